// lego_wire.h — PointCloud2 decode plan and launcher (lego_wire.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lego_loam.h"

namespace lego {

constexpr int kPc2Fields = 5;  // x, y, z, intensity, ring

// One message of a decode launch: where its points are and where each
// PointXYZIR field sits in a point (-1: no matching field, stays 0).
struct Pc2Desc {
  const uint8_t* data;
  uint32_t height, width, pointStep, rowStep;
  int off[kPc2Fields];
  int _pad;
  uint64_t outBase;  // first output point
};

int pc2_plan(const lego_pc2_msg* m, Pc2Desc* d);
int launch_pc2_decode(const Pc2Desc* dDescs, int K, uint64_t maxPoints, lego_point_xyzir* out, hipStream_t s);

}  // namespace lego
