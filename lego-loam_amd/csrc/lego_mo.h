// lego_mo.h — device buffers and entry points of the scan-to-map step
// (lego_mo.hip).  One MoDev per stream context.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>

namespace lego {

// mapOptimization member state that persists across mapping steps
// (mapOptmization.cpp:145-260), device-resident.
struct MoState {
  float transformSum[6], transformIncre[6], transformTobeMapped[6];
  float transformBefMapped[6], transformAftMapped[6];
  float matP[36];
  int isDegenerate;
  float cRoll, sRoll, cPitch, sPitch, cYaw, sYaw;  // updatePointAssociateToMapSinCos cache
  int optimized, converged, iterations, rowsLast;
};

// Cloud sizes produced on the device.
struct MoCounts {
  int cornerMapDS, surfMapDS;
  int cornerDS, surfDS, outlierDS, surfTotal, surfTotalDS;
  int _pad;
};

// VoxelGrid / index-build scratch for clouds of up to cap points.
struct VgScratch {
  unsigned* keys;
  unsigned* keys2;
  int* vals;
  int* vals2;
  int* heads;
  int* scan;
  int* mm;        // [6] ordered-int min / max
  int* overflow;  // [1]
  void* tmp;
  size_t tmpBytes;
  int cap;
};

// 1 m hashed cells over a map cloud: points sorted by bucket (w = index).
struct MoIndex {
  int* begin;
  int* end;
  float4* sorted;
  int T, cap;
};

struct MoDev {
  MoState* st;
  MoCounts* cnt;
  VgScratch vg;
  // fixed map (config C5) and its voxel-filtered form
  float4 *cornerMap, *surfMap, *cornerMapDS, *surfMapDS;
  int mapCornerCap, mapSurfCap;
  MoIndex cornerIx, surfIx;
  // the scan's clouds and their filtered forms
  float4 *cornerLast, *surfLast, *outlierLast;
  float4 *cornerDS, *surfDS, *outlierDS, *surfTotal, *surfTotalDS;
  int scanCap;
  float* rows;  // [rowCap x 8]
  int rowCap;
};

struct MoStepArgs {
  double quat[4];  // /laser_odom_to_init orientation (x, y, z, w)
  double pos[3];
  int nCorner, nSurf, nOutlier;
};

size_t voxel_scratch_tmp_bytes(int cap);
int voxel_grid_device(const float4* in, int n, const int* nDev, float leaf, float4* out, int* nOut,
                      const VgScratch& v, hipStream_t s);
int mo_set_map_device(MoDev& m, int nCornerMap, int nSurfMap, hipStream_t s);
int mo_step_device(const MoDev& m, const MoStepArgs& a, hipStream_t s);

}  // namespace lego
