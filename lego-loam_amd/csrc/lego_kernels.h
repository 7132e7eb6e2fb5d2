// lego_kernels.h — host-side launchers of the gfx950 kernels + stage timer.
#pragma once
#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "lego_device.h"

namespace lego {

// Optional per-stage hipEvent timeline (bench / profiling).  mark(name) closes
// the previous stage and opens `name` on the stream.
class StageTimer {
 public:
  bool enabled = false;
  void begin() {
    names_.clear();
    used_ = 0;
  }
  void mark(const char* name, hipStream_t s) {
    if (!enabled) return;
    if (used_ >= events_.size()) {
      hipEvent_t e;
      if (hipEventCreate(&e) != hipSuccess) {  // timing is diagnostic: drop it, never fail the call
        enabled = false;
        return;
      }
      events_.push_back(e);
    }
    if (hipEventRecord(events_[used_], s) != hipSuccess) return;
    ++used_;
    names_.push_back(name);
  }
  void end(hipStream_t s) { mark("__end__", s); }
  // Collapses repeated names into totals.  Call after a stream sync.
  void collect(std::vector<std::string>& names, std::vector<float>& ms) const {
    names.clear();
    ms.clear();
    for (size_t i = 0; i + 1 < used_; ++i) {
      float t = 0;
      if (hipEventElapsedTime(&t, events_[i], events_[i + 1]) != hipSuccess) t = 0;
      size_t k = 0;
      for (; k < names.size(); ++k)
        if (names[k] == names_[i]) break;
      if (k == names.size()) {
        names.push_back(names_[i]);
        ms.push_back(0);
      }
      ms[k] += t;
    }
  }
  ~StageTimer() {
    for (auto e : events_) (void)hipEventDestroy(e);
  }

 private:
  std::vector<hipEvent_t> events_;
  std::vector<std::string> names_;
  size_t used_ = 0;
};

// Hash-grid nearest-neighbour index over a snapshot of a last cloud.
struct NNGrid {
  unsigned long long* keys;  // [T]
  int* cnt;                  // [T]
  int* start;                // [T]
  int* slot;                 // [cap] per-point slot (build scratch)
  float4* pts;               // [cap] cell-ordered snapshot
  int* idx;                  // [cap] original index
};

// Odometry state kept on the device for one stream (featureAssociation.cpp
// member variables that persist across scans).
struct OdomState {
  float transformCur[6];
  float transformSum[6];
  float matP[9];
  int isDegenerate;
  int inited;            // systemInitedLM
  int cornerLastNum, surfLastNum;
  int nnCornerNum, nnSurfNum;  // point sets the NN structures were built on
  int frameCount;
  int _pad[3];
};

struct OdomBufs {
  OdomState* st;
  float4* cornerLast;   // [capCorner]
  float4* surfLast;     // [capSurf]
  NNGrid gC, gS;        // hash grids over snapshots of the last clouds
  int capCorner, capSurf;
  // per-scan outputs of the batch
  float* sumOut;        // [B*6]
  float* curOut;        // [B*6]
  int* validOut;        // [B]
  int* pubOut;          // [B]
  float4* cornerEnd;    // [B*capLS]  less-sharp after TransformToEnd
  float4* surfEnd;      // [B*P]      less-flat after TransformToEnd
  int capLS;
};

void launch_ip(const BatchBufs& bb, const DevCfg& c, int B, int want_labels, hipStream_t s,
               StageTimer* tm);
void launch_fa(const BatchBufs& bb, const DevCfg& c, int B, FaCarry* d_carry, hipStream_t s,
               StageTimer* tm);
void launch_odom(const BatchBufs& bb, const OdomBufs& ob, const DevCfg& c, int B, hipStream_t s,
                 StageTimer* tm, unsigned long long* gkeys, int* gqi, unsigned long long* prof);
size_t odom_grid_table(int npts);

}  // namespace lego
