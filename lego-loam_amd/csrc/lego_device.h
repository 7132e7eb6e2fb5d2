// lego_device.h — shared device-side types for the gfx950 kernels.
//
// Data layout in HBM (one stream context, batch of B scans, P = N*H pixels):
//   range image / label / parent / root / ground : [B][P]  (row-major pixels)
//   full cloud                                    : [B][P]  float4 (x,y,z,I)
//   segmented cloud + cloud_info arrays           : [B][P]  (first Ns valid)
//   feature ring slots                            : [B][N][cap]
//   compacted features                            : [B][cap]
// Everything a later stage reads stays resident; nothing round-trips to host
// inside lego_odom_batch except the 64-B pose records at the end.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lego_loam.h"
#include "lego_numerics.h"

namespace lego {

constexpr int kMaxRings = 128;        // rowmask = 2 x u64
constexpr int kMaxHorizon = 2048;     // col fits u16; a ring's less-flat VoxelGrid sort holds <= 2048 keys (lego_vgsort.h)
constexpr int kSharpPerRing = 12;     // 2 per sector (featureAssociation.cpp:709)
constexpr int kLessSharpPerRing = 120;// 20 per sector (:713)
constexpr int kFlatPerRing = 24;      // 4 per sector (:746-748)
constexpr int kExtractThreads = 256;
constexpr int kSortCap = 1024;        // sector sort buffer (sector <= H/6 + 2)
constexpr int kVoxCap = 4096;         // per-ring less-flat voxel sort

struct DevCfg {
  int N, H, P, g;
  float ang_res_x, min_range, mount_angle, theta;
  float sinAX, cosAX, sinAY, cosAY;
  int valid_pt, valid_line;
  float edge_thr, surf_thr, nn_sq, scan_period;
  int skip;  // skipFrameNum (featureAssociation.cpp:284)
  // the segmentation angle test's quotient band (seg_edge_fast, lego_ip.hip):
  // tan(theta -+ 1e-5), and whether theta < pi / 2 - 1e-3
  double tanLo, tanHi;
  int quad1;
  int segHbm;  // diagnostic (LEGO_SEG_HBM): the HBM union-find for every image size
  // useCloudRing (utility.h:60): 1 = the row is the point's ring channel; 0 =
  // the row from the vertical angle, (angle + ang_bottom) / ang_res_y
  // (imageProjection.cpp:228-231), and non-finite points are removed first
  // (pcl::removeNaNFromPointCloud, :170) instead of rejecting the scan
  int ringRow;
  float ang_res_y, ang_bottom;
};

// ---- IMU (featureAssociation.cpp:84-159, 317-459, 525-614)
constexpr int kImuQ = 200;  // imuQueLength, utility.h:109
enum { IV_ROLL, IV_PITCH, IV_YAW, IV_VX, IV_VY, IV_VZ, IV_SX, IV_SY, IV_SZ, IV_AX, IV_AY, IV_AZ, kImuV };

// featureAssociation's IMU queue as adjustDistortion sees it for one scan
// (the host runs imuHandler / AccumulateIMUShiftAndRotation as messages are
// delivered and snapshots the queue per scan).
struct ImuSnap {
  double stamp;           // timeScanCur
  double time[kImuQ];
  float v[kImuV][kImuQ];  // imuRoll, imuPitch, imuYaw, imuVelo*, imuShift*, imuAngularRotation*
  int last;               // imuPointerLast (-1: no message yet)
  int lastIter;           // imuPointerLastIteration
  int _pad[2];
};

// Per-scan IMU terms.  k_fa_imu_start / k_fa_point write this scan's raw
// values; k_fa_fixup resolves the members that persist across scans (a scan
// with no IMU message yet, or too few points, leaves them as they were) in
// stream order; the odometry reads the resolved values.
struct ImuScan {
  int active;    // imuPointerLast >= 0
  int hasFirst;  // the loop reached point 0 (ns >= 1)
  int hasLast;   // ... and a later point (ns >= 2)
  int _pad;
  float rollStart, pitchStart, yawStart;
  float veloStart[3];
  float cRS, cPS, cYS, sRS, sPS, sYS;  // updateImuRollPitchYawStartSinCos
  float ar0[3];                        // imuAngularRotation*Cur at point 0
  float rollCur, pitchCur, yawCur;     // at the last point
  float vfs[3];                        // imuVeloFromStart*Cur at the last point
  float angFromStart[3];               // imuAngularFromStart* (resolved)
};

// Per-stream feature-extraction carry: the stale
// cloudSmoothness[4] entry (value is always 0.0f, only its index moves) and the
// sticky cloudNeighborPicked[0].  S* = {0, 1} is the steady state.  Then the
// featureAssociation IMU members that persist from scan to scan.
struct FaCarry {
  int phantom_ind;
  int picked0;
  int flags;
  int _pad;
  float rollStart, pitchStart, yawStart, rollCur, pitchCur, yawCur;
  float vfs[3], arLast[3], angFromStart[3];
};

// Batch-wide device pointers (filled by the host, passed by value).
// The gated imageProjection topics of one scan (lego_ip_process with
// LEGO_IP_GATED), allocated on first use.
struct GatedBufs {
  float4* info;    // [P] /full_cloud_info
  float4* ground;  // [P] /ground_cloud
  float4* pure;    // [P] /segmented_cloud_pure
  int* n;          // [2] ground, pure counts
};

// BatchBufs::bad bits (per scan, zeroed before each batch): the host returns
// LEGO_E_NOT_DENSE for the first, LEGO_E_DEVICE for the second (a VoxelGrid
// sort handed back a payload outside its input: it cannot happen unless the
// device's LDS or registers are corrupted, and is never clamped into range).
// kBadLfLate (LEGO_E_DEVICE): a node call's hand-off gave up waiting for the
// less-flat VoxelGrid on the side stream (launch_odom's lfReady).
constexpr int kBadNotDense = 1, kBadPermutation = 2, kBadLfLate = 4;
struct BatchBufs {
  int B;
  const ImuSnap* imu;        // [B] or null: no IMU message delivered to this batch's stream(s)
  ImuScan* imuScan;          // [B]
  int Nmax;                  // max input points per scan
  // ---- image projection
  const void* pts;           // lego_point_xyzir [*], or with bit 0 set the node call's packed float4 [*] (pts_view)
  const int64_t* off;        // [B+1]
  int* owner;                // [B*P]
  float* range;              // [B*P]
  float4* full;              // [B*P]
  int8_t* ground;            // [B*P]
  int* label;                // [B*P]  init label, then final label image
  int* parent;               // [B*P]
  int* root;                 // [B*P]
  uint8_t* edges;            // [B*P]
  int* csize;                // [B*P]
  unsigned long long* rowmask;  // [B*P*2]
  float* rawang;             // [B*2]
  int* bad;                  // [B]  kBadNotDense: non-finite xyz seen (imageProjection.cpp:174-176); kBadPermutation
  // ---- segmented cloud + cloud_info
  float4* seg;               // [B*P]
  uint8_t* gflag;            // [B*P]
  uint32_t* col;             // [B*P]
  float* srange;             // [B*P]
  float4* outl;              // [B*P]
  int* ns;                   // [B]  segmented count
  int* nout;                 // [B]
  int* sri;                  // [B*N]
  int* eri;                  // [B*N]
  float* orient;             // [B*3]
  // ---- feature association
  int* firsthalf;            // [B]
  float4* dsk;               // [B*P] deskewed segmented cloud
  float* curv;               // [B*P]
  uint8_t* pick0;            // [B*P] occlusion marks
  float4* r_sharp;           // [B*N*12]
  float4* r_lsharp;          // [B*N*120]
  float4* r_flat;            // [B*N*24]
  float4* r_lflat;           // [B*P]   ring r at [b*P + r*H]
  int* r_cnt;                // [B*N*4]
  FaCarry* spec_out;         // [B] carry produced under S*
  int* fa_flags;             // [B]
  unsigned long long* xprof; // k_extract phase stamps (lego_extract_profile) or nullptr
  float4* f_sharp;           // [B*N*12]
  float4* f_lsharp;          // [B*N*120]
  float4* f_flat;            // [B*N*24]
  float4* f_lflat;           // [B*P]
  int* f_cnt;                // [B*4]
};

// Buffer views inside the batch for scan b.
__device__ __forceinline__ int scan_npts(const BatchBufs& bb, int b) {
  return (int)(bb.off[b + 1] - bb.off[b]);
}

}  // namespace lego
