// lego_mo.h — device buffers and entry points of the scan-to-map step
// (lego_mo.hip).  One MoDev per stream context.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>

#include "lego_icp.h"

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
  int derr;  // the step's VoxelGrids' error word (VgScratch::err): nonzero = a sort returned a foreign payload
};

// VoxelGrid / index-build scratch for clouds of up to cap points (lego_vg.hip).
struct VgScratch {
  unsigned* keys;   // [cap] voxel index per point, sorted in place
  int* vals;        // [cap] point index, moved with the keys
  int* pl;          // [cap] a round's swapped left stops, by partner rank
  int* pr;          // [cap] a round's swapped right stops, by rank
  int2* big;        // [2][capBig] segments partitioned by the current / next round
  int* cut;         // [capBig] the round's cut per segment
  int* kcnt;        // [capBig] the round's swap count per segment
  int* tileOff;     // [capBig + 1] first tile of each segment
  int* tileSeg;     // [capTiles] the round's tile -> its segment | its index in the segment << 16
  int* tileL;       // [capTiles] left stops per tile
  int* tileR;       // [capTiles] right stops per tile
  int4* loc;        // [capLoc] segments sorted in one workgroup (s, e, depth budget)
  int* scanTiles;   // [capScanTiles] tile sums of the scans
  int* ctl;         // [16] counters (lego_vg.hip C_*)
  int* mm;          // [6] ordered-int min / max
  int* overflow;    // [1]
  // error word: set (atomicOr 1) when a sorted payload lies outside the cloud,
  // which no sort can produce unless the device's LDS / registers were
  // corrupted; the payload is then not read.  ctl + C_ERR after
  // vg_scratch_alloc (lego_voxel_grid reads it per call); a mapping context
  // points its scratches at MoCounts::derr (read after every step).
  int* err;
  int cap, capBig, capTiles, capLoc, capScanTiles;
  int rounds = -1;  // host only: lego_ctx_opts::vg_rounds (-1: by the cloud's size)
};

// 1 m cells of the mapping NN index, hashed into T buckets
__device__ __forceinline__ unsigned mo_cell_hash(int ix, int iy, int iz) {
  unsigned long long k = ((unsigned long long)(unsigned)(ix + (1 << 20)) << 42) |
                         ((unsigned long long)(unsigned)(iy + (1 << 20)) << 21) |
                         (unsigned long long)(unsigned)(iz + (1 << 20));
  k ^= k >> 33; k *= 0xff51afd7ed558ccdULL; k ^= k >> 33;
  return (unsigned)k;
}
__device__ __forceinline__ int cell1(float v) { return (int)floorf(v); }  // 1 m cells

// 1 m hashed cells over a map cloud: points grouped by bucket (w = index).
// k_mo_rows' candidate cache (MoDev::cand): points per query, queries cached,
// the radius kept around the reference point and how far the query may move
// from it (kCandR >= 1 + kCandMove, with room for rounding).
constexpr int kCand = 96, kCandQueries = 65536;
constexpr float kCandMove = 0.25f, kCandR = 1.27f;

struct MoIndex {
  int* begin;
  int* end;
  float4* sorted;
  int T, cap;
};

// Keyframe store (saveKeyFramesAndFactor :1353-1454 without iSAM2: the chain
// estimate equals the initial values when there are no loop factors) and the
// surrounding-map bookkeeping of extractSurroundingKeyFrames (:1001-1065).
struct MoKeyframes {
  float4* pos3;      // [kcap] x, y, z, intensity = key index (cloudKeyPoses3D)
  float* pose6;      // [kcap * 6] x, y, z, roll, pitch, yaw (cloudKeyPoses6D)
  double* time;      // [kcap] cloudKeyPoses6D[i].time
  int* seg;          // [kcap * 6] arena offset / count of corner, surf, outlier DS clouds
  float4* arena;     // [acap] keyframe clouds
  int* exID;         // [kcap] surroundingExistingKeyPosesID
  int* plan;         // [kcap * 4] per existing key: key, corner offset, surf offset, -
  float* planPose;   // [kcap * 6] loop-closure mode: the pose each planned key is transformed with
  float4* sur;       // [kcap] surrounding key poses (radius hits, distance order)
  float4* surDS;     // [kcap] their 1 m voxel filter
  unsigned long long* sortKeys;  // [kcap] (distance bits, index) of the hits
  int* meta;         // [kKfMeta] K, arenaTop, nEx, nSur, nSurDS, nCornerFromMap, nSurfFromMap, store full
                     // (sticky), saved this step, radius hits over the sort capacity (this step)
  float* robot;      // previousRobotPos xyz, currentRobotPos xyz
  int kcap, acap;
};
enum { KF_K = 0, KF_TOP = 1, KF_NEX = 2, KF_NSUR = 3, KF_NSURDS = 4, KF_NCM = 5, KF_NSM = 6, KF_OVF = 7,
       KF_SAVED = 8, KF_HITOVF = 9, kKfMeta = 16 };
// mo_step_device / mo_loop_closure_device status codes
enum { MO_OK = 0, MO_E_LAUNCH = -1, MO_E_STORE_FULL = -2, MO_E_RADIUS_HITS = -3, MO_E_MAP_CAP = -4 };

struct MoDev {
  MoState* st;
  MoCounts* cnt;
  VgScratch vg;
  // fixed map (config C5) and its voxel-filtered form
  float4 *cornerMap, *surfMap, *cornerMapDS, *surfMapDS;
  int mapCornerCap, mapSurfCap;
  int nCornerMap, nSurfMap;  // the installed map's raw sizes
  int mapPerStep;            // lego_mo_opts.fixed_map_per_step: filter + index every step
  MoIndex cornerIx, surfIx;
  // the scan's clouds and their filtered forms
  float4 *cornerLast, *surfLast, *outlierLast;
  float4 *cornerDS, *surfDS, *outlierDS, *surfTotal, *surfTotalDS;
  int scanCap;
  float* rows;  // [rowCap x 8]
  int rowCap;
  // Per-query 5-NN candidates across the LM iterations (k_mo_rows): the map
  // points of the query's 27-cell block within kCandR of where its last full
  // search put it (candRef.xyz; .w = their count, or < 0: none kept), so a
  // later iteration that leaves the query in the same cell and within
  // kCandMove of that point searches only those (every point within 1 m of
  // it is among them: exact).  Queries [0, candQ).
  float4* cand;     // [candQ x kCand]
  float4* candRef;  // [candQ]
  int candQ;
  double* part;  // [partCap x 28] the rows' AtA / AtB sums per k_mo_rows workgroup
  int partCap;
  // keyframe-built map (when no fixed map is installed)
  MoKeyframes kf;
  float4 *cornerFromMap, *surfFromMap;  // [fromMapCap]
  int fromMapCap;
  // Fork-join of a step's independent VoxelGrids (each is latency-bound and
  // fills a small part of the GPU): fork[0] (the context's odometry stream)
  // takes the scan's outlier cloud, then surf + outlier; fork[1] the scan's
  // surf cloud, then the map's corner cloud and its index; the step's stream
  // the map's surf cloud and index, then the scan's corner cloud.
  // Each chain has its own VoxelGrid scratch.
  hipStream_t fork[2];
  hipEvent_t ev[6];
  hipEvent_t prof[6] = {};  // lego_ctx_opts::mo_evprof (diagnostic): the step's chain ends, timed
  VgScratch vgMap2, vgScan1, vgScan2;
  bool hostprof = false, evprof = false;  // lego_ctx_opts::mo_hostprof / mo_evprof (host only)
};

struct MoStepArgs {
  double quat[4];  // /laser_odom_to_init orientation (x, y, z, w)
  double pos[3];
  int nCorner, nSurf, nOutlier;
  int imuOn;              // transformUpdate's IMU blend (:465-490), roll / pitch from the host queue
  float imuRoll, imuPitch;
  double stamp;           // timeLaserOdometry (the keyframe's time)
  // loop-closure mode's recent-keyframe map: nPlan >= 0 entries of kf.plan /
  // kf.planPose (uploaded by the host), nCM / nSM the map clouds' sizes;
  // nPlan = -1: the radius-search map
  int nPlan = -1, nCM = 0, nSM = 0;
  // the scan's clouds on the device when they need no upload (lego_mo_process:
  // the context's own fa output); null: MoDev's cornerLast / surfLast /
  // outlierLast.  outlierRaw is the outlier cloud before adjustOutlierCloud.
  const float4* corner = nullptr;
  const float4* surf = nullptr;
  const float4* outlierRaw = nullptr;
};

// Loop closure (lego_loop.hip): the detection result and gather plan, the
// ICP state.  Device-resident; the host reads it back.
constexpr int kLcPlan = 2 + 2 * 51;  // latest corner + surf, then +-25 keyframes x 2 clouds
struct LcState {
  int K, latest, closest, detected;
  int nPlan, nPlanSrc, nSrcRaw, nTgtRaw;
  int plan[kLcPlan][4];  // key, arena offset, count, output offset
  int nSrc, nTgt;
  int iterations, converged, done, nFit;
  float T[4][4], fin[4][4];
  IcpCriteria crit;
  double fitness;
};
struct LcDev {
  LcState* st;
  float4 *srcRaw, *src, *cur, *tgtRaw, *tgt;
  int* cIdx;
  float* cD;
  MoIndex ix;
  int cap;
};

// allocates every VgScratch buffer for clouds of up to cap points through
// alloc (0 = success)
int vg_scratch_alloc(VgScratch& v, int cap, void* ctx, int (*alloc)(void* ctx, void** p, size_t bytes));
int voxel_grid_device(const float4* in, int n, const int* nDev, float leaf, float4* out, int* nOut,
                      const VgScratch& v, hipStream_t s);
// partition rounds voxel_grid_device launches for a cloud of n points
// (LEGO_VG_ROUNDS overrides: diagnostic)
// partition rounds for a cloud of n points; forced >= 0 (lego_ctx_opts::vg_rounds) overrides
int vg_rounds_for(int n, int forced = -1);
void mo_evprof_print(MoDev& m);  // after the step's stream is synchronised
// the VgScratch counters of the last voxel_grid_device on s (16 ints, synchronous)
int vg_read_ctl(const VgScratch& v, int* ctl16, hipStream_t s);
int mo_set_map_device(MoDev& m, int nCornerMap, int nSurfMap, hipStream_t s);
// libstdc++'s std::sort permutation of (key, index) by key on the device
// (lego_vg.hip): mode 0..8 picks the form, block size and sum-order rule
// (lego_sort_permutation); heap: the heap-sorted pieces are counted into it.
// sort_perm_cap: the largest n of a mode, -1 for an unknown mode.
int sort_perm_cap(int mode);
int sort_perm_device(const uint32_t* keys, int n, int mode, int* perm, int* heap, hipStream_t s);
int index_build_device(const float4* pts, int n, const int* nDev, MoIndex& ix, const VgScratch& v, hipStream_t s);
// One performLoopClosure over the keyframe store (tnow = timeLaserOdometry).
// Returns MO_OK (hostState holds the result), MO_E_LAUNCH, or MO_E_MAP_CAP when
// the clouds exceed the loop buffers.
int mo_loop_closure_device(MoDev& m, LcDev& lc, double tnow, LcState* hostState, hipStream_t s);
// One mapping step.  fixedMap: the installed map; otherwise the keyframe map.
// Returns MO_OK, MO_E_LAUNCH, MO_E_STORE_FULL (an earlier step could not save
// its keyframe), MO_E_RADIUS_HITS (more key poses within the search radius
// than the sort holds) or MO_E_MAP_CAP (the surrounding map exceeds its
// buffers), the last three before anything of the step ran.  That a keyframe
// of THIS step did not fit is reported through meta[KF_OVF] after the step.
int mo_step_device(MoDev& m, const MoStepArgs& a, bool fixedMap, float radius, hipStream_t s);

}  // namespace lego
