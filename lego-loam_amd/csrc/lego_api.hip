// lego_api.hip — the C-ABI (include/lego_loam.h) over the gfx950 kernels.
//
// One lego_ctx = one lidar stream = one HIP stream on one device.  All
// per-scan work is device resident; the node-shaped calls (lego_ip_process,
// lego_fa_process) are the batch path at B = 1 followed by the copies the
// reference's publishers would serialise.  There is no CPU fallback: every
// entry point fails with LEGO_E_DEVICE if HIP cannot run.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <array>
#include <atomic>
#include <cstring>
#include <deque>
#include <new>
#include <string>
#include <vector>

#include "lego_device.h"
#include "lego_fusion_host.h"
#include "lego_imu_host.h"
#include "lego_kernels.h"
#include "lego_mo.h"
#include "lego_loam.h"
#include "lego_pack_host.h"
#include "lego_pgo_host.h"
#include "lego_seg.h"
#include "lego_wire.h"

using namespace lego;

namespace {

thread_local char g_err[512] = "";

void set_err(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

#define HIPCHK(x)                                                                 \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      set_err("%s:%d %s: %s", __FILE__, __LINE__, #x, hipGetErrorString(e_));     \
      return LEGO_E_DEVICE;                                                       \
    }                                                                             \
  } while (0)

// tf::Quaternion::setRPY + publishOdometry axis shuffle (featureAssociation.cpp:1728-1737)
void odom_quat(const float ts[6], double q[4], double pos[3]) {
  const double roll = ts[2], pitch = -ts[0], yaw = -ts[1];
  const double hy = yaw * 0.5, hp = pitch * 0.5, hr = roll * 0.5;
  const double cy = std::cos(hy), sy = std::sin(hy), cp = std::cos(hp), sp = std::sin(hp);
  const double cr = std::cos(hr), sr = std::sin(hr);
  const double g0 = sr * cp * cy - cr * sp * sy, g1 = cr * sp * cy + sr * cp * sy;
  const double g2 = cr * cp * sy - sr * sp * cy, g3 = cr * cp * cy + sr * sp * sy;
  q[0] = -g1; q[1] = -g2; q[2] = g0; q[3] = g3;
  pos[0] = ts[3]; pos[1] = ts[4]; pos[2] = ts[5];
}

template <typename T>
hipError_t dalloc(T** p, size_t n) {
  return hipMalloc((void**)p, sizeof(T) * (n ? n : 1));
}

}  // namespace

// for the other translation units of the library (lego_comm.hip)
void lego_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

constexpr int kFetchHdr = 32;  // header words of the host staging block (fetch_ip / fetch_fa)
constexpr size_t kMoResBytes = ((sizeof(MoState) + 15) & ~(size_t)15) + ((sizeof(MoCounts) + 15) & ~(size_t)15) +
                               sizeof(int) * kKfMeta;

struct lego_ctx {
  lego_sensor_cfg cfg;
  DevCfg dc;
  lego_ctx_opts opts;  // fixed at creation (lego_create_ex)
  LaunchOpts lo;       // its launch-shape part, as launch_ip / launch_fa take it
  // a node call's hand-off gave up waiting for the VoxelGrid (kBadLfLate):
  // the stream's state was not advanced and the odometry calls refuse to run
  // until lego_reset
  bool needReset = false;
  int device = 0;
  int maxPoints = 0, maxBatch = 0;  // maxBatch: scans per call over all streams
  int nStreams = 1;                   // a fleet context carries nStreams independent streams
  int cus = 1;                        // the device's CUs (hipDeviceAttributeMultiprocessorCount)
  hipStream_t stream = nullptr;   // image projection + feature extraction (and everything else)
  hipStream_t ostream = nullptr;  // the odometry chain (overlaps the next batch's extraction)
  // Two batch slots: the per-scan buffers hold 2 x maxBatch scans; batch n
  // uses slot n % 2, so batch n + 1's projection + extraction (stream) run
  // while batch n's odometry (ostream) still reads its slot.
  hipEvent_t faDone[2] = {nullptr, nullptr};    // extraction of the slot's batch finished
  hipEvent_t recsDone[2] = {nullptr, nullptr};  // the slot's packed records are on the host
  hipEvent_t oJoin = nullptr;                   // ostream work so far (node calls order after it)
  hipEvent_t lfFork = nullptr;                  // a node call's features, before its side-stream VoxelGrid
  unsigned* d_lfReady = nullptr;                // [1] its rings counted as their less-flat clouds land
  // A fleet batch's projection + extraction in parts of whole streams, part
  // p > 0 on fstream[p - 1] (created on first use; front_parts)
  static constexpr int kFrontPartsMax = 4;
  hipStream_t fstream[kFrontPartsMax - 1] = {};
  hipEvent_t fFork = nullptr, fJoin[kFrontPartsMax - 1] = {};
  int nextSlot = 0, inflight = 0, oldest = 0;
  int slotB[2] = {0, 0};
  std::vector<double> slotStamps[2];
  int lastBase = 0;  // first scan slot of the batch lego_batch_fetch reads
  BatchBufs bb{};
  OdomBufs ob{};
  FaCarry* d_carry = nullptr;
  unsigned long long* d_prof = nullptr;  // in-kernel phase stamps (lego_odom_profile)
  bool profOn = false;
  lego_point_xyzir* d_pts = nullptr;
  int64_t* d_off = nullptr;
  std::vector<void*> allocs;
  StageTimer tm, otm;            // node-shaped calls
  StageTimer stm[2], sotm[2];    // per batch slot: extraction / odometry stages
  StageTimer ftm;                // the front-end parts p > 0 (never enabled)
  // last batch
  int lastB = 0;
  std::vector<double> stamps;
  // host staging (library-owned outputs): regions of one pinned block
  // (hostBlock) that k_fetch writes directly, one launch and one sync per
  // fetched scan (pageable staging cost a synchronous copy per array)
  unsigned char* hostBlock = nullptr;
  int32_t* h_hdr = nullptr;  // k_fetch's header words (counts, flags, orientation, transforms)
  void* h_moRes = nullptr;   // lego_mo_process's MoState / MoCounts / keyframe words (kMoResBytes)
  lego_point_xyzi *h_seg = nullptr, *h_outl = nullptr, *h_full = nullptr, *h_sharp = nullptr, *h_lsharp = nullptr,
                  *h_flat = nullptr, *h_lflat = nullptr;
  GatedBufs gb{};  // LEGO_IP_GATED outputs (first use)
  uint8_t* d_handoff = nullptr;  // lego_handoff_pack's packet (grown on demand)
  hipStream_t hstream = nullptr; // the hand-off packing (first use)
  size_t handoffCap = 0;
  hipEvent_t handoffFence = nullptr;  // a lego_comm send of d_handoff in flight (lego_handoff_fence)
  bool handoffFenced = false;
  std::vector<uint8_t> h_handoffHead;
  lego_point_xyzi *h_info = nullptr, *h_gcloud = nullptr, *h_pure = nullptr;
  lego_point_xyzi *h_cornerLast = nullptr, *h_surfLast = nullptr, *h_outlLast = nullptr;
  // the device work generation: every call that launches into the batch
  // slots bumps it; fetch_fa records the slot and generation its published
  // clouds (h_cornerLast / h_surfLast / h_outlLast) came from, so that
  // lego_mo_process can take them from the device when handed them back
  uint64_t devGen = 0, faGen = ~0ull;
  int faK = -1, faCnt[3] = {0, 0, 0};
  int32_t *h_sri = nullptr, *h_eri = nullptr, *h_label = nullptr, *h_bad = nullptr;
  uint8_t* h_gflag = nullptr;
  uint32_t* h_col = nullptr;
  float *h_range = nullptr, *h_rimg = nullptr;
  int8_t* h_gimg = nullptr;
  lego_ip_out lastIp{};
  bool lastIpDevice = false;  // lastIp describes batch slot 0 on device
  bool lastBatch = false;     // lastB / lastBase describe a waited batch (lego_handoff_pack)
  // /imu_raw: featureAssociation's and mapOptimization's queues (host), the
  // per-scan snapshots of the former for a batch
  // raw PointCloud2 staging (lego_*_pc2): grown on demand
  uint8_t* d_raw = nullptr;
  size_t rawCap = 0;
  Pc2Desc* d_desc = nullptr;
  std::vector<Pc2Desc> h_desc;
  PackedRec* d_pack = nullptr;  // h_pack's device address: k_pack_recs writes the records there
  PackedRec* h_pack = nullptr;  // pinned
  int64_t* h_offp = nullptr;    // pinned [maxBatch + 1]: device offsets read back for validation
  float4* h_stage = nullptr;  // pinned [maxPoints] packed points, created by the first host-buffer node call
  std::unique_ptr<lego::PackPool> pack;  // the upload pass's helper threads (clouds of more than two chunks)
  OdomState* h_resetSt = nullptr;   // pinned [S]: construction state (ctx_reset)
  FaCarry* h_resetCarry = nullptr;  // pinned [S]
  Fusion fusion;  // transformFusion state
  FaImuQueue faImu;
  MoImuQueue moImu;
  std::vector<ImuSnap> h_imu;
  ImuSnap* d_imu = nullptr;
  // scan-to-map (lego_mo_*): buffers allocated by the first lego_mo_set_map
  MoDev mo{};
  bool moAlloc = false, moFixed = false;
  // lego_voxel_grid: its own scratch and device cloud buffers, grown on demand
  VgScratch vgApi{};
  float4 *vgIn = nullptr, *vgOut = nullptr;
  int* vgN = nullptr;
  int vgCap = 0;
  int vgStats[8] = {};
  hipEvent_t vgEv[2] = {nullptr, nullptr};  // lego_voxel_grid's timing events (first use)
  lego_mo_opts moOpts{};
  double moTimeLast = -1;
  bool moStoreFull = false;  // sticky KF_OVF seen: no step runs until lego_reset
  double moTimeOdom = 0;  // timeLaserOdometry: the last hand-off's stamp (laserOdometryHandler :630)
  LcDev lc{};             // loop closure buffers (first lego_mo_loop_closure)
  // loop-closure mode (lego_mo_opts.loop_closure_enable): the pose graph, the
  // recent-keyframe queue (key + the pose it was transformed with) and host
  // mirrors of the saved keyframes' poses and arena segments
  struct RecentKf {
    int key;
    std::array<float, 6> pose;
  };
  PoseGraph pg;
  std::deque<RecentKf> recent;
  int latestFrameID = 0;  // mapOptmization.cpp:373
  bool aLoopIsClosed = false;
  float transformLast[6] = {0, 0, 0, 0, 0, 0};
  std::vector<std::array<float, 6>> kfPose;  // x y z roll pitch yaw (cloudKeyPoses6D)
  std::vector<std::array<int, 6>> kfSeg;
  std::vector<std::string> tnames;
  std::vector<float> tms;

  template <typename T>
  hipError_t alloc(T** p, size_t n) {
    hipError_t e = dalloc(p, n);
    if (e == hipSuccess) allocs.push_back((void*)*p);
    return e;
  }
  ~lego_ctx() {
    if (device >= 0) (void)hipSetDevice(device);
    if (stream) (void)hipStreamSynchronize(stream);  // batches still in flight
    if (ostream) (void)hipStreamSynchronize(ostream);
    for (auto f : fstream)
      if (f) (void)hipStreamSynchronize(f);
    if (mo.fork[1]) (void)hipStreamSynchronize(mo.fork[1]);  // the mapping VoxelGrids' fork
    if (d_raw) (void)hipFree(d_raw);
    if (handoffFenced) (void)hipEventSynchronize(handoffFence);  // a send still reading d_handoff
    if (handoffFence) (void)hipEventDestroy(handoffFence);
    for (auto e : vgEv)
      if (e) (void)hipEventDestroy(e);
    if (d_handoff) (void)hipFree(d_handoff);
    if (h_pack) (void)hipHostFree(h_pack);
    if (h_offp) (void)hipHostFree(h_offp);
    if (h_stage) (void)hipHostFree(h_stage);
    if (h_resetSt) (void)hipHostFree(h_resetSt);
    if (h_resetCarry) (void)hipHostFree(h_resetCarry);
    if (hostBlock) (void)hipHostFree(hostBlock);
    for (void* p : allocs) (void)hipFree(p);
    if (oJoin) (void)hipEventDestroy(oJoin);
    if (lfFork) (void)hipEventDestroy(lfFork);
    if (fFork) (void)hipEventDestroy(fFork);
    for (auto e : fJoin)
      if (e) (void)hipEventDestroy(e);
    for (auto f : fstream)
      if (f) (void)hipStreamDestroy(f);
    for (int i = 0; i < 2; ++i) {
      if (faDone[i]) (void)hipEventDestroy(faDone[i]);
      if (recsDone[i]) (void)hipEventDestroy(recsDone[i]);
    }
    if (mo.fork[1]) (void)hipStreamDestroy(mo.fork[1]);
    for (auto e : mo.ev)
      if (e) (void)hipEventDestroy(e);
    for (auto e : mo.prof)
      if (e) (void)hipEventDestroy(e);
    if (hstream) (void)hipStreamSynchronize(hstream);
    if (hstream) (void)hipStreamDestroy(hstream);
    if (ostream) (void)hipStreamDestroy(ostream);
    if (stream) (void)hipStreamDestroy(stream);
  }
};

static int make_devcfg(const lego_sensor_cfg* c, const lego_ctx_opts& o, DevCfg* d) {
  if (c->n_scan <= 0 || c->n_scan > kMaxRings || c->horizon_scan <= 0 ||
      c->horizon_scan > kMaxHorizon || c->ground_scan_ind < 0 || c->ground_scan_ind >= c->n_scan)
    return LEGO_E_ARG;
  if (!c->use_cloud_ring && !(c->ang_res_y > 0.0f && std::isfinite(c->ang_bottom)))
    return LEGO_E_ARG;  // the vertical-angle row needs a positive resolution
  d->N = c->n_scan;
  d->H = c->horizon_scan;
  d->P = c->n_scan * c->horizon_scan;
  d->g = c->ground_scan_ind;
  d->ang_res_x = c->ang_res_x;
  d->min_range = c->sensor_minimum_range;
  d->mount_angle = c->sensor_mount_angle;
  d->theta = c->segment_theta;
  const TanBand tb = seg_tan_band_host(d->theta);  // seg_edge_fast's quotient band (lego_seg.h)
  d->tanLo = tb.lo;
  d->tanHi = tb.hi;
  d->quad1 = tb.quad1 ? 1 : 0;
  d->segHbm = o.seg_hbm ? 1 : 0;  // diagnostic: the k_seg_lds cross-check
  // labelComponents re-evaluates sin/cos(alpha) per edge (imageProjection.cpp:421);
  // they are per-sensor constants, evaluated with the same libm restatement.
  d->sinAX = lego_sinf(c->segment_alpha_x);
  d->cosAX = lego_cosf(c->segment_alpha_x);
  d->sinAY = lego_sinf(c->segment_alpha_y);
  d->cosAY = lego_cosf(c->segment_alpha_y);
  d->valid_pt = c->segment_valid_point_num;
  d->valid_line = c->segment_valid_line_num;
  d->edge_thr = c->edge_threshold;
  d->surf_thr = c->surf_threshold;
  d->nn_sq = c->nearest_feature_search_sq_dist;
  d->scan_period = c->scan_period;
  d->skip = c->skip_frame_num;
  d->ringRow = c->use_cloud_ring ? 1 : 0;
  d->ang_res_y = c->ang_res_y;
  d->ang_bottom = c->ang_bottom;
  return LEGO_OK;
}

// Back to construction state.  The device state is reset in stream order —
// the odometry state on the odometry stream, the FA carry on the extraction
// stream — so batches already submitted finish with the old state and the
// next one starts fresh (from a constant pinned image).
static int ctx_reset(lego_ctx* x) {
  ++x->devGen;
  x->needReset = false;
  HIPCHK(hipMemcpyAsync(x->ob.st, x->h_resetSt, sizeof(OdomState) * x->nStreams, hipMemcpyHostToDevice,
                        x->ostream));
  // the hand-off tags restart with the state: no granule of the old stream may match
  HIPCHK(hipMemsetAsync(x->ob.xh, 0, x->ob.xhBytes, x->ostream));
  HIPCHK(hipMemcpyAsync(x->d_carry, x->h_resetCarry, sizeof(FaCarry) * x->nStreams, hipMemcpyHostToDevice,
                        x->stream));
  // the next batch's odometry must also follow the reset of its own stream's
  // carry: it already waits for that batch's extraction (faDone)
  x->lastIpDevice = false;
  x->lastB = 0;
  x->lastBatch = false;
  x->faImu = FaImuQueue{};
  x->moImu = MoImuQueue{};
  x->fusion = Fusion{};
  if (x->moAlloc) {
    HIPCHK(hipMemsetAsync(x->mo.st, 0, sizeof(MoState), x->stream));
    if (x->mo.kf.kcap) {
      HIPCHK(hipMemsetAsync(x->mo.kf.meta, 0, sizeof(int) * kKfMeta, x->stream));
      HIPCHK(hipMemsetAsync(x->mo.kf.robot, 0, sizeof(float) * 8, x->stream));
    }
    HIPCHK(hipStreamSynchronize(x->stream));
  }
  x->moTimeLast = -1;
  x->moStoreFull = false;
  x->moTimeOdom = 0;
  x->pg.clear();
  x->recent.clear();
  x->latestFrameID = 0;
  x->aLoopIsClosed = false;
  std::memset(x->transformLast, 0, sizeof(x->transformLast));
  x->kfPose.clear();
  x->kfSeg.clear();
  return LEGO_OK;
}

extern "C" {

const char* lego_last_error(void) { return g_err; }

void lego_ctx_opts_init(lego_ctx_opts* o) {
  if (!o) return;
  std::memset(o, 0, sizeof(*o));
  o->size = (int32_t)sizeof(*o);
  o->node_overlap = 1;
  o->front_parts = 2;  // profiles/r05_ab_front_parts.txt
  o->lfv_wave = 1;
  o->lfv_block_rings = 0;
  o->lfv_wide = -1;
  o->ccl_tiles = 1;
  o->seg_hbm = 0;
  o->odom_workgroups = 0;
  o->odom_gridless = -1;
  o->odom_integ = -1;
  o->odom_silent_wg = -1;
  o->odom_late_wg = -1;
  o->lf_wait_ms = 2000;
  o->mo_cand_cache = 1;
  o->kf_cap = 0;
  o->vg_rounds = -1;
  o->ip_fused = 1;
}

int lego_sensor_preset(const char* name, lego_sensor_cfg* o) {
  if (!name || !o) return LEGO_E_ARG;
  std::memset(o, 0, sizeof(*o));
  if (!std::strcmp(name, "VLP-16")) {  // utility.h:63-68
    o->n_scan = 16; o->horizon_scan = 1800; o->ang_res_x = 0.2f; o->ang_res_y = 2.0f;
    o->ang_bottom = (float)(15.0 + 0.1); o->ground_scan_ind = 7;
  } else if (!std::strcmp(name, "HDL-32E")) {  // utility.h:71-76
    o->n_scan = 32; o->horizon_scan = 1800; o->ang_res_x = (float)(360.0 / (float)1800);
    o->ang_res_y = (float)(41.33 / (float)(32 - 1)); o->ang_bottom = 30.67f; o->ground_scan_ind = 20;
  } else if (!std::strcmp(name, "VLS-128")) {  // utility.h:79-84
    o->n_scan = 128; o->horizon_scan = 1800; o->ang_res_x = 0.2f; o->ang_res_y = 0.3f;
    o->ang_bottom = 25.0f; o->ground_scan_ind = 10;
  } else if (!std::strcmp(name, "OS1-16")) {  // utility.h:89-94
    o->n_scan = 16; o->horizon_scan = 1024; o->ang_res_x = (float)(360.0 / (float)1024);
    o->ang_res_y = (float)(33.2 / (float)(16 - 1)); o->ang_bottom = (float)(16.6 + 0.1);
    o->ground_scan_ind = 7;
  } else if (!std::strcmp(name, "OS1-64")) {  // utility.h:97-102
    o->n_scan = 64; o->horizon_scan = 1024; o->ang_res_x = (float)(360.0 / (float)1024);
    o->ang_res_y = (float)(33.2 / (float)(64 - 1)); o->ang_bottom = (float)(16.6 + 0.1);
    o->ground_scan_ind = 15;
  } else if (!std::strcmp(name, "HDL-64E")) {  // KITTI-shaped, DESIGN.md §2
    o->n_scan = 64; o->horizon_scan = 2048; o->ang_res_x = (float)(360.0 / (float)2048);
    o->ang_res_y = (float)(26.8 / (float)(64 - 1)); o->ang_bottom = 24.8f;
    o->ground_scan_ind = 55;
  } else {
    return LEGO_E_ARG;
  }
  o->use_cloud_ring = 1;
  o->sensor_minimum_range = 1.0f;
  o->sensor_mount_angle = 0.0f;
  o->segment_theta = (float)(60.0 / 180.0 * M_PI);
  o->segment_valid_point_num = 5;
  o->segment_valid_line_num = 3;
  o->segment_alpha_x = (float)(o->ang_res_x / 180.0 * M_PI);
  o->segment_alpha_y = (float)(o->ang_res_y / 180.0 * M_PI);
  o->edge_threshold = 0.1f;
  o->surf_threshold = 0.1f;
  o->nearest_feature_search_sq_dist = 25.f;
  o->scan_period = 0.1f;
  o->mapping_process_interval = 0.3;
  o->surrounding_keyframe_search_radius = 50.0f;
  o->skip_frame_num = 1;
  return LEGO_OK;
}

static int create_ctx(const lego_sensor_cfg* cfg, int device, int32_t n_streams, int32_t max_points,
                      int32_t max_batch, const lego_ctx_opts* optsIn, lego_ctx** out) {
  if (!cfg || !out || max_points <= 0 || max_batch <= 0 || n_streams <= 0) return LEGO_E_ARG;
  lego_ctx_opts opts;
  lego_ctx_opts_init(&opts);
  if (optsIn) {
    if (optsIn->size != (int32_t)sizeof(lego_ctx_opts)) {
      set_err("lego_ctx_opts.size %d != %d (lego_ctx_opts_init first)", optsIn->size, (int)sizeof(lego_ctx_opts));
      return LEGO_E_ARG;
    }
    opts = *optsIn;
  }
  if (opts.front_parts < 1 || opts.lf_wait_ms < 0) {
    set_err("lego_ctx_opts: front_parts >= 1 and lf_wait_ms >= 0");
    return LEGO_E_ARG;
  }
  DevCfg dc;
  if (make_devcfg(cfg, opts, &dc) != LEGO_OK) {
    set_err("unsupported sensor configuration");
    return LEGO_E_ARG;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= device || device < 0) {
    set_err("no HIP device %d (count %d)", device, ndev);
    return LEGO_E_DEVICE;
  }
  lego_ctx* x = new (std::nothrow) lego_ctx;
  if (!x) return LEGO_E_CAPACITY;
  x->cfg = *cfg;
  x->dc = dc;
  x->opts = opts;
  x->lo.cclTiles = opts.ccl_tiles;
  x->lo.lfvWave = opts.lfv_wave;
  x->lo.lfvBlockRings = opts.lfv_block_rings;
  x->lo.lfvWide = opts.lfv_wide;
  x->lo.faSyncCheck = opts.fa_synccheck;
  x->lo.ipFused = opts.ip_fused;
  x->vgApi.rounds = opts.vg_rounds;
  x->mo.hostprof = opts.mo_hostprof != 0;
  x->mo.evprof = opts.mo_evprof != 0;
  for (VgScratch* v : {&x->mo.vg, &x->mo.vgMap2, &x->mo.vgScan1, &x->mo.vgScan2}) v->rounds = opts.vg_rounds;
  x->device = device;
  x->maxPoints = max_points;
  x->maxBatch = max_batch;
  x->nStreams = n_streams;
  auto fail = [&](int st) { delete x; return st; };
  if (hipSetDevice(device) != hipSuccess) return fail(LEGO_E_DEVICE);
  if (hipStreamCreateWithFlags(&x->stream, hipStreamNonBlocking) != hipSuccess) return fail(LEGO_E_DEVICE);
  if (hipStreamCreateWithFlags(&x->ostream, hipStreamNonBlocking) != hipSuccess) return fail(LEGO_E_DEVICE);
  if (hipEventCreateWithFlags(&x->oJoin, hipEventDisableTiming) != hipSuccess) return fail(LEGO_E_DEVICE);
  if (hipEventCreateWithFlags(&x->lfFork, hipEventDisableTiming) != hipSuccess) return fail(LEGO_E_DEVICE);
  for (int i = 0; i < 2; ++i)
    if (hipEventCreateWithFlags(&x->faDone[i], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&x->recsDone[i], hipEventDisableTiming) != hipSuccess)
      return fail(LEGO_E_DEVICE);
  // B: per-scan slots (two batches); input staging is one batch
  const size_t B = 2 * (size_t)max_batch, B1 = max_batch, P = dc.P, N = dc.N;
  BatchBufs& bb = x->bb;
  bb.B = max_batch;
  bb.Nmax = max_points;
#define A(ptr, n)                                           \
  if (x->alloc(&(ptr), (n)) != hipSuccess) {                \
    set_err("hipMalloc failed for %s", #ptr);               \
    return fail(LEGO_E_DEVICE);                             \
  }
  A(x->d_pts, B1 * max_points);
  A(x->d_off, B1 + 1);
  A(bb.owner, B * P);
  if (hipMemset(bb.owner, 0xff, sizeof(int) * (size_t)B * P) != hipSuccess) {  // -1: no owner (k_pixels keeps it so)
    set_err("hipMemset failed for the owner image");
    return fail(LEGO_E_DEVICE);
  }
  A(bb.range, B * P);
  A(bb.full, B * P);
  A(bb.ground, B * P);
  A(bb.label, B * P);
  A(bb.parent, B * P);
  A(bb.root, B * P);
  A(bb.edges, B * P);
  A(bb.csize, B * P);
  A(bb.rowmask, B * P * 2);
  A(bb.rawang, B * 2);
  A(bb.bad, B);
  A(bb.seg, B * P);
  A(bb.gflag, B * P);
  A(bb.col, B * P);
  A(bb.srange, B * P);
  A(bb.outl, B * P);
  A(bb.ns, B);
  A(bb.nout, B);
  A(bb.sri, B * N);
  A(bb.eri, B * N);
  A(bb.orient, B * 3);
  A(bb.firsthalf, B);
  A(bb.dsk, B * P);
  A(bb.curv, B * P);
  A(bb.pick0, B * P);
  A(bb.r_sharp, B * N * kSharpPerRing);
  A(bb.r_lsharp, B * N * kLessSharpPerRing);
  A(bb.r_flat, B * N * kFlatPerRing);
  A(bb.r_lflat, B * P);
  A(bb.r_cnt, B * N * 4);
  A(bb.spec_out, B);
  A(bb.fa_flags, B);
  A(bb.f_sharp, B * N * kSharpPerRing);
  A(bb.f_lsharp, B * N * kLessSharpPerRing);
  A(bb.f_flat, B * N * kFlatPerRing);
  A(bb.f_lflat, B * P);
  A(bb.f_cnt, B * 4);
  A(x->d_lfReady, 1);
  A(bb.imuScan, B);
  A(x->d_desc, B);
  if (hipHostMalloc(&x->h_pack, sizeof(PackedRec) * 2 * (B1 + 1), hipHostMallocMapped | hipHostMallocCoherent) !=
          hipSuccess ||
      hipHostGetDevicePointer((void**)&x->d_pack, x->h_pack, 0) != hipSuccess) {
    if (x->h_pack) (void)hipHostFree(x->h_pack);
    x->h_pack = nullptr;
    set_err("hipHostMalloc failed for the record buffer");
    return fail(LEGO_E_DEVICE);
  }
  if (hipHostMalloc(&x->h_offp, sizeof(int64_t) * (B1 + 1), hipHostMallocDefault) != hipSuccess) {
    x->h_offp = nullptr;
    set_err("hipHostMalloc failed for the offsets buffer");
    return fail(LEGO_E_DEVICE);
  }
  A(x->d_imu, B1);
  bb.imu = nullptr;
  OdomBufs& ob = x->ob;
  ob.capLS = (int)(N * kLessSharpPerRing);
  ob.capCorner = ob.capLS;
  ob.capSurf = (int)P;
  if (ob.capSurf >= (1 << 21) - 1 || ob.capCorner >= (1 << 21) - 1) {  // the NN exchange's 21-bit indices
    set_err("max_points too large for the odometry exchange (< 2097151 points per scan)");
    return fail(LEGO_E_ARG);
  }
  const size_t S = n_streams;
  ob.S = n_streams;
  A(ob.st, S);
  A(ob.stIn, S);
  {
    // workgroups of the odometry launch
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) cus = 1;
    x->cus = cus;
    ob.G = odom_workgroups((int)N, cus);
    // a fleet's streams share the device: S x G workgroups, all resident
    if (n_streams > 1) ob.G = std::max(1, std::min(ob.G, cus / n_streams));
    // override (profiling / scaling studies); at most one workgroup per CU
    // over the fleet's streams
    if (const int g = opts.odom_workgroups; g >= 1 && (long)g * (long)n_streams <= (long)cus) ob.G = g;
    // without grids an NN round's wave searches its query's whole LDS cloud:
    // worth it when that is about one query per wave (the grids' build is on
    // every scan's chain); a fleet's few workgroups per stream keep them
    ob.gridless = ob.G >= kGridlessMinWG ? 1 : 0;
    if (opts.odom_gridless >= 0) ob.gridless = opts.odom_gridless ? 1 : 0;  // diagnostic
    ob.wg = S == 1 && opts.odom_silent_wg >= 0 ? opts.odom_silent_wg : -1;
    ob.late = S == 1 && opts.odom_late_wg >= 0 ? opts.odom_late_wg : -1;
    const int copies = ob.wg >= 0 ? 2 : 1;  // exchange copies (OdomBufs::wg)
    const size_t G = S * ob.G;  // private copies over all streams' workgroups
    for (int k = 0; k < 2; ++k) {
      A(ob.cornerLast[k], G * ob.capCorner);
      A(ob.surfLast[k], G * ob.capSurf);
    }
    int gTC = 0, gTS = 0;
    odom_index_caps(ob.capCorner, ob.capSurf, &gTC, &gTS);
    ob.gTC = gTC;
    ob.gTS = gTS;
    A(ob.nC.gPts, G * ob.capCorner);
    A(ob.nS.gPts, G * ob.capSurf);
    ob.capH = ob.capSurf + ob.capCorner;
    ob.ring = nullptr;
    ob.ringR = 0;
    ob.ringStride = ob.ringCtl = ob.ringCopy = 0;
    if (odom_ring_sensor((int)N)) {  // one copy of the last clouds and grids per stream (OdomBufs::ring)
      ob.ringR = ring_slots((int)((B1 + S - 1) / S));
      ob.ringStride = ring_stride(ob.G, gTS, gTC, ob.capH);
      ob.ringCtl = ring_ctl_bytes(ob.G, gTS, gTC);
      const size_t ringCopies = ob.wg >= 0 ? 2 : 1;
      ob.ringCopy = ringCopies > 1 ? (size_t)ob.ringR * ob.ringStride : 0;
      A(ob.ring, S * ringCopies * (size_t)ob.ringR * ob.ringStride);
    }
    ob.capQ = (int)(N * kFlatPerRing);
    A(ob.qi, G * 3 * ob.capQ);
    // exchange block: 16-byte error word, then per stream one slot of capQ
    // granules per NN round a launch can run (10 per scan)
    ob.roundsCap = 10 * (int)((B1 + S - 1) / S);
    const size_t xslots = S * (size_t)ob.roundsCap * (size_t)ob.capQ;
    ob.xbytes = 16 + copies * sizeof(unsigned long long) * xslots;
    unsigned char* xb = nullptr;
    A(xb, ob.xbytes);
    ob.xblock = xb;
    ob.xerr = (unsigned*)xb;
    ob.xg = (unsigned long long*)(xb + 16);
    ob.capH = ob.capSurf + ob.capCorner;
    const size_t hslots = S * 2 * 3 * (size_t)ob.capH;
    ob.xhBytes = copies * sizeof(unsigned long long) * hslots;
    unsigned char* hb = nullptr;
    A(hb, ob.xhBytes);
    ob.xh = (unsigned long long*)hb;
    if (hipMemset(ob.xh, 0, ob.xhBytes) != hipSuccess) {
      set_err("hipMemset failed for the hand-off exchange");
      return fail(LEGO_E_DEVICE);
    }
    {  // header: the error word, then the silent workgroup's copy distances
      const unsigned hdr[4] = {0u, 0u, copies > 1 ? (unsigned)xslots : 0u, copies > 1 ? (unsigned)hslots : 0u};
      if (hipMemcpy(xb, hdr, sizeof(hdr), hipMemcpyHostToDevice) != hipSuccess) {
        set_err("hipMemcpy failed for the exchange header");
        return fail(LEGO_E_DEVICE);
      }
    }
  }
  A(ob.sumOut, B * 6);
  A(ob.intX, B * 6);
  ob.integ = ob.G > 1 ? 1 : 0;  // integration on its own workgroup per stream (OdomBufs::integ)
  if (opts.odom_integ >= 0) ob.integ = ob.G > 1 && opts.odom_integ != 0;  // diagnostic A/B
  A(ob.curOut, B * 6);
  A(ob.validOut, B);
  A(ob.pubOut, B);
  A(ob.cornerEnd, B * ob.capLS);
  A(ob.surfEnd, B * P);
  A(x->d_carry, S);
  if (hipHostMalloc(&x->h_resetSt, sizeof(OdomState) * S, hipHostMallocDefault) != hipSuccess ||
      hipHostMalloc(&x->h_resetCarry, sizeof(FaCarry) * S, hipHostMallocDefault) != hipSuccess) {
    set_err("hipHostMalloc failed for the reset image");
    return fail(LEGO_E_DEVICE);
  }
  for (size_t i = 0; i < S; ++i) {
    std::memset(&x->h_resetSt[i], 0, sizeof(OdomState));
    x->h_resetSt[i].frameCount = cfg->skip_frame_num;  // frameCount = skipFrameNum (:314)
    x->h_resetCarry[i] = FaCarry{};  // fresh member arrays: phantom {0.0f, 0}, picked[0] = 0
  }
  A(x->d_prof, 48);  // [0, 32) k_odom phases, [32, 40) k_extract phases, [40] its in-flight counter
#undef A
  bb.pts = x->d_pts;
  bb.off = x->d_off;
  {  // the pinned host staging block and its regions (256-byte aligned)
    size_t at = 0;
    std::vector<std::pair<void**, size_t>> reg;
    auto R = [&](auto** ptr, size_t bytes) { reg.push_back({(void**)ptr, at}); at += (bytes + 255) & ~(size_t)255; };
    const size_t P16 = sizeof(lego_point_xyzi) * P;
    R(&x->h_hdr, sizeof(int32_t) * kFetchHdr);
    R(&x->h_moRes, kMoResBytes);
    R(&x->h_seg, P16); R(&x->h_outl, P16); R(&x->h_full, P16); R(&x->h_lflat, P16);
    R(&x->h_surfLast, P16); R(&x->h_outlLast, P16); R(&x->h_info, P16); R(&x->h_gcloud, P16); R(&x->h_pure, P16);
    R(&x->h_sharp, sizeof(lego_point_xyzi) * N * kSharpPerRing);
    R(&x->h_lsharp, sizeof(lego_point_xyzi) * N * kLessSharpPerRing);
    R(&x->h_cornerLast, sizeof(lego_point_xyzi) * N * kLessSharpPerRing);
    R(&x->h_flat, sizeof(lego_point_xyzi) * N * kFlatPerRing);
    R(&x->h_sri, sizeof(int32_t) * N); R(&x->h_eri, sizeof(int32_t) * N);
    R(&x->h_label, sizeof(int32_t) * P); R(&x->h_col, sizeof(uint32_t) * P);
    R(&x->h_range, sizeof(float) * P); R(&x->h_rimg, sizeof(float) * P);
    R(&x->h_gflag, P); R(&x->h_gimg, P);
    R(&x->h_bad, sizeof(int32_t) * (size_t)x->maxBatch);
    if (hipHostMalloc((void**)&x->hostBlock, at, hipHostMallocDefault) != hipSuccess) {
      set_err("hipHostMalloc failed for the host staging block (%zu bytes)", at);
      return fail(LEGO_E_DEVICE);
    }
    for (auto& r : reg) *r.first = x->hostBlock + r.second;
  }
  int st = ctx_reset(x);
  if (st != LEGO_OK) return fail(st);
  *out = x;
  return LEGO_OK;
}

int lego_create_ex(const lego_sensor_cfg* cfg, int device, int32_t max_points, int32_t max_batch,
                   const lego_ctx_opts* opts, lego_ctx** out) {
  return create_ctx(cfg, device, 1, max_points, max_batch, opts, out);
}

int lego_create(const lego_sensor_cfg* cfg, int device, int32_t max_points, int32_t max_batch,
                lego_ctx** out) {
  return create_ctx(cfg, device, 1, max_points, max_batch, nullptr, out);
}

int lego_fleet_create_ex(const lego_sensor_cfg* cfg, int device, int32_t n_streams, int32_t max_points,
                         int32_t scans_per_stream, const lego_ctx_opts* opts, lego_ctx** out) {
  if (n_streams <= 0 || scans_per_stream <= 0 || (int64_t)n_streams * scans_per_stream > (1 << 24))
    return LEGO_E_ARG;
  return create_ctx(cfg, device, n_streams, max_points, n_streams * scans_per_stream, opts, out);
}

int lego_fleet_create(const lego_sensor_cfg* cfg, int device, int32_t n_streams, int32_t max_points,
                      int32_t scans_per_stream, lego_ctx** out) {
  return lego_fleet_create_ex(cfg, device, n_streams, max_points, scans_per_stream, nullptr, out);
}

int lego_destroy(lego_ctx* x) {
  delete x;
  return LEGO_OK;
}

int lego_reset(lego_ctx* x) {
  if (!x) return LEGO_E_ARG;
  HIPCHK(hipSetDevice(x->device));
  return ctx_reset(x);
}

// Delivers /imu_raw messages to both nodes' queues (host imuHandlers).
static void imu_deliver(lego_ctx* x, const lego_imu_msg* m, int n) {
  for (int i = 0; i < n; ++i) {
    x->faImu.push(m[i], x->cfg.scan_period);
    x->moImu.push(m[i]);
  }
}

// The featureAssociation queue of scans 0..B-1 (x->stamps): messages
// imu[0 .. before[k]) are delivered before scan k, the rest after the last
// scan.  Returns the device snapshots, or null while the stream has never
// received a message (adjustDistortion's imuPointerLast < 0 branch).
static int imu_stage(lego_ctx* x, int B, const lego_imu_msg* imu, int n_imu, const int32_t* before,
                     const ImuSnap** out) {
  *out = nullptr;
  const bool any = x->faImu.last >= 0 || (n_imu > 0 && before && before[B - 1] > 0);
  if (!any) {  // adjustDistortion still ends with imuPointerLastIteration = imuPointerLast (-1)
    x->faImu.lastIter = x->faImu.last;
    imu_deliver(x, imu, n_imu);
    return LEGO_OK;
  }
  x->h_imu.resize(B);
  int j = 0;
  for (int k = 0; k < B; ++k) {
    const int upto = before ? before[k] : 0;
    imu_deliver(x, imu + j, upto - j);
    j = upto;
    x->faImu.snapshot(x->stamps[k], &x->h_imu[k]);
  }
  imu_deliver(x, imu + j, n_imu - j);
  HIPCHK(hipMemcpyAsync(x->d_imu, x->h_imu.data(), sizeof(ImuSnap) * B, hipMemcpyHostToDevice, x->stream));
  *out = x->d_imu;
  return LEGO_OK;
}

// ---------------------------------------------------------------- batch slots
// The per-scan device views of scan slots [c0, c0 + n).
static BatchBufs bb_slice(const BatchBufs& a, const DevCfg& c, int c0, int n) {
  BatchBufs b = a;
  const size_t k = (size_t)c0, P = c.P, N = c.N;
  b.B = n;
  if (b.imu) b.imu += k;
  b.imuScan += k;
  b.off += k;
  b.owner += k * P; b.range += k * P; b.full += k * P; b.ground += k * P; b.label += k * P;
  b.parent += k * P; b.root += k * P; b.edges += k * P; b.csize += k * P;
  b.rowmask += k * P * 2; b.rawang += k * 2; b.bad += k;
  b.seg += k * P; b.gflag += k * P; b.col += k * P; b.srange += k * P; b.outl += k * P;
  b.ns += k; b.nout += k; b.sri += k * N; b.eri += k * N; b.orient += k * 3;
  b.firsthalf += k; b.dsk += k * P; b.curv += k * P; b.pick0 += k * P;
  b.r_sharp += k * N * kSharpPerRing; b.r_lsharp += k * N * kLessSharpPerRing;
  b.r_flat += k * N * kFlatPerRing; b.r_lflat += k * P; b.r_cnt += k * N * 4;
  b.spec_out += k; b.fa_flags += k;
  b.f_sharp += k * N * kSharpPerRing; b.f_lsharp += k * N * kLessSharpPerRing;
  b.f_flat += k * N * kFlatPerRing; b.f_lflat += k * P; b.f_cnt += k * 4;
  return b;
}

// The odometry view of streams [s0, s0 + S) whose scans are the slots from c0.
static OdomBufs ob_slice(const OdomBufs& a, const DevCfg& c, int c0, int s0, int S) {
  OdomBufs o = a;
  o.S = S;
  o.st += s0;
  o.stIn += s0;
  const size_t w = (size_t)s0 * a.G, k = (size_t)c0;
  for (int i = 0; i < 2; ++i) {
    o.cornerLast[i] += w * a.capCorner;
    o.surfLast[i] += w * a.capSurf;
  }
  o.nC.gPts += w * a.capCorner;
  o.nS.gPts += w * a.capSurf;
  o.qi += w * 3 * a.capQ;
  o.xg += (size_t)s0 * a.roundsCap * a.capQ;
  o.xh += (size_t)s0 * 2 * 3 * a.capH;
  if (a.ring) o.ring += (size_t)s0 * (a.ringCopy ? 2 : 1) * a.ringR * a.ringStride;
  o.sumOut += k * 6; o.curOut += k * 6; o.validOut += k; o.pubOut += k; o.intX += k * 6;
  o.cornerEnd += k * a.capLS; o.surfEnd += k * c.P;
  return o;
}

// Validates a batch and points bb (a slot view) at its input points: the
// caller's device arrays, or a copy of host arrays in the staging buffer.
// node: the caller synchronises before returning (run_ip), so the offsets may
// go through the pinned h_offp
static int stage_inputs(lego_ctx* x, const lego_point_xyzir* pts, const int64_t* offsets, int B,
                        int on_device, BatchBufs& bb, bool node = false, bool staged = false) {
  HIPCHK(hipSetDevice(x->device));
  // Per-scan sizes are validated on the host in both modes: an empty scan is
  // undefined upstream (findStartEndAngle reads points[0] and points[size-1],
  // imageProjection.cpp:201-203) and a scan above capacity would overrun the
  // per-point work buffers.
  std::vector<int64_t> off(B + 1);
  if (on_device) {
    HIPCHK(hipMemcpyAsync(x->h_offp, offsets, sizeof(int64_t) * (B + 1), hipMemcpyDeviceToHost, x->stream));
    HIPCHK(hipStreamSynchronize(x->stream));
    for (int k = 0; k <= B; ++k) off[k] = x->h_offp[k];
  } else {
    for (int k = 0; k <= B; ++k) off[k] = offsets[k];
  }
  int mx = 0;
  for (int k = 0; k < B; ++k) {
    const int64_t n = off[k + 1] - off[k];
    if (n <= 0) {
      set_err("scan %d of the batch is empty (offsets must be strictly increasing)", k);
      return LEGO_E_ARG;
    }
    if (n > x->maxPoints) {
      set_err("scan %d has %lld points > capacity %d", k, (long long)n, x->maxPoints);
      return LEGO_E_CAPACITY;
    }
    mx = std::max<int>(mx, (int)n);
  }
  if (on_device) {
    bb.pts = pts;
    bb.off = offsets;
  } else {
    const int64_t total = off[B] - off[0];
    if (total > (int64_t)x->maxPoints * x->maxBatch) return LEGO_E_CAPACITY;
    const int64_t base = off[0];
    for (int k = 0; k <= B; ++k) off[k] -= base;
    if (!staged)  // (staged: upload_checked already queued the points' copies on x->stream)
      HIPCHK(hipMemcpyAsync(x->d_pts, pts + base, sizeof(lego_point_xyzir) * total,
                            hipMemcpyHostToDevice, x->stream));
    if (node) {  // pinned: an asynchronous copy (a pageable source is a synchronous staged one)
      for (int k = 0; k <= B; ++k) x->h_offp[k] = off[k];
      HIPCHK(hipMemcpyAsync(x->d_off, x->h_offp, sizeof(int64_t) * (B + 1), hipMemcpyHostToDevice, x->stream));
    } else {
      HIPCHK(hipMemcpyAsync(x->d_off, off.data(), sizeof(int64_t) * (B + 1), hipMemcpyHostToDevice, x->stream));
    }
    // staged: the packed form (bit 0 of the pointer, pts_view in lego_ip.hip)
    bb.pts = staged ? (const void*)((uintptr_t)x->d_pts | 1) : (const void*)x->d_pts;
    bb.off = x->d_off;
  }
  bb.Nmax = mx;
  return LEGO_OK;
}

static int fetch_ip(lego_ctx* x, int k, bool images, lego_ip_out* o, bool gated = false, int badN = 0);

// Image projection only (lego_ip_process*): slot 0, synchronous; scan 0's
// outputs are fetched into *out with the batch's not-dense flags (one sync).
static int run_ip(lego_ctx* x, const lego_point_xyzir* pts, const int64_t* offsets, int B, int on_device,
                  bool images, lego_ip_out* out, bool gated = false, bool staged = false) {
  const int want_labels = images ? 1 : 0;
  if (x->inflight) {
    set_err("node-shaped call while batches are in flight (lego_odom_batch_wait first)");
    return LEGO_E_STATE;
  }
  BatchBufs bb = x->bb;
  int st = stage_inputs(x, pts, offsets, B, on_device, bb, true, staged);
  if (st != LEGO_OK) return st;
  // this launch writes slot 0 (the outlier cloud among it): a resident
  // hand-off of an earlier lego_fa_process is stale from here on
  // (lego_ip_process and lego_ip_process_pc2 alike).  A call
  // rejected above launched nothing and leaves it valid.
  ++x->devGen;
  x->lastBatch = false;
  if (!ip_clears_bad(x->dc, B, x->lo)) HIPCHK(hipMemsetAsync(bb.bad, 0, sizeof(int) * B, x->stream));
  if (gated && !x->gb.n) {
    const size_t P = x->dc.P;
#define MA(ptr, n) \
  if (x->alloc(&(ptr), (size_t)(n)) != hipSuccess) { set_err("hipMalloc failed for %s", #ptr); return LEGO_E_DEVICE; }
    MA(x->gb.info, P); MA(x->gb.ground, P); MA(x->gb.pure, P); MA(x->gb.n, 2);
#undef MA
  }
  x->tm.begin();
  launch_ip(bb, x->dc, B, want_labels || gated ? 1 : 0, x->stream, &x->tm, x->lo);
  if (gated) {
    x->tm.mark("ip.gated", x->stream);
    launch_gated(bb, x->dc, x->gb, x->stream);
  }
  x->tm.end(x->stream);
  HIPCHK(hipGetLastError());
  x->lastB = B;
  x->lastBase = 0;
  st = fetch_ip(x, 0, images, out, gated, B);
  if (st != LEGO_OK) return st;
  x->tnames.clear();
  x->tms.clear();
  std::vector<int> cnt;
  x->tm.collect(x->tnames, x->tms, cnt);
  for (int k = 0; k < B; ++k)
    if (x->h_bad[k] & kBadNotDense) {
      x->lastB = 0;
      set_err(x->dc.ringRow ? "scan %d of the batch has non-finite xyz (the cloud must be dense)"
                            : "scan %d of the batch has no finite point", k);
      return LEGO_E_NOT_DENSE;
    }
  return LEGO_OK;
}

// Parts of a fleet batch's front end (submit_batch): lego_ctx_opts::front_parts
// (default 2, profiles/r05_ab_front_parts.txt), at most kFrontPartsMax,
// reduced until it divides the streams.  A single stream is one part (its
// scans chain through the extraction's carry).
static int front_parts(const lego_ctx* x, int S) {
  int p = std::max(1, std::min(x->opts.front_parts, lego_ctx::kFrontPartsMax));
  while (S % p) --p;
  return p;
}

static int front_streams(lego_ctx* x, int parts) {
  HIPCHK(hipSetDevice(x->device));
  if (!x->fFork) HIPCHK(hipEventCreateWithFlags(&x->fFork, hipEventDisableTiming));
  for (int p = 1; p < parts; ++p) {
    if (!x->fstream[p - 1]) HIPCHK(hipStreamCreateWithFlags(&x->fstream[p - 1], hipStreamNonBlocking));
    if (!x->fJoin[p - 1]) HIPCHK(hipEventCreateWithFlags(&x->fJoin[p - 1], hipEventDisableTiming));
  }
  return LEGO_OK;
}

// Enqueues ip + fa + odometry for a batch (x->stamps) in the next slot and
// returns.  Projection and extraction run on x->stream, the odometry on
// x->ostream after them, so they overlap the previous batch's odometry.
static int submit_batch(lego_ctx* x, const lego_point_xyzir* pts, const int64_t* offsets, int B, int on_device,
                        const lego_imu_msg* imu, int n_imu, const int32_t* imu_before) {
  if (x->needReset) {
    set_err("an earlier odometry call failed on the device: lego_reset first");
    return LEGO_E_STATE;
  }
  ++x->devGen;
  if (x->inflight >= 2) {
    set_err("two batches in flight: lego_odom_batch_wait before submitting another");
    return LEGO_E_STATE;
  }
  const int h = x->nextSlot, base = h * x->maxBatch;
  // the waited batch in this slot is about to be overwritten: no hand-off of it after this
  if (x->lastBatch && x->lastBase == base) x->lastBatch = false;
  BatchBufs bb = bb_slice(x->bb, x->dc, base, B);
  int st = stage_inputs(x, pts, offsets, B, on_device, bb);
  if (st != LEGO_OK) return st;
  st = imu_stage(x, B, imu, n_imu, imu_before, &bb.imu);
  if (st != LEGO_OK) return st;
  const int S = x->nStreams;
  StageTimer& tm = x->stm[h];
  StageTimer& otm = x->sotm[h];
  tm.enabled = otm.enabled = x->tm.enabled;
  const int parts = front_parts(x, S);
  // k_ip_lds clears its scans' words itself: no fill queued behind the
  // previous batch's odometry, whose workgroups hold every CU's registers
  if (!ip_clears_bad(x->dc, B / parts, x->lo)) HIPCHK(hipMemsetAsync(bb.bad, 0, sizeof(int) * B, x->stream));
  bb.xprof = x->profOn ? x->d_prof + 32 : nullptr;
  tm.begin();
  otm.begin();
  // a fleet's streams are independent up to the odometry: their projection
  // and extraction in parts of whole streams (the batch is stream-major), on
  // HIP streams of their own, so that one part's LDS-bound kernels
  // (segmentation, VoxelGrids) share the CUs with another's HBM-bound ones
  if (parts > 1) {
    st = front_streams(x, parts);
    if (st != LEGO_OK) return st;
    HIPCHK(hipEventRecord(x->fFork, x->stream));
    for (int p = 1; p < parts; ++p) HIPCHK(hipStreamWaitEvent(x->fstream[p - 1], x->fFork, 0));
  }
  const int Sp = S / parts, Bp = B / parts;
  for (int p = 0; p < parts; ++p) {
    hipStream_t s = p ? x->fstream[p - 1] : x->stream;
    StageTimer* t = p ? &x->ftm : &tm;  // the stage times are part 0's
    BatchBufs q = parts > 1 ? bb_slice(bb, x->dc, p * Bp, Bp) : bb;
    if (p) q.xprof = nullptr;
    launch_ip(q, x->dc, Bp, 0, s, t, x->lo);
    launch_fa(q, x->dc, Bp, Sp, x->d_carry + p * Sp, s, t, x->lo);
  }
  for (int p = 1; p < parts; ++p) {
    HIPCHK(hipEventRecord(x->fJoin[p - 1], x->fstream[p - 1]));
    HIPCHK(hipStreamWaitEvent(x->stream, x->fJoin[p - 1], 0));
  }
  tm.end(x->stream);
  HIPCHK(hipEventRecord(x->faDone[h], x->stream));
  HIPCHK(hipStreamWaitEvent(x->ostream, x->faDone[h], 0));
  const OdomBufs ob = ob_slice(x->ob, x->dc, base, 0, S);  // launch_odom zeroes *ob.xerr
  if (launch_odom(bb, ob, x->dc, B / S, x->ostream, &otm, x->profOn ? x->d_prof : nullptr) != 0) {
    set_err("odometry launch failed (%d workgroups)", x->ob.G);
    return LEGO_E_DEVICE;
  }
  otm.end(x->ostream);
  // the batch's records, non-dense flags and the error word, written by the
  // kernel straight into the pinned (coherent, mapped) host slot
  launch_pack_recs(bb, ob, B, x->d_pack + (size_t)h * (x->maxBatch + 1), x->ostream);
  HIPCHK(hipEventRecord(x->recsDone[h], x->ostream));
  HIPCHK(hipGetLastError());
  x->slotB[h] = B;
  x->slotStamps[h] = x->stamps;
  if (x->inflight == 0) x->oldest = h;
  x->inflight++;
  x->nextSlot = h ^ 1;
  return LEGO_OK;
}

// Waits for the oldest batch in flight and writes its pose records.
static int wait_batch(lego_ctx* x, lego_pose_rec* recs, int cap, int* nOut) {
  if (!x->inflight) {
    set_err("no batch in flight");
    return LEGO_E_STATE;
  }
  const int h = x->oldest, B = x->slotB[h];
  HIPCHK(hipEventSynchronize(x->recsDone[h]));
  x->inflight--;
  x->oldest = h ^ 1;
  const PackedRec* pk = x->h_pack + (size_t)h * (x->maxBatch + 1);
  x->tnames.clear();
  x->tms.clear();
  std::vector<int> cnt;
  x->stm[h].collect(x->tnames, x->tms, cnt);
  x->sotm[h].collect(x->tnames, x->tms, cnt);
  for (size_t i = 0, m = x->tnames.size(); i < m; ++i) {  // launches per stage, as "n:<stage>"
    x->tnames.push_back("n:" + x->tnames[i]);
    x->tms.push_back((float)cnt[i]);
  }
  x->lastB = 0;
  x->lastBatch = false;
  if (pk[B].bad) {
    set_err("odometry error word %d (1: more NN rounds than slots, 2: a ring share never done, 3: the "
            "integration never saw a scan's transform)", pk[B].bad);
    return LEGO_E_DEVICE;
  }
  for (int k = 0; k < B; ++k)
    if (pk[k].bad & kBadNotDense) {
      set_err(x->dc.ringRow ? "scan %d of the batch has non-finite xyz (the cloud must be dense)"
                            : "scan %d of the batch has no finite point", k);
      return LEGO_E_NOT_DENSE;
    }
  for (int k = 0; k < B; ++k)
    if (pk[k].bad & kBadPermutation) {
      set_err("scan %d: per-ring VoxelGrid sort returned a payload outside its input (device fault)", k);
      return LEGO_E_DEVICE;
    }
  if (cap < B) {
    set_err("record buffer of %d < %d scans", cap, B);
    return LEGO_E_ARG;
  }
  const std::vector<double>& stamps = x->slotStamps[h];
  for (int k = 0; k < B; ++k) {
    const PackedRec& p = pk[k];
    lego_pose_rec& r = recs[k];
    std::memset(&r, 0, sizeof(r));
    r.stamp = k < (int)stamps.size() ? stamps[k] : 0.0;
    for (int i = 0; i < 6; ++i) r.transform_sum[i] = p.sum[i];
    r.n_segmented = p.ns;
    r.n_sharp = p.cnt[0];
    r.n_less_sharp = p.cnt[1];
    r.n_flat = p.cnt[2];
    r.n_less_flat = p.cnt[3];
    r.odom_valid = p.valid;
    r.flags = p.flags;
  }
  x->stamps = stamps;
  x->lastB = B;
  x->lastBase = h * x->maxBatch;
  x->lastBatch = true;
  if (nOut) *nOut = B;
  return LEGO_OK;
}

// ---------------------------------------------------------------- fetch
// One scan's host outputs in one launch: k_fetch copies every array of the
// list straight into the pinned staging block (the counts read on the device,
// so no round trip sizes the copies), then the caller synchronises once.
struct FetchItem {
  const void* src;
  void* dst;
  const int* cnt;  // element count on the device (nullptr: n)
  int n, elem, cap;  // elements, bytes per element, capacity of dst in elements
};
constexpr int kFetchItems = 24;
struct FetchList {
  FetchItem it[kFetchItems];
};
__global__ void __launch_bounds__(256) k_fetch(FetchList L) {
  const FetchItem f = L.it[blockIdx.y];
  int n = f.cnt ? *f.cnt : f.n;
  n = n < 0 ? 0 : (n > f.cap ? f.cap : n);
  const size_t bytes = (size_t)n * (size_t)f.elem;
  const unsigned char* src = (const unsigned char*)f.src;
  unsigned char* dst = (unsigned char*)f.dst;
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x, T = (size_t)gridDim.x * blockDim.x;
  const uintptr_t al = (uintptr_t)src | (uintptr_t)dst;
  size_t done = 0;
  if ((al & 15) == 0) {
    const size_t v = bytes / 16;
    for (size_t i = t; i < v; i += T) ((uint4*)dst)[i] = ((const uint4*)src)[i];
    done = v * 16;
  } else if ((al & 3) == 0) {
    const size_t v = bytes / 4;
    for (size_t i = t; i < v; i += T) ((uint32_t*)dst)[i] = ((const uint32_t*)src)[i];
    done = v * 4;
  }
  for (size_t i = done + t; i < bytes; i += T) dst[i] = src[i];
}
struct FetchBuilder {
  FetchList L{};
  int n = 0;
  void add(const void* src, void* dst, const int* cnt, size_t num, int elem, size_t cap) {
    L.it[n++] = FetchItem{src, dst, cnt, (int)num, elem, (int)cap};
  }
  hipError_t run(hipStream_t s) {
    k_fetch<<<dim3(8, n), 256, 0, s>>>(L);
    const hipError_t e = hipGetLastError();
    return e != hipSuccess ? e : hipStreamSynchronize(s);
  }
};
// header words of h_hdr
enum { FH_NS = 0, FH_NOUT = 1, FH_ORIENT = 2, FH_NG = 5, FH_CNT = 8, FH_VALID = 12, FH_PUB = 13, FH_FNOUT = 14,
       FH_SUM = 16, FH_CUR = 22, FH_XERR = 28, FH_BAD = 29 };

// copy scan k's image-projection outputs of the last batch into host staging
// (badN: also the first badN not-dense flags into h_bad)
static int fetch_ip(lego_ctx* x, int k, bool images, lego_ip_out* o, bool gated, int badN) {
  const DevCfg& c = x->dc;
  const size_t P = c.P, N = c.N;
  const BatchBufs& bb = x->bb;
  int32_t* hd = x->h_hdr;
  FetchBuilder F;
  F.add(bb.ns + k, hd + FH_NS, nullptr, 1, 4, 1);
  F.add(bb.nout + k, hd + FH_NOUT, nullptr, 1, 4, 1);
  F.add(bb.orient + 3 * k, hd + FH_ORIENT, nullptr, 3, 4, 3);
  F.add(bb.sri + k * N, x->h_sri, nullptr, N, 4, N);
  F.add(bb.eri + k * N, x->h_eri, nullptr, N, 4, N);
  F.add(bb.seg + k * P, x->h_seg, bb.ns + k, 0, 16, P);
  F.add(bb.gflag + k * P, x->h_gflag, bb.ns + k, 0, 1, P);
  F.add(bb.col + k * P, x->h_col, bb.ns + k, 0, 4, P);
  F.add(bb.srange + k * P, x->h_range, bb.ns + k, 0, 4, P);
  F.add(bb.outl + k * P, x->h_outl, bb.nout + k, 0, 16, P);
  if (gated) {  // scan 0 of a node-shaped call
    F.add(x->gb.n, hd + FH_NG, nullptr, 2, 4, 2);
    F.add(x->gb.info, x->h_info, nullptr, P, 16, P);
    F.add(x->gb.ground, x->h_gcloud, x->gb.n, 0, 16, P);
    F.add(x->gb.pure, x->h_pure, x->gb.n + 1, 0, 16, P);
  }
  if (images) {
    F.add(bb.full + k * P, x->h_full, nullptr, P, 16, P);
    F.add(bb.range + k * P, x->h_rimg, nullptr, P, 4, P);
    F.add(bb.ground + k * P, x->h_gimg, nullptr, P, 1, P);
    F.add(bb.label + k * P, x->h_label, nullptr, P, 4, P);
  }
  if (badN > 0) F.add(bb.bad, x->h_bad, nullptr, badN, 4, x->maxBatch);
  HIPCHK(F.run(x->stream));
  const int ns = hd[FH_NS], nout = hd[FH_NOUT];
  float orient[3];
  std::memcpy(orient, hd + FH_ORIENT, sizeof(orient));
  std::memset(o, 0, sizeof(*o));
  const int kr = k - x->lastBase;  // index within the batch
  o->info.stamp = (kr < (int)x->stamps.size()) ? x->stamps[kr] : 0.0;
  o->info.start_ring_index = x->h_sri;
  o->info.end_ring_index = x->h_eri;
  o->info.start_orientation = orient[0];
  o->info.end_orientation = orient[1];
  o->info.orientation_diff = orient[2];
  o->info.segmented_cloud_ground_flag = x->h_gflag;
  o->info.segmented_cloud_col_ind = x->h_col;
  o->info.segmented_cloud_range = x->h_range;
  o->segmented_cloud = x->h_seg;
  o->n_segmented = ns;
  o->outlier_cloud = x->h_outl;
  o->n_outlier = nout;
  if (images) {
    o->full_cloud = x->h_full;
    o->range_image = x->h_rimg;
    o->ground_image = x->h_gimg;
    o->label_image = x->h_label;
  }
  if (gated) {
    o->full_info_cloud = x->h_info;
    o->ground_cloud = x->h_gcloud;
    o->n_ground = hd[FH_NG];
    o->segmented_cloud_pure = x->h_pure;
    o->n_segmented_pure = hd[FH_NG + 1];
  }
  return LEGO_OK;
}

// scan k's extraction + odometry outputs; withXerr: also the batch's exchange
// error word (h_hdr[FH_XERR], lego_fa_process)
static int fetch_fa(lego_ctx* x, int k, lego_fa_out* o, bool withXerr = false) {
  const DevCfg& c = x->dc;
  const size_t P = c.P, N = c.N;
  const BatchBufs& bb = x->bb;
  int32_t* hd = x->h_hdr;
  const int* fc = bb.f_cnt + 4 * k;
  FetchBuilder F;
  F.add(fc, hd + FH_CNT, nullptr, 4, 4, 4);
  F.add(x->ob.validOut + k, hd + FH_VALID, nullptr, 1, 4, 1);
  F.add(x->ob.pubOut + k, hd + FH_PUB, nullptr, 1, 4, 1);
  F.add(bb.nout + k, hd + FH_FNOUT, nullptr, 1, 4, 1);
  F.add(x->ob.sumOut + 6 * k, hd + FH_SUM, nullptr, 6, 4, 6);
  F.add(x->ob.curOut + 6 * k, hd + FH_CUR, nullptr, 6, 4, 6);
  if (withXerr) {
    F.add(x->ob.xerr, hd + FH_XERR, nullptr, 1, 4, 1);
    F.add(bb.bad + k, hd + FH_BAD, nullptr, 1, 4, 1);
  }
  F.add(bb.f_sharp + k * N * kSharpPerRing, x->h_sharp, fc + 0, 0, 16, N * kSharpPerRing);
  F.add(bb.f_lsharp + k * N * kLessSharpPerRing, x->h_lsharp, fc + 1, 0, 16, N * kLessSharpPerRing);
  F.add(bb.f_flat + k * N * kFlatPerRing, x->h_flat, fc + 2, 0, 16, N * kFlatPerRing);
  F.add(bb.f_lflat + k * P, x->h_lflat, fc + 3, 0, 16, P);
  F.add(x->ob.cornerEnd + (size_t)k * x->ob.capLS, x->h_cornerLast, fc + 1, 0, 16, N * kLessSharpPerRing);
  F.add(x->ob.surfEnd + k * P, x->h_surfLast, fc + 3, 0, 16, P);
  F.add(bb.outl + k * P, x->h_outlLast, bb.nout + k, 0, 16, P);
  HIPCHK(F.run(x->stream));
  int cnt[4];
  float sum[6], cur[6];
  std::memcpy(cnt, hd + FH_CNT, sizeof(cnt));
  std::memcpy(sum, hd + FH_SUM, sizeof(sum));
  std::memcpy(cur, hd + FH_CUR, sizeof(cur));
  const int valid = hd[FH_VALID], pub = hd[FH_PUB], nout = hd[FH_FNOUT];
  // adjustOutlierCloud :1746-1757 (axis swap) on the published copy
  for (int i = 0; i < nout; ++i) {
    const lego_point_xyzi p = x->h_outlLast[i];
    x->h_outlLast[i] = {p.y, p.z, p.x, p.intensity};
  }
  std::memset(o, 0, sizeof(*o));
  const int kr = k - x->lastBase;
  o->stamp = (kr < (int)x->stamps.size()) ? x->stamps[kr] : 0.0;
  o->sharp = x->h_sharp; o->n_sharp = cnt[0];
  o->less_sharp = x->h_lsharp; o->n_less_sharp = cnt[1];
  o->flat = x->h_flat; o->n_flat = cnt[2];
  o->less_flat = x->h_lflat; o->n_less_flat = cnt[3];
  o->odom_valid = valid;
  for (int i = 0; i < 6; ++i) { o->transform_sum[i] = sum[i]; o->transform_cur[i] = cur[i]; }
  odom_quat(sum, o->odom_quat, o->odom_pos);
  o->publish_to_mapping = pub;
  if (pub) {
    o->corner_last = x->h_cornerLast; o->n_corner_last = cnt[1];
    o->surf_last = x->h_surfLast; o->n_surf_last = cnt[3];
    o->outlier_last = x->h_outlLast; o->n_outlier_last = nout;
  }
  x->faGen = x->devGen;
  x->faK = k;
  x->faCnt[0] = cnt[1]; x->faCnt[1] = cnt[3]; x->faCnt[2] = nout;
  return LEGO_OK;
}

// The node call's upload of a host cloud (lego_ip_process): one pass over
// the caller's records packs them (x, y, z, ring: the 16 bytes the
// projection reads of each 32-byte record) into the context's pinned staging
// buffer and accumulates the dense check (imageProjection.cpp:174; an all-ones
// exponent is inf / nan, branch-free so the loop vectorises), chunk by chunk,
// each chunk's DMA to x->d_pts queued as soon as it is staged, so the copy
// engine works beside the next chunk's pass; clouds of more than two chunks
// (dense sensors) are packed by three helper threads and the caller
// (lego_pack_host.h).  It replaces a separate check
// pass plus the runtime's staged copy of pageable memory: VLS-128's 7.4 MB
// were read twice and all of them crossed PCIe.  A non-dense cloud (with
// use_cloud_ring) is refused here, before any kernel: nothing but d_pts has
// changed.  Without useCloudRing k_project drops such points (:170).
static int upload_checked(lego_ctx* x, const lego_point_xyzir* pts, int32_t n) {
  HIPCHK(hipSetDevice(x->device));
  static_assert(sizeof(float4) * 2 == sizeof(lego_point_xyzir), "the packed form fits d_pts");
  if (!x->h_stage &&
      hipHostMalloc((void**)&x->h_stage, sizeof(float4) * (size_t)x->maxPoints, hipHostMallocDefault) != hipSuccess) {
    x->h_stage = nullptr;
    set_err("hipHostMalloc failed for the node call's staging buffer");
    return LEGO_E_DEVICE;
  }
  float4* d = (float4*)x->d_pts;
  uint32_t nonfinite = 0;
  constexpr int kChunk = PackPool::kChunk;
  if (n > 2 * kChunk) {  // a dense sensor's cloud: three helper threads beside the caller
    if (!x->pack) x->pack.reset(new PackPool(3, x->maxPoints));
    hipError_t err = hipSuccess;
    nonfinite = x->pack->run(pts, (uint32_t*)x->h_stage, n, [&](int c0, int c1) {
      if (err == hipSuccess)
        err = hipMemcpyAsync(d + c0, x->h_stage + c0, sizeof(float4) * (size_t)(c1 - c0), hipMemcpyHostToDevice,
                             x->stream);
    });
    HIPCHK(err);
  } else {
    for (int c0 = 0; c0 < n; c0 += kChunk) {
      const int c1 = std::min(n, c0 + kChunk);
      nonfinite |= pack_points(pts, (uint32_t*)x->h_stage, c0, c1);
      HIPCHK(hipMemcpyAsync(d + c0, x->h_stage + c0, sizeof(float4) * (size_t)(c1 - c0), hipMemcpyHostToDevice,
                            x->stream));
    }
  }
  if (nonfinite && x->dc.ringRow) {
    HIPCHK(hipStreamSynchronize(x->stream));  // the staging buffer is free again when this returns
    set_err("the cloud has non-finite xyz (it must be dense with use_cloud_ring)");
    return LEGO_E_NOT_DENSE;
  }
  return LEGO_OK;
}

int lego_ip_process(lego_ctx* x, const lego_point_xyzir* pts, int32_t n, double stamp,
                    uint32_t flags, lego_ip_out* out) {
  if (!x || !pts || !out || n <= 0) return LEGO_E_ARG;
  if (n > x->maxPoints) return LEGO_E_CAPACITY;
  if (x->inflight) {
    set_err("node-shaped call while batches are in flight (lego_odom_batch_wait first)");
    return LEGO_E_STATE;
  }
  const int up = upload_checked(x, pts, n);
  if (up != LEGO_OK) return up;
  int64_t off[2] = {0, n};
  x->stamps.assign(1, stamp);
  const bool gated = (flags & LEGO_IP_GATED) != 0;
  const int st = run_ip(x, pts, off, 1, 0, (flags & LEGO_IP_IMAGES) != 0, out, gated, true);
  if (st != LEGO_OK) return st;
  x->lastIp = *out;
  x->lastIpDevice = true;
  return LEGO_OK;
}

// Uploads a host cloud_info + segmented cloud into batch slot 0 (used when the
// caller's input did not come from this context's lego_ip_process).
static int upload_ip(lego_ctx* x, const lego_ip_out* in) {
  const DevCfg& c = x->dc;
  const int ns = in->n_segmented;
  if (ns < 0 || ns > c.P || in->n_outlier < 0 || in->n_outlier > c.P) return LEGO_E_CAPACITY;
  hipStream_t s = x->stream;
  std::vector<float4> seg(ns);
  for (int i = 0; i < ns; ++i) {
    const lego_point_xyzi& p = in->segmented_cloud[i];
    seg[i] = make_float4(p.x, p.y, p.z, p.intensity);
  }
  float orient[3] = {in->info.start_orientation, in->info.end_orientation, in->info.orientation_diff};
  HIPCHK(hipMemcpyAsync(x->bb.seg, seg.data(), sizeof(float4) * ns, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(x->bb.gflag, in->info.segmented_cloud_ground_flag, ns, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(x->bb.col, in->info.segmented_cloud_col_ind, sizeof(uint32_t) * ns, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(x->bb.srange, in->info.segmented_cloud_range, sizeof(float) * ns, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(x->bb.outl, in->outlier_cloud, sizeof(float4) * in->n_outlier, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(x->bb.ns, &ns, sizeof(int), hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(x->bb.nout, &in->n_outlier, sizeof(int), hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(x->bb.sri, in->info.start_ring_index, sizeof(int) * c.N, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(x->bb.eri, in->info.end_ring_index, sizeof(int) * c.N, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(x->bb.orient, orient, sizeof(orient), hipMemcpyHostToDevice, s));
  HIPCHK(hipStreamSynchronize(s));
  return LEGO_OK;
}

int lego_fa_process(lego_ctx* x, const lego_ip_out* in, lego_fa_out* out) {
  if (!x || !in || !out) return LEGO_E_ARG;
  if (x->inflight) {
    set_err("node-shaped call while batches are in flight (lego_odom_batch_wait first)");
    return LEGO_E_STATE;
  }
  if (x->nStreams != 1) {
    set_err("lego_fa_process needs a single-stream context");
    return LEGO_E_ARG;
  }
  if (x->needReset) {
    set_err("an earlier odometry call failed on the device: lego_reset first");
    return LEGO_E_STATE;
  }
  HIPCHK(hipSetDevice(x->device));
  ++x->devGen;
  const bool resident = x->lastIpDevice && in->segmented_cloud == x->h_seg &&
                        in->n_segmented == x->lastIp.n_segmented;
  if (!resident) {
    int st = upload_ip(x, in);
    if (st != LEGO_OK) return st;
  }
  x->stamps.assign(1, in->info.stamp);
  BatchBufs bb = x->bb;
  bb.xprof = x->profOn ? x->d_prof + 32 : nullptr;  // k_extract's stamps (lego_extract_profile)
  HIPCHK(hipEventRecord(x->oJoin, x->ostream));  // e.g. a reset of the odometry state
  HIPCHK(hipStreamWaitEvent(x->stream, x->oJoin, 0));
  {
    const int st = imu_stage(x, 1, nullptr, 0, nullptr, &bb.imu);
    if (st != LEGO_OK) return st;
  }
  HIPCHK(hipMemsetAsync(bb.bad, 0, sizeof(int), x->stream));  // ip reported its own bit; k_lf_voxel's below
  x->tm.begin();
  // the per-ring less-flat VoxelGrid (featureAssociation.cpp:778-782) feeds
  // only the hand-off (publishCloudsLast, :1759-1815): it runs on ostream
  // beside the LM, and the hand-off waits for it (OdomBufs::lfWait)
  // (lego_ctx_opts::node_overlap = 0: everything on one stream).  Only
  // while the odometry's workgroups, each holding a CU's registers, leave
  // room for the VoxelGrid's rings (a partitioned device with as many CUs as
  // workgroups would starve it until the hand-off's wait gives up)
  const int odomWGs = x->ob.G + (x->ob.integ ? 1 : 0);
  const bool overlap = x->opts.node_overlap != 0 && odomWGs <= x->cus - x->dc.N / 2;
  launch_fa(bb, x->dc, 1, 1, x->d_carry, x->stream, &x->tm, x->lo, overlap ? x->ostream : nullptr, x->lfFork,
            x->d_lfReady);
  // launch_odom's prep zeroes *ob.xerr; the hand-off's wait bound in ticks of
  // the 100 MHz wall clock (s_memrealtime)
  const unsigned long long lfTicks = (unsigned long long)x->opts.lf_wait_ms * 100000ull;
  if (launch_odom(bb, x->ob, x->dc, 1, x->stream, &x->tm, x->profOn ? x->d_prof : nullptr,
                  overlap ? x->d_lfReady : nullptr, lfTicks) != 0) {
    set_err("odometry launch failed (%d workgroups)", x->ob.G);
    return LEGO_E_DEVICE;
  }
  x->tm.end(x->stream);
  if (overlap) {  // the fetch reads f_lflat: the side stream first
    HIPCHK(hipEventRecord(x->oJoin, x->ostream));
    HIPCHK(hipStreamWaitEvent(x->stream, x->oJoin, 0));
  }
  HIPCHK(hipGetLastError());
  x->lastB = 1;
  x->lastBase = 0;
  x->lastBatch = false;  // slot 0's buffers now hold this scan, not a waited batch
  x->lastIpDevice = false;
  const int st = fetch_fa(x, 0, out, true);  // the exchange error word with the outputs: one sync
  if (st != LEGO_OK) return st;
  {  // the call's stage times (fa.*, odom.lm) for lego_stage_times; events are complete after the sync
    x->tnames.clear();
    x->tms.clear();
    std::vector<int> cnt;
    x->tm.collect(x->tnames, x->tms, cnt);
  }
  if (x->h_hdr[FH_XERR]) {
    x->faK = -1;  // no resident hand-off of a failed scan
    set_err("odometry error word %u (1: more NN rounds than slots, 2: a ring share never done, 3: the "
            "integration never saw a scan's transform)", (unsigned)x->h_hdr[FH_XERR]);
    return LEGO_E_DEVICE;
  }
  if (x->h_hdr[FH_BAD] & kBadPermutation) {
    x->faK = -1;
    set_err("per-ring VoxelGrid: the device sort returned a payload outside its input (device fault)");
    return LEGO_E_DEVICE;
  }
  if (x->h_hdr[FH_BAD] & kBadLfLate) {
    x->faK = -1;
    x->needReset = true;
    set_err("the hand-off waited more than %d ms for the per-ring VoxelGrid on the side stream "
            "(the stream state was not advanced: lego_reset to go on)", x->opts.lf_wait_ms);
    return LEGO_E_DEVICE;
  }
  return LEGO_OK;
}

int lego_odom_batch(lego_ctx* x, const lego_point_xyzir* pts, const int64_t* offsets,
                    const double* stamps, int32_t nscans, int32_t on_device, lego_pose_rec* recs) {
  return lego_odom_batch_imu(x, pts, offsets, stamps, nscans, on_device, nullptr, 0, nullptr, recs);
}

int lego_imu_push(lego_ctx* x, const lego_imu_msg* msgs, int32_t n) {
  if (!x || n < 0 || (n > 0 && !msgs)) return LEGO_E_ARG;
  if (x->nStreams != 1) {
    set_err("IMU input needs a single-stream context");
    return LEGO_E_ARG;
  }
  imu_deliver(x, msgs, n);
  return LEGO_OK;
}

int lego_odom_batch_submit(lego_ctx* x, const lego_point_xyzir* pts, const int64_t* offsets,
                           const double* stamps, int32_t nscans, int32_t on_device, const lego_imu_msg* imu,
                           int32_t n_imu, const int32_t* imu_before) {
  if (!x || !pts || !offsets || nscans <= 0) return LEGO_E_ARG;
  if (n_imu < 0 || (n_imu > 0 && (!imu || !imu_before))) return LEGO_E_ARG;
  if (n_imu > 0) {
    if (x->nStreams != 1) {
      set_err("IMU input needs a single-stream context");
      return LEGO_E_ARG;
    }
    for (int k = 0; k < nscans; ++k)
      if (imu_before[k] < (k ? imu_before[k - 1] : 0) || imu_before[k] > n_imu) {
        set_err("imu_before must be non-decreasing within [0, n_imu]");
        return LEGO_E_ARG;
      }
  }
  if (nscans > x->maxBatch) {
    set_err("batch of %d scans > context capacity %d", nscans, x->maxBatch);
    return LEGO_E_CAPACITY;
  }
  if (nscans % x->nStreams) {
    set_err("batch of %d scans is not %d streams x K scans", nscans, x->nStreams);
    return LEGO_E_ARG;
  }
  HIPCHK(hipSetDevice(x->device));
  x->stamps.assign(stamps ? stamps : nullptr, stamps ? stamps + nscans : nullptr);
  if (!stamps) x->stamps.assign(nscans, 0.0);
  x->lastIpDevice = false;
  return submit_batch(x, pts, offsets, nscans, on_device, imu, n_imu, imu_before);
}

int lego_odom_batch_wait(lego_ctx* x, lego_pose_rec* recs, int32_t cap, int32_t* nscans) {
  if (!x || !recs) return LEGO_E_ARG;
  HIPCHK(hipSetDevice(x->device));
  int n = 0;
  const int st = wait_batch(x, recs, cap, &n);
  if (nscans) *nscans = n;
  return st;
}

int lego_odom_batch_imu(lego_ctx* x, const lego_point_xyzir* pts, const int64_t* offsets,
                        const double* stamps, int32_t nscans, int32_t on_device, const lego_imu_msg* imu,
                        int32_t n_imu, const int32_t* imu_before, lego_pose_rec* recs) {
  if (!x || !recs) return LEGO_E_ARG;
  if (x->inflight) {
    set_err("lego_odom_batch with batches in flight (lego_odom_batch_wait first)");
    return LEGO_E_STATE;
  }
  const int st = lego_odom_batch_submit(x, pts, offsets, stamps, nscans, on_device, imu, n_imu, imu_before);
  if (st != LEGO_OK) return st;
  return lego_odom_batch_wait(x, recs, nscans, nullptr);
}

int lego_batch_fetch(lego_ctx* x, int32_t k, lego_ip_out* ip, lego_fa_out* fa) {
  if (!x || k < 0 || k >= x->lastB) return LEGO_E_ARG;
  HIPCHK(hipSetDevice(x->device));
  if (ip) {
    int st = fetch_ip(x, x->lastBase + k, false, ip);
    if (st != LEGO_OK) return st;
  }
  if (fa) return fetch_fa(x, x->lastBase + k, fa);
  return LEGO_OK;
}

// Device buffers of the scan-to-map step for maps of up to nc / ns points.
static int mo_alloc(lego_ctx* x, int nc, int ns) {
  MoDev& m = x->mo;
  const int N = x->dc.N, P = x->dc.P;
  auto fail = [&](const char* what) {
    set_err("hipMalloc failed for %s", what);
    return LEGO_E_DEVICE;
  };
#define MA(ptr, n) \
  if (x->alloc(&(ptr), (size_t)(n)) != hipSuccess) return fail(#ptr);
  if (!x->moAlloc) {
    MA(m.st, 1);
    MA(m.cnt, 1);
    m.scanCap = P;
    MA(m.cornerLast, N * kLessSharpPerRing); MA(m.surfLast, P); MA(m.outlierLast, P);
    MA(m.cornerDS, N * kLessSharpPerRing); MA(m.surfDS, P); MA(m.outlierDS, P);
    MA(m.surfTotal, 2 * P); MA(m.surfTotalDS, 2 * P);
    m.rowCap = N * kLessSharpPerRing + 2 * P;
    MA(m.rows, (size_t)m.rowCap * 8);
    m.candQ = std::min(m.rowCap, kCandQueries);
    if (!x->opts.mo_cand_cache) m.candQ = 0;  // no cache (device memory)
    MA(m.cand, (size_t)m.candQ * kCand);
    MA(m.candRef, (size_t)m.candQ);
    m.partCap = 4096;  // k_mo_rows' grid cap (grid_for)
    MA(m.part, (size_t)m.partCap * 28);
    HIPCHK(hipMemsetAsync(m.st, 0, sizeof(MoState), x->stream));
    HIPCHK(hipMemsetAsync(m.cnt, 0, sizeof(MoCounts), x->stream));
    // the VoxelGrids' fork streams (lego_mo.h): created with the mapping
    // buffers, so contexts that never map keep two streams
    m.fork[0] = x->ostream;
    if (hipStreamCreateWithFlags(&m.fork[1], hipStreamNonBlocking) != hipSuccess) return fail("fork stream");
    for (auto& e : m.ev)
      if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return fail("fork event");
    x->moAlloc = true;
  }
  auto ctx_alloc = [](void* c, void** p, size_t bytes) {
    return static_cast<lego_ctx*>(c)->alloc(reinterpret_cast<unsigned char**>(p), bytes) == hipSuccess ? 0 : -1;
  };
  // buffers are never freed before the context: grow by reallocating
  const int vcap = std::max(std::max(nc, ns), 2 * P);
  if (vcap > m.vg.cap && vg_scratch_alloc(m.vg, vcap, x, ctx_alloc)) return fail("VoxelGrid scratch");
  const int v2cap = std::max(nc, N * kLessSharpPerRing);
  if (v2cap > m.vgMap2.cap && vg_scratch_alloc(m.vgMap2, v2cap, x, ctx_alloc)) return fail("VoxelGrid scratch");
  if (2 * P > m.vgScan1.cap && vg_scratch_alloc(m.vgScan1, 2 * P, x, ctx_alloc)) return fail("VoxelGrid scratch");
  if (P > m.vgScan2.cap && vg_scratch_alloc(m.vgScan2, P, x, ctx_alloc)) return fail("VoxelGrid scratch");
  for (VgScratch* v : {&m.vg, &m.vgMap2, &m.vgScan1, &m.vgScan2}) v->err = &m.cnt->derr;  // read after every step
  if (nc > m.mapCornerCap) {
    m.mapCornerCap = nc;
    MA(m.cornerMap, nc); MA(m.cornerMapDS, nc);
    int T = 64;
    while (T < nc) T <<= 1;
    MA(m.cornerIx.begin, T); MA(m.cornerIx.end, T); MA(m.cornerIx.sorted, nc);
    m.cornerIx.cap = nc;
  }
  if (ns > m.mapSurfCap) {
    m.mapSurfCap = ns;
    MA(m.surfMap, ns); MA(m.surfMapDS, ns);
    int T = 64;
    while (T < ns) T <<= 1;
    MA(m.surfIx.begin, T); MA(m.surfIx.end, T); MA(m.surfIx.sorted, ns);
    m.surfIx.cap = ns;
  }
#undef MA
  return LEGO_OK;
}

// Keyframe store for the keyframe-built map (first use without a fixed map).
static int mo_alloc_keyframes(lego_ctx* x) {
  MoDev& m = x->mo;
  if (m.kf.kcap) return LEGO_OK;
  const int fromCap = 2 << 20;
  int st = mo_alloc(x, fromCap, fromCap);
  if (st != LEGO_OK) return st;
  MoKeyframes& kf = m.kf;
  int kcap = 16384, acap = 16 << 20;
  if (x->opts.kf_cap > 0) kcap = std::min(kcap, x->opts.kf_cap);  // diagnostic
#define MA(ptr, n) \
  if (x->alloc(&(ptr), (size_t)(n)) != hipSuccess) { set_err("hipMalloc failed for %s", #ptr); return LEGO_E_DEVICE; }
  MA(kf.pos3, kcap); MA(kf.pose6, kcap * 6); MA(kf.time, kcap); MA(kf.seg, kcap * 6); MA(kf.arena, acap);
  MA(kf.exID, kcap); MA(kf.plan, kcap * 4); MA(kf.planPose, kcap * 6); MA(kf.sur, kcap); MA(kf.surDS, kcap); MA(kf.sortKeys, kcap);
  MA(kf.meta, kKfMeta); MA(kf.robot, 8);
  MA(m.cornerFromMap, fromCap); MA(m.surfFromMap, fromCap);
#undef MA
  m.fromMapCap = fromCap;
  HIPCHK(hipMemsetAsync(kf.meta, 0, sizeof(int) * kKfMeta, x->stream));
  HIPCHK(hipMemsetAsync(kf.robot, 0, sizeof(float) * 8, x->stream));
  kf.kcap = kcap;
  kf.acap = acap;
  return LEGO_OK;
}

int lego_mo_set_map(lego_ctx* x, const lego_point_xyzi* corner, int32_t n_corner,
                    const lego_point_xyzi* surf, int32_t n_surf) {
  if (x && x->nStreams != 1) {
    set_err("mapping needs a single-stream context");
    return LEGO_E_ARG;
  }
  if (!x) return LEGO_E_ARG;
  HIPCHK(hipSetDevice(x->device));
  if (!corner && !surf) {
    x->moFixed = false;
    return LEGO_OK;
  }
  if (!corner || !surf || n_corner < 0 || n_surf < 0) return LEGO_E_ARG;
  int st = mo_alloc(x, std::max(n_corner, 1), std::max(n_surf, 1));
  if (st != LEGO_OK) return st;
  MoDev& m = x->mo;
  HIPCHK(hipMemcpyAsync(m.cornerMap, corner, sizeof(float4) * n_corner, hipMemcpyHostToDevice, x->stream));
  HIPCHK(hipMemcpyAsync(m.surfMap, surf, sizeof(float4) * n_surf, hipMemcpyHostToDevice, x->stream));
  m.nCornerMap = n_corner;
  m.nSurfMap = n_surf;
  if (mo_set_map_device(m, n_corner, n_surf, x->stream) != 0) {
    set_err("scan-to-map: map voxel filter / index launch failed");
    return LEGO_E_DEVICE;
  }
  HIPCHK(hipStreamSynchronize(x->stream));
  x->moFixed = true;
  return LEGO_OK;
}

int lego_sort_permutation(lego_ctx* x, const uint32_t* keys, int32_t n, int32_t wave, int32_t* perm,
                          int32_t* heap_pieces) {
  const int cap = sort_perm_cap(wave);
  if (!x || n < 0 || (n > 0 && (!keys || !perm)) || cap < 0) return LEGO_E_ARG;
  if (n > cap) {
    set_err("lego_sort_permutation: n = %d above the mode-%d sort's %d", n, wave, cap);
    return LEGO_E_CAPACITY;
  }
  HIPCHK(hipSetDevice(x->device));
  uint32_t* dk = nullptr;
  int* dp = nullptr;
  HIPCHK(hipMallocAsync((void**)&dk, sizeof(uint32_t) * (size_t)(n + 1) + sizeof(int) * (size_t)(n + 2), x->stream));
  dp = (int*)(dk + n + 1);
  HIPCHK(hipMemsetAsync(dp, 0, sizeof(int), x->stream));
  if (n) HIPCHK(hipMemcpyAsync(dk, keys, sizeof(uint32_t) * n, hipMemcpyHostToDevice, x->stream));
  const int rc = sort_perm_device(dk, n, wave, dp + 1, dp, x->stream);
  int h = 0;
  if (rc == 0) {
    if (n) HIPCHK(hipMemcpyAsync(perm, dp + 1, sizeof(int) * n, hipMemcpyDeviceToHost, x->stream));
    HIPCHK(hipMemcpyAsync(&h, dp, sizeof(int), hipMemcpyDeviceToHost, x->stream));
  }
  HIPCHK(hipFreeAsync(dk, x->stream));
  HIPCHK(hipStreamSynchronize(x->stream));
  if (rc) {
    set_err("lego_sort_permutation: launch failed");
    return LEGO_E_DEVICE;
  }
  if (heap_pieces) *heap_pieces = h;
  return LEGO_OK;
}

int lego_voxel_grid(lego_ctx* x, const lego_point_xyzi* in, int32_t n, float leaf, lego_point_xyzi* out,
                    int32_t* n_out) {
  if (!x || !n_out || n < 0 || (n > 0 && (!in || !out)) || !(leaf > 0.f)) return LEGO_E_ARG;
  HIPCHK(hipSetDevice(x->device));
  if (n > x->vgCap) {
    auto ctx_alloc = [](void* c, void** p, size_t bytes) {
      return static_cast<lego_ctx*>(c)->alloc(reinterpret_cast<unsigned char**>(p), bytes) == hipSuccess ? 0 : -1;
    };
    if (vg_scratch_alloc(x->vgApi, n, x, ctx_alloc)) {
      set_err("hipMalloc failed for the VoxelGrid scratch");
      return LEGO_E_DEVICE;
    }
    if (x->alloc(&x->vgIn, n) != hipSuccess || x->alloc(&x->vgOut, n) != hipSuccess ||
        (!x->vgN && x->alloc(&x->vgN, 1) != hipSuccess)) {
      set_err("hipMalloc failed for the VoxelGrid clouds");
      return LEGO_E_DEVICE;
    }
    x->vgCap = n;
  }
  if (n == 0) {
    *n_out = 0;
    std::fill(x->vgStats, x->vgStats + 8, 0);
    return LEGO_OK;
  }
  for (auto& e : x->vgEv)
    if (!e) HIPCHK(hipEventCreate(&e));  // once per context (destroyed with it)
  hipEvent_t e0 = x->vgEv[0], e1 = x->vgEv[1];
  HIPCHK(hipMemcpyAsync(x->vgIn, in, sizeof(float4) * n, hipMemcpyHostToDevice, x->stream));
  HIPCHK(hipEventRecord(e0, x->stream));
  const int rc = voxel_grid_device(x->vgIn, n, nullptr, leaf, x->vgOut, x->vgN, x->vgApi, x->stream);
  HIPCHK(hipEventRecord(e1, x->stream));
  int nOut = 0, ctl[16];
  HIPCHK(hipMemcpyAsync(&nOut, x->vgN, sizeof(int), hipMemcpyDeviceToHost, x->stream));
  HIPCHK(hipStreamSynchronize(x->stream));
  float ms = 0.f;
  HIPCHK(hipEventElapsedTime(&ms, e0, e1));
  if (rc != 0 || vg_read_ctl(x->vgApi, ctl, x->stream) != 0) {
    set_err("VoxelGrid launch failed");
    return LEGO_E_DEVICE;
  }
  if (ctl[10]) {  // C_ERR (lego_vg.hip): a sorted payload outside the cloud
    set_err("VoxelGrid: the sort returned a payload outside the cloud (device fault)");
    return LEGO_E_DEVICE;
  }
  HIPCHK(hipMemcpy(out, x->vgOut, sizeof(float4) * nOut, hipMemcpyDeviceToHost));
  *n_out = nOut;
  // ctl: C_M 0, C_NLOC 4, C_NONFIN 5, C_NOUT 6, C_SLOW 7, C_HEAP 8, C_NLOCB 9 (lego_vg.hip)
  const int st[8] = {ctl[0], ctl[6], vg_rounds_for(n, x->vgApi.rounds), ctl[4] + ctl[9], ctl[7], ctl[8], ctl[5], (int)(ms * 1000.f)};
  std::copy(st, st + 8, x->vgStats);
  return LEGO_OK;
}

int lego_voxel_grid_stats(lego_ctx* x, int32_t stats[8]) {
  if (!x || !stats) return LEGO_E_ARG;
  std::copy(x->vgStats, x->vgStats + 8, stats);
  return LEGO_OK;
}

int lego_mo_configure(lego_ctx* x, const lego_mo_opts* o) {
  if (!x || !o) return LEGO_E_ARG;
  if (x->nStreams != 1) {
    set_err("mapping needs a single-stream context");
    return LEGO_E_ARG;
  }
  if ((o->loop_closure_enable != 0) != (x->moOpts.loop_closure_enable != 0) && x->mo.kf.kcap) {
    int K = 0;
    HIPCHK(hipSetDevice(x->device));
    HIPCHK(hipMemcpy(&K, x->mo.kf.meta + KF_K, sizeof(int), hipMemcpyDeviceToHost));
    if (K > 0) {
      set_err("loop_closure_enable changes the keyframe bookkeeping: lego_reset first");
      return LEGO_E_STATE;
    }
  }
  x->moOpts = *o;
  x->mo.mapPerStep = o->fixed_map_per_step ? 1 : 0;
  return LEGO_OK;
}

int lego_mo_loop_closure(lego_ctx* x, lego_loop_out* out) {
  if (x && x->nStreams != 1) {
    set_err("loop closure needs a single-stream context");
    return LEGO_E_ARG;
  }
  if (!x || !out) return LEGO_E_ARG;
  std::memset(out, 0, sizeof(*out));
  out->latest_id = out->closest_id = -1;
  if (x->moFixed) {
    set_err("loop closure runs over the keyframe store (no fixed map installed)");
    return LEGO_E_ARG;
  }
  MoDev& m = x->mo;
  if (!m.kf.kcap) return LEGO_OK;  // no mapping step yet: cloudKeyPoses3D is empty
  HIPCHK(hipSetDevice(x->device));
  LcDev& lc = x->lc;
  if (!lc.cap) {
    const int cap = m.fromMapCap;
    int T = 64;
    while (T < cap) T <<= 1;
#define MA(ptr, n) \
  if (x->alloc(&(ptr), (size_t)(n)) != hipSuccess) { set_err("hipMalloc failed for %s", #ptr); return LEGO_E_DEVICE; }
    MA(lc.st, 1); MA(lc.srcRaw, cap); MA(lc.src, cap); MA(lc.cur, cap); MA(lc.tgtRaw, cap); MA(lc.tgt, cap);
    MA(lc.cIdx, cap); MA(lc.cD, cap); MA(lc.ix.begin, T); MA(lc.ix.end, T); MA(lc.ix.sorted, cap);
#undef MA
    lc.ix.cap = cap;
    lc.cap = cap;
  }
  LcState hs;
  const int rs = mo_loop_closure_device(m, lc, x->moTimeOdom, &hs, x->stream);
  if (rs == MO_E_MAP_CAP) {
    set_err("loop closure: clouds larger than the loop buffers");
    return LEGO_E_CAPACITY;
  }
  if (rs != 0) {
    set_err("loop closure launch failed");
    return LEGO_E_DEVICE;
  }
  {  // the history cloud's VoxelGrid error word (MoCounts::derr; the state read above synchronised)
    int derr = 0;
    HIPCHK(hipMemcpy(&derr, &m.cnt->derr, sizeof(int), hipMemcpyDeviceToHost));
    if (derr) {
      HIPCHK(hipMemset(&m.cnt->derr, 0, sizeof(int)));
      set_err("loop closure: a VoxelGrid sort returned a payload outside its cloud (device fault)");
      return LEGO_E_DEVICE;
    }
  }
  if (!hs.detected) return LEGO_OK;
  out->detected = 1;
  out->latest_id = hs.latest;
  out->closest_id = hs.closest;
  out->n_source = hs.nSrc;
  out->n_target = hs.nTgt;
  out->iterations = hs.iterations;
  out->converged = hs.converged;
  out->fitness = hs.fitness;
  std::memcpy(out->icp_transform, hs.fin, sizeof(hs.fin));
  out->accepted = hs.converged && !(hs.fitness > 0.3);  // historyKeyframeFitnessScore, utility.h:134
  if (out->accepted) {
    float p6[2][6];
    HIPCHK(hipMemcpy(p6[0], m.kf.pose6 + 6 * hs.latest, sizeof(p6[0]), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(p6[1], m.kf.pose6 + 6 * hs.closest, sizeof(p6[1]), hipMemcpyDeviceToHost));
    LoopFactor f;
    loop_factor(hs.fin, p6[0], p6[1], &f);
    std::memcpy(out->from_rotation, f.fromR, sizeof(f.fromR));
    std::memcpy(out->from_translation, f.fromT, sizeof(f.fromT));
    std::memcpy(out->to_rotation, f.toR, sizeof(f.toR));
    std::memcpy(out->to_translation, f.toT, sizeof(f.toT));
    std::memcpy(out->between_rotation, f.betweenR, sizeof(f.betweenR));
    std::memcpy(out->between_translation, f.betweenT, sizeof(f.betweenT));
    if (x->moOpts.loop_closure_enable) {  // gtSAMgraph.add + isam->update (:930-944)
      const double noise = (double)(float)hs.fitness;  // float noiseScore (:931)
      const double var[6] = {noise, noise, noise, noise, noise, noise};
      Pose3d z;
      std::memcpy(z.R, f.betweenR, sizeof(z.R));
      std::memcpy(z.t, f.betweenT, sizeof(z.t));
      x->pg.add_between(hs.latest, hs.closest, z, var, true);
      x->aLoopIsClosed = true;
    }
  }
  return LEGO_OK;
}

// loopClosureEnableFlag's extractSurroundingKeyFrames (mapOptmization.cpp:
// 961-999): the queue of the most recent keyframes, each with the pose its
// clouds were transformed with, and the gather plan of the map it makes
// (corner clouds, then surf + outlier per key), uploaded on the stream.
static int lc_recent_plan(lego_ctx* x, MoStepArgs& a) {
  const int K = (int)x->kfPose.size();
  const int num = x->moOpts.surrounding_keyframe_search_num > 0 ? x->moOpts.surrounding_keyframe_search_num : 50;
  a.nPlan = a.nCM = a.nSM = 0;
  if (K == 0) return LEGO_OK;  // cloudKeyPoses3D empty: no map (:958-959)
  auto& q = x->recent;
  if ((int)q.size() < num) {  // not full: rebuilt from the newest keys (:963-977)
    q.clear();
    for (int i = K - 1; i >= 0; --i) {
      q.push_front({i, x->kfPose[i]});
      if ((int)q.size() >= num) break;
    }
  } else if (x->latestFrameID != K - 1) {  // full: the oldest out, the newest in (:978-991)
    q.pop_front();
    x->latestFrameID = K - 1;
    q.push_back({K - 1, x->kfPose[K - 1]});
  }
  const int n = (int)q.size();
  std::vector<int> plan((size_t)n * 4);
  std::vector<float> pose((size_t)n * 6);
  int oc = 0, os = 0;
  for (int i = 0; i < n; ++i) {
    const int key = q[i].key;
    plan[4 * i] = key;
    plan[4 * i + 1] = oc;
    plan[4 * i + 2] = os;
    plan[4 * i + 3] = 0;
    std::memcpy(&pose[6 * i], q[i].pose.data(), sizeof(float) * 6);
    oc += x->kfSeg[key][1];
    os += x->kfSeg[key][3] + x->kfSeg[key][5];
  }
  MoKeyframes& kf = x->mo.kf;
  HIPCHK(hipMemcpyAsync(kf.plan, plan.data(), sizeof(int) * plan.size(), hipMemcpyHostToDevice, x->stream));
  HIPCHK(hipMemcpyAsync(kf.planPose, pose.data(), sizeof(float) * pose.size(), hipMemcpyHostToDevice, x->stream));
  HIPCHK(hipStreamSynchronize(x->stream));  // the host vectors go out of scope
  a.nPlan = n;
  a.nCM = oc;
  a.nSM = os;
  return LEGO_OK;
}

static std::array<float, 6> t6_of_pose6(const std::array<float, 6>& p) {  // x y z r p y -> transform order
  return {p[3], p[4], p[5], p[0], p[1], p[2]};
}

// Writes keyframe i's pose (transform order r p y x y z) to the device store
// (cloudKeyPoses3D / 6D) and the host mirror.
static int lc_put_key(lego_ctx* x, int i, const float (&t)[6]) {
  MoKeyframes& kf = x->mo.kf;
  const std::array<float, 6> p6 = {t[3], t[4], t[5], t[0], t[1], t[2]};
  const float4 p3 = make_float4(t[3], t[4], t[5], (float)i);
  if (i < (int)x->kfPose.size()) x->kfPose[i] = p6;  // the loop-closure mode's host mirror
  HIPCHK(hipMemcpyAsync(kf.pose6 + 6 * i, p6.data(), sizeof(float) * 6, hipMemcpyHostToDevice, x->stream));
  HIPCHK(hipMemcpyAsync(kf.pos3 + i, &p3, sizeof(float4), hipMemcpyHostToDevice, x->stream));
  HIPCHK(hipStreamSynchronize(x->stream));
  return LEGO_OK;
}

// Key K - 1 (just saved by k_kf_save from the chain's transform) takes iSAM2's
// latest estimate t as the reference stores it (:1412-1432): the key pose,
// and past the first key transformAftMapped = transformTobeMapped = t.
// Device writes only where t differs from what the device holds.
static int kf_put_estimate(lego_ctx* x, MoState& hs, int K, const float (&t)[6]) {
  const float* chain = K == 1 ? hs.transformTobeMapped : hs.transformAftMapped;
  if (std::memcmp(chain, t, sizeof(t)) == 0) return LEGO_OK;
  const int st = lc_put_key(x, K - 1, t);
  if (st != LEGO_OK) return st;
  if (K > 1) {
    for (int i = 0; i < 6; ++i) hs.transformAftMapped[i] = hs.transformTobeMapped[i] = t[i];
    MoDev& m = x->mo;
    HIPCHK(hipMemcpyAsync((char*)m.st + offsetof(MoState, transformAftMapped), t, sizeof(t), hipMemcpyHostToDevice,
                          x->stream));
    HIPCHK(hipMemcpyAsync((char*)m.st + offsetof(MoState, transformTobeMapped), t, sizeof(t), hipMemcpyHostToDevice,
                          x->stream));
    HIPCHK(hipStreamSynchronize(x->stream));  // t may be a stack array
  }
  return LEGO_OK;
}

// the chain's transform of the key just saved, round-tripped (no loop factor:
// iSAM2's estimate is the chain itself)
static void kf_chain_estimate(const MoState& hs, int K, float (&t)[6]) {
  float c[6];
  for (int i = 0; i < 6; ++i) c[i] = K == 1 ? hs.transformTobeMapped[i] : hs.transformAftMapped[i];
  transform_roundtrip(c, t);
}

// saveKeyFramesAndFactor's graph part and correctPoses (:1372-1438, 1456-1478)
// after the device saved (or not) this step's keyframe; hs is updated to what
// the reference publishes.
static int lc_after_step(lego_ctx* x, MoState& hs, int saved, int K) {
  MoDev& m = x->mo;
  if (saved) {
    std::array<float, 6> p6;
    std::array<int, 6> sg;
    HIPCHK(hipMemcpyAsync(p6.data(), m.kf.pose6 + 6 * (K - 1), sizeof(float) * 6, hipMemcpyDeviceToHost, x->stream));
    HIPCHK(hipMemcpyAsync(sg.data(), m.kf.seg + 6 * (K - 1), sizeof(int) * 6, hipMemcpyDeviceToHost, x->stream));
    HIPCHK(hipStreamSynchronize(x->stream));
    x->kfPose.push_back(p6);
    x->kfSeg.push_back(sg);
    const double(&var)[6] = pgo_odometry_variances();
    if (K == 1) {
      float t[6];
      for (int i = 0; i < 6; ++i) t[i] = hs.transformTobeMapped[i];
      x->pg.add_prior(pose_from_transform(t), var);
      x->pg.insert(pose_from_transform(t));
      std::memcpy(x->transformLast, t, sizeof(t));
    } else {
      float aft[6];
      for (int i = 0; i < 6; ++i) aft[i] = hs.transformAftMapped[i];
      x->pg.add_between(K - 2, K - 1, pose_between(pose_from_transform(x->transformLast), pose_from_transform(aft)),
                        var);
      x->pg.insert(pose_from_transform(aft));
    }
    float t[6];  // latestEstimate
    if (x->pg.loops > 0) {
      x->pg.optimize();
      transform_from_pose(x->pg.est[K - 1], t);
    } else {
      kf_chain_estimate(hs, K, t);
    }
    const int st = kf_put_estimate(x, hs, K, t);
    if (st != LEGO_OK) return st;
    if (K > 1) std::memcpy(x->transformLast, t, sizeof(t));  // transformLast = latestEstimate
  }
  if (x->aLoopIsClosed) {  // correctPoses: the estimate of the last save, every key
    x->recent.clear();
    for (int i = 0; i < (int)x->pg.est.size(); ++i) {
      float t[6];
      transform_from_pose(x->pg.est[i], t);
      const int st = lc_put_key(x, i, t);
      if (st != LEGO_OK) return st;
    }
    x->aLoopIsClosed = false;
  }
  HIPCHK(hipStreamSynchronize(x->stream));
  return LEGO_OK;
}

int lego_mo_process(lego_ctx* x, const lego_fa_out* in, lego_mo_out* out) {
  if (x && x->nStreams != 1) {
    set_err("mapping needs a single-stream context");
    return LEGO_E_ARG;
  }
  if (!x || !in || !out) return LEGO_E_ARG;
  std::memset(out, 0, sizeof(*out));
  // run() gates (mapOptmization.cpp:1487-1499): a new hand-off, then the interval
  if (!in->publish_to_mapping || !in->odom_valid) return LEGO_OK;
  x->moTimeOdom = in->stamp;
  if (!(in->stamp - x->moTimeLast >= x->cfg.mapping_process_interval)) return LEGO_OK;
  if (!x->moFixed) {
    const int st = mo_alloc_keyframes(x);
    if (st != LEGO_OK) return st;
  }
  x->moTimeLast = in->stamp;
  MoDev& m = x->mo;
  if (x->moStoreFull) {  // both map modes: nothing of the step runs (lego_mo.h MO_E_STORE_FULL)
    set_err("scan-to-map: the keyframe store is full (%d keyframes / %d arena points); lego_reset to go on",
            m.kf.kcap, m.kf.acap);
    return LEGO_E_CAPACITY;
  }
  const int N = x->dc.N, P = x->dc.P;
  if (in->n_corner_last < 0 || in->n_corner_last > N * kLessSharpPerRing || in->n_surf_last < 0 ||
      in->n_surf_last > P || in->n_outlier_last < 0 || in->n_outlier_last > P) {
    set_err("scan-to-map: cloud larger than the sensor's capacity");
    return LEGO_E_CAPACITY;
  }
  HIPCHK(hipSetDevice(x->device));
  hipStream_t s = x->stream;
  MoStepArgs a;
  // the clouds of this context's own last fa output (the node path's hand-off
  // within one process): read where fetch_fa copied them from, on the device
  const bool resident = x->faK >= 0 && x->faGen == x->devGen && in->corner_last == x->h_cornerLast &&
                        in->surf_last == x->h_surfLast && in->outlier_last == x->h_outlLast &&
                        in->n_corner_last == x->faCnt[0] && in->n_surf_last == x->faCnt[1] &&
                        in->n_outlier_last == x->faCnt[2];
  if (resident) {
    a.corner = x->ob.cornerEnd + (size_t)x->faK * x->ob.capLS;
    a.surf = x->ob.surfEnd + (size_t)x->faK * P;
    a.outlierRaw = x->bb.outl + (size_t)x->faK * P;  // adjustOutlierCloud's axis swap on the device
  } else {
    if (in->n_corner_last)
      HIPCHK(hipMemcpyAsync(m.cornerLast, in->corner_last, sizeof(float4) * in->n_corner_last, hipMemcpyHostToDevice,
                            s));
    if (in->n_surf_last)
      HIPCHK(hipMemcpyAsync(m.surfLast, in->surf_last, sizeof(float4) * in->n_surf_last, hipMemcpyHostToDevice, s));
    if (in->n_outlier_last)
      HIPCHK(hipMemcpyAsync(m.outlierLast, in->outlier_last, sizeof(float4) * in->n_outlier_last,
                            hipMemcpyHostToDevice, s));
  }
  for (int i = 0; i < 4; ++i) a.quat[i] = in->odom_quat[i];
  for (int i = 0; i < 3; ++i) a.pos[i] = in->odom_pos[i];
  a.nCorner = in->n_corner_last;
  a.nSurf = in->n_surf_last;
  a.nOutlier = in->n_outlier_last;
  a.stamp = in->stamp;
  int moFront = x->moImu.front;
  a.imuOn = x->moImu.at(in->stamp, x->cfg.scan_period, &a.imuRoll, &a.imuPitch, &moFront) ? 1 : 0;
  if (!a.imuOn) a.imuRoll = a.imuPitch = 0.f;
  const bool lcMode = x->moOpts.loop_closure_enable && !x->moFixed;
  if (lcMode) {
    const int st = lc_recent_plan(x, a);
    if (st != LEGO_OK) return st;
  }
  const int rs = mo_step_device(m, a, x->moFixed, x->cfg.surrounding_keyframe_search_radius, s);
  switch (rs) {
    case MO_OK: break;
    case MO_E_STORE_FULL:  // sticky: the stream's keyframe history is incomplete from here on
      x->moStoreFull = true;
      set_err("scan-to-map: the keyframe store is full (%d keyframes / %d arena points); lego_reset to go on",
              m.kf.kcap, m.kf.acap);
      return LEGO_E_CAPACITY;
    case MO_E_RADIUS_HITS:  // this step only; nothing of it ran
      set_err("scan-to-map: more than 8192 key poses within surroundingKeyframeSearchRadius");
      return LEGO_E_CAPACITY;
    case MO_E_MAP_CAP:  // this step only; nothing of it ran
      set_err("scan-to-map: the surrounding map exceeds %d points", m.fromMapCap);
      return LEGO_E_CAPACITY;
    default:
      set_err("scan-to-map launch failed");
      return LEGO_E_DEVICE;
  }
  MoState hs;
  MoCounts hc;
  int meta[kKfMeta] = {};
  {  // the step's state, counts and keyframe words in one k_fetch (pinned staging)
    unsigned char* hb = (unsigned char*)x->h_moRes;
    const size_t oc = (sizeof(MoState) + 15) & ~(size_t)15, om = oc + ((sizeof(MoCounts) + 15) & ~(size_t)15);
    FetchBuilder F;
    F.add(m.st, hb, nullptr, sizeof(MoState), 1, sizeof(MoState));
    F.add(m.cnt, hb + oc, nullptr, sizeof(MoCounts), 1, sizeof(MoCounts));
    if (!x->moFixed) F.add(m.kf.meta, hb + om, nullptr, sizeof(meta), 1, sizeof(meta));
    HIPCHK(F.run(s));
    std::memcpy(&hs, hb, sizeof(hs));
    std::memcpy(&hc, hb + oc, sizeof(hc));
    if (!x->moFixed) std::memcpy(meta, hb + om, sizeof(meta));
  }
  mo_evprof_print(m);
  if (hc.derr) {  // a VoxelGrid sort handed back a payload outside its cloud (MoCounts::derr)
    HIPCHK(hipMemsetAsync(&m.cnt->derr, 0, sizeof(int), s));
    set_err("scan-to-map: a VoxelGrid sort returned a payload outside its cloud (device fault)");
    return LEGO_E_DEVICE;
  }
  if (meta[KF_OVF]) {  // saveKeyFramesAndFactor of this very step found the store full (k_kf_save)
    x->moStoreFull = true;
    set_err("scan-to-map: the keyframe store is full (%d keyframes / %d arena points): this step's keyframe "
            "was not saved; lego_reset to go on", m.kf.kcap, m.kf.acap);
    return LEGO_E_CAPACITY;
  }
  if (lcMode) {
    const int st = lc_after_step(x, hs, meta[KF_SAVED], meta[KF_K]);
    if (st != LEGO_OK) return st;
  } else if (!x->moFixed && meta[KF_SAVED]) {  // the key pose as iSAM2's estimate of the chain
    float t[6];
    kf_chain_estimate(hs, meta[KF_K], t);
    const int st = kf_put_estimate(x, hs, meta[KF_K], t);
    if (st != LEGO_OK) return st;
  }
  if (hs.optimized) x->moImu.front = moFront;  // transformUpdate ran (:1345)
  out->processed = 1;
  out->optimized = hs.optimized;
  out->iterations = hs.iterations;
  for (int i = 0; i < 6; ++i) {
    out->transform_tobe_mapped[i] = hs.transformTobeMapped[i];
    out->transform_aft_mapped[i] = hs.transformAftMapped[i];
    out->transform_bef_mapped[i] = hs.transformBefMapped[i];
  }
  out->n_corner_map_ds = hc.cornerMapDS;
  out->n_surf_map_ds = hc.surfMapDS;
  out->n_corner_scan_ds = hc.cornerDS;
  out->n_surf_scan_ds = hc.surfTotalDS;
  out->n_rows_last = hs.rowsLast;
  return LEGO_OK;
}

// ---------------------------------------------------------------- PointCloud2
// Decodes K messages (pcl::fromROSMsg, lego_wire.hip) into the context's
// point buffer, scan k at points [off[k], off[k+1]).  Host data is staged
// through one device copy per message.
static int pc2_stage(lego_ctx* x, const lego_pc2_msg* msgs, int K, bool onDevice, std::vector<int64_t>& off) {
  x->h_desc.resize(K);
  off.assign(K + 1, 0);
  size_t raw = 0;
  uint64_t maxPts = 0;
  for (int k = 0; k < K; ++k) {
    if (pc2_plan(&msgs[k], &x->h_desc[k]) != LEGO_OK) {
      set_err("PointCloud2 %d: bad layout (big-endian, point_step, row_step or a field past point_step)", k);
      return LEGO_E_ARG;
    }
    // imageProjection.cpp:172-176: with useCloudRing a non-dense message is an
    // error; without it removeNaNFromPointCloud (:170) drops its NaN points
    if (!msgs[k].is_dense && x->dc.ringRow) {
      set_err("PointCloud2 %d is not dense (is_dense = false)", k);
      return LEGO_E_NOT_DENSE;
    }
    const uint64_t n = (uint64_t)msgs[k].height * msgs[k].width;
    if (n == 0) {
      set_err("PointCloud2 %d is empty", k);
      return LEGO_E_ARG;
    }
    if (n > (uint64_t)x->maxPoints) {
      set_err("PointCloud2 %d has %llu points > capacity %d", k, (unsigned long long)n, x->maxPoints);
      return LEGO_E_CAPACITY;
    }
    if (!msgs[k].data) return LEGO_E_ARG;
    x->h_desc[k].outBase = (uint64_t)off[k];
    off[k + 1] = off[k] + (int64_t)n;
    raw += (size_t)msgs[k].height * msgs[k].row_step;
    maxPts = std::max(maxPts, n);
  }
  if (!onDevice) {
    if (raw > x->rawCap) {
      if (x->d_raw) HIPCHK(hipFree(x->d_raw));
      x->d_raw = nullptr;
      x->rawCap = 0;
      HIPCHK(hipMalloc(&x->d_raw, raw));
      x->rawCap = raw;
    }
    size_t o = 0;
    for (int k = 0; k < K; ++k) {
      const size_t bytes = (size_t)msgs[k].height * msgs[k].row_step;
      HIPCHK(hipMemcpyAsync(x->d_raw + o, msgs[k].data, bytes, hipMemcpyHostToDevice, x->stream));
      x->h_desc[k].data = x->d_raw + o;
      o += bytes;
    }
  }
  HIPCHK(hipMemcpyAsync(x->d_desc, x->h_desc.data(), sizeof(Pc2Desc) * K, hipMemcpyHostToDevice, x->stream));
  if (launch_pc2_decode(x->d_desc, K, maxPts, x->d_pts, x->stream) != 0) {
    set_err("PointCloud2 decode launch failed");
    return LEGO_E_DEVICE;
  }
  HIPCHK(hipMemcpyAsync(x->d_off, off.data(), sizeof(int64_t) * (K + 1), hipMemcpyHostToDevice, x->stream));
  return LEGO_OK;
}

int lego_pc2_decode(lego_ctx* x, const lego_pc2_msg* msg, lego_point_xyzir* out, int32_t cap, int32_t* n_out) {
  if (!x || !msg || !out || !n_out) return LEGO_E_ARG;
  HIPCHK(hipSetDevice(x->device));
  std::vector<int64_t> off;
  const int st = pc2_stage(x, msg, 1, false, off);
  if (st != LEGO_OK) return st;
  if (off[1] > cap) return LEGO_E_CAPACITY;
  HIPCHK(hipMemcpyAsync(out, x->d_pts, sizeof(lego_point_xyzir) * off[1], hipMemcpyDeviceToHost, x->stream));
  HIPCHK(hipStreamSynchronize(x->stream));
  *n_out = (int32_t)off[1];
  return LEGO_OK;
}

int lego_ip_process_pc2(lego_ctx* x, const lego_pc2_msg* msg, uint32_t flags, lego_ip_out* out) {
  if (!x || !msg || !out) return LEGO_E_ARG;
  if (x->inflight) {  // before the decode, which writes the staging points a batch in flight may read
    set_err("node-shaped call while batches are in flight (lego_odom_batch_wait first)");
    return LEGO_E_STATE;
  }
  HIPCHK(hipSetDevice(x->device));
  std::vector<int64_t> off;
  int st = pc2_stage(x, msg, 1, false, off);
  if (st != LEGO_OK) return st;
  x->stamps.assign(1, msg->stamp);
  const bool gated = (flags & LEGO_IP_GATED) != 0;
  st = run_ip(x, x->d_pts, x->d_off, 1, 1, (flags & LEGO_IP_IMAGES) != 0, out, gated);
  if (st != LEGO_OK) return st;
  x->lastIp = *out;
  x->lastIpDevice = true;
  return LEGO_OK;
}

int lego_odom_batch_pc2(lego_ctx* x, const lego_pc2_msg* msgs, int32_t nscans, int32_t on_device,
                        lego_pose_rec* recs) {
  if (!x || !msgs || nscans <= 0 || !recs) return LEGO_E_ARG;
  if (nscans > x->maxBatch) {
    set_err("batch of %d scans > context capacity %d", nscans, x->maxBatch);
    return LEGO_E_CAPACITY;
  }
  HIPCHK(hipSetDevice(x->device));
  std::vector<int64_t> off;
  const int st = pc2_stage(x, msgs, nscans, on_device != 0, off);
  if (st != LEGO_OK) return st;
  std::vector<double> stamps(nscans);
  for (int k = 0; k < nscans; ++k) stamps[k] = msgs[k].stamp;
  return lego_odom_batch(x, x->d_pts, x->d_off, stamps.data(), nscans, 1, recs);
}

// ---------------------------------------------------------------- hand-off packet
// Packs the last waited batch into dst (cap bytes) or, dst == NULL, into the
// context's buffer, on the hand-off stream (the batch is complete: no other
// stream's work is waited for).
static int handoff_pack(lego_ctx* x, uint8_t* dst, uint64_t cap, const void** packet, uint64_t* bytes) {
  const int B = x->lastB;
  if (B <= 0 || !x->lastBatch) {
    set_err("lego_handoff_pack: no batch result (lego_odom_batch / lego_odom_batch_wait first)");
    return LEGO_E_STATE;
  }
  const int slot = x->lastBase / x->maxBatch;
  const PackedRec* pk = x->h_pack + (size_t)slot * (x->maxBatch + 1);
  const std::vector<double>& stamps = x->slotStamps[slot];  // the waited batch's, whatever was submitted since
  const size_t head = sizeof(lego_handoff_hdr) + sizeof(lego_handoff_scan) * (size_t)B;
  x->h_handoffHead.assign(head, 0);
  lego_handoff_hdr* h = reinterpret_cast<lego_handoff_hdr*>(x->h_handoffHead.data());
  lego_handoff_scan* e = reinterpret_cast<lego_handoff_scan*>(h + 1);
  uint64_t off = head, npub = 0;
  for (int k = 0; k < B; ++k) {
    const PackedRec& p = pk[k];
    lego_pose_rec& r = e[k].rec;
    r.stamp = k < (int)stamps.size() ? stamps[k] : 0.0;
    for (int i = 0; i < 6; ++i) { r.transform_sum[i] = p.sum[i]; e[k].transform_cur[i] = p.cur[i]; }
    r.n_segmented = p.ns;
    r.n_sharp = p.cnt[0]; r.n_less_sharp = p.cnt[1]; r.n_flat = p.cnt[2]; r.n_less_flat = p.cnt[3];
    r.odom_valid = p.valid;
    r.flags = p.flags;
    e[k].publish_to_mapping = p.pub;
    e[k].offset = off;
    if (p.pub) {  // publishCloudsLast: less-sharp / less-flat after TransformToEnd, the outliers
      e[k].n_corner_last = p.cnt[1];
      e[k].n_surf_last = p.cnt[3];
      e[k].n_outlier_last = p.nout;
      off += sizeof(lego_point_xyzi) * (uint64_t)(p.cnt[1] + p.cnt[3] + p.nout);
      ++npub;
    }
  }
  h->magic = LEGO_HANDOFF_MAGIC;
  h->version = 1;
  h->nscans = B;
  h->npub = (int32_t)npub;
  h->bytes = off;
  *bytes = off;
  if (!packet && !dst) return LEGO_OK;  // lego_handoff_pack_into size query
  if (dst && cap < off) {
    set_err("lego_handoff_pack_into: %llu bytes needed, %llu given", (unsigned long long)off,
            (unsigned long long)cap);
    return LEGO_E_CAPACITY;
  }
  if (!dst) {
    if (x->handoffFenced) {  // a lego_comm send still reads the buffer (lego_handoff_fence)
      HIPCHK(hipEventSynchronize(x->handoffFence));
      x->handoffFenced = false;
    }
    if (off > x->handoffCap) {
      if (x->d_handoff) HIPCHK(hipFree(x->d_handoff));
      x->d_handoff = nullptr;
      x->handoffCap = 0;
      HIPCHK(hipMalloc(&x->d_handoff, off));
      x->handoffCap = off;
    }
    dst = x->d_handoff;
  }
  if (!x->hstream) HIPCHK(hipStreamCreateWithFlags(&x->hstream, hipStreamNonBlocking));
  hipStream_t s = x->hstream;
  HIPCHK(hipMemcpyAsync(dst, x->h_handoffHead.data(), head, hipMemcpyHostToDevice, s));
  launch_pack_handoff(bb_slice(x->bb, x->dc, x->lastBase, B), ob_slice(x->ob, x->dc, x->lastBase, 0, x->nStreams), B,
                      x->dc.P, dst, s);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(s));
  if (packet) *packet = dst;
  return LEGO_OK;
}

// lego_comm.hip: the packet buffer is read by a send enqueued on stream s;
// the next pack into it waits for that point of s.
int lego_handoff_fence(lego_ctx* x, hipStream_t s) {
  if (!x->handoffFence) HIPCHK(hipEventCreateWithFlags(&x->handoffFence, hipEventDisableTiming));
  HIPCHK(hipEventRecord(x->handoffFence, s));
  x->handoffFenced = true;
  return LEGO_OK;
}

int lego_handoff_pack(lego_ctx* x, const void** packet, uint64_t* bytes) {
  if (!x || !packet || !bytes) return LEGO_E_ARG;
  HIPCHK(hipSetDevice(x->device));
  return handoff_pack(x, nullptr, 0, packet, bytes);
}

int lego_handoff_pack_into(lego_ctx* x, void* dst, uint64_t cap, uint64_t* bytes) {
  if (!x || !bytes) return LEGO_E_ARG;
  HIPCHK(hipSetDevice(x->device));
  return handoff_pack(x, static_cast<uint8_t*>(dst), dst ? cap : 0, nullptr, bytes);
}

int lego_handoff_unpack(const void* packet, uint64_t bytes, int32_t k, lego_pose_rec* rec, lego_fa_out* out) {
  if (!packet || bytes < sizeof(lego_handoff_hdr)) return LEGO_E_ARG;
  const uint8_t* base = static_cast<const uint8_t*>(packet);
  const lego_handoff_hdr* h = reinterpret_cast<const lego_handoff_hdr*>(base);
  if (h->magic != LEGO_HANDOFF_MAGIC || h->version != 1 || h->bytes != bytes || h->nscans < 0 ||
      sizeof(lego_handoff_hdr) + sizeof(lego_handoff_scan) * (uint64_t)h->nscans > bytes) {
    set_err("lego_handoff_unpack: not a version-1 hand-off packet of %llu bytes", (unsigned long long)bytes);
    return LEGO_E_ARG;
  }
  if (k < 0 || k >= h->nscans) return LEGO_E_ARG;
  const lego_handoff_scan& e = reinterpret_cast<const lego_handoff_scan*>(h + 1)[k];
  const uint64_t n = (uint64_t)e.n_corner_last + (uint64_t)e.n_surf_last + (uint64_t)e.n_outlier_last;
  if (e.n_corner_last < 0 || e.n_surf_last < 0 || e.n_outlier_last < 0 || e.offset > bytes ||
      n * sizeof(lego_point_xyzi) > bytes - e.offset) {
    set_err("lego_handoff_unpack: scan %d's clouds lie outside the packet", k);
    return LEGO_E_ARG;
  }
  if (rec) *rec = e.rec;
  if (out) {
    std::memset(out, 0, sizeof(*out));
    out->stamp = e.rec.stamp;
    out->n_sharp = e.rec.n_sharp;
    out->n_less_sharp = e.rec.n_less_sharp;
    out->n_flat = e.rec.n_flat;
    out->n_less_flat = e.rec.n_less_flat;
    out->odom_valid = e.rec.odom_valid;
    for (int i = 0; i < 6; ++i) {
      out->transform_sum[i] = e.rec.transform_sum[i];
      out->transform_cur[i] = e.transform_cur[i];
    }
    odom_quat(e.rec.transform_sum, out->odom_quat, out->odom_pos);  // publishOdometry (:1727-1744)
    out->publish_to_mapping = e.publish_to_mapping;
    if (e.publish_to_mapping) {
      const lego_point_xyzi* p = reinterpret_cast<const lego_point_xyzi*>(base + e.offset);
      out->corner_last = p;
      out->n_corner_last = e.n_corner_last;
      out->surf_last = p + e.n_corner_last;
      out->n_surf_last = e.n_surf_last;
      out->outlier_last = p + e.n_corner_last + e.n_surf_last;
      out->n_outlier_last = e.n_outlier_last;
    }
  }
  return LEGO_OK;
}

// ---------------------------------------------------------------- transformFusion
int lego_fusion_odometry(lego_ctx* x, const lego_fa_out* odom, lego_fusion_out* out) {
  if (!x || !odom || !out) return LEGO_E_ARG;
  x->fusion.odometry(odom->odom_quat, odom->odom_pos);
  std::memset(out, 0, sizeof(*out));
  out->stamp = odom->stamp;
  for (int i = 0; i < 6; ++i) out->transform_mapped[i] = x->fusion.transformMapped[i];
  odom_quat(x->fusion.transformMapped, out->quat, out->pos);  // the same setRPY + axis shuffle (:187-196)
  return LEGO_OK;
}

int lego_fusion_aft_mapped(lego_ctx* x, const lego_mo_out* mo) {
  if (!x || !mo) return LEGO_E_ARG;
  if (!mo->processed) return LEGO_OK;  // nothing was published
  double q[4], pos[3];
  odom_quat(mo->transform_aft_mapped, q, pos);  // publishTF (mapOptmization.cpp:656-665)
  x->fusion.aft_mapped(q, pos, mo->transform_bef_mapped);
  return LEGO_OK;
}

int lego_odom_profile(lego_ctx* x, int32_t enable, uint64_t* out32) {
  if (!x) return LEGO_E_ARG;
  HIPCHK(hipSetDevice(x->device));
  if (out32) {
    HIPCHK(hipMemcpy(out32, x->d_prof, 32 * sizeof(uint64_t), hipMemcpyDeviceToHost));
  }
  if (enable >= 0) {
    x->profOn = enable != 0;
    HIPCHK(hipMemset(x->d_prof, 0, 48 * sizeof(uint64_t)));
  }
  return LEGO_OK;
}

int lego_extract_profile(lego_ctx* x, uint64_t* out8) {
  if (!x || !out8) return LEGO_E_ARG;
  HIPCHK(hipSetDevice(x->device));
  HIPCHK(hipMemcpy(out8, x->d_prof + 32, 8 * sizeof(uint64_t), hipMemcpyDeviceToHost));
  return LEGO_OK;
}

int lego_stage_times(lego_ctx* x, const char** names, float* ms, int32_t cap, int32_t* n) {
  if (!x || !n) return LEGO_E_ARG;
  if (cap == 0) {  // toggle: cap 0 with names == NULL enables/disables the timer
    x->tm.enabled = x->otm.enabled = ms != nullptr;
    *n = 0;
    return LEGO_OK;
  }
  const int m = std::min<int>((int)x->tnames.size(), cap);
  for (int i = 0; i < m; ++i) {
    if (names) names[i] = x->tnames[i].c_str();
    if (ms) ms[i] = x->tms[i];
  }
  *n = m;
  return LEGO_OK;
}

}  // extern "C"
