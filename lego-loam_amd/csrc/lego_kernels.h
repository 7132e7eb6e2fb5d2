// lego_kernels.h — host-side launchers of the gfx950 kernels + stage timer.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

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
  // Collapses repeated names into totals (appended to names / ms, with the
  // number of intervals per name in counts; "__gap__" marks time that belongs
  // to no stage).  Call after a stream sync.
  void collect(std::vector<std::string>& names, std::vector<float>& ms, std::vector<int>& counts) const {
    for (size_t i = 0; i + 1 < used_; ++i) {
      if (names_[i] == "__gap__") continue;
      float t = 0;
      if (hipEventElapsedTime(&t, events_[i], events_[i + 1]) != hipSuccess) t = 0;
      size_t k = 0;
      for (; k < names.size(); ++k)
        if (names[k] == names_[i]) break;
      if (k == names.size()) {
        names.push_back(names_[i]);
        ms.push_back(0);
        counts.push_back(0);
      }
      ms[k] += t;
      counts[k] += 1;
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

// HBM form of the two NN indexes over one last cloud (sensors whose working
// set does not fit LDS); see lego_odom.hip.
struct NNIndexBufs {
  float4* gPts;  // [cap] the cloud in fine-grid bucket order, .w = the point's index (int bits);
                 // the bucket ends live in LDS (lego_odom.hip, hbm_grid_ends)
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
  int nnCornerNum, nnSurfNum;  // sizes of the clouds the NN indexes were built on
  int frameCount;
  // HBM copy holding the current last clouds: 0 / 1 a workgroup-private
  // buffer (LDS-resident sensors), >= 2 the stream's ring slot curBuf - 2
  // (HBM-resident sensors, OdomBufs::ring)
  int curBuf;
  int snapBuf;   // the copy the indexes were built over (== curBuf unless stale), same encoding
  int resident;  // current last clouds (and indexes) are LDS-resident
  // LDS-resident sensors: hand-offs so far (the hand-off exchange's tag; its
  // granules are zeroed with it).  Ring sensors: ring picks so far (ring_next).
  unsigned seq;
};

// Device buffers of the odometry kernel for S independent streams (a fleet;
// S = 1 for a plain context).  Arrays marked [G x] hold one private copy per
// workgroup of the launch (the G workgroups of a stream redundantly run the
// same serial chain and split only the NN searches); they and st are [S x]
// over the streams.  The kernel offsets them.
struct OdomBufs {
  OdomState* st;          // [S] the state after the last launch (written by each stream's lead workgroup)
  // [S] read-only copy of st taken on the odometry stream before each launch:
  // every workgroup starts from it, so one dispatched after its lead finished
  // still sees the launch's input state (launch_odom)
  OdomState* stIn;
  float4* cornerLast[2];  // [G x capCorner] double-buffered: current / stale snapshot
  float4* surfLast[2];    // [G x capSurf]
  NNIndexBufs nC, nS;     // [G x] HBM indexes (sensors too large for LDS)
  int* qi;                // [G x 3 * capQ] HBM correspondences
  int gTC, gTS;           // bucket caps of the HBM-resident grids
  int capCorner, capSurf, capQ;
  int G;                  // workgroups per stream
  int S;                  // streams
  int roundsCap;          // exchange slots (NN rounds) per stream and launch
  // LDS-resident clouds without hash grids (host: G large enough that an NN
  // round is about one query per wave): the closest point is an exhaustive
  // pass over the LDS cloud and the index build keeps only the key tables
  int gridless;
  // set in the kernel: this workgroup's index within its stream.  On the
  // host: -1, or the diagnostic LEGO_ODOM_SILENT_WG of a single-stream
  // context, a workgroup that uses private copies of both exchanges (placed
  // after the shared ones, distances in xerr[2], xerr[3]): the others never see
  // its results and take its share through the steal-on-timeout paths, and it
  // takes theirs the same way (tests)
  int wg;
  // diagnostic LEGO_ODOM_LATE_WG of a single-stream context (-1: none): that
  // workgroup waits at its start until the lead has written the launch's
  // final state (xerr[1], zeroed per launch), so it replays the whole chain
  // from the input state and the published rounds (tests)
  int late;
  // exchange: an error word shared by the streams (zeroed per batch), then
  // per stream roundsCap x capQ granules (zeroed per launch)
  void* xblock;
  size_t xbytes;
  unsigned* xerr;
  unsigned long long* xg;
  // hand-off exchange: per stream 2 (hand-off parity) x 3 x capH granules
  // {seq, TransformToEnd'ed x / y / z}, zeroed at creation and reset
  unsigned long long* xh;
  size_t xhBytes;
  int capH;  // capSurf + capCorner

  // Sensors whose last clouds do not fit LDS (HDL-64E, VLS-128): the stream's
  // ONE copy of each hand-off's TransformToEnd'ed clouds and of their grids,
  // as featureAssociation.cpp:1759-1815 keeps one per stream, instead of a
  // private copy per workgroup.  ringR slots per stream, ringStride bytes
  // each: control words (per share: claim / done of the two phases), the key
  // tables and bucket counts / cursors (agent-scope atomics), then the clouds
  // in index order (P) and in bucket order (Q).  Each workgroup transforms and
  // stores its share of the points; a share whose owner has not claimed it in
  // kStealTicks is done by the waiting workgroup.  Within a launch no slot is
  // written twice and the indexes' snapshot slot is skipped (ring_next), so a
  // slower workgroup never reads a rewritten slot; k_ring_prep zeroes the
  // control words of the slots a launch can pick.  ring == nullptr: the
  // LDS-resident sensors' private path.
  unsigned char* ring;     // [S x copies x ringR x ringStride]
  size_t ringStride;       // bytes per slot
  size_t ringCtl;          // bytes of a slot's control words (zeroed per pick)
  size_t ringCopy;         // the diagnostic silent workgroup's private ring (bytes past the stream's), else 0
  int ringR;

  // integrateTransformation off the chain (G > 1): one more workgroup per
  // stream, launched after the S x G chain workgroups, integrates every scan
  // of the launch in order from the lead's transformCur, published per scan
  // as six 8-byte granules {tag, float} (intX, zeroed per launch; tag =
  // 2 (b + 1) + valid), and writes sumOut and the state's transformSum.  The
  // chain's TransformToEnd then runs on all eight waves.  0: wave 0 of every
  // chain workgroup integrates beside TransformToEnd (G = 1, LEGO_ODOM_INTEG=0).
  int integ;
  unsigned long long* intX;  // [B*6]


  // per-scan outputs of the batch (workgroup 0)
  float* sumOut;        // [B*6]
  float* curOut;        // [B*6]
  int* validOut;        // [B]
  int* pubOut;          // [B]
  float4* cornerEnd;    // [B*capLS]  less-sharp after TransformToEnd
  float4* surfEnd;      // [B*P]      less-flat after TransformToEnd
  int capLS;
};

// Ring slot layout (OdomBufs::ring), shared by the host's allocation and the
// kernels: [claimA, doneA, claimB, doneB] x G words, the key tables
// (kRingKey words), the bucket counts and cursors (gTS + gTC words each), then
// P and Q (capH points each).  Everything before P is a slot's control words.
constexpr int kRingKey = 4 * kMaxRings + 2;
__host__ __device__ inline size_t ring_al(size_t x) { return (x + 255) & ~(size_t)255; }
__host__ __device__ inline size_t ring_ctl_bytes(int G, int gTS, int gTC) {
  return ring_al((size_t)16 * G) + ring_al((size_t)4 * kRingKey) + 2 * ring_al((size_t)4 * (gTS + gTC));
}
__host__ __device__ inline size_t ring_stride(int G, int gTS, int gTC, int capH) {
  return ring_ctl_bytes(G, gTS, gTC) + 2 * ring_al((size_t)16 * capH);
}
// Ring slots per stream for launches of up to K scans per stream: K picks,
// the snapshot's slot and the launch's first current slot are never rewritten.
__host__ __device__ inline int ring_slots(int K) { return K + 3; }

// The launch-shape switches of a context (lego_ctx_opts, fixed at creation):
// host only, never a kernel argument.
struct LaunchOpts {
  int cclTiles = 1;       // lego_ctx_opts::ccl_tiles
  int lfvWave = 1;        // ::lfv_wave
  int lfvBlockRings = 0;  // ::lfv_block_rings
  int lfvWide = -1;       // ::lfv_wide
  int faSyncCheck = 0;    // ::fa_synccheck
  int ipFused = 1;        // ::ip_fused
};

void launch_gated(const BatchBufs& bb, const DevCfg& c, const GatedBufs& gb, hipStream_t s);
void launch_ip(const BatchBufs& bb, const DevCfg& c, int B, int want_labels, hipStream_t s,
               StageTimer* tm, const LaunchOpts& lo);
// launch_ip of B scans takes k_ip_lds, which clears each scan's bb.bad word
// itself (the caller's fill of bb.bad is then redundant)
bool ip_clears_bad(const DevCfg& c, int B, const LaunchOpts& lo);
// B = S x K scans, stream-major (scans [s*K, s*K + K) are stream s's, in
// order); d_carry[S].
// side (node calls, B = 1): the per-ring less-flat VoxelGrid and its
// compaction go to that stream after `fork` is recorded on s, beside the
// odometry launched next on s, each ring counted into lfReady[b] (release;
// zeroed here first); the caller passes lfReady to launch_odom and joins side
// into s before reading f_lflat.  null: everything on s.
void launch_fa(const BatchBufs& bb, const DevCfg& c, int B, int S, FaCarry* d_carry, hipStream_t s,
               StageTimer* tm, const LaunchOpts& lo, hipStream_t side = nullptr, hipEvent_t fork = nullptr,
               unsigned* lfReady = nullptr);
// K scans per stream over ob.S streams (the caller zeroes *ob.xerr once per
// batch).  Returns 0 on a successful launch.  lfReady (a node call, launch_fa
// with a side stream): the scan's less-flat VoxelGrid is still running when
// the LM starts; the hand-off, its only reader (publishCloudsLast,
// featureAssociation.cpp:1759-1815), first waits until lfReady[b] counts
// every ring (bounded: lfTicks of the 100 MHz wall clock, 0 = none, then
// bad[b] |= kBadLfLate and no less-flat points; the host then fails the call
// and requires lego_reset).  The lead workgroup decides and publishes the
// decision in lfReady[b]'s flag bits (kLfDecided*), which every other
// workgroup follows.
int launch_odom(const BatchBufs& bb, const OdomBufs& ob, const DevCfg& c, int K, hipStream_t s,
                StageTimer* tm, unsigned long long* prof, unsigned* lfReady = nullptr,
                unsigned long long lfTicks = 0);
int odom_workgroups(int N, int cusAvailable);
// sensors whose last clouds never fit LDS: the stream keeps one ring copy (OdomBufs::ring)
bool odom_ring_sensor(int N);
// workgroups per stream from which the LDS-resident odometry runs without grids
constexpr int kGridlessMinWG = 16;

// One scan's pose-record fields, gathered on the device so a batch returns in
// one copy; slot B of the array carries the exchange timeout word in `bad`.
struct PackedRec {
  float sum[6];
  int ns, cnt[4], valid, flags, bad;
  float cur[6];
  int pub, nout;  // publish_to_mapping, outlier cloud size (the hand-off packet)
};
// The hand-off packet's clouds (lego_handoff_pack): scan b of the batch reads
// its lego_handoff_scan entry at packet + 32 + 128 b.
void launch_pack_handoff(const BatchBufs& bb, const OdomBufs& ob, int B, int maxPts, uint8_t* packet, hipStream_t s);
void launch_pack_recs(const BatchBufs& bb, const OdomBufs& ob, int B, PackedRec* out, hipStream_t s);
// HBM index sizes for clouds of up to capCorner / capSurf points.
void odom_index_caps(int capCorner, int capSurf, int* gTC, int* gTS);

}  // namespace lego
