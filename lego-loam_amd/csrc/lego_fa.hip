// lego_fa.hip — featureAssociation feature extraction on gfx950.
//
//   k_fa_half     1 lane / segmented point: the !halfPassed orientation test;
//                 the first point that flips halfPassed is an atomicMin
//                 (adjustDistortion, featureAssociation.cpp:491-523)
//   k_fa_point    1 lane / point: deskew (axis swap + relTime), 11-tap
//                 curvature (:621-641), occlusion marks as a gather (:643-678)
//   k_extract     1 workgroup / (scan, ring): per sector a bitonic sort of
//                 (curvature, index) in LDS — libstdc++ introsort port when the
//                 sector holds ties (equal keys are ordered by std::sort's
//                 unstable algorithm) — then the edge/flat picking scans as
//                 wave ballots, the less-flat set and the per-ring 0.2 m
//                 VoxelGrid (:680-784).  Rings are independent except through
//                 the ring-0 carry: extraction runs for every
//                 scan under the steady carry S*; k_fa_fixup walks the batch in
//                 stream order and re-runs ring 0 where the real carry differs.
//   k_fa_compact  concatenates the per-ring slots in ring order.
#include <climits>
#include <cstdio>

#include "lego_device.h"
#include "lego_introsort.h"
#include "lego_vgsort.h"
#include "lego_vgsort_wave.h"
#include "lego_kernels.h"

namespace lego {

// ---------------------------------------------------------------- deskew
__device__ __forceinline__ float ori_not_half(float ori, float so) {
  if ((double)ori < (double)so - M_PI / 2) ori = (float)((double)ori + 2 * M_PI);
  else if ((double)ori > (double)so + M_PI * 3 / 2) ori = (float)((double)ori - 2 * M_PI);
  return ori;
}

__global__ void k_fa_half(BatchBufs bb, DevCfg c) {
  const int b = blockIdx.y;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= bb.ns[b]) return;
  const float4 p = bb.seg[(size_t)b * c.P + i];
  const float so = bb.orient[3 * b];
  const float ori = ori_not_half(-lego_atan2f(p.y, p.x), so);        // point.x = y, point.z = x
  if ((double)(ori - so) > M_PI) atomicMin(&bb.firsthalf[b], i);
}

__device__ __forceinline__ bool occ_fwd(const float* r, const uint32_t* col, int i, int ns) {
  if (i < 5 || i >= ns - 6) return false;
  const int cd = abs((int)(col[i + 1] - col[i]));
  return cd < 10 && (double)(r[i] - r[i + 1]) > 0.3;
}
__device__ __forceinline__ bool occ_bwd(const float* r, const uint32_t* col, int i, int ns) {
  if (i < 5 || i >= ns - 6) return false;
  const int cd = abs((int)(col[i + 1] - col[i]));
  return cd < 10 && !((double)(r[i] - r[i + 1]) > 0.3) && (double)(r[i + 1] - r[i]) > 0.3;
}
__device__ __forceinline__ bool occ_par(const float* r, int i, int ns) {
  if (i < 5 || i >= ns - 6) return false;
  const float d1 = lfabsf(r[i - 1] - r[i]), d2 = lfabsf(r[i + 1] - r[i]);
  return (double)d1 > 0.02 * (double)r[i] && (double)d2 > 0.02 * (double)r[i];
}

// ---------------------------------------------------------------- IMU
// adjustDistortion's queue lookup (:526-566) for the point at timeScanCur +
// pointTime: the first entry after imuPointerLastIteration stamped later than
// the point (or imuPointerLast), interpolated with the entry before it.
struct ImuAt {
  float roll, pitch, yaw, vx, vy, vz;
  float rf, rb;  // ratioFront / ratioBack (interpolated case)
  int f, b;
  bool exact;    // timeScanCur + pointTime > imuTime[front]: no interpolation
};
__device__ __forceinline__ void imu_lookup(const ImuSnap& S, float pointTime, ImuAt& a) {
  const double t = S.stamp + pointTime;
  int f = S.lastIter;
  while (f != S.last) {
    if (t < S.time[f]) break;
    f = (f + 1) % kImuQ;
  }
  a.f = f;
  a.exact = t > S.time[f];
  if (a.exact) {
    a.roll = S.v[IV_ROLL][f]; a.pitch = S.v[IV_PITCH][f]; a.yaw = S.v[IV_YAW][f];
    a.vx = S.v[IV_VX][f]; a.vy = S.v[IV_VY][f]; a.vz = S.v[IV_VZ][f];
    return;
  }
  const int b = (f + kImuQ - 1) % kImuQ;
  a.b = b;
  a.rf = (float)((S.stamp + pointTime - S.time[b]) / (S.time[f] - S.time[b]));
  a.rb = (float)((S.time[f] - S.stamp - pointTime) / (S.time[f] - S.time[b]));
  a.roll = S.v[IV_ROLL][f] * a.rf + S.v[IV_ROLL][b] * a.rb;
  a.pitch = S.v[IV_PITCH][f] * a.rf + S.v[IV_PITCH][b] * a.rb;
  const float yf = S.v[IV_YAW][f], yb = S.v[IV_YAW][b];
  if ((double)(yf - yb) > M_PI) a.yaw = (float)(yf * a.rf + (yb + 2 * M_PI) * a.rb);
  else if ((double)(yf - yb) < -M_PI) a.yaw = (float)(yf * a.rf + (yb - 2 * M_PI) * a.rb);
  else a.yaw = yf * a.rf + yb * a.rb;
  a.vx = S.v[IV_VX][f] * a.rf + S.v[IV_VX][b] * a.rb;
  a.vy = S.v[IV_VY][f] * a.rf + S.v[IV_VY][b] * a.rb;
  a.vz = S.v[IV_VZ][f] * a.rf + S.v[IV_VZ][b] * a.rb;
}

// Point 0 of each scan (the i == 0 branch of :568-610): the start attitude and
// velocity, their sines / cosines, and the angular rotation at point 0.  One
// lane per scan.  Defaults rollCur.. to the start values (a one-point scan).
__global__ void k_fa_imu_start(BatchBufs bb, DevCfg c) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= bb.B) return;
  const ImuSnap& S = bb.imu[b];
  ImuScan o = {};
  const int ns = bb.ns[b];
  o.active = S.last >= 0;
  o.hasFirst = o.active && ns >= 1;
  o.hasLast = o.active && ns >= 2;
  if (o.hasFirst) {
    const float4 p = bb.seg[(size_t)b * c.P];
    const float so = bb.orient[3 * b], od = bb.orient[3 * b + 2];
    const float ori = ori_not_half(-lego_atan2f(p.y, p.x), so);
    const float relTime = (ori - so) / od;
    ImuAt a;
    imu_lookup(S, relTime * c.scan_period, a);
    o.rollStart = a.roll; o.pitchStart = a.pitch; o.yawStart = a.yaw;
    o.veloStart[0] = a.vx; o.veloStart[1] = a.vy; o.veloStart[2] = a.vz;
    if (a.exact) {
      for (int k = 0; k < 3; ++k) o.ar0[k] = S.v[IV_AX + k][a.f];
    } else {
      for (int k = 0; k < 3; ++k) o.ar0[k] = S.v[IV_AX + k][a.f] * a.rf + S.v[IV_AX + k][a.b] * a.rb;
    }
    o.cRS = lego_cosf(o.rollStart); o.cPS = lego_cosf(o.pitchStart); o.cYS = lego_cosf(o.yawStart);
    o.sRS = lego_sinf(o.rollStart); o.sPS = lego_sinf(o.pitchStart); o.sYS = lego_sinf(o.yawStart);
    o.rollCur = o.rollStart; o.pitchCur = o.pitchStart; o.yawCur = o.yawStart;
  }
  bb.imuScan[b] = o;
}

// TransformToStartIMU :365-390 (imuShiftFromStart*Cur stays 0: ShiftToStartIMU
// is never called)
__device__ __forceinline__ float4 to_start_imu(float4 p, const ImuAt& a, const ImuScan& s) {
  const float cr = lego_cosf(a.roll), sr = lego_sinf(a.roll);
  const float cp = lego_cosf(a.pitch), sp = lego_sinf(a.pitch);
  const float cy = lego_cosf(a.yaw), sy = lego_sinf(a.yaw);
  const float x1 = cr * p.x - sr * p.y;
  const float y1 = sr * p.x + cr * p.y;
  const float z1 = p.z;
  const float x2 = x1;
  const float y2 = cp * y1 - sp * z1;
  const float z2 = sp * y1 + cp * z1;
  const float x3 = cy * x2 + sy * z2;
  const float y3 = y2;
  const float z3 = -sy * x2 + cy * z2;
  const float x4 = s.cYS * x3 - s.sYS * z3;
  const float y4 = y3;
  const float z4 = s.sYS * x3 + s.cYS * z3;
  const float x5 = x4;
  const float y5 = s.cPS * y4 + s.sPS * z4;
  const float z5 = -s.sPS * y4 + s.cPS * z4;
  return make_float4(s.cRS * x5 + s.sRS * y5 + 0.0f, -s.sRS * x5 + s.cRS * y5 + 0.0f, z5 + 0.0f, p.w);
}

__global__ void k_fa_point(BatchBufs bb, DevCfg c) {
  const int b = blockIdx.y;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int ns = bb.ns[b];
  if (i >= ns) return;
  const size_t base = (size_t)b * c.P;
  // adjustDistortion (imuPointerLast < 0): :498-523
  const float4 p = bb.seg[base + i];
  const float so = bb.orient[3 * b], eo = bb.orient[3 * b + 1], od = bb.orient[3 * b + 2];
  float ori = -lego_atan2f(p.y, p.x);
  if (i <= bb.firsthalf[b]) {
    ori = ori_not_half(ori, so);
  } else {
    ori = (float)((double)ori + 2 * M_PI);
    if ((double)ori < (double)eo - M_PI * 3 / 2) ori = (float)((double)ori + 2 * M_PI);
    else if ((double)ori > (double)eo + M_PI / 2) ori = (float)((double)ori - 2 * M_PI);
  }
  const float relTime = (ori - so) / od;
  const float inten = (float)(int)p.w + c.scan_period * relTime;
  float4 q = make_float4(p.y, p.z, p.x, inten);
  if (bb.imu && i > 0) {
    ImuScan& is = bb.imuScan[b];
    if (is.active) {
      ImuAt a;
      imu_lookup(bb.imu[b], relTime * c.scan_period, a);
      if (i == ns - 1) {  // the members the scan leaves behind: the last point's
        // VeloToStartIMU :346-363
        float vx = a.vx - is.veloStart[0], vy = a.vy - is.veloStart[1], vz = a.vz - is.veloStart[2];
        const float x1 = is.cYS * vx - is.sYS * vz;
        const float y1 = vy;
        const float z1 = is.sYS * vx + is.cYS * vz;
        const float x2 = x1;
        const float y2 = is.cPS * y1 + is.sPS * z1;
        const float z2 = -is.sPS * y1 + is.cPS * z1;
        is.vfs[0] = is.cRS * x2 + is.sRS * y2;
        is.vfs[1] = -is.sRS * x2 + is.cRS * y2;
        is.vfs[2] = z2;
        is.rollCur = a.roll; is.pitchCur = a.pitch; is.yawCur = a.yaw;
      }
      q = to_start_imu(q, a, is);
    }
  }
  bb.dsk[base + i] = q;
  // calculateSmoothness :624-640
  const float* r = bb.srange + base;
  float cv = 0.f;
  if (i >= 5 && i < ns - 5) {
    const float d = r[i - 5] + r[i - 4] + r[i - 3] + r[i - 2] + r[i - 1] - r[i] * 10 + r[i + 1] +
                    r[i + 2] + r[i + 3] + r[i + 4] + r[i + 5];
    cv = d * d;
  }
  bb.curv[base + i] = cv;
  // markOccludedPoints as a gather: which i' mark index i
  const uint32_t* col = bb.col + base;
  bool m = occ_par(r, i, ns);
  for (int k = i; k <= i + 5 && !m; ++k) m = occ_fwd(r, col, k, ns);
  for (int k = i - 6; k <= i - 1 && !m; ++k) m = occ_bwd(r, col, k, ns);
  bb.pick0[base + i] = m ? 1 : 0;
}

// ---------------------------------------------------------------- extraction
struct ExtractLds {
  float* curv;
  uint16_t* col;
  uint8_t* picked;
  int8_t* label;
  uint8_t* gfl;
  uint16_t* lf;
  uint16_t* perm;
  SmoothEntry* srt;
  SmoothEntry* orig;
  int* misc;
  float* red;
};

__host__ __device__ inline int next_pow2(int x) {
  int m = 1;
  while (m < x) m <<= 1;
  return m;
}

// LDS of one (scan, ring) workgroup, laid out by phase so that six fit a CU
// for VLP-16-class rings (W = H + 32 window positions; the kernel's time
// scales with the resident workgroups: two per CU took 1.86x the time of
// four).  Region A, then region B, then misc / red:
//   sorts    A: the waves' sector scratch          B: curv, perm, gfl
//   picking  A: pick lists [0, 1 KB), the initial  B: curv, perm, gfl
//               picked copy, picked, label, col
//   less-flat                                      B: lf (its tail)
//   less-flat   lf in B's tail (its points go to the ring's slot; the
//               VoxelGrid is k_lf_voxel's)
// col, picked and label are loaded once the sorts are done.
// A sector holds n <= (H + 32) / 6 + 2 entries plus the fallback sort's
// stack (kIntroStack words) behind it.
__host__ __device__ inline int extract_sector_cap(int H) { return next_pow2((H + 32) / 6 + 2 + (kIntroStack + 1) / 2); }
constexpr int kSortWaves = 3;  // waves sorting sectors at once (the scratch holds their sectors)
struct ExtractLayout {
  size_t A, B, colOff, lfOff;  // region sizes; col's offset in A, lf's in B
};
__host__ __device__ inline ExtractLayout extract_layout(int H) {
  const size_t W = (size_t)H + 32;
  ExtractLayout e;
  const size_t sec = (size_t)kSortWaves * extract_sector_cap(H) * 8;
  e.colOff = (1024 + 3 * W + 1) & ~(size_t)1;  // after the pick lists, the picked copy, picked, label
  size_t a = e.colOff + 2 * W;
  if (sec > a) a = sec;
  e.lfOff = (5 * W + 1) & ~(size_t)1;          // over perm / gfl, dead once the walks are done
  e.B = (e.lfOff + 2 * W + 15) & ~(size_t)15;
  e.A = (a + 15) & ~(size_t)15;
  return e;
}
__host__ __device__ inline size_t extract_lds_bytes(int H) {
  const ExtractLayout e = extract_layout(H);
  return e.A + e.B + 64 * 4 + 64 * 4;  // + misc + red
}

__device__ __forceinline__ ExtractLds carve(unsigned char* base, int H) {
  const size_t W = (size_t)H + 32;
  const ExtractLayout e = extract_layout(H);
  ExtractLds L;
  unsigned char* A = base;
  unsigned char* B = base + e.A;
  L.srt = (SmoothEntry*)A;
  L.orig = nullptr;
  L.picked = A + 1024 + W;  // [1024, 1024 + W): the initial picked copy of the speculative walks
  L.label = (int8_t*)(A + 1024 + 2 * W);
  L.col = (uint16_t*)(A + e.colOff);
  L.curv = (float*)B;
  L.perm = (uint16_t*)(B + 4 * W);
  L.gfl = B + 6 * W;
  L.lf = (uint16_t*)(B + e.lfOff);
  L.misc = (int*)(B + e.B);
  L.red = (float*)(B + e.B + 64 * 4);
  return L;
}

enum { M_TIE = 0, M_LF = 1, M_OVF = 2, M_NSH = 3, M_NLS = 4, M_NFL = 5, M_D0 = 6, M_D1 = 7,
       M_MB0 = 8, M_MB1 = 9, M_MB2 = 10, M_PH = 11, M_REWALK = 12, M_P0 = 13, M_WOFF = 16, M_SEC = 24,
       M_NEF = 48 };
// per-sector pick list: 2 sharp, 20 less sharp, 4 flat (featureAssociation.cpp:709-748)
constexpr int kPickListStride = 32;

// Bitonic sort of m (power of two) entries in LDS by value, all threads.
__device__ __forceinline__ void bitonic_entries(SmoothEntry* a, int m) {
  for (int k = 2; k <= m; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int t = threadIdx.x; t < m / 2; t += blockDim.x) {
        const int i = (t / j) * 2 * j + (t % j);
        const int l = i + j;
        const bool up = (i & k) == 0;
        const SmoothEntry x = a[i], y = a[l];
        if ((x.value > y.value) == up) { a[i] = y; a[l] = x; }
      }
      __syncthreads();
    }
  }
}
// The same network by one wave on its own LDS buffer (no block barrier).
__device__ __forceinline__ void wave_sync_lds() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ void wave_bitonic_entries(SmoothEntry* a, int m) {
  const int lane = threadIdx.x & 63;
  for (int k = 2; k <= m; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int t = lane; t < m / 2; t += 64) {
        const int i = (t / j) * 2 * j + (t % j);
        const int l = i + j;
        const bool up = (i & k) == 0;
        const SmoothEntry x = a[i], y = a[l];
        if ((x.value > y.value) == up) { a[i] = y; a[l] = x; }
      }
      wave_sync_lds();
    }
  }
}
// Ordered block compaction helper: returns this thread's exclusive rank among
// flagged threads of the block and the block total (256 threads = 4 waves).
__device__ __forceinline__ int block_rank(bool f, int* woff, int* total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const unsigned long long m = __ballot(f);
  const int r = __popcll(m & ((1ull << lane) - 1));
  if (lane == 0) woff[wave] = __popcll(m);
  __syncthreads();
  int off = 0, tot = 0;
  const int nw = blockDim.x >> 6;
  for (int w = 0; w < nw; ++w) {
    if (w < wave) off += woff[w];
    tot += woff[w];
  }
  __syncthreads();
  *total = tot;
  return off + r;
}

struct RingCtx {
  int b, ring, lo, Wn, ns;
  size_t base;
  float4* osh;
  float4* ols;
  float4* ofl;
};

// neighbour suppression (:720-732, :751-767); negative indices break (the
// reference reads colInd[-1] there — UB; SURVEY.md §9.7 policy).
__device__ __forceinline__ void suppress(const RingCtx& R, volatile uint8_t* picked, const uint16_t* col, int ind) {
  const int w = ind - R.lo;
  picked[w] = 1;
  for (int l = 1; l <= 5; l++) {
    const int q = w + l;
    if (q >= R.Wn) break;
    if (abs((int)col[q] - (int)col[q - 1]) > 10) break;
    picked[q] = 1;
  }
  for (int l = -1; l >= -5; l--) {
    const int q = w + l;
    if (ind + l < 0 || q < 0) break;
    if (abs((int)col[q] - (int)col[q + 1]) > 10) break;
    picked[q] = 1;
  }
}

// the reference's cloudSmoothness[k].ind after the sector sort (ep itself is
// not sorted, :699): perm holds window positions, 0xFFFF the phantom entry
__device__ __forceinline__ int entry_ind(const uint16_t* perm, int sp, int ep, int k, int lo, int ph) {
  if (k == ep) return ep;
  const int v = perm[k - sp];
  return v == 0xFFFF ? ph : v + lo;
}

__device__ __forceinline__ bool in_win(const RingCtx& R, int ind) {
  return ind >= R.lo && ind - R.lo < R.Wn;
}

__device__ __forceinline__ void extract_ring(const BatchBufs& bb, const DevCfg& c, int b, int ring, FaCarry* carry,
                             const ExtractLds& L) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ns = bb.ns[b];
  const int s = bb.sri[b * c.N + ring], e = bb.eri[b * c.N + ring];
  unsigned long long* const xp = bb.xprof;  // diagnostic phase stamps (thread 0, 100 MHz)
  unsigned long long tp = (xp && tid == 0) ? wall_clock64() : 0;
  if (xp && tid == 0) atomicAdd(xp + 7, atomicAdd(xp + 8, 1ull) + 1);  // workgroups in flight
  auto stamp = [&](int slot) {
    if (xp && tid == 0) {
      const unsigned long long now = wall_clock64();
      atomicAdd(xp + slot, now - tp);
      tp = now;
    }
  };
  RingCtx R;
  R.b = b; R.ring = ring; R.ns = ns;
  R.base = (size_t)b * c.P;
  R.lo = max(0, s - 5);
  int hi = min(ns, e + 6);
  if (hi < R.lo) hi = R.lo;
  R.Wn = hi - R.lo;
  R.osh = bb.r_sharp + ((size_t)b * c.N + ring) * kSharpPerRing;
  R.ols = bb.r_lsharp + ((size_t)b * c.N + ring) * kLessSharpPerRing;
  R.ofl = bb.r_flat + ((size_t)b * c.N + ring) * kFlatPerRing;
  float4* olf = bb.r_lflat + R.base + (size_t)ring * c.H;
  volatile uint8_t* picked = L.picked;
  volatile int8_t* label = L.label;
  for (int t = tid; t < R.Wn; t += blockDim.x) {  // what the sorts read (col, picked, label: after them)
    const size_t g = R.base + R.lo + t;
    L.curv[t] = bb.curv[g];
    L.gfl[t] = bb.gflag[g];
  }
  if (tid < 64) L.misc[tid] = 0;
  __syncthreads();
  int ph = 0;
  if (ring == 0 && carry) ph = carry->phantom_ind;
  if (tid == 0) L.misc[M_PH] = ph;  // the phantom entry's index unless a sector sort replaces it
  __syncthreads();
  int flags = 0;
  // sector j: [sp, ep] (ep scanned, excluded from the sort, :699-702), sorted
  // by value in its own buffer at off(j) = sum of the earlier padded sizes
  auto sector = [&](int j, int* sp, int* ep, int* off) {
    int o = 0;
    for (int i = 0; i < j; ++i) {
      const int a0 = (s * (6 - i) + e * i) / 6, b0 = (s * (5 - i) + e * (i + 1)) / 6 - 1;
      if (a0 < b0) o += next_pow2(b0 - a0);
    }
    *sp = (s * (6 - j) + e * j) / 6;
    *ep = (s * (5 - j) + e * (j + 1)) / 6 - 1;
    *off = o;
  };
  // ---- the six sector sorts, one wave per sector at a time (they do not
  // depend on the picking; only the picking runs in sector order).  Each is
  // sorted in its wave's scratch and kept as window positions in perm.
  //
  // Rings other than ring 0 sort only what a walk can pick: the edge walk
  // (:704-734) takes points with curvature > edge_thr off the ground, the flat
  // walk (:736-769) points with curvature < surf_thr on the ground, and it
  // passes over every other point without effect.  So the edge candidates
  // and the flat candidates are each sorted by value alone and kept back to
  // back in perm (counts in misc): the walks over them see the candidates in
  // the same order as over the whole sorted sector.  Equal values within a
  // candidate list fall back to std::sort of the whole sector, filtered in
  // its order.  Ring 0 sorts the whole sector: its phantom entry (the carried
  // index, perm 0xFFFF) is not a position of the sector.
  const int nw = blockDim.x >> 6;
  constexpr int kPhantom = -2;
  const int secCap = extract_sector_cap(c.H);
  const bool filtered = ring != 0;
  // three waves sort (two rounds of three sectors, as four waves would take
  // two rounds too), so the scratch holds three sectors
  for (int j = wave; j < 6 && wave < kSortWaves; j += kSortWaves) {
    int sp, ep, off;
    sector(j, &sp, &ep, &off);
    if (sp >= ep) continue;
    const int n = ep - sp;
    SmoothEntry* a = L.srt + wave * secCap;
    uint16_t* pm = L.perm + (sp - s);
    if (filtered) {
      int nl[2] = {0, 0};
      for (int list = 0; list < 2; ++list) {
        auto cand = [&](int w, float v) {
          return list == 0 ? (v > c.edge_thr && L.gfl[w] == 0) : (v < c.surf_thr && L.gfl[w] == 1);
        };
        int cnt = 0;
        for (int t0 = 0; t0 < n; t0 += 64) {  // ordered wave compaction
          const int t = t0 + lane;
          bool f = false;
          float v = 0.0f;
          if (t < n) {
            v = L.curv[sp + t - R.lo];
            f = cand(sp + t - R.lo, v);
          }
          const unsigned long long msk = __ballot(f);
          if (f) a[cnt + __popcll(msk & ((1ull << lane) - 1))] = SmoothEntry{v, sp + t};
          cnt += __popcll(msk);
        }
        nl[list] = cnt;
        if (cnt == 0) continue;
        const int m = next_pow2(cnt);
        for (int t = cnt + lane; t < m; t += 64) a[t] = {__builtin_inff(), INT_MAX};
        wave_sync_lds();
        wave_bitonic_entries(a, m);
        bool tie = false;
        for (int t = lane; t < cnt - 1; t += 64) tie |= a[t].value == a[t + 1].value;
        uint16_t* out = pm + (list == 0 ? 0 : nl[0]);
        if (__ballot(tie)) {
          if (lane == 0) {
            atomicOr(&bb.fa_flags[b], LEGO_REC_SORT_TIES);  // the record shows the fallback ran
            for (int t = 0; t < n; ++t) a[t] = SmoothEntry{L.curv[sp + t - R.lo], sp + t};
            std_sort_by_value(a, n, (uint32_t*)(a + n));  // stack in the scratch behind the sector
            int k = 0;
            for (int t = 0; t < n; ++t)
              if (cand(a[t].ind - R.lo, a[t].value)) out[k++] = (uint16_t)(a[t].ind - R.lo);
          }
        } else {
          for (int t = lane; t < cnt; t += 64) out[t] = (uint16_t)(a[t].ind - R.lo);
        }
        wave_sync_lds();  // the scratch is refilled for the next list
      }
      if (lane == 0) {
        L.misc[M_NEF + 2 * j] = nl[0];
        L.misc[M_NEF + 2 * j + 1] = nl[1];
      }
      continue;
    }
    const int m = next_pow2(n);
    const bool phantom_here = (ring == 0 && sp <= 4 && 4 < ep);
    for (int t = lane; t < m; t += 64) {
      SmoothEntry en;
      if (t < n) {
        const int pos = sp + t;
        en = (phantom_here && pos == 4) ? SmoothEntry{0.0f, kPhantom} : SmoothEntry{L.curv[pos - R.lo], pos};
      } else {
        en = {__builtin_inff(), INT_MAX};
      }
      a[t] = en;
    }
    wave_sync_lds();
    wave_bitonic_entries(a, m);
    bool tie = false;
    for (int t = lane; t < n - 1; t += 64) tie |= a[t].value == a[t + 1].value;
    if (__ballot(tie)) {
      // equal curvatures: their relative order is std::sort's
      if (lane == 0) {
        atomicOr(&bb.fa_flags[b], LEGO_REC_SORT_TIES);  // the record shows the fallback ran
        for (int t = 0; t < n; ++t) {
          const int pos = sp + t;
          a[t] = (phantom_here && pos == 4) ? SmoothEntry{0.0f, kPhantom} : SmoothEntry{L.curv[pos - R.lo], pos};
        }
        std_sort_by_value(a, n, (uint32_t*)(a + n));  // stack in the scratch behind the sector
      }
      wave_sync_lds();
    }
    for (int t = lane; t < n; t += 64) {
      const int ind = a[t].ind;
      pm[t] = ind == kPhantom ? (uint16_t)0xFFFF : (uint16_t)(ind - R.lo);
    }
    if (phantom_here && lane == 0) {
      const int ind = a[4 - sp].ind;
      L.misc[M_PH] = ind == kPhantom ? ph : ind;
    }
    wave_sync_lds();  // the scratch is refilled for the wave's next sector
  }
  __syncthreads();
  // the walks' arrays, in the sort scratch now that the sorts are done
  for (int t = tid; t < R.Wn; t += blockDim.x) {
    const size_t g = R.base + R.lo + t;
    L.col[t] = (uint16_t)bb.col[g];
    L.picked[t] = bb.pick0[g];
    L.label[t] = 0;
  }
  __syncthreads();
  if (ring == 0 && carry && tid == 0 && R.lo == 0 && R.Wn > 0 && carry->picked0) L.picked[0] = 1;
  __syncthreads();
  stamp(0);  // window load + the six sector sorts
  const int newph = L.misc[M_PH];
  // per-sector pick lists (sharp, less sharp, flat) in pick order, in the
  // sort scratch, which is free until the VoxelGrid keys; the counts and the
  // spill masks in misc
  int* const pk = (int*)L.srt;
  static_assert(6 * kPickListStride * 4 <= 1024, "pick lists fit the scratch head");
  // ---- picking (:699-769).  Sector j's walk only interacts with sector j+1
  // through the suppression of its picks near ep_j (positions sp_{j+1} ..
  // sp_{j+1}+4).  Rings other than ring 0 (whose phantom entry may point
  // anywhere in the window) with every sector at least 8 long run the six
  // walks speculatively in parallel (one wave per sector, suppression kept
  // inside the sector and the rest recorded as spill bits), then validate in
  // sector order: sector j's walk is exactly the serial one unless sector
  // j-1's final spill marks a position that sector j's walk picked (a position
  // the walk reached and found eligible; one it skipped or never reached
  // changes nothing).  Such a sector is re-walked by wave 0 from its initial
  // state plus the spill.  Ring 0 and short rings walk serially on wave 0.
  bool parallel = !(ring == 0);
  for (int j = 0; j < 6 && parallel; ++j) {
    int sp, ep, off;
    sector(j, &sp, &ep, &off);
    parallel = ep - sp >= 8;
  }
  if (parallel) {  // the initial picked state, for re-walks
    uint8_t* p0 = (uint8_t*)L.srt + 1024;
    for (int t = tid; t < R.Wn; t += blockDim.x) p0[t] = picked[t];
  }
  if (tid < 6 * 4) L.misc[M_SEC + tid] = 0;
  __syncthreads();
  auto walk = [&](int j, bool local) {
    int sp, ep, off;
    sector(j, &sp, &ep, &off);
    if (sp >= ep) return;
    int* const lst = pk + j * kPickListStride;
    int* const cnt3 = L.misc + M_SEC + 4 * j;
    const int lo = local ? sp - R.lo : 0, hi = local ? ep - R.lo : R.Wn - 1;
    const uint16_t* srt = L.perm + (sp - s);
    // the walks' items: position ep (scanned, never sorted, :699-702) first
    // in the edge walk and last in the flat walk, the sorted entries between
    const int nE = filtered ? L.misc[M_NEF + 2 * j] : 0, nF = filtered ? L.misc[M_NEF + 2 * j + 1] : 0;
    const int nEdge = filtered ? nE + 1 : ep - sp + 1, nFlat = filtered ? nF + 1 : ep - sp + 1;
    auto edge_item = [&](int q) {
      if (!filtered) return entry_ind(srt, sp, ep, ep - q, R.lo, ph);
      return q == 0 ? ep : (int)srt[nE - q] + R.lo;
    };
    auto flat_item = [&](int q) {
      if (!filtered) return entry_ind(srt, sp, ep, sp + q, R.lo, ph);
      return q == nF ? ep : (int)srt[nE + q] + R.lo;
    };
    int nsh = 0, nls = 0, nfl = 0;
    unsigned spill = 0;  // bit i: position ep+1+i suppressed; bit 8+i: sp-1-i
    auto sup = [&](int ind) {
      const int w = ind - R.lo;
      picked[w] = 1;
      for (int l = 1; l <= 5; l++) {
        const int q = w + l;
        if (q >= R.Wn) break;
        if (abs((int)L.col[q] - (int)L.col[q - 1]) > 10) break;
        if (q <= hi) picked[q] = 1;
        else spill |= 1u << (q - hi - 1);
      }
      for (int l = -1; l >= -5; l--) {
        const int q = w + l;
        if (ind + l < 0 || q < 0) break;
        if (abs((int)L.col[q] - (int)L.col[q + 1]) > 10) break;
        if (q >= lo) picked[q] = 1;
        else spill |= 1u << (8 + lo - 1 - q);
      }
    };
    {
      int cnt = 0;
      bool done = false;
      for (int q0 = 0; q0 < nEdge && !done; q0 += 64) {
        const int q = q0 + lane;
        bool act = q < nEdge;
        const int ind = act ? edge_item(q) : -1;
        if (act && !in_win(R, ind)) { act = false; flags |= 1; }
        while (true) {
          bool el = false;
          if (act) {
            const int w = ind - R.lo;
            el = picked[w] == 0 && L.curv[w] > c.edge_thr && L.gfl[w] == 0;
          }
          const unsigned long long msk = __ballot(el);
          if (msk == 0) break;
          const int l = __ffsll((long long)msk) - 1;
          cnt++;
          if (cnt > 20) { done = true; break; }
          if (lane == l) {  // the points are copied after the picking (no HBM latency per pick)
            label[ind - R.lo] = cnt <= 2 ? 2 : 1;
            if (cnt <= 2) lst[nsh] = ind;
            lst[2 + nls] = ind;
            sup(ind);
          }
          if (cnt <= 2) nsh++;
          nls++;
          act = act && lane > l;
        }
      }
    }
    {
      int cnt = 0;
      bool done = false;
      for (int q0 = 0; q0 < nFlat && !done; q0 += 64) {
        const int q = q0 + lane;
        bool act = q < nFlat;
        const int ind = act ? flat_item(q) : -1;
        if (act && !in_win(R, ind)) { act = false; flags |= 1; }
        while (true) {
          bool el = false;
          if (act) {
            const int w = ind - R.lo;
            el = picked[w] == 0 && L.curv[w] < c.surf_thr && L.gfl[w] == 1;
          }
          const unsigned long long msk = __ballot(el);
          if (msk == 0) break;
          const int l = __ffsll((long long)msk) - 1;
          if (lane == l) {
            label[ind - R.lo] = -1;
            lst[22 + nfl] = ind;
          }
          nfl++;
          cnt++;
          if (cnt >= 4) { done = true; break; }
          if (lane == l) sup(ind);
          act = act && lane > l;
        }
      }
    }
    unsigned sm = 0;
    for (int bit = 0; bit < 16; ++bit)
      if (__ballot((spill >> bit) & 1u)) sm |= 1u << bit;
    if (lane == 0) { cnt3[0] = nsh; cnt3[1] = nls; cnt3[2] = nfl; cnt3[3] = (int)sm; }
    wave_sync_lds();
  };
  if (parallel) {
    for (int j = wave; j < 6; j += nw) walk(j, true);
    __syncthreads();
    if (wave == 0) {
      const uint8_t* p0 = (const uint8_t*)L.srt + 1024;
      for (int j = 1; j < 6; ++j) {
        int sp, ep, off;
        sector(j, &sp, &ep, &off);
        const unsigned in = (unsigned)L.misc[M_SEC + 4 * (j - 1) + 3] & 0x1fu;
        bool bad = false;
        for (int i = 0; i < 5; ++i) bad |= ((in >> i) & 1u) && label[sp + i - R.lo] != 0;
        if (!bad) continue;
        // re-walk: the sector's initial state plus the spill, labels cleared
        for (int t = sp + lane; t <= ep; t += 64) {
          const int w = t - R.lo;
          picked[w] = p0[w] | ((t - sp < 5 && ((in >> (t - sp)) & 1u)) ? 1 : 0);
          label[w] = 0;
        }
        wave_sync_lds();
        if (lane == 0) atomicAdd(&L.misc[M_REWALK], 1);
        walk(j, true);
      }
    }
  } else if (wave == 0) {
    for (int j = 0; j < 6; j++) walk(j, false);
  }
  __syncthreads();
  stamp(1);  // the picking walks
  if (xp && tid == 0) {
    atomicAdd(xp + 5, (unsigned long long)L.misc[M_REWALK]);
    if (parallel) atomicAdd(xp + 6, 1ull);
  }
  {  // the picked points in pick order (sector by sector), all loads independent
    int nsh = 0, nls = 0, nfl = 0;
    for (int j = 0; j < 6; ++j) {
      nsh += L.misc[M_SEC + 4 * j];
      nls += L.misc[M_SEC + 4 * j + 1];
      nfl += L.misc[M_SEC + 4 * j + 2];
    }
    auto at = [&](int t, int which, int head) {  // t-th entry of list `which` over the sectors
      for (int j = 0;; ++j) {
        const int n = L.misc[M_SEC + 4 * j + which];
        if (t < n || j == 5) return pk[j * kPickListStride + head + t];
        t -= n;
      }
    };
    for (int t = tid; t < nsh + nls + nfl; t += blockDim.x) {
      if (t < nsh) R.osh[t] = bb.dsk[R.base + at(t, 0, 0)];
      else if (t < nsh + nls) R.ols[t - nsh] = bb.dsk[R.base + at(t - nsh, 1, 2)];
      else R.ofl[t - nsh - nls] = bb.dsk[R.base + at(t - nsh - nls, 2, 22)];
    }
    __syncthreads();
    if (tid == 0) { L.misc[M_NSH] = nsh; L.misc[M_NLS] = nls; L.misc[M_NFL] = nfl; }
  }
  // ---- less-flat set: per sector the positions k in [sp, ep] with label <= 0,
  // in order (:771-775); the sectors are consecutive ranges, so one ordered
  // pass over [s, e - 1] restricted to the sectors that ran.  One block scan
  // for the whole range: a flag per position in 256-position chunks (a bit
  // per chunk), the waves' counts per chunk through LDS (L.red, free until
  // the VoxelGrid bounds), then every position's rank.
  {
    int sp0, ep0, o0;
    sector(0, &sp0, &ep0, &o0);
    int sp5, ep5, o5;
    sector(5, &sp5, &ep5, &o5);
    const int nC = ep5 >= sp0 ? (ep5 - sp0 + blockDim.x) / blockDim.x : 0;  // <= 16 (W <= 4096)
    int* cnt = (int*)L.red;  // [chunk][wave], nC * nw <= 64
    unsigned fm = 0;
    for (int ch = 0; ch < nC; ++ch) {
      const int k = sp0 + ch * (int)blockDim.x + tid;
      bool f = false;
      if (k <= ep5 && label[k - R.lo] <= 0) {
        int j = 0;
        int sp, ep, off;
        for (; j < 6; ++j) {
          sector(j, &sp, &ep, &off);
          if (k <= ep) break;
        }
        f = j < 6 && k >= sp && sp < ep;
      }
      fm |= (f ? 1u : 0u) << ch;
      const unsigned long long m = __ballot(f);
      if (lane == 0) cnt[ch * nw + wave] = (int)__popcll(m);
    }
    __syncthreads();
    const unsigned long long lt = (1ull << lane) - 1;
    int total = 0;
    for (int ch = 0; ch < nC; ++ch) {
      int base = total;
      for (int w = 0; w < nw; ++w) {
        const int v = cnt[ch * nw + w];
        if (w < wave) base += v;
        total += v;
      }
      const bool f = (fm >> ch) & 1u;
      const unsigned long long m = __ballot(f);
      if (f) L.lf[base + (int)__popcll(m & lt)] = (uint16_t)(sp0 + ch * (int)blockDim.x + tid - R.lo);  // window positions
    }
    if (tid == 0) L.misc[M_LF] = total;
    __syncthreads();
  }
  if (tid == 0) L.misc[M_P0] = (R.Wn > 0 && L.picked[0]) ? 1 : 0;  // the carry's
  stamp(2);  // picked-point copies + the ordered less-flat set
  // ---- the less-flat set's points, in order, to the ring's slot: the
  // VoxelGrid (:778-782) runs in k_lf_voxel over every ring of the batch
  const int K = L.misc[M_LF];
  for (int t = tid; t < K; t += blockDim.x) olf[t] = bb.dsk[R.base + R.lo + L.lf[t]];
  const int nlf = K;
  __syncthreads();
  stamp(3);  // the less-flat points to the ring's slot
  if (xp && tid == 0) {
    atomicAdd(xp + 4, 1ull);
    atomicAdd(xp + 8, ~0ull);  // leaves the in-flight count
  }
  if (tid == 0) {
    int* cnt = bb.r_cnt + ((size_t)b * c.N + ring) * 4;
    cnt[0] = L.misc[M_NSH];
    cnt[1] = L.misc[M_NLS];
    cnt[2] = L.misc[M_NFL];
    static_assert(kMaxHorizon < (1 << 15), "r_cnt[3] packs two ring counts (<= H) in 16 bits each");
    cnt[3] = nlf | (nlf << 16);  // high half: the less-flat count k_lf_voxel decides on (never overwritten)
  }
  if (ring == 0 && carry) {
    // wave 0 holds the picking flags; lane values of `flags` are merged below
    int fl = __ballot(flags != 0) ? 1 : 0;
    if (tid == 0) {
      carry->phantom_ind = newph;
      carry->picked0 = (R.lo == 0 && R.Wn > 0) ? L.misc[M_P0] : carry->picked0;
      carry->flags |= fl;
    }
  }
  __syncthreads();
}

// ---------------------------------------------------------------- less-flat VoxelGrid
// pcl::VoxelGrid<PointType> downSizeFilter, leaf 0.2 (featureAssociation.cpp:
// 778-782) on each ring's less-flat set, one (scan, ring) workgroup: the
// points from the ring's slot (L2-resident: k_extract just wrote them),
// getMinMax3D, the voxel index per point, PCL's std::sort of (idx, point) by
// idx (lego_vgsort.h: libstdc++'s order of each voxel's points, which is the
// summation order), one lane per voxel summing its points in that order into
// registers, then the centroids over the slot.  The slot's count goes from
// the less-flat set's size to the voxels'.
// the per-voxel centroid of PCL's VoxelGrid: the points of sorted positions
// [t, u) (one voxel), summed in that order from the ring's slot
// A payload at or past K cannot come out of a sort (every form only moves
// the payloads 0..K-1 it was given); if one does, the scan's error word gets
// kBadPermutation (the host returns LEGO_E_DEVICE) and the addend is skipped.
__device__ __forceinline__ float4 lfv_centroid(const float4* slot, const uint16_t* val, const uint32_t* key, int t,
                                               int K, int* bad) {
  const uint32_t k = key[t];
  float cx = 0, cy = 0, cz = 0, ci = 0;
  int u = t;
  for (; u < K && key[u] == k; ++u) {
    const int vi = (int)val[u];
    if (vi >= K) {
      atomicOr(bad, kBadPermutation);
      continue;
    }
    const float4 q = slot[vi];
    cx += q.x; cy += q.y; cz += q.z; ci += q.w;
  }
  const float n = (float)(u - t);
  return make_float4(cx / n, cy / n, cz / n, ci / n);
}

// A ring of up to kVgWaveMax less-flat points by ONE wave (lego_vgsort_wave.h:
// the same permutation as the block sort, no workgroup barrier): the same
// steps as lfv_block below, wave-wide.  lds: the wave's key / payload /
// scratch words.
constexpr int kLfvWaveRows = kVgWaveMax / 64;
constexpr size_t kLfvWaveLds = (size_t)4 * kVgWaveMax * 10;  // four waves' key (4 B), payload (2 B), scratch (4 B)
__device__ __forceinline__ void lfv_wave(const BatchBufs& bb, const DevCfg& c, int ring, int b, unsigned char* lds) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (ring >= c.N) return;
  int* cnt = bb.r_cnt + ((size_t)b * c.N + ring) * 4;
  // the count as k_extract wrote it (high half): a large ring's workgroup may
  // already have replaced the low half with its voxel count, which must not
  // make this wave filter the filtered ring again
  const int K = cnt[3] >> 16;
  if (K <= 0 || K > kVgWaveMax) return;  // wave-uniform
  float4* slot = bb.r_lflat + (size_t)b * c.P + (size_t)ring * c.H;
  uint32_t* key = (uint32_t*)lds + (size_t)wave * kVgWaveMax;
  uint16_t* val = (uint16_t*)(lds + (size_t)16 * kVgWaveMax) + (size_t)wave * kVgWaveMax;
  uint32_t* scw = (uint32_t*)(lds + (size_t)24 * kVgWaveMax) + (size_t)wave * kVgWaveMax;
  const float inv = 1.0f / 0.2f;
  float mn[3] = {__builtin_inff(), __builtin_inff(), __builtin_inff()};
  float mx[3] = {-__builtin_inff(), -__builtin_inff(), -__builtin_inff()};
  for (int t = lane; t < K; t += 64) {
    const float4 p = slot[t];
    mn[0] = fminf(mn[0], p.x); mn[1] = fminf(mn[1], p.y); mn[2] = fminf(mn[2], p.z);
    mx[0] = fmaxf(mx[0], p.x); mx[1] = fmaxf(mx[1], p.y); mx[2] = fmaxf(mx[2], p.z);
  }
  for (int q = 0; q < 3; ++q) {
    for (int o = 32; o > 0; o >>= 1) {
      mn[q] = fminf(mn[q], __shfl_xor(mn[q], o, 64));
      mx[q] = fmaxf(mx[q], __shfl_xor(mx[q], o, 64));
    }
  }
  const long long dx = (long long)((mx[0] - mn[0]) * inv) + 1;
  const long long dy = (long long)((mx[1] - mn[1]) * inv) + 1;
  const long long dz = (long long)((mx[2] - mn[2]) * inv) + 1;
  if (dx * dy * dz > (long long)INT_MAX) return;  // PCL keeps the cloud (it is in the slot already)
  int mb[3], xb[3];
  for (int q = 0; q < 3; ++q) {
    mb[q] = (int)floorf(mn[q] * inv);
    xb[q] = (int)floorf(mx[q] * inv);
  }
  const int d0 = xb[0] - mb[0] + 1, d1 = xb[1] - mb[1] + 1;
  for (int t = lane; t < K; t += 64) {
    const float4 p = slot[t];
    const int i0 = (int)(floorf(p.x * inv) - (float)mb[0]);
    const int i1 = (int)(floorf(p.y * inv) - (float)mb[1]);
    const int i2 = (int)(floorf(p.z * inv) - (float)mb[2]);
    key[t] = (uint32_t)(i0 + i1 * d0 + i2 * d0 * d1);
    val[t] = (uint16_t)t;
  }
  vg_wave_sync();
  vg_wave_sort(key, val, scw, K);  // a whole array: budget 2 lg K
  // centroids into registers (every read of the slot done), then over the slot
  float4 cen[kLfvWaveRows];
  int at[kLfvWaveRows];
  int outc = 0;
  const unsigned long long below = (1ull << lane) - 1;
#pragma unroll
  for (int j = 0; j < kLfvWaveRows; ++j) {
    at[j] = -1;
    const int t = (j << 6) + lane;
    const bool head = t < K && (t == 0 || key[t] != key[t - 1]);
    const unsigned long long m = __ballot(head);
    if (head) {
      cen[j] = lfv_centroid(slot, val, key, t, K, bb.bad + b);
      at[j] = outc + (int)__popcll(m & below);
    }
    outc += (int)__popcll(m);
  }
  vg_wave_sync();  // the wave's slot reads have returned
#pragma unroll
  for (int j = 0; j < kLfvWaveRows; ++j)
    if (at[j] >= 0) slot[at[j]] = cen[j];
  if (lane == 0) cnt[3] = outc | (K << 16);
}

constexpr int kLfvBlockRings = 2;  // rings per large-ring workgroup (k_lf_voxel; 1 / 2 / 4 / 8: fleet 254 / 256 / 245 / 253 k)
// A launch of at most this many rings leaves part of the device idle (one
// scan through the node API, C2's 100-scan batch beside the odometry, C3):
// one large ring per workgroup there, so a workgroup lasts one ring's sort
// instead of two in sequence (C2 at 20 steps: fa.voxel 0.695 -> 0.667 ms,
// profiles/r04_ab_lfv_rings.txt).  A fleet call keeps two (kLfvBlockRings).
constexpr int kLfvSmallLaunchRings = 4096;
// launches of up to this many rings (a node call) take 1024-thread workgroups:
// node fa 0.30 -> 0.28 ms; a C2 batch's VoxelGrid 0.67 -> 1.52 ms that way
// (profiles/r04_ab_lfv_wide.txt)
constexpr int kLfvWideLaunchRings = 128;
#ifndef LFV_DIAG
#define LFV_DIAG 0
#endif
#if LFV_DIAG
__device__ int g_lfv_diag;  // printed violations (capped)
#endif
__host__ __device__ inline size_t lfvox_lds_bytes(int H) {
  return (((size_t)H * 6 + 15) & ~(size_t)15) + vg_sort_scratch_bytes(H, kExtractThreads) + 64;
}
template <int T>
__device__ __forceinline__ void lfv_block(const BatchBufs& bb, const DevCfg& c, int ring, int b, int waveMax,
                          unsigned char* lds_raw) {
  constexpr int MP = (kMaxHorizon + T - 1) / T;  // voxels per thread (<= H of them per ring)
  int tid = threadIdx.x;
  asm volatile("" : "+v"(tid));  // the lane terms computed per ring, not held across k_lf_voxel's ring loop
  const int lane = tid & 63, wave = tid >> 6;
  const int H = c.H;
  uint32_t* key = (uint32_t*)lds_raw;
  uint16_t* val = (uint16_t*)(lds_raw + (size_t)H * 4);
  unsigned char* sc = lds_raw + (((size_t)H * 6 + 15) & ~(size_t)15);
  int* misc = (int*)(sc + vg_sort_scratch_bytes(H, kExtractThreads));  // [16]
  __shared__ float mm[16][6];  // per wave (up to 1024 threads)
  int* cnt = bb.r_cnt + ((size_t)b * c.N + ring) * 4;
  float4* slot = bb.r_lflat + (size_t)b * c.P + (size_t)ring * H;
  const int K = cnt[3] >> 16;  // as k_extract wrote it (lfv_wave)
  if (K <= waveMax) return;  // a wave's (or empty)
  const float inv = 1.0f / 0.2f;
  float mn[3] = {__builtin_inff(), __builtin_inff(), __builtin_inff()};
  float mx[3] = {-__builtin_inff(), -__builtin_inff(), -__builtin_inff()};
  for (int t = tid; t < K; t += blockDim.x) {
    const float4 p = slot[t];
    mn[0] = fminf(mn[0], p.x); mn[1] = fminf(mn[1], p.y); mn[2] = fminf(mn[2], p.z);
    mx[0] = fmaxf(mx[0], p.x); mx[1] = fmaxf(mx[1], p.y); mx[2] = fmaxf(mx[2], p.z);
  }
  for (int q = 0; q < 3; ++q) {
    for (int o = 32; o > 0; o >>= 1) {
      mn[q] = fminf(mn[q], __shfl_xor(mn[q], o, 64));
      mx[q] = fmaxf(mx[q], __shfl_xor(mx[q], o, 64));
    }
  }
  if (lane == 0)
    for (int q = 0; q < 3; ++q) { mm[wave][q] = mn[q]; mm[wave][3 + q] = mx[q]; }
  __syncthreads();
  float lo[3], hi[3];
  for (int q = 0; q < 3; ++q) {
    lo[q] = mm[0][q];
    hi[q] = mm[0][3 + q];
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w) { lo[q] = fminf(lo[q], mm[w][q]); hi[q] = fmaxf(hi[q], mm[w][3 + q]); }
  }
  const long long dx = (long long)((hi[0] - lo[0]) * inv) + 1;
  const long long dy = (long long)((hi[1] - lo[1]) * inv) + 1;
  const long long dz = (long long)((hi[2] - lo[2]) * inv) + 1;
  if (dx * dy * dz > (long long)INT_MAX) return;  // PCL keeps the cloud (it is in the slot already)
  int mb[3], xb[3];
  for (int q = 0; q < 3; ++q) {
    mb[q] = (int)floorf(lo[q] * inv);
    xb[q] = (int)floorf(hi[q] * inv);
  }
  const int d0 = xb[0] - mb[0] + 1, d1 = xb[1] - mb[1] + 1;
  for (int t = tid; t < K; t += blockDim.x) {
    const float4 p = slot[t];
    const int i0 = (int)(floorf(p.x * inv) - (float)mb[0]);
    const int i1 = (int)(floorf(p.y * inv) - (float)mb[1]);
    const int i2 = (int)(floorf(p.z * inv) - (float)mb[2]);
    key[t] = (uint32_t)(i0 + i1 * d0 + i2 * d0 * d1);
    val[t] = (uint16_t)t;
  }
  __syncthreads();
  // The LDS-id form of the block sort.  The register form (vg_block_sort,
  // segment ids in registers, five barriers per level instead of seven) is
  // not built into this kernel: both builds of it here spilled under the
  // 128-VGPR cap and both faulted on the GPU (round 4's
  // 256-thread build; round 5's 1024-thread instance, a VM fault on VLS-128
  // scan 0, gpurun_out r05a / r05c, profiles/r05_lfv_fault.txt), while the
  // same sort is exact at both block sizes in kernels of its own.
  vg_block_sort_sid(vg_sort_carve(key, val, sc, K, (int)blockDim.x), K, -1, nullptr, true);
#if LFV_DIAG  // diagnostic build (scripts/lfv_diag.sh): the sort's output checked before any use
  for (int t = tid; t < K; t += blockDim.x) {
    const bool badv = (int)val[t] >= K, bado = t > 0 && key[t - 1] > key[t];
    if ((badv || bado) && atomicAdd(&g_lfv_diag, 1) < 24)
      printf("LFV_DIAG sort T=%d b=%d ring=%d K=%d t=%d val=%d key[t-1]=%u key[t]=%u\n", (int)blockDim.x, b, ring,
             K, t, (int)val[t], t > 0 ? key[t - 1] : 0u, key[t]);
  }
  __syncthreads();
#endif
  // centroids into registers (every read of the slot done), then over the slot
  float4 cen[MP];
  int at[MP];
  int outc = 0;
#pragma unroll
  for (int j = 0; j < MP; ++j) {
    at[j] = -1;
    const int t = j * (int)blockDim.x + tid;
    if (j * (int)blockDim.x >= K) continue;  // uniform
    const bool head = t < K && (t == 0 || key[t] != key[t - 1]);
    int tot;
    const int r = block_rank(head, misc, &tot);
    if (head) {
      cen[j] = lfv_centroid(slot, val, key, t, K, bb.bad + b);
      at[j] = outc + r;
    }
    outc += tot;
  }
  __syncthreads();
#if LFV_DIAG
  for (int j = 0; j < MP; ++j)
    if (at[j] >= K && atomicAdd(&g_lfv_diag, 1) < 24) {
      printf("LFV_DIAG store T=%d b=%d ring=%d K=%d j=%d at=%d outc=%d\n", (int)blockDim.x, b, ring, K, j, at[j],
             outc);
      at[j] = -1;
    }
  if (tid == 0 && (outc > K || outc < 0) && atomicAdd(&g_lfv_diag, 1) < 24)
    printf("LFV_DIAG count T=%d b=%d ring=%d K=%d outc=%d\n", (int)blockDim.x, b, ring, K, outc);
#endif
#pragma unroll
  for (int j = 0; j < MP; ++j)
    if (at[j] >= 0) slot[at[j]] = cen[j];
  if (tid == 0) cnt[3] = outc | (K << 16);
}

// The batch's per-ring VoxelGrids in one launch, so small and large rings
// interleave: workgroups [0, g4) of each scan take four rings each, a ring of
// up to kVgWaveMax points per wave (lfv_wave); workgroups [g4, g4 + gb) the
// larger rings with the whole workgroup (lfv_block), workgroup k the rings
// k, k + gb, ... (gb < N: fewer workgroups that find no large ring).  g4 = 0
// (diagnostic LEGO_LFV_WAVE=0): every ring by a workgroup.
// T = 1024 (small launches): every ring by a whole workgroup (g4 = 0).
// LFV_MINB: lego_vgsort.h.
template <int T>
__global__ void __launch_bounds__(T, T == kExtractThreads ? LFV_MINB : 1) k_lf_voxel(BatchBufs bb, DevCfg c, int g4,
                                                                                   int gb) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
  const int b = blockIdx.y;
  if (T == kExtractThreads && (int)blockIdx.x < g4) {
    lfv_wave(bb, c, (int)blockIdx.x * 4 + (int)(threadIdx.x >> 6), b, lds_raw);
    return;
  }
  for (int ring = (int)blockIdx.x - g4; ring < c.N; ring += gb) {
    lfv_block<T>(bb, c, ring, b, g4 > 0 ? kVgWaveMax : 0, lds_raw);
    __syncthreads();  // the next ring reuses the LDS
  }
}

#ifndef EXTRACT_MINWAVES
#define EXTRACT_MINWAVES 6
#endif
__global__ void __launch_bounds__(kExtractThreads, EXTRACT_MINWAVES) k_extract(BatchBufs bb, DevCfg c) {  // six waves per SIMD: six workgroups per CU
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
  const ExtractLds L = carve(lds_raw, c.H);
  const int ring = blockIdx.x, b = blockIdx.y;
  if (ring == 0) {
    __shared__ FaCarry cs;
    if (threadIdx.x == 0) cs = FaCarry{0, 1, 0, 0};  // S*
    __syncthreads();
    extract_ring(bb, c, b, 0, &cs, L);
    if (threadIdx.x == 0) bb.spec_out[b] = cs;
  } else {
    extract_ring(bb, c, b, ring, nullptr, L);
  }
}

// Walks each stream's scans in order (block s: scans [s*K, s*K + K), carry
// d_carry[s]); re-runs ring 0 wherever the real carry is not S* (the first
// scan of a stream, or after a 0.0-curvature tie).
__global__ void __launch_bounds__(kExtractThreads) k_fa_fixup(BatchBufs bb, DevCfg c, int K,
                                                             FaCarry* carries) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
  const ExtractLds L = carve(lds_raw, c.H);
  __shared__ FaCarry cs;
  FaCarry* carry = carries + blockIdx.x;
  if (threadIdx.x == 0) cs = *carry;
  __syncthreads();
  for (int b = blockIdx.x * K; b < (int)(blockIdx.x + 1) * K; ++b) {
    const bool steady = cs.phantom_ind == 0 && cs.picked0 == 1;
    if (steady) {
      __syncthreads();
      if (threadIdx.x == 0) {
        const FaCarry s = bb.spec_out[b];
        cs.phantom_ind = s.phantom_ind;
        cs.picked0 = s.picked0;
        cs.flags |= s.flags;
      }
      __syncthreads();
    } else {
      extract_ring(bb, c, b, 0, &cs, L);
      if (threadIdx.x == 0) atomicOr(&bb.fa_flags[b], LEGO_REC_RING0_REDONE);  // ring 0 recomputed with the real carry
    }
    if (bb.imu && threadIdx.x == 0) {  // the IMU members in stream order (:568-612, 1641-1651)
      ImuScan& o = bb.imuScan[b];
      if (o.hasFirst) {
        cs.rollStart = o.rollStart; cs.pitchStart = o.pitchStart; cs.yawStart = o.yawStart;
        for (int k = 0; k < 3; ++k) {
          cs.angFromStart[k] = o.ar0[k] - cs.arLast[k];
          cs.arLast[k] = o.ar0[k];
        }
        cs.rollCur = o.rollCur; cs.pitchCur = o.pitchCur; cs.yawCur = o.yawCur;
        if (o.hasLast)
          for (int k = 0; k < 3; ++k) cs.vfs[k] = o.vfs[k];
      }
      o.rollStart = cs.rollStart; o.pitchStart = cs.pitchStart; o.yawStart = cs.yawStart;
      o.rollCur = cs.rollCur; o.pitchCur = cs.pitchCur; o.yawCur = cs.yawCur;
      for (int k = 0; k < 3; ++k) { o.vfs[k] = cs.vfs[k]; o.angFromStart[k] = cs.angFromStart[k]; }
    }
  }
  if (threadIdx.x == 0) *carry = cs;
}

// One workgroup per (scan, ring): the ring's offsets are the sums of the
// earlier rings' counts (wave 0, a lane per ring), then its four slots are
// copied.  (A workgroup per scan walking its rings serially cost ~185 us on
// a single VLS-128 scan: 128 dependent rounds of small copies.)
// PART: 0 all four clouds; 1 the LM's three (sharp, less-sharp, flat: a node
// call, before the odometry); 2 the less-flat cloud only (the node call's
// side stream, after k_lf_voxel), each workgroup then counting its ring into
// lfReady (release) for the hand-off's wait.
template <int PART>
__global__ void k_fa_compact(BatchBufs bb, DevCfg c, unsigned* lfReady) {
  constexpr int F0 = PART == 2 ? 3 : 0, F1 = PART == 1 ? 3 : 4;  // the clouds [F0, F1)
  __shared__ int off[4];
  const int r = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  const int* cnt = bb.r_cnt + (size_t)b * c.N * 4;
  if (tid < 64) {
    int s[4] = {0, 0, 0, 0};
    for (int q = tid; q < r; q += 64)
#pragma unroll
      for (int f = F0; f < F1; ++f) s[f] += cnt[q * 4 + f] & 0xffff;  // [3]: the VoxelGrid's count, low half
#pragma unroll
    for (int f = F0; f < F1; ++f)
      for (int o = 32; o > 0; o >>= 1) s[f] += __shfl_xor(s[f], o, 64);
    if (tid == 0) {
#pragma unroll
      for (int f = F0; f < F1; ++f) {
        off[f] = s[f];
        if (r == c.N - 1) bb.f_cnt[b * 4 + f] = s[f] + (cnt[r * 4 + f] & 0xffff);
      }
    }
  }
  __syncthreads();
#if LFV_DIAG
  if (tid == 0 && ((cnt[r * 4 + 3] & 0xffff) > c.H || off[3] + (cnt[r * 4 + 3] & 0xffff) > c.P) &&
      atomicAdd(&g_lfv_diag, 1) < 24)
    printf("LFV_DIAG compact b=%d ring=%d cnt3=%x off3=%d\n", b, r, cnt[r * 4 + 3], off[3]);
#endif
  const size_t rb = (size_t)b * c.N + r;
  if (PART != 2) {
    for (int t = tid; t < cnt[r * 4 + 0]; t += blockDim.x)
      bb.f_sharp[(size_t)b * c.N * kSharpPerRing + off[0] + t] = bb.r_sharp[rb * kSharpPerRing + t];
    for (int t = tid; t < cnt[r * 4 + 1]; t += blockDim.x)
      bb.f_lsharp[(size_t)b * c.N * kLessSharpPerRing + off[1] + t] = bb.r_lsharp[rb * kLessSharpPerRing + t];
    for (int t = tid; t < cnt[r * 4 + 2]; t += blockDim.x)
      bb.f_flat[(size_t)b * c.N * kFlatPerRing + off[2] + t] = bb.r_flat[rb * kFlatPerRing + t];
  }
  if (PART != 1)
    for (int t = tid; t < (cnt[r * 4 + 3] & 0xffff); t += blockDim.x)
      bb.f_lflat[(size_t)b * c.P + off[3] + t] = bb.r_lflat[(size_t)b * c.P + (size_t)r * c.H + t];
  if (PART == 2) {
    __threadfence();  // every wave's stores (and, ring N-1, f_cnt) visible device-wide
    __syncthreads();  // ... before the ring's count
    if (tid == 0) __hip_atomic_fetch_add(lfReady + b, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// the batch's per-scan words k_fa_half / the extraction accumulate into (one
// launch instead of two fills)
__global__ void k_fa_init(BatchBufs bb, int B, unsigned* lfReady) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < B) {
    bb.firsthalf[b] = 0x7f7f7f7f;  // atomicMin's identity for the first-half index
    bb.fa_flags[b] = 0;
    if (lfReady) lfReady[b] = 0u;
  }
}

// lego_ctx_opts::fa_synccheck (diagnostic, host only): synchronise after
// every launch of launch_fa and name the kernel whose execution returned an
// error.
static void fa_synccheck(const LaunchOpts& lo, hipStream_t s, const char* what) {
  if (!lo.faSyncCheck) return;
  const hipError_t e = hipStreamSynchronize(s);
  std::fprintf(stderr, "fa_synccheck %s: %s\n", what, hipGetErrorString(e));
}

void launch_fa(const BatchBufs& bb, const DevCfg& c, int B, int S, FaCarry* d_carry, hipStream_t s,
               StageTimer* tm, const LaunchOpts& lo, hipStream_t side, hipEvent_t fork, unsigned* lfReady) {
  tm->mark("fa.deskew", s);
  k_fa_init<<<(B + 255) / 256, 256, 0, s>>>(bb, B, side ? lfReady : nullptr);
  fa_synccheck(lo, s, "k_fa_init");
  dim3 gpts((c.P + 255) / 256, B);
  k_fa_half<<<gpts, 256, 0, s>>>(bb, c);
  fa_synccheck(lo, s, "k_fa_half");
  if (bb.imu) k_fa_imu_start<<<(B + 63) / 64, 64, 0, s>>>(bb, c);
  k_fa_point<<<gpts, 256, 0, s>>>(bb, c);
  fa_synccheck(lo, s, "k_fa_point");
  tm->mark("fa.extract", s);
  const size_t lds = extract_lds_bytes(c.H);
  k_extract<<<dim3(c.N, B), kExtractThreads, lds, s>>>(bb, c);
  fa_synccheck(lo, s, "k_extract");
  tm->mark("fa.fixup", s);
  k_fa_fixup<<<S, kExtractThreads, lds, s>>>(bb, c, B / S, d_carry);
  fa_synccheck(lo, s, "k_fa_fixup");
  if (side) {  // a node call: the LM's clouds now, the less-flat VoxelGrid beside the odometry
    tm->mark("fa.compact", s);
    k_fa_compact<1><<<dim3(c.N, B), 256, 0, s>>>(bb, c, nullptr);
    fa_synccheck(lo, s, "k_fa_compact<1>");
    (void)hipEventRecord(fork, s);
    (void)hipStreamWaitEvent(side, fork, 0);
    s = side;
  } else {
    tm->mark("fa.voxel", s);
  }
  const bool waveOn = lo.lfvWave != 0;
  const int g4 = waveOn ? (c.N + 3) / 4 : 0;
  // rings per large-ring workgroup (lego_ctx_opts::lfv_block_rings; 1 = one
  // workgroup per ring)
  const int rpb = lo.lfvBlockRings > 0 ? lo.lfvBlockRings
                                       : (waveOn && B * c.N > kLfvSmallLaunchRings ? kLfvBlockRings : 1);
  const int gb = (c.N + rpb - 1) / rpb;
  // a launch that leaves the device idle but for itself (a node call): every
  // ring by a 1024-thread workgroup, the sort's levels over four times the
  // lanes (lego_ctx_opts::lfv_wide overrides)
  const bool wide = lo.lfvWide >= 0 ? lo.lfvWide != 0 : B * c.N <= kLfvWideLaunchRings;
  if (wide)
    k_lf_voxel<1024><<<dim3(c.N, B), 1024, lfvox_lds_bytes(c.H), s>>>(bb, c, 0, c.N);
  else
    k_lf_voxel<kExtractThreads>
        <<<dim3(g4 + gb, B), kExtractThreads, std::max(kLfvWaveLds, lfvox_lds_bytes(c.H)), s>>>(bb, c, g4, gb);
  fa_synccheck(lo, s, wide ? "k_lf_voxel<1024>" : "k_lf_voxel<256>");
  if (side) {
    k_fa_compact<2><<<dim3(c.N, B), 256, 0, s>>>(bb, c, lfReady);
    fa_synccheck(lo, s, "k_fa_compact<2>");
    return;
  }
  tm->mark("fa.compact", s);
  k_fa_compact<0><<<dim3(c.N, B), 256, 0, s>>>(bb, c, nullptr);
  fa_synccheck(lo, s, "k_fa_compact");
}

}  // namespace lego
