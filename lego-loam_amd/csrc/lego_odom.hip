// lego_odom.hip — the two-step LM odometry of featureAssociation on gfx950.
//
// One persistent 512-thread workgroup walks the batch's scans in stream order
// (scan k's problem depends on scan k-1's result through transformCur and the
// TransformToEnd'ed "last" clouds, featureAssociation.cpp:1759-1815), so the
// per-scan chain never returns to the host.  Per LM iteration:
//   every 5th iteration, one 32-lane group per query: TransformToStart
//     (:860-883), the exact nearest neighbour in a hash grid over the last
//     cloud (replaces KdTreeFLANN, :1054, :1165; ties -> lower index, FLANN's
//     tie order is traversal dependent) and the scan-line search loops as
//     written (:1062-1099, :1173-1220, incl. the loop-bound quirk);
//   one lane per query: line / plane residual, weight and Jacobian row
//     (:1106-1151, :1228-1321);
//   block reduce: AtA, AtB with double accumulation (cv::gemm's float path);
//   lane 0: QR solve, iteration-0 eigen degeneracy projection, update, NaN
//     reset, convergence test (:1324-1376, :1425-1477).
// Then integrateTransformation (:1697-1725) and publishCloudsLast (ToEnd,
// swap, grid rebuild).  The last clouds, the odometry state and the
// correspondence indices live in LDS when they fit (VLP-16 always does).
#include <climits>

#include "lego_device.h"
#include "lego_kernels.h"

namespace lego {

constexpr int kOdomThreads = 512;
constexpr int kOdomWaves = kOdomThreads / 64;
// LDS residency caps (VLP-16 fits entirely; larger sensors fall back to HBM)
constexpr int kLdsSurf = 4096;      // last surf cloud points
constexpr int kLdsCorner = 2048;    // last corner cloud points
constexpr int kLdsQ = 512;          // queries with LDS-resident correspondence indices

// ---------------------------------------------------------------- transforms
struct Trig3 {
  float srx, crx, sry, cry, srz, crz;
};
__device__ __forceinline__ Trig3 trig3(float rx, float ry, float rz) {
  return {lego_sinf(rx), lego_cosf(rx), lego_sinf(ry), lego_cosf(ry), lego_sinf(rz), lego_cosf(rz)};
}

__device__ __forceinline__ float4 to_start(float4 pi, const float* tc) {  // :860-883
  const float s = 10 * (pi.w - (float)(int)pi.w);
  const float rx = s * tc[0], ry = s * tc[1], rz = s * tc[2];
  const float tx = s * tc[3], ty = s * tc[4], tz = s * tc[5];
  const float cz = lego_cosf(rz), sz = lego_sinf(rz), cx = lego_cosf(rx), sx = lego_sinf(rx);
  const float cy = lego_cosf(ry), sy = lego_sinf(ry);
  const float x1 = cz * (pi.x - tx) + sz * (pi.y - ty);
  const float y1 = -sz * (pi.x - tx) + cz * (pi.y - ty);
  const float z1 = (pi.z - tz);
  const float x2 = x1;
  const float y2 = cx * y1 + sx * z1;
  const float z2 = -sx * y1 + cx * z1;
  return make_float4(cy * x2 - sy * z2, y2, sy * x2 + cy * z2, pi.w);
}

// TransformToEnd :885-953 with the IMU terms of an IMU-less run
// (cos/sin of the zero IMU angles; imuShiftFromStart = 0).
struct ImuEnd {
  float cRS, cPS, cYS, sRS, sPS, sYS;  // cosImu*Start / sinImu*Start
  float cYL, sYL, cPL, sPL, cRL, sRL;  // imu*Last
};
__device__ __forceinline__ float4 to_end(float4 pi, const float* tc, const ImuEnd& im) {
  const float s = 10 * (pi.w - (float)(int)pi.w);
  float rx = s * tc[0], ry = s * tc[1], rz = s * tc[2];
  float tx = s * tc[3], ty = s * tc[4], tz = s * tc[5];
  float cz = lego_cosf(rz), sz = lego_sinf(rz), cx = lego_cosf(rx), sx = lego_sinf(rx);
  float cy = lego_cosf(ry), sy = lego_sinf(ry);
  const float x1 = cz * (pi.x - tx) + sz * (pi.y - ty);
  const float y1 = -sz * (pi.x - tx) + cz * (pi.y - ty);
  const float z1 = (pi.z - tz);
  const float x2 = x1;
  const float y2 = cx * y1 + sx * z1;
  const float z2 = -sx * y1 + cx * z1;
  const float x3 = cy * x2 - sy * z2;
  const float y3 = y2;
  const float z3 = sy * x2 + cy * z2;
  rx = tc[0]; ry = tc[1]; rz = tc[2]; tx = tc[3]; ty = tc[4]; tz = tc[5];
  cz = lego_cosf(rz); sz = lego_sinf(rz); cx = lego_cosf(rx); sx = lego_sinf(rx);
  cy = lego_cosf(ry); sy = lego_sinf(ry);
  const float x4 = cy * x3 + sy * z3;
  const float y4 = y3;
  const float z4 = -sy * x3 + cy * z3;
  const float x5 = x4;
  const float y5 = cx * y4 - sx * z4;
  const float z5 = sx * y4 + cx * z4;
  const float x6 = cz * x5 - sz * y5 + tx;
  const float y6 = sz * x5 + cz * y5 + ty;
  const float z6 = z5 + tz;
  const float x7 = im.cRS * (x6 - 0.0f) - im.sRS * (y6 - 0.0f);
  const float y7 = im.sRS * (x6 - 0.0f) + im.cRS * (y6 - 0.0f);
  const float z7 = z6 - 0.0f;
  const float x8 = x7;
  const float y8 = im.cPS * y7 - im.sPS * z7;
  const float z8 = im.sPS * y7 + im.cPS * z7;
  const float x9 = im.cYS * x8 + im.sYS * z8;
  const float y9 = y8;
  const float z9 = -im.sYS * x8 + im.cYS * z8;
  const float x10 = im.cYL * x9 - im.sYL * z9;
  const float y10 = y9;
  const float z10 = im.sYL * x9 + im.cYL * z9;
  const float x11 = x10;
  const float y11 = im.cPL * y10 + im.sPL * z10;
  const float z11 = -im.sPL * y10 + im.cPL * z10;
  return make_float4(im.cRL * x11 + im.sRL * y11, -im.sRL * x11 + im.cRL * y11, z11,
                     (float)(int)pi.w);
}

// AccumulateRotation :1015-1032
__device__ __forceinline__ void accumulate_rotation(float cx, float cy, float cz, float lx, float ly, float lz,
                                    float& ox, float& oy, float& oz) {
  const float clx = lego_cosf(lx), slx = lego_sinf(lx), cly = lego_cosf(ly), sly = lego_sinf(ly);
  const float clz = lego_cosf(lz), slz = lego_sinf(lz);
  const float ccx = lego_cosf(cx), scx = lego_sinf(cx), ccy = lego_cosf(cy), scy = lego_sinf(cy);
  const float ccz = lego_cosf(cz), scz = lego_sinf(cz);
  const float srx = clx * ccx * sly * scz - ccx * ccz * slx - clx * cly * scx;
  ox = -lego_asinf(srx);
  const float srycrx = slx * (ccy * scz - ccz * scx * scy) + clx * sly * (ccy * ccz + scx * scy * scz) +
                       clx * cly * ccx * scy;
  const float crycrx = clx * cly * ccx * ccy - clx * sly * (ccz * scy - ccy * scx * scz) -
                       slx * (scy * scz + ccy * ccz * scx);
  oy = lego_atan2f(srycrx / lego_cosf(ox), crycrx / lego_cosf(ox));
  const float srzcrx = scx * (clz * sly - cly * slx * slz) + ccx * scz * (cly * clz + slx * sly * slz) +
                       clx * ccx * ccz * slz;
  const float crzcrx = clx * clz * ccx * ccz - ccx * scz * (cly * slz - clz * slx * sly) -
                       scx * (sly * slz + cly * clz * slx);
  oz = lego_atan2f(srzcrx / lego_cosf(ox), crzcrx / lego_cosf(ox));
}

// PluginIMURotation :955-1013
__device__ __forceinline__ void plugin_imu_rotation(float bcx, float bcy, float bcz, float blx, float bly, float blz,
                                    float alx, float aly, float alz, float& acx, float& acy,
                                    float& acz) {
  const float sbcx = lego_sinf(bcx), cbcx = lego_cosf(bcx), sbcy = lego_sinf(bcy), cbcy = lego_cosf(bcy);
  const float sbcz = lego_sinf(bcz), cbcz = lego_cosf(bcz);
  const float sblx = lego_sinf(blx), cblx = lego_cosf(blx), sbly = lego_sinf(bly), cbly = lego_cosf(bly);
  const float sblz = lego_sinf(blz), cblz = lego_cosf(blz);
  const float salx = lego_sinf(alx), calx = lego_cosf(alx), saly = lego_sinf(aly), caly = lego_cosf(aly);
  const float salz = lego_sinf(alz), calz = lego_cosf(alz);
  const float srx = -sbcx * (salx * sblx + calx * caly * cblx * cbly + calx * cblx * saly * sbly) -
                    cbcx * cbcz * (calx * saly * (cbly * sblz - cblz * sblx * sbly) -
                                   calx * caly * (sbly * sblz + cbly * cblz * sblx) + cblx * cblz * salx) -
                    cbcx * sbcz * (calx * caly * (cblz * sbly - cbly * sblx * sblz) -
                                   calx * saly * (cbly * cblz + sblx * sbly * sblz) + cblx * salx * sblz);
  acx = -lego_asinf(srx);
  const float srycrx = (cbcy * sbcz - cbcz * sbcx * sbcy) *
                           (calx * saly * (cbly * sblz - cblz * sblx * sbly) -
                            calx * caly * (sbly * sblz + cbly * cblz * sblx) + cblx * cblz * salx) -
                       (cbcy * cbcz + sbcx * sbcy * sbcz) *
                           (calx * caly * (cblz * sbly - cbly * sblx * sblz) -
                            calx * saly * (cbly * cblz + sblx * sbly * sblz) + cblx * salx * sblz) +
                       cbcx * sbcy * (salx * sblx + calx * caly * cblx * cbly + calx * cblx * saly * sbly);
  const float crycrx = (cbcz * sbcy - cbcy * sbcx * sbcz) *
                           (calx * caly * (cblz * sbly - cbly * sblx * sblz) -
                            calx * saly * (cbly * cblz + sblx * sbly * sblz) + cblx * salx * sblz) -
                       (sbcy * sbcz + cbcy * cbcz * sbcx) *
                           (calx * saly * (cbly * sblz - cblz * sblx * sbly) -
                            calx * caly * (sbly * sblz + cbly * cblz * sblx) + cblx * cblz * salx) +
                       cbcx * cbcy * (salx * sblx + calx * caly * cblx * cbly + calx * cblx * saly * sbly);
  acy = lego_atan2f(srycrx / lego_cosf(acx), crycrx / lego_cosf(acx));
  const float srzcrx = sbcx * (cblx * cbly * (calz * saly - caly * salx * salz) -
                               cblx * sbly * (caly * calz + salx * saly * salz) + calx * salz * sblx) -
                       cbcx * cbcz * ((caly * calz + salx * saly * salz) * (cbly * sblz - cblz * sblx * sbly) +
                                      (calz * saly - caly * salx * salz) * (sbly * sblz + cbly * cblz * sblx) -
                                      calx * cblx * cblz * salz) +
                       cbcx * sbcz * ((caly * calz + salx * saly * salz) * (cbly * cblz + sblx * sbly * sblz) +
                                      (calz * saly - caly * salx * salz) * (cblz * sbly - cbly * sblx * sblz) +
                                      calx * cblx * salz * sblz);
  const float crzcrx = sbcx * (cblx * sbly * (caly * salz - calz * salx * saly) -
                               cblx * cbly * (saly * salz + caly * calz * salx) + calx * calz * sblx) +
                       cbcx * cbcz * ((saly * salz + caly * calz * salx) * (sbly * sblz + cbly * cblz * sblx) +
                                      (caly * salz - calz * salx * saly) * (cbly * sblz - cblz * sblx * sbly) +
                                      calx * calz * cblx * cblz) -
                       cbcx * sbcz * ((saly * salz + caly * calz * salx) * (cblz * sbly - cbly * sblx * sblz) +
                                      (caly * salz - calz * salx * saly) * (cbly * cblz + sblx * sbly * sblz) -
                                      calx * calz * cblx * sblz);
  acz = lego_atan2f(srzcrx / lego_cosf(acx), crzcrx / lego_cosf(acx));
}

// In-kernel phase stamps (diagnostic; enabled per launch).  Thread 0 adds
// wall_clock64 deltas (100 MHz) into prof[k].
enum { P_SURF_NN = 0, P_SURF = 1, P_CORN_NN = 2, P_CORN = 3, P_SOLVE = 4, P_INTEG = 5,
       P_TOEND = 6, P_BUILD = 7, P_RESID = 8, P_ITERS_S = 9, P_ITERS_C = 10, P_NNR = 11,
       P_QUERY = 12, P_SCANLINE = 13, P_NN_SHELL1 = 14, P_NN_BRUTE = 15, P_NPROF = 16 };
struct Stamp {
  unsigned long long* prof;
  unsigned long long t;
  __device__ void start() { if (prof && threadIdx.x == 0) t = wall_clock64(); }
  __device__ void add(int k) {
    if (prof && threadIdx.x == 0) { const unsigned long long n = wall_clock64(); prof[k] += n - t; t = n; }
  }
  __device__ void count(int k) { if (prof && threadIdx.x == 0) prof[k] += 1; }
};

// ---------------------------------------------------------------- LDS layout
struct OdomLds {
  float4* lastS;     // [kLdsSurf]  (also the NN-build key scratch)
  float4* lastC;     // [kLdsCorner]
  int* qi;           // [3 * kLdsQ] correspondence indices
  double* red;       // [kOdomWaves * 10]
  float* f;          // 64 scalars
  int* n;            // 64 scalars
  OdomState* st;     // the stream state, resident for the kernel's lifetime
};

__host__ __device__ inline size_t odom_lds_bytes() {
  size_t s = 0;
  s += (size_t)kLdsSurf * 16 + (size_t)kLdsCorner * 16;
  s += (size_t)3 * kLdsQ * 4;
  s += (size_t)kOdomWaves * 10 * 8;
  s += 64 * 4 + 64 * 4;
  s += 128;  // OdomState
  return s;
}

__device__ __forceinline__ OdomLds odom_carve(unsigned char* base) {
  OdomLds L;
  size_t o = 0;
  L.lastS = (float4*)(base + o); o += (size_t)kLdsSurf * 16;
  L.lastC = (float4*)(base + o); o += (size_t)kLdsCorner * 16;
  L.red = (double*)(base + o); o += (size_t)kOdomWaves * 10 * 8;
  L.qi = (int*)(base + o); o += (size_t)3 * kLdsQ * 4;
  L.f = (float*)(base + o); o += 64 * 4;
  L.n = (int*)(base + o); o += 64 * 4;
  L.st = (OdomState*)(base + o); o += 128;
  return L;
}

enum { F_BB = 0 /* bbox 6 */ };
enum { N_BREAK = 0, N_M = 1 };

// ---------------------------------------------------------------- NN index
// Hash grid over a snapshot of the last cloud (taken when the reference would
// rebuild its kd-tree, featureAssociation.cpp:1785-1788): 0.5 m cells, open-
// addressing table, points scattered into cell order by atomic cursors (no
// sort).  A query is served by a 32-lane group: the 27 cells around it, then
// the 98-cell shell, each accepted only when the best distance is provably
// smaller than the covered radius; otherwise (or for small clouds) an exact
// group-wide brute force.  Ties resolve to the lower original index.
constexpr int kG = 32;              // lanes per query group
constexpr float kCell = 0.5f;
constexpr unsigned long long kEmpty = ~0ull;

struct GridView {
  const unsigned long long* keys;
  const int* cnt;
  const int* start;
  const float4* pts;  // cell-ordered snapshot
  const int* idx;     // original index of each slot
  int T, n;
};

__device__ __forceinline__ unsigned long long cell_key(int ix, int iy, int iz) {
  return ((unsigned long long)(unsigned)(ix + (1 << 20)) << 42) |
         ((unsigned long long)(unsigned)(iy + (1 << 20)) << 21) | (unsigned long long)(unsigned)(iz + (1 << 20));
}
__device__ __forceinline__ unsigned hash_key(unsigned long long k) {
  k ^= k >> 33; k *= 0xff51afd7ed558ccdULL; k ^= k >> 33;
  return (unsigned)k;
}
__device__ __forceinline__ int cell_of(float v) { return (int)floorf(v * (1.0f / kCell)); }

__host__ __device__ inline int grid_table_size(int n) {
  int t = 64;
  while (t < 2 * n) t <<= 1;
  return t;
}

// Builds the grid over src[0..n) (all threads; global buffers).
__device__ __forceinline__ void grid_build(const float4* src, int n, unsigned long long* keys, int* cnt, int* start,
                           int* slotOf, float4* pts, int* idx, const OdomLds& L) {
  const int tid = threadIdx.x;
  const int T = grid_table_size(n);
  for (int t = tid; t < T; t += blockDim.x) { keys[t] = kEmpty; cnt[t] = 0; }
  __syncthreads();
  for (int i = tid; i < n; i += blockDim.x) {
    const float4 p = src[i];
    const unsigned long long k = cell_key(cell_of(p.x), cell_of(p.y), cell_of(p.z));
    unsigned s = hash_key(k) & (T - 1);
    while (true) {
      const unsigned long long old = atomicCAS(&keys[s], kEmpty, k);
      if (old == kEmpty || old == k) break;
      s = (s + 1) & (T - 1);
    }
    slotOf[i] = (int)s;
    atomicAdd(&cnt[s], 1);
  }
  __syncthreads();
  // exclusive scan of cnt into start: each thread owns T/blockDim consecutive slots
  {
    const int per = (T + blockDim.x - 1) / blockDim.x;
    const int b0 = tid * per, b1 = min(T, b0 + per);
    int local = 0;
    for (int t = b0; t < b1; ++t) local += cnt[t];
    const int lane = tid & 63, wave = tid >> 6;
    int x = local;
    for (int o2 = 1; o2 < 64; o2 <<= 1) {
      const int y = __shfl_up(x, o2, 64);
      if (lane >= o2) x += y;
    }
    if (lane == 63) L.n[8 + wave] = x;
    __syncthreads();
    int woff = 0;
    for (int w = 0; w < wave; ++w) woff += L.n[8 + w];
    int run = woff + x - local;
    for (int t = b0; t < b1; ++t) { start[t] = run; run += cnt[t]; cnt[t] = 0; }
    __syncthreads();
  }
  for (int i = tid; i < n; i += blockDim.x) {
    const int s = slotOf[i];
    const int pos = start[s] + atomicAdd(&cnt[s], 1);
    pts[pos] = src[i];
    idx[pos] = i;
  }
  __syncthreads();
}

// L2_Simple distance order ((0 + d0^2) + d1^2) + d2^2 (FLANN)
__device__ __forceinline__ float flann_d2(float4 q, float4 p) {
  float r = 0.f, d;
  d = q.x - p.x; r += d * d;
  d = q.y - p.y; r += d * d;
  d = q.z - p.z; r += d * d;
  return r;
}

__device__ __forceinline__ void lex_min(float& d, int& i, float d2, int i2) {
  if (d2 < d || (d2 == d && i2 < i)) { d = d2; i = i2; }
}
__device__ __forceinline__ void group_lex_min(float& d, int& i) {
  for (int o = kG / 2; o > 0; o >>= 1) {
    const float d2 = __shfl_xor(d, o, 64);
    const int i2 = __shfl_xor(i, o, 64);
    lex_min(d, i, d2, i2);
  }
}

__device__ __forceinline__ void scan_cell(const GridView& v, float4 q, int ix, int iy, int iz, float& bd,
                                          int& bi) {
  const unsigned long long k = cell_key(ix, iy, iz);
  unsigned s = hash_key(k) & (v.T - 1);
  while (true) {
    const unsigned long long kk = v.keys[s];
    if (kk == kEmpty) return;
    if (kk == k) break;
    s = (s + 1) & (v.T - 1);
  }
  const int b = v.start[s], e = b + v.cnt[s];
  for (int t = b; t < e; ++t) lex_min(bd, bi, flann_d2(q, v.pts[t]), v.idx[t]);
}

// Exact nearest neighbour with d2 < bound, by the calling 32-lane group.
__device__ __forceinline__ int grid_nn(const GridView& v, float4 q, float bound, int g,
                                       unsigned long long* prof) {
  if (v.n <= 0) return -1;
  float bd = bound;
  int bi = INT_MAX;
  if (v.n > 4 * kG) {
    const int cx = cell_of(q.x), cy = cell_of(q.y), cz = cell_of(q.z);
    // shell 1: the 27 cells (covered radius >= 1 cell)
    if (g < 27) scan_cell(v, q, cx + g % 3 - 1, cy + (g / 3) % 3 - 1, cz + g / 9 - 1, bd, bi);
    group_lex_min(bd, bi);
    if (bd < kCell * kCell * 0.99999f) {
      if (prof && g == 0) atomicAdd(&prof[P_NN_SHELL1], 1ull);
      return (bi != INT_MAX && bd < bound) ? bi : -1;
    }
    // shell 2: the 98 cells at Chebyshev distance 2 (covered radius >= 2 cells)
    for (int c = g; c < 125; c += kG) {
      const int dx = c % 5 - 2, dy = (c / 5) % 5 - 2, dz = c / 25 - 2;
      if (abs(dx) == 2 || abs(dy) == 2 || abs(dz) == 2) scan_cell(v, q, cx + dx, cy + dy, cz + dz, bd, bi);
    }
    group_lex_min(bd, bi);
    if (bd < 4 * kCell * kCell * 0.99999f) return (bi != INT_MAX && bd < bound) ? bi : -1;
  }
  // exact fallback: every point
  if (prof && g == 0) atomicAdd(&prof[P_NN_BRUTE], 1ull);
  for (int t = g; t < v.n; t += kG) lex_min(bd, bi, flann_d2(q, v.pts[t]), v.idx[t]);
  group_lex_min(bd, bi);
  return (bi != INT_MAX && bd < bound) ? bi : -1;
}

__device__ __forceinline__ float line_d2(float4 a, float4 s) {  // the scan-line distance
  return (a.x - s.x) * (a.x - s.x) + (a.y - s.y) * (a.y - s.y) + (a.z - s.z) * (a.z - s.z);
}

// ordered (d, visit order) argmin over the group's candidate lanes
__device__ __forceinline__ void group_argmin(bool cand, float d, int ord, int j, float* bd, int* bj) {
  float v = cand ? d : __builtin_inff();
  int o = cand ? ord : INT_MAX;
  int jj = cand ? j : -1;
  for (int s = kG / 2; s > 0; s >>= 1) {
    const float v2 = __shfl_xor(v, s, 64);
    const int o2 = __shfl_xor(o, s, 64);
    const int j2 = __shfl_xor(jj, s, 64);
    if (v2 < v || (v2 == v && o2 < o)) { v = v2; o = o2; jj = j2; }
  }
  *bd = v;
  *bj = jj;
}

__device__ __forceinline__ unsigned group_ballot(bool p, int gbase) {
  return (unsigned)(__ballot(p) >> gbase);
}

// Scan-line search around `ci` (corner :1062-1099, surf :1173-1220): the
// reference's sequential loops, kG indices per step.  The sequential running
// minimum with a strict < keeps the FIRST point in visiting order among equal
// distances, so every lane keeps a lexicographic (distance, visit rank) minimum
// over the indices it visits and one group reduction combines them.
// int(I) > cScan + 2.5 <=> int(I) > cScan + 2 (and < cScan - 2.5 <=> < cScan - 2).
__device__ __forceinline__ void group_lex_min3(float& d, int& r, int& j) {
  for (int s = kG / 2; s > 0; s >>= 1) {
    const float d2 = __shfl_xor(d, s, 64);
    const int r2 = __shfl_xor(r, s, 64);
    const int j2 = __shfl_xor(j, s, 64);
    if (d2 < d || (d2 == d && r2 < r)) { d = d2; r = r2; j = j2; }
  }
}

__device__ __forceinline__ void scanline_group(const float4* last, int jend, int ci, float4 sel, bool surf,
                                               float nn_sq, int g, int gbase, int* o2, int* o3) {
  const int cScan = (int)last[ci].w;
  float m2 = nn_sq, m3 = nn_sq;
  int r2 = INT_MAX, r3 = INT_MAX, i2 = -1, i3 = -1;
  for (int j0 = ci + 1; j0 < jend; j0 += kG) {
    const int j = j0 + g;
    const bool inr = j < jend;
    float4 p = make_float4(0, 0, 0, 0);
    int rj = 0;
    if (inr) { p = last[j]; rj = (int)p.w; }
    const unsigned bm = group_ballot(inr && rj > cScan + 2, gbase);
    const int lim = bm ? (__ffs(bm) - 1) : kG;
    if (inr && g < lim) {
      const float d = line_d2(p, sel);
      const int rank = j - ci;
      if (surf) {
        if (rj <= cScan) { if (d < m2) { m2 = d; r2 = rank; i2 = j; } }
        else if (d < m3) { m3 = d; r3 = rank; i3 = j; }
      } else if (rj > cScan && d < m2) { m2 = d; r2 = rank; i2 = j; }
    }
    if (bm) break;
  }
  const int fwdSpan = jend - ci;
  for (int j0 = ci - 1; j0 >= 0; j0 -= kG) {
    const int j = j0 - g;
    const bool inr = j >= 0;
    float4 p = make_float4(0, 0, 0, 0);
    int rj = 0;
    if (inr) { p = last[j]; rj = (int)p.w; }
    const unsigned bm = group_ballot(inr && rj < cScan - 2, gbase);
    const int lim = bm ? (__ffs(bm) - 1) : kG;
    if (inr && g < lim) {
      const float d = line_d2(p, sel);
      const int rank = fwdSpan + (ci - j);
      if (surf) {
        if (rj >= cScan) { if (d < m2) { m2 = d; r2 = rank; i2 = j; } }
        else if (d < m3) { m3 = d; r3 = rank; i3 = j; }
      } else if (rj < cScan && d < m2) { m2 = d; r2 = rank; i2 = j; }
    }
    if (bm) break;
  }
  group_lex_min3(m2, r2, i2);
  if (surf) group_lex_min3(m3, r3, i3);
  *o2 = i2;
  *o3 = surf ? i3 : -1;
}

// ---------------------------------------------------------------- reduction
// 9 doubles (AtA upper triangle 6 + AtB 3) + the row count over the block.
__device__ __forceinline__ void block_sum9(double v[9], int m, const OdomLds& L, double out[9], int* mt) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int k = 0; k < 9; ++k)
    for (int o = 32; o > 0; o >>= 1) v[k] += __shfl_xor(v[k], o, 64);
  for (int o = 32; o > 0; o >>= 1) m += __shfl_xor(m, o, 64);
  if (lane == 0) {
    for (int k = 0; k < 9; ++k) L.red[wave * 10 + k] = v[k];
    L.red[wave * 10 + 9] = (double)m;
  }
  __syncthreads();
  for (int k = 0; k < 9; ++k) {
    double s = 0;
    for (int w = 0; w < kOdomWaves; ++w) s += L.red[w * 10 + k];
    out[k] = s;
  }
  double ms = 0;
  for (int w = 0; w < kOdomWaves; ++w) ms += L.red[w * 10 + 9];
  *mt = (int)ms;
}

struct ScanFeat {
  const float4* sharp; int nSharp;
  const float4* lsharp; int nLS;
  const float4* flat; int nFlat;
  const float4* lflat; int nLF;
};

// Shared tail of calculateTransformationSurf / Corner.  Thread 0 only.
__device__ __forceinline__ void solve_step(float (&AtA)[3][3], float (&AtB)[3], int iter, OdomState* st,
                           float (&X)[3]) {
  float Aq[3][3];
  for (int a = 0; a < 3; ++a) for (int b = 0; b < 3; ++b) Aq[a][b] = AtA[a][b];
  cv_solve_qr<3, 3>(Aq, AtB, X);
  float (&P)[3][3] = *reinterpret_cast<float(*)[3][3]>(st->matP);
  if (iter == 0) {
    float E[3], V[3][3], V2[3][3], Ae[3][3];
    for (int a = 0; a < 3; ++a) for (int b = 0; b < 3; ++b) Ae[a][b] = AtA[a][b];
    cv_eigen_sym<3>(Ae, E, V);
    for (int a = 0; a < 3; ++a) for (int b = 0; b < 3; ++b) V2[a][b] = V[a][b];
    st->isDegenerate = 0;
    for (int i = 2; i >= 0; i--) {
      if (E[i] < 10) {
        for (int j = 0; j < 3; j++) V2[i][j] = 0;
        st->isDegenerate = 1;
      } else {
        break;
      }
    }
    float Vi[3][3];
    cv_inv3(V, Vi);
    cv_matmul<3>(Vi, V2, P);
  }
  if (st->isDegenerate) {
    float X2[3] = {X[0], X[1], X[2]};
    cv_matvec<3>(P, X2, X);
  }
}

__device__ __forceinline__ double r2d(double r) { return r * 180.0 / M_PI; }

// One LM loop (surf: <= 25 x {findCorrespondingSurfFeatures;
// calculateTransformationSurf}; corner likewise) — updateTransformation :1666-1695.
__device__ __forceinline__ void lm_loop(bool surf, const ScanFeat& F, const float4* last, int lastN,
                        const GridView& nn, OdomState* st, const OdomLds& L, int* gqi,
                        const DevCfg& c, Stamp& S) {
  const int tid = threadIdx.x;
  const float4* qp = surf ? F.flat : F.sharp;
  const int nQ = surf ? F.nFlat : F.nSharp;
  const int jend = min(nQ, lastN);  // the reference bounds by the query count (:1062, :1173)
  int* qi = (nQ <= kLdsQ) ? L.qi : gqi;
  const int qs = (nQ <= kLdsQ) ? kLdsQ : nQ;  // stride between the three index arrays
  const int g = tid & (kG - 1), gbase = tid & 63 & ~(kG - 1), grp = tid / kG;
  const int ngrp = blockDim.x / kG;
  for (int it = 0; it < 25; it++) {
    S.start();
    S.count(surf ? P_ITERS_S : P_ITERS_C);
    if (it % 5 == 0) S.count(P_NNR);
    float tc[6];
    for (int i = 0; i < 6; ++i) tc[i] = st->transformCur[i];
    const float srx = lego_sinf(tc[0]), crx = lego_cosf(tc[0]);
    const float sry = lego_sinf(tc[1]), cry = lego_cosf(tc[1]);
    const float srz = lego_sinf(tc[2]), crz = lego_cosf(tc[2]);
    const float tx = tc[3], ty = tc[4], tz = tc[5];
    double acc[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    int mloc = 0;
    if (it % 5 == 0) {
      // nearest neighbour + scan-line search, one 32-lane group per query
      for (int q = grp; q < nQ; q += ngrp) {
        const float4 sel = to_start(qp[q], tc);
        int i1 = grid_nn(nn, sel, c.nn_sq, g, S.prof);
        if (i1 >= lastN) i1 = -1;  // stale snapshot of a larger cloud
        int i2 = -1, i3 = -1;
        if (i1 >= 0) scanline_group(last, jend, i1, sel, surf, c.nn_sq, g, gbase, &i2, &i3);
        if (g == 0) { qi[q] = i1; qi[qs + q] = i2; qi[2 * qs + q] = i3; }
      }
      __syncthreads();
      S.add(P_QUERY);
    }
    for (int q = tid; q < nQ; q += blockDim.x) {
      const float4 po = qp[q];
      const float4 sel = to_start(po, tc);
      const int i1 = qi[q], i2 = qi[qs + q], i3 = qi[2 * qs + q];
      float4 cf;
      bool ok = false;
      if (surf) {
        if (i2 >= 0 && i3 >= 0) {
          const float4 t1 = last[i1], t2 = last[i2], t3 = last[i3];
          float pa = (t2.y - t1.y) * (t3.z - t1.z) - (t3.y - t1.y) * (t2.z - t1.z);
          float pb = (t2.z - t1.z) * (t3.x - t1.x) - (t3.z - t1.z) * (t2.x - t1.x);
          float pc = (t2.x - t1.x) * (t3.y - t1.y) - (t3.x - t1.x) * (t2.y - t1.y);
          float pd = -(pa * t1.x + pb * t1.y + pc * t1.z);
          const float ps = __builtin_sqrtf(pa * pa + pb * pb + pc * pc);
          pa /= ps; pb /= ps; pc /= ps; pd /= ps;
          const float pd2 = pa * sel.x + pb * sel.y + pc * sel.z + pd;
          float s = 1;
          if (it >= 5)
            s = (float)(1 - 1.8 * (double)lfabsf(pd2) /
                                (double)__builtin_sqrtf(__builtin_sqrtf(sel.x * sel.x + sel.y * sel.y + sel.z * sel.z)));
          if ((double)s > 0.1 && pd2 != 0) {
            ok = true;
            cf = make_float4(s * pa, s * pb, s * pc, s * pd2);
          }
        }
      } else {
        if (i2 >= 0) {
          const float4 t1 = last[i1], t2 = last[i2];
          const float x0 = sel.x, y0 = sel.y, z0 = sel.z;
          const float x1 = t1.x, y1 = t1.y, z1 = t1.z, x2 = t2.x, y2 = t2.y, z2 = t2.z;
          const float m11 = ((x0 - x1) * (y0 - y2) - (x0 - x2) * (y0 - y1));
          const float m22 = ((x0 - x1) * (z0 - z2) - (x0 - x2) * (z0 - z1));
          const float m33 = ((y0 - y1) * (z0 - z2) - (y0 - y2) * (z0 - z1));
          const float a012 = __builtin_sqrtf(m11 * m11 + m22 * m22 + m33 * m33);
          const float l12 = __builtin_sqrtf((x1 - x2) * (x1 - x2) + (y1 - y2) * (y1 - y2) + (z1 - z2) * (z1 - z2));
          const float la = ((y1 - y2) * m11 + (z1 - z2) * m22) / a012 / l12;
          const float lb = -((x1 - x2) * m11 - (z1 - z2) * m33) / a012 / l12;
          const float lc = -((x1 - x2) * m22 + (y1 - y2) * m33) / a012 / l12;
          const float ld2 = a012 / l12;
          float s = 1;
          if (it >= 5) s = (float)(1 - 1.8 * (double)lfabsf(ld2));
          if ((double)s > 0.1 && ld2 != 0) {
            ok = true;
            cf = make_float4(s * la, s * lb, s * lc, s * ld2);
          }
        }
      }
      if (ok) {
        float a0, a1, a2;
        if (surf) {  // :1291-1321
          const float a1_ = crx * sry * srz, a2_ = crx * crz * sry, a3 = srx * sry, a4 = tx * a1_ - ty * a2_ - tz * a3;
          const float a5 = srx * srz, a6 = crz * srx, a7 = ty * a6 - tz * crx - tx * a5;
          const float a8 = crx * cry * srz, a9 = crx * cry * crz, a10 = cry * srx, a11 = tz * a10 + ty * a9 - tx * a8;
          const float b1 = -crz * sry - cry * srx * srz, b2 = cry * crz * srx - sry * srz;
          const float b5 = cry * crz - srx * sry * srz, b6 = cry * srz + crz * srx * sry;
          const float c1 = -b6, c2 = b5, c3 = tx * b6 - ty * b5, c4 = -crx * crz, c5 = crx * srz;
          const float c6 = ty * c5 + tx * -c4;
          const float c7 = b2, c8 = -b1, c9 = tx * -b2 - ty * -b1;
          a0 = (-a1_ * po.x + a2_ * po.y + a3 * po.z + a4) * cf.x +
               (a5 * po.x - a6 * po.y + crx * po.z + a7) * cf.y +
               (a8 * po.x - a9 * po.y - a10 * po.z + a11) * cf.z;
          a1 = (c1 * po.x + c2 * po.y + c3) * cf.x + (c4 * po.x - c5 * po.y + c6) * cf.y +
               (c7 * po.x + c8 * po.y + c9) * cf.z;
          a2 = -b6 * cf.x + c4 * cf.y + b2 * cf.z;
        } else {  // :1400-1423
          const float b1 = -crz * sry - cry * srx * srz, b2 = cry * crz * srx - sry * srz, b3 = crx * cry;
          const float b4 = tx * -b1 + ty * -b2 + tz * b3;
          const float b5 = cry * crz - srx * sry * srz, b6 = cry * srz + crz * srx * sry, b7 = crx * sry;
          const float b8 = tz * b7 - ty * b6 - tx * b5;
          const float c5 = crx * srz;
          a0 = (b1 * po.x + b2 * po.y - b3 * po.z + b4) * cf.x + (b5 * po.x + b6 * po.y - b7 * po.z + b8) * cf.z;
          a1 = -b5 * cf.x + c5 * cf.y + b1 * cf.z;
          a2 = b7 * cf.x - srx * cf.y - b3 * cf.z;
        }
        const float bb = (float)(-0.05 * (double)cf.w);
        const double d0 = a0, d1 = a1, d2 = a2, db = bb;
        acc[0] += d0 * d0; acc[1] += d0 * d1; acc[2] += d0 * d2;
        acc[3] += d1 * d1; acc[4] += d1 * d2; acc[5] += d2 * d2;
        acc[6] += d0 * db; acc[7] += d1 * db; acc[8] += d2 * db;
        mloc++;
      }
    }
    double tot[9];
    int M;
    block_sum9(acc, mloc, L, tot, &M);
    S.add(surf ? (it % 5 == 0 ? P_SURF_NN : P_SURF) : (it % 5 == 0 ? P_CORN_NN : P_CORN));
    if (tid == 0) {
      L.n[N_BREAK] = 0;
      if (M >= 10) {
        float AtA[3][3] = {{(float)tot[0], (float)tot[1], (float)tot[2]},
                           {(float)tot[1], (float)tot[3], (float)tot[4]},
                           {(float)tot[2], (float)tot[4], (float)tot[5]}};
        float AtB[3] = {(float)tot[6], (float)tot[7], (float)tot[8]};
        float X[3];
        solve_step(AtA, AtB, it, st, X);
        float* t = st->transformCur;
        double dR, dT;
        if (surf) {
          t[0] += X[0]; t[2] += X[1]; t[4] += X[2];
        } else {
          t[1] += X[0]; t[3] += X[1]; t[5] += X[2];
        }
        for (int i = 0; i < 6; i++) if (__builtin_isnan(t[i])) t[i] = 0;
        if (surf) {
          const double r0 = r2d(X[0]), r1 = r2d(X[1]), t2 = (double)(X[2] * 100);
          dR = (double)(float)__builtin_sqrt(r0 * r0 + r1 * r1);
          dT = (double)(float)__builtin_sqrt(t2 * t2);
        } else {
          const double r0 = r2d(X[0]), t1 = (double)(X[1] * 100), t2 = (double)(X[2] * 100);
          dR = (double)(float)__builtin_sqrt(r0 * r0);
          dT = (double)(float)__builtin_sqrt(t1 * t1 + t2 * t2);
        }
        if (dR < 0.1 && dT < 0.1) L.n[N_BREAK] = 1;
      }
      __threadfence_block();
    }
    __syncthreads();
    S.add(P_SOLVE);
    const int brk = L.n[N_BREAK];
    __syncthreads();
    if (brk) break;
  }
}

// Copies the last clouds into LDS when they fit.
struct Resident {
  const float4* lastS;
  const float4* lastC;
  GridView nnS, nnC;
};

__device__ __forceinline__ void make_resident(const OdomBufs& ob, const OdomState* st, const OdomLds& L, Resident& R) {
  const int tid = threadIdx.x;
  const int ns = st->surfLastNum, nc = st->cornerLastNum;
  R.lastS = ns <= kLdsSurf ? L.lastS : ob.surfLast;
  R.lastC = nc <= kLdsCorner ? L.lastC : ob.cornerLast;
  R.nnS = GridView{ob.gS.keys, ob.gS.cnt, ob.gS.start, ob.gS.pts, ob.gS.idx,
                   grid_table_size(st->nnSurfNum), st->nnSurfNum};
  R.nnC = GridView{ob.gC.keys, ob.gC.cnt, ob.gC.start, ob.gC.pts, ob.gC.idx,
                   grid_table_size(st->nnCornerNum), st->nnCornerNum};
  if (ns <= kLdsSurf) for (int t = tid; t < ns; t += blockDim.x) L.lastS[t] = ob.surfLast[t];
  if (nc <= kLdsCorner) for (int t = tid; t < nc; t += blockDim.x) L.lastC[t] = ob.cornerLast[t];
  __syncthreads();
}

__global__ void __launch_bounds__(kOdomThreads) k_odom(BatchBufs bb, OdomBufs ob, DevCfg c, int B,
                                                      unsigned long long* gkeys, int* gqi,
                                                      unsigned long long* prof) {
  Stamp S{prof, 0};
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
  const OdomLds L = odom_carve(lds_raw);
  const int tid = threadIdx.x;
  static_assert(sizeof(OdomState) <= 128, "OdomState LDS slot");
  OdomState* st = L.st;
  if (tid < (int)(sizeof(OdomState) / 4)) ((int*)st)[tid] = ((const int*)ob.st)[tid];
  __syncthreads();
  Resident R;
  S.start();
  make_resident(ob, st, L, R);
  S.add(P_RESID);
  const ImuEnd im{1.f, 1.f, 1.f, 0.f, 0.f, 0.f, 1.f, 0.f, 1.f, 0.f, 1.f, 0.f};
  for (int b = 0; b < B; ++b) {
    ScanFeat F;
    const int* fc = bb.f_cnt + b * 4;
    F.sharp = bb.f_sharp + (size_t)b * c.N * kSharpPerRing; F.nSharp = fc[0];
    F.lsharp = bb.f_lsharp + (size_t)b * c.N * kLessSharpPerRing; F.nLS = fc[1];
    F.flat = bb.f_flat + (size_t)b * c.N * kFlatPerRing; F.nFlat = fc[2];
    F.lflat = bb.f_lflat + (size_t)b * c.P; F.nLF = fc[3];
    float4* cEnd = ob.cornerEnd + (size_t)b * ob.capLS;
    float4* sEnd = ob.surfEnd + (size_t)b * c.P;
    const bool init = !st->inited;
    if (!init) {
      // updateInitialGuess is a no-op without IMU
      if (st->cornerLastNum >= 10 && st->surfLastNum >= 100) {
        lm_loop(true, F, R.lastS, st->surfLastNum, R.nnS, st, L, gqi, c, S);
        lm_loop(false, F, R.lastC, st->cornerLastNum, R.nnC, st, L, gqi, c, S);
      }
      // integrateTransformation :1697-1725
      S.start();
      if (tid == 0) {
        float* ts = st->transformSum;
        const float* tc = st->transformCur;
        float rx, ry, rz;
        accumulate_rotation(ts[0], ts[1], ts[2], -tc[0], -tc[1], -tc[2], rx, ry, rz);
        const float x1 = lego_cosf(rz) * (tc[3] - 0.0f) - lego_sinf(rz) * (tc[4] - 0.0f);
        const float y1 = lego_sinf(rz) * (tc[3] - 0.0f) + lego_cosf(rz) * (tc[4] - 0.0f);
        const float z1 = tc[5] - 0.0f;
        const float x2 = x1;
        const float y2 = lego_cosf(rx) * y1 - lego_sinf(rx) * z1;
        const float z2 = lego_sinf(rx) * y1 + lego_cosf(rx) * z1;
        const float tx = ts[3] - (lego_cosf(ry) * x2 + lego_sinf(ry) * z2);
        const float ty = ts[4] - y2;
        const float tz = ts[5] - (-lego_sinf(ry) * x2 + lego_cosf(ry) * z2);
        plugin_imu_rotation(rx, ry, rz, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, rx, ry, rz);
        ts[0] = rx; ts[1] = ry; ts[2] = rz; ts[3] = tx; ts[4] = ty; ts[5] = tz;
        __threadfence_block();
      }
      __syncthreads();
      S.add(P_INTEG);
    }
    S.start();
    // hand-off: checkSystemInitialization (:1605-1637, no TransformToEnd) or
    // publishCloudsLast (:1759-1815)
    float tcur[6];
    for (int i = 0; i < 6; ++i) tcur[i] = st->transformCur[i];
    for (int t = tid; t < F.nLS; t += blockDim.x) {
      const float4 p = init ? F.lsharp[t] : to_end(F.lsharp[t], tcur, im);
      ob.cornerLast[t] = p;
      cEnd[t] = p;
    }
    for (int t = tid; t < F.nLF; t += blockDim.x) {
      const float4 p = init ? F.lflat[t] : to_end(F.lflat[t], tcur, im);
      ob.surfLast[t] = p;
      sEnd[t] = p;
    }
    __syncthreads();
    S.add(P_TOEND);
    const bool rebuild = init || (F.nLS > 10 && F.nLF > 100);
    unsigned long long tb = 0;
    if (prof && tid == 0) tb = wall_clock64();
    if (rebuild) {
      grid_build(ob.cornerLast, F.nLS, ob.gC.keys, ob.gC.cnt, ob.gC.start, ob.gC.slot, ob.gC.pts, ob.gC.idx, L);
      grid_build(ob.surfLast, F.nLF, ob.gS.keys, ob.gS.cnt, ob.gS.start, ob.gS.slot, ob.gS.pts, ob.gS.idx, L);
    }
    if (prof && tid == 0) prof[P_BUILD] += wall_clock64() - tb;
    if (tid == 0) {
      st->cornerLastNum = F.nLS;
      st->surfLastNum = F.nLF;
      if (rebuild) { st->nnCornerNum = F.nLS; st->nnSurfNum = F.nLF; }
      int pub = 0;
      if (init) {
        st->transformSum[0] += 0.0f;  // += imuPitchStart
        st->transformSum[2] += 0.0f;  // += imuRollStart
        st->inited = 1;
      } else {
        st->frameCount++;
        if (st->frameCount >= c.skip + 1) { st->frameCount = 0; pub = 1; }
      }
      ob.validOut[b] = init ? 0 : 1;
      ob.pubOut[b] = pub;
      for (int i = 0; i < 6; ++i) { ob.sumOut[b * 6 + i] = st->transformSum[i]; ob.curOut[b * 6 + i] = st->transformCur[i]; }
      __threadfence_block();
    }
    __syncthreads();
    S.start();
    make_resident(ob, st, L, R);
    S.add(P_RESID);
  }
  __syncthreads();
  if (tid < (int)(sizeof(OdomState) / 4)) ((int*)ob.st)[tid] = ((const int*)st)[tid];
}

size_t odom_grid_table(int npts) { return (size_t)grid_table_size(npts); }

void launch_odom(const BatchBufs& bb, const OdomBufs& ob, const DevCfg& c, int B, hipStream_t s,
                 StageTimer* tm, unsigned long long* gkeys, int* gqi, unsigned long long* prof) {
  tm->mark("odom.lm", s);
  k_odom<<<1, kOdomThreads, odom_lds_bytes(), s>>>(bb, ob, c, B, gkeys, gqi, prof);
}

}  // namespace lego
