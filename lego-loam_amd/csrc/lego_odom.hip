// lego_odom.hip — the two-step LM odometry of featureAssociation on gfx950.
//
// One persistent 1024-thread workgroup walks the batch's scans in stream order
// (scan k's problem depends on scan k-1's result through transformCur and the
// TransformToEnd'ed "last" clouds, featureAssociation.cpp:1759-1815), so the
// per-scan chain never returns to the host.  Per LM iteration:
//   A  1 lane / query : TransformToStart                         (:860-883)
//   B  1 wave / query : nearest neighbour (every 5th iteration) in an LBVH
//                       over the last cloud — exact, replaces KdTreeFLANN
//                       (:1054,1165; ties -> lower index, FLANN's are
//                       traversal-order dependent) — then the scan-line search
//                       as ordered wave ballots (:1062-1099, :1173-1220),
//                       keeping the reference's loop-bound quirk
//   C  1 lane / query : line / plane residual, weight, row      (:1106-1151, 1228-1266)
//   D  block reduce   : AtA, AtB with double accumulation (cv::gemm's float
//                       path accumulates in double)
//   E  lane 0         : QR solve, iteration-0 eigen degeneracy projection,
//                       update, NaN reset, convergence (:1324-1376, :1425-1477)
// then integrateTransformation (:1697-1725) and publishCloudsLast.
#include <climits>

#include "lego_device.h"
#include "lego_kernels.h"

namespace lego {

constexpr int kOdomThreads = 1024;
constexpr int kOdomWaves = kOdomThreads / 64;
constexpr int kLeaf = 64;
constexpr int kLdsSortKeys = 16384;

// ---------------------------------------------------------------- transforms
struct Trig3 {
  float srx, crx, sry, cry, srz, crz;
};
__device__ __forceinline__ Trig3 trig3(float rx, float ry, float rz) {
  return {lego_sinf(rx), lego_cosf(rx), lego_sinf(ry), lego_cosf(ry), lego_sinf(rz), lego_cosf(rz)};
}

__device__ float4 to_start(float4 pi, const float* tc) {  // :860-883
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
__device__ float4 to_end(float4 pi, const float* tc, const ImuEnd& im) {
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
__device__ void accumulate_rotation(float cx, float cy, float cz, float lx, float ly, float lz,
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
__device__ void plugin_imu_rotation(float bcx, float bcy, float bcz, float blx, float bly, float blz,
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

// ---------------------------------------------------------------- LDS layout
struct OdomLds {
  unsigned long long* keys;  // NN build (union with the query arrays)
  float4* sel;               // [capQ] transformed queries
  int* i1;                   // [capQ]
  int* i2;
  int* i3;
  int* acc;                  // [capQ] row accepted
  int* stack;                // [kOdomWaves * 64]
  double* red;               // [kOdomWaves * 10]
  float* f;                  // scalars: transformCur etc.
  int* n;                    // int scalars
};

__host__ __device__ inline size_t odom_lds_bytes() {
  size_t s = (size_t)kLdsSortKeys * 8;                   // keys / query union
  s += (size_t)kOdomWaves * 64 * 4;                      // stacks
  s += (size_t)kOdomWaves * 10 * 8;                      // reduce
  s += 64 * 4 + 64 * 4;                                  // scalars
  return s;
}
__host__ __device__ inline int odom_cap_q() {
  // sel(16) + i1,i2,i3,acc(16) per query inside the 128 KiB union
  return (kLdsSortKeys * 8) / 32;
}

__device__ OdomLds odom_carve(unsigned char* base) {
  OdomLds L;
  size_t o = 0;
  L.keys = (unsigned long long*)(base + o);
  const int capQ = odom_cap_q();
  L.sel = (float4*)(base + o);
  L.i1 = (int*)(base + o + (size_t)capQ * 16);
  L.i2 = L.i1 + capQ;
  L.i3 = L.i2 + capQ;
  L.acc = L.i3 + capQ;
  o += (size_t)kLdsSortKeys * 8;
  L.stack = (int*)(base + o); o += (size_t)kOdomWaves * 64 * 4;
  L.red = (double*)(base + o); o += (size_t)kOdomWaves * 10 * 8;
  L.f = (float*)(base + o); o += 64 * 4;
  L.n = (int*)(base + o); o += 64 * 4;
  return L;
}

// scalar slots in L.f / L.n
enum { F_CUR = 0, F_SUM = 6, F_MATP = 12, F_BB = 21 /* bbox 6 */ };
enum { N_BREAK = 0, N_M = 1, N_DONE = 2, N_TMP = 3 };

// ---------------------------------------------------------------- NN index
struct NNIndex {
  float4* pts;   // sorted points (w = original intensity)
  int* idx;      // original index of each sorted slot
  float4* box;   // [2 * 2*L2]: lo at 2*node, hi at 2*node+1
  int n, L2;
};

__device__ void bitonic_u64_any(unsigned long long* a, int m) {
  for (int k = 2; k <= m; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int t = threadIdx.x; t < m / 2; t += blockDim.x) {
        const int i = (t / j) * 2 * j + (t % j);
        const int l = i + j;
        const bool up = (i & k) == 0;
        const unsigned long long x = a[i], y = a[l];
        if ((x > y) == up) { a[i] = y; a[l] = x; }
      }
      __syncthreads();
    }
  }
}

__device__ __forceinline__ unsigned spread10(unsigned v) {
  v &= 1023u;
  v = (v | (v << 16)) & 0x030000FFu;
  v = (v | (v << 8)) & 0x0300F00Fu;
  v = (v | (v << 4)) & 0x030C30C3u;
  v = (v | (v << 2)) & 0x09249249u;
  return v;
}

// Builds the LBVH over src[0..n): Morton-sorted 64-point leaves under an
// implicit complete binary tree (node 1 = root, leaves at [L2, 2*L2)).
__device__ void nn_build(const float4* src, int n, NNIndex& ix, const OdomLds& L,
                         unsigned long long* gkeys) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  float mn[3] = {__builtin_inff(), __builtin_inff(), __builtin_inff()};
  float mx[3] = {-__builtin_inff(), -__builtin_inff(), -__builtin_inff()};
  for (int t = tid; t < n; t += blockDim.x) {
    const float4 p = src[t];
    mn[0] = fminf(mn[0], p.x); mn[1] = fminf(mn[1], p.y); mn[2] = fminf(mn[2], p.z);
    mx[0] = fmaxf(mx[0], p.x); mx[1] = fmaxf(mx[1], p.y); mx[2] = fmaxf(mx[2], p.z);
  }
  for (int q = 0; q < 3; ++q)
    for (int o = 32; o > 0; o >>= 1) {
      mn[q] = fminf(mn[q], __shfl_xor(mn[q], o, 64));
      mx[q] = fmaxf(mx[q], __shfl_xor(mx[q], o, 64));
    }
  float* red = (float*)L.red;
  if (lane == 0)
    for (int q = 0; q < 3; ++q) { red[wave * 6 + q] = mn[q]; red[wave * 6 + 3 + q] = mx[q]; }
  __syncthreads();
  if (tid < 6) {
    float v = red[tid];
    for (int w = 1; w < kOdomWaves; ++w) v = tid < 3 ? fminf(v, red[w * 6 + tid]) : fmaxf(v, red[w * 6 + tid]);
    L.f[F_BB + tid] = v;
  }
  __syncthreads();
  const float lo0 = L.f[F_BB], lo1 = L.f[F_BB + 1], lo2 = L.f[F_BB + 2];
  const float s0 = 1023.0f / fmaxf(L.f[F_BB + 3] - lo0, 1e-6f);
  const float s1 = 1023.0f / fmaxf(L.f[F_BB + 4] - lo1, 1e-6f);
  const float s2 = 1023.0f / fmaxf(L.f[F_BB + 5] - lo2, 1e-6f);
  int m = 1;
  while (m < n) m <<= 1;
  unsigned long long* keys = (m <= kLdsSortKeys) ? L.keys : gkeys;
  for (int t = tid; t < m; t += blockDim.x) {
    unsigned long long k = ~0ull;
    if (t < n) {
      const float4 p = src[t];
      const unsigned mc = (spread10((unsigned)((p.x - lo0) * s0)) << 2) |
                          (spread10((unsigned)((p.y - lo1) * s1)) << 1) |
                          spread10((unsigned)((p.z - lo2) * s2));
      k = ((unsigned long long)mc << 32) | (unsigned)t;
    }
    keys[t] = k;
  }
  __syncthreads();
  bitonic_u64_any(keys, m);
  for (int t = tid; t < n; t += blockDim.x) {
    const int o = (int)(keys[t] & 0xffffffffu);
    ix.pts[t] = src[o];
    ix.idx[t] = o;
  }
  __syncthreads();
  const int nleaf = (n + kLeaf - 1) / kLeaf;
  int L2 = 1;
  while (L2 < nleaf) L2 <<= 1;
  ix.n = n;
  ix.L2 = L2;
  // leaf boxes: one wave per leaf
  for (int l = wave; l < L2; l += kOdomWaves) {
    const int s = l * kLeaf + lane;
    float a[3] = {__builtin_inff(), __builtin_inff(), __builtin_inff()};
    float z[3] = {-__builtin_inff(), -__builtin_inff(), -__builtin_inff()};
    if (s < n) {
      const float4 p = ix.pts[s];
      a[0] = z[0] = p.x; a[1] = z[1] = p.y; a[2] = z[2] = p.z;
    }
    for (int q = 0; q < 3; ++q)
      for (int o = 32; o > 0; o >>= 1) {
        a[q] = fminf(a[q], __shfl_xor(a[q], o, 64));
        z[q] = fmaxf(z[q], __shfl_xor(z[q], o, 64));
      }
    if (lane == 0) {
      ix.box[2 * (L2 + l)] = make_float4(a[0], a[1], a[2], 0);
      ix.box[2 * (L2 + l) + 1] = make_float4(z[0], z[1], z[2], 0);
    }
  }
  __syncthreads();
  for (int lvl = L2 >> 1; lvl >= 1; lvl >>= 1) {
    for (int nd = lvl + tid; nd < 2 * lvl; nd += blockDim.x) {
      const float4 al = ix.box[2 * (2 * nd)], ah = ix.box[2 * (2 * nd) + 1];
      const float4 bl = ix.box[2 * (2 * nd + 1)], bh = ix.box[2 * (2 * nd + 1) + 1];
      ix.box[2 * nd] = make_float4(fminf(al.x, bl.x), fminf(al.y, bl.y), fminf(al.z, bl.z), 0);
      ix.box[2 * nd + 1] = make_float4(fmaxf(ah.x, bh.x), fmaxf(ah.y, bh.y), fmaxf(ah.z, bh.z), 0);
    }
    __syncthreads();
  }
}

__device__ __forceinline__ float box_d2(const NNIndex& ix, int nd, float4 q) {
  const float4 lo = ix.box[2 * nd], hi = ix.box[2 * nd + 1];
  const float gx = lo.x - q.x > 0 ? lo.x - q.x : (q.x - hi.x > 0 ? q.x - hi.x : 0.f);
  const float gy = lo.y - q.y > 0 ? lo.y - q.y : (q.y - hi.y > 0 ? q.y - hi.y : 0.f);
  const float gz = lo.z - q.z > 0 ? lo.z - q.z : (q.z - hi.z > 0 ? q.z - hi.z : 0.f);
  return gx * gx + gy * gy + gz * gz;
}

// L2_Simple distance order ((0 + d0^2) + d1^2) + d2^2 (FLANN)
__device__ __forceinline__ float flann_d2(float4 q, float4 p) {
  float r = 0.f, d;
  d = q.x - p.x; r += d * d;
  d = q.y - p.y; r += d * d;
  d = q.z - p.z; r += d * d;
  return r;
}

// One wave: exact nearest neighbour with d2 < bound (ties -> lower original
// index).  Returns the original index or -1.
__device__ int nn_query_wave(const NNIndex& ix, float4 q, float bound, int* stack) {
  const int lane = threadIdx.x & 63;
  if (ix.n <= 0) return -1;
  float best = bound;
  int bestIdx = INT_MAX;
  int sp = 0;
  if (lane == 0) stack[0] = 1;
  sp = 1;
  __builtin_amdgcn_wave_barrier();
  while (sp > 0) {
    const int nd = ((volatile int*)stack)[sp - 1];
    --sp;
    const float bd = box_d2(ix, nd, q);
    if (bd > best * 1.0001f + 1e-6f) continue;
    if (nd >= ix.L2) {
      const int s = (nd - ix.L2) * kLeaf + lane;
      float d = __builtin_inff();
      int id = INT_MAX;
      if (s < ix.n) {
        d = flann_d2(q, ix.pts[s]);
        id = ix.idx[s];
      }
      // wave lexicographic min of (d, id)
      for (int o = 32; o > 0; o >>= 1) {
        const float d2 = __shfl_xor(d, o, 64);
        const int i2 = __shfl_xor(id, o, 64);
        if (d2 < d || (d2 == d && i2 < id)) { d = d2; id = i2; }
      }
      if (d < best || (d == best && id < bestIdx)) { best = d; bestIdx = id; }
    } else {
      const int a = 2 * nd, b = 2 * nd + 1;
      const float da = box_d2(ix, a, q), db = box_d2(ix, b, q);
      const int nearC = da <= db ? a : b, farC = da <= db ? b : a;
      if (lane == 0) {
        ((volatile int*)stack)[sp] = farC;
        ((volatile int*)stack)[sp + 1] = nearC;
      }
      sp += 2;
      __builtin_amdgcn_wave_barrier();
    }
  }
  return (bestIdx != INT_MAX && best < bound) ? bestIdx : -1;
}

// lexicographic (d, order) min across the wave among `cand` lanes
__device__ __forceinline__ void wave_argmin(bool cand, float d, int order, int j, float* bd, int* bo,
                                            int* bj) {
  float v = cand ? d : __builtin_inff();
  int o = cand ? order : INT_MAX;
  int jj = cand ? j : -1;
  for (int s = 32; s > 0; s >>= 1) {
    const float v2 = __shfl_xor(v, s, 64);
    const int o2 = __shfl_xor(o, s, 64);
    const int j2 = __shfl_xor(jj, s, 64);
    if (v2 < v || (v2 == v && o2 < o)) { v = v2; o = o2; jj = j2; }
  }
  *bd = v;
  *bo = o;
  *bj = jj;
}

__device__ __forceinline__ float line_d2(float4 a, float4 s) {  // the scan-line distance
  return (a.x - s.x) * (a.x - s.x) + (a.y - s.y) * (a.y - s.y) + (a.z - s.z) * (a.z - s.z);
}

// Scan-line search around `ci` (featureAssociation.cpp:1062-1099 corner,
// :1173-1220 surf).  Sequential semantics: the running minimum with strict <
// keeps the first point in visiting order.
__device__ void scanline_wave(const float4* last, int lastN, int jend, int ci, float4 sel,
                              bool surf, float nn_sq, int* o2, int* o3) {
  const int lane = threadIdx.x & 63;
  const int cScan = (int)last[ci].w;
  float m2 = nn_sq, m3 = nn_sq;
  int i2 = -1, i3 = -1;
  // forward
  for (int j0 = ci + 1; j0 < jend; j0 += 64) {
    const int j = j0 + lane;
    const bool inr = j < jend;
    float4 p = make_float4(0, 0, 0, 0);
    int rj = 0;
    if (inr) { p = last[j]; rj = (int)p.w; }
    const bool brk = inr && (double)rj > cScan + 2.5;
    const unsigned long long bm = __ballot(brk);
    const int lim = bm ? (__ffsll((long long)bm) - 1) : 64;
    const bool v = inr && lane < lim;
    const float d = v ? line_d2(p, sel) : 0.f;
    float bd; int bo, bj;
    if (surf) {
      wave_argmin(v && rj <= cScan, d, lane, j, &bd, &bo, &bj);
      if (bj >= 0 && bd < m2) { m2 = bd; i2 = bj; }
      wave_argmin(v && rj > cScan, d, lane, j, &bd, &bo, &bj);
      if (bj >= 0 && bd < m3) { m3 = bd; i3 = bj; }
    } else {
      wave_argmin(v && rj > cScan, d, lane, j, &bd, &bo, &bj);
      if (bj >= 0 && bd < m2) { m2 = bd; i2 = bj; }
    }
    if (bm) break;
  }
  // backward
  for (int j0 = ci - 1; j0 >= 0; j0 -= 64) {
    const int j = j0 - lane;
    const bool inr = j >= 0;
    float4 p = make_float4(0, 0, 0, 0);
    int rj = 0;
    if (inr) { p = last[j]; rj = (int)p.w; }
    const bool brk = inr && (double)rj < cScan - 2.5;
    const unsigned long long bm = __ballot(brk);
    const int lim = bm ? (__ffsll((long long)bm) - 1) : 64;
    const bool v = inr && lane < lim;
    const float d = v ? line_d2(p, sel) : 0.f;
    float bd; int bo, bj;
    if (surf) {
      wave_argmin(v && rj >= cScan, d, lane, j, &bd, &bo, &bj);
      if (bj >= 0 && bd < m2) { m2 = bd; i2 = bj; }
      wave_argmin(v && rj < cScan, d, lane, j, &bd, &bo, &bj);
      if (bj >= 0 && bd < m3) { m3 = bd; i3 = bj; }
    } else {
      wave_argmin(v && rj < cScan, d, lane, j, &bd, &bo, &bj);
      if (bj >= 0 && bd < m2) { m2 = bd; i2 = bj; }
    }
    if (bm) break;
  }
  *o2 = i2;
  *o3 = i3;
}

// ---------------------------------------------------------------- reduction
// 9 doubles (AtA upper triangle 6 + AtB 3) summed over the block.
__device__ void block_sum9(double v[9], const OdomLds& L, double out[9]) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int k = 0; k < 9; ++k)
    for (int o = 32; o > 0; o >>= 1) v[k] += __shfl_xor(v[k], o, 64);
  if (lane == 0)
    for (int k = 0; k < 9; ++k) L.red[wave * 10 + k] = v[k];
  __syncthreads();
  for (int k = 0; k < 9; ++k) {
    double s = 0;
    for (int w = 0; w < kOdomWaves; ++w) s += L.red[w * 10 + k];
    out[k] = s;
  }
  __syncthreads();
}

struct ScanFeat {
  const float4* sharp; int nSharp;
  const float4* lsharp; int nLS;
  const float4* flat; int nFlat;
  const float4* lflat; int nLF;
};

// Shared tail of calculateTransformationSurf / Corner.  Thread 0 only.
__device__ bool solve_step(float (&AtA)[3][3], float (&AtB)[3], int iter, OdomState* st,
                           float (&X)[3]) {
  float Aq[3][3];
  for (int a = 0; a < 3; ++a) for (int b = 0; b < 3; ++b) Aq[a][b] = AtA[a][b];
  float bq[3] = {AtB[0], AtB[1], AtB[2]};
  cv_solve_qr<3, 3>(Aq, bq, X);
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
  return true;
}

__device__ __forceinline__ double r2d(double r) { return r * 180.0 / M_PI; }

// One LM loop (surf: 25 iterations of findCorrespondingSurfFeatures +
// calculateTransformationSurf; corner likewise).  updateTransformation :1666-1695.
__device__ void lm_loop(bool surf, const ScanFeat& F, const float4* last, int lastN,
                        const NNIndex& nn, OdomState* st, const OdomLds& L, const DevCfg& c) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const float4* qp = surf ? F.flat : F.sharp;
  const int nQ = surf ? F.nFlat : F.nSharp;
  const int jend = min(nQ, lastN);  // the reference bounds by the query count (:1062, :1173)
  for (int it = 0; it < 25; it++) {
    // A: TransformToStart
    for (int q = tid; q < nQ; q += blockDim.x) L.sel[q] = to_start(qp[q], st->transformCur);
    __syncthreads();
    // B: correspondences
    if (it % 5 == 0) {
      for (int q = wave; q < nQ; q += kOdomWaves) {
        const float4 sel = L.sel[q];
        int ci = nn_query_wave(nn, sel, c.nn_sq, L.stack + wave * 64);
        if (ci >= lastN) ci = -1;  // stale tree over a smaller cloud
        int i2 = -1, i3 = -1;
        if (ci >= 0) scanline_wave(last, lastN, jend, ci, sel, surf, c.nn_sq, &i2, &i3);
        if (lane == 0) { L.i1[q] = ci; L.i2[q] = i2; L.i3[q] = i3; }
      }
      __syncthreads();
    }
    // C + D: rows and normal equations
    const float* tc = st->transformCur;
    const Trig3 T = trig3(tc[0], tc[1], tc[2]);
    const float srx = T.srx, crx = T.crx, sry = T.sry, cry = T.cry, srz = T.srz, crz = T.crz;
    const float tx = tc[3], ty = tc[4], tz = tc[5];
    double acc[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    int mloc = 0;
    for (int q = tid; q < nQ; q += blockDim.x) {
      const float4 sel = L.sel[q];
      float4 cf;
      bool ok = false;
      if (surf) {
        if (L.i2[q] >= 0 && L.i3[q] >= 0) {
          const float4 t1 = last[L.i1[q]], t2 = last[L.i2[q]], t3 = last[L.i3[q]];
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
        if (L.i2[q] >= 0) {
          const float4 t1 = last[L.i1[q]], t2 = last[L.i2[q]];
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
        const float4 po = qp[q];
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
    // row count
    int mw = mloc;
    for (int o = 32; o > 0; o >>= 1) mw += __shfl_xor(mw, o, 64);
    if (lane == 0) L.stack[wave * 64] = mw;
    double tot[9];
    block_sum9(acc, L, tot);
    if (tid == 0) {
      int M = 0;
      for (int w = 0; w < kOdomWaves; ++w) M += L.stack[w * 64];
      L.n[N_M] = M;
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
    const int brk = L.n[N_BREAK];
    __syncthreads();
    if (brk) break;
  }
}

__global__ void __launch_bounds__(kOdomThreads) k_odom(BatchBufs bb, OdomBufs ob, DevCfg c, int B,
                                                      unsigned long long* gkeys) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
  const OdomLds L = odom_carve(lds_raw);
  const int tid = threadIdx.x;
  OdomState* st = ob.st;
  NNIndex nnC{ob.nnCorner, ob.nnCornerIdx, ob.nnCornerBox, st->nnCornerNum, 0};
  NNIndex nnS{ob.nnSurf, ob.nnSurfIdx, ob.nnSurfBox, st->nnSurfNum, 0};
  // L2 of the stored trees follows from n
  {
    int l2 = 1; while (l2 < (nnC.n + kLeaf - 1) / kLeaf) l2 <<= 1; nnC.L2 = l2;
    l2 = 1; while (l2 < (nnS.n + kLeaf - 1) / kLeaf) l2 <<= 1; nnS.L2 = l2;
  }
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
    if (!st->inited) {
      // checkSystemInitialization :1605-1637 (no TransformToEnd)
      for (int t = tid; t < F.nLS; t += blockDim.x) { ob.cornerLast[t] = F.lsharp[t]; cEnd[t] = F.lsharp[t]; }
      for (int t = tid; t < F.nLF; t += blockDim.x) { ob.surfLast[t] = F.lflat[t]; sEnd[t] = F.lflat[t]; }
      __syncthreads();
      nn_build(ob.cornerLast, F.nLS, nnC, L, gkeys);
      nn_build(ob.surfLast, F.nLF, nnS, L, gkeys);
      if (tid == 0) {
        st->cornerLastNum = F.nLS;
        st->surfLastNum = F.nLF;
        st->nnCornerNum = F.nLS;
        st->nnSurfNum = F.nLF;
        st->transformSum[0] += 0.0f;  // += imuPitchStart
        st->transformSum[2] += 0.0f;  // += imuRollStart
        st->inited = 1;
        ob.validOut[b] = 0;
        ob.pubOut[b] = 0;
        for (int i = 0; i < 6; ++i) { ob.sumOut[b * 6 + i] = st->transformSum[i]; ob.curOut[b * 6 + i] = st->transformCur[i]; }
        __threadfence_block();
      }
      __syncthreads();
      continue;
    }
    // updateInitialGuess: a no-op without IMU
    if (st->cornerLastNum >= 10 && st->surfLastNum >= 100) {
      lm_loop(true, F, ob.surfLast, st->surfLastNum, nnS, st, L, c);
      lm_loop(false, F, ob.cornerLast, st->cornerLastNum, nnC, st, L, c);
    }
    // integrateTransformation :1697-1725
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
      ob.validOut[b] = 1;
      for (int i = 0; i < 6; ++i) { ob.sumOut[b * 6 + i] = ts[i]; ob.curOut[b * 6 + i] = tc[i]; }
      __threadfence_block();
    }
    __syncthreads();
    // publishCloudsLast :1759-1815
    for (int t = tid; t < F.nLS; t += blockDim.x) {
      const float4 p = to_end(F.lsharp[t], st->transformCur, im);
      ob.cornerLast[t] = p;
      cEnd[t] = p;
    }
    for (int t = tid; t < F.nLF; t += blockDim.x) {
      const float4 p = to_end(F.lflat[t], st->transformCur, im);
      ob.surfLast[t] = p;
      sEnd[t] = p;
    }
    __syncthreads();
    const bool rebuild = F.nLS > 10 && F.nLF > 100;
    if (rebuild) {
      nn_build(ob.cornerLast, F.nLS, nnC, L, gkeys);
      nn_build(ob.surfLast, F.nLF, nnS, L, gkeys);
    }
    if (tid == 0) {
      st->cornerLastNum = F.nLS;
      st->surfLastNum = F.nLF;
      if (rebuild) { st->nnCornerNum = F.nLS; st->nnSurfNum = F.nLF; }
      st->frameCount++;
      int pub = 0;
      if (st->frameCount >= c.skip + 1) { st->frameCount = 0; pub = 1; }
      ob.pubOut[b] = pub;
      __threadfence_block();
    }
    __syncthreads();
  }
}

size_t odom_nn_box_count(int npts) {
  int l2 = 1;
  while (l2 < (npts + kLeaf - 1) / kLeaf) l2 <<= 1;
  return (size_t)4 * l2;  // 2 float4 per node, 2*L2 nodes
}

void launch_odom(const BatchBufs& bb, const OdomBufs& ob, const DevCfg& c, int B, hipStream_t s,
                 StageTimer* tm, unsigned long long* gkeys) {
  tm->mark("odom.lm", s);
  k_odom<<<1, kOdomThreads, odom_lds_bytes(), s>>>(bb, ob, c, B, gkeys);
}

}  // namespace lego
