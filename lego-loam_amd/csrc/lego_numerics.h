// lego_numerics.h — bit-exact float libm + small dense solvers shared by the
// HIP kernels (gfx950) and the host code (g++).  Everything here restates
// THIRD-PARTY arithmetic that the reference calls on its hot path, so that the
// device produces the same bits as the reference does on its CPU host:
//
//   * glibc 2.35 atan2f / atanf  (fdlibm e_atan2f.c / s_atanf.c, glibc table)
//     — used by imageProjection.cpp:201,235,284,421 and featureAssociation.cpp:504
//   * glibc 2.35 sinf / cosf     (sysdeps/ieee754/flt-32/s_sinf.c, s_cosf.c,
//     sincosf.h, sincosf_data.c — the double-evaluated polynomial form)
//     — used by featureAssociation.cpp:871-881,1281-1286,1390-1395 etc.
//   * glibc 2.35 asinf           (sysdeps/ieee754/flt-32/e_asinf.c)
//     — used by featureAssociation.cpp:1019,984 and mapOptmization.cpp:418
//
// The pinning tests (tests/test_numerics_shim.py) compare these against the
// container's glibc bit for bit.  Compile every TU that includes this header
// with -ffp-contract=off: contraction into FMA changes discrete decisions.
#pragma once
#include <stdint.h>
#include <string.h>

#if defined(__HIPCC__)
#define LEGO_HD __host__ __device__ inline
#else
#define LEGO_HD inline
#endif

namespace lego {

LEGO_HD uint32_t f2u(float f) { return __builtin_bit_cast(uint32_t, f); }
LEGO_HD float u2f(uint32_t u) { return __builtin_bit_cast(float, u); }
LEGO_HD uint64_t d2u(double d) { return __builtin_bit_cast(uint64_t, d); }

LEGO_HD float lfabsf(float x) { return u2f(f2u(x) & 0x7fffffffu); }
LEGO_HD float lsqrtf(float x) { return __builtin_sqrtf(x); }

// ---------------------------------------------------------------- atanf
LEGO_HD float lego_atanf(float x) {
  const float atanhi0 = u2f(0x3eed6338u), atanhi1 = u2f(0x3f490fdau),
              atanhi2 = u2f(0x3f7b985eu), atanhi3 = u2f(0x3fc90fdau);
  const float atanlo0 = u2f(0x31ac3769u), atanlo1 = u2f(0x33222168u),
              atanlo2 = u2f(0x33140fb4u), atanlo3 = u2f(0x33a22168u);
  const float aT0 = u2f(0x3eaaaaabu), aT1 = u2f(0xbe4ccccdu), aT2 = u2f(0x3e124925u),
              aT3 = u2f(0xbde38e38u), aT4 = u2f(0x3dba2e6eu), aT5 = u2f(0xbd9d8795u),
              aT6 = u2f(0x3d886b35u), aT7 = u2f(0xbd6ef16bu), aT8 = u2f(0x3d4bda59u),
              aT9 = u2f(0xbd15a221u), aT10 = u2f(0x3c8569d7u);
  const float one = 1.0f;
  int32_t hx = (int32_t)f2u(x);
  int32_t ix = hx & 0x7fffffff;
  int id;
  if (ix >= 0x4c000000) {             // |x| >= 2^25
    if (ix > 0x7f800000) return x + x; // NaN
    if (hx > 0) return atanhi3 + atanlo3;
    return -atanhi3 - atanlo3;
  }
  if (ix < 0x3ee00000) {              // |x| < 0.4375
    if (ix < 0x31000000) return x;    // |x| < 2^-29
    id = -1;
  } else {
    x = lfabsf(x);
    if (ix < 0x3f980000) {            // |x| < 1.1875
      if (ix < 0x3f300000) { id = 0; x = (2.0f * x - one) / (2.0f + x); }
      else                 { id = 1; x = (x - one) / (x + one); }
    } else {
      if (ix < 0x401c0000) { id = 2; x = (x - 1.5f) / (one + 1.5f * x); }
      else                 { id = 3; x = -1.0f / x; }
    }
  }
  float z = x * x;
  float w = z * z;
  float s1 = z * (aT0 + w * (aT2 + w * (aT4 + w * (aT6 + w * (aT8 + w * aT10)))));
  float s2 = w * (aT1 + w * (aT3 + w * (aT5 + w * (aT7 + w * aT9))));
  if (id < 0) return x - x * (s1 + s2);
  float hi = id == 0 ? atanhi0 : id == 1 ? atanhi1 : id == 2 ? atanhi2 : atanhi3;
  float lo = id == 0 ? atanlo0 : id == 1 ? atanlo1 : id == 2 ? atanlo2 : atanlo3;
  z = hi - ((x * (s1 + s2) - lo) - x);
  return (hx < 0) ? -z : z;
}

// ---------------------------------------------------------------- atan2f
LEGO_HD float lego_atan2f(float y, float x) {
  const float tiny = 1.0e-30f;
  const float pi_o_4 = u2f(0x3f490fdbu), pi_o_2 = u2f(0x3fc90fdbu),
              pi = u2f(0x40490fdbu), pi_lo = u2f(0xb3bbbd2eu);
  int32_t hx = (int32_t)f2u(x), ix = hx & 0x7fffffff;
  int32_t hy = (int32_t)f2u(y), iy = hy & 0x7fffffff;
  if (ix > 0x7f800000 || iy > 0x7f800000) return x + y;
  if (hx == 0x3f800000) return lego_atanf(y);
  int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);
  if (iy == 0) {
    switch (m) {
      case 0: case 1: return y;
      case 2: return pi + tiny;
      default: return -pi - tiny;
    }
  }
  if (ix == 0) return (hy < 0) ? -pi_o_2 - tiny : pi_o_2 + tiny;
  if (ix == 0x7f800000) {
    if (iy == 0x7f800000) {
      switch (m) {
        case 0: return pi_o_4 + tiny;
        case 1: return -pi_o_4 - tiny;
        case 2: return 3.0f * pi_o_4 + tiny;
        default: return -3.0f * pi_o_4 - tiny;
      }
    } else {
      switch (m) {
        case 0: return 0.0f;
        case 1: return -0.0f;
        case 2: return pi + tiny;
        default: return -pi - tiny;
      }
    }
  }
  if (iy == 0x7f800000) return (hy < 0) ? -pi_o_2 - tiny : pi_o_2 + tiny;
  int32_t k = (iy - ix) >> 23;
  float z;
  if (k > 60) z = pi_o_2 + 0.5f * pi_lo;
  else if (hx < 0 && k < -60) z = 0.0f;
  else z = lego_atanf(lfabsf(y / x));
  switch (m) {
    case 0: return z;
    case 1: return u2f(f2u(z) ^ 0x80000000u);
    case 2: return pi - (z - pi_lo);
    default: return (z - pi_lo) - pi;
  }
}

// ---------------------------------------------------------------- sinf/cosf
// glibc's sincosf tables (sincosf_data.c), non-TOINT_INTRINSICS variant.
// Entry 1 is entry 0 with the cosine polynomial negated; sign[] = {1,-1,-1,1}.
struct SinCosTab {
  double hpi_inv, hpi, c0, c1, c2, c3, c4, s1, s2, s3;
};

LEGO_HD SinCosTab sincos_tab(int which) {
  const double neg = which ? -1.0 : 1.0;
  SinCosTab t;
  t.hpi_inv = 0x1.45F306DC9C883p+23;
  t.hpi = 0x1.921FB54442D18p0;
  t.c0 = neg * 0x1p0;
  t.c1 = neg * -0x1.ffffffd0c621cp-2;
  t.c2 = neg * 0x1.55553e1068f19p-5;
  t.c3 = neg * -0x1.6c087e89a359dp-10;
  t.c4 = neg * 0x1.99343027bf8c3p-16;
  t.s1 = -0x1.555545995a603p-3;
  t.s2 = 0x1.1107605230bc4p-7;
  t.s3 = -0x1.994eb3774cf24p-13;
  return t;
}

LEGO_HD double sincos_sign(int q) { return (q == 1 || q == 2) ? -1.0 : 1.0; }

LEGO_HD uint32_t abstop12(float x) { return (f2u(x) >> 20) & 0x7ff; }

// glibc x86_64 dispatches sinf/cosf to the FMA build (s_sinf-fma.c) on any
// FMA-capable host: the same source with every a + b*c contracted.  We write
// those contractions explicitly so host (-ffp-contract=off) and device agree.
LEGO_HD double fmad(double a, double b, double c) { return __builtin_fma(a, b, c); }

LEGO_HD float sinf_poly(double x, double x2, const SinCosTab p, int n) {
  if ((n & 1) == 0) {
    double x3 = x * x2;
    double s1 = fmad(x2, p.s3, p.s2);
    double x7 = x3 * x2;
    double s = fmad(x3, p.s1, x);
    return (float)fmad(x7, s1, s);
  } else {
    double x4 = x2 * x2;
    double c2 = fmad(x2, p.c4, p.c3);
    double c1 = fmad(x2, p.c1, p.c0);
    double x6 = x4 * x2;
    double c = fmad(x4, p.c2, c1);
    return (float)fmad(x6, c2, c);
  }
}

LEGO_HD double reduce_fast(double x, const SinCosTab p, int* np) {
  double r = x * p.hpi_inv;
  int n = ((int32_t)r + 0x800000) >> 24;
  *np = n;
  return fmad(-(double)n, p.hpi, x);
}

LEGO_HD double reduce_large(uint32_t xi, int* np) {
  const uint32_t inv_pio4[24] = {
      0xa2,       0xa2f9,     0xa2f983,   0xa2f9836e, 0xf9836e4e, 0x836e4e44,
      0x6e4e4415, 0x4e441529, 0x441529fc, 0x1529fc27, 0x29fc2757, 0xfc2757d1,
      0x2757d1f5, 0x57d1f534, 0xd1f534dd, 0xf534ddc0, 0x34ddc0db, 0xddc0db62,
      0xc0db6295, 0xdb629599, 0x6295993c, 0x95993c43, 0x993c4390, 0x3c439041};
  const uint32_t* arr = &inv_pio4[(xi >> 26) & 15];
  int shift = (xi >> 23) & 7;
  uint64_t n, res0, res1, res2;
  xi = (xi & 0xffffff) | 0x800000;
  xi <<= shift;
  res0 = xi * arr[0];
  res1 = (uint64_t)xi * arr[4];
  res2 = (uint64_t)xi * arr[8];
  res0 = (res2 >> 32) | (res0 << 32);
  res0 += res1;
  n = (res0 + (1ULL << 61)) >> 62;
  res0 -= n << 62;
  double x = (double)(int64_t)res0;
  *np = (int)n;
  return x * 0x1.921FB54442D18p-62;
}

// |y| >= 120 and non-finite y (sin, cos): out of line.  The Payne-Hanek
// reduction's table and 64-bit products are code every inlined sinf / cosf
// would carry through the kernels' hot loops, where the angles are small.
struct SinCos {
  float s, c;
};
LEGO_HD __attribute__((noinline)) SinCos lego_sincosf_huge(float y) {
  SinCos r;
  if (abstop12(y) < abstop12(__builtin_inff())) {
    uint32_t xi = f2u(y);
    int sign = xi >> 31, n;
    const double x = reduce_large(xi, &n);
    double s = sincos_sign((n + sign) & 3);
    const SinCosTab p = sincos_tab(((n + sign) & 2) ? 1 : 0);
    r.s = sinf_poly(x * s, x * x, p, n);
    r.c = sinf_poly(x * s, x * x, p, n ^ 1);
  } else {
    r.s = r.c = (y - y) / (y - y);
  }
  return r;
}

LEGO_HD float lego_sinf(float y) {
  double x = y;
  int n;
  const float pio4 = 0x1.921FB6p-1f;
  if (abstop12(y) < abstop12(pio4)) {
    double s = x * x;
    if (abstop12(y) < abstop12(0x1p-12f)) return y;
    return sinf_poly(x, s, sincos_tab(0), 0);
  } else if (abstop12(y) < abstop12(120.0f)) {
    x = reduce_fast(x, sincos_tab(0), &n);
    double s = sincos_sign(n & 3);
    const SinCosTab p = sincos_tab((n & 2) ? 1 : 0);
    return sinf_poly(x * s, x * x, p, n);
  }
  return lego_sincosf_huge(y).s;
}

LEGO_HD float lego_cosf(float y) {
  double x = y;
  int n;
  const float pio4 = 0x1.921FB6p-1f;
  if (abstop12(y) < abstop12(pio4)) {
    double x2 = x * x;
    if (abstop12(y) < abstop12(0x1p-12f)) return 1.0f;
    return sinf_poly(x, x2, sincos_tab(0), 1);
  } else if (abstop12(y) < abstop12(120.0f)) {
    x = reduce_fast(x, sincos_tab(0), &n);
    double s = sincos_sign(n & 3);
    const SinCosTab p = sincos_tab((n & 2) ? 1 : 0);
    return sinf_poly(x * s, x * x, p, n ^ 1);
  }
  return lego_sincosf_huge(y).c;
}

// sinf and cosf of one argument (glibc's sincosf structure): the range
// reduction, sign and table are shared and each result is the very
// expression lego_sinf / lego_cosf evaluate, so both are bit-identical to them.
LEGO_HD void lego_sincosf(float y, float* sp, float* cp) {
  double x = y;
  int n;
  const float pio4 = 0x1.921FB6p-1f;
  if (abstop12(y) < abstop12(pio4)) {
    const double x2 = x * x;
    if (abstop12(y) < abstop12(0x1p-12f)) {
      *sp = y;
      *cp = 1.0f;
      return;
    }
    *sp = sinf_poly(x, x2, sincos_tab(0), 0);
    *cp = sinf_poly(x, x2, sincos_tab(0), 1);
  } else if (abstop12(y) < abstop12(120.0f)) {
    x = reduce_fast(x, sincos_tab(0), &n);
    const double s = sincos_sign(n & 3);
    const SinCosTab p = sincos_tab((n & 2) ? 1 : 0);
    *sp = sinf_poly(x * s, x * x, p, n);
    *cp = sinf_poly(x * s, x * x, p, n ^ 1);
  } else {
    const SinCos r = lego_sincosf_huge(y);
    *sp = r.s;
    *cp = r.c;
  }
}

// ---------------------------------------------------------------- asinf
LEGO_HD float lego_asinf(float x) {
  const float one = 1.0f;
  const float pio2_hi = 1.57079637050628662109375f;
  const float pio2_lo = -4.37113900018624283e-8f;
  const float pio4_hi = 0.785398185253143310546875f;
  const float p0 = 1.666675248e-1f, p1 = 7.495297643e-2f, p2 = 4.547037598e-2f,
              p3 = 2.417951451e-2f, p4 = 4.216630880e-2f;
  float t, w, p, q, c, r, s;
  int32_t hx = (int32_t)f2u(x);
  int32_t ix = hx & 0x7fffffff;
  if (ix == 0x3f800000) return x * pio2_hi + x * pio2_lo;
  if (ix > 0x3f800000) return (x - x) / (x - x);
  if (ix < 0x3f000000) {
    if (ix < 0x32000000) return x;
    t = x * x;
    w = t * (p0 + t * (p1 + t * (p2 + t * (p3 + t * p4))));
    return x + x * w;
  }
  w = one - lfabsf(x);
  t = w * 0.5f;
  p = t * (p0 + t * (p1 + t * (p2 + t * (p3 + t * p4))));
  s = lsqrtf(t);
  if (ix >= 0x3F79999A) {
    t = pio2_hi - (2.0f * (s + s * p) - pio2_lo);
  } else {
    w = u2f(f2u(s) & 0xfffff000u);
    c = (t - w * w) / (s + w);
    r = p;
    p = 2.0f * s * r - (pio2_lo - 2.0f * c);
    q = pio4_hi - 2.0f * w;
    t = pio4_hi - (p - q);
  }
  return (hx > 0) ? t : -t;
}


// ===================================================================== solvers
// The reference solves its normal equations with OpenCV 3.x (ROS kinetic /
// melodic): cv::solve(..., DECOMP_QR) -> hal::QR32f (Householder QRImpl),
// cv::eigen -> hal::Jacobi (JacobiImpl_), Mat::inv() -> cv::invert(DECOMP_LU)
// (closed form for n <= 3, hal::LU32f otherwise).  OpenCV is not in this image,
// so these are restatements of those published algorithms (parity with
// OpenCV's float internals is unpinned); the oracle and the
// kernels share them, so the GPU reproduces the oracle bit for bit.
// Call sites: featureAssociation.cpp:1327,1334,1349 / 1428,1435,1450;
// mapOptmization.cpp:1126,1189,1276,1283,1298.

LEGO_HD float lfabs(float x) { return lfabsf(x); }

// cv::hypot (lapack.cpp) — used by the Jacobi rotation.
LEGO_HD float cv_hypot(float a, float b) {
  a = lfabsf(a);
  b = lfabsf(b);
  if (a > b) {
    b /= a;
    return a * lsqrtf(1 + b * b);
  }
  if (b > 0) {
    a /= b;
    return b * lsqrtf(1 + a * a);
  }
  return 0;
}

// cv::eigen for a symmetric float matrix: eigenvalues W in descending order,
// eigenvectors as the ROWS of V.  A is destroyed.
// The pivot bookkeeping indR/indC is caller-provided so device code can keep
// it (and A, W, V) in LDS: the Jacobi sweep indexes them dynamically, which in
// registers would become scratch memory.
template <int N>
LEGO_HD void cv_eigen_sym_ws(float (&A)[N][N], float (&W)[N], float (&V)[N][N], int (&indR)[N],
                             int (&indC)[N]) {
  const float eps = 1.1920928955078125e-07f;  // FLT_EPSILON
  int i, j, k, m;
  for (i = 0; i < N; i++) {
    for (j = 0; j < N; j++) V[i][j] = 0.f;
    V[i][i] = 1.f;
  }
  float mv = 0.f;
  for (k = 0; k < N; k++) {
    W[k] = A[k][k];
    if (k < N - 1) {
      for (m = k + 1, mv = lfabsf(A[k][m]), i = k + 2; i < N; i++) {
        float val = lfabsf(A[k][i]);
        if (mv < val) mv = val, m = i;
      }
      indR[k] = m;
    }
    if (k > 0) {
      for (m = 0, mv = lfabsf(A[0][k]), i = 1; i < k; i++) {
        float val = lfabsf(A[i][k]);
        if (mv < val) mv = val, m = i;
      }
      indC[k] = m;
    }
  }
  if (N > 1) {
    const int maxIters = N * N * 30;
    for (int iters = 0; iters < maxIters; iters++) {
      for (k = 0, mv = lfabsf(A[0][indR[0]]), i = 1; i < N - 1; i++) {
        float val = lfabsf(A[i][indR[i]]);
        if (mv < val) mv = val, k = i;
      }
      int l = indR[k];
      for (i = 1; i < N; i++) {
        float val = lfabsf(A[indC[i]][i]);
        if (mv < val) mv = val, k = indC[i], l = i;
      }
      float p = A[k][l];
      if (lfabsf(p) <= eps) break;
      float y = (float)((double)(W[l] - W[k]) * 0.5);
      float t = lfabsf(y) + cv_hypot(p, y);
      float s = cv_hypot(p, t);
      float c = t / s;
      s = p / s;
      t = (p / t) * p;
      if (y < 0) s = -s, t = -t;
      A[k][l] = 0;
      W[k] -= t;
      W[l] += t;
      float a0, b0;
#define LEGO_ROT(v0, v1) a0 = v0, b0 = v1, v0 = a0 * c - b0 * s, v1 = a0 * s + b0 * c
      for (i = 0; i < k; i++) LEGO_ROT(A[i][k], A[i][l]);
      for (i = k + 1; i < l; i++) LEGO_ROT(A[k][i], A[i][l]);
      for (i = l + 1; i < N; i++) LEGO_ROT(A[k][i], A[l][i]);
      for (i = 0; i < N; i++) LEGO_ROT(V[k][i], V[l][i]);
#undef LEGO_ROT
      for (j = 0; j < 2; j++) {
        int idx = j == 0 ? k : l;
        if (idx < N - 1) {
          for (m = idx + 1, mv = lfabsf(A[idx][m]), i = idx + 2; i < N; i++) {
            float val = lfabsf(A[idx][i]);
            if (mv < val) mv = val, m = i;
          }
          indR[idx] = m;
        }
        if (idx > 0) {
          for (m = 0, mv = lfabsf(A[0][idx]), i = 1; i < idx; i++) {
            float val = lfabsf(A[i][idx]);
            if (mv < val) mv = val, m = i;
          }
          indC[idx] = m;
        }
      }
    }
  }
  for (k = 0; k < N - 1; k++) {
    m = k;
    for (i = k + 1; i < N; i++)
      if (W[m] < W[i]) m = i;
    if (k != m) {
      float tw = W[m]; W[m] = W[k]; W[k] = tw;
      for (i = 0; i < N; i++) { float tv = V[m][i]; V[m][i] = V[k][i]; V[k][i] = tv; }
    }
  }
}

template <int N>
LEGO_HD void cv_eigen_sym(float (&A)[N][N], float (&W)[N], float (&V)[N][N]) {
  int indR[N], indC[N];
  cv_eigen_sym_ws<N>(A, W, V, indR, indC);
}

// cv_eigen_sym<3> with every index resolved at compile time, so device code
// keeps the whole Jacobi state in registers.  Same operations in the same
// order as the generic form above (tests/native/eigen3_check.cpp compares the
// two bit for bit): only the pivot bookkeeping is spelled out.  For N = 3 the
// pivots are (0,1), (0,2), (1,2); indR[1] = 2 and indC[1] = 0 are constant.
LEGO_HD void cv_eigen_sym3(const float (&Ain)[3][3], float (&W)[3], float (&V)[3][3]) {
  const float eps = 1.1920928955078125e-07f;
  float a01 = Ain[0][1], a02 = Ain[0][2], a12 = Ain[1][2];
  float w0 = Ain[0][0], w1 = Ain[1][1], w2 = Ain[2][2];
  float v00 = 1.f, v01 = 0.f, v02 = 0.f, v10 = 0.f, v11 = 1.f, v12 = 0.f, v20 = 0.f, v21 = 0.f, v22 = 1.f;
  int indR0 = (lfabsf(a01) < lfabsf(a02)) ? 2 : 1;
  int indC2 = (lfabsf(a02) < lfabsf(a12)) ? 1 : 0;
  for (int iters = 0; iters < 3 * 3 * 30; iters++) {
    int k = 0, l;
    float mv = indR0 == 1 ? lfabsf(a01) : lfabsf(a02);
    float val = lfabsf(a12);
    if (mv < val) mv = val, k = 1;
    l = k == 0 ? indR0 : 2;
    val = lfabsf(a01);
    if (mv < val) mv = val, k = 0, l = 1;
    val = indC2 == 0 ? lfabsf(a02) : lfabsf(a12);
    if (mv < val) mv = val, k = indC2, l = 2;
    const int pr = k == 0 ? (l == 1 ? 0 : 1) : 2;  // (0,1) (0,2) (1,2)
    float p = pr == 0 ? a01 : (pr == 1 ? a02 : a12);
    if (lfabsf(p) <= eps) break;
    const float wk = pr == 2 ? w1 : w0, wl = pr == 0 ? w1 : w2;
    float y = (float)((double)(wl - wk) * 0.5);
    float t = lfabsf(y) + cv_hypot(p, y);
    float s = cv_hypot(p, t);
    float c = t / s;
    s = p / s;
    t = (p / t) * p;
    if (y < 0) s = -s, t = -t;
    float a0, b0;
#define LEGO_ROT(v0_, v1_) a0 = v0_, b0 = v1_, v0_ = a0 * c - b0 * s, v1_ = a0 * s + b0 * c
    if (pr == 0) {
      a01 = 0; w0 -= t; w1 += t;
      LEGO_ROT(a02, a12);
      LEGO_ROT(v00, v10); LEGO_ROT(v01, v11); LEGO_ROT(v02, v12);
    } else if (pr == 1) {
      a02 = 0; w0 -= t; w2 += t;
      LEGO_ROT(a01, a12);
      LEGO_ROT(v00, v20); LEGO_ROT(v01, v21); LEGO_ROT(v02, v22);
    } else {
      a12 = 0; w1 -= t; w2 += t;
      LEGO_ROT(a01, a02);
      LEGO_ROT(v10, v20); LEGO_ROT(v11, v21); LEGO_ROT(v12, v22);
    }
#undef LEGO_ROT
    // indR / indC of rows and columns k and l (the only ones that change)
    if (k == 0 || l == 0) indR0 = (lfabsf(a01) < lfabsf(a02)) ? 2 : 1;
    if (k == 2 || l == 2) indC2 = (lfabsf(a02) < lfabsf(a12)) ? 1 : 0;
  }
  // selection sort, descending (strict <), rows of V follow
  float r0[3] = {v00, v01, v02}, r1[3] = {v10, v11, v12}, r2[3] = {v20, v21, v22};
  {
    int m = 0;
    if (w0 < w1) m = 1;
    if ((m == 0 ? w0 : w1) < w2) m = 2;
    if (m == 1) {
      float tw = w1; w1 = w0; w0 = tw;
      for (int i = 0; i < 3; i++) { float tv = r1[i]; r1[i] = r0[i]; r0[i] = tv; }
    } else if (m == 2) {
      float tw = w2; w2 = w0; w0 = tw;
      for (int i = 0; i < 3; i++) { float tv = r2[i]; r2[i] = r0[i]; r0[i] = tv; }
    }
  }
  if (w1 < w2) {
    float tw = w2; w2 = w1; w1 = tw;
    for (int i = 0; i < 3; i++) { float tv = r2[i]; r2[i] = r1[i]; r1[i] = tv; }
  }
  W[0] = w0; W[1] = w1; W[2] = w2;
  for (int i = 0; i < 3; i++) { V[0][i] = r0[i]; V[1][i] = r1[i]; V[2][i] = r2[i]; }
}

// cv::solve(A, b, x, DECOMP_QR) for a square float system with one rhs
// (hal::QR32f, eps = 10*FLT_EPSILON).  A and b are destroyed; x written.
// On failure OpenCV zeroes dst (lapack.cpp: `if (!result) dst = Scalar(0)`).
template <int M, int N>
LEGO_HD bool cv_solve_qr(float (&A)[M][N], const float (&bin)[M], float (&x)[N]) {
  const float eps = 1.1920928955078125e-07f * 10;
  float b[M];
  for (int i = 0; i < M; i++) b[i] = bin[i];
  float vl[M];
  float hF[N];
#pragma unroll
  for (int l = 0; l < N; l++) {
    int vlSize = M - l;
    float vlNorm = 0.f;
#pragma unroll
    for (int i = 0; i < vlSize; i++) {
      vl[i] = A[l + i][l];
      vlNorm += vl[i] * vl[i];
    }
    float tmpV = vl[0];
    vl[0] = vl[0] + (vl[0] >= 0 ? 1.f : -1.f) * lsqrtf(vlNorm);
    vlNorm = lsqrtf(vlNorm + vl[0] * vl[0] - tmpV * tmpV);
#pragma unroll
    for (int i = 0; i < vlSize; i++) vl[i] /= vlNorm;
#pragma unroll
    for (int j = l; j < N; j++) {
      float v_lA = 0.f;
#pragma unroll
      for (int i = l; i < M; i++) v_lA += vl[i - l] * A[i][j];
#pragma unroll
      for (int i = l; i < M; i++) A[i][j] -= 2 * vl[i - l] * v_lA;
    }
    hF[l] = vl[0] * vl[0];
#pragma unroll
    for (int i = 1; i < vlSize; i++) A[l + i][l] = vl[i] / vl[0];
  }
#pragma unroll
  for (int l = 0; l < N; l++) {
    vl[0] = 1.f;
#pragma unroll
    for (int j = 1; j < M - l; j++) vl[j] = A[j + l][l];
    float v_lB = 0.f;
#pragma unroll
    for (int i = l; i < M; i++) v_lB += vl[i - l] * b[i];
#pragma unroll
    for (int i = l; i < M; i++) b[i] -= 2 * vl[i - l] * v_lB * hF[l];
  }
#pragma unroll
  for (int i = N - 1; i >= 0; i--) {
#pragma unroll
    for (int j = N - 1; j > i; j--) b[i] -= b[j] * A[i][j];
    if (lfabsf(A[i][i]) < eps) {
      for (int q = 0; q < N; q++) x[q] = 0.f;
      return false;
    }
    b[i] /= A[i][i];
  }
  for (int q = 0; q < N; q++) x[q] = b[q];
  return true;
}

// Mat::inv() for 3x3 float (cv::invert closed form, determinant in float via
// det3, cofactors in double).  Zeroes the output if det == 0.
LEGO_HD bool cv_inv3(const float (&S)[3][3], float (&D)[3][3]) {
  float df = S[0][0] * (S[1][1] * S[2][2] - S[1][2] * S[2][1]) -
             S[0][1] * (S[1][0] * S[2][2] - S[1][2] * S[2][0]) +
             S[0][2] * (S[1][0] * S[2][1] - S[1][1] * S[2][0]);
  double d = df;
  if (d == 0.) {
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++) D[i][j] = 0.f;
    return false;
  }
  d = 1. / d;
  double t[9];
  t[0] = (((double)S[1][1] * S[2][2] - (double)S[1][2] * S[2][1]) * d);
  t[1] = (((double)S[0][2] * S[2][1] - (double)S[0][1] * S[2][2]) * d);
  t[2] = (((double)S[0][1] * S[1][2] - (double)S[0][2] * S[1][1]) * d);
  t[3] = (((double)S[1][2] * S[2][0] - (double)S[1][0] * S[2][2]) * d);
  t[4] = (((double)S[0][0] * S[2][2] - (double)S[0][2] * S[2][0]) * d);
  t[5] = (((double)S[0][2] * S[1][0] - (double)S[0][0] * S[1][2]) * d);
  t[6] = (((double)S[1][0] * S[2][1] - (double)S[1][1] * S[2][0]) * d);
  t[7] = (((double)S[0][1] * S[2][0] - (double)S[0][0] * S[2][1]) * d);
  t[8] = (((double)S[0][0] * S[1][1] - (double)S[0][1] * S[1][0]) * d);
  for (int i = 0; i < 9; i++) D[i / 3][i % 3] = (float)t[i];
  return true;
}

// Mat::inv() for n > 3: hal::LU32f with the identity as right-hand side.
template <int N>
LEGO_HD bool cv_inv_lu(const float (&S)[N][N], float (&D)[N][N]) {
  const float eps = 1.1920928955078125e-07f * 10;
  float A[N][N];
  for (int i = 0; i < N; i++)
    for (int j = 0; j < N; j++) { A[i][j] = S[i][j]; D[i][j] = (i == j) ? 1.f : 0.f; }
  for (int i = 0; i < N; i++) {
    int k = i;
    for (int j = i + 1; j < N; j++)
      if (lfabsf(A[j][i]) > lfabsf(A[k][i])) k = j;
    if (lfabsf(A[k][i]) < eps) {
      for (int a = 0; a < N; a++)
        for (int b = 0; b < N; b++) D[a][b] = 0.f;
      return false;
    }
    if (k != i) {
      for (int j = i; j < N; j++) { float t = A[i][j]; A[i][j] = A[k][j]; A[k][j] = t; }
      for (int j = 0; j < N; j++) { float t = D[i][j]; D[i][j] = D[k][j]; D[k][j] = t; }
    }
    float d = -1 / A[i][i];
    for (int j = i + 1; j < N; j++) {
      float alpha = A[j][i] * d;
      for (int q = i + 1; q < N; q++) A[j][q] += alpha * A[i][q];
      for (int q = 0; q < N; q++) D[j][q] += alpha * D[i][q];
    }
    A[i][i] = -d;
  }
  for (int i = N - 1; i >= 0; i--)
    for (int j = 0; j < N; j++) {
      float s = D[i][j];
      for (int q = i + 1; q < N; q++) s -= A[i][q] * D[q][j];
      D[i][j] = s * A[i][i];
    }
  return true;
}

// True when every eigenvalue of the symmetric AtA provably exceeds thr by a
// margin that dwarfs the float Jacobi's error (1e-4 of ||AtA||_F, ~10^3 ulp):
// then cv::eigen's smallest eigenvalue is >= thr as well, the degeneracy test
// of :1336-1347 / :1437-1448 finds nothing, and the 3x3 Jacobi can be skipped.
// LDL^T of AtA - t I in double: positive definite iff all pivots are > 0
// (NaN fails every comparison and takes the Jacobi path).
LEGO_HD bool eig_min_above(const float (&A)[3][3], double thr) {
  const double a00 = A[0][0], a01 = A[0][1], a02 = A[0][2], a11 = A[1][1], a12 = A[1][2], a22 = A[2][2];
  const double fro = __builtin_sqrt(a00 * a00 + a11 * a11 + a22 * a22 + 2 * (a01 * a01 + a02 * a02 + a12 * a12));
  const double t = thr + 1e-4 * fro;
  const double d0 = a00 - t;
  if (!(d0 > 0)) return false;
  const double l10 = a01 / d0, l20 = a02 / d0;
  const double d1 = (a11 - t) - l10 * a01;
  if (!(d1 > 0)) return false;
  const double l21 = (a12 - l20 * a01) / d1;
  const double d2 = (a22 - t) - l20 * a02 - l21 * l21 * d1;
  return d2 > 0;
}

// The same proof for an N x N system (mapOptimization's 6 x 6 AtA, threshold
// 100, mapOptmization.cpp:1281-1296): A - t I positive definite by an LDL^T in
// double, t = thr + 1e-4 * ||A||_F, so every eigenvalue, and the Jacobi
// restatement's computed ones, exceed thr.  Checked against cv_eigen_sym<6>
// by tests/native/eigmin_check.cpp.
template <int N>
LEGO_HD bool eig_min_above_n(const float (&A)[N][N], double thr) {
  double fro2 = 0;
#pragma unroll
  for (int i = 0; i < N; i++)
#pragma unroll
    for (int j = 0; j < N; j++) fro2 += (double)A[i][j] * (double)A[i][j];
  const double t = thr + 1e-4 * __builtin_sqrt(fro2);
  double Lm[N][N], D[N];
#pragma unroll
  for (int j = 0; j < N; j++) {
    double d = (double)A[j][j] - t;
#pragma unroll
    for (int k = 0; k < j; k++) d -= Lm[j][k] * Lm[j][k] * D[k];
    if (!(d > 0)) return false;
    D[j] = d;
#pragma unroll
    for (int i = j + 1; i < N; i++) {
      double v = (double)A[i][j];
#pragma unroll
      for (int k = 0; k < j; k++) v -= Lm[i][k] * Lm[j][k] * D[k];
      Lm[i][j] = v / d;
    }
  }
  return true;
}

// matP = matV.inv() * matV2 (cv gemm: double accumulation, float store).
template <int N>
LEGO_HD void cv_matmul(const float (&A)[N][N], const float (&B)[N][N], float (&C)[N][N]) {
  for (int i = 0; i < N; i++)
    for (int j = 0; j < N; j++) {
      double s = 0;
      for (int q = 0; q < N; q++) s += (double)A[i][q] * (double)B[q][j];
      C[i][j] = (float)s;
    }
}
template <int N>
LEGO_HD void cv_matvec(const float (&A)[N][N], const float (&x)[N], float (&y)[N]) {
  for (int i = 0; i < N; i++) {
    double s = 0;
    for (int q = 0; q < N; q++) s += (double)A[i][q] * (double)x[q];
    y[i] = (float)s;
  }
}

}  // namespace lego
