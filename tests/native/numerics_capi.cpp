// C entry points over the solver restatements of lego_numerics.h (shared by
// the oracle and the gfx950 kernels), so tests/test_numerics_witness.py can
// compare them with the independently written numpy witness
// (tests/witness_numerics.py).  Test infrastructure; built by the test with
// g++ -ffp-contract=off.
#include <cstring>

#include "lego_numerics.h"

extern "C" {

// cv::solve(A, b, x, DECOMP_QR) for (m, n) in {(3,3), (5,3), (6,6)}; A row-major m x n.
int lw_solve_qr(int m, int n, const float* A, const float* b, float* x) {
#define CASE(M, N)                                                   \
  if (m == M && n == N) {                                            \
    float a[M][N], bb[M], xx[N];                                     \
    std::memcpy(a, A, sizeof(a));                                    \
    std::memcpy(bb, b, sizeof(bb));                                  \
    const bool ok = lego::cv_solve_qr<M, N>(a, bb, xx);             \
    std::memcpy(x, xx, sizeof(xx));                                  \
    return ok ? 1 : 0;                                               \
  }
  CASE(3, 3) CASE(5, 3) CASE(6, 6)
#undef CASE
  return -1;
}

// cv::eigen of a symmetric n x n (n = 3 or 6): W descending, eigenvectors as rows of V.
// form = 1: the register form cv_eigen_sym3 (n = 3 only).
int lw_eigen(int n, int form, const float* A, float* W, float* V) {
  if (n == 3 && form == 1) {
    float a[3][3], w[3], v[3][3];
    std::memcpy(a, A, sizeof(a));
    lego::cv_eigen_sym3(a, w, v);
    std::memcpy(W, w, sizeof(w));
    std::memcpy(V, v, sizeof(v));
    return 0;
  }
#define CASE(N)                                    \
  if (n == N) {                                    \
    float a[N][N], w[N], v[N][N];                  \
    std::memcpy(a, A, sizeof(a));                  \
    lego::cv_eigen_sym<N>(a, w, v);                \
    std::memcpy(W, w, sizeof(w));                  \
    std::memcpy(V, v, sizeof(v));                  \
    return 0;                                      \
  }
  CASE(3) CASE(6)
#undef CASE
  return -1;
}

// Mat::inv(): n = 3 closed form (cv_inv3), n = 6 LU (cv_inv_lu<6>).
int lw_inv(int n, const float* A, float* D) {
  if (n == 3) {
    float a[3][3], d[3][3];
    std::memcpy(a, A, sizeof(a));
    const bool ok = lego::cv_inv3(a, d);
    std::memcpy(D, d, sizeof(d));
    return ok ? 1 : 0;
  }
  if (n == 6) {
    float a[6][6], d[6][6];
    std::memcpy(a, A, sizeof(a));
    const bool ok = lego::cv_inv_lu<6>(a, d);
    std::memcpy(D, d, sizeof(d));
    return ok ? 1 : 0;
  }
  return -1;
}

}  // extern "C"

#include "lego_icp.h"

extern "C" {

// Eigen JacobiSVD<Matrix3f> restatement: U, S (descending), V; 0 on invalid input.
int lw_svd3(const float* A, float* U, float* S, float* V) {
  float a[3][3], u[3][3], s[3], v[3][3];
  std::memcpy(a, A, sizeof(a));
  const bool ok = lego::jacobi_svd3(a, u, s, v);
  std::memcpy(U, u, sizeof(u));
  std::memcpy(S, s, sizeof(s));
  std::memcpy(V, v, sizeof(v));
  return ok ? 1 : 0;
}

// pcl::umeyama (no scaling) from the float means and the 1/n-scaled cross-covariance.
void lw_umeyama(const float* srcMean, const float* dstMean, const float* sigma, float* T) {
  float sm[3], dm[3], sg[3][3], t[4][4];
  std::memcpy(sm, srcMean, sizeof(sm));
  std::memcpy(dm, dstMean, sizeof(dm));
  std::memcpy(sg, sigma, sizeof(sg));
  lego::umeyama_finish(sm, dm, sg, t);
  std::memcpy(T, t, sizeof(t));
}

}  // extern "C"
