// The Eigen JacobiSVD<Matrix3f> / umeyama restatement (lego_icp.h) on random
// and degenerate 3x3 matrices: U S V^T reproduces A, U and V are orthonormal,
// S is non-negative and descending; umeyama_finish recovers a known rigid
// motion from exact correspondences; icp_converged follows PCL's criteria.
#include <cmath>
#include <cstdio>
#include <random>

#include "../../lego-loam_amd/csrc/lego_icp.h"

int main(int argc, char** argv) {
  const long n = argc > 1 ? std::atol(argv[1]) : 100000;
  std::mt19937_64 rng(99);
  std::uniform_real_distribution<float> U(-1.f, 1.f);
  std::uniform_int_distribution<int> E(-6, 6), K(0, 5);
  long bad = 0;
  for (long it = 0; it < n; ++it) {
    float A[3][3];
    const int kind = K(rng);
    for (auto& r : A)
      for (float& v : r) v = U(rng) * std::ldexp(1.f, kind < 2 ? E(rng) : 0);
    if (kind == 3)  // rank 2
      for (int j = 0; j < 3; ++j) A[2][j] = A[0][j] + A[1][j];
    if (kind == 4)  // rank 1
      for (int j = 0; j < 3; ++j) A[1][j] = 2 * A[0][j], A[2][j] = -A[0][j];
    if (kind == 5) A[0][1] = A[1][0] = A[0][2] = A[2][0] = 0;  // partly diagonal
    float Uu[3][3], S[3], V[3][3];
    lego::jacobi_svd3(A, Uu, S, V);
    double amax = 0, err = 0, orth = 0;
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) {
        amax = std::fmax(amax, std::fabs(A[i][j]));
        double r = 0, uu = 0, vv = 0;
        for (int k = 0; k < 3; ++k) {
          r += (double)Uu[i][k] * S[k] * V[j][k];
          uu += (double)Uu[k][i] * Uu[k][j];
          vv += (double)V[k][i] * V[k][j];
        }
        err = std::fmax(err, std::fabs(r - A[i][j]));
        orth = std::fmax(orth, std::fmax(std::fabs(uu - (i == j)), std::fabs(vv - (i == j))));
      }
    const bool ok = err <= 1e-5 * std::fmax(amax, 1e-30) + 1e-30 && orth <= 1e-5 && S[0] >= S[1] && S[1] >= S[2] &&
                    S[2] >= 0;
    if (!ok && bad++ < 5) std::printf("svd mismatch at %ld (kind %d): err %g orth %g S %g %g %g\n", it, kind, err, orth,
                                      S[0], S[1], S[2]);
  }
  // umeyama: rotation about a random axis + translation, 50 exact point pairs
  long badU = 0;
  for (int it = 0; it < 2000; ++it) {
    const double ax = U(rng), ay = U(rng), az = U(rng), nn = std::sqrt(ax * ax + ay * ay + az * az) + 1e-9;
    const double th = U(rng) * 0.5, c = std::cos(th), s = std::sin(th), x = ax / nn, y = ay / nn, z = az / nn;
    const double R[3][3] = {{c + x * x * (1 - c), x * y * (1 - c) - z * s, x * z * (1 - c) + y * s},
                            {y * x * (1 - c) + z * s, c + y * y * (1 - c), y * z * (1 - c) - x * s},
                            {z * x * (1 - c) - y * s, z * y * (1 - c) + x * s, c + z * z * (1 - c)}};
    const double t[3] = {U(rng) * 2.0, U(rng) * 2.0, U(rng) * 2.0};
    float src[50][3], dst[50][3];
    double ss[3] = {0, 0, 0}, sd[3] = {0, 0, 0};
    for (int k = 0; k < 50; ++k) {
      for (int r = 0; r < 3; ++r) src[k][r] = U(rng) * 10.f;
      for (int r = 0; r < 3; ++r)
        dst[k][r] = (float)(R[r][0] * src[k][0] + R[r][1] * src[k][1] + R[r][2] * src[k][2] + t[r]);
      for (int r = 0; r < 3; ++r) ss[r] += src[k][r], sd[r] += dst[k][r];
    }
    const float on = 1.0f / 50.f;
    float sm[3], dm[3], sigma[3][3], T[4][4];
    for (int r = 0; r < 3; ++r) sm[r] = (float)ss[r] * on, dm[r] = (float)sd[r] * on;
    double sg[3][3] = {};
    for (int k = 0; k < 50; ++k)
      for (int r = 0; r < 3; ++r)
        for (int q = 0; q < 3; ++q) sg[r][q] += (double)(dst[k][r] - dm[r]) * (double)(src[k][q] - sm[q]);
    for (int r = 0; r < 3; ++r)
      for (int q = 0; q < 3; ++q) sigma[r][q] = (float)sg[r][q] * on;
    lego::umeyama_finish(sm, dm, sigma, T);
    double e = 0;
    for (int r = 0; r < 3; ++r) {
      for (int q = 0; q < 3; ++q) e = std::fmax(e, std::fabs(T[r][q] - R[r][q]));
      e = std::fmax(e, std::fabs(T[r][3] - t[r]) / 10);
    }
    if (e > 1e-4 && badU++ < 5) std::printf("umeyama error %g at %d\n", e, it);
  }
  // criteria: an identity increment converges on the transformation test; a
  // large one does not, then the relative-MSE test fires on a repeated MSE
  long badC = 0;
  {
    lego::IcpCriteria c = lego::icp_criteria(100, 1e-6, 1e-6);
    float I[4][4] = {{1, 0, 0, 0}, {0, 1, 0, 0}, {0, 0, 1, 0}, {0, 0, 0, 1}};
    float B[4][4] = {{1, 0, 0, 0.5f}, {0, 1, 0, 0}, {0, 0, 1, 0}, {0, 0, 0, 1}};
    badC += lego::icp_converged(c, 1, B, 2.0) ? 1 : 0;
    badC += lego::icp_converged(c, 2, B, 2.0) ? 0 : 1;  // |dMSE| < 1e-12
    lego::IcpCriteria c2 = lego::icp_criteria(100, 1e-6, 1e-6);
    badC += lego::icp_converged(c2, 1, I, 1.0) ? 0 : 1;
    lego::IcpCriteria c3 = lego::icp_criteria(5, 1e-6, 1e-6);
    badC += lego::icp_converged(c3, 5, B, 3.0) ? 0 : 1;  // iteration cap
  }
  std::printf("svd3: %ld / %ld bad; umeyama %ld / 2000 bad; criteria %ld bad\n", bad, n, badU, badC);
  return bad || badU || badC ? 1 : 0;
}
