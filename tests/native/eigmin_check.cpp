// eig_min_above (the odometry's shortcut past the iteration-0 Jacobi) is
// sound: whenever it claims every eigenvalue exceeds the threshold, the
// OpenCV JacobiImpl_ restatement's smallest eigenvalue is >= the threshold
// too, so the degeneracy test (featureAssociation.cpp:1336-1347) finds
// nothing either way.  Matrices are built with a chosen smallest eigenvalue
// just above / at / below the threshold, large spreads, and LM-shaped AtA.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>

#include "../../lego-loam_amd/csrc/lego_numerics.h"

int main(int argc, char** argv) {
  const long n = argc > 1 ? std::atol(argv[1]) : 200000;
  std::mt19937_64 rng(777);
  std::uniform_real_distribution<double> U(-1.0, 1.0), L(0.0, 1.0);
  long bad = 0, taken = 0;
  const double thr = 10.0;
  for (long it = 0; it < n; ++it) {
    float A[3][3];
    const int kind = it % 3;
    if (kind < 2) {
      // random rotation (Gram-Schmidt) and spectrum {lmin, l1, l2}
      double q[3][3];
      for (auto& r : q)
        for (double& x : r) x = U(rng);
      for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < i; ++j) {
          double d = 0;
          for (int k = 0; k < 3; ++k) d += q[i][k] * q[j][k];
          for (int k = 0; k < 3; ++k) q[i][k] -= d * q[j][k];
        }
        double nrm = std::sqrt(q[i][0] * q[i][0] + q[i][1] * q[i][1] + q[i][2] * q[i][2]);
        for (int k = 0; k < 3; ++k) q[i][k] /= nrm;
      }
      const double spread = std::pow(10.0, 6 * L(rng));
      const double lmin = kind == 0 ? thr * (1 + std::ldexp(U(rng), -(int)(20 * L(rng)))) : thr * spread * L(rng);
      const double lam[3] = {lmin, lmin + spread * L(rng), lmin + spread};
      for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
          double s = 0;
          for (int k = 0; k < 3; ++k) s += q[k][i] * lam[k] * q[k][j];
          A[i][j] = (float)s;
        }
      for (int i = 0; i < 3; ++i)
        for (int j = 0; j < i; ++j) A[i][j] = A[j][i];
    } else {  // AtA of M LM-like rows
      const int M = 10 + (int)(200 * L(rng));
      const double sc = std::pow(10.0, 2 * U(rng));
      double S[3][3] = {};
      for (int r = 0; r < M; ++r) {
        const float row[3] = {(float)(U(rng) * sc), (float)(U(rng) * sc * 0.1), (float)(U(rng))};
        for (int i = 0; i < 3; ++i)
          for (int j = 0; j < 3; ++j) S[i][j] += (double)row[i] * row[j];
      }
      for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) A[i][j] = (float)S[i][j];
    }
    float Ac[3][3], W[3], V[3][3];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) Ac[i][j] = A[i][j];
    lego::cv_eigen_sym<3>(Ac, W, V);
    if (lego::eig_min_above(A, thr)) {
      ++taken;
      if (!(W[2] >= thr) && bad++ < 5) std::printf("unsound at %ld: lmin %.9g\n", it, W[2]);
    }
  }
  std::printf("eigmin: %ld unsound of %ld shortcuts, %ld matrices\n", bad, taken, n);
  // The mapping's 6 x 6 form (eig_min_above_n<6>, threshold 100) against
  // cv_eigen_sym<6>: spectra whose smallest eigenvalue sits just above / at /
  // below 100 under random rotations, wide spreads, and AtA of LM-shaped rows.
  long bad6 = 0, taken6 = 0;
  const long n6 = n / 3;
  const double thr6 = 100.0;
  for (long it = 0; it < n6; ++it) {
    float A[6][6];
    const int kind = it % 3;
    if (kind < 2) {
      double q[6][6];
      for (auto& r : q)
        for (double& x : r) x = U(rng);
      for (int i = 0; i < 6; ++i) {
        for (int j = 0; j < i; ++j) {
          double d = 0;
          for (int k = 0; k < 6; ++k) d += q[i][k] * q[j][k];
          for (int k = 0; k < 6; ++k) q[i][k] -= d * q[j][k];
        }
        double nrm = 0;
        for (int k = 0; k < 6; ++k) nrm += q[i][k] * q[i][k];
        nrm = std::sqrt(nrm);
        for (int k = 0; k < 6; ++k) q[i][k] /= nrm;
      }
      const double spread = std::pow(10.0, 6 * L(rng));
      const double lmin = kind == 0 ? thr6 * (1 + std::ldexp(U(rng), -(int)(20 * L(rng)))) : thr6 * spread * L(rng);
      double lam[6];
      lam[0] = lmin;
      for (int k = 1; k < 6; ++k) lam[k] = lmin + spread * L(rng);
      for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 6; ++j) {
          double s2 = 0;
          for (int k = 0; k < 6; ++k) s2 += q[k][i] * lam[k] * q[k][j];
          A[i][j] = (float)s2;
        }
      for (int i = 0; i < 6; ++i)
        for (int j = 0; j < i; ++j) A[i][j] = A[j][i];
    } else {  // AtA of M rows shaped like LMOptimization's (angles, then unit-normal translations)
      const int M = 50 + (int)(4000 * L(rng));
      const double sc = std::pow(10.0, 1.5 * U(rng));
      double S[6][6] = {};
      for (int r = 0; r < M; ++r) {
        float row[6];
        for (int k = 0; k < 3; ++k) row[k] = (float)(U(rng) * sc);
        for (int k = 3; k < 6; ++k) row[k] = (float)(U(rng) * (k == 5 ? 0.05 + L(rng) : 1.0));
        for (int i = 0; i < 6; ++i)
          for (int j = 0; j < 6; ++j) S[i][j] += (double)row[i] * row[j];
      }
      for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 6; ++j) A[i][j] = (float)S[i][j];
    }
    float Ac[6][6], W[6], V[6][6];
    for (int i = 0; i < 6; ++i)
      for (int j = 0; j < 6; ++j) Ac[i][j] = A[i][j];
    lego::cv_eigen_sym<6>(Ac, W, V);
    if (lego::eig_min_above_n<6>(A, thr6)) {
      ++taken6;
      if (!(W[5] >= thr6) && bad6++ < 5) std::printf("6x6 unsound at %ld: lmin %.9g\n", it, W[5]);
    }
  }
  std::printf("eigmin 6x6: %ld unsound of %ld shortcuts, %ld matrices\n", bad6, taken6, n6);
  return bad || taken == 0 || bad6 || taken6 == 0 ? 1 : 0;
}
