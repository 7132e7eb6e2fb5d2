// lego_pgo_host.h — the keyframe pose graph of mapOptimization (iSAM2's role,
// mapOptmization.cpp:229-231, 936-941, 1372-1420, 1456-1478), host C++.
//
// GTSAM is not in this image.  This restates the factor graph the reference
// builds and solves it in batch:
//   * variables: one gtsam::Pose3 per saved keyframe, Pose3(Rot3::RzRyRx(
//     t[2], t[0], t[1]), Point3(t[5], t[3], t[4])) of the camera-frame
//     transform t (:1376-1392);
//   * PriorFactor on pose 0 and BetweenFactor(i-1, i, poseFrom.between(poseTo))
//     per keyframe, both with Diagonal::Variances(1e-6, 1e-6, 1e-6, 1e-8,
//     1e-8, 1e-6) (:345-350); the loop factors of performLoopClosure with
//     variances = the ICP fitness (:930-939);
//   * errors in GTSAM 4's default charts (GTSAM_POSE3_EXPMAP off): the local
//     coordinates of measured^-1 * h(x) are [Rot3::Logmap(R), translation];
//     updates retract as (R Exp(w), t + R v);
//   * Gauss-Newton to convergence over the whole graph (central-difference
//     Jacobians of those errors), the block-tridiagonal-plus-loops information
//     matrix factored by a block skyline (envelope) Cholesky, so a chain with a
//     few loops costs O(K) blocks plus the loops' spans.
// iSAM2 (relinearizeThreshold 0.01, relinearizeSkip 1) reaches the same
// optimum incrementally; its intermediate estimates, and GTSAM's float /
// ordering details, are not reproduced: parity against GTSAM is unpinned
// (DESIGN.md §2).  tests/test_pose_graph.py checks this solver against an
// independent scipy restatement and a closed-loop known answer.
//
// Without a loop factor every factor is satisfied by the initial values, so
// the estimate IS the chain and no solve runs (the product's keyframe store
// then needs no host round trip, as before).
#pragma once

#include <cmath>
#include <cstring>
#include <vector>

namespace lego {

struct Pose3d {
  double R[3][3];
  double t[3];
};

inline Pose3d pose_identity() {
  Pose3d p{};
  for (int i = 0; i < 3; ++i) p.R[i][i] = 1.0;
  return p;
}

inline void mat3_mul(const double (&A)[3][3], const double (&B)[3][3], double (&C)[3][3]) {
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) C[i][j] = A[i][0] * B[0][j] + A[i][1] * B[1][j] + A[i][2] * B[2][j];
}

// gtsam::Rot3::RzRyRx(x, y, z) = Rz(z) Ry(y) Rx(x)
inline void pgo_rzryrx(double x, double y, double z, double (&R)[3][3]) {
  const double cx = std::cos(x), sx = std::sin(x), cy = std::cos(y), sy = std::sin(y), cz = std::cos(z),
               sz = std::sin(z);
  R[0][0] = cy * cz; R[0][1] = -cx * sz + sx * sy * cz; R[0][2] = sx * sz + cx * sy * cz;
  R[1][0] = cy * sz; R[1][1] = cx * cz + sx * sy * sz; R[1][2] = -sx * cz + cx * sy * sz;
  R[2][0] = -sy; R[2][1] = sx * cy; R[2][2] = cx * cy;
}

// gtsam::Rot3::xyz() (the RQ decomposition by Givens rotations, Matrix.cpp RQ):
// x, y, z with R = Rz(z) Ry(y) Rx(x); roll() = x, pitch() = y, yaw() = z.
inline void pgo_xyz(const double (&A)[3][3], double* x, double* y, double* z) {
  *x = -std::atan2(-A[2][1], A[2][2]);
  const double cx = std::cos(-*x), sx = std::sin(-*x);
  double B[3][3];  // A * Rx(-x)
  for (int i = 0; i < 3; ++i) {
    B[i][0] = A[i][0];
    B[i][1] = A[i][1] * cx + A[i][2] * sx;
    B[i][2] = -A[i][1] * sx + A[i][2] * cx;
  }
  *y = -std::atan2(B[2][0], B[2][2]);
  const double cy = std::cos(-*y), sy = std::sin(-*y);
  double C[3][3];  // B * Ry(-y)
  for (int i = 0; i < 3; ++i) {
    C[i][0] = B[i][0] * cy - B[i][2] * sy;
    C[i][1] = B[i][1];
    C[i][2] = B[i][0] * sy + B[i][2] * cy;
  }
  *z = -std::atan2(-C[1][0], C[1][1]);
}

// The camera-frame transform (roll, pitch, yaw, x, y, z as transformTobeMapped)
// <-> gtsam::Pose3 (:1376-1392 and :1412-1438)
inline Pose3d pose_from_transform(const float (&t)[6]) {
  Pose3d p;
  pgo_rzryrx((double)t[2], (double)t[0], (double)t[1], p.R);
  p.t[0] = (double)t[5];
  p.t[1] = (double)t[3];
  p.t[2] = (double)t[4];
  return p;
}
inline void transform_from_pose(const Pose3d& p, float (&t)[6]) {
  double x, y, z;
  pgo_xyz(p.R, &x, &y, &z);
  t[0] = (float)y;  // rotation().pitch()
  t[1] = (float)z;  // rotation().yaw()
  t[2] = (float)x;  // rotation().roll()
  t[3] = (float)p.t[1];
  t[4] = (float)p.t[2];
  t[5] = (float)p.t[0];
}

// A transform through gtsam::Pose3 and back: what the reference stores as
// every key pose and, past the first key, as transformAftMapped /
// TobeMapped / Last (mapOptmization.cpp:1412-1432 read latestEstimate's
// rotation().pitch() / yaw() / roll()).  Wraps a yaw past +-pi, re-branches
// |pitch| > pi/2, and may move a last bit.
inline void transform_roundtrip(const float (&in)[6], float (&out)[6]) { transform_from_pose(pose_from_transform(in), out); }

// a^-1 b
inline Pose3d pose_between(const Pose3d& a, const Pose3d& b) {
  Pose3d r;
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j) r.R[i][j] = a.R[0][i] * b.R[0][j] + a.R[1][i] * b.R[1][j] + a.R[2][i] * b.R[2][j];
    double d[3] = {b.t[0] - a.t[0], b.t[1] - a.t[1], b.t[2] - a.t[2]};
    r.t[i] = a.R[0][i] * d[0] + a.R[1][i] * d[1] + a.R[2][i] * d[2];
  }
  return r;
}

// SO(3) exponential and logarithm (Rodrigues)
inline void so3_exp(const double (&w)[3], double (&R)[3][3]) {
  const double th2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2], th = std::sqrt(th2);
  double a, b;
  if (th < 1e-8) {
    a = 1.0 - th2 / 6.0;
    b = 0.5 - th2 / 24.0;
  } else {
    a = std::sin(th) / th;
    b = (1.0 - std::cos(th)) / th2;
  }
  const double W[3][3] = {{0, -w[2], w[1]}, {w[2], 0, -w[0]}, {-w[1], w[0], 0}};
  double W2[3][3];
  mat3_mul(W, W, W2);
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) R[i][j] = (i == j ? 1.0 : 0.0) + a * W[i][j] + b * W2[i][j];
}
inline void so3_log(const double (&R)[3][3], double (&w)[3]) {
  const double tr = R[0][0] + R[1][1] + R[2][2];
  const double v[3] = {R[2][1] - R[1][2], R[0][2] - R[2][0], R[1][0] - R[0][1]};
  double c = 0.5 * (tr - 1.0);
  if (c > 1.0) c = 1.0;
  if (c < -1.0) c = -1.0;
  const double th = std::acos(c);
  if (th < 1e-6) {  // sin th / th ~ 1 - th^2/6
    const double f = 0.5 * (1.0 + th * th / 6.0);
    for (int i = 0; i < 3; ++i) w[i] = f * v[i];
    return;
  }
  if (M_PI - th < 1e-6) {  // near pi: from the symmetric part
    int k = 0;
    for (int i = 1; i < 3; ++i)
      if (R[i][i] > R[k][k]) k = i;
    double col[3];
    for (int i = 0; i < 3; ++i) col[i] = R[i][k] + (i == k ? 1.0 : 0.0);
    const double n = std::sqrt(col[0] * col[0] + col[1] * col[1] + col[2] * col[2]);
    for (int i = 0; i < 3; ++i) w[i] = th * col[i] / n;
    return;
  }
  const double f = th / (2.0 * std::sin(th));
  for (int i = 0; i < 3; ++i) w[i] = f * v[i];
}

// retract (GTSAM 4 default Pose3 chart): x (+) d = (R Exp(d_w), t + R d_v)
inline Pose3d pose_retract(const Pose3d& x, const double* d) {
  Pose3d r;
  double E[3][3];
  const double w[3] = {d[0], d[1], d[2]};
  so3_exp(w, E);
  mat3_mul(x.R, E, r.R);
  for (int i = 0; i < 3; ++i) r.t[i] = x.t[i] + x.R[i][0] * d[3] + x.R[i][1] * d[4] + x.R[i][2] * d[5];
  return r;
}
// local coordinates of z^-1 h: [Logmap(Rz^T Rh), Rz^T (th - tz)]
inline void pose_local(const Pose3d& z, const Pose3d& h, double (&e)[6]) {
  const Pose3d d = pose_between(z, h);
  double w[3];
  so3_log(d.R, w);
  for (int i = 0; i < 3; ++i) {
    e[i] = w[i];
    e[3 + i] = d.t[i];
  }
}

struct PoseGraph {
  struct Factor {
    int i, j;       // j < 0: a prior on i
    Pose3d z;       // measurement (prior value)
    double info[6]; // 1 / variance (Diagonal::Variances)
  };
  std::vector<Pose3d> est;  // the estimate, initial values until a solve
  std::vector<Factor> f;
  int loops = 0;            // loop factors added

  void clear() {
    est.clear();
    f.clear();
    loops = 0;
  }
  static void info_of(const double (&var)[6], double (&info)[6]) {
    for (int k = 0; k < 6; ++k) info[k] = 1.0 / var[k];
  }
  // saveKeyFramesAndFactor: the first keyframe (prior) or the next (between)
  void add_prior(const Pose3d& p, const double (&var)[6]) {
    Factor q{0, -1, p, {}};
    info_of(var, q.info);
    f.push_back(q);
  }
  void add_between(int i, int j, const Pose3d& z, const double (&var)[6], bool loop = false) {
    Factor q{i, j, z, {}};
    info_of(var, q.info);
    f.push_back(q);
    if (loop) ++loops;
  }
  void insert(const Pose3d& initial) { est.push_back(initial); }

  void error(const Factor& q, const std::vector<Pose3d>& x, double (&e)[6]) const {
    if (q.j < 0) pose_local(q.z, x[q.i], e);
    else pose_local(q.z, pose_between(x[q.i], x[q.j]), e);
  }

  // Gauss-Newton to convergence; returns the iterations run.
  int optimize(int maxIter = 30, double tol = 1e-10) {
    const int K = (int)est.size();
    if (K == 0) return 0;
    // block envelope: first[r] = lowest column coupled to row r
    std::vector<int> first(K);
    for (int r = 0; r < K; ++r) first[r] = r;
    for (const Factor& q : f)
      if (q.j >= 0) {
        const int lo = q.i < q.j ? q.i : q.j, hi = q.i < q.j ? q.j : q.i;
        if (lo < first[hi]) first[hi] = lo;
      }
    std::vector<size_t> off(K + 1, 0);
    for (int r = 0; r < K; ++r) off[r + 1] = off[r] + (size_t)(r - first[r] + 1) * 36;
    std::vector<double> H(off[K]), g((size_t)K * 6);
    auto blk = [&](int r, int c) { return &H[off[r] + (size_t)(c - first[r]) * 36]; };
    int it = 0;
    for (; it < maxIter; ++it) {
      std::fill(H.begin(), H.end(), 0.0);
      std::fill(g.begin(), g.end(), 0.0);
      std::vector<Pose3d> xp = est;
      for (const Factor& q : f) {
        const int nv = q.j < 0 ? 1 : 2;
        const int var[2] = {q.i, q.j};
        double e[6], J[2][6][6];
        error(q, est, e);
        for (int v = 0; v < nv; ++v)
          for (int k = 0; k < 6; ++k) {  // central differences along the retraction
            const double h = 1e-6;
            double d[6] = {0, 0, 0, 0, 0, 0}, ep[6], em[6];
            d[k] = h;
            xp[var[v]] = pose_retract(est[var[v]], d);
            error(q, xp, ep);
            d[k] = -h;
            xp[var[v]] = pose_retract(est[var[v]], d);
            error(q, xp, em);
            xp[var[v]] = est[var[v]];
            for (int r = 0; r < 6; ++r) J[v][r][k] = (ep[r] - em[r]) / (2 * h);
          }
        for (int a = 0; a < nv; ++a) {
          double* ga = &g[(size_t)var[a] * 6];
          for (int r = 0; r < 6; ++r)
            for (int k = 0; k < 6; ++k) ga[k] += J[a][r][k] * q.info[r] * e[r];
          for (int b = 0; b < nv; ++b) {
            if (var[b] > var[a]) continue;  // lower triangle: row var[a] >= column var[b]
            double* B = blk(var[a], var[b]);
            for (int k = 0; k < 6; ++k)
              for (int l = 0; l < 6; ++l) {
                double s = 0;
                for (int r = 0; r < 6; ++r) s += J[a][r][k] * q.info[r] * J[b][r][l];
                B[k * 6 + l] += s;
              }
          }
        }
      }
      // block skyline Cholesky H = L L^T in place (lower blocks)
      for (int r = 0; r < K; ++r) {
        for (int c = first[r]; c <= r; ++c) {
          double* A = blk(r, c);
          const int k0 = first[r] > first[c] ? first[r] : first[c];
          for (int k = k0; k < c; ++k) {  // A -= L[r][k] L[c][k]^T
            const double* Lr = blk(r, k);
            const double* Lc = blk(c, k);
            for (int a = 0; a < 6; ++a)
              for (int b = 0; b < 6; ++b) {
                double s = 0;
                for (int m = 0; m < 6; ++m) s += Lr[a * 6 + m] * Lc[b * 6 + m];
                A[a * 6 + b] -= s;
              }
          }
          if (c < r) {  // A L[c][c]^-T: forward substitution on each row of A
            const double* Lcc = blk(c, c);
            for (int a = 0; a < 6; ++a)
              for (int b = 0; b < 6; ++b) {
                double s = A[a * 6 + b];
                for (int m = 0; m < b; ++m) s -= A[a * 6 + m] * Lcc[b * 6 + m];
                A[a * 6 + b] = s / Lcc[b * 6 + b];
              }
          } else {  // dense 6x6 Cholesky of the diagonal block
            for (int a = 0; a < 6; ++a) {
              for (int b = 0; b <= a; ++b) {
                double s = A[a * 6 + b];
                for (int m = 0; m < b; ++m) s -= A[a * 6 + m] * A[b * 6 + m];
                if (a == b) A[a * 6 + a] = s > 0 ? std::sqrt(s) : 1e-300;
                else A[a * 6 + b] = s / A[b * 6 + b];
              }
              for (int b = a + 1; b < 6; ++b) A[a * 6 + b] = 0.0;
            }
          }
        }
      }
      // L y = -g, L^T d = y
      std::vector<double> y((size_t)K * 6);
      for (int r = 0; r < K; ++r)
        for (int a = 0; a < 6; ++a) {
          double s = -g[(size_t)r * 6 + a];
          for (int c = first[r]; c < r; ++c) {
            const double* L = blk(r, c);
            for (int m = 0; m < 6; ++m) s -= L[a * 6 + m] * y[(size_t)c * 6 + m];
          }
          const double* Lrr = blk(r, r);
          for (int m = 0; m < a; ++m) s -= Lrr[a * 6 + m] * y[(size_t)r * 6 + m];
          y[(size_t)r * 6 + a] = s / Lrr[a * 6 + a];
        }
      for (int r = K - 1; r >= 0; --r)  // row-oriented back substitution: scatter L^T
        for (int a = 5; a >= 0; --a) {
          const double* Lrr = blk(r, r);
          const double v = y[(size_t)r * 6 + a] / Lrr[a * 6 + a];
          y[(size_t)r * 6 + a] = v;
          for (int m = 0; m < a; ++m) y[(size_t)r * 6 + m] -= Lrr[a * 6 + m] * v;
          for (int c = first[r]; c < r; ++c) {
            const double* L = blk(r, c);
            for (int m = 0; m < 6; ++m) y[(size_t)c * 6 + m] -= L[a * 6 + m] * v;
          }
        }
      double dmax = 0;
      for (int r = 0; r < K; ++r) {
        est[r] = pose_retract(est[r], &y[(size_t)r * 6]);
        for (int a = 0; a < 6; ++a) dmax = std::fmax(dmax, std::fabs(y[(size_t)r * 6 + a]));
      }
      if (dmax < tol) {
        ++it;
        break;
      }
    }
    return it;
  }
};

// The variances of priorNoise / odometryNoise (mapOptmization.cpp:347-350)
inline const double (&pgo_odometry_variances())[6] {
  static const double v[6] = {1e-6, 1e-6, 1e-6, 1e-8, 1e-8, 1e-6};
  return v;
}

}  // namespace lego
