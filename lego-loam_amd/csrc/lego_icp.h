// lego_icp.h — restatements of the arithmetic mapOptimization's loop closure
// (mapOptmization.cpp:875-945) takes from PCL 1.8 and Eigen 3.3 and GTSAM,
// shared by the oracle and the kernels (as lego_numerics.h is for libm and
// OpenCV):
//   * Eigen JacobiSVD<Matrix3f> (two-sided Jacobi, Jacobi/Jacobi.h and
//     SVD/JacobiSVD.h) and pcl::umeyama (Eigen/Geometry/Umeyama.h) as
//     pcl::registration::TransformationEstimationSVD uses it;
//   * pcl::registration::DefaultConvergenceCriteria<float>::hasConverged;
//   * pcl::transformPointCloud's per-point form (common/impl/transforms.hpp);
//   * pcl::getTranslationAndEulerAngles / pcl::getTransformation
//     (common/impl/eigen.hpp), gtsam::Rot3::RzRyRx and Pose3::between.
// None of these libraries is in the image: the restatements follow their
// published algorithms and are unpinned against them.
// Deviation: Eigen sums umeyama's means and cross-covariance in float with a
// vectorisation-dependent order; here they are summed in double (exact
// float products) and rounded once, so the parallel reductions of the kernels
// and the sequential ones of the oracle agree.
#pragma once
#include <cfloat>
#include <cmath>

#include "lego_numerics.h"

namespace lego {

// ---------------------------------------------------------------- Jacobi SVD
struct JRot {
  float c, s;
};
LEGO_HD JRot jrot_mul(JRot a, JRot b) {  // JacobiRotation::operator* (real)
  return {a.c * b.c - a.s * b.s, a.c * b.s + a.s * b.c};
}
LEGO_HD JRot jrot_t(JRot a) { return {a.c, -a.s}; }  // transpose()

// JacobiRotation::makeJacobi(x, y, z) for real scalars
LEGO_HD bool make_jacobi(float x, float y, float z, JRot* r) {
  const float deno = 2.0f * lfabsf(y);
  if (deno < FLT_MIN) {
    r->c = 1.0f;
    r->s = 0.0f;
    return false;
  }
  const float tau = (x - z) / deno;
  const float w = lsqrtf(tau * tau + 1.0f);
  float t;
  if (tau > 0.0f) t = 1.0f / (tau + w);
  else t = 1.0f / (tau - w);
  const float sign_t = t > 0.0f ? 1.0f : -1.0f;
  const float n = 1.0f / lsqrtf(t * t + 1.0f);
  r->s = -sign_t * (y / lfabsf(y)) * lfabsf(t) * n;
  r->c = n;
  return true;
}

// apply_rotation_in_the_plane on rows p, q (applyOnTheLeft) and on columns
// p, q with j^T (applyOnTheRight); identity rotations are skipped as Eigen does
LEGO_HD void rot_left(float (&m)[3][3], int p, int q, JRot j) {
  if (j.c == 1.0f && j.s == 0.0f) return;
  for (int i = 0; i < 3; ++i) {
    const float xi = m[p][i], yi = m[q][i];
    m[p][i] = j.c * xi + j.s * yi;
    m[q][i] = -j.s * xi + j.c * yi;
  }
}
LEGO_HD void rot_right(float (&m)[3][3], int p, int q, JRot j) {
  const JRot t = jrot_t(j);
  if (t.c == 1.0f && t.s == 0.0f) return;
  for (int i = 0; i < 3; ++i) {
    const float xi = m[i][p], yi = m[i][q];
    m[i][p] = t.c * xi + t.s * yi;
    m[i][q] = -t.s * xi + t.c * yi;
  }
}

// internal::real_2x2_jacobi_svd
LEGO_HD void real_2x2_jacobi_svd(const float (&a)[3][3], int p, int q, JRot* jl, JRot* jr) {
  float m[2][2] = {{a[p][p], a[p][q]}, {a[q][p], a[q][q]}};
  JRot rot1;
  const float t = m[0][0] + m[1][1];
  const float d = m[1][0] - m[0][1];
  if (lfabsf(d) < FLT_MIN) {
    rot1.s = 0.0f;
    rot1.c = 1.0f;
  } else {
    const float u = t / d;
    const float tmp = lsqrtf(1.0f + u * u);
    rot1.s = 1.0f / tmp;
    rot1.c = u / tmp;
  }
  if (!(rot1.c == 1.0f && rot1.s == 0.0f)) {  // m.applyOnTheLeft(0, 1, rot1)
    for (int i = 0; i < 2; ++i) {
      const float xi = m[0][i], yi = m[1][i];
      m[0][i] = rot1.c * xi + rot1.s * yi;
      m[1][i] = -rot1.s * xi + rot1.c * yi;
    }
  }
  make_jacobi(m[0][0], m[0][1], m[1][1], jr);
  *jl = jrot_mul(rot1, jrot_t(*jr));
}

// JacobiSVD<Matrix3f>(A, ComputeFullU | ComputeFullV): U, singular values
// (descending), V.  Returns false for a non-finite input (InvalidInput).
LEGO_HD bool jacobi_svd3(const float (&A)[3][3], float (&U)[3][3], float (&S)[3], float (&V)[3][3]) {
  const float precision = 2.0f * FLT_EPSILON;
  const float considerAsZero = FLT_MIN;
  float scale = 0.0f;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {  // cwiseAbs().maxCoeff(), column-major visit
      const float v = lfabsf(A[j][i]);
      if (v > scale || (i == 0 && j == 0)) scale = v;
    }
  if (!(scale - scale == 0.0f)) return false;
  if (scale == 0.0f) scale = 1.0f;
  float W[3][3];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      W[i][j] = A[i][j] / scale;
      U[i][j] = i == j ? 1.0f : 0.0f;
      V[i][j] = i == j ? 1.0f : 0.0f;
    }
  float maxDiag = lfabsf(W[0][0]);
  for (int i = 1; i < 3; ++i)
    if (lfabsf(W[i][i]) > maxDiag) maxDiag = lfabsf(W[i][i]);
  bool finished = false;
  for (int sweep = 0; !finished && sweep < 64; ++sweep) {  // converges in a few sweeps; the cap only bounds NaN
    finished = true;
    for (int p = 1; p < 3; ++p)
      for (int q = 0; q < p; ++q) {
        const float pm = precision * maxDiag;
        const float threshold = considerAsZero > pm ? considerAsZero : pm;
        if (lfabsf(W[p][q]) > threshold || lfabsf(W[q][p]) > threshold) {
          finished = false;
          JRot jl, jr;
          real_2x2_jacobi_svd(W, p, q, &jl, &jr);
          rot_left(W, p, q, jl);
          rot_right(U, p, q, jrot_t(jl));
          rot_right(W, p, q, jr);
          rot_right(V, p, q, jr);
          const float ap = lfabsf(W[p][p]), aq = lfabsf(W[q][q]);
          const float mpq = ap > aq ? ap : aq;
          if (mpq > maxDiag) maxDiag = mpq;
        }
      }
  }
  for (int i = 0; i < 3; ++i) {
    const float a = W[i][i];
    S[i] = lfabsf(a);
    if (a < 0.0f)
      for (int r = 0; r < 3; ++r) U[r][i] = -U[r][i];
  }
  for (int i = 0; i < 3; ++i) S[i] *= scale;
  for (int i = 0; i < 3; ++i) {  // sort descending: tail(3 - i).maxCoeff(&pos), first maximum
    int pos = i;
    float mx = S[i];
    for (int k = i + 1; k < 3; ++k)
      if (S[k] > mx) { mx = S[k]; pos = k; }
    if (mx == 0.0f) break;
    if (pos != i) {
      const float t = S[i]; S[i] = S[pos]; S[pos] = t;
      for (int r = 0; r < 3; ++r) {
        float u = U[r][i]; U[r][i] = U[r][pos]; U[r][pos] = u;
        float v = V[r][i]; V[r][i] = V[r][pos]; V[r][pos] = v;
      }
    }
  }
  return true;
}

// Eigen's 3x3 determinant (bruteforce_det3_helper)
LEGO_HD float det3f(const float (&m)[3][3]) {
  auto h = [&](int a, int b, int c) { return m[0][a] * (m[1][b] * m[2][c] - m[1][c] * m[2][b]); };
  return h(0, 1, 2) - h(1, 0, 2) + h(2, 0, 1);
}

// umeyama(src, dst, false) given the float means and the (already scaled by
// 1/n) cross-covariance sigma = dst_demean * src_demean^T / n.  Row-major 4x4.
LEGO_HD void umeyama_finish(const float (&srcMean)[3], const float (&dstMean)[3], const float (&sigma)[3][3],
                            float (&Rt)[4][4]) {
  float U[3][3], S[3], V[3][3];
  jacobi_svd3(sigma, U, S, V);
  float Sd[3] = {1.0f, 1.0f, 1.0f};
  if (det3f(U) * det3f(V) < 0.0f) Sd[2] = -1.0f;
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) Rt[i][j] = i == j ? 1.0f : 0.0f;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {  // (U * S.asDiagonal()) * V^T
      float acc = (U[i][0] * Sd[0]) * V[j][0];
      acc = acc + (U[i][1] * Sd[1]) * V[j][1];
      acc = acc + (U[i][2] * Sd[2]) * V[j][2];
      Rt[i][j] = acc;
    }
  for (int i = 0; i < 3; ++i) {  // t = dst_mean - R src_mean
    float rs = Rt[i][0] * srcMean[0];
    rs = rs + Rt[i][1] * srcMean[1];
    rs = rs + Rt[i][2] * srcMean[2];
    Rt[i][3] = dstMean[i] - rs;
  }
}

// final = T * final (Matrix4f product, k in order)
LEGO_HD void mat4_mul(const float (&A)[4][4], const float (&B)[4][4], float (&C)[4][4]) {
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) {
      float acc = A[i][0] * B[0][j];
      acc = acc + A[i][1] * B[1][j];
      acc = acc + A[i][2] * B[2][j];
      acc = acc + A[i][3] * B[3][j];
      C[i][j] = acc;
    }
}

// pcl::transformPointCloud per point (transforms.hpp, PCL 1.8)
LEGO_HD void xform_point(const float* T /*row-major 4x4*/, float x, float y, float z, float* ox, float* oy,
                         float* oz) {
  *ox = T[0] * x + T[1] * y + T[2] * z + T[3];
  *oy = T[4] * x + T[5] * y + T[6] * z + T[7];
  *oz = T[8] * x + T[9] * y + T[10] * z + T[11];
}

// DefaultConvergenceCriteria<float> as IterativeClosestPoint configures it
// (max iterations, relative MSE = euclidean fitness epsilon, translation
// threshold = transformation epsilon, rotation threshold = 1 - epsilon)
struct IcpCriteria {
  int maxIterations;
  double relMse, transThr, rotThr, absMse;
  double prevMse;
  int similar, maxSimilar;
};
LEGO_HD IcpCriteria icp_criteria(int maxIt, double transEps, double fitnessEps) {
  return IcpCriteria{maxIt, fitnessEps, transEps, 1.0 - transEps, 1e-12, DBL_MAX, 0, 0};
}
// hasConverged() after iteration `iterations` (already incremented);
// T = this iteration's transformation_, mse = calculateMSE of its correspondences
LEGO_HD bool icp_converged(IcpCriteria& c, int iterations, const float (&T)[4][4], double mse) {
  if (iterations >= c.maxIterations) return true;  // failure_after_max_iter_ = false
  const double cos_angle = 0.5 * ((double)T[0][0] + (double)T[1][1] + (double)T[2][2] - 1);
  const double translation_sqr = (double)T[0][3] * (double)T[0][3] + (double)T[1][3] * (double)T[1][3] +
                                 (double)T[2][3] * (double)T[2][3];
  if (cos_angle >= c.rotThr && translation_sqr <= c.transThr) {
    if (c.similar < c.maxSimilar) { ++c.similar; return false; }
    c.similar = 0;
    return true;
  }
  if (fabs(mse - c.prevMse) < c.absMse) {
    if (c.similar < c.maxSimilar) { ++c.similar; return false; }
    c.similar = 0;
    return true;
  }
  if (fabs(mse - c.prevMse) / c.prevMse < c.relMse) {
    if (c.similar < c.maxSimilar) { ++c.similar; return false; }
    c.similar = 0;
    return true;
  }
  c.prevMse = mse;
  return false;
}

// ---------------------------------------------------------------- pose math (host)
// pcl::getTranslationAndEulerAngles (Affine3f, row-major 4x4 here)
LEGO_HD void pcl_translation_euler(const float (&t)[4][4], float* x, float* y, float* z, float* roll, float* pitch,
                                   float* yaw) {
  *x = t[0][3];
  *y = t[1][3];
  *z = t[2][3];
  *roll = lego_atan2f(t[2][1], t[2][2]);
  *pitch = lego_asinf(-t[2][0]);
  *yaw = lego_atan2f(t[1][0], t[0][0]);
}
// pcl::getTransformation(x, y, z, roll, pitch, yaw)
LEGO_HD void pcl_transformation(float x, float y, float z, float roll, float pitch, float yaw, float (&t)[4][4]) {
  const float A = lego_cosf(yaw), B = lego_sinf(yaw), C = lego_cosf(pitch), D = lego_sinf(pitch),
              E = lego_cosf(roll), F = lego_sinf(roll), DE = D * E, DF = D * F;
  t[0][0] = A * C; t[0][1] = A * DF - B * E; t[0][2] = B * F + A * DE; t[0][3] = x;
  t[1][0] = B * C; t[1][1] = A * E + B * DF; t[1][2] = B * DE - A * F; t[1][3] = y;
  t[2][0] = -D; t[2][1] = C * F; t[2][2] = C * E; t[2][3] = z;
  t[3][0] = 0; t[3][1] = 0; t[3][2] = 0; t[3][3] = 1;
}
// gtsam::Rot3::RzRyRx(x, y, z) = Rz(z) Ry(y) Rx(x), double
LEGO_HD void rot3_rzryrx(double x, double y, double z, double (&R)[3][3]) {
  const double cx = cos(x), sx = sin(x), cy = cos(y), sy = sin(y), cz = cos(z), sz = sin(z);
  const double ss_ = sx * sy, cs_ = cx * sy;
  R[0][0] = cy * cz; R[0][1] = -cx * sz + ss_ * cz; R[0][2] = sx * sz + cs_ * cz;
  R[1][0] = cy * sz; R[1][1] = cx * cz + ss_ * sz; R[1][2] = -sx * cz + cs_ * sz;
  R[2][0] = -sy; R[2][1] = sx * cy; R[2][2] = cx * cy;
}
// gtsam::Pose3::between(p2) = inverse() * p2 with inverse() = (R1^T, R1^T (-t1))
// and compose (Ra Rb, ta + Ra tb)
LEGO_HD void pose3_between(const double (&R1)[3][3], const double (&t1)[3], const double (&R2)[3][3],
                           const double (&t2)[3], double (&R)[3][3], double (&t)[3]) {
  double ti[3];
  for (int i = 0; i < 3; ++i) ti[i] = R1[0][i] * -t1[0] + R1[1][i] * -t1[1] + R1[2][i] * -t1[2];
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j) R[i][j] = R1[0][i] * R2[0][j] + R1[1][i] * R2[1][j] + R1[2][i] * R2[2][j];
    t[i] = ti[i] + (R1[0][i] * t2[0] + R1[1][i] * t2[1] + R1[2][i] * t2[2]);
  }
}

// The loop constraint of performLoopClosure (:919-934) from the ICP's final
// transformation and the two keyframes' poses6 (x y z roll pitch yaw, the
// camera-frame keyframe pose of cloudKeyPoses6D): gtsam poseFrom, poseTo and
// poseFrom.between(poseTo) as rotation matrix + translation.
struct LoopFactor {
  double fromR[3][3], fromT[3], toR[3][3], toT[3], betweenR[3][3], betweenT[3];
  float fromRpy[3];  // roll, pitch, yaw of tCorrect (float, as the reference passes them)
};
LEGO_HD void loop_factor(const float (&finalT)[4][4], const float* latest6, const float* closest6, LoopFactor* f) {
  float x, y, z, roll, pitch, yaw;
  pcl_translation_euler(finalT, &x, &y, &z, &roll, &pitch, &yaw);
  float corr[4][4], wrong[4][4], correct[4][4];
  pcl_transformation(z, x, y, yaw, roll, pitch, corr);  // correctionLidarFrame
  // pclPointToAffine3fCameraToLidar: getTransformation(p.z, p.x, p.y, p.yaw, p.roll, p.pitch)
  pcl_transformation(latest6[2], latest6[0], latest6[1], latest6[5], latest6[3], latest6[4], wrong);
  mat4_mul(corr, wrong, correct);
  pcl_translation_euler(correct, &x, &y, &z, &roll, &pitch, &yaw);
  rot3_rzryrx(roll, pitch, yaw, f->fromR);
  f->fromT[0] = x; f->fromT[1] = y; f->fromT[2] = z;
  f->fromRpy[0] = roll; f->fromRpy[1] = pitch; f->fromRpy[2] = yaw;
  // pclPointTogtsamPose3: RzRyRx(yaw, roll, pitch), Point3(z, x, y)
  rot3_rzryrx((double)closest6[5], (double)closest6[3], (double)closest6[4], f->toR);
  f->toT[0] = (double)closest6[2]; f->toT[1] = (double)closest6[0]; f->toT[2] = (double)closest6[1];
  pose3_between(f->fromR, f->fromT, f->toR, f->toT, f->betweenR, f->betweenT);
}

}  // namespace lego
