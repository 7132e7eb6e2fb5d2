// lego_fusion_host.h — transformFusion (transformFusion.cpp:94-239) on the
// host: the serial per-message consumer that composes each /laser_odom_to_init
// pose with the latest /aft_mapped_to_init correction into /integrated_to_init.
// Scalar float math per message, mirrored expression by expression (glibc
// float sinf / cosf / asinf / atan2f through lego_numerics.h).
#pragma once
#include "lego_imu_host.h"  // tf_get_rpy
#include "lego_numerics.h"

namespace lego {

struct Fusion {
  float transformSum[6] = {0, 0, 0, 0, 0, 0};
  float transformIncre[6] = {0, 0, 0, 0, 0, 0};
  float transformMapped[6] = {0, 0, 0, 0, 0, 0};
  float transformBefMapped[6] = {0, 0, 0, 0, 0, 0};
  float transformAftMapped[6] = {0, 0, 0, 0, 0, 0};

  // transformAssociateToMap :94-172
  void associate() {
    const float* s = transformSum;
    const float* b = transformBefMapped;
    const float* a = transformAftMapped;
    float* m = transformMapped;
    float x1 = lego_cosf(s[1]) * (b[3] - s[3]) - lego_sinf(s[1]) * (b[5] - s[5]);
    float y1 = b[4] - s[4];
    float z1 = lego_sinf(s[1]) * (b[3] - s[3]) + lego_cosf(s[1]) * (b[5] - s[5]);
    float x2 = x1;
    float y2 = lego_cosf(s[0]) * y1 + lego_sinf(s[0]) * z1;
    float z2 = -lego_sinf(s[0]) * y1 + lego_cosf(s[0]) * z1;
    transformIncre[3] = lego_cosf(s[2]) * x2 + lego_sinf(s[2]) * y2;
    transformIncre[4] = -lego_sinf(s[2]) * x2 + lego_cosf(s[2]) * y2;
    transformIncre[5] = z2;
    const float sbcx = lego_sinf(s[0]), cbcx = lego_cosf(s[0]);
    const float sbcy = lego_sinf(s[1]), cbcy = lego_cosf(s[1]);
    const float sbcz = lego_sinf(s[2]), cbcz = lego_cosf(s[2]);
    const float sblx = lego_sinf(b[0]), cblx = lego_cosf(b[0]);
    const float sbly = lego_sinf(b[1]), cbly = lego_cosf(b[1]);
    const float sblz = lego_sinf(b[2]), cblz = lego_cosf(b[2]);
    const float salx = lego_sinf(a[0]), calx = lego_cosf(a[0]);
    const float saly = lego_sinf(a[1]), caly = lego_cosf(a[1]);
    const float salz = lego_sinf(a[2]), calz = lego_cosf(a[2]);
    const float srx = -sbcx * (salx * sblx + calx * cblx * salz * sblz + calx * calz * cblx * cblz) -
                      cbcx * sbcy * (calx * calz * (cbly * sblz - cblz * sblx * sbly) -
                                     calx * salz * (cbly * cblz + sblx * sbly * sblz) + cblx * salx * sbly) -
                      cbcx * cbcy * (calx * salz * (cblz * sbly - cbly * sblx * sblz) -
                                     calx * calz * (sbly * sblz + cbly * cblz * sblx) + cblx * cbly * salx);
    m[0] = -lego_asinf(srx);
    const float srycrx = sbcx * (cblx * cblz * (caly * salz - calz * salx * saly) -
                                 cblx * sblz * (caly * calz + salx * saly * salz) + calx * saly * sblx) -
                         cbcx * cbcy * ((caly * calz + salx * saly * salz) * (cblz * sbly - cbly * sblx * sblz) +
                                        (caly * salz - calz * salx * saly) * (sbly * sblz + cbly * cblz * sblx) -
                                        calx * cblx * cbly * saly) +
                         cbcx * sbcy * ((caly * calz + salx * saly * salz) * (cbly * cblz + sblx * sbly * sblz) +
                                        (caly * salz - calz * salx * saly) * (cbly * sblz - cblz * sblx * sbly) +
                                        calx * cblx * saly * sbly);
    const float crycrx = sbcx * (cblx * sblz * (calz * saly - caly * salx * salz) -
                                 cblx * cblz * (saly * salz + caly * calz * salx) + calx * caly * sblx) +
                         cbcx * cbcy * ((saly * salz + caly * calz * salx) * (sbly * sblz + cbly * cblz * sblx) +
                                        (calz * saly - caly * salx * salz) * (cblz * sbly - cbly * sblx * sblz) +
                                        calx * caly * cblx * cbly) -
                         cbcx * sbcy * ((saly * salz + caly * calz * salx) * (cbly * sblz - cblz * sblx * sbly) +
                                        (calz * saly - caly * salx * salz) * (cbly * cblz + sblx * sbly * sblz) -
                                        calx * caly * cblx * sbly);
    m[1] = lego_atan2f(srycrx / lego_cosf(m[0]), crycrx / lego_cosf(m[0]));
    const float srzcrx = (cbcz * sbcy - cbcy * sbcx * sbcz) *
                             (calx * salz * (cblz * sbly - cbly * sblx * sblz) -
                              calx * calz * (sbly * sblz + cbly * cblz * sblx) + cblx * cbly * salx) -
                         (cbcy * cbcz + sbcx * sbcy * sbcz) *
                             (calx * calz * (cbly * sblz - cblz * sblx * sbly) -
                              calx * salz * (cbly * cblz + sblx * sbly * sblz) + cblx * salx * sbly) +
                         cbcx * sbcz * (salx * sblx + calx * cblx * salz * sblz + calx * calz * cblx * cblz);
    const float crzcrx = (cbcy * sbcz - cbcz * sbcx * sbcy) *
                             (calx * calz * (cbly * sblz - cblz * sblx * sbly) -
                              calx * salz * (cbly * cblz + sblx * sbly * sblz) + cblx * salx * sbly) -
                         (sbcy * sbcz + cbcy * cbcz * sbcx) *
                             (calx * salz * (cblz * sbly - cbly * sblx * sblz) -
                              calx * calz * (sbly * sblz + cbly * cblz * sblx) + cblx * cbly * salx) +
                         cbcx * cbcz * (salx * sblx + calx * cblx * salz * sblz + calx * calz * cblx * cblz);
    m[2] = lego_atan2f(srzcrx / lego_cosf(m[0]), crzcrx / lego_cosf(m[0]));
    x1 = lego_cosf(m[2]) * transformIncre[3] - lego_sinf(m[2]) * transformIncre[4];
    y1 = lego_sinf(m[2]) * transformIncre[3] + lego_cosf(m[2]) * transformIncre[4];
    z1 = transformIncre[5];
    x2 = x1;
    y2 = lego_cosf(m[0]) * y1 - lego_sinf(m[0]) * z1;
    z2 = lego_sinf(m[0]) * y1 + lego_cosf(m[0]) * z1;
    m[3] = a[3] - (lego_cosf(m[1]) * x2 + lego_sinf(m[1]) * z2);
    m[4] = a[4] - y2;
    m[5] = a[5] - (-lego_sinf(m[1]) * x2 + lego_cosf(m[1]) * z2);
  }

  // the roll/pitch/yaw of an Odometry orientation, as both handlers read it:
  // tf::Matrix3x3(tf::Quaternion(q.z, -q.x, -q.y, q.w)).getRPY (:178-180, :209-211)
  static void msg_rpy(const double q[4], double* roll, double* pitch, double* yaw) {
    const double t[4] = {q[2], -q[0], -q[1], q[3]};
    tf_get_rpy(t, roll, pitch, yaw);
  }

  // laserOdometryHandler :174-205 -> transformMapped
  void odometry(const double q[4], const double pos[3]) {
    double roll, pitch, yaw;
    msg_rpy(q, &roll, &pitch, &yaw);
    transformSum[0] = (float)-pitch;
    transformSum[1] = (float)-yaw;
    transformSum[2] = (float)roll;
    transformSum[3] = (float)pos[0];
    transformSum[4] = (float)pos[1];
    transformSum[5] = (float)pos[2];
    associate();
  }

  // odomAftMappedHandler :207-227 (pose = transformAftMapped, twist = transformBefMapped)
  void aft_mapped(const double q[4], const double pos[3], const float bef[6]) {
    double roll, pitch, yaw;
    msg_rpy(q, &roll, &pitch, &yaw);
    transformAftMapped[0] = (float)-pitch;
    transformAftMapped[1] = (float)-yaw;
    transformAftMapped[2] = (float)roll;
    transformAftMapped[3] = (float)pos[0];
    transformAftMapped[4] = (float)pos[1];
    transformAftMapped[5] = (float)pos[2];
    for (int i = 0; i < 6; ++i) transformBefMapped[i] = bef[i];
  }
};

}  // namespace lego
