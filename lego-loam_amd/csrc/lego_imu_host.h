// lego_imu_host.h — the /imu_raw callbacks of featureAssociation and
// mapOptimization, on the host.  Each message is a short serial update of a
// 200-entry queue (the reference runs it in its ROS callback); the per-point
// use of the queue (adjustDistortion) runs on the device from a per-scan
// snapshot (ImuSnap).
#pragma once
#include <cmath>
#include <cstring>

#include "lego_device.h"
#include "lego_loam.h"

namespace lego {

// tf::Matrix3x3(q).getRPY, solution 1 (tf/LinearMath/Matrix3x3.h), double.
inline void tf_get_rpy(const double q[4], double* roll, double* pitch, double* yaw) {
  const double x = q[0], y = q[1], z = q[2], w = q[3];
  const double d = x * x + y * y + z * z + w * w;
  const double s = 2.0 / d;
  const double xs = x * s, ys = y * s, zs = z * s;
  const double wx = w * xs, wy = w * ys, wz = w * zs;
  const double xx = x * xs, xy = x * ys, xz = x * zs;
  const double yy = y * ys, yz = y * zs, zz = z * zs;
  const double m00 = 1.0 - (yy + zz), m10 = xy + wz, m20 = xz - wy, m21 = yz + wx, m22 = 1.0 - (xx + yy);
  if (std::fabs(m20) >= 1) {
    *yaw = 0;
    *pitch = m20 < 0 ? M_PI / 2.0 : -M_PI / 2.0;
    *roll = std::atan2(m21, m22);
  } else {
    *pitch = -std::asin(m20);
    const double cp = std::cos(*pitch);
    *roll = std::atan2(m21 / cp, m22 / cp);
    *yaw = std::atan2(m10 / cp, m00 / cp);
  }
}

// featureAssociation's queue: imuHandler :431-458 + AccumulateIMUShiftAndRotation :392-429.
struct FaImuQueue {
  int last = -1;      // imuPointerLast
  int lastIter = 0;   // imuPointerLastIteration
  double time[kImuQ] = {};
  float v[kImuV][kImuQ] = {};
  float acc[3][kImuQ] = {};
  float angVelo[3][kImuQ] = {};

  void push(const lego_imu_msg& m, float scanPeriod) {
    double roll, pitch, yaw;
    tf_get_rpy(m.orientation, &roll, &pitch, &yaw);
    const float accX = (float)(m.linear_acceleration[1] - std::sin(roll) * std::cos(pitch) * 9.81);
    const float accY = (float)(m.linear_acceleration[2] - std::cos(roll) * std::cos(pitch) * 9.81);
    const float accZ = (float)(m.linear_acceleration[0] + std::sin(pitch) * 9.81);
    last = (last + 1) % kImuQ;
    const int l = last;
    time[l] = m.stamp;
    v[IV_ROLL][l] = (float)roll; v[IV_PITCH][l] = (float)pitch; v[IV_YAW][l] = (float)yaw;
    acc[0][l] = accX; acc[1][l] = accY; acc[2][l] = accZ;
    for (int k = 0; k < 3; ++k) angVelo[k][l] = (float)m.angular_velocity[k];
    // AccumulateIMUShiftAndRotation
    const float r = v[IV_ROLL][l], p = v[IV_PITCH][l], y = v[IV_YAW][l];
    float ax = acc[0][l], ay = acc[1][l], az = acc[2][l];
    const float x1 = lego_cosf(r) * ax - lego_sinf(r) * ay;
    const float y1 = lego_sinf(r) * ax + lego_cosf(r) * ay;
    const float z1 = az;
    const float x2 = x1;
    const float y2 = lego_cosf(p) * y1 - lego_sinf(p) * z1;
    const float z2 = lego_sinf(p) * y1 + lego_cosf(p) * z1;
    ax = lego_cosf(y) * x2 + lego_sinf(y) * z2;
    ay = y2;
    az = -lego_sinf(y) * x2 + lego_cosf(y) * z2;
    const int b = (l + kImuQ - 1) % kImuQ;
    const double dt = time[l] - time[b];
    if (dt < scanPeriod) {
      const float a3[3] = {ax, ay, az};
      for (int k = 0; k < 3; ++k) {
        v[IV_SX + k][l] = (float)(v[IV_SX + k][b] + v[IV_VX + k][b] * dt + a3[k] * dt * dt / 2);
        v[IV_VX + k][l] = (float)(v[IV_VX + k][b] + a3[k] * dt);
        v[IV_AX + k][l] = (float)(v[IV_AX + k][b] + angVelo[k][b] * dt);
      }
    }
  }

  // The queue as adjustDistortion of a scan stamped `stamp` sees it; then
  // the end of adjustDistortion (imuPointerLastIteration = imuPointerLast).
  // The reference starts the search at imuPointerLastIteration, which is -1
  // when the previous scan saw no message yet: it then reads imuTime[-1]
  // (undefined; SURVEY.md §9.7 policy) — restated as a zero slot, which any
  // scan time passes, i.e. the search starts at entry 0.
  void snapshot(double stamp, ImuSnap* o) {
    o->stamp = stamp;
    std::memcpy(o->time, time, sizeof(time));
    std::memcpy(o->v, v, sizeof(v));
    o->last = last;
    o->lastIter = lastIter < 0 ? 0 : lastIter;
    o->_pad[0] = o->_pad[1] = 0;
    lastIter = last;
  }
};

// mapOptimization's queue (:181-190, imuHandler :643-652) and the roll /
// pitch transformUpdate blends in (:465-490).  The front pointer persists.
struct MoImuQueue {
  int front = 0, last = -1;
  double time[kImuQ] = {};
  float roll[kImuQ] = {}, pitch[kImuQ] = {};

  void push(const lego_imu_msg& m) {
    double r, p, y;
    tf_get_rpy(m.orientation, &r, &p, &y);
    last = (last + 1) % kImuQ;
    time[last] = m.stamp;
    roll[last] = (float)r;
    pitch[last] = (float)p;
  }

  // imuRollLast / imuPitchLast at timeLaserOdometry + scanPeriod; *f = the
  // advanced front pointer (committed by the caller only when transformUpdate
  // ran, i.e. the scan-to-map guard passed).  False without a message.
  bool at(double tOdom, float scanPeriod, float* r, float* p, int* f) const {
    if (last < 0) return false;
    int k = front;
    while (k != last) {
      if (tOdom + scanPeriod < time[k]) break;
      k = (k + 1) % kImuQ;
    }
    *f = k;
    if (tOdom + scanPeriod > time[k]) {
      *r = roll[k];
      *p = pitch[k];
    } else {
      const int b = (k + kImuQ - 1) % kImuQ;
      const float rf = (float)((tOdom + scanPeriod - time[b]) / (time[k] - time[b]));
      const float rb = (float)((time[k] - tOdom - scanPeriod) / (time[k] - time[b]));
      *r = roll[k] * rf + roll[b] * rb;
      *p = pitch[k] * rf + pitch[b] * rb;
    }
    return true;
  }
};

}  // namespace lego
