// lego_odom.hip — the two-step LM odometry of featureAssociation on gfx950.
//
// k_odom walks a batch's scans in stream order (scan k's problem depends on
// scan k-1's result through transformCur and the TransformToEnd'ed "last"
// clouds, featureAssociation.cpp:1759-1815), so the per-scan chain never
// returns to the host.  One launch runs G workgroups of 512 threads per
// stream (24 for VLP-16, odom_workgroups); each runs the whole serial chain
// redundantly and they split only the correspondence searches, exchanging the
// results through tagged granules ("exchange" below).  Per LM iteration:
//   every 5th iteration: each workgroup searches its slice of the queries,
//     one wave (kGL = 64 lanes) per query:
//       - the exact nearest neighbour in the last cloud (replaces KdTreeFLANN,
//         :1054, :1165; ties -> lower index, FLANN's tie order is traversal
//         dependent): an exhaustive pass over the LDS cloud when a stream has
//         enough workgroups for about one query per wave (OdomBufs::gridless)
//         or the cloud is small, else a 0.5 m hash grid with provable
//         coverage, falling back to the exhaustive pass;
//       - the scan-line neighbours (:1062-1099, :1173-1220, incl. the
//         loop-bound quirk): the reference's sequential loops visit an index
//         window bounded by ring breaks; the window is read off per-ring
//         first/last tables, keeping the (distance, visit order) tie rule;
//     then publishes (i1, i2, i3) as one packed granule per query and reads
//     the other slices' granules;
//   one lane per query: line / plane residual, weight and Jacobian row
//     (:1106-1151, :1228-1321);
//   reduction of AtA, AtB with double accumulation (DPP row sums, one barrier);
//   every wave: 3x3 QR solve, iteration-0 eigen degeneracy projection, update,
//     NaN reset, convergence test (:1324-1376, :1425-1477).
// Then integrateTransformation (:1697-1725) and publishCloudsLast (ToEnd, swap,
// index rebuild).  For VLP-16-class sensors the last clouds, both NN indexes,
// the queries, correspondences and the state all live in LDS; the same code
// runs from per-workgroup HBM copies for larger sensors.  Every workgroup
// starts from a read-only copy of the stream state (OdomBufs::stIn) and only
// the lead workgroup writes the state back.
#include <climits>
#include <cstdint>
#include <type_traits>

#include "lego_device.h"
#include "lego_kernels.h"

namespace lego {

constexpr int kOdomThreads = 512;
constexpr int kOdomWaves = kOdomThreads / 64;
constexpr int kGL = 64;                       // lanes per query group (one wave)
constexpr int kNGrp = kOdomThreads / kGL;
// LDS residency caps (VLP-16 / OS1-16 fit; larger sensors use the HBM path)
constexpr int kLdsSurf = 4096;                // last surf cloud points
constexpr int kLdsCorner = 2048;              // last corner cloud points
constexpr int kLdsQ = 384;                    // queries (flat <= 24 N, sharp <= 12 N)
constexpr int kLdsGridS = 2048, kLdsGridC = 1024;  // fine-grid buckets
constexpr int kKeyTab = kMaxRings + 4;
constexpr int kLdsCnt = kLdsGridS + kLdsGridC;
constexpr float kCell = 0.5f;

// ---------------------------------------------------------------- transforms
struct Trig3 {
  float srx, crx, sry, cry, srz, crz;
};
__device__ __forceinline__ Trig3 trig3(float rx, float ry, float rz) {
  return {lego_sinf(rx), lego_cosf(rx), lego_sinf(ry), lego_cosf(ry), lego_sinf(rz), lego_cosf(rz)};
}

__device__ __forceinline__ float start_s(float4 pi) { return 10 * (pi.w - (float)(int)pi.w); }
// TransformToStart given the point's s and the six sines / cosines of s * tc[0..2]
__device__ __forceinline__ float4 to_start_t(float4 pi, float s, const float* tc, float cx, float sx, float cy,
                                             float sy, float cz, float sz) {
  const float tx = s * tc[3], ty = s * tc[4], tz = s * tc[5];
  const float x1 = cz * (pi.x - tx) + sz * (pi.y - ty);
  const float y1 = -sz * (pi.x - tx) + cz * (pi.y - ty);
  const float z1 = (pi.z - tz);
  const float x2 = x1;
  const float y2 = cx * y1 + sx * z1;
  const float z2 = -sx * y1 + cx * z1;
  return make_float4(cy * x2 - sy * z2, y2, sy * x2 + cy * z2, pi.w);
}
__device__ __forceinline__ float4 to_start(float4 pi, const float* tc) {  // :860-883
  const float s = start_s(pi);
  float cx, sx, cy, sy, cz, sz;
  lego_sincosf(s * tc[0], &sx, &cx);
  lego_sincosf(s * tc[1], &sy, &cy);
  lego_sincosf(s * tc[2], &sz, &cz);
  return to_start_t(pi, s, tc, cx, sx, cy, sy, cz, sz);
}
// One LM step moves only three of transformCur's components (surf: rx, rz,
// ty; corner: ry, tx, tz), so the sines / cosines of the other angles are the
// same in every iteration of the step.  A lane keeps them for its first query,
// keyed by the bits of the angle they were computed from.
struct FixTrig {
  float sa, ca, sb, cb;
  unsigned ka, kb;
  bool have;
};
__device__ __forceinline__ float4 to_start_fix(float4 pi, const float* tc, bool surf, FixTrig& f) {
  const float s = start_s(pi);
  if (surf) {  // ry fixed
    if (!f.have || __float_as_uint(tc[1]) != f.ka) {
      lego_sincosf(s * tc[1], &f.sa, &f.ca);
      f.ka = __float_as_uint(tc[1]);
      f.have = true;
    }
    float cx, sx, cz, sz;
    lego_sincosf(s * tc[0], &sx, &cx);
    lego_sincosf(s * tc[2], &sz, &cz);
    return to_start_t(pi, s, tc, cx, sx, f.ca, f.sa, cz, sz);
  }
  if (!f.have || __float_as_uint(tc[0]) != f.ka || __float_as_uint(tc[2]) != f.kb) {  // rx, rz fixed
    lego_sincosf(s * tc[0], &f.sa, &f.ca);
    f.ka = __float_as_uint(tc[0]);
    lego_sincosf(s * tc[2], &f.sb, &f.cb);
    f.kb = __float_as_uint(tc[2]);
    f.have = true;
  }
  float cy, sy;
  lego_sincosf(s * tc[1], &sy, &cy);
  return to_start_t(pi, s, tc, f.ca, f.sa, cy, sy, f.cb, f.sb);
}

// TransformToEnd :885-953 with the IMU terms of an IMU-less run
// (cos/sin of the zero IMU angles; imuShiftFromStart = 0).
struct ImuEnd {
  float cRS, cPS, cYS, sRS, sPS, sYS;  // cosImu*Start / sinImu*Start
  float cYL, sYL, cPL, sPL, cRL, sRL;  // imu*Last
};
// The second half of TransformToEnd rotates by the full transformCur: its
// sines and cosines are the same for every point, computed once per scan.
struct EndTrig {
  float cx, sx, cy, sy, cz, sz;
};
__device__ __forceinline__ EndTrig end_trig(const float* tc) {
  EndTrig e;
  lego_sincosf(tc[0], &e.sx, &e.cx);
  lego_sincosf(tc[1], &e.sy, &e.cy);
  lego_sincosf(tc[2], &e.sz, &e.cz);
  return e;
}
__device__ __forceinline__ float4 to_end_t(float4 pi, const float* tc, const EndTrig& et, const ImuEnd& im) {
  const float s = 10 * (pi.w - (float)(int)pi.w);
  float tx = s * tc[3], ty = s * tc[4], tz = s * tc[5];
  float cx, sx, cy, sy, cz, sz;
  lego_sincosf(s * tc[0], &sx, &cx);
  lego_sincosf(s * tc[1], &sy, &cy);
  lego_sincosf(s * tc[2], &sz, &cz);
  const float x1 = cz * (pi.x - tx) + sz * (pi.y - ty);
  const float y1 = -sz * (pi.x - tx) + cz * (pi.y - ty);
  const float z1 = (pi.z - tz);
  const float x2 = x1;
  const float y2 = cx * y1 + sx * z1;
  const float z2 = -sx * y1 + cx * z1;
  const float x3 = cy * x2 - sy * z2;
  const float y3 = y2;
  const float z3 = sy * x2 + cy * z2;
  tx = tc[3]; ty = tc[4]; tz = tc[5];
  cz = et.cz; sz = et.sz; cx = et.cx; sx = et.sx; cy = et.cy; sy = et.sy;
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

// The IMU terms of an IMU-less stream are cos 0 = 1 and sin 0 = 0: with them
// as literals the compiler drops only the exact identities (x * 1, x - 0), the
// same bits as the general expression.
__device__ __forceinline__ float4 to_end(float4 pi, const float* tc, const EndTrig& et, const ImuEnd& im, bool imu) {
  if (imu) return to_end_t(pi, tc, et, im);
  return to_end_t(pi, tc, et, ImuEnd{1.f, 1.f, 1.f, 0.f, 0.f, 0.f, 1.f, 0.f, 1.f, 0.f, 1.f, 0.f});
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

// integrateTransformation (:1697-1725) by one wave: the same expressions as
// accumulate_rotation / plugin_imu_rotation above, with their independent
// sines and cosines evaluated on separate lanes and broadcast by readlane, and
// the two atan2f of each step on two lanes.  bl / al: the IMU angles
// (imuPitchStart, imuYawStart, imuRollStart) / (imuPitchLast, imuYawLast,
// imuRollLast); all zero without an IMU.
__device__ __forceinline__ float rl_f(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ float sel6(int m, float a0, float a1, float a2, float a3, float a4, float a5) {
  return m == 0 ? a0 : m == 1 ? a1 : m == 2 ? a2 : m == 3 ? a3 : m == 4 ? a4 : a5;
}
__device__ __forceinline__ void integrate_wave(float* ts, const float* tc, const float bl[3], const float al[3]) {
  const int lane = threadIdx.x & 63;
  // accumulate_rotation(ts[0..2], -tc[0..2]): lanes 0-5 sin, 6-11 cos of {lx, ly, lz, cx, cy, cz};
  // plugin_imu_rotation's bl / al: lanes 12-17 sin, 18-23 cos
  float v = 0.f;
  if (lane < 12) {
    const float a = sel6(lane % 6, -tc[0], -tc[1], -tc[2], ts[0], ts[1], ts[2]);
    v = lane < 6 ? lego_sinf(a) : lego_cosf(a);
  } else if (lane < 24) {
    const float a = sel6(lane % 6, bl[0], bl[1], bl[2], al[0], al[1], al[2]);
    v = lane < 18 ? lego_sinf(a) : lego_cosf(a);
  }
  const float slx = rl_f(v, 0), sly = rl_f(v, 1), slz = rl_f(v, 2), scx = rl_f(v, 3), scy = rl_f(v, 4), scz = rl_f(v, 5);
  const float clx = rl_f(v, 6), cly = rl_f(v, 7), clz = rl_f(v, 8), ccx = rl_f(v, 9), ccy = rl_f(v, 10), ccz = rl_f(v, 11);
  const float srx = clx * ccx * sly * scz - ccx * ccz * slx - clx * cly * scx;
  const float ox = -lego_asinf(srx);
  const float cox = lego_cosf(ox);
  const float srycrx = slx * (ccy * scz - ccz * scx * scy) + clx * sly * (ccy * ccz + scx * scy * scz) +
                       clx * cly * ccx * scy;
  const float crycrx = clx * cly * ccx * ccy - clx * sly * (ccz * scy - ccy * scx * scz) -
                       slx * (scy * scz + ccy * ccz * scx);
  const float srzcrx = scx * (clz * sly - cly * slx * slz) + ccx * scz * (cly * clz + slx * sly * slz) +
                       clx * ccx * ccz * slz;
  const float crzcrx = clx * clz * ccx * ccz - ccx * scz * (cly * slz - clz * slx * sly) -
                       scx * (sly * slz + cly * clz * slx);
  const float at = lane == 0 ? lego_atan2f(srycrx / cox, crycrx / cox) : lego_atan2f(srzcrx / cox, crzcrx / cox);
  const float rx = ox, ry = rl_f(at, 0), rz = rl_f(at, 1);
  // sin / cos of the accumulated angles: the translation and plugin_imu_rotation's bc terms
  float w = 0.f;
  if (lane < 6) {
    const float a = sel6(lane % 3, rx, ry, rz, rx, ry, rz);
    w = lane < 3 ? lego_sinf(a) : lego_cosf(a);
  }
  const float sbcx = rl_f(w, 0), sbcy = rl_f(w, 1), sbcz = rl_f(w, 2);
  const float cbcx = rl_f(w, 3), cbcy = rl_f(w, 4), cbcz = rl_f(w, 5);
  const float x1 = cbcz * (tc[3] - 0.0f) - sbcz * (tc[4] - 0.0f);
  const float y1 = sbcz * (tc[3] - 0.0f) + cbcz * (tc[4] - 0.0f);
  const float z1 = tc[5] - 0.0f;
  const float x2 = x1;
  const float y2 = cbcx * y1 - sbcx * z1;
  const float z2 = sbcx * y1 + cbcx * z1;
  const float tx = ts[3] - (cbcy * x2 + sbcy * z2);
  const float ty = ts[4] - y2;
  const float tz = ts[5] - (-sbcy * x2 + cbcy * z2);
  // plugin_imu_rotation(rx, ry, rz, bl, al)
  const float sblx = rl_f(v, 12), sbly = rl_f(v, 13), sblz = rl_f(v, 14);
  const float salx = rl_f(v, 15), saly = rl_f(v, 16), salz = rl_f(v, 17);
  const float cblx = rl_f(v, 18), cbly = rl_f(v, 19), cblz = rl_f(v, 20);
  const float calx = rl_f(v, 21), caly = rl_f(v, 22), calz = rl_f(v, 23);
  const float psrx = -sbcx * (salx * sblx + calx * caly * cblx * cbly + calx * cblx * saly * sbly) -
                     cbcx * cbcz * (calx * saly * (cbly * sblz - cblz * sblx * sbly) -
                                    calx * caly * (sbly * sblz + cbly * cblz * sblx) + cblx * cblz * salx) -
                     cbcx * sbcz * (calx * caly * (cblz * sbly - cbly * sblx * sblz) -
                                    calx * saly * (cbly * cblz + sblx * sbly * sblz) + cblx * salx * sblz);
  const float acx = -lego_asinf(psrx);
  const float cacx = lego_cosf(acx);
  const float psrycrx = (cbcy * sbcz - cbcz * sbcx * sbcy) *
                            (calx * saly * (cbly * sblz - cblz * sblx * sbly) -
                             calx * caly * (sbly * sblz + cbly * cblz * sblx) + cblx * cblz * salx) -
                        (cbcy * cbcz + sbcx * sbcy * sbcz) *
                            (calx * caly * (cblz * sbly - cbly * sblx * sblz) -
                             calx * saly * (cbly * cblz + sblx * sbly * sblz) + cblx * salx * sblz) +
                        cbcx * sbcy * (salx * sblx + calx * caly * cblx * cbly + calx * cblx * saly * sbly);
  const float pcrycrx = (cbcz * sbcy - cbcy * sbcx * sbcz) *
                            (calx * caly * (cblz * sbly - cbly * sblx * sblz) -
                             calx * saly * (cbly * cblz + sblx * sbly * sblz) + cblx * salx * sblz) -
                        (sbcy * sbcz + cbcy * cbcz * sbcx) *
                            (calx * saly * (cbly * sblz - cblz * sblx * sbly) -
                             calx * caly * (sbly * sblz + cbly * cblz * sblx) + cblx * cblz * salx) +
                        cbcx * cbcy * (salx * sblx + calx * caly * cblx * cbly + calx * cblx * saly * sbly);
  const float psrzcrx = sbcx * (cblx * cbly * (calz * saly - caly * salx * salz) -
                                cblx * sbly * (caly * calz + salx * saly * salz) + calx * salz * sblx) -
                        cbcx * cbcz * ((caly * calz + salx * saly * salz) * (cbly * sblz - cblz * sblx * sbly) +
                                       (calz * saly - caly * salx * salz) * (sbly * sblz + cbly * cblz * sblx) -
                                       calx * cblx * cblz * salz) +
                        cbcx * sbcz * ((caly * calz + salx * saly * salz) * (cbly * cblz + sblx * sbly * sblz) +
                                       (calz * saly - caly * salx * salz) * (cblz * sbly - cbly * sblx * sblz) +
                                       calx * cblx * salz * sblz);
  const float pcrzcrx = sbcx * (cblx * sbly * (caly * salz - calz * salx * saly) -
                                cblx * cbly * (saly * salz + caly * calz * salx) + calx * calz * sblx) +
                        cbcx * cbcz * ((saly * salz + caly * calz * salx) * (sbly * sblz + cbly * cblz * sblx) +
                                       (caly * salz - calz * salx * saly) * (cbly * sblz - cblz * sblx * sbly) +
                                       calx * calz * cblx * cblz) -
                        cbcx * sbcz * ((saly * salz + caly * calz * salx) * (cblz * sbly - cbly * sblx * sblz) +
                                       (caly * salz - calz * salx * saly) * (cbly * cblz + sblx * sbly * sblz) -
                                       calx * calz * cblx * sblz);
  const float pt = lane == 0 ? lego_atan2f(psrycrx / cacx, pcrycrx / cacx) : lego_atan2f(psrzcrx / cacx, pcrzcrx / cacx);
  const float acy = rl_f(pt, 0), acz = rl_f(pt, 1);
  if (lane == 0) { ts[0] = acx; ts[1] = acy; ts[2] = acz; ts[3] = tx; ts[4] = ty; ts[5] = tz; }
}

// In-kernel phase stamps (diagnostic; enabled per launch).  Thread 0 adds
// wall_clock64 deltas (100 MHz) into prof[k].
enum { P_SURF_NN = 0, P_SURF = 1, P_CORN_NN = 2, P_CORN = 3, P_SOLVE = 4, P_INTEG = 5,
       P_TOEND = 6, P_BUILD = 7, P_RESID = 8, P_ITERS_S = 9, P_ITERS_C = 10, P_NNR = 11,
       P_QUERY = 12, P_SCANLINE = 13, P_NN_SHELL1 = 14, P_NN_BRUTE = 15,
       P_G0_TOSTART = 16, P_G0_NN = 17, P_G0_SCAN = 18, P_G0_Q = 19, P_AZLINE = 20,
       P_T_ROWS = 21, P_T_SOLVE0 = 22, P_T_SOLVE = 23, P_X_LOCAL = 24, P_TOEND_LOOP = 25,
       P_B_PASS1 = 26, P_B_SCAN = 27, P_B_SCATTER = 29, P_B_ENDS = 31,  // index-build sub-phases
       P_NPROF = 32 };
// ODOM_RESID_PROBE (diagnostic build, scripts/build_ab.sh): the stretches of a
// scan outside the stamped phases, on the build sub-phase slots (unused by the
// gridless C2 stream): 26 scan top -> first LM iteration, 27 the LM loops'
// prologues / epilogues, 29 the hand-off before its loop, 31 after it to the
// scan's end (includes P_BUILD)
#ifndef ODOM_RESID_PROBE
#define ODOM_RESID_PROBE 0
#endif
#define RP_START(S) do { if (ODOM_RESID_PROBE) (S).start(); } while (0)
#define RP_ADD(S, k) do { if (ODOM_RESID_PROBE) (S).add(k); } while (0)
struct Stamp {
  unsigned long long* prof;
  unsigned long long t;
  __device__ __forceinline__ void start() { if (prof && threadIdx.x == 0) t = wall_clock64(); }
  __device__ __forceinline__ void add(int k) {
    if (prof && threadIdx.x == 0) { const unsigned long long n = wall_clock64(); prof[k] += n - t; t = n; }
  }
  __device__ __forceinline__ void count(int k) { if (prof && threadIdx.x == 0) prof[k] += 1; }
};

// ---------------------------------------------------------------- NN index
// Fine grid over one last cloud: 0.5 m cells hashed into T buckets, built by
// counting sort (bucket array = END offsets into a point-order array, begin =
// the previous bucket's end; order inside a bucket is arbitrary, every search
// keeps a lexicographic minimum).  Plus per-key first/last tables, key =
// int(intensity), the ring the scan-line loops test.
template <class Idx>
struct NNView {
  const float4* pts;
  int n;
  const Idx* gEnd;
  const Idx* gOrd;     // LDS grids: point order
  const float4* gPts;  // HBM grids: the points themselves in bucket order (.w = index bits)
  int T, NK;
  const int* sufFirst;  // [NK + 1] first index whose key >= k (INT_MAX if none)
  const int* preLast;   // [NK]     last index whose key <= k (-1 if none)
  int irregular;        // a key outside [0, NK): tables unusable
  int gridless;         // no grid (OdomBufs::gridless): exhaustive closest-point search
};

template <class Idx>
struct NNStore {
  Idx *gEnd, *gOrd;
  float4* gPts;
  int *sufFirst, *preLast, *irregular;
  int Tcap;
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
__device__ __forceinline__ int fine_bucket(int ix, int iy, int iz, int T) {
  return (int)(hash_key(cell_key(ix, iy, iz)) & (unsigned)(T - 1));
}
__host__ __device__ inline int fine_T(int n, int cap) {
  int t = 64;
  while (t < n / 2 && t < cap) t <<= 1;
  return t;
}

// exclusive scan of a[0..n) in place, all threads of the block
__device__ __forceinline__ void block_exscan(unsigned* a, int n, int* wtot) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int per = (n + kOdomThreads - 1) / kOdomThreads;
  const int b0 = min(n, tid * per), b1 = min(n, b0 + per);
  unsigned local = 0;
  for (int t = b0; t < b1; ++t) local += a[t];
  unsigned x = local;
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) wtot[wave] = (int)x;
  __syncthreads();
  unsigned run = x - local;
  for (int w = 0; w < wave; ++w) run += (unsigned)wtot[w];
  for (int t = b0; t < b1; ++t) {
    const unsigned cnt = a[t];
    a[t] = run;
    run += cnt;
  }
  __syncthreads();
}

// Builds both clouds' fine grids and key tables in shared passes (all
// threads; half the barriers of two builds): ptsS[0..nS) then ptsC[0..nC) as
// one index range, surf buckets [0, TS) then corner buckets [TS, TS + TC) in
// one counter array (>= TS + TC entries), kfirst / klast [2 * NK].  Three
// phases: build_zero, build_count (per wave chunk of 64 consecutive indices;
// the hand-off runs it on the points TransformToEnd has just produced, so the
// clouds are not read back for it) and build_finish.
template <class Idx>
struct BuildArgs {
  const float4 *ptsS, *ptsC;
  int nS, nC, TS, TC, NK;
  NNStore<Idx> S, Cs;
  unsigned* cnt;
  int *wtot, *kfirst, *klast;
  int gridless;  // key tables only (OdomBufs::gridless)
};
template <class Idx>
__device__ __forceinline__ BuildArgs<Idx> build_args(const float4* ptsS, int nS, const NNStore<Idx>& S,
                                                     const float4* ptsC, int nC, const NNStore<Idx>& Cs, int NK,
                                                     unsigned* cnt, int* wtot, int* kfirst, int* klast,
                                                     int gridless = 0) {
  return BuildArgs<Idx>{ptsS, ptsC, nS, nC, fine_T(nS, S.Tcap), fine_T(nC, Cs.Tcap), NK, S, Cs,
                        cnt, wtot, kfirst, klast, gridless};
}
// zeroes the counters and key tables (all threads; the caller's barrier follows)
template <class Idx>
__device__ __forceinline__ void build_zero(const BuildArgs<Idx>& B) {
  const int tid = threadIdx.x;
  if (!B.gridless)
    for (int b = tid; b < B.TS + B.TC; b += kOdomThreads) B.cnt[b] = 0;
  for (int k = tid; k < 2 * B.NK; k += kOdomThreads) { B.kfirst[k] = INT_MAX; B.klast[k] = -1; }
  if (tid == 0) { *B.S.irregular = 0; *B.Cs.irregular = 0; }
}
// The keys of index i's neighbours in its cloud: kp of i - 1 (INT_MIN at the
// cloud's start), kn of i + 1 (INT_MAX at its end), from the .w words wp of
// point i - 1 and wn of point i + 1 (loaded beside point i itself, so the
// chunk waits for one load latency).
__device__ __forceinline__ void nbr_keys(int i, int nS, int n, float wp, float wn, int& kp, int& kn) {
  kp = i == 0 || i == nS ? INT_MIN : (int)wp;
  kn = i == nS - 1 || i == n - 1 ? INT_MAX : (int)wn;
}
// counts the wave's chunk [i0, i0 + 64) of the combined index range; lane
// i0 + lane holds point p (ignored past nS + nC) and its neighbours' keys
// (nbr_keys).  The clouds come ring after ring, so a key's first / last index
// is where the key changes: one plain store per run.  A key that decreases
// along a cloud marks the cloud irregular (the searches then use the literal
// scan-line loop), as does a key outside [0, NK).
template <class Idx>
__device__ __forceinline__ void build_count(const BuildArgs<Idx>& B, int i0, float4 p, int kp, int kn,
                                            bool active = true) {
  const int lane = threadIdx.x & 63, i = i0 + lane, n = B.nS + B.nC;
  if (i < n && active) {
    const bool corner = i >= B.nS;
    const int T = corner ? B.TC : B.TS;
    if (!B.gridless)
      atomicAdd(&B.cnt[(corner ? B.TS : 0) + fine_bucket(cell_of(p.x), cell_of(p.y), cell_of(p.z), T)], 1u);
    const int k = (int)p.w;
    if (k < 0 || k >= B.NK || kp > k) {
      *(corner ? B.Cs.irregular : B.S.irregular) = 1;
    } else {
      const int kk = k + (corner ? B.NK : 0), j = i - (corner ? B.nS : 0);
      if (kp != k) B.kfirst[kk] = j;
      if (kn != k) B.klast[kk] = j;
    }
  }
}
// key tables, bucket starts, scatter, bucket ends (all threads, after a
// barrier that follows the last build_count)
template <class Idx>
__device__ __forceinline__ void build_finish(const BuildArgs<Idx>& B, unsigned long long* prof) {
  const int tid = threadIdx.x;
  const int nS = B.nS, TS = B.TS, TC = B.TC, NK = B.NK, n = B.nS + B.nC;
  const NNStore<Idx>& S = B.S;
  const NNStore<Idx>& Cs = B.Cs;
  unsigned* cnt = B.cnt;
  unsigned long long tp = (prof && tid == 0) ? wall_clock64() : 0;
  auto stamp = [&](int k) {
    if (prof && tid == 0) { const unsigned long long t = wall_clock64(); prof[k] += t - tp; tp = t; }
  };
  // suffix-min of first / prefix-max of last, one thread per (cloud, key)
  for (int t = tid; t < 2 * NK; t += kOdomThreads) {
    const int c0 = t >= NK ? NK : 0, k = t - c0;
    int m = INT_MAX, M = -1;
    for (int j = k; j < NK; ++j) m = min(m, B.kfirst[c0 + j]);
    for (int j = 0; j <= k; ++j) M = max(M, B.klast[c0 + j]);
    (c0 ? Cs : S).sufFirst[k] = m;
    (c0 ? Cs : S).preLast[k] = M;
  }
  if (tid == 0) { S.sufFirst[NK] = INT_MAX; Cs.sufFirst[NK] = INT_MAX; }
  if (B.gridless) {
    __syncthreads();
    return;
  }
  block_exscan(cnt, TS + TC, B.wtot);  // corner starts come out offset by nS
  stamp(P_B_SCAN);
  constexpr int kBuildU = 8;  // points per lane in flight
  for (int j = tid; j < n; j += kBuildU * kOdomThreads) {
    float4 pu[kBuildU];
#pragma unroll
    for (int u = 0; u < kBuildU; ++u) {
      const int i = j + u * kOdomThreads;
      if (i < n) pu[u] = i >= nS ? B.ptsC[i - nS] : B.ptsS[i];
    }
#pragma unroll
    for (int u = 0; u < kBuildU; ++u) {
      const int i = j + u * kOdomThreads;
      if (i >= n) break;
      const bool corner = i >= nS;
      const float4 p = pu[u];
      const int T = corner ? TC : TS;
      const unsigned pos =
          atomicAdd(&cnt[(corner ? TS : 0) + fine_bucket(cell_of(p.x), cell_of(p.y), cell_of(p.z), T)], 1u);
      if constexpr (std::is_same<Idx, uint32_t>::value) {  // HBM grids: the point itself, one load per visit
        if (corner) Cs.gPts[pos - nS] = make_float4(p.x, p.y, p.z, __int_as_float(i - nS));
        else S.gPts[pos] = make_float4(p.x, p.y, p.z, __int_as_float(i));
      } else {
        if (corner) Cs.gOrd[pos - nS] = (Idx)(i - nS);
        else S.gOrd[pos] = (Idx)i;
      }
    }
  }
  __syncthreads();
  stamp(P_B_SCATTER);
  for (int b = tid; b < TS + TC; b += kOdomThreads) {
    if (b < TS) S.gEnd[b] = (Idx)cnt[b];
    else Cs.gEnd[b - TS] = (Idx)(cnt[b] - nS);
  }
  __syncthreads();
  stamp(P_B_ENDS);
}
template <class Idx>
__device__ __forceinline__ void nn_build2(const BuildArgs<Idx>& B, unsigned long long* prof = nullptr) {
  const int tid = threadIdx.x, lane = tid & 63, n = B.nS + B.nC;
  const unsigned long long tp = (prof && tid == 0) ? wall_clock64() : 0;
  build_zero(B);
  __syncthreads();
  constexpr int kBuildU = 4;  // points per lane in flight
  for (int j0 = tid - lane; j0 < n; j0 += kBuildU * kOdomThreads) {  // wave-uniform loop
    float4 pu[kBuildU];
#pragma unroll
    for (int u = 0; u < kBuildU; ++u) {
      const int i = j0 + u * kOdomThreads + lane;
      if (i < n) pu[u] = i >= B.nS ? B.ptsC[i - B.nS] : B.ptsS[i];
    }
    auto w_at = [&](int j) { return j >= B.nS ? B.ptsC[j - B.nS].w : B.ptsS[j].w; };
#pragma unroll
    for (int u = 0; u < kBuildU; ++u) {
      const int i0 = j0 + u * kOdomThreads, i = i0 + lane;
      if (i0 >= n) break;
      int kp = 0, kn = 0;
      if (i < n) nbr_keys(i, B.nS, n, w_at(max(i - 1, 0)), w_at(min(i + 1, n - 1)), kp, kn);
      build_count(B, i0, pu[u], kp, kn);
    }
  }
  __syncthreads();
  if (prof && tid == 0) prof[P_B_PASS1] += wall_clock64() - tp;
  build_finish(B, prof);
}

template <class Idx>
__device__ __forceinline__ void bucket_range(const Idx* E, int b, int& lo, int& hi) {
  lo = b ? (int)E[b - 1] : 0;
  hi = (int)E[b];
}

// L2_Simple distance order ((0 + d0^2) + d1^2) + d2^2 (FLANN)
__device__ __forceinline__ float flann_d2(float4 q, float4 p) {
  float r = 0.f, d;
  d = q.x - p.x; r += d * d;
  d = q.y - p.y; r += d * d;
  d = q.z - p.z; r += d * d;
  return r;
}
__device__ __forceinline__ float line_d2(float4 a, float4 s) {  // the scan-line distance
  return (a.x - s.x) * (a.x - s.x) + (a.y - s.y) * (a.y - s.y) + (a.z - s.z) * (a.z - s.z);
}

__device__ __forceinline__ void lex_min(float& d, int& i, float d2, int i2) {
  if (d2 < d || (d2 == d && i2 < i)) { d = d2; i = i2; }
}
// Wave-wide lexicographic minima through DPP lane moves (VALU, no LDS):
// quad swaps, half-row and row mirrors leave every lane its 16-lane row
// minimum; the four row minima are then combined from readlanes.  The
// order is a total one (ties broken by the second key), so the result does not
// depend on the pairing.
template <int kCtrl>
__device__ __forceinline__ float dpp_f32(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), kCtrl, 0xf, 0xf, false));
}
template <int kCtrl>
__device__ __forceinline__ int dpp_i32(int v) {
  return __builtin_amdgcn_mov_dpp(v, kCtrl, 0xf, 0xf, false);
}
// Wave minima through DPP lane moves: quad swaps, half-row and row mirrors
// leave every lane its row's minimum, four readlanes combine the rows.
__device__ __forceinline__ float wave_min_f32(float v) {
  v = fminf(v, dpp_f32<0xB1>(v));
  v = fminf(v, dpp_f32<0x4E>(v));
  v = fminf(v, dpp_f32<0x141>(v));
  v = fminf(v, dpp_f32<0x140>(v));
  const float a = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
  const float b = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16));
  const float c = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
  const float e = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48));
  return fminf(fminf(a, b), fminf(c, e));
}
__device__ __forceinline__ int wave_min_i32(int v) {
  v = min(v, dpp_i32<0xB1>(v));
  v = min(v, dpp_i32<0x4E>(v));
  v = min(v, dpp_i32<0x141>(v));
  v = min(v, dpp_i32<0x140>(v));
  return min(min(__builtin_amdgcn_readlane(v, 0), __builtin_amdgcn_readlane(v, 16)),
             min(__builtin_amdgcn_readlane(v, 32), __builtin_amdgcn_readlane(v, 48)));
}
// Lexicographic (distance, second key) minimum over the wave in two plain
// minima: the smallest distance (distances are finite and >= 0), then the
// smallest second key among the lanes that hold it.  The order is a total
// one, so this equals any pairwise lexicographic reduction.
__device__ __forceinline__ void group_lex_min(float& d, int& i) {
  static_assert(kGL == 64, "DPP reductions span one wave");
  const float dm = wave_min_f32(d);
  i = wave_min_i32(d == dm ? i : INT_MAX);
  d = dm;
}
// (distance, visit rank) minimum carrying the index of the lane that holds it
// (ranks are distinct among candidates; without one every lane holds j = -1)
__device__ __forceinline__ void group_lex_min3(float& d, int& r, int& j) {
  const float dm = wave_min_f32(d);
  const int rm = wave_min_i32(d == dm ? r : INT_MAX);
  const int owner = __ffsll((long long)__ballot(d == dm && r == rm)) - 1;
  j = __builtin_amdgcn_readlane(j, owner);
  d = dm;
  r = rm;
}

constexpr int kBruteSmall = 4 * kGL;
// Exact nearest neighbour with d2 < bound over pts[0, n), by the calling wave.
// A lane visits ascending indices, so a strict < keeps its lexicographic
// (distance, index) minimum; the group reduction breaks ties by index.
__device__ __forceinline__ int nn_brute(const float4* pts, int n, float4 q, float bound, int g) {
  float bd = bound;
  int bi = INT_MAX;
#pragma unroll 4
  for (int j = g; j < n; j += kGL) {
    const float d2 = flann_d2(q, pts[j]);
    if (d2 < bd) { bd = d2; bi = j; }
  }
  group_lex_min(bd, bi);
  return (bi != INT_MAX && bd < bound) ? bi : -1;
}

// Exact nearest neighbour with d2 < bound, by the calling wave: the fine
// grid's 27 cells (accepted when the best distance is provably below the one
// cell they cover), else every point (nn_brute, which covers the cells' points
// too).  Going to nn_brute directly for a query that fell back in the previous
// NN round measured 1.5% slower: the fallback is VALU-bound and its waves then
// contend for the SIMDs with the shell searches' latency-bound waves.
template <class Idx>
__device__ __forceinline__ int nn_i1(const NNView<Idx>& v, float4 q, float bound, int g, unsigned long long* prof) {
  if (v.n <= 0) return -1;
  // a small cloud (the corner clouds: ~100-200 points) is searched whole:
  // four points per lane cost less than the bucket lookups the shell needs
  if (v.n <= kBruteSmall || v.gridless) return nn_brute(v.pts, v.n, q, bound, g);
  float bd = bound;
  int bi = INT_MAX;
  const int cx = cell_of(q.x), cy = cell_of(q.y), cz = cell_of(q.z);
  if (g < 54) {  // two lanes per cell, alternate points of the bucket
    const int cc = g % 27, half = g / 27;
    int lo, hi;
    bucket_range(v.gEnd, fine_bucket(cx + cc % 3 - 1, cy + (cc / 3) % 3 - 1, cz + cc / 9 - 1, v.T), lo, hi);
    if constexpr (std::is_same<Idx, uint32_t>::value) {
#pragma unroll 2
      for (int t = lo + half; t < hi; t += 2) {
        const float4 p = v.gPts[t];
        lex_min(bd, bi, flann_d2(q, p), __float_as_int(p.w));
      }
    } else {
#pragma unroll 2
      for (int t = lo + half; t < hi; t += 2) {
        const int j = (int)v.gOrd[t];
        lex_min(bd, bi, flann_d2(q, v.pts[j]), j);
      }
    }
  }
  group_lex_min(bd, bi);
  if (bd < kCell * kCell * 0.99999f) {
    if (prof && g == 0) atomicAdd(&prof[P_NN_SHELL1], 1ull);
    return (bi != INT_MAX && bd < bound) ? bi : -1;
  }
  if (prof && g == 0) atomicAdd(&prof[P_NN_BRUTE], 1ull);
  return nn_brute(v.pts, v.n, q, bound, g);
}

// Scan-line neighbours of closest point ci (corner :1062-1099, surf
// :1173-1220), by the calling wave.  The forward loop visits
// (ci, min(F, jend)) where F is the first index after ci whose key exceeds
// cScan + 2 (int(I) > cScan + 2.5); the backward loop visits (B, ci) where B is
// the last index before ci whose key is below cScan - 2.  With the key tables
// F and B are known up front (when the keys are ordered enough for that to be
// exact; otherwise false: the caller runs the loops literally), so the window
// is scanned with independent contiguous loads.  Every point in it is classed
// by its key and side exactly as the loops do; their strict < keeps the first
// visited among equal distances, i.e. the smallest visit rank.
template <class Idx>
__device__ __forceinline__ bool nn_lines(const NNView<Idx>& v, int ci, int jend, float4 sel, bool surf, float nn_sq,
                                         int g, int* o2, int* o3) {
  if (v.irregular) return false;
  const int cScan = (int)v.pts[ci].w;
  const int F = (cScan + 3 <= v.NK) ? v.sufFirst[cScan + 3] : INT_MAX;
  const int B = (cScan - 3 >= 0) ? v.preLast[cScan - 3] : -1;
  if (F <= ci || B >= ci) return false;
  const int fwdEnd = min(F, jend);
  float m2 = nn_sq, m3 = nn_sq;
  int r2 = INT_MAX, r3 = INT_MAX, i2 = -1, i3 = -1;
  auto visit = [&](int j, bool fwd) {
    const float4 p = v.pts[j];
    const int kj = (int)p.w;
    bool cls2 = true;
    if (surf) cls2 = fwd ? (kj <= cScan) : (kj >= cScan);
    else if (fwd ? kj <= cScan : kj >= cScan) return;
    const float d = line_d2(p, sel);
    if (!(d < nn_sq)) return;
    const int rank = fwd ? j - ci : (jend - ci) + (ci - j);
    // selects, not a branch between the two minima (keeps them in registers)
    const bool u2 = cls2 && (d < m2 || (d == m2 && rank < r2));
    const bool u3 = !cls2 && (d < m3 || (d == m3 && rank < r3));
    m2 = u2 ? d : m2; r2 = u2 ? rank : r2; i2 = u2 ? j : i2;
    m3 = u3 ? d : m3; r3 = u3 ? rank : r3; i3 = u3 ? j : i3;
  };
#pragma unroll 2
  for (int j = ci + 1 + g; j < fwdEnd; j += kGL) visit(j, true);
#pragma unroll 4
  for (int j = B + 1 + g; j < ci; j += kGL) visit(j, false);
  group_lex_min3(m2, r2, i2);
  if (surf) group_lex_min3(m3, r3, i3);
  *o2 = i2;
  *o3 = surf ? i3 : -1;
  return true;
}


// Corner query against a small cloud (<= kBruteSmall points, ordered keys):
// the closest point and the scan-line neighbour from the same four points per
// lane, loaded once (nn_brute + nn_lines without reloading the window).  The
// candidates, their classes and visit ranks are nn_lines' exactly, and the
// lexicographic minima do not depend on which lane visits what.  Returns i1;
// *o2 the neighbour, *ok false when the key tables cannot bound the loops
// (the caller then runs them literally).
template <class Idx>
__device__ __forceinline__ int nn_corner_small(const NNView<Idx>& v, int jend, float4 sel, float bound,
                                               float nn_sq, int g, int* o2, bool* ok) {
  float4 p[4];
  float bd = bound;
  int bi = INT_MAX;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int j = g + k * kGL;
    p[k] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (j < v.n) {
      p[k] = v.pts[j];
      const float d2 = flann_d2(sel, p[k]);
      if (d2 < bd) { bd = d2; bi = j; }
    }
  }
  group_lex_min(bd, bi);
  *o2 = -1;
  *ok = true;
  if (bi == INT_MAX || !(bd < bound)) return -1;
  const int ci = bi;
  const int kc = ci / kGL;  // wave-uniform
  const float wc = kc == 0 ? p[0].w : (kc == 1 ? p[1].w : (kc == 2 ? p[2].w : p[3].w));
  const int cScan = (int)__int_as_float(__builtin_amdgcn_readlane(__float_as_int(wc), ci % kGL));
  const int F = (cScan + 3 <= v.NK) ? v.sufFirst[cScan + 3] : INT_MAX;
  const int B = (cScan - 3 >= 0) ? v.preLast[cScan - 3] : -1;
  if (F <= ci || B >= ci) {
    *ok = false;
    return ci;
  }
  const int fwdEnd = min(F, jend);
  float m2 = nn_sq;
  int r2 = INT_MAX, i2 = -1;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int j = g + k * kGL;
    const bool fwd = j > ci && j < fwdEnd, bwd = j > B && j < ci;
    const int kj = (int)p[k].w;
    if ((fwd && kj > cScan) || (bwd && kj < cScan)) {
      const float d = line_d2(p[k], sel);
      const int rank = fwd ? j - ci : (jend - ci) + (ci - j);
      const bool u = d < nn_sq && (d < m2 || (d == m2 && rank < r2));
      m2 = u ? d : m2; r2 = u ? rank : r2; i2 = u ? j : i2;
    }
  }
  group_lex_min3(m2, r2, i2);
  *o2 = i2;
  return ci;
}

// The reference's sequential loops, kGL indices per step (fallback).  Every
// lane keeps a lexicographic (distance, visit rank) minimum over the indices
// it visits and one group reduction combines them.
// int(I) > cScan + 2.5 <=> int(I) > cScan + 2 (and < cScan - 2.5 <=> < cScan - 2).
__device__ __forceinline__ void scanline_group(const float4* last, int jend, int ci, float4 sel, bool surf,
                                               float nn_sq, int g, int* o2, int* o3) {
  const int cScan = (int)last[ci].w;
  float m2 = nn_sq, m3 = nn_sq;
  int r2 = INT_MAX, r3 = INT_MAX, i2 = -1, i3 = -1;
  for (int j0 = ci + 1; j0 < jend; j0 += kGL) {
    const int j = j0 + g;
    const bool inr = j < jend;
    float4 p = make_float4(0, 0, 0, 0);
    int rj = 0;
    if (inr) { p = last[j]; rj = (int)p.w; }
    const unsigned long long bm = __ballot(inr && rj > cScan + 2);
    const int lim = bm ? (__ffsll((long long)bm) - 1) : kGL;
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
  for (int j0 = ci - 1; j0 >= 0; j0 -= kGL) {
    const int j = j0 - g;
    const bool inr = j >= 0;
    float4 p = make_float4(0, 0, 0, 0);
    int rj = 0;
    if (inr) { p = last[j]; rj = (int)p.w; }
    const unsigned long long bm = __ballot(inr && rj < cScan - 2);
    const int lim = bm ? (__ffsll((long long)bm) - 1) : kGL;
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

// Picks one of two buffers without indexing the kernel-argument struct (a
// dynamic index would move the struct to scratch memory).
__device__ __forceinline__ float4* buf2(float4* const (&a)[2], int k) { return k ? a[1] : a[0]; }

// ---------------------------------------------------------------- LDS layout
struct SolveWs {  // thread-0 solver workspace (dynamically indexed by the Jacobi sweep)
  float A[3][3], W[3], V[3][3], V2[3][3], Vi[3][3];
  int indR[3], indC[3];
};

struct OdomLds {
  float4* lastS;     // [kLdsSurf]
  float4* lastC;     // [kLdsCorner]
  int* qi;           // [3 * kLdsQ] correspondence indices
  float4* qflat;     // [2][kLdsQ]      flat features (LM queries): scan k in buffer k & 1
  float4* qsharp;    // [2][kLdsQ / 2]  sharp features
  unsigned* cnt;     // [kLdsGridS] index-build counters
  uint16_t *gEndS, *gOrdS, *gEndC, *gOrdC;  // fine grids
  int *sufS, *preS, *sufC, *preC;           // [kKeyTab] per-key first / last
  int *kfirst, *klast;                      // [2 * kMaxRings] build scratch
  double* red;       // [2][kOdomWaves * 4 * 10] reduction row partials (iteration parity)
  SolveWs* sw;
  int* wtot;         // [kOdomWaves]
  int* n;            // [16] flags
  OdomState* st;     // the stream state, resident for the kernel's lifetime
};
enum { N_BREAK = 0, N_IRR_S = 1, N_IRR_C = 2, N_ROUND = 3, N_RING = 4, N_CLAIM = 5,
       N_NEXT = 8, N_PRE = 12, N_LF = 13 };  // [8, 12): the next scan's f_cnt, prefetched; N_PRE: it and its queries are

__host__ __device__ constexpr size_t odom_lds_bytes() {
  size_t s = 0;
  s += (size_t)kLdsSurf * 16 + (size_t)kLdsCorner * 16 + (size_t)kLdsCnt * 4 + (size_t)3 * kLdsQ * 4;
  s += 2 * ((size_t)kLdsQ * 16 + (size_t)(kLdsQ / 2) * 16);
  s += (size_t)(kLdsGridS + kLdsSurf + kLdsGridC + kLdsCorner) * 2;
  s += (size_t)4 * kKeyTab * 4 + (size_t)4 * kMaxRings * 4;
  s += (size_t)2 * kOdomWaves * 4 * 10 * 8 + 256 + (size_t)kOdomWaves * 4 + 16 * 4 + 128;
  return s;
}

static_assert(odom_lds_bytes() + 32 * 8 <= 160 * 1024, "odometry LDS (+ the stamp accumulators) fits one CU");

__device__ __forceinline__ OdomLds odom_carve(unsigned char* base) {
  OdomLds L;
  size_t o = 0;
  L.lastS = (float4*)(base + o); o += (size_t)kLdsSurf * 16;
  L.lastC = (float4*)(base + o); o += (size_t)kLdsCorner * 16;
  L.qflat = (float4*)(base + o); o += (size_t)2 * kLdsQ * 16;
  L.qsharp = (float4*)(base + o); o += (size_t)2 * (kLdsQ / 2) * 16;
  L.cnt = (unsigned*)(base + o); o += (size_t)kLdsCnt * 4;
  L.qi = (int*)(base + o); o += (size_t)3 * kLdsQ * 4;
  L.red = (double*)(base + o); o += (size_t)2 * kOdomWaves * 4 * 10 * 8;
  L.sw = (SolveWs*)(base + o); o += 256;
  L.gEndS = (uint16_t*)(base + o); o += (size_t)kLdsGridS * 2;
  L.gOrdS = (uint16_t*)(base + o); o += (size_t)kLdsSurf * 2;
  L.gEndC = (uint16_t*)(base + o); o += (size_t)kLdsGridC * 2;
  L.gOrdC = (uint16_t*)(base + o); o += (size_t)kLdsCorner * 2;
  L.sufS = (int*)(base + o); o += (size_t)kKeyTab * 4;
  L.preS = (int*)(base + o); o += (size_t)kKeyTab * 4;
  L.sufC = (int*)(base + o); o += (size_t)kKeyTab * 4;
  L.preC = (int*)(base + o); o += (size_t)kKeyTab * 4;
  L.kfirst = (int*)(base + o); o += (size_t)2 * kMaxRings * 4;
  L.klast = (int*)(base + o); o += (size_t)2 * kMaxRings * 4;
  L.wtot = (int*)(base + o); o += (size_t)kOdomWaves * 4;
  L.n = (int*)(base + o); o += 16 * 4;
  L.st = (OdomState*)(base + o); o += 128;
  return L;
}

// The VLP-16-class configuration whose whole working set fits LDS.
__device__ __forceinline__ bool sensor_resident(const DevCfg& c) {
  return c.N * kFlatPerRing <= kLdsQ && c.N * kSharpPerRing <= kLdsQ / 2;
}

// Views of the current indexes (valid when the snapshot is current).
__device__ __forceinline__ NNView<uint16_t> view_lds(bool surf, const OdomLds& L, const OdomState* st, const DevCfg& c,
                                                    int gridless) {
  if (surf)
    return NNView<uint16_t>{L.lastS, st->surfLastNum, L.gEndS, L.gOrdS, nullptr, fine_T(st->surfLastNum, kLdsGridS),
                            c.N, L.sufS, L.preS, L.n[N_IRR_S], gridless};
  return NNView<uint16_t>{L.lastC, st->cornerLastNum, L.gEndC, L.gOrdC, nullptr, fine_T(st->cornerLastNum, kLdsGridC),
                          c.N, L.sufC, L.preC, L.n[N_IRR_C], gridless};
}
// A stream's ring slot (OdomBufs::ring; the protocol under "ring" below).
struct RingSlot {
  unsigned *claimA, *doneA, *claimB, *doneB;  // [G] each
  int* key;        // [kRingKey]: first (max of INT_MAX - j), last (max of j + 1) per (cloud, key), irregular x 2
  unsigned* cnt;   // [TS + TC] bucket counts
  unsigned* fill;  // [TS + TC] scatter cursors
  float4* P;       // [capH] less-flat [0, nS) then less-sharp [nS, nS + nC), TransformToEnd'ed
  float4* Q;       // [capH] the same in bucket order (corner buckets after nS), .w = index in its cloud
};
__device__ __forceinline__ RingSlot ring_slot(const OdomBufs& ob, int slot) {
  unsigned char* b = ob.ring + (size_t)slot * ob.ringStride;
  RingSlot r;
  r.claimA = (unsigned*)b;
  r.doneA = r.claimA + ob.G;
  r.claimB = r.doneA + ob.G;
  r.doneB = r.claimB + ob.G;
  b += ring_al((size_t)16 * ob.G);
  r.key = (int*)b;
  b += ring_al((size_t)4 * kRingKey);
  r.cnt = (unsigned*)b;
  b += ring_al((size_t)4 * (ob.gTS + ob.gTC));
  r.fill = (unsigned*)b;
  b += ring_al((size_t)4 * (ob.gTS + ob.gTC));
  r.P = (float4*)b;
  b += ring_al((size_t)16 * ob.capH);
  r.Q = (float4*)b;
  return r;
}
// The HBM copy `buf` of a last cloud (curBuf / snapBuf encoding, OdomState):
// a private buffer, or the ring slot's P (the corner cloud after nSurf points).
template <bool RING>
__device__ __forceinline__ const float4* hbm_cloud(const OdomBufs& ob, int buf, bool surf, int nSurf) {
  if (RING && buf >= 2) {
    const float4* P = ring_slot(ob, buf - 2).P;
    return surf ? P : P + nSurf;
  }
  return surf ? buf2(ob.surfLast, buf) : buf2(ob.cornerLast, buf);
}
// HBM-resident clouds: the LDS that holds the clouds, queries and counters of
// the resident layout (lastS .. cnt, contiguous) is free, and takes both
// grids' bucket arrays (the counting sort's counters, which end the build as
// the bucket ends); the point-order arrays stay in HBM.
constexpr int kHbmLdsCnt = (kLdsSurf * 16 + kLdsCorner * 16 + kLdsQ * 16 + (kLdsQ / 2) * 16 + kLdsCnt * 4) / 4;
__device__ __forceinline__ unsigned* hbm_grid_ends(const OdomLds& L) { return (unsigned*)L.lastS; }
template <bool RING>
__device__ __forceinline__ NNView<uint32_t> view_hbm(bool surf, const OdomLds& L, const OdomBufs& ob,
                                                     const OdomState* st, const DevCfg& c) {
  unsigned* ends = hbm_grid_ends(L);
  const int TS = fine_T(st->surfLastNum, ob.gTS);
  const float4* last = hbm_cloud<RING>(ob, st->curBuf, surf, st->surfLastNum);
  const float4* gq = nullptr;
  if (RING && st->curBuf >= 2) {  // the stream's ring slot: Q holds both clouds, corner after the surf points
    const float4* Q = ring_slot(ob, st->curBuf - 2).Q;
    gq = surf ? Q : Q + st->surfLastNum;
  } else {
    gq = surf ? ob.nS.gPts : ob.nC.gPts;
  }
  if (surf)
    return NNView<uint32_t>{last, st->surfLastNum, ends, nullptr, gq, TS, c.N, L.sufS, L.preS, L.n[N_IRR_S], 0};
  return NNView<uint32_t>{last, st->cornerLastNum, ends + TS, nullptr, gq, fine_T(st->cornerLastNum, ob.gTC), c.N,
                          L.sufC, L.preC, L.n[N_IRR_C], 0};
}

// The build arguments of both clouds' indexes over the current last clouds
// (st->curBuf, st->*LastNum) in the layout `resident` selects.
__device__ __forceinline__ BuildArgs<uint16_t> lds_build_args(const OdomLds& L, const OdomState* st,
                                                              const DevCfg& c, int gridless) {
  NNStore<uint16_t> sS{L.gEndS, L.gOrdS, nullptr, L.sufS, L.preS, &L.n[N_IRR_S], kLdsGridS};
  NNStore<uint16_t> sC{L.gEndC, L.gOrdC, nullptr, L.sufC, L.preC, &L.n[N_IRR_C], kLdsGridC};
  return build_args<uint16_t>(L.lastS, st->surfLastNum, sS, L.lastC, st->cornerLastNum, sC, c.N, L.cnt, L.wtot,
                              L.kfirst, L.klast, gridless);
}
__device__ __forceinline__ BuildArgs<uint32_t> hbm_build_args(const OdomLds& L, const OdomBufs& ob,
                                                              const OdomState* st, const DevCfg& c) {
  // counters in LDS; the bucket ends are the counters themselves (the
  // build's final pass rewrites each in place, corner ends less nS)
  unsigned* cnt = hbm_grid_ends(L);
  const int TS = fine_T(st->surfLastNum, ob.gTS);
  NNStore<uint32_t> sS{cnt, nullptr, ob.nS.gPts, L.sufS, L.preS, &L.n[N_IRR_S], ob.gTS};
  NNStore<uint32_t> sC{cnt + TS, nullptr, ob.nC.gPts, L.sufC, L.preC, &L.n[N_IRR_C], ob.gTC};
  return build_args<uint32_t>(buf2(ob.surfLast, st->curBuf), st->surfLastNum, sS, buf2(ob.cornerLast, st->curBuf),
                              st->cornerLastNum, sC, c.N, cnt, L.wtot, L.kfirst, L.klast);
}

// Rebuilds both clouds' indexes (all threads) over the current last clouds.
__device__ __forceinline__ void build_indexes(const OdomLds& L, const OdomBufs& ob, const OdomState* st,
                                              const DevCfg& c, unsigned long long* prof = nullptr) {
  if (st->resident) nn_build2(lds_build_args(L, st, c, ob.gridless), prof);
  else nn_build2(hbm_build_args(L, ob, st, c), prof);
}

// ---------------------------------------------------------------- reduction
// Wave sum of a double through DPP lane moves (VALU, no LDS traffic): quad
// swaps, half-row and row mirrors give every lane its 16-lane row sum, then
// the four row sums are read out in a fixed order.  Deterministic.
template <int kCtrl>
__device__ __forceinline__ double dpp_f64(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp((int)b, kCtrl, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), kCtrl, 0xf, 0xf, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double rdlane_f64(double v, int l) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)b, l), hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// Row sums (16 lanes) of a double through DPP lane moves: quad swaps, then
// half-row and row mirrors leave every lane of a row its row's sum.
__device__ __forceinline__ double row_sum_f64(double v) {
  v += dpp_f64<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_f64<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_f64<0x141>(v);  // row_half_mirror
  v += dpp_f64<0x140>(v);  // row_mirror
  return v;
}

// 9 doubles (AtA upper triangle 6 + AtB 3) + the row count over the block.
// The waves that hold queries (nw) reduce each quantity to four row sums and
// their row leaders put them in LDS; after the barrier lane 4k + r of every
// wave sums row r of quantity k over the waves in order, a quad DPP adds the
// four rows, and readlanes hand every wave the same totals, so the solve
// that follows runs redundantly in every wave without a second barrier.
// Deterministic (a fixed tree).  The partials are double-buffered by
// iteration parity: a wave can run at most one iteration ahead of the
// slowest reader.
__device__ __forceinline__ void block_sum9(double v[9], int m, int nQ, int parity, const OdomLds& L, double out[9],
                                           int* mt) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nw = min(kOdomWaves, (nQ + 63) >> 6);
  double* red = L.red + parity * kOdomWaves * 4 * 10;
  if (wave < nw) {
    double r[10];
#pragma unroll
    for (int k = 0; k < 9; ++k) r[k] = row_sum_f64(v[k]);
    r[9] = row_sum_f64((double)m);
    if ((lane & 15) == 0) {
      double* dst = red + (wave * 4 + (lane >> 4)) * 10;
#pragma unroll
      for (int k = 0; k < 10; ++k) dst[k] = r[k];
    }
  }
  __syncthreads();
  double s = 0;
  if (lane < 40) {
    const int row = lane & 3, k = lane >> 2;
    for (int w = 0; w < nw; ++w) s += red[(w * 4 + row) * 10 + k];
  }
  s += dpp_f64<0xB1>(s);
  s += dpp_f64<0x4E>(s);
#pragma unroll
  for (int k = 0; k < 9; ++k) out[k] = rdlane_f64(s, 4 * k);
  *mt = (int)rdlane_f64(s, 36);
}

struct ScanFeat {
  const float4* sharp; int nSharp;
  const float4* lsharp; int nLS;
  const float4* flat; int nFlat;
  const float4* lflat; int nLF;
  int qpar;  // LDS-resident path: the query buffer (OdomLds::qflat / qsharp) this scan's queries are in
};

// The degeneracy analysis of iteration 0 (:1336-1357, :1437-1458): Jacobi
// eigen-decomposition, the eigenvalues < 10 zeroed, matP = V^-1 V2.  Out of
// line: it runs only when eig_min_above cannot rule degeneracy out, and its
// unrolled Jacobi would otherwise sit inside the LM loop's instruction stream.
// Arguments and result by value: a reference into the caller's matrices
// would give them an address and keep them in scratch memory for the whole
// LM loop.
struct Mat3 {
  float m[3][3];
};
struct DegOut {
  Mat3 P;
  int deg;
};
__device__ __attribute__((noinline)) DegOut degeneracy_cold(const Mat3 in) {
  float AtA[3][3], P[3][3];
#pragma unroll
  for (int a = 0; a < 3; ++a)
#pragma unroll
    for (int b = 0; b < 3; ++b) AtA[a][b] = in.m[a][b];
  float E[3], V[3][3], V2[3][3], Vi[3][3];
  cv_eigen_sym3(AtA, E, V);
#pragma unroll
  for (int a = 0; a < 3; ++a)
#pragma unroll
    for (int b = 0; b < 3; ++b) V2[a][b] = V[a][b];
  int deg = 0;
  bool stop = false;
#pragma unroll
  for (int i = 2; i >= 0; i--) {
    if (!stop && E[i] < 10) {
#pragma unroll
      for (int j = 0; j < 3; j++) V2[i][j] = 0;
      deg = 1;
    } else {
      stop = true;
    }
  }
  cv_inv3(V, Vi);
  cv_matmul<3>(Vi, V2, P);
  DegOut o;
#pragma unroll
  for (int a = 0; a < 3; ++a)
#pragma unroll
    for (int b = 0; b < 3; ++b) o.P.m[a][b] = P[a][b];
  o.deg = deg;
  return o;
}

// Shared tail of calculateTransformationSurf / Corner.  Thread 0 only, all in
// registers (cv_eigen_sym3 is the index-resolved 3x3 Jacobi).
__device__ __forceinline__ void solve_step(float (&AtA)[3][3], float (&AtB)[3], int iter, float (&P)[3][3],
                                           int& isDeg, float (&X)[3]) {
  float Aq[3][3];
#pragma unroll
  for (int a = 0; a < 3; ++a)
#pragma unroll
    for (int b = 0; b < 3; ++b) Aq[a][b] = AtA[a][b];
  cv_solve_qr<3, 3>(Aq, AtB, X);
  if (iter == 0 && eig_min_above(AtA, 10.0)) {
    isDeg = 0;  // P is read only while isDeg is set, and the next iteration 0 rewrites both
  } else if (iter == 0) {
    Mat3 a;
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) a.m[i][j] = AtA[i][j];
    const DegOut d = degeneracy_cold(a);
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) P[i][j] = d.P.m[i][j];
    isDeg = d.deg;
  }
  if (isDeg) {
    float X2[3] = {X[0], X[1], X[2]};
    cv_matvec<3>(P, X2, X);
  }
}

__device__ __forceinline__ double r2d(double r) { return r * 180.0 / M_PI; }

// The convergence test of calculateTransformationSurf / Corner (:1362-1368,
// :1463-1469): deltaR = float(sqrt(sum of rad2deg(x)^2)) < 0.1 and deltaT =
// float(sqrt(sum of (100 x)^2)) < 0.1.  The squared sums are first bounded
// with a multiply by 180/pi (a few ulp from the reference's divide): when
// they are clearly on one side of 0.1^2 the verdict is the reference's; only
// near the threshold is the exact expression evaluated.
__device__ __forceinline__ bool conv_exact(bool surf, const float (&X)[3]) {
  double dR, dT;
  if (surf) {
    const double r0 = r2d(X[0]), r1 = r2d(X[1]), t2 = (double)(X[2] * 100);
    dR = (double)(float)__builtin_sqrt(r0 * r0 + r1 * r1);
    dT = (double)(float)__builtin_sqrt(t2 * t2);
  } else {
    const double r0 = r2d(X[0]), t1 = (double)(X[1] * 100), t2 = (double)(X[2] * 100);
    dR = (double)(float)__builtin_sqrt(r0 * r0);
    dT = (double)(float)__builtin_sqrt(t1 * t1 + t2 * t2);
  }
  return dR < 0.1 && dT < 0.1;
}
__device__ __forceinline__ bool converged3(bool surf, const float (&X)[3]) {
  constexpr double k = 180.0 / M_PI;
  double qR, qT;
  if (surf) {
    const double r0 = X[0] * k, r1 = X[1] * k, t2 = (double)(X[2] * 100);
    qR = r0 * r0 + r1 * r1;
    qT = t2 * t2;
  } else {
    const double r0 = X[0] * k, t1 = (double)(X[1] * 100), t2 = (double)(X[2] * 100);
    qR = r0 * r0;
    qT = t1 * t1 + t2 * t2;
  }
  // float(sqrt(q)) < 0.1 holds for q < 0.0099 and fails for q > 0.0101 (the
  // float rounding of sqrt and the divide-vs-multiply difference are ~1e-7 relative)
  if (qR > 0.0101 || qT > 0.0101) return false;
  if (qR < 0.0099 && qT < 0.0099) return true;
  return conv_exact(surf, X);
}

// ---------------------------------------------------------------- exchange
// The workgroups of a launch run the same serial chain on identical inputs
// and split only the correspondence searches.  Results travel as one 8-byte
// granule per query (x_pack: the three indices and a valid bit; MI355X L2s
// are per XCD: agent-scope relaxed atomics, the data is its own flag), one
// slot per NN round of the launch, zeroed before the launch.  Nothing assumes the launch's workgroups
// are resident together: a granule that has not arrived within kStealTicks is
// computed by the waiting wave itself (the search is deterministic: the same
// bits as its owner's), and a workgroup that starts late replays the chain
// from the rounds already published.  So a plain launch is safe next to any
// other work on the device.
typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned gu32;
constexpr unsigned long long kStealTicks = 4000;  // 40 us at the 100 MHz wall clock
constexpr unsigned long long kLateTicks = 200000000;  // 2 s: the diagnostic late workgroup's bound
// odom_integrate's polls of one scan's granules before it gives up (each
// s_sleep 2 = 128 clocks; ~20 M polls, seconds)
constexpr unsigned kIntegPolls = 20000000u;
// A node call's hand-off waits for the less-flat cloud (launch_odom's
// lfTicks, lego_ctx_opts::lf_wait_ms).  lfReady[b] counts the rings in its
// low bits; the lead workgroup decides (ready, or late after lfTicks) and
// ORs one of these flags in, and every other workgroup follows that decision
// (bounded by lfTicks + kLfFollowTicks), so all take the same cloud size.
constexpr unsigned kLfCountMask = 0xffffu, kLfDecidedOk = 1u << 30, kLfDecidedLate = 1u << 29;
constexpr unsigned long long kLfFollowTicks = 100000000;  // 1 s past the lead's own bound
__device__ __forceinline__ void x_publish(unsigned long long* p, unsigned long long v) {
  __hip_atomic_store((gu64*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// The NN exchange's granule: (i1, i2, i3) of one query, each + 1 in 21 bits,
// and bit 63 set (the round's slots are zeroed before the launch, so a
// nonzero granule is a published one).  Clouds stay below 2^21 - 1 points
// (checked at context creation).
__device__ __forceinline__ unsigned long long x_pack(int i1, int i2, int i3) {
  return (1ull << 63) | ((unsigned long long)(unsigned)(i1 + 1) << 42) |
         ((unsigned long long)(unsigned)(i2 + 1) << 21) | (unsigned long long)(unsigned)(i3 + 1);
}
__device__ __forceinline__ int x_field(unsigned long long x, int k) {  // k = 0: i1, 1: i2, 2: i3
  return (int)((x >> (42 - 21 * k)) & 0x1fffffu) - 1;
}
// Bounded wait for a granule; false when it did not arrive in time.  The
// clock (an SMEM read) is consulted only every 32 polls.
__device__ __forceinline__ bool x_try(const unsigned long long* p, unsigned long long* v) {
  unsigned long long t0 = 0;
  for (unsigned n = 0;; ++n) {
    const unsigned long long x = __hip_atomic_load((gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (x >> 63) {
      *v = x;
      return true;
    }
    if ((n & 31) == 0) {
      const unsigned long long t = wall_clock64();
      if (n == 0) t0 = t;
      else if (t - t0 > kStealTicks) return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

constexpr int kHU = 6;  // hand-off chunks whose granules are in flight together
// Hand-off exchange (TransformToEnd split over the workgroups): workgroup w
// transforms its share of the new last clouds and publishes each point as
// three {seq, x / y / z} granules; every workgroup then takes all points from
// the granules.  A point whose granules have not arrived in kStealTicks is
// transformed by the waiting lane itself (the same bits).  Relaxed loads, as
// the NN exchange.
__device__ __forceinline__ unsigned long long x_load(const unsigned long long* p) {
  return __hip_atomic_load((gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool x_tagged3(unsigned long long a, unsigned long long b, unsigned long long c,
                                          unsigned long long tag) {
  return ((a & b & c) >> 32) == (tag >> 32) && ((a | b | c) >> 32) == (tag >> 32);
}
// The granules of point i (prefetched as a, b, c), polled until they carry
// the tag; false after kStealTicks (the caller transforms the point itself).
__device__ __forceinline__ bool x_point(const unsigned long long* xh, int i, unsigned long long tag,
                                        unsigned long long a, unsigned long long b, unsigned long long c,
                                        float w, float4& p) {
  if (!x_tagged3(a, b, c, tag)) {
    unsigned long long t0 = 0;
    for (unsigned n = 0;; ++n) {
      __builtin_amdgcn_s_sleep(1);
      a = x_load(xh + 3 * i); b = x_load(xh + 3 * i + 1); c = x_load(xh + 3 * i + 2);
      if (x_tagged3(a, b, c, tag)) break;
      if ((n & 31) == 0) {
        const unsigned long long t = wall_clock64();
        if (n == 0) t0 = t;
        else if (t - t0 > kStealTicks) return false;
      }
    }
  }
  p = make_float4(__uint_as_float((unsigned)a), __uint_as_float((unsigned)b), __uint_as_float((unsigned)c),
                  (float)(int)w);
  return true;
}

// ---------------------------------------------------------------- ring
// HBM-resident sensors keep ONE copy per stream of each hand-off's last
// clouds and grids (OdomBufs::ring; featureAssociation.cpp:1759-1815 keeps one
// per stream), built in two phases over shares of whole 64-point chunks:
//   A  TransformToEnd of the share into P (index order), the per-scan output
//      clouds, the bucket counts and key tables (agent-scope atomics);
//   B  the share scattered into Q (bucket order, .w = the point's index) at
//      its bucket's start (from the counts) plus an agent-scope cursor.
// A share is claimed (compare-and-swap) before it is done and flagged done
// after: the owner claims its own at once; a share still unclaimed after
// kStealTicks is claimed and done by a waiting workgroup, so nothing needs the
// launch's workgroups to be resident together.  Stores are 8-byte agent-scope
// (sc1) stores; every storing wave waits for its stores (vmcnt 0) before the
// workgroup barrier behind which one lane flags the share; readers poll the
// flags, then one agent acquire, then plain loads.  Within a launch no slot is
// written twice (ring_next), so a slot is never read before it is complete.
// The slot of the next hand-off: the next of the ring, skipping the indexes'
// snapshot the launch started with (k_ring_prep replays the same picks).
__device__ __forceinline__ int ring_next(unsigned seq, int snapBuf, int R, unsigned* seqOut) {
  const int snap = snapBuf >= 2 ? snapBuf - 2 : -1;
  int s = (int)(seq % (unsigned)R);
  if (s == snap) {
    ++seq;
    s = (int)(seq % (unsigned)R);
  }
  *seqOut = seq + 1;
  return s;
}
__device__ __forceinline__ void ring_put(float4* p, float4 v) {
  unsigned long long* q = (unsigned long long*)p;
  x_publish(q, ((unsigned long long)__float_as_uint(v.y) << 32) | __float_as_uint(v.x));
  x_publish(q + 1, ((unsigned long long)__float_as_uint(v.w) << 32) | __float_as_uint(v.z));
}
__device__ __forceinline__ unsigned ring_add(unsigned* p) {
  return __hip_atomic_fetch_add((gu32*)p, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void ring_max(int* p, int v) {
  __hip_atomic_fetch_max((__attribute__((address_space(1))) int*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool ring_claim(unsigned* p, unsigned who) {
  unsigned e = 0u;
  return __hip_atomic_compare_exchange_strong((gu32*)p, &e, who, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned ring_peek(const unsigned* p) {
  return __hip_atomic_load((gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Per-key first / last tables (suffix minimum / prefix maximum) from
// kfirst / klast, both clouds (all threads; a barrier follows).
__device__ __forceinline__ void key_tables_lds(const OdomLds& L, int NK) {
  for (int t = threadIdx.x; t < 2 * NK; t += kOdomThreads) {
    const int c0 = t >= NK ? NK : 0, k = t - c0;
    int m = INT_MAX, M = -1;
    for (int j = k; j < NK; ++j) m = min(m, L.kfirst[c0 + j]);
    for (int j = 0; j <= k; ++j) M = max(M, L.klast[c0 + j]);
    (c0 ? L.sufC : L.sufS)[k] = m;
    (c0 ? L.preC : L.preS)[k] = M;
  }
  if (threadIdx.x == 0) { L.sufS[NK] = INT_MAX; L.sufC[NK] = INT_MAX; }
}
// A ring slot's grids into LDS: bucket ends (counts scanned; corner ends less
// nS, the corner cloud's points sit after nS in Q) and the key tables.
__device__ __forceinline__ void ring_index_lds(const OdomLds& L, const RingSlot& R, int nS, int TS, int TC, int NK,
                                               bool ends) {
  unsigned* hc = hbm_grid_ends(L);
  const int tid = threadIdx.x;
  for (int b = tid; b < TS + TC; b += kOdomThreads) hc[b] = R.cnt[b];
  for (int t = tid; t < 2 * NK; t += kOdomThreads) {
    L.kfirst[t] = INT_MAX - R.key[t];
    L.klast[t] = R.key[2 * NK + t] - 1;
  }
  if (tid == 0) {
    L.n[N_IRR_S] = R.key[4 * NK] != 0;
    L.n[N_IRR_C] = R.key[4 * NK + 1] != 0;
  }
  __syncthreads();
  block_exscan(hc, TS + TC, L.wtot);  // bucket starts
  key_tables_lds(L, NK);
  if (ends) {
    for (int b = tid; b < TS + TC; b += kOdomThreads) {
      const unsigned e = hc[b] + R.cnt[b];
      hc[b] = b >= TS ? e - (unsigned)nS : e;
    }
  }
  __syncthreads();
}

// One LM loop (surf: <= 25 x {findCorrespondingSurfFeatures;
// calculateTransformationSurf}; corner likewise) — updateTransformation
// :1666-1695.  R: the last clouds and indexes are LDS-resident.
template <bool R, bool RING>
__device__ __forceinline__ void lm_loop(bool surf, const ScanFeat& F, const OdomLds& L, const OdomBufs& ob,
                                        const DevCfg& c, Stamp& S) {
  using Idx = typename std::conditional<R, uint16_t, uint32_t>::type;
  OdomState* st = L.st;
  const int tid = threadIdx.x;
  const float4* last;
  int* qi;
  int qs;
  NNView<Idx> nn;
  if constexpr (R) {
    last = surf ? L.lastS : L.lastC;
    qi = L.qi; qs = kLdsQ;
    nn = view_lds(surf, L, st, c, ob.gridless);
  } else {
    last = hbm_cloud<RING>(ob, st->curBuf, surf, st->surfLastNum);
    qi = ob.qi; qs = ob.capQ;
    nn = view_hbm<RING>(surf, L, ob, st, c);
  }
  const int lastN = surf ? st->surfLastNum : st->cornerLastNum;
  const bool stale = st->curBuf != st->snapBuf;
  const float4* snap = hbm_cloud<RING>(ob, st->snapBuf, surf, st->nnSurfNum);
  const int snapN = surf ? st->nnSurfNum : st->nnCornerNum;
  const float4* qp;
  if constexpr (R) qp = surf ? L.qflat + F.qpar * kLdsQ : L.qsharp + F.qpar * (kLdsQ / 2);  // staged in LDS
  else qp = surf ? F.flat : F.sharp;
  const int nQ = surf ? F.nFlat : F.nSharp;
  const int jend = min(nQ, lastN);  // the reference bounds by the query count (:1062, :1173)
  const int g = tid & (kGL - 1), grp = tid / kGL;
  // transformCur, matP and isDegenerate live in registers for the loop: every
  // wave computes the same solve (st is written back once at the end)
  float tc[6], Pm[3][3];
  int isDeg = st->isDegenerate;
#pragma unroll
  for (int i = 0; i < 6; ++i) tc[i] = st->transformCur[i];
#pragma unroll
  for (int i = 0; i < 9; ++i) Pm[i / 3][i % 3] = st->matP[i];
  FixTrig fix;
  fix.have = false;
  // Waves 0-3 (one per SIMD) issue ahead of waves 4-7 during the loop: the
  // rows sit on the low waves, and every wave's redundant 3x3 solve then
  // yields the SIMD to the wave that carries the chain on (+0.45% on C2, A/B;
  // the same for the whole kernel, or only around the solve: equal / -0.8%)
  if (tid < 4 * 64) __builtin_amdgcn_s_setprio(2);
  RP_ADD(S, P_B_SCAN);
  for (int it = 0; it < 25; it++) {
    S.start();
    S.count(surf ? P_ITERS_S : P_ITERS_C);
    const bool nnIter = it % 5 == 0;
    if (nnIter) S.count(P_NNR);
    // sin / cos of the three angles: lanes 0-2 and 3-5 of each wave, then broadcast
    float trig;
    {  // lanes 0-2 the sines, 3-5 the cosines: one fused evaluation, no divergence
      const int l = tid & 63;
      float sv, cv;
      const int l3 = l % 3;  // selects, not tc[l % 3]: a lane-varying index would put tc in scratch
      lego_sincosf(l3 == 0 ? tc[0] : (l3 == 1 ? tc[1] : tc[2]), &sv, &cv);
      trig = l < 3 ? sv : cv;
    }
    const float srx = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(trig), 0));
    const float sry = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(trig), 1));
    const float srz = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(trig), 2));
    const float crx = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(trig), 3));
    const float cry = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(trig), 4));
    const float crz = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(trig), 5));
    const float tx = tc[3], ty = tc[4], tz = tc[5];
    double acc[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    int mloc = 0;
    if (nnIter) {
      // This workgroup's slice of the queries, one wave per query; the slices
      // of the other workgroups of the launch arrive through the exchange.
      const int G = ob.G, per = (nQ + G - 1) / G;
      const int q0 = min(nQ, ob.wg * per), q1 = min(nQ, q0 + per);
      int round = L.n[N_ROUND];
      const bool xch = G > 1 && round < ob.roundsCap;
      if (G > 1 && !xch && tid == 0) *ob.xerr = 1;  // more rounds than the slots (cannot happen: 10 per scan)
      unsigned long long* xg = ob.xg + (size_t)round * ob.capQ;  // this stream's (odom_private)
      const bool w0 = S.prof && tid == 0;
      // findCorresponding{Surf,Corner}Features for query q by one wave
      auto search = [&](int q, int& i1, int& i2, int& i3) {
        // wave 0's sub-phase stamps (diagnostic): to_start, closest point, scan-line neighbours
        unsigned long long tq = w0 ? wall_clock64() : 0;
        auto sub = [&](int k) {
          if (w0) {
            const unsigned long long n = wall_clock64();
            S.prof[k] += n - tq;
            tq = n;
          }
        };
        // TransformToStart of the wave's query: the three sines / cosines on
        // lanes 0-2 at once (the same calls as to_start), then broadcast
        const float4 pq = qp[q];
        const float s = start_s(pq);
        float sv, cv;
        {
          const int l3 = g % 3;  // selects, not tc[l3] (a lane-varying index would put tc in scratch)
          lego_sincosf(s * (l3 == 0 ? tc[0] : (l3 == 1 ? tc[1] : tc[2])), &sv, &cv);
        }
        const float sx = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(sv), 0));
        const float sy = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(sv), 1));
        const float sz = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(sv), 2));
        const float cx = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cv), 0));
        const float cy = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cv), 1));
        const float cz = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cv), 2));
        const float4 sel = to_start_t(pq, s, tc, cx, sx, cy, sy, cz, sz);
        sub(P_G0_TOSTART);
        // a corner query against a small cloud: one pass over registers
        // (+0.35% on C2, A/B)
        if (!surf && !stale && !nn.irregular && nn.n <= kBruteSmall) {
          bool ok;
          i3 = -1;
          i1 = nn_corner_small(nn, jend, sel, c.nn_sq, c.nn_sq, g, &i2, &ok);
          if (i1 >= lastN) i1 = -1;
          if (i1 >= 0 && !ok) scanline_group(last, jend, i1, sel, surf, c.nn_sq, g, &i2, &i3);
          if (i1 < 0) i2 = -1;
          sub(P_G0_SCAN);
          return;
        }
        i1 = stale ? nn_brute(snap, snapN, sel, c.nn_sq, g) : nn_i1(nn, sel, c.nn_sq, g, S.prof);
        if (i1 >= lastN) i1 = -1;  // an index past a stale snapshot's cloud
        sub(P_G0_NN);
        i2 = -1; i3 = -1;
        if (i1 >= 0 && (stale || !nn_lines(nn, i1, jend, sel, surf, c.nn_sq, g, &i2, &i3))) {
          if (S.prof && g == 0) atomicAdd(&S.prof[P_SCANLINE], 1ull);
          scanline_group(last, jend, i1, sel, surf, c.nn_sq, g, &i2, &i3);
        }
        sub(P_G0_SCAN);
      };
      const int qa = xch ? q0 : 0, qb = xch ? q1 : nQ;  // no exchange: every query here
      for (int q = qa + grp; q < qb; q += kNGrp) {
        unsigned long long ta = w0 ? wall_clock64() : 0;
        int i1, i2, i3;
        search(q, i1, i2, i3);
        if (w0) {
          S.prof[28] += wall_clock64() - ta; S.prof[30] += 1;
        }
        if (g == 0) {
          qi[q] = i1; qi[qs + q] = i2; qi[2 * qs + q] = i3;
          if (xch) x_publish(xg + q, x_pack(i1, i2, i3));
        }
      }
      S.add(P_X_LOCAL);
      if (xch) {
        // the other slices: lane l of a wave waits for the granule of query
        // base + l (64 queries per pass); what does not arrive in time the
        // wave computes itself
        for (int base = grp * kGL; base < nQ; base += kNGrp * kGL) {
          const int q = base + g;
          const bool want = q < nQ && !(q >= q0 && q < q1);
          bool got = !want;
          if (want) {
            unsigned long long x;
            got = x_try(xg + q, &x);
            if (got) {
              qi[q] = x_field(x, 0); qi[qs + q] = x_field(x, 1); qi[2 * qs + q] = x_field(x, 2);
            }
          }
          unsigned long long miss = __ballot(!got);
          while (miss) {
            const int qm = base + __ffsll((long long)miss) - 1;
            int i1, i2, i3;
            search(qm, i1, i2, i3);
            if (g == 0) {
              qi[qm] = i1; qi[qs + qm] = i2; qi[2 * qs + qm] = i3;
              x_publish(xg + qm, x_pack(i1, i2, i3));
            }
            miss &= miss - 1;
          }
        }
      }
      __syncthreads();
      if (tid == 0) L.n[N_ROUND] = round + 1;
      S.add(P_QUERY);
    }
    for (int q = tid; q < nQ; q += kOdomThreads) {
      const float4 po = qp[q];
      const float4 sel = q == tid ? to_start_fix(po, tc, surf, fix) : to_start(po, tc);
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
        // a product of two floats is exact in double, so one fma rounds the
        // sum exactly as the separate multiply and add do
        const double d0 = a0, d1 = a1, d2 = a2, db = bb;
        acc[0] = __builtin_fma(d0, d0, acc[0]); acc[1] = __builtin_fma(d0, d1, acc[1]);
        acc[2] = __builtin_fma(d0, d2, acc[2]); acc[3] = __builtin_fma(d1, d1, acc[3]);
        acc[4] = __builtin_fma(d1, d2, acc[4]); acc[5] = __builtin_fma(d2, d2, acc[5]);
        acc[6] = __builtin_fma(d0, db, acc[6]); acc[7] = __builtin_fma(d1, db, acc[7]);
        acc[8] = __builtin_fma(d2, db, acc[8]);
        mloc++;
      }
    }
    double tot[9];
    int M = 0;
    S.add(P_T_ROWS);
    block_sum9(acc, mloc, nQ, it & 1, L, tot, &M);
    S.add(surf ? (nnIter ? P_SURF_NN : P_SURF) : (nnIter ? P_CORN_NN : P_CORN));
    bool brk = false;
    if (M >= 10) {
      float AtA[3][3] = {{(float)tot[0], (float)tot[1], (float)tot[2]},
                         {(float)tot[1], (float)tot[3], (float)tot[4]},
                         {(float)tot[2], (float)tot[4], (float)tot[5]}};
      float AtB[3] = {(float)tot[6], (float)tot[7], (float)tot[8]};
      float X[3];
      solve_step(AtA, AtB, it, Pm, isDeg, X);
      S.add(it == 0 ? P_T_SOLVE0 : P_T_SOLVE);
      if (surf) {
        tc[0] += X[0]; tc[2] += X[1]; tc[4] += X[2];
      } else {
        tc[1] += X[0]; tc[3] += X[1]; tc[5] += X[2];
      }
#pragma unroll
      for (int i = 0; i < 6; i++) if (__builtin_isnan(tc[i])) tc[i] = 0;
      brk = converged3(surf, X);
    }
    S.add(P_SOLVE);
    if (brk) break;
  }
  RP_START(S);
  __builtin_amdgcn_s_setprio(0);
  // write the loop's state back once (all waves hold the same values)
  if (tid == 0) {
#pragma unroll
    for (int i = 0; i < 6; ++i) st->transformCur[i] = tc[i];
#pragma unroll
    for (int i = 0; i < 9; ++i) st->matP[i] = Pm[i / 3][i % 3];
    st->isDegenerate = isDeg;
  }
  __syncthreads();
  RP_ADD(S, P_B_SCAN);
}

// This workgroup's private HBM buffers (the launch's workgroups never share
// them) and its stream's state and exchange granules.  Block i of the launch
// is workgroup i % G of stream i / G.
__device__ __forceinline__ OdomBufs odom_private(OdomBufs ob) {
  const int s = blockIdx.x / ob.G;
  const int silent = ob.wg;  // the host's value (OdomBufs::wg)
  ob.wg = blockIdx.x - s * ob.G;
  if (ob.wg == silent) {
    ob.xg += ob.xerr[2];
    ob.xh += ob.xerr[3];
  }
  const size_t w = blockIdx.x;  // index into the [S x G x] arrays
  ob.st += s;
  ob.stIn += s;
  ob.xg += (size_t)s * ob.roundsCap * ob.capQ;
  ob.xh += (size_t)s * 2 * 3 * ob.capH;
  ob.cornerLast[0] += w * ob.capCorner;
  ob.cornerLast[1] += w * ob.capCorner;
  ob.surfLast[0] += w * ob.capSurf;
  ob.surfLast[1] += w * ob.capSurf;
  ob.nC.gPts += w * ob.capCorner;
  ob.nS.gPts += w * ob.capSurf;
  ob.qi += w * 3 * ob.capQ;
  if (ob.ring) {  // the stream's ring (the silent workgroup: its private copy after it)
    ob.ring += (size_t)s * (ob.ringCopy ? 2 : 1) * ob.ringR * ob.ringStride;
    if (ob.wg == silent) ob.ring += ob.ringCopy;
  }
  return ob;
}

// K scans of each of the ob.S streams: block i runs stream i / G's scans
// [s*K, s*K + K) of the batch.
// integrateTransformation (:1697-1725) of every scan of the launch, in order,
// off the odometry chain (OdomBufs::integ): wave 0 of the stream's extra
// workgroup, from the launch's input transformSum and the lead's published
// transformCur / valid flag of each scan (checkSystemInitialization's
// increment at a stream's first scan, :1633-1634); writes sumOut and, at the
// end, the state's transformSum (the lead leaves those words alone).
__device__ __forceinline__ void odom_integrate(const BatchBufs& bb, const OdomBufs& ob, int K) {
  const int lane = threadIdx.x;
  const int s = blockIdx.x - ob.S * ob.G;
  __shared__ float ts[6], tc[6];
  if (lane < 6) ts[lane] = ob.stIn[s].transformSum[lane];
  for (int b = s * K; b < s * K + K; ++b) {
    unsigned long long g = 0;
    const unsigned want = (unsigned)(b + 1);
    unsigned polls = 0;
    if (lane < 6) {
      for (;;) {
        g = x_load(ob.intX + (size_t)b * 6 + lane);
        if ((unsigned)(g >> 33) == want || ++polls > kIntegPolls) break;
        __builtin_amdgcn_s_sleep(2);
      }
      tc[lane] = __uint_as_float((unsigned)g);
    }
    if (__ballot(polls > kIntegPolls)) {  // the batch's error word (3), not a hung device
      if (lane == 0) *ob.xerr = 3u;
      return;
    }
    const bool valid = (__builtin_amdgcn_readfirstlane((int)(unsigned)(g >> 32)) & 1) != 0;
    ImuScan iq = {};
    if (bb.imu) iq = bb.imuScan[b];
    if (!valid) {
      if (lane == 0) {  // checkSystemInitialization :1633-1634
        ts[0] += iq.pitchStart;
        ts[2] += iq.rollStart;
      }
    } else {
      const float bl[3] = {iq.pitchStart, iq.yawStart, iq.rollStart};
      const float al[3] = {iq.pitchCur, iq.yawCur, iq.rollCur};  // imu*Last = imu*Cur (:1641-1643)
      integrate_wave(ts, tc, bl, al);
    }
    if (lane < 6) ob.sumOut[(size_t)b * 6 + lane] = ts[lane];
  }
  if (lane < 6) ob.st[s].transformSum[lane] = ts[lane];
}

// RING: the sensor keeps its last clouds in the stream's ring (OdomBufs::ring,
// HDL-64E / VLS-128); a separate instantiation, so the LDS-resident sensors'
// kernel carries none of its code or registers.  LFW: a node call's form,
// whose hand-off waits for the side stream's less-flat cloud (launch_odom's
// lfReady, a trailing argument so the batch kernels' arguments keep their
// offsets); also separate, so the batch kernels keep their registers.
template <bool RING, bool LFW>
__global__ void __launch_bounds__(kOdomThreads) k_odom(BatchBufs bb, OdomBufs obShared, DevCfg c, int K,
                                                      unsigned long long* prof, unsigned* lfReady,
                                                      unsigned long long lfTicks) {
  // Claim the whole register file of the SIMD (2 waves x 256): no other
  // kernel's waves share a SIMD with the latency-bound chain while the next
  // chunk's extraction runs beside it.
  asm volatile("v_mov_b32 v255, 0" ::: "v255");
  if (obShared.integ && (int)blockIdx.x >= obShared.S * obShared.G) {  // the stream's integrating workgroup
    if (threadIdx.x < 64) odom_integrate(bb, obShared, K);
    return;
  }
  const OdomBufs ob = odom_private(obShared);
  const int b0 = (int)(blockIdx.x / ob.G) * K;
  const bool lead = ob.wg == 0;  // writes the stream's outputs and state
  if (blockIdx.x != 0) prof = nullptr;
  // stamps accumulate in LDS (a global read-modify-write per stamp would put
  // an L2 round trip on the chain it measures); added to prof at the end
  __shared__ unsigned long long sprof[P_NPROF];
  unsigned long long* const gprof = prof;
  if (gprof) {
    if (threadIdx.x < P_NPROF) sprof[threadIdx.x] = 0;
    prof = sprof;
  }
  Stamp S{prof, 0};
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
  const OdomLds L = odom_carve(lds_raw);
  const int tid = threadIdx.x;
  static_assert(sizeof(OdomState) <= 128, "OdomState LDS slot");
  OdomState* st = L.st;
  if (ob.wg == ob.late) {  // diagnostic: start only once the lead has finished
    if (tid == 0) {
      const unsigned long long t0 = wall_clock64();
      while (__hip_atomic_load((gu32*)&ob.xerr[1], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == 0u &&
             wall_clock64() - t0 < kLateTicks)
        __builtin_amdgcn_s_sleep(8);
    }
    __syncthreads();
  }
  // the launch's input state (never the lead's output: ob.st)
  if (tid < (int)(sizeof(OdomState) / 4)) ((int*)st)[tid] = ((const int*)ob.stIn)[tid];
  if (tid == 0) L.n[N_ROUND] = 0;
  __syncthreads();
  const bool sensorRes = sensor_resident(c);
  // LDS does not survive launches: reload the current last clouds and rebuild
  // the indexes over them (unless the snapshot is stale: brute force then).
  S.start();
  if (st->inited) {
    if (!RING && st->resident) {
      const float4* gS = buf2(ob.surfLast, st->curBuf);
      const float4* gC = buf2(ob.cornerLast, st->curBuf);
      for (int t = tid; t < st->surfLastNum; t += kOdomThreads) L.lastS[t] = gS[t];
      for (int t = tid; t < st->cornerLastNum; t += kOdomThreads) L.lastC[t] = gC[t];
      __syncthreads();
    }
    if (st->curBuf == st->snapBuf) {
      if (RING && st->curBuf >= 2) {  // the stream's ring slot: its grids' ends and key tables into LDS
        ring_index_lds(L, ring_slot(ob, st->curBuf - 2), st->nnSurfNum, fine_T(st->nnSurfNum, ob.gTS),
                       fine_T(st->nnCornerNum, ob.gTC), c.N, true);
      } else if (!RING) {
        build_indexes(L, ob, st, c);
      }
    }
  }
  S.add(P_RESID);
  for (int b = b0; b < b0 + K; ++b) {
    RP_START(S);
    ScanFeat F;
    // the counts and (LDS-resident path) the queries of every scan but the
    // launch's first were fetched during the previous scan's hand-off (N_PRE):
    // no global-memory round trip on the chain between two scans
    const bool pre = !RING && b > b0 && __builtin_amdgcn_readfirstlane(L.n[N_PRE]);
    const int par = (b - b0) & 1;
    int4 fc;
    // (readfirstlane: an LDS word is a VGPR to the compiler, and a count it
    // cannot prove uniform turns the loops it bounds divergent: +26 spills)
    if (pre) fc = make_int4(__builtin_amdgcn_readfirstlane(L.n[N_NEXT]), __builtin_amdgcn_readfirstlane(L.n[N_NEXT + 1]),
                            __builtin_amdgcn_readfirstlane(L.n[N_NEXT + 2]), __builtin_amdgcn_readfirstlane(L.n[N_NEXT + 3]));
    else fc = *(const int4*)(bb.f_cnt + b * 4);
    F.sharp = bb.f_sharp + (size_t)b * c.N * kSharpPerRing; F.nSharp = fc.x;
    F.lsharp = bb.f_lsharp + (size_t)b * c.N * kLessSharpPerRing; F.nLS = fc.y;
    F.flat = bb.f_flat + (size_t)b * c.N * kFlatPerRing; F.nFlat = fc.z;
    F.lflat = bb.f_lflat + (size_t)b * c.P; F.nLF = fc.w;
    F.qpar = par;
    float4* cEnd = ob.cornerEnd + (size_t)b * ob.capLS;
    float4* sEnd = ob.surfEnd + (size_t)b * c.P;
    const bool init = !st->inited;
    // this scan's IMU terms (all zero without an IMU message: cos 0 = 1)
    ImuScan iq = {};
    if (bb.imu) iq = bb.imuScan[b];
    if (!init) {
      // updateInitialGuess :1639-1664 (imuShiftFromStart* stays 0; a no-op
      // until the stream's first IMU message)
      if (bb.imu) {
      if (tid == 0) {
        float* tc = st->transformCur;
        if (iq.angFromStart[0] != 0 || iq.angFromStart[1] != 0 || iq.angFromStart[2] != 0) {
          tc[0] = -iq.angFromStart[1];
          tc[1] = -iq.angFromStart[2];
          tc[2] = -iq.angFromStart[0];
        }
        if (iq.vfs[0] != 0 || iq.vfs[1] != 0 || iq.vfs[2] != 0) {
          tc[3] -= iq.vfs[0] * c.scan_period;
          tc[4] -= iq.vfs[1] * c.scan_period;
          tc[5] -= iq.vfs[2] * c.scan_period;
        }
      }
      __syncthreads();
      }
      if (st->cornerLastNum >= 10 && st->surfLastNum >= 100) {
        if (!RING && st->resident) {
          if (!pre) {
            for (int t = tid; t < F.nFlat; t += kOdomThreads) L.qflat[par * kLdsQ + t] = F.flat[t];
            for (int t = tid; t < F.nSharp; t += kOdomThreads) L.qsharp[par * (kLdsQ / 2) + t] = F.sharp[t];
            __syncthreads();
          }
          RP_ADD(S, P_B_PASS1);
          lm_loop<true, RING>(true, F, L, ob, c, S);
          lm_loop<true, RING>(false, F, L, ob, c, S);
        } else {
          RP_ADD(S, P_B_PASS1);
          lm_loop<false, RING>(true, F, L, ob, c, S);
          lm_loop<false, RING>(false, F, L, ob, c, S);
        }
      }
    }
    if (LFW) {  // a node call: the less-flat cloud comes from the side stream (launch_fa)
      if (tid == 0) {
        const unsigned long long t0 = wall_clock64();
        bool ok = false;
        if (lead) {  // decides for the launch (kLfDecided*)
          if (lfTicks)
            while (!(ok = (__hip_atomic_load(lfReady + b, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) &
                           kLfCountMask) >= (unsigned)c.N) &&
                   wall_clock64() - t0 < lfTicks)
              __builtin_amdgcn_s_sleep(2);
          __hip_atomic_fetch_or(lfReady + b, ok ? kLfDecidedOk : kLfDecidedLate, __ATOMIC_RELEASE,
                                __HIP_MEMORY_SCOPE_AGENT);
        } else {  // follows the lead's decision
          unsigned v;
          while (!((v = __hip_atomic_load(lfReady + b, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT)) &
                   (kLfDecidedOk | kLfDecidedLate)) &&
                 wall_clock64() - t0 < lfTicks + kLfFollowTicks)
            __builtin_amdgcn_s_sleep(2);
          ok = (v & kLfDecidedOk) != 0;
        }
        L.n[N_LF] = ok ? __hip_atomic_load(bb.f_cnt + b * 4 + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
        // the host fails the call and the context until lego_reset (never a silent empty cloud)
        if (!ok) atomicOr(bb.bad + b, kBadLfLate);
      }
      __syncthreads();
      F.nLF = __builtin_amdgcn_readfirstlane(L.n[N_LF]);
    }
    S.start();
    // hand-off: checkSystemInitialization (:1605-1637, no TransformToEnd) or
    // publishCloudsLast (:1759-1815).  The new last clouds go to the HBM
    // buffer that is not the index snapshot (so a stale snapshot survives),
    // to the per-scan outputs, and to LDS when they fit.
    const int nbuf = st->snapBuf ^ 1;
    float4* gCn = buf2(ob.cornerLast, nbuf);
    float4* gSn = buf2(ob.surfLast, nbuf);
    const bool fits = !RING && sensorRes && F.nLS <= kLdsCorner && F.nLF <= kLdsSurf;
    float tcur[6];
    for (int i = 0; i < 6; ++i) tcur[i] = st->transformCur[i];
    const EndTrig et = end_trig(tcur);
    if (ODOM_RESID_PROBE == 2) S.add(P_B_ENDS);
    // updateImuRollPitchYawStartSinCos (:1761) and the imu*Last terms of TransformToEnd
    ImuEnd im{1.f, 1.f, 1.f, 0.f, 0.f, 0.f, 1.f, 0.f, 1.f, 0.f, 1.f, 0.f};  // cos 0 / sin 0
    const bool hasImu = bb.imu != nullptr;
    if (hasImu)
      im = ImuEnd{lego_cosf(iq.rollStart), lego_cosf(iq.pitchStart), lego_cosf(iq.yawStart),
                  lego_sinf(iq.rollStart), lego_sinf(iq.pitchStart), lego_sinf(iq.yawStart),
                  lego_cosf(iq.yawCur), lego_sinf(iq.yawCur), lego_cosf(iq.pitchCur),
                  lego_sinf(iq.pitchCur), lego_cosf(iq.rollCur), lego_sinf(iq.rollCur)};
    // integrateTransformation (:1697-1725) on wave 0 while waves 1-7 run
    // TransformToEnd: both read the final transformCur, only the former
    // writes (transformSum)
    const bool waves8 = init || ob.integ;  // TransformToEnd on every wave (integration elsewhere or none)
    const int t0 = waves8 ? tid : tid - 64, tstep = waves8 ? kOdomThreads : kOdomThreads - 64;
    const bool rebuild = init || (F.nLS > 10 && F.nLF > 100);
    // the new clouds' build arguments in the layout they will use
    NNStore<uint16_t> nsS{L.gEndS, L.gOrdS, nullptr, L.sufS, L.preS, &L.n[N_IRR_S], kLdsGridS};
    NNStore<uint16_t> nsC{L.gEndC, L.gOrdC, nullptr, L.sufC, L.preC, &L.n[N_IRR_C], kLdsGridC};
    const BuildArgs<uint16_t> BL = build_args<uint16_t>(L.lastS, F.nLF, nsS, L.lastC, F.nLS, nsC, c.N, L.cnt,
                                                        L.wtot, L.kfirst, L.klast, ob.gridless);
    unsigned* hcnt = hbm_grid_ends(L);
    const int hTS = fine_T(F.nLF, ob.gTS);
    NNStore<uint32_t> hsS{hcnt, nullptr, ob.nS.gPts, L.sufS, L.preS, &L.n[N_IRR_S], ob.gTS};
    NNStore<uint32_t> hsC{hcnt + hTS, nullptr, ob.nC.gPts, L.sufC, L.preC, &L.n[N_IRR_C], ob.gTC};
    const BuildArgs<uint32_t> BH = build_args<uint32_t>(gSn, F.nLF, hsS, gCn, F.nLS, hsC, c.N, hcnt, L.wtot,
                                                        L.kfirst, L.klast);
    // HBM-resident sensors: the stream's ring slot of this hand-off, its shares
    // (whole 64-point chunks) and this workgroup's claim on its own share
    const bool ringMode = RING && ob.ring != nullptr && !fits;
    unsigned rseq = 0;
    // the skip is the LAUNCH's input snapshot (ob.stIn), the slot k_ring_prep
    // left alone: a snapshot this launch makes is a slot already behind seq,
    // never picked again within the launch (<= K + 1 consecutive picks of
    // R = K + 3), so the kernel replays prep's picks exactly
    const int rslot = ringMode ? ring_next(st->seq, ob.stIn->snapBuf, ob.ringR, &rseq) : -1;
    const int rn = F.nLF + F.nLS;
    const int rper = max(64, ((rn + ob.G - 1) / ob.G + 63) & ~63);
    const int rnsh = (rn + rper - 1) / rper;
    if (ringMode && tid == 0)
      L.n[N_CLAIM] = ob.wg < rnsh && ring_claim(&ring_slot(ob, rslot).claimA[ob.wg], (unsigned)ob.wg + 1u);
    if (rebuild && !RING) {  // the counters must be zero before the first chunk is counted
      if (fits) build_zero(BL);
      else build_zero(BH);
    }
    __syncthreads();
    // the next scan's counts and queries, copied into the other query buffer
    // while this hand-off runs: direct global -> LDS loads (no VGPRs held;
    // the LDS image is lane-linear, slot = thread), every query slot up to the
    // sensor's caps so nothing waits for the counts (slots past a scan's count
    // hold whatever the extraction left, never read).  The barriers after the
    // hand-off retire them.
    const bool nxt = !RING && sensorRes && b + 1 < b0 + K;
    if (nxt) {
      // (the lane index laundered through an empty asm: otherwise the compiler
      // hoists the three per-lane addresses out of the scan loop and spills
      // them, and each copy then waits for a scratch reload)
      int t = tid;
      asm volatile("" : "+v"(t));
      const size_t bn = (size_t)b + 1;
      const int nf = c.N * kFlatPerRing, nsh = c.N * kSharpPerRing, wb = t & ~63;
      if (t < nf)
        __builtin_amdgcn_global_load_lds((const void*)(bb.f_flat + bn * nf + t),
                                         (void*)(L.qflat + (par ^ 1) * kLdsQ + wb), 16, 0, 0);
      if (t < nsh)
        __builtin_amdgcn_global_load_lds((const void*)(bb.f_sharp + bn * nsh + t),
                                         (void*)(L.qsharp + (par ^ 1) * (kLdsQ / 2) + wb), 16, 0, 0);
      if (t < 4)
        __builtin_amdgcn_global_load_lds((const void*)(bb.f_cnt + bn * 4 + t), (void*)(L.n + N_NEXT), 4, 0, 0);
    }
    // hand-off exchange: this workgroup's share of TransformToEnd, published.
    // Only for the HBM-resident sensors: C3 +2.5%, while the LDS-resident
    // VLP-16 stream and the fleet measured equal (their chunks are few, and
    // the granules' latency costs what the transform saves).
    const bool hx = ob.G > 1 && !init && !fits && !ringMode;
    const unsigned seq = st->seq + 1u;
    const unsigned long long xtag = (unsigned long long)seq << 32;
    unsigned long long* const xh = ob.xh + (size_t)(seq & 1u) * 3 * ob.capH;
    if (hx && t0 >= 0) {
      const int n = F.nLF + F.nLS, per = (n + ob.G - 1) / ob.G;
      const int a = min(n, ob.wg * per), e = min(n, a + per);
      for (int i = a + t0; i < e; i += tstep) {
        const float4 p = to_end(i < F.nLF ? F.lflat[i] : F.lsharp[i - F.nLF], tcur, et, im, hasImu);
        x_publish(xh + 3 * i, xtag | __float_as_uint(p.x));
        x_publish(xh + 3 * i + 1, xtag | __float_as_uint(p.y));
        x_publish(xh + 3 * i + 2, xtag | __float_as_uint(p.z));
      }
    }
    const unsigned long long tw = prof && (tid == 0 || tid == 64) ? wall_clock64() : 0;
    if (!init && tid < 64 && !ob.integ) {
      const float bl[3] = {iq.pitchStart, iq.yawStart, iq.rollStart};
      const float al[3] = {iq.pitchCur, iq.yawCur, iq.rollCur};  // imu*Last = imu*Cur (:1641-1643)
      integrate_wave(st->transformSum, st->transformCur, bl, al);
    }
    if (prof && tid == 0) prof[P_INTEG] += wall_clock64() - tw;
    // TransformToEnd of less-flat then less-sharp as one index range in
    // wave-uniform chunks, each chunk counted into the next index as it is
    // produced (build_count: no read-back of the clouds for the counting pass)
    auto hand_off = [&](const auto& B) {
      if (t0 >= 0) {
        const int nS = F.nLF, n = F.nLF + F.nLS, lane = tid & 63;
        auto w_at = [&](int j) { return j < nS ? F.lflat[j].w : F.lsharp[j - nS].w; };
        // the point and its neighbours' .w words, one chunk ahead
        auto fetch = [&](int i, float4& r, float& wp, float& wn) {
          if (i < n) {
            r = i >= nS ? F.lsharp[i - nS] : F.lflat[i];
            wp = w_at(max(i - 1, 0));
            wn = w_at(min(i + 1, n - 1));
          }
        };
        float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
        float wp = 0.f, wn = 0.f;
        fetch(t0, r, wp, wn);
        for (int i0 = t0 - lane; i0 < n; i0 += tstep) {  // wave-uniform
          const int i = i0 + lane;
          float4 rN = r;
          float wpN = wp, wnN = wn;
          fetch(i + tstep, rN, wpN, wnN);
          float4 p = make_float4(0.f, 0.f, 0.f, 0.f);
          int kp = 0, kn = 0;
          if (i < n) {
            const bool corner = i >= nS;
            if (rebuild) nbr_keys(i, nS, n, wp, wn, kp, kn);
            p = init ? r : to_end(r, tcur, et, im, hasImu);
            if (corner) {
              gCn[i - nS] = p;
              if (lead) cEnd[i - nS] = p;
              if (fits) L.lastC[i - nS] = p;
            } else {
              gSn[i] = p;
              if (lead) sEnd[i] = p;
              if (fits) L.lastS[i] = p;
            }
          }
          if (rebuild) build_count(B, i0, p, kp, kn);
          r = rN; wp = wpN; wn = wnN;
        }
      }
    };
    // the same with the points taken from the exchange: kHU chunks' granules
    // and inputs are loaded before any of them is used (one latency per group)
    auto hand_off_x = [&](const auto& B) {
      if (t0 >= 0) {
        const int nS = F.nLF, n = F.nLF + F.nLS, lane = tid & 63;
        auto w_at = [&](int j) { return j < nS ? F.lflat[j].w : F.lsharp[j - nS].w; };
        auto put = [&](int i, float4 p) {
          if (i >= nS) {
            gCn[i - nS] = p;
            if (lead) cEnd[i - nS] = p;
            if (fits) L.lastC[i - nS] = p;
          } else {
            gSn[i] = p;
            if (lead) sEnd[i] = p;
            if (fits) L.lastS[i] = p;
          }
        };
        for (int c0 = t0 - lane; c0 < n; c0 += kHU * tstep) {  // wave-uniform
          float wr[kHU], wp[kHU], wn[kHU];
          unsigned long long ga[kHU], gb[kHU], gc[kHU];
#pragma unroll
          for (int u = 0; u < kHU; ++u) {
            const int i = c0 + u * tstep + lane;
            wr[u] = wp[u] = wn[u] = 0.f;
            ga[u] = gb[u] = gc[u] = 0;
            if (i < n) {
              wr[u] = w_at(i);
              wp[u] = w_at(max(i - 1, 0));
              wn[u] = w_at(min(i + 1, n - 1));
              ga[u] = x_load(xh + 3 * i);
              gb[u] = x_load(xh + 3 * i + 1);
              gc[u] = x_load(xh + 3 * i + 2);
            }
          }
          unsigned miss = 0;  // bit u: point c0 + u * tstep + lane did not arrive
#pragma unroll
          for (int u = 0; u < kHU; ++u) {
            const int i0 = c0 + u * tstep, i = i0 + lane;
            if (i0 >= n) break;
            float4 p = make_float4(0.f, 0.f, 0.f, 0.f);
            int kp = 0, kn = 0;
            bool ok = false;
            if (i < n) {
              if (rebuild) nbr_keys(i, nS, n, wp[u], wn[u], kp, kn);
              ok = x_point(xh, i, xtag, ga[u], gb[u], gc[u], wr[u], p);
              if (ok) put(i, p);
              else miss |= 1u << u;
            }
            if (rebuild) build_count(B, i0, p, kp, kn, ok);
          }
          // the points whose granules did not arrive: transformed here
          for (unsigned long long mw = __ballot(miss != 0); mw; mw = __ballot(miss != 0)) {
            const int u = miss ? __ffs(miss) - 1 : 0;
            const int i = c0 + u * tstep + lane;
            float4 p = make_float4(0.f, 0.f, 0.f, 0.f);
            int kp = 0, kn = 0;
            if (miss) {
              p = to_end(i < nS ? F.lflat[i] : F.lsharp[i - nS], tcur, et, im, hasImu);
              put(i, p);
              nbr_keys(i, nS, n, w_at(max(i - 1, 0)), w_at(min(i + 1, n - 1)), kp, kn);
            }
            if (rebuild) build_count(B, i - lane, p, kp, kn, miss != 0);
            miss &= miss - 1;
          }
        }
      }
    };
    // the stream's ring slot (HBM-resident sensors; see "ring"): phase A over
    // the own share (waves 1-7 beside the integrating wave 0; at the first
    // scan every wave), the other shares awaited or stolen; then, when the
    // indexes are rebuilt, the counts and key tables into LDS and phase B
    auto hand_off_ring = [&]() {
      const RingSlot R = ring_slot(ob, rslot);
      const int nS = F.nLF, n = rn, NK = c.N;
      const int TS = fine_T(F.nLF, ob.gTS), TC = fine_T(F.nLS, ob.gTC);
      unsigned* hc = hbm_grid_ends(L);
      auto w_at = [&](int j) { return j < nS ? F.lflat[j].w : F.lsharp[j - nS].w; };
      auto shareA = [&](int j, int u0, int ustep) {
        const int a = j * rper, e = min(n, a + rper);
        for (int i = a + u0; i < e; i += ustep) {
          const bool corner = i >= nS;
          const float4 r = corner ? F.lsharp[i - nS] : F.lflat[i];
          const float wp = w_at(max(i - 1, 0)), wn = w_at(min(i + 1, n - 1));
          const float4 p = init ? r : to_end(r, tcur, et, im, hasImu);
          ring_put(R.P + i, p);
          if (corner) cEnd[i - nS] = p;
          else sEnd[i] = p;
          if (rebuild) {
            ring_add(&R.cnt[(corner ? TS : 0) + fine_bucket(cell_of(p.x), cell_of(p.y), cell_of(p.z), corner ? TC : TS)]);
            int kp, kn;
            nbr_keys(i, nS, n, wp, wn, kp, kn);
            const int k = (int)p.w;
            if (k < 0 || k >= NK || kp > k) {
              ring_max(&R.key[4 * NK + (corner ? 1 : 0)], 1);
            } else {
              const int kk = k + (corner ? NK : 0), jj = i - (corner ? nS : 0);
              if (kp != k) ring_max(&R.key[kk], INT_MAX - jj);
              if (kn != k) ring_max(&R.key[2 * NK + kk], jj + 1);
            }
          }
        }
      };
      auto shareB = [&](int j, int u0, int ustep) {
        const int a = j * rper, e = min(n, a + rper);
        for (int i = a + u0; i < e; i += ustep) {
          const bool corner = i >= nS;
          const float4 p = R.P[i];
          const int bk = (corner ? TS : 0) + fine_bucket(cell_of(p.x), cell_of(p.y), cell_of(p.z), corner ? TC : TS);
          const unsigned pos = hc[bk] + ring_add(&R.fill[bk]);
          ring_put(R.Q + pos, make_float4(p.x, p.y, p.z, __int_as_float(i - (corner ? nS : 0))));
        }
      };
      // every share of a phase done: wave 0 polls the done flags; a share still
      // unclaimed after kStealTicks is claimed and done here by every wave;
      // then one agent acquire before the plain loads of what the shares wrote
      auto wait_shares = [&](unsigned* claim, unsigned* done, auto&& share) {
        const unsigned long long tw0 = wall_clock64();
        for (;;) {
          if (tid < 64) {
            int steal = INT_MAX;
            bool pend = false;
            const bool late = wall_clock64() - tw0 > kStealTicks;
            for (int j = tid; j < rnsh; j += 64) {
              if (ring_peek(&done[j])) continue;
              pend = true;
              if (late && ring_peek(&claim[j]) == 0u) steal = min(steal, j);
            }
            const bool any = __ballot(pend) != 0;
            steal = wave_min_i32(steal);
            // a share claimed but never flagged in kLateTicks (cannot happen: the
            // claimer is running) ends the wait with the batch's error word set
            // rather than hanging the device
            const bool lost = any && wall_clock64() - tw0 > kLateTicks;
            if (tid == 0) {
              if (lost) *ob.xerr = 2u;
              L.n[N_RING] = (!any || lost) ? -1 : (steal != INT_MAX ? steal : -2);
            }
          }
          __syncthreads();
          const int j = L.n[N_RING];
          if (j == -1) break;
          if (j >= 0) {
            if (tid == 0) L.n[N_CLAIM] = ring_claim(&claim[j], (unsigned)ob.wg + 1u);
            __syncthreads();
            if (L.n[N_CLAIM]) {
              share(j, tid, kOdomThreads);
              asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
              __syncthreads();
              if (tid == 0) __hip_atomic_store((gu32*)&done[j], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
          } else if (tid == 0) {
            __builtin_amdgcn_s_sleep(2);
          }
          __syncthreads();
        }
        if (tid == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
      };
      const bool mineA = L.n[N_CLAIM] != 0;  // claimed before the barrier above
      if (mineA && t0 >= 0) shareA(ob.wg, t0, tstep);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();  // wave 0 joins after integrating
      if (mineA && tid == 0)
        __hip_atomic_store((gu32*)&R.doneA[ob.wg], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      wait_shares(R.claimA, R.doneA, shareA);
      if (!rebuild) return;  // the indexes stay on their snapshot (stale: brute force next scan)
      ring_index_lds(L, R, nS, TS, TC, NK, false);  // bucket starts + key tables
      if (tid == 0) L.n[N_CLAIM] = ob.wg < rnsh && ring_claim(&R.claimB[ob.wg], (unsigned)ob.wg + 1u);
      __syncthreads();
      if (L.n[N_CLAIM]) {
        shareB(ob.wg, tid, kOdomThreads);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) __hip_atomic_store((gu32*)&R.doneB[ob.wg], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      wait_shares(R.claimB, R.doneB, shareB);
      for (int bk = tid; bk < TS + TC; bk += kOdomThreads) {  // starts -> ends (corner ends less nS)
        const unsigned e = hc[bk] + R.cnt[bk];
        hc[bk] = bk >= TS ? e - (unsigned)nS : e;
      }
    };
    RP_ADD(S, P_B_SCATTER);
    if (ringMode) {
      hand_off_ring();
    } else if (!RING && hx) {
      if (fits) hand_off_x(BL);
      else hand_off_x(BH);
    } else if (!RING) {
      if (fits) hand_off(BL);
      else hand_off(BH);
    }
    if (prof && tid == 64) prof[P_TOEND_LOOP] += wall_clock64() - tw;  // wave 1's chunks
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's LDS-DMA copies have landed
    if (tid == 0) L.n[N_PRE] = nxt ? 1 : 0;  // read at the next scan's top, after the barriers below
    __syncthreads();
    S.add(P_TOEND);
    if (tid == 0) {
      st->cornerLastNum = F.nLS;
      st->surfLastNum = F.nLF;
      st->curBuf = ringMode ? rslot + 2 : nbuf;
      // the record's flag: this scan's LM ran on HBM-resident last clouds
      if (lead && !init && !st->resident) bb.fa_flags[b] |= LEGO_REC_ODOM_HBM;
      st->resident = fits ? 1 : 0;
      if (hx) st->seq = seq;
      if (ringMode) st->seq = rseq;
      if (rebuild) { st->snapBuf = ringMode ? rslot + 2 : nbuf; st->nnCornerNum = F.nLS; st->nnSurfNum = F.nLF; }
      int pub = 0;
      if (init) {
        st->transformSum[0] += iq.pitchStart;  // checkSystemInitialization :1633-1634
        st->transformSum[2] += iq.rollStart;
        st->inited = 1;
      } else {
        st->frameCount++;
        if (st->frameCount >= c.skip + 1) { st->frameCount = 0; pub = 1; }
      }
      if (lead) {
        ob.validOut[b] = init ? 0 : 1;
        ob.pubOut[b] = pub;
        for (int i = 0; i < 6; ++i) ob.curOut[b * 6 + i] = st->transformCur[i];
        if (ob.integ) {  // the integrating workgroup's input: {tag, transformCur[i]} granules
          const unsigned long long tag = (unsigned long long)(2u * (unsigned)(b + 1) + (init ? 0u : 1u)) << 32;
          for (int i = 0; i < 6; ++i) x_publish(ob.intX + (size_t)b * 6 + i, tag | __float_as_uint(st->transformCur[i]));
        } else {
          for (int i = 0; i < 6; ++i) ob.sumOut[b * 6 + i] = st->transformSum[i];
        }
      }
      __threadfence_block();
    }
    __syncthreads();
    unsigned long long tb = 0;
    if (prof && tid == 0) tb = wall_clock64();
    if (rebuild && !RING) {
      if (fits) build_finish(BL, prof);
      else build_finish(BH, prof);
    }
    if (prof && tid == 0) prof[P_BUILD] += wall_clock64() - tb;
    if (ODOM_RESID_PROBE == 1) S.add(P_B_ENDS);
  }
  __syncthreads();
  // (with the integrating workgroup, transformSum's words 6..11 are its)
  if (lead && tid < (int)(sizeof(OdomState) / 4) && !(ob.integ && tid >= 6 && tid < 12))
    ((int*)ob.st)[tid] = ((const int*)st)[tid];
  if (lead && ob.late >= 0) {  // releases the diagnostic late workgroup
    __syncthreads();
    if (tid == 0) __hip_atomic_store((gu32*)&ob.xerr[1], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (gprof && tid < P_NPROF) gprof[tid] += sprof[tid];
}

// Bucket caps of the HBM-resident grids: both bucket arrays live in LDS
// (kHbmLdsCnt counters), so at most 16 k surf + 8 k corner buckets.
constexpr int kHbmTS = 16384, kHbmTC = 8192;
static_assert(kHbmTS + kHbmTC <= kHbmLdsCnt, "HBM-path grid ends fit the free LDS");
void odom_index_caps(int capCorner, int capSurf, int* gTC, int* gTS) {
  int t = 64;
  while (t < capCorner / 2 && t < kHbmTC) t <<= 1;
  *gTC = t;
  t = 64;
  while (t < capSurf / 2 && t < kHbmTS) t <<= 1;
  *gTS = t;
}

// Workgroups of the odometry launch: LDS-resident sensors split each NN round
// over one wave per query of the largest round (flat <= 24 N queries).
__global__ void k_pack_recs(BatchBufs bb, OdomBufs ob, int B, PackedRec* out) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b > B) return;
  PackedRec r = {};
  if (b == B) {
    r.bad = (int)*ob.xerr;
  } else {
    for (int i = 0; i < 6; ++i) r.sum[i] = ob.sumOut[b * 6 + i];
    r.ns = bb.ns[b];
    for (int i = 0; i < 4; ++i) r.cnt[i] = bb.f_cnt[b * 4 + i];
    r.valid = ob.validOut[b];
    r.flags = bb.fa_flags[b];
    r.bad = bb.bad[b];
    for (int i = 0; i < 6; ++i) r.cur[i] = ob.curOut[b * 6 + i];
    r.pub = ob.pubOut[b];
    r.nout = bb.nout[b];
  }
  out[b] = r;
}

// publishCloudsLast's clouds into the hand-off packet (lego_handoff_pack): one
// y-block row per scan, the entries (offsets, counts) already in the packet.
__global__ void k_pack_handoff(BatchBufs bb, OdomBufs ob, int P, uint8_t* packet) {
  const int b = blockIdx.y;
  const lego_handoff_scan& e = *reinterpret_cast<const lego_handoff_scan*>(packet + sizeof(lego_handoff_hdr) +
                                                                           sizeof(lego_handoff_scan) * b);
  if (!e.publish_to_mapping) return;
  const int nc = e.n_corner_last, ns = e.n_surf_last, no = e.n_outlier_last;
  float4* dst = reinterpret_cast<float4*>(packet + e.offset);
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < nc + ns + no; i += gridDim.x * blockDim.x) {
    float4 p;
    if (i < nc) {
      p = ob.cornerEnd[(size_t)b * ob.capLS + i];
    } else if (i < nc + ns) {
      p = ob.surfEnd[(size_t)b * P + i - nc];
    } else {
      const float4 q = bb.outl[(size_t)b * P + i - nc - ns];
      p = make_float4(q.y, q.z, q.x, q.w);  // adjustOutlierCloud :1746-1757
    }
    dst[i] = p;
  }
}

void launch_pack_handoff(const BatchBufs& bb, const OdomBufs& ob, int B, int P, uint8_t* packet, hipStream_t s) {
  k_pack_handoff<<<dim3(16, B), 256, 0, s>>>(bb, ob, P, packet);
}

void launch_pack_recs(const BatchBufs& bb, const OdomBufs& ob, int B, PackedRec* out, hipStream_t s) {
  k_pack_recs<<<(B + 1 + 63) / 64, 64, 0, s>>>(bb, ob, B, out);
}

// LDS-resident sensors: one wave per query of the corner NN rounds (the sharp
// features, 12 per ring; three of a scan's four rounds) — 24 workgroups for
// VLP-16, whose single surf round then takes two queries per wave (measured
// on C2 with the gridless search: 16 → 13.2 k, 20 → 13.7 k, 24–32 → 14.05 k,
// 40–64 → 13.85–13.95 k scans/s; fewer workgroups also poll fewer
// granules per round).  Larger sensors keep
// their clouds and indexes in HBM, and each workgroup builds its own index
// copy per scan: four queries per wave balance that redundant build against
// the search split (HDL-64E: 48 workgroups; measured 1.4 k scans/s at 192,
// 2.7 k at 48, 2.6 k at 24).  Capped at the CU count.
// LDS-resident sensors: one wave per corner query.  HBM-resident ones (the
// ring): two flat queries per wave, at most 128 workgroups — C3 (HDL-64E,
// 20-scan batches beside the next batch's front end) measured 9.3 / 9.8 /
// 9.8 / 9.0 k scans/s at 64 / 96 / 128 / 160 workgroups, 8.9 k at the four
// queries per wave of round 4 (48; profiles/r05_wg_c3.txt): more workgroups
// shorten the chain's NN rounds and hand-off shares but take CUs from the
// overlapped front end.
int odom_workgroups(int N, int cusAvailable) {
  const bool resident = N * kFlatPerRing <= kLdsQ && N * kSharpPerRing <= kLdsQ / 2;
  int g = resident ? (N * kSharpPerRing + kOdomWaves - 1) / kOdomWaves
                   : (N * kFlatPerRing + 2 * kOdomWaves - 1) / (2 * kOdomWaves);
  if (!resident && g > 128) g = 128;
  return g < cusAvailable ? g : cusAvailable;
}

// The launch's preparation in one kernel (it was two memsets and a copy, each
// a dependent operation on the odometry stream between two k_odom launches):
// the error word, the exchange slots of the rounds this launch can use, and
// the read-only input state (OdomBufs::stIn) from the state the previous
// launch left.
__global__ void k_odom_prep(unsigned* xerr, uint4* xg, size_t xgVec, const uint4* st, uint4* stIn, int stVec,
                            uint4* ix, int ixVec) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x, T = (size_t)gridDim.x * blockDim.x;
  if (t == 0) *xerr = 0u;
  for (size_t i = t; i < xgVec; i += T) xg[i] = make_uint4(0u, 0u, 0u, 0u);
  for (size_t i = t; i < (size_t)ixVec; i += T) ix[i] = make_uint4(0u, 0u, 0u, 0u);  // the integration granules
  for (size_t i = t; i < (size_t)stVec; i += T) stIn[i] = st[i];
}

// Zeroes the control words of the ring slots a launch of K scans per stream
// can pick (ring_next from the state the previous launch left; the launch's
// picks that skip the ring, LDS-resident hand-offs, only shorten that prefix),
// in every copy (OdomBufs::ringCopy).  Block row s = stream s.
__global__ void k_ring_prep(OdomBufs ob, int K) {
  const int s = blockIdx.y;
  const int copies = ob.ringCopy ? 2 : 1;
  unsigned char* base = ob.ring + (size_t)s * copies * ob.ringR * ob.ringStride;
  const size_t words = ob.ringCtl / 16;
  unsigned seq = ob.st[s].seq;
  const int snapBuf = ob.st[s].snapBuf;
  for (int j = 0; j < K; ++j) {
    unsigned nx;
    const int slot = ring_next(seq, snapBuf, ob.ringR, &nx);
    seq = nx;
    for (int cp = 0; cp < copies; ++cp) {
      uint4* w = (uint4*)(base + (size_t)cp * ob.ringCopy + (size_t)slot * ob.ringStride);
      for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < words; i += (size_t)gridDim.x * blockDim.x)
        w[i] = make_uint4(0u, 0u, 0u, 0u);
    }
  }
}

bool odom_ring_sensor(int N) { return !(N * kFlatPerRing <= kLdsQ && N * kSharpPerRing <= kLdsQ / 2); }

int launch_odom(const BatchBufs& bb, const OdomBufs& ob, const DevCfg& c, int K, hipStream_t s, StageTimer* tm,
                unsigned long long* prof, unsigned* lfReady, unsigned long long lfTicks) {
  tm->mark("odom.lm", s);
  if (ob.ring) {
    const int gx = (int)std::min<size_t>(64, (ob.ringCtl / 16 + 255) / 256);
    k_ring_prep<<<dim3(gx, ob.S), 256, 0, s>>>(ob, K);
  }
  // zero the exchange slots of the rounds this launch can use (10 per scan)
  const size_t slot = (size_t)ob.capQ * sizeof(unsigned long long);
  const size_t bytes = ob.G <= 1 ? 0
                       : ob.S == 1 ? std::min<size_t>(ob.roundsCap, (size_t)10 * K) * slot
                                   : (size_t)ob.S * ob.roundsCap * slot;
  static_assert(sizeof(OdomState) % 16 == 0, "OdomState copies as 16-byte words");
  const int stVec = (int)(sizeof(OdomState) * ob.S / 16);
  const size_t xgVec = bytes / 16;  // capQ is even: whole 16-byte words
  const int grid = (int)std::max<size_t>(1, std::min<size_t>(512, (std::max<size_t>(xgVec, stVec) + 255) / 256));
  const int ixVec = ob.integ ? ob.S * K * 6 * 8 / 16 : 0;  // 6 granules of 8 bytes per scan
  k_odom_prep<<<grid, 256, 0, s>>>(ob.xerr, (uint4*)ob.xg, xgVec, (const uint4*)ob.st, (uint4*)ob.stIn, stVec,
                                   (uint4*)ob.intX, ixVec);
  if (ob.late >= 0 && hipMemsetAsync(ob.xerr + 1, 0, sizeof(unsigned), s) != hipSuccess) return -1;
  if (ob.wg >= 0 && ob.G > 1 &&  // the diagnostic silent workgroup's copy (single-stream contexts)
      hipMemsetAsync((unsigned char*)ob.xblock + 16, 0, ob.xbytes - 16, s) != hipSuccess)
    return -1;
  // A plain launch: the exchange needs no co-residency (see "exchange").
  const int blocks = ob.S * ob.G + (ob.integ ? ob.S : 0);  // the chains, then one integrating workgroup per stream
  const size_t lds = odom_lds_bytes();
  if (lfReady) {
    if (ob.ring) k_odom<true, true><<<blocks, kOdomThreads, lds, s>>>(bb, ob, c, K, prof, lfReady, lfTicks);
    else k_odom<false, true><<<blocks, kOdomThreads, lds, s>>>(bb, ob, c, K, prof, lfReady, lfTicks);
  } else {
    if (ob.ring) k_odom<true, false><<<blocks, kOdomThreads, lds, s>>>(bb, ob, c, K, prof, nullptr, 0ull);
    else k_odom<false, false><<<blocks, kOdomThreads, lds, s>>>(bb, ob, c, K, prof, nullptr, 0ull);
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace lego
