// lego_mo.hip — mapOptimization's scan-to-map step on gfx950.
//
// Per mapping step (mapOptmization.cpp:1487-1522 with the loop closure off):
//   k_mo_associate   1 thread: laserOdometryHandler's quaternion -> RPY
//                    (:629-641), transformAssociateToMap (:376-461)
//   VoxelGrid        PCL's filter (voxel_grid.hpp, lego_vg.hip): min/max,
//                    voxel index per point, std::sort's permutation of
//                    (index, point) reproduced (lego_vgsort.h), one lane per
//                    voxel summing its points in that order — the map (once
//                    per installed map) and the scan's corner / surf /
//                    outlier / surf+outlier clouds (:1067-1091)
//   NN index         1 m cells hashed into buckets by a counting sort,
//                    begin/end per bucket (lego_vg.hip); replaces KdTreeFLANN
//                    on the map (:1335-1336).  Every use is thresholded (5th nearest
//                    within 1 m, :1101, :1183), so the 27 cells around a query
//                    hold every candidate; ties resolve to the lower index.
//   per LM iteration (<= 10, :1337-1345):
//     k_mo_rows      one 32-lane group per query: pointAssociateToMap (:513-527), 5-NN
//                    (a lane per cell of the 3x3x3 block, then a group merge),
//                    corner line fit (mean, covariance, 3x3 Jacobi, :1093-1174)
//                    or surf plane fit (5x3 QR, :1176-1227), weight and
//                    Jacobian row (:1244-1270)
//     k_mo_solve     one workgroup: AtA / AtB with double accumulation, 6x6 QR,
//                    iteration-0 eigen degeneracy projection, update,
//                    convergence (:1229-1327); later iterations exit at once
//                    once converged
//   k_mo_finish      transformUpdate (:463-496)
// The fixed map (config C5, lego_mo_set_map) is voxel-filtered and indexed once
// per map: the filter of an unchanged cloud is the same cloud every step.  With
// lego_mo_opts.fixed_map_per_step it is filtered and indexed on every step, the
// work the reference does on its surrounding map (like-for-like timing).
#include <algorithm>
#include <cfloat>
#include <climits>

#include "lego_device.h"
#include "lego_kernels.h"
#include "lego_mo.h"

#include <chrono>
#include <cstdio>

namespace lego {

constexpr unsigned kInvalidKey = 0xffffffffu;
constexpr int kMoSolveThreads = 1024;  // the partials in two rounds of loads (1536 / 1024)

static int grid_for(int n, int bs = 256) {
  int g = (n + bs - 1) / bs;
  return g < 1 ? 1 : (g > 4096 ? 4096 : g);
}

// VoxelGrid and the NN index build: lego_vg.hip.

// The 5 nearest map points with squared distance < 1 (FLANN L2_Simple order),
// sorted by (distance, index), found by a 32-lane group: lane l < 27 scans cell
// l of the 3x3x3 block around the query into its own sorted top 5, then five
// rounds of a group-wide lexicographic minimum pick the overall five (the
// result depends only on the (distance, index) order, not on the split).
// Every lane of the group returns the same list; the count (<= 5) is returned.
#ifndef MO_KNN_LANES
#define MO_KNN_LANES 32
#endif
constexpr int kKnnLanes = MO_KNN_LANES;  // lanes per query (a power of two, <= 32)
__device__ __forceinline__ bool knn_less(float da, int ia, float db, int ib) {
  return da < db || (da == db && ia < ib);
}
// The five rounds of the group's lexicographic (distance, index) minimum over
// the lanes' sorted top-5 lists (ld / li, n entries each).
__device__ __forceinline__ int knn5_merge(const float* ld, const int* li, int n, int* oi, float* od) {
  int head = 0, found = 0;
  for (int r = 0; r < 5; ++r) {
    float cd = head < n ? ld[head] : FLT_MAX;
    int ci = head < n ? li[head] : INT_MAX;
    float md = cd;
    int mi = ci;
    for (int o = kKnnLanes / 2; o > 0; o >>= 1) {
      const float d2 = __shfl_xor(md, o, kKnnLanes);
      const int i2 = __shfl_xor(mi, o, kKnnLanes);
      if (knn_less(d2, i2, md, mi)) { md = d2; mi = i2; }
    }
    if (mi == INT_MAX) break;  // fewer than five points within 1 m
    od[r] = md;
    oi[r] = mi;
    ++found;
    if (head < n && ci == mi) ++head;  // indices are unique: exactly one lane advances
  }
  return found;
}
// point p into the lane's sorted top 5 when it is within 1 m of q
__device__ __forceinline__ void knn5_offer(float4 q, float4 p, float* ld, int* li, int& n) {
  float d2 = 0.f, d;
  d = q.x - p.x; d2 += d * d;
  d = q.y - p.y; d2 += d * d;
  d = q.z - p.z; d2 += d * d;
  if (!(d2 < 1.0f)) return;
  const int id = __float_as_int(p.w);
  if (n == 5 && !knn_less(d2, id, ld[4], li[4])) return;
  int pos = n < 5 ? n++ : 4;
  while (pos > 0 && knn_less(d2, id, ld[pos - 1], li[pos - 1])) {
    ld[pos] = ld[pos - 1];
    li[pos] = li[pos - 1];
    --pos;
  }
  ld[pos] = d2;
  li[pos] = id;
}
// The 5-NN from the query's cached candidates (k_mo_rows): lane l takes
// candidates l, l + 32, l + 64.
__device__ __forceinline__ int knn5_cached(const float4* cand, int nc, float4 q, int* oi, float* od) {
  const int gl = threadIdx.x & (kKnnLanes - 1);
  float ld[5];
  int li[5];
  int n = 0;
  for (int t = gl; t < nc; t += kKnnLanes) knn5_offer(q, cand[t], ld, li, n);
  return knn5_merge(ld, li, n, oi, od);
}

// keep: the query's candidate list to refill (nullptr: none), *kept its count
// via the group's LDS counter (-1 when it overflowed kCand)
__device__ __forceinline__ int knn5_group(const MoIndex& ix, float4 q, int* oi, float* od, float4* keep = nullptr,
                                          int* kept = nullptr) {
  const int gl = threadIdx.x & (kKnnLanes - 1);
  float ld[5];
  int li[5];
  int n = 0;
  for (int cl = gl; cl < 27; cl += kKnnLanes) {  // the 3x3x3 cells over the group's lanes
    const int bx = cell1(q.x) + cl % 3 - 1, by = cell1(q.y) + (cl / 3) % 3 - 1, bz = cell1(q.z) + cl / 9 - 1;
    const unsigned b = mo_cell_hash(bx, by, bz) & (unsigned)(ix.T - 1);
    const int lo = ix.begin[b], hi = ix.end[b];
    for (int t = lo; t < hi; ++t) {
      const float4 p = ix.sorted[t];
      if (cell1(p.x) != bx || cell1(p.y) != by || cell1(p.z) != bz) continue;  // another cell's bucket mate
      if (keep) {  // a candidate of the later iterations: within kCandR of q
        float r2 = 0.f, d;
        d = q.x - p.x; r2 += d * d;
        d = q.y - p.y; r2 += d * d;
        d = q.z - p.z; r2 += d * d;
        if (r2 < kCandR * kCandR) {
          const int k = atomicAdd(kept, 1);
          if (k < kCand) keep[k] = p;
        }
      }
      knn5_offer(q, p, ld, li, n);
    }
  }
  return knn5_merge(ld, li, n, oi, od);
}

// ---------------------------------------------------------------- state
__device__ __forceinline__ void quat_from_rpy(double roll, double pitch, double yaw, double q[4]) {
  const double hy = yaw * 0.5, hp = pitch * 0.5, hr = roll * 0.5;
  const double cy = cos(hy), sy = sin(hy), cp = cos(hp), sp = sin(hp), cr = cos(hr), sr = sin(hr);
  q[0] = sr * cp * cy - cr * sp * sy;
  q[1] = cr * sp * cy + sr * cp * sy;
  q[2] = cr * cp * sy - sr * sp * cy;
  q[3] = cr * cp * cy + sr * sp * sy;
}
// tf::Matrix3x3(q).getRPY, solution 1
__device__ __forceinline__ void rpy_from_quat(double x, double y, double z, double w, double* roll, double* pitch,
                                              double* yaw) {
  const double d = x * x + y * y + z * z + w * w;
  const double s = 2.0 / d;
  const double xs = x * s, ys = y * s, zs = z * s;
  const double wx = w * xs, wy = w * ys, wz = w * zs;
  const double xx = x * xs, xy = x * ys, xz = x * zs;
  const double yy = y * ys, yz = y * zs, zz = z * zs;
  const double m00 = 1.0 - (yy + zz), m10 = xy + wz, m20 = xz - wy, m21 = yz + wx, m22 = 1.0 - (xx + yy);
  if (fabs(m20) >= 1) {
    *yaw = 0;
    const double delta = atan2(m21, m22);
    *pitch = m20 < 0 ? M_PI / 2.0 : -M_PI / 2.0;
    *roll = delta;
  } else {
    *pitch = -asin(m20);
    const double cp = cos(*pitch);
    *roll = atan2(m21 / cp, m22 / cp);
    *yaw = atan2(m10 / cp, m00 / cp);
  }
}

__device__ __forceinline__ void mo_update_trig(MoState* st) {  // updatePointAssociateToMapSinCos :498-511
  const float* t = st->transformTobeMapped;
  st->cRoll = lego_cosf(t[0]); st->sRoll = lego_sinf(t[0]);
  st->cPitch = lego_cosf(t[1]); st->sPitch = lego_sinf(t[1]);
  st->cYaw = lego_cosf(t[2]); st->sYaw = lego_sinf(t[2]);
}

// laserOdometryHandler (:629-641) and transformAssociateToMap (:376-461)
__global__ void k_mo_associate(MoState* st, double qx, double qy, double qz, double qw, double px,
                               double py, double pz) {
  if (threadIdx.x != 0) return;
  double roll, pitch, yaw;
  rpy_from_quat(qz, -qx, -qy, qw, &roll, &pitch, &yaw);
  float* ts = st->transformSum;
  ts[0] = (float)-pitch; ts[1] = (float)-yaw; ts[2] = (float)roll;
  ts[3] = (float)px; ts[4] = (float)py; ts[5] = (float)pz;
  const float* bef = st->transformBefMapped;
  const float* aft = st->transformAftMapped;
  float* tbm = st->transformTobeMapped;
  float* inc = st->transformIncre;
  float x1 = lego_cosf(ts[1]) * (bef[3] - ts[3]) - lego_sinf(ts[1]) * (bef[5] - ts[5]);
  float y1 = bef[4] - ts[4];
  float z1 = lego_sinf(ts[1]) * (bef[3] - ts[3]) + lego_cosf(ts[1]) * (bef[5] - ts[5]);
  float x2 = x1;
  float y2 = lego_cosf(ts[0]) * y1 + lego_sinf(ts[0]) * z1;
  float z2 = -lego_sinf(ts[0]) * y1 + lego_cosf(ts[0]) * z1;
  inc[3] = lego_cosf(ts[2]) * x2 + lego_sinf(ts[2]) * y2;
  inc[4] = -lego_sinf(ts[2]) * x2 + lego_cosf(ts[2]) * y2;
  inc[5] = z2;
  const float sbcx = lego_sinf(ts[0]), cbcx = lego_cosf(ts[0]);
  const float sbcy = lego_sinf(ts[1]), cbcy = lego_cosf(ts[1]);
  const float sbcz = lego_sinf(ts[2]), cbcz = lego_cosf(ts[2]);
  const float sblx = lego_sinf(bef[0]), cblx = lego_cosf(bef[0]);
  const float sbly = lego_sinf(bef[1]), cbly = lego_cosf(bef[1]);
  const float sblz = lego_sinf(bef[2]), cblz = lego_cosf(bef[2]);
  const float salx = lego_sinf(aft[0]), calx = lego_cosf(aft[0]);
  const float saly = lego_sinf(aft[1]), caly = lego_cosf(aft[1]);
  const float salz = lego_sinf(aft[2]), calz = lego_cosf(aft[2]);
  const float srx = -sbcx * (salx * sblx + calx * cblx * salz * sblz + calx * calz * cblx * cblz) -
                    cbcx * sbcy * (calx * calz * (cbly * sblz - cblz * sblx * sbly) -
                                   calx * salz * (cbly * cblz + sblx * sbly * sblz) + cblx * salx * sbly) -
                    cbcx * cbcy * (calx * salz * (cblz * sbly - cbly * sblx * sblz) -
                                   calx * calz * (sbly * sblz + cbly * cblz * sblx) + cblx * cbly * salx);
  tbm[0] = -lego_asinf(srx);
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
  tbm[1] = lego_atan2f(srycrx / lego_cosf(tbm[0]), crycrx / lego_cosf(tbm[0]));
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
  tbm[2] = lego_atan2f(srzcrx / lego_cosf(tbm[0]), crzcrx / lego_cosf(tbm[0]));
  x1 = lego_cosf(tbm[2]) * inc[3] - lego_sinf(tbm[2]) * inc[4];
  y1 = lego_sinf(tbm[2]) * inc[3] + lego_cosf(tbm[2]) * inc[4];
  z1 = inc[5];
  x2 = x1;
  y2 = lego_cosf(tbm[0]) * y1 - lego_sinf(tbm[0]) * z1;
  z2 = lego_sinf(tbm[0]) * y1 + lego_cosf(tbm[0]) * z1;
  tbm[3] = aft[3] - (lego_cosf(tbm[1]) * x2 + lego_sinf(tbm[1]) * z2);
  tbm[4] = aft[4] - y2;
  tbm[5] = aft[5] - (-lego_sinf(tbm[1]) * x2 + lego_cosf(tbm[1]) * z2);
  mo_update_trig(st);
  st->converged = 0;
  st->iterations = 0;
  st->optimized = 0;
}

// scan2MapOptimization's guard (:1331), once the map is filtered
__global__ void k_mo_guard(MoState* st, const MoCounts* cnt) {
  if (threadIdx.x == 0) st->optimized = (cnt->cornerMapDS > 10 && cnt->surfMapDS > 100) ? 1 : 0;
}

// adjustOutlierCloud (featureAssociation.cpp:1746-1757): (x, y, z) -> (y, z, x)
__global__ void k_mo_outlier_in(const float4* raw, int n, float4* out) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const float4 p = raw[i];
    out[i] = make_float4(p.y, p.z, p.x, p.w);
  }
}

// surfTotalLast = surfLastDS + outlierLastDS (:1084-1086)
__global__ void k_mo_concat(const float4* a, const float4* b, MoCounts* cnt, float4* out) {
  const int na = cnt->surfDS, nb = cnt->outlierDS;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < na + nb; i += gridDim.x * blockDim.x)
    out[i] = i < na ? a[i] : b[i - na];
  if (blockIdx.x == 0 && threadIdx.x == 0) cnt->surfTotal = na + nb;
}

// ---------------------------------------------------------------- LM rows
__device__ __forceinline__ float4 associate_to_map(float4 pi, const MoState* st) {  // :513-527
  const float x1 = st->cYaw * pi.x - st->sYaw * pi.y;
  const float y1 = st->sYaw * pi.x + st->cYaw * pi.y;
  const float z1 = pi.z;
  const float x2 = x1;
  const float y2 = st->cRoll * y1 - st->sRoll * z1;
  const float z2 = st->sRoll * y1 + st->cRoll * z1;
  const float* t = st->transformTobeMapped;
  return make_float4(st->cPitch * x2 + st->sPitch * z2 + t[3], y2 + t[4], -st->sPitch * x2 + st->cPitch * z2 + t[5],
                     pi.w);
}

// One 32-lane group per query: corner queries [0, nCornerDS), then
// surf+outlier queries.  Row r = {arx, ary, arz, cf.x, cf.y, cf.z, B, valid},
// written by the group's lane 0 (the fit runs on every lane of the group).
__device__ __forceinline__ bool mo_row(MoState* st, int nC, const float4* cornerDS, const float4* surfTotalDS,
                                       const MoIndex& cornerIx, const MoIndex& surfIx, const float4* cornerMap,
                                       const float4* surfMap, float* rows, int q, double* red, float4* cand,
                                       float4* candRef, int candQ, int it, int* kept) {
  const bool lead = (threadIdx.x & (kKnnLanes - 1)) == 0;
  float* row = rows + (size_t)q * 8;
  if (lead) row[7] = 0.f;
  const bool corner = q < nC;
  const float4 po = corner ? cornerDS[q] : surfTotalDS[q - nC];
  const float4 sel = associate_to_map(po, st);
  int ind[5];
  float sq[5];
  // the query's candidates from its last full search, when it has stayed in
  // that search's cell and within kCandMove of its point (MoDev::cand)
  bool cached = false;
  float4 ref = make_float4(0.f, 0.f, 0.f, -1.f);
  if (it > 0 && q < candQ) {
    ref = candRef[q];
    const float dx = sel.x - ref.x, dy = sel.y - ref.y, dz = sel.z - ref.z;
    cached = ref.w >= 0.f && cell1(sel.x) == cell1(ref.x) && cell1(sel.y) == cell1(ref.y) &&
             cell1(sel.z) == cell1(ref.z) && dx * dx + dy * dy + dz * dz <= kCandMove * kCandMove;
  }
  int found;
  if (cached) {
    found = knn5_cached(cand + (size_t)q * kCand, (int)ref.w, sel, ind, sq);
  } else if (q < candQ) {  // a full search, refilling the query's candidates
    if (lead) *kept = 0;
    __builtin_amdgcn_wave_barrier();
    found = knn5_group(corner ? cornerIx : surfIx, sel, ind, sq, cand + (size_t)q * kCand, kept);
    __builtin_amdgcn_wave_barrier();
    if (lead) {
      const int k = *kept;
      candRef[q] = make_float4(sel.x, sel.y, sel.z, k <= kCand ? (float)k : -1.f);
    }
  } else {
    found = knn5_group(corner ? cornerIx : surfIx, sel, ind, sq);
  }
  if (found < 5) return false;
  float4 cf;
  if (corner) {  // cornerOptimization :1093-1174
    float cx = 0, cy = 0, cz = 0;
    for (int j = 0; j < 5; j++) {
      const float4 m = cornerMap[ind[j]];
      cx += m.x; cy += m.y; cz += m.z;
    }
    cx /= 5; cy /= 5; cz /= 5;
    float a11 = 0, a12 = 0, a13 = 0, a22 = 0, a23 = 0, a33 = 0;
    for (int j = 0; j < 5; j++) {
      const float4 m = cornerMap[ind[j]];
      const float ax = m.x - cx, ay = m.y - cy, az = m.z - cz;
      a11 += ax * ax; a12 += ax * ay; a13 += ax * az;
      a22 += ay * ay; a23 += ay * az; a33 += az * az;
    }
    a11 /= 5; a12 /= 5; a13 /= 5; a22 /= 5; a23 /= 5; a33 /= 5;
    const float A1[3][3] = {{a11, a12, a13}, {a12, a22, a23}, {a13, a23, a33}};
    float D1[3], V1[3][3];
    cv_eigen_sym3(A1, D1, V1);
    if (!(D1[0] > 3 * D1[1])) return false;
    const float x0 = sel.x, y0 = sel.y, z0 = sel.z;
    const float x1 = (float)(cx + 0.1 * (double)V1[0][0]);
    const float y1 = (float)(cy + 0.1 * (double)V1[0][1]);
    const float z1 = (float)(cz + 0.1 * (double)V1[0][2]);
    const float x2 = (float)(cx - 0.1 * (double)V1[0][0]);
    const float y2 = (float)(cy - 0.1 * (double)V1[0][1]);
    const float z2 = (float)(cz - 0.1 * (double)V1[0][2]);
    const float m11 = (x0 - x1) * (y0 - y2) - (x0 - x2) * (y0 - y1);
    const float m22 = (x0 - x1) * (z0 - z2) - (x0 - x2) * (z0 - z1);
    const float m33 = (y0 - y1) * (z0 - z2) - (y0 - y2) * (z0 - z1);
    const float a012 = __builtin_sqrtf(m11 * m11 + m22 * m22 + m33 * m33);
    const float l12 = __builtin_sqrtf((x1 - x2) * (x1 - x2) + (y1 - y2) * (y1 - y2) + (z1 - z2) * (z1 - z2));
    const float la = ((y1 - y2) * m11 + (z1 - z2) * m22) / a012 / l12;
    const float lb = -((x1 - x2) * m11 - (z1 - z2) * m33) / a012 / l12;
    const float lc = -((x1 - x2) * m22 + (y1 - y2) * m33) / a012 / l12;
    const float ld2 = a012 / l12;
    const float s = (float)(1 - 0.9 * (double)lfabsf(ld2));
    if (!((double)s > 0.1)) return false;
    cf = make_float4(s * la, s * lb, s * lc, s * ld2);
  } else {  // surfOptimization :1176-1227
    float A0[5][3];
    const float B0[5] = {-1, -1, -1, -1, -1};
#pragma unroll
    for (int j = 0; j < 5; j++) {
      const float4 m = surfMap[ind[j]];
      A0[j][0] = m.x; A0[j][1] = m.y; A0[j][2] = m.z;
    }
    float X0[3];
    cv_solve_qr<5, 3>(A0, B0, X0);
    float pa = X0[0], pb = X0[1], pc = X0[2], pd = 1;
    const float ps = __builtin_sqrtf(pa * pa + pb * pb + pc * pc);
    pa /= ps; pb /= ps; pc /= ps; pd /= ps;
    for (int j = 0; j < 5; j++) {
      const float4 m = surfMap[ind[j]];
      if ((double)lfabsf(pa * m.x + pb * m.y + pc * m.z + pd) > 0.2) return false;
    }
    const float pd2 = pa * sel.x + pb * sel.y + pc * sel.z + pd;
    const float s = (float)(1 - 0.9 * (double)lfabsf(pd2) /
                                    (double)__builtin_sqrtf(__builtin_sqrtf(sel.x * sel.x + sel.y * sel.y + sel.z * sel.z)));
    if (!((double)s > 0.1)) return false;
    cf = make_float4(s * pa, s * pb, s * pc, s * pd2);
  }
  // LMOptimization's Jacobian row (:1244-1270)
  const float* t = st->transformTobeMapped;
  const float srx = st->sRoll, crx = st->cRoll, sry = st->sPitch, cry = st->cPitch, srz = st->sYaw, crz = st->cYaw;
  (void)t;
  const float arx = (crx * sry * srz * po.x + crx * crz * sry * po.y - srx * sry * po.z) * cf.x +
                    (-srx * srz * po.x - crz * srx * po.y - crx * po.z) * cf.y +
                    (crx * cry * srz * po.x + crx * cry * crz * po.y - cry * srx * po.z) * cf.z;
  const float ary = ((cry * srx * srz - crz * sry) * po.x + (sry * srz + cry * crz * srx) * po.y + crx * cry * po.z) * cf.x +
                    ((-cry * crz - srx * sry * srz) * po.x + (cry * srz - crz * srx * sry) * po.y - crx * sry * po.z) * cf.z;
  const float arz = ((crz * srx * sry - cry * srz) * po.x + (-cry * crz - srx * sry * srz) * po.y) * cf.x +
                    (crx * crz * po.x - crx * srz * po.y) * cf.y +
                    ((sry * srz + cry * crz * srx) * po.x + (crz * sry - cry * srx * srz) * po.y) * cf.z;
  if (lead) {
    row[0] = arx; row[1] = ary; row[2] = arz;
    row[3] = cf.x; row[4] = cf.y; row[5] = cf.z;
    row[6] = -cf.w;
    row[7] = 1.f;
    // the workgroup's AtA / AtB sums (products of floats are exact in double)
    const float ra[7] = {arx, ary, arz, cf.x, cf.y, cf.z, -cf.w};
    int o = 0;
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
      for (int j = i; j < 6; ++j) red[o++] += (double)ra[i] * (double)ra[j];
#pragma unroll
    for (int i = 0; i < 6; ++i) red[21 + i] += (double)ra[i] * (double)ra[6];
    red[27] += 1.0;
  }
  return true;
}

constexpr int kMoRowsThreads = 256, kMoRowsGrid = 1536;
constexpr int kMoSums = 21 + 6 + 1;  // AtA upper triangle, AtB, row count
// One 32-lane group per query; each workgroup also sums its rows' AtA / AtB
// terms in double (products of floats are exact in double) into part[block],
// so k_mo_solve reduces one partial per workgroup instead of every row.
__global__ void __launch_bounds__(kMoRowsThreads, 6) k_mo_rows(  // six waves per SIMD: kMoRowsGrid resident at once
MoState* st, const MoCounts* cnt, const float4* cornerDS,
                                                           const float4* surfTotalDS, MoIndex cornerIx,
                                                           MoIndex surfIx, const float4* cornerMap,
                                                           const float4* surfMap, float* rows, int qcap,
                                                           double* part, float4* cand, float4* candRef, int candQ,
                                                           int it) {
  if (!st->optimized || st->converged) return;
  const int nC = cnt->cornerDS, nQ = min(nC + cnt->surfTotalDS, qcap);
  constexpr int kGroups = kMoRowsThreads / kKnnLanes;
  __shared__ double red[kGroups][kMoSums];
  __shared__ int kept[kGroups];  // a full search's candidate count (mo_row)
  const int g = (int)threadIdx.x / kKnnLanes;
  const bool lead = (threadIdx.x & (kKnnLanes - 1)) == 0;
  if (lead)
    for (int k = 0; k < kMoSums; ++k) red[g][k] = 0.0;
  for (int q0 = blockIdx.x * kGroups; q0 < nQ; q0 += gridDim.x * kGroups) {  // group-uniform
    const int q = q0 + g;
    if (q < nQ)
      mo_row(st, nC, cornerDS, surfTotalDS, cornerIx, surfIx, cornerMap, surfMap, rows, q, red[g], cand, candRef,
             candQ, it, &kept[g]);
  }
  __syncthreads();
  if (threadIdx.x < kMoSums) {
    double sum = 0.0;
#pragma unroll
    for (int w = 0; w < kGroups; ++w) sum += red[w][threadIdx.x];
    part[(size_t)blockIdx.x * kMoSums + threadIdx.x] = sum;
  }
}

// ---------------------------------------------------------------- LM solve
// Wave sum of a double through DPP (see lego_odom.hip).
template <int kCtrl>
__device__ __forceinline__ double mo_dpp(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp((int)b, kCtrl, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), kCtrl, 0xf, 0xf, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double mo_rdlane(double v, int l) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)b, l), hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double mo_wave_sum(double v) {
  v += mo_dpp<0xB1>(v);
  v += mo_dpp<0x4E>(v);
  v += mo_dpp<0x141>(v);
  v += mo_dpp<0x140>(v);
  return (mo_rdlane(v, 0) + mo_rdlane(v, 16)) + (mo_rdlane(v, 32) + mo_rdlane(v, 48));
}

__device__ __forceinline__ void mo_solve_tail(MoState* st, const double* tot, int iterCount, float* ws, int* wsi);

// nb: the partials k_mo_rows wrote (its grid)
__global__ void __launch_bounds__(kMoSolveThreads) k_mo_solve(MoState* st, const double* part, int nb,
                                                             int iterCount) {
  if (!st->optimized || st->converged) return;
  __shared__ double red[kMoSolveThreads / 64][kMoSums];
  __shared__ float ws[6 * 6 * 6 + 16];  // eigen / inverse workspace (thread 0)
  __shared__ int wsi[16];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  double acc[kMoSums];
#pragma unroll
  for (int k = 0; k < kMoSums; ++k) acc[k] = 0.0;
  for (int b = tid; b < nb; b += kMoSolveThreads) {
    const double* pb = part + (size_t)b * kMoSums;
#pragma unroll
    for (int k = 0; k < kMoSums; ++k) acc[k] += pb[k];
  }
#pragma unroll
  for (int k = 0; k < kMoSums; ++k) {
    const double w = mo_wave_sum(acc[k]);
    if (lane == 0) red[wave][k] = w;
  }
  __syncthreads();
  __shared__ double totS[kMoSums];
  if (tid < kMoSums) {  // a thread per quantity over the waves, in wave order
    double sum = 0;
#pragma unroll
    for (int w = 0; w < kMoSolveThreads / 64; ++w) sum += red[w][tid];
    totS[tid] = sum;
  }
  __syncthreads();
  if (tid != 0) return;
  double tot[kMoSums];
#pragma unroll
  for (int k = 0; k < kMoSums; ++k) tot[k] = totS[k];
  mo_solve_tail(st, tot, iterCount, ws, wsi);
}

// LMOptimization (:1229-1327) from the reduced sums, one thread: the 6x6 QR
// solve, the iteration-0 eigen analysis (degeneracy), the update and the
// convergence test.  ws / wsi: LDS workspace of the eigen / inverse.
__device__ __forceinline__ void mo_solve_tail(MoState* st, const double* tot, int iterCount, float* ws, int* wsi) {
  const int M = (int)tot[27];
  st->rowsLast = M;
  st->iterations = iterCount + 1;
  if (M < 50) return;  // LMOptimization returns false: not converged
  float AtA[6][6], AtB[6];
  int o = 0;
#pragma unroll
  for (int i = 0; i < 6; ++i)
#pragma unroll
    for (int j = i; j < 6; ++j) { AtA[i][j] = AtA[j][i] = (float)tot[o++]; }
#pragma unroll
  for (int i = 0; i < 6; ++i) AtB[i] = (float)tot[21 + i];
  float Aq[6][6], X[6];
#pragma unroll
  for (int i = 0; i < 6; ++i)
#pragma unroll
    for (int j = 0; j < 6; ++j) Aq[i][j] = AtA[i][j];
  cv_solve_qr<6, 6>(Aq, AtB, X);
  float (&P)[6][6] = *reinterpret_cast<float(*)[6][6]>(st->matP);
  if (iterCount == 0 && eig_min_above_n<6>(AtA, 100.0)) {
    // every eigenvalue provably above the threshold: the degeneracy test finds
    // nothing, and matP is read only while isDegenerate is set (:1281-1296);
    // the Jacobi (most of this launch's time at iteration 0) is not needed
    st->isDegenerate = 0;
  } else if (iterCount == 0) {
    // eigen / inverse on LDS arrays (their loops index dynamically)
    float (&Ae)[6][6] = *reinterpret_cast<float(*)[6][6]>(ws);
    float (&V)[6][6] = *reinterpret_cast<float(*)[6][6]>(ws + 36);
    float (&V2)[6][6] = *reinterpret_cast<float(*)[6][6]>(ws + 72);
    float (&Vi)[6][6] = *reinterpret_cast<float(*)[6][6]>(ws + 108);
    float (&E)[6] = *reinterpret_cast<float(*)[6]>(ws + 144);
    int (&indR)[6] = *reinterpret_cast<int(*)[6]>(wsi);
    int (&indC)[6] = *reinterpret_cast<int(*)[6]>(wsi + 6);
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
      for (int j = 0; j < 6; ++j) Ae[i][j] = AtA[i][j];
    cv_eigen_sym_ws<6>(Ae, E, V, indR, indC);
    for (int i = 0; i < 6; ++i)
      for (int j = 0; j < 6; ++j) V2[i][j] = V[i][j];
    st->isDegenerate = 0;
    for (int i = 5; i >= 0; i--) {
      if (E[i] < 100) {
        for (int j = 0; j < 6; j++) V2[i][j] = 0;
        st->isDegenerate = 1;
      } else {
        break;
      }
    }
    cv_inv_lu<6>(V, Vi);
    cv_matmul<6>(Vi, V2, P);
  }
  if (st->isDegenerate) {
    float X2[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) X2[i] = X[i];
    cv_matvec<6>(P, X2, X);
  }
  float* t = st->transformTobeMapped;
#pragma unroll
  for (int i = 0; i < 6; i++) t[i] += X[i];
  // pcl::rad2deg(float) = a * 57.29578f
  const double d0 = X[0] * 57.29578f, d1 = X[1] * 57.29578f, d2 = X[2] * 57.29578f;
  const double t0 = X[3] * 100, t1 = X[4] * 100, t2 = X[5] * 100;
  const float deltaR = (float)sqrt(d0 * d0 + d1 * d1 + d2 * d2);
  const float deltaT = (float)sqrt(t0 * t0 + t1 * t1 + t2 * t2);
  mo_update_trig(st);
  if ((double)deltaR < 0.05 && (double)deltaT < 0.05) st->converged = 1;
}

// transformUpdate :463-496.  imuOn: the host's mapOptimization IMU queue had a
// message; imuRoll / imuPitch are imuRollLast / imuPitchLast at
// timeLaserOdometry + scanPeriod.
__global__ void k_mo_finish(MoState* st, int imuOn, float imuRoll, float imuPitch) {
  if (threadIdx.x != 0 || !st->optimized) return;
  if (imuOn) {
    float* t = st->transformTobeMapped;
    t[0] = (float)(0.998 * t[0] + 0.002 * imuPitch);
    t[2] = (float)(0.998 * t[2] + 0.002 * imuRoll);
  }
  for (int i = 0; i < 6; i++) {
    st->transformBefMapped[i] = st->transformSum[i];
    st->transformAftMapped[i] = st->transformTobeMapped[i];
  }
}

// ---------------------------------------------------------------- keyframe map
// extractSurroundingKeyFrames (:1001-1065), radius search part: key poses
// within surroundingKeyframeSearchRadius of the last saved position, in
// (distance, index) order (the kd-tree's sorted radius search; ties unpinned).
constexpr int kKfSortCap = 8192;
__global__ void __launch_bounds__(1024) k_kf_select(MoKeyframes kf, float radius) {
  __shared__ unsigned long long keys[kKfSortCap];
  __shared__ int nHit;
  const int tid = threadIdx.x;
  const int K = kf.meta[KF_K];
  if (tid == 0) { nHit = 0; kf.meta[KF_HITOVF] = 0; }
  __syncthreads();
  const float cx = kf.robot[3], cy = kf.robot[4], cz = kf.robot[5];
  const double r = (double)radius;
  for (int i = tid; i < K; i += blockDim.x) {
    const float4 p = kf.pos3[i];
    float d = 0.f, e;
    e = cx - p.x; d += e * e;
    e = cy - p.y; d += e * e;
    e = cz - p.z; d += e * e;
    if ((double)d <= r * r) {
      const int j = atomicAdd(&nHit, 1);
      if (j < kKfSortCap) keys[j] = ((unsigned long long)__float_as_uint(d) << 32) | (unsigned)i;
    }
  }
  __syncthreads();
  const int n = min(nHit, kKfSortCap);
  int np = 1;
  while (np < n) np <<= 1;
  for (int i = n + tid; i < np; i += blockDim.x) keys[i] = ~0ull;
  __syncthreads();
  for (int k = 2; k <= np; k <<= 1)  // bitonic sort, ascending (distance >= 0: bits order = value order)
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = tid; i < np; i += blockDim.x) {
        const int l = i ^ j;
        if (l > i) {
          const unsigned long long a = keys[i], b = keys[l];
          if (((i & k) == 0) == (a > b)) { keys[i] = b; keys[l] = a; }
        }
      }
      __syncthreads();
    }
  for (int i = tid; i < n; i += blockDim.x) kf.sur[i] = kf.pos3[(int)(keys[i] & 0xffffffffu)];
  if (tid == 0) {
    kf.meta[KF_NSUR] = n;
    if (nHit > kKfSortCap) kf.meta[KF_HITOVF] = 1;  // the step is refused (MO_E_RADIUS_HITS)
  }
}

// The existing-key bookkeeping (erase the keys no longer around, append the
// new ones in filtered order) and the concatenation plan: per existing key its
// corner offset and its surf + outlier offset in the map clouds.
__global__ void k_kf_plan(MoKeyframes kf) {
  if (threadIdx.x != 0) return;
  const int nSurDS = kf.meta[KF_NSURDS];
  int nEx = kf.meta[KF_NEX], w = 0;
  for (int i = 0; i < nEx; ++i) {
    const int id = kf.exID[i];
    bool exist = false;
    for (int j = 0; j < nSurDS && !exist; ++j) exist = (int)kf.surDS[j].w == id;
    if (exist) kf.exID[w++] = id;
  }
  nEx = w;
  for (int j = 0; j < nSurDS; ++j) {
    const int key = (int)kf.surDS[j].w;
    bool exist = false;
    for (int i = 0; i < nEx && !exist; ++i) exist = kf.exID[i] == key;
    if (!exist && nEx < kf.kcap) kf.exID[nEx++] = key;
  }
  int oc = 0, os = 0;
  for (int i = 0; i < nEx; ++i) {
    const int key = kf.exID[i];
    kf.plan[4 * i + 0] = key;
    kf.plan[4 * i + 1] = oc;
    kf.plan[4 * i + 2] = os;
    oc += kf.seg[6 * key + 1];
    os += kf.seg[6 * key + 3] + kf.seg[6 * key + 5];
  }
  kf.meta[KF_NEX] = nEx;
  kf.meta[KF_NCM] = oc;
  kf.meta[KF_NSM] = os;
}

// transformPointCloud (:529-575) of every planned key's clouds into the map
// clouds, one workgroup per key: corner, then surf followed by outlier.  The
// pose is the key's current one, or (planPose) the one the recent-keyframe
// queue transformed it with when it was queued (:961-999).
__global__ void k_kf_gather(MoKeyframes kf, const float* planPose, float4* cornerFromMap, float4* surfFromMap) {
  const int i = blockIdx.x;
  const int key = kf.plan[4 * i + 0], oc = kf.plan[4 * i + 1], os = kf.plan[4 * i + 2];
  const float* pose = planPose ? planPose + 6 * i : kf.pose6 + 6 * key;
  const float ctRoll = lego_cosf(pose[3]), stRoll = lego_sinf(pose[3]);
  const float ctPitch = lego_cosf(pose[4]), stPitch = lego_sinf(pose[4]);
  const float ctYaw = lego_cosf(pose[5]), stYaw = lego_sinf(pose[5]);
  const float tx = pose[0], ty = pose[1], tz = pose[2];
  auto tf = [&](float4 p) {
    const float x1 = ctYaw * p.x - stYaw * p.y;
    const float y1 = stYaw * p.x + ctYaw * p.y;
    const float z1 = p.z;
    const float x2 = x1;
    const float y2 = ctRoll * y1 - stRoll * z1;
    const float z2 = stRoll * y1 + ctRoll * z1;
    return make_float4(ctPitch * x2 + stPitch * z2 + tx, y2 + ty, -stPitch * x2 + ctPitch * z2 + tz, p.w);
  };
  const int* sg = kf.seg + 6 * key;
  for (int j = threadIdx.x; j < sg[1]; j += blockDim.x) cornerFromMap[oc + j] = tf(kf.arena[sg[0] + j]);
  for (int j = threadIdx.x; j < sg[3]; j += blockDim.x) surfFromMap[os + j] = tf(kf.arena[sg[2] + j]);
  for (int j = threadIdx.x; j < sg[5]; j += blockDim.x) surfFromMap[os + sg[3] + j] = tf(kf.arena[sg[4] + j]);
}

// saveKeyFramesAndFactor (:1353-1454) with iSAM2's chain estimate: keyframe
// decision, pose append, arena slots for this step's filtered clouds.
__global__ void k_kf_save(MoKeyframes kf, MoState* st, const MoCounts* cnt, double stamp) {
  if (threadIdx.x != 0) return;
  float* prev = kf.robot;
  float* cur = kf.robot + 3;
  const float* aft = st->transformAftMapped;
  cur[0] = aft[3]; cur[1] = aft[4]; cur[2] = aft[5];
  const float dx = prev[0] - cur[0], dy = prev[1] - cur[1], dz = prev[2] - cur[2];
  const bool save = !(__builtin_sqrtf(dx * dx + dy * dy + dz * dz) < 0.3f);
  const int K = kf.meta[KF_K];
  kf.meta[KF_SAVED] = 0;  // no copy unless saved
  if (!save && K > 0) return;
  const int top = kf.meta[KF_TOP];
  const int nc = cnt->cornerDS, ns = cnt->surfDS, no = cnt->outlierDS;
  if (K >= kf.kcap || top + nc + ns + no > kf.acap) {
    kf.meta[KF_OVF] = 1;
    return;
  }
  prev[0] = cur[0]; prev[1] = cur[1]; prev[2] = cur[2];
  const float* est = K == 0 ? st->transformTobeMapped : aft;
  float e[6];
  for (int i = 0; i < 6; ++i) e[i] = est[i];
  kf.pos3[K] = make_float4(e[3], e[4], e[5], (float)K);
  float* p6 = kf.pose6 + 6 * K;
  p6[0] = e[3]; p6[1] = e[4]; p6[2] = e[5]; p6[3] = e[0]; p6[4] = e[1]; p6[5] = e[2];
  kf.time[K] = stamp;  // thisPose6D.time = timeLaserOdometry (:1424)
  if (K + 1 > 1)
    for (int i = 0; i < 6; ++i) st->transformTobeMapped[i] = aft[i];
  int* sg = kf.seg + 6 * K;
  sg[0] = top; sg[1] = nc; sg[2] = top + nc; sg[3] = ns; sg[4] = top + nc + ns; sg[5] = no;
  kf.meta[KF_TOP] = top + nc + ns + no;
  kf.meta[KF_K] = K + 1;
  kf.meta[KF_SAVED] = 1;
}
__global__ void k_kf_copy(MoKeyframes kf, const float4* cornerDS, const float4* surfDS, const float4* outlierDS) {
  if (!kf.meta[KF_SAVED]) return;
  const int* sg = kf.seg + 6 * (kf.meta[KF_K] - 1);
  for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < sg[1] + sg[3] + sg[5]; j += gridDim.x * blockDim.x) {
    float4 p;
    if (j < sg[1]) p = cornerDS[j];
    else if (j < sg[1] + sg[3]) p = surfDS[j - sg[1]];
    else p = outlierDS[j - sg[1] - sg[3]];
    kf.arena[sg[0] + j] = p;
  }
}

enum { EV_MAP_FORK, EV_MAP_CORNER, EV_SCAN_FORK, EV_SCAN_CORNER, EV_SURF, EV_SCAN_DONE };

static bool fork_wait(MoDev& m, int ev, hipStream_t from, hipStream_t to) {
  return hipEventRecord(m.ev[ev], from) == hipSuccess && hipStreamWaitEvent(to, m.ev[ev], 0) == hipSuccess;
}

// The map's VoxelGrids (corner 0.2 m, surf 0.4 m, :1058-1064) and NN indexes
// (:1333-1334): the surf cloud on s, the corner cloud on f; joined on s here
// when `join` (installing a map), else by the step's join_scan (f = fork[1],
// after the scan's surf cloud there).
static int map_filter(MoDev& m, const float4* corner, int nC, const float4* surf, int nS, hipStream_t s,
                      hipStream_t f, bool join) {
  // enqueued longest first: the host's launches take longer than the GPU's
  // short kernels, so the order of enqueueing is the order the chains start
  if (hipEventRecord(m.ev[EV_MAP_FORK], s) != hipSuccess) return -1;
  if (voxel_grid_device(surf, nS, nullptr, 0.4f, m.surfMapDS, &m.cnt->surfMapDS, m.vg, s)) return -1;
  if (index_build_device(m.surfMapDS, nS, &m.cnt->surfMapDS, m.surfIx, m.vg, s)) return -1;
  if (hipStreamWaitEvent(f, m.ev[EV_MAP_FORK], 0) != hipSuccess) return -1;
  const bool ok = voxel_grid_device(corner, nC, nullptr, 0.2f, m.cornerMapDS, &m.cnt->cornerMapDS, m.vgMap2, f) == 0 &&
                  index_build_device(m.cornerMapDS, nC, &m.cnt->cornerMapDS, m.cornerIx, m.vgMap2, f) == 0;
  if (!join) return ok ? 0 : -1;  // the step's join_scan joins f (also on failure)
  return fork_wait(m, EV_MAP_CORNER, f, s) && ok ? 0 : -1;  // joined on failure too
}

// downsampleCurrentScan (:1067-1091) forked off s at EV_SCAN_FORK, in two
// parts around the map's launches so that every chain starts early (the
// host's launches are serial): first the outlier cloud on fork[0] and the
// surf cloud on fork[1] (the map's corner cloud follows it there); after the
// map's launches the concatenation, its VoxelGrid and the corner cloud's on
// fork[0] (after the outlier cloud and, through EV_SURF, the surf cloud);
// join_scan makes s wait for the forks.  The three chains come out about
// equal on C5 (r04o VoxelGrid times alone: outlier 0.42 + surf+outlier 0.36 +
// corner 0.11 ms; surf 0.35 + map corner 0.62 ms; map surf 0.93 ms); with the
// map's corner cloud after the outlier cloud fork[0] was the longest.
// (Enqueueing the concatenation before the map's launches delayed the map's
// surf cloud by the host's ~0.3 ms: 2.6 vs 2.3 ms in round 3.)
// (Two forks: with the step's stream that is three hardware queues, as many
// as a process gets besides the runtime's own; a third fork shared one.)
static int scan_filter_begin(MoDev& m, const MoStepArgs& a) {
  const hipStream_t f0 = m.fork[0], f1 = m.fork[1];
  if (hipStreamWaitEvent(f0, m.ev[EV_SCAN_FORK], 0) != hipSuccess) return -1;
  if (hipStreamWaitEvent(f1, m.ev[EV_SCAN_FORK], 0) != hipSuccess) return -1;
  if (a.outlierRaw && a.nOutlier > 0)
    k_mo_outlier_in<<<grid_for(a.nOutlier), 256, 0, f0>>>(a.outlierRaw, a.nOutlier, m.outlierLast);
  if (voxel_grid_device(m.outlierLast, a.nOutlier, nullptr, 0.4f, m.outlierDS, &m.cnt->outlierDS, m.vgScan2, f0))
    return -1;
  if (voxel_grid_device(a.surf ? a.surf : m.surfLast, a.nSurf, nullptr, 0.4f, m.surfDS, &m.cnt->surfDS, m.vgScan1, f1))
    return -1;
  if (hipEventRecord(m.ev[EV_SURF], f1) != hipSuccess) return -1;
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
static int scan_filter_end(MoDev& m, const MoStepArgs& a, bool cornerOnF0) {
  const hipStream_t f0 = m.fork[0];
  if (hipStreamWaitEvent(f0, m.ev[EV_SURF], 0) != hipSuccess) return -1;
  k_mo_concat<<<grid_for(a.nSurf + a.nOutlier), 256, 0, f0>>>(m.surfDS, m.outlierDS, m.cnt, m.surfTotal);
  if (voxel_grid_device(m.surfTotal, a.nSurf + a.nOutlier, &m.cnt->surfTotal, 0.4f, m.surfTotalDS,
                        &m.cnt->surfTotalDS, m.vgScan2, f0))
    return -1;
  // the scan's corner cloud (:1069-1073) last on fork[0] when s filters a
  // map this step (its surf cloud is then the longest chain)
  if (cornerOnF0 &&
      voxel_grid_device(a.corner ? a.corner : m.cornerLast, a.nCorner, nullptr, 0.2f, m.cornerDS, &m.cnt->cornerDS,
                        m.vgScan2, f0))
    return -1;
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
static int join_scan(MoDev& m, hipStream_t s) {
  return fork_wait(m, EV_SCAN_CORNER, m.fork[0], s) && fork_wait(m, EV_SCAN_DONE, m.fork[1], s) ? 0 : -1;
}

static int kf_map_filter(MoDev& m, int nCM, int nSM, hipStream_t s) {
  return map_filter(m, m.cornerFromMap, nCM, m.surfFromMap, nSM, s, m.fork[1], false);
}

// The surrounding map of the keyframe store, filtered and indexed.
static int kf_map(MoDev& m, float radius, hipStream_t s) {
  MoKeyframes& kf = m.kf;
  k_kf_select<<<1, 1024, 0, s>>>(kf, radius);
  if (voxel_grid_device(kf.sur, kf.kcap, &kf.meta[KF_NSUR], 1.0f, kf.surDS, &kf.meta[KF_NSURDS], m.vg, s))
    return -1;
  k_kf_plan<<<1, 64, 0, s>>>(kf);
  int meta[kKfMeta];
  if (hipMemcpyAsync(meta, kf.meta, sizeof(meta), hipMemcpyDeviceToHost, s) != hipSuccess) return -1;
  if (hipStreamSynchronize(s) != hipSuccess) return -1;
  if (meta[KF_OVF]) return MO_E_STORE_FULL;
  if (meta[KF_HITOVF]) return MO_E_RADIUS_HITS;
  if (meta[KF_NCM] > m.fromMapCap || meta[KF_NSM] > m.fromMapCap) return MO_E_MAP_CAP;
  if (meta[KF_NEX] > 0) k_kf_gather<<<meta[KF_NEX], 256, 0, s>>>(kf, nullptr, m.cornerFromMap, m.surfFromMap);
  return kf_map_filter(m, meta[KF_NCM], meta[KF_NSM], s);
}

// The recent-keyframe map of loopClosureEnableFlag (:961-999): the host's
// queue plan (kf.plan / kf.planPose, uploaded on stream s) of nPlan keys.
static int kf_map_recent(MoDev& m, const MoStepArgs& a, hipStream_t s) {
  if (a.nCM > m.fromMapCap || a.nSM > m.fromMapCap) return MO_E_MAP_CAP;
  if (a.nPlan > 0) k_kf_gather<<<a.nPlan, 256, 0, s>>>(m.kf, m.kf.planPose, m.cornerFromMap, m.surfFromMap);
  return kf_map_filter(m, a.nCM, a.nSM, s);
}

// lego_ctx_opts::mo_hostprof (diagnostic): the host's enqueue time of the
// step's parts to stderr (map, scan VoxelGrids, LM).
#define MO_HOSTPROF(k)                                                                                  \
  if (m.hostprof) {                                                                                     \
    hp[k] = std::chrono::steady_clock::now();                                                           \
    if (k == 3)                                                                                         \
      std::fprintf(stderr, "mo enqueue us: map %.0f scan %.0f lm %.0f\n",                              \
                   std::chrono::duration<double, std::micro>(hp[1] - hp[0]).count(),                    \
                   std::chrono::duration<double, std::micro>(hp[2] - hp[1]).count(),                    \
                   std::chrono::duration<double, std::micro>(hp[3] - hp[2]).count());                   \
  }

// lego_ctx_opts::mo_evprof (diagnostic): timing events at the step's start
// and at the end of each chain (s: the map's surf cloud; fork[1]: surf, map
// corner; fork[0]: outlier, surf + outlier, corner), after the join and after
// the LM; mo_evprof_print writes their offsets (us) to stderr.
static void evprof(MoDev& m, int k, hipStream_t st) {
  if (!m.evprof) return;
  if (!m.prof[k] && hipEventCreate(&m.prof[k]) != hipSuccess) return;
  (void)hipEventRecord(m.prof[k], st);
}
void mo_evprof_print(MoDev& m) {
  if (!m.evprof || !m.prof[0]) return;
  static const char* names[6] = {"start", "s_map_surf", "f1_surf_mapcorner", "f0_outlier_total_corner", "join", "lm"};
  std::fprintf(stderr, "mo evprof us:");
  for (int k = 1; k < 6; ++k) {
    float ms = -1.f;
    if (m.prof[k] && hipEventElapsedTime(&ms, m.prof[0], m.prof[k]) != hipSuccess) ms = -1.f;
    std::fprintf(stderr, " %s %.0f", names[k], ms * 1000.f);
  }
  std::fprintf(stderr, "\n");
}

int mo_step_device(MoDev& m, const MoStepArgs& a, bool fixedMap, float radius, hipStream_t s) {
  std::chrono::steady_clock::time_point hp[4];
  evprof(m, 0, s);
  k_mo_associate<<<1, 64, 0, s>>>(m.st, a.quat[0], a.quat[1], a.quat[2], a.quat[3], a.pos[0], a.pos[1], a.pos[2]);
  if (hipGetLastError() != hipSuccess) return -1;
  MO_HOSTPROF(0);
  // the scan's VoxelGrids fork here: they need only the uploaded clouds
  if (hipEventRecord(m.ev[EV_SCAN_FORK], s) != hipSuccess) return -1;
  // Any return from here on first joins the forks into s: the next step's
  // uploads on s must not overwrite clouds a fork still reads.
  auto fail = [&](int st) {
    (void)join_scan(m, s);
    return st;
  };
  if (scan_filter_begin(m, a)) return fail(-1);
  if (!fixedMap && a.nPlan >= 0) {  // extractSurroundingKeyFrames, loop-closure branch :961-999
    const int st = kf_map_recent(m, a, s);
    if (st) return fail(st);
  } else if (!fixedMap) {  // extractSurroundingKeyFrames :1001-1065
    const int st = kf_map(m, radius, s);
    if (st) return fail(st);
  } else if (m.mapPerStep) {  // the map VoxelGrids (:1058-1064) and kd-tree builds (:1333-1334) of every step
    if (map_filter(m, m.cornerMap, m.nCornerMap, m.surfMap, m.nSurfMap, s, m.fork[1], false)) return fail(-1);
  }
  evprof(m, 1, s);
  evprof(m, 2, m.fork[1]);
  MO_HOSTPROF(1);
  // an installed map filtered once leaves s idle: the corner cloud runs there
  const bool mapOnS = !fixedMap || m.mapPerStep;
  if (scan_filter_end(m, a, mapOnS)) return fail(-1);
  if (!mapOnS && voxel_grid_device(a.corner ? a.corner : m.cornerLast, a.nCorner, nullptr, 0.2f, m.cornerDS,
                                   &m.cnt->cornerDS, m.vg, s))
    return fail(-1);
  evprof(m, 3, m.fork[0]);
  if (join_scan(m, s)) return -1;
  evprof(m, 4, s);
  MO_HOSTPROF(2);
  k_mo_guard<<<1, 64, 0, s>>>(m.st, m.cnt);
  // scan2MapOptimization :1329-1350 — the iterations exit on the device once converged
  const int qcap = a.nCorner + a.nSurf + a.nOutlier;
  if (qcap > m.rowCap) return -1;
  // qcap bounds the filtered query count from above (the raw clouds): 1536
  // workgroups (six per CU) cover C5's ~12 k queries in one pass and keep
  // thousands of empty workgroups off the dispatcher; larger clouds loop
  const int nb = qcap > 0 ? std::min(grid_for(qcap, kMoRowsThreads / kKnnLanes), kMoRowsGrid) : 0;
  if (nb > m.partCap) return -1;
  for (int it = 0; it < 10; ++it) {
    if (qcap > 0)
      k_mo_rows<<<nb, kMoRowsThreads, 0, s>>>(m.st, m.cnt, m.cornerDS, m.surfTotalDS, m.cornerIx, m.surfIx,
                                                m.cornerMapDS, m.surfMapDS, m.rows, qcap, m.part, m.cand, m.candRef,
                                                m.candQ, it);
    k_mo_solve<<<1, kMoSolveThreads, 0, s>>>(m.st, m.part, nb, it);
  }
  k_mo_finish<<<1, 64, 0, s>>>(m.st, a.imuOn, a.imuRoll, a.imuPitch);
  evprof(m, 5, s);
  MO_HOSTPROF(3);
  if (!fixedMap) {  // saveKeyFramesAndFactor :1353-1454
    k_kf_save<<<1, 64, 0, s>>>(m.kf, m.st, m.cnt, a.stamp);
    k_kf_copy<<<grid_for(qcap), 256, 0, s>>>(m.kf, m.cornerDS, m.surfDS, m.outlierDS);
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Installs a fixed map: voxel filter (corner 0.2 m, surf 0.4 m, :1062-1064) and
// NN index, once.
int mo_set_map_device(MoDev& m, int nCornerMap, int nSurfMap, hipStream_t s) {
  return map_filter(m, m.cornerMap, nCornerMap, m.surfMap, nSurfMap, s, m.fork[0], true);
}

}  // namespace lego
