// lego_oracle.cpp — TEST INFRASTRUCTURE ONLY (see lego_oracle.h).
//
// A sequential, line-by-line CPU restatement of LeGO-LOAM's per-scan hot path:
//   imageProjection.cpp:163-460     (projection, ground, BFS segmentation)
//   featureAssociation.cpp:491-784  (deskew, curvature, occlusion, extraction)
//   featureAssociation.cpp:860-1032, 1044-1478, 1605-1815 (two-step LM odometry)
// Third-party arithmetic (glibc libm, OpenCV solvers) comes from the shared
// restatement lego-loam_amd/csrc/lego_numerics.h; std::sort is libstdc++'s own.
// Compiled with -O2 -ffp-contract=off (the reference builds without FMA).
#include "lego_oracle.h"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <deque>
#include <limits>
#include <memory>
#include <vector>

#include "../lego-loam_amd/csrc/lego_numerics.h"
#include "../lego-loam_amd/csrc/lego_icp.h"
#include "../lego-loam_amd/csrc/lego_pgo_host.h"

using lego::lego_atan2f;
using lego::lego_cosf;
using lego::lego_sinf;
using lego::lego_asinf;

namespace oracle {

// ============================================================ config presets
// utility.h:53-136 (float constants evaluated exactly as the C++ initialisers).
int sensor_preset(const char* name, lego_sensor_cfg* o) {
  if (!name || !o) return LEGO_E_ARG;
  std::memset(o, 0, sizeof(*o));
  if (!std::strcmp(name, "VLP-16")) {  // utility.h:63-68
    o->n_scan = 16; o->horizon_scan = 1800; o->ang_res_x = 0.2f; o->ang_res_y = 2.0f;
    o->ang_bottom = (float)(15.0 + 0.1); o->ground_scan_ind = 7;
  } else if (!std::strcmp(name, "HDL-32E")) {  // utility.h:71-76
    o->n_scan = 32; o->horizon_scan = 1800; o->ang_res_x = (float)(360.0 / (float)1800);
    o->ang_res_y = (float)(41.33 / (float)(32 - 1)); o->ang_bottom = 30.67f; o->ground_scan_ind = 20;
  } else if (!std::strcmp(name, "VLS-128")) {  // utility.h:79-84
    o->n_scan = 128; o->horizon_scan = 1800; o->ang_res_x = 0.2f; o->ang_res_y = 0.3f;
    o->ang_bottom = 25.0f; o->ground_scan_ind = 10;
  } else if (!std::strcmp(name, "OS1-16")) {  // utility.h:89-94
    o->n_scan = 16; o->horizon_scan = 1024; o->ang_res_x = (float)(360.0 / (float)1024);
    o->ang_res_y = (float)(33.2 / (float)(16 - 1)); o->ang_bottom = (float)(16.6 + 0.1);
    o->ground_scan_ind = 7;
  } else if (!std::strcmp(name, "OS1-64")) {  // utility.h:97-102
    o->n_scan = 64; o->horizon_scan = 1024; o->ang_res_x = (float)(360.0 / (float)1024);
    o->ang_res_y = (float)(33.2 / (float)(64 - 1)); o->ang_bottom = (float)(16.6 + 0.1);
    o->ground_scan_ind = 15;
  } else if (!std::strcmp(name, "HDL-64E")) {
    // No preset in the reference (README.md:86).  KITTI-shaped: 64 rings over
    // [-24.8, +2.0] deg, 2048 columns; groundScanInd = last ring that still
    // points below -1 deg (a 1.7 m mount reaches the ground within ~100 m).
    o->n_scan = 64; o->horizon_scan = 2048; o->ang_res_x = (float)(360.0 / (float)2048);
    o->ang_res_y = (float)(26.8 / (float)(64 - 1)); o->ang_bottom = 24.8f;
    o->ground_scan_ind = 55;
  } else {
    return LEGO_E_ARG;
  }
  o->use_cloud_ring = 1;
  o->sensor_minimum_range = 1.0f;
  o->sensor_mount_angle = 0.0f;
  o->segment_theta = (float)(60.0 / 180.0 * M_PI);
  o->segment_valid_point_num = 5;
  o->segment_valid_line_num = 3;
  o->segment_alpha_x = (float)(o->ang_res_x / 180.0 * M_PI);
  o->segment_alpha_y = (float)(o->ang_res_y / 180.0 * M_PI);
  o->edge_threshold = 0.1f;
  o->surf_threshold = 0.1f;
  o->nearest_feature_search_sq_dist = 25.f;
  o->scan_period = 0.1f;
  o->mapping_process_interval = 0.3;
  o->surrounding_keyframe_search_radius = 50.0f;
  o->skip_frame_num = 1;
  return LEGO_OK;
}

using Pt = lego_point_xyzi;

// ============================================================ VoxelGrid
// pcl::VoxelGrid<PointXYZI>::applyFilter (PCL 1.8, downsample_all_data_=true,
// min_points_per_voxel_=0).  In-voxel summation order: PCL std::sorts the
// (idx, point) pairs by idx only, so equal-idx order is libstdc++ introsort's
// (pcl_sort=1 reproduces it, the product's order: lego_vgsort.h); pcl_sort=0
// sums in input order (std::stable_sort), kept for comparison.
void voxel_grid(const std::vector<Pt>& in, float leaf, bool pcl_sort, std::vector<Pt>& out) {
  out.clear();
  if (in.empty()) return;
  const float inv = 1.0f / leaf;
  float minp[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, maxp[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
  for (const Pt& p : in) {
    if (!std::isfinite(p.x) || !std::isfinite(p.y) || !std::isfinite(p.z)) continue;
    const float v[3] = {p.x, p.y, p.z};
    for (int k = 0; k < 3; ++k) {
      minp[k] = std::min(minp[k], v[k]);
      maxp[k] = std::max(maxp[k], v[k]);
    }
  }
  int64_t dx = (int64_t)((maxp[0] - minp[0]) * inv) + 1;
  int64_t dy = (int64_t)((maxp[1] - minp[1]) * inv) + 1;
  int64_t dz = (int64_t)((maxp[2] - minp[2]) * inv) + 1;
  if (dx * dy * dz > (int64_t)std::numeric_limits<int32_t>::max()) {
    out = in;  // PCL: "Leaf size is too small ... Integer indices would overflow"
    return;
  }
  int minb[3], maxb[3];
  for (int k = 0; k < 3; ++k) {
    minb[k] = (int)std::floor(minp[k] * inv);
    maxb[k] = (int)std::floor(maxp[k] * inv);
  }
  const int divb0 = maxb[0] - minb[0] + 1, divb1 = maxb[1] - minb[1] + 1;
  struct Idx { int idx; unsigned cpi; bool operator<(const Idx& o) const { return idx < o.idx; } };
  std::vector<Idx> iv;
  iv.reserve(in.size());
  for (size_t i = 0; i < in.size(); ++i) {
    const Pt& p = in[i];
    if (!std::isfinite(p.x) || !std::isfinite(p.y) || !std::isfinite(p.z)) continue;
    int i0 = (int)(std::floor(p.x * inv) - (float)minb[0]);
    int i1 = (int)(std::floor(p.y * inv) - (float)minb[1]);
    int i2 = (int)(std::floor(p.z * inv) - (float)minb[2]);
    iv.push_back({i0 + i1 * divb0 + i2 * divb0 * divb1, (unsigned)i});
  }
  if (const char* dump = std::getenv("LEGO_ORACLE_VG_DUMP")) {  // diagnostic: the sort's keys, per call
    if (FILE* f = std::fopen(dump, "ab")) {
      const int32_t m = (int32_t)iv.size();
      std::fwrite(&m, 4, 1, f);
      for (const Idx& e : iv) std::fwrite(&e.idx, 4, 1, f);
      std::fclose(f);
    }
  }
  if (pcl_sort) std::sort(iv.begin(), iv.end(), std::less<Idx>());
  else std::stable_sort(iv.begin(), iv.end(), std::less<Idx>());
  size_t idx = 0;
  while (idx < iv.size()) {
    size_t j = idx + 1;
    while (j < iv.size() && iv[j].idx == iv[idx].idx) ++j;
    float c[4] = {0, 0, 0, 0};
    for (size_t l = idx; l < j; ++l) {
      const Pt& p = in[iv[l].cpi];
      c[0] += p.x; c[1] += p.y; c[2] += p.z; c[3] += p.intensity;
    }
    const float cnt = (float)(j - idx);
    out.push_back({c[0] / cnt, c[1] / cnt, c[2] / cnt, c[3] / cnt});
    idx = j;
  }
}

// ============================================================ kd-tree
// Exact nearest-neighbour search as pcl::KdTreeFLANN (KDTreeSingleIndex, leaf
// 15, L2_Simple distance ((0+d0^2)+d1^2)+d2^2, sorted results).  FLANN's tie
// order is traversal-dependent (unpinned); ties resolve to the lower index.
struct KdTree {
  std::vector<Pt> pts;
  std::vector<int> idx;
  struct Node { int lo, hi, left, right, dim; float split; };
  std::vector<Node> nodes;

  static float dist(const Pt& q, const Pt& p) {
    float r = 0.f, d;
    d = q.x - p.x; r += d * d;
    d = q.y - p.y; r += d * d;
    d = q.z - p.z; r += d * d;
    return r;
  }
  void build(const std::vector<Pt>& cloud) {
    pts = cloud;
    idx.resize(pts.size());
    for (size_t i = 0; i < idx.size(); ++i) idx[i] = (int)i;
    nodes.clear();
    if (!pts.empty()) build_rec(0, (int)pts.size());
  }
  int build_rec(int lo, int hi) {
    int id = (int)nodes.size();
    nodes.push_back({lo, hi, -1, -1, 0, 0.f});
    if (hi - lo <= 15) return id;
    float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    for (int i = lo; i < hi; ++i) {
      const Pt& p = pts[idx[i]];
      const float v[3] = {p.x, p.y, p.z};
      for (int k = 0; k < 3; ++k) { mn[k] = std::min(mn[k], v[k]); mx[k] = std::max(mx[k], v[k]); }
    }
    int dim = 0;
    for (int k = 1; k < 3; ++k) if (mx[k] - mn[k] > mx[dim] - mn[dim]) dim = k;
    int mid = (lo + hi) / 2;
    auto key = [&](int i) { const Pt& p = pts[i]; return dim == 0 ? p.x : dim == 1 ? p.y : p.z; };
    std::nth_element(idx.begin() + lo, idx.begin() + mid, idx.begin() + hi,
                     [&](int a, int b) { return key(a) < key(b); });
    float split = key(idx[mid]);
    int l = build_rec(lo, mid);
    int r = build_rec(mid, hi);
    nodes[id].left = l; nodes[id].right = r; nodes[id].dim = dim; nodes[id].split = split;
    return id;
  }
  // k nearest (k <= 8), sorted by (distance, index).
  int knn(const Pt& q, int k, int* oi, float* od) const {
    int n = 0;
    if (nodes.empty()) return 0;
    search(0, q, k, oi, od, n);
    return n;
  }
  void search(int ni, const Pt& q, int k, int* oi, float* od, int& n) const {
    const Node& nd = nodes[ni];
    if (nd.left < 0) {
      for (int i = nd.lo; i < nd.hi; ++i) {
        int id = idx[i];
        float d = dist(q, pts[id]);
        if (n == k && !(d < od[n - 1] || (d == od[n - 1] && id < oi[n - 1]))) continue;
        int pos = (n < k) ? n++ : n - 1;
        while (pos > 0 && (d < od[pos - 1] || (d == od[pos - 1] && id < oi[pos - 1]))) {
          od[pos] = od[pos - 1]; oi[pos] = oi[pos - 1]; --pos;
        }
        od[pos] = d; oi[pos] = id;
      }
      return;
    }
    float qv = nd.dim == 0 ? q.x : nd.dim == 1 ? q.y : q.z;
    float diff = qv - nd.split;
    int first = diff < 0 ? nd.left : nd.right, second = diff < 0 ? nd.right : nd.left;
    search(first, q, k, oi, od, n);
    if (n < k || (double)diff * diff <= (double)od[n - 1] * 1.0000001 + 1e-30)
      search(second, q, k, oi, od, n);
  }
};

// ============================================================ ImageProjection
struct ImageProjection {
  lego_sensor_cfg c;
  int N, H, P;
  float sinAX, cosAX, sinAY, cosAY;
  std::vector<float> rangeMat;
  std::vector<int8_t> groundMat;
  std::vector<int32_t> labelMat;
  std::vector<Pt> fullCloud, fullInfoCloud;
  std::vector<Pt> segmentedCloud, outlierCloud, groundCloud, segmentedCloudPure;
  std::vector<int32_t> startRingIndex, endRingIndex;
  std::vector<uint8_t> groundFlag;
  std::vector<uint32_t> colInd;
  std::vector<float> segRange;
  float startOrientation = 0, endOrientation = 0, orientationDiff = 0;
  std::vector<uint16_t> qx, qy, apx, apy;
  int labelCount = 1;

  explicit ImageProjection(const lego_sensor_cfg& cfg) : c(cfg) {
    N = c.n_scan; H = c.horizon_scan; P = N * H;
    rangeMat.resize(P); groundMat.resize(P); labelMat.resize(P);
    fullCloud.resize(P); fullInfoCloud.resize(P);
    startRingIndex.assign(N, 0); endRingIndex.assign(N, 0);   // :125-126
    groundFlag.assign(P, 0); colInd.assign(P, 0); segRange.assign(P, 0.f);  // :128-130
    qx.resize(P); qy.resize(P); apx.resize(P); apy.resize(P);
    // labelComponents evaluates sin/cos(alpha) per edge (:421); the values are
    // per-sensor constants, taken from the same libm.
    sinAX = lego_sinf(c.segment_alpha_x); cosAX = lego_cosf(c.segment_alpha_x);
    sinAY = lego_sinf(c.segment_alpha_y); cosAY = lego_cosf(c.segment_alpha_y);
  }

  void reset() {  // resetParameters :145-159
    segmentedCloud.clear(); outlierCloud.clear(); groundCloud.clear(); segmentedCloudPure.clear();
    std::fill(rangeMat.begin(), rangeMat.end(), FLT_MAX);
    std::fill(groundMat.begin(), groundMat.end(), 0);
    std::fill(labelMat.begin(), labelMat.end(), 0);
    labelCount = 1;
    const float qn = std::numeric_limits<float>::quiet_NaN();
    std::fill(fullCloud.begin(), fullCloud.end(), Pt{qn, qn, qn, -1.f});
    std::fill(fullInfoCloud.begin(), fullInfoCloud.end(), Pt{qn, qn, qn, -1.f});
  }

  // findStartEndAngle :199-209
  void findStartEndAngle(const lego_point_xyzir* in, int n) {
    startOrientation = -lego_atan2f(in[0].y, in[0].x);
    endOrientation = (float)(-lego_atan2f(in[n - 1].y, in[n - 1].x) + 2 * M_PI);
    if ((double)(endOrientation - startOrientation) > 3 * M_PI)
      endOrientation = (float)((double)endOrientation - 2 * M_PI);
    else if ((double)(endOrientation - startOrientation) < M_PI)
      endOrientation = (float)((double)endOrientation + 2 * M_PI);
    orientationDiff = endOrientation - startOrientation;
  }

  // The (size_t) conversion of :230.  Out of range it is UB in C++; the
  // reference's x86-64 build converts a float below 2^63 by truncation toward
  // zero through int64 (cvttss2si), so (-1, 0) gives row 0 and v <= -1 wraps
  // to an index past N_SCAN.  Stated explicitly so this build cannot differ.
  static size_t row_of(float v) {
    if (!(v < 9.2233720e18f)) return ~(size_t)0;  // NaN or >= 2^63: never a row
    return (size_t)(int64_t)v;
  }

  // projectPointCloud :211-257, both branches of useCloudRing (:225-231)
  void project(const lego_point_xyzir* in, int n) {
    for (int i = 0; i < n; ++i) {
      const float x = in[i].x, y = in[i].y, z = in[i].z;
      size_t row;
      if (c.use_cloud_ring) {
        row = in[i].ring;
      } else {
        // float atan2 / sqrt (utility.h's `using namespace std`), * 180 in
        // float, / M_PI in double, stored to the float verticalAngle
        const float va = (float)((double)(lego_atan2f(z, std::sqrt(x * x + y * y)) * 180.0f) / M_PI);
        row = row_of((va + c.ang_bottom) / c.ang_res_y);
      }
      if (row >= (size_t)N) continue;
      float h = (float)((double)(lego_atan2f(x, y) * 180.0f) / M_PI);
      double cd = -std::round(((double)h - 90.0) / (double)c.ang_res_x) + (double)(H / 2);
      if (cd < 0) continue;  // (size_t) of a negative double; unreachable for the presets
      size_t col = (size_t)cd;
      if (col >= (size_t)H) col -= H;
      if (col >= (size_t)H) continue;
      float range = std::sqrt(x * x + y * y + z * z);
      if (range < c.sensor_minimum_range) continue;
      rangeMat[row * H + col] = range;
      float inten = (float)((double)(float)row + (double)(float)col / 10000.0);
      size_t index = col + row * H;
      fullCloud[index] = {x, y, z, inten};
      fullInfoCloud[index] = {x, y, z, range};
    }
  }

  // groundRemoval :260-310
  void groundRemoval(bool want_ground_cloud) {
    const int g = c.ground_scan_ind;
    for (int j = 0; j < H; ++j) {
      for (int i = 0; i < g; ++i) {
        size_t lo = j + i * H, up = j + (i + 1) * H;
        if (fullCloud[lo].intensity == -1 || fullCloud[up].intensity == -1) {
          groundMat[i * H + j] = -1;
          continue;
        }
        float dX = fullCloud[up].x - fullCloud[lo].x;
        float dY = fullCloud[up].y - fullCloud[lo].y;
        float dZ = fullCloud[up].z - fullCloud[lo].z;
        float angle = (float)((double)(lego_atan2f(dZ, std::sqrt(dX * dX + dY * dY)) * 180.0f) / M_PI);
        if (lego::lfabsf(angle - c.sensor_mount_angle) <= 10) {
          groundMat[i * H + j] = 1;
          groundMat[(i + 1) * H + j] = 1;
        }
      }
    }
    for (int i = 0; i < N; ++i)
      for (int j = 0; j < H; ++j)
        if (groundMat[i * H + j] == 1 || rangeMat[i * H + j] == FLT_MAX) labelMat[i * H + j] = -1;
    if (want_ground_cloud)
      for (int i = 0; i <= g && i < N; ++i)
        for (int j = 0; j < H; ++j)
          if (groundMat[i * H + j] == 1) groundCloud.push_back(fullCloud[j + i * H]);
  }

  // labelComponents :370-460 (BFS with the reference's queue discipline)
  void labelComponents(int row, int col) {
    std::vector<char> lineCountFlag(N, 0);
    qx[0] = row; qy[0] = col;
    int queueSize = 1, queueStartInd = 0, queueEndInd = 1;
    apx[0] = row; apy[0] = col;
    int allPushedIndSize = 1;
    static const int nb[4][2] = {{-1, 0}, {0, 1}, {0, -1}, {1, 0}};  // :133-136
    while (queueSize > 0) {
      int fx = qx[queueStartInd], fy = qy[queueStartInd];
      --queueSize; ++queueStartInd;
      labelMat[fx * H + fy] = labelCount;
      for (int k = 0; k < 4; ++k) {
        int tx = fx + nb[k][0], ty = fy + nb[k][1];
        if (tx < 0 || tx >= N) continue;
        if (ty < 0) ty = H - 1;
        if (ty >= H) ty = 0;
        if (labelMat[tx * H + ty] != 0) continue;
        float d1 = std::max(rangeMat[fx * H + fy], rangeMat[tx * H + ty]);
        float d2 = std::min(rangeMat[fx * H + fy], rangeMat[tx * H + ty]);
        float sa = nb[k][0] == 0 ? sinAX : sinAY, ca = nb[k][0] == 0 ? cosAX : cosAY;
        float angle = lego_atan2f(d2 * sa, (d1 - d2 * ca));
        if (angle > c.segment_theta) {
          qx[queueEndInd] = tx; qy[queueEndInd] = ty;
          ++queueSize; ++queueEndInd;
          labelMat[tx * H + ty] = labelCount;
          lineCountFlag[tx] = 1;
          apx[allPushedIndSize] = tx; apy[allPushedIndSize] = ty;
          ++allPushedIndSize;
        }
      }
    }
    bool feasible = false;
    if (allPushedIndSize >= 30) feasible = true;
    else if (allPushedIndSize >= c.segment_valid_point_num) {
      int lineCount = 0;
      for (int i = 0; i < N; ++i) if (lineCountFlag[i]) ++lineCount;
      if (lineCount >= c.segment_valid_line_num) feasible = true;
    }
    if (feasible) ++labelCount;
    else
      for (int i = 0; i < allPushedIndSize; ++i) labelMat[apx[i] * H + apy[i]] = 999999;
  }

  // cloudSegmentation :312-368
  void cloudSegmentation(bool want_pure) {
    for (int i = 0; i < N; ++i)
      for (int j = 0; j < H; ++j)
        if (labelMat[i * H + j] == 0) labelComponents(i, j);
    int size = 0;
    const int g = c.ground_scan_ind;
    for (int i = 0; i < N; ++i) {
      startRingIndex[i] = size - 1 + 5;
      for (int j = 0; j < H; ++j) {
        const int L = labelMat[i * H + j];
        const int8_t G = groundMat[i * H + j];
        if (L > 0 || G == 1) {
          if (L == 999999) {
            if (i > g && j % 5 == 0) outlierCloud.push_back(fullCloud[j + i * H]);
            continue;
          }
          if (G == 1 && (j % 5 != 0 && j > 5 && j < H - 5)) continue;
          groundFlag[size] = (G == 1);
          colInd[size] = j;
          segRange[size] = rangeMat[i * H + j];
          segmentedCloud.push_back(fullCloud[j + i * H]);
          ++size;
        }
      }
      endRingIndex[i] = size - 1 - 5;
    }
    if (want_pure)
      for (int i = 0; i < N; ++i)
        for (int j = 0; j < H; ++j) {
          const int L = labelMat[i * H + j];
          if (L > 0 && L != 999999) {
            Pt p = fullCloud[j + i * H];
            p.intensity = (float)L;
            segmentedCloudPure.push_back(p);
          }
        }
  }

  std::vector<lego_point_xyzir> finite;

  int process(const lego_point_xyzir* in, int n, bool images, bool gated = false) {
    if (n <= 0 || !in) return LEGO_E_ARG;
    auto ok = [](const lego_point_xyzir& p) {
      return std::isfinite(p.x) && std::isfinite(p.y) && std::isfinite(p.z);
    };
    if (c.use_cloud_ring) {
      for (int i = 0; i < n; ++i)
        if (!ok(in[i])) return LEGO_E_NOT_DENSE;  // :173-176
    } else {
      // pcl::removeNaNFromPointCloud (:170) of a non-dense cloud: the finite
      // points in order (a dense-flagged cloud is projected unchanged upstream;
      // here non-finite points are always removed, DESIGN.md §2 deviation 4)
      bool all = true;
      for (int i = 0; i < n && all; ++i) all = ok(in[i]);
      if (!all) {
        finite.clear();
        for (int i = 0; i < n; ++i)
          if (ok(in[i])) finite.push_back(in[i]);
        if (finite.empty()) return LEGO_E_NOT_DENSE;  // points[0] of an empty cloud: UB upstream
        in = finite.data();
        n = (int)finite.size();
      }
    }
    reset();
    findStartEndAngle(in, n);
    project(in, n);
    groundRemoval(gated);
    cloudSegmentation(gated);
    return LEGO_OK;
  }
};

// ============================================================ FeatureAssociation
// tf::Matrix3x3(q).getRPY, defined with the mapping restatement (oracle_mo.inc)
inline void rpy_from_quat(double x, double y, double z, double w, double* roll, double* pitch, double* yaw);

static constexpr int kImuQ = 200;  // imuQueLength, utility.h:109

struct Smooth { float value; size_t ind; };           // utility.h:139-142
struct ByValue {                                       // utility.h:144-148
  bool operator()(Smooth const& l, Smooth const& r) const { return l.value < r.value; }
};

// Diagnostic log of the dense systems handed to the OpenCV-shaped solvers, so
// tests/test_numerics_witness.py can re-solve the real LM systems of a stream
// with an independent restatement.  Kinds: 0 odometry AtA|AtB (3x3 + 3),
// 1 mapping AtA|AtB (6x6 + 6), 2 mapping plane fit A0 (5x3, rhs -1),
// 3 mapping corner covariance (3x3).  Off unless enabled; capped per kind.
struct SysLog {
  bool on = false;
  int cap = 4096;  // systems per kind
  std::vector<float> v[4];
  int n[4] = {0, 0, 0, 0};
  void add(int kind, const float* a, int len) {
    if (!on || n[kind] >= cap) return;
    v[kind].insert(v[kind].end(), a, a + len);
    ++n[kind];
  }
};

struct FeatureAssociation {
  lego_sensor_cfg c;
  int N, H, P;
  bool pcl_sort = false;
  SysLog* log = nullptr;
  // persistent member arrays (:210-223); zero-initialised
  std::vector<float> cloudCurvature;
  std::vector<int> cloudNeighborPicked, cloudLabel;
  std::vector<Smooth> cloudSmoothness;
  std::vector<float> ind1, ind2, ind3;   // pointSearch*Ind (float arrays :214-221)
  // per-scan inputs
  std::vector<Pt> segmentedCloud, outlierCloud;
  std::vector<int32_t> sri, eri;
  std::vector<uint8_t> gflag;
  std::vector<uint32_t> colInd;
  std::vector<float> segRange;
  float startOri = 0, endOri = 0, oriDiff = 0;
  double stamp = 0;
  // features
  std::vector<Pt> sharp, lessSharp, flat, lessFlat, lessFlatScan, lessFlatScanDS;
  // odometry state
  bool systemInitedLM = false;
  float transformCur[6] = {0, 0, 0, 0, 0, 0}, transformSum[6] = {0, 0, 0, 0, 0, 0};
  std::vector<Pt> cornerLast, surfLast;
  KdTree kdCorner, kdSurf;
  int cornerLastNum = 0, surfLastNum = 0;
  std::vector<Pt> laserCloudOri, coeffSel;
  bool isDegenerate = false;
  float matP[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
  int frameCount;
  // IMU state (:84-159, initialised :251-295); all zero until the first
  // /imu_raw message (imuPointerLast = -1)
  float cosImuRollStart = 0, cosImuPitchStart = 0, cosImuYawStart = 0;
  float sinImuRollStart = 0, sinImuPitchStart = 0, sinImuYawStart = 0;
  float imuRollStart = 0, imuPitchStart = 0, imuYawStart = 0;
  float imuRollLast = 0, imuPitchLast = 0, imuYawLast = 0;
  float imuShiftFromStartX = 0, imuShiftFromStartY = 0, imuShiftFromStartZ = 0;
  float imuVeloFromStartX = 0, imuVeloFromStartY = 0, imuVeloFromStartZ = 0;
  int imuPointerFront = 0, imuPointerLast = -1, imuPointerLastIteration = 0;
  double imuTime[kImuQ] = {};
  float imuRoll[kImuQ] = {}, imuPitch[kImuQ] = {}, imuYaw[kImuQ] = {};
  float imuAccX[kImuQ] = {}, imuAccY[kImuQ] = {}, imuAccZ[kImuQ] = {};
  float imuVeloX[kImuQ] = {}, imuVeloY[kImuQ] = {}, imuVeloZ[kImuQ] = {};
  float imuShiftX[kImuQ] = {}, imuShiftY[kImuQ] = {}, imuShiftZ[kImuQ] = {};
  float imuAngularVeloX[kImuQ] = {}, imuAngularVeloY[kImuQ] = {}, imuAngularVeloZ[kImuQ] = {};
  float imuAngularRotationX[kImuQ] = {}, imuAngularRotationY[kImuQ] = {}, imuAngularRotationZ[kImuQ] = {};
  float imuRollCur = 0, imuPitchCur = 0, imuYawCur = 0;
  float imuVeloXStart = 0, imuVeloYStart = 0, imuVeloZStart = 0;
  float imuShiftXStart = 0, imuShiftYStart = 0, imuShiftZStart = 0;
  float imuVeloXCur = 0, imuVeloYCur = 0, imuVeloZCur = 0;
  float imuShiftXCur = 0, imuShiftYCur = 0, imuShiftZCur = 0;
  float imuShiftFromStartXCur = 0, imuShiftFromStartYCur = 0, imuShiftFromStartZCur = 0;
  float imuVeloFromStartXCur = 0, imuVeloFromStartYCur = 0, imuVeloFromStartZCur = 0;
  float imuAngularRotationXCur = 0, imuAngularRotationYCur = 0, imuAngularRotationZCur = 0;
  float imuAngularRotationXLast = 0, imuAngularRotationYLast = 0, imuAngularRotationZLast = 0;
  float imuAngularFromStartX = 0, imuAngularFromStartY = 0, imuAngularFromStartZ = 0;
  // outputs
  bool odomValid = false, publishToMapping = false;
  std::vector<Pt> outCornerLast, outSurfLast, outOutlierLast;

  explicit FeatureAssociation(const lego_sensor_cfg& cfg) : c(cfg) {
    N = c.n_scan; H = c.horizon_scan; P = N * H;
    cloudCurvature.assign(P, 0.f);
    cloudNeighborPicked.assign(P, 0);
    cloudLabel.assign(P, 0);
    cloudSmoothness.assign(P, Smooth{0.f, 0});
    ind1.assign(P, 0.f); ind2.assign(P, 0.f); ind3.assign(P, 0.f);
    frameCount = c.skip_frame_num;
  }

  // updateImuRollPitchYawStartSinCos :317-324
  void updateImuStartSinCos() {
    cosImuRollStart = lego_cosf(imuRollStart); cosImuPitchStart = lego_cosf(imuPitchStart);
    cosImuYawStart = lego_cosf(imuYawStart); sinImuRollStart = lego_sinf(imuRollStart);
    sinImuPitchStart = lego_sinf(imuPitchStart); sinImuYawStart = lego_sinf(imuYawStart);
  }

  // AccumulateIMUShiftAndRotation :392-429
  void accumulateIMUShiftAndRotation() {
    const int l = imuPointerLast;
    const float roll = imuRoll[l], pitch = imuPitch[l], yaw = imuYaw[l];
    float accX = imuAccX[l], accY = imuAccY[l], accZ = imuAccZ[l];
    const float x1 = lego_cosf(roll) * accX - lego_sinf(roll) * accY;
    const float y1 = lego_sinf(roll) * accX + lego_cosf(roll) * accY;
    const float z1 = accZ;
    const float x2 = x1;
    const float y2 = lego_cosf(pitch) * y1 - lego_sinf(pitch) * z1;
    const float z2 = lego_sinf(pitch) * y1 + lego_cosf(pitch) * z1;
    accX = lego_cosf(yaw) * x2 + lego_sinf(yaw) * z2;
    accY = y2;
    accZ = -lego_sinf(yaw) * x2 + lego_cosf(yaw) * z2;
    const int b = (l + kImuQ - 1) % kImuQ;
    const double timeDiff = imuTime[l] - imuTime[b];
    if (timeDiff < c.scan_period) {
      imuShiftX[l] = (float)(imuShiftX[b] + imuVeloX[b] * timeDiff + accX * timeDiff * timeDiff / 2);
      imuShiftY[l] = (float)(imuShiftY[b] + imuVeloY[b] * timeDiff + accY * timeDiff * timeDiff / 2);
      imuShiftZ[l] = (float)(imuShiftZ[b] + imuVeloZ[b] * timeDiff + accZ * timeDiff * timeDiff / 2);
      imuVeloX[l] = (float)(imuVeloX[b] + accX * timeDiff);
      imuVeloY[l] = (float)(imuVeloY[b] + accY * timeDiff);
      imuVeloZ[l] = (float)(imuVeloZ[b] + accZ * timeDiff);
      imuAngularRotationX[l] = (float)(imuAngularRotationX[b] + imuAngularVeloX[b] * timeDiff);
      imuAngularRotationY[l] = (float)(imuAngularRotationY[b] + imuAngularVeloY[b] * timeDiff);
      imuAngularRotationZ[l] = (float)(imuAngularRotationZ[b] + imuAngularVeloZ[b] * timeDiff);
    }
  }

  // imuHandler :431-458
  void imuHandler(const lego_imu_msg& m) {
    double roll, pitch, yaw;
    rpy_from_quat(m.orientation[0], m.orientation[1], m.orientation[2], m.orientation[3], &roll, &pitch, &yaw);
    const float accX = (float)(m.linear_acceleration[1] - std::sin(roll) * std::cos(pitch) * 9.81);
    const float accY = (float)(m.linear_acceleration[2] - std::cos(roll) * std::cos(pitch) * 9.81);
    const float accZ = (float)(m.linear_acceleration[0] + std::sin(pitch) * 9.81);
    imuPointerLast = (imuPointerLast + 1) % kImuQ;
    const int l = imuPointerLast;
    imuTime[l] = m.stamp;
    imuRoll[l] = (float)roll; imuPitch[l] = (float)pitch; imuYaw[l] = (float)yaw;
    imuAccX[l] = accX; imuAccY[l] = accY; imuAccZ[l] = accZ;
    imuAngularVeloX[l] = (float)m.angular_velocity[0];
    imuAngularVeloY[l] = (float)m.angular_velocity[1];
    imuAngularVeloZ[l] = (float)m.angular_velocity[2];
    accumulateIMUShiftAndRotation();
  }

  // VeloToStartIMU :346-363
  void veloToStartIMU() {
    imuVeloFromStartXCur = imuVeloXCur - imuVeloXStart;
    imuVeloFromStartYCur = imuVeloYCur - imuVeloYStart;
    imuVeloFromStartZCur = imuVeloZCur - imuVeloZStart;
    const float x1 = cosImuYawStart * imuVeloFromStartXCur - sinImuYawStart * imuVeloFromStartZCur;
    const float y1 = imuVeloFromStartYCur;
    const float z1 = sinImuYawStart * imuVeloFromStartXCur + cosImuYawStart * imuVeloFromStartZCur;
    const float x2 = x1;
    const float y2 = cosImuPitchStart * y1 + sinImuPitchStart * z1;
    const float z2 = -sinImuPitchStart * y1 + cosImuPitchStart * z1;
    imuVeloFromStartXCur = cosImuRollStart * x2 + sinImuRollStart * y2;
    imuVeloFromStartYCur = -sinImuRollStart * x2 + cosImuRollStart * y2;
    imuVeloFromStartZCur = z2;
  }

  // TransformToStartIMU :365-390
  void transformToStartIMU(Pt* p) const {
    const float x1 = lego_cosf(imuRollCur) * p->x - lego_sinf(imuRollCur) * p->y;
    const float y1 = lego_sinf(imuRollCur) * p->x + lego_cosf(imuRollCur) * p->y;
    const float z1 = p->z;
    const float x2 = x1;
    const float y2 = lego_cosf(imuPitchCur) * y1 - lego_sinf(imuPitchCur) * z1;
    const float z2 = lego_sinf(imuPitchCur) * y1 + lego_cosf(imuPitchCur) * z1;
    const float x3 = lego_cosf(imuYawCur) * x2 + lego_sinf(imuYawCur) * z2;
    const float y3 = y2;
    const float z3 = -lego_sinf(imuYawCur) * x2 + lego_cosf(imuYawCur) * z2;
    const float x4 = cosImuYawStart * x3 - sinImuYawStart * z3;
    const float y4 = y3;
    const float z4 = sinImuYawStart * x3 + cosImuYawStart * z3;
    const float x5 = x4;
    const float y5 = cosImuPitchStart * y4 + sinImuPitchStart * z4;
    const float z5 = -sinImuPitchStart * y4 + cosImuPitchStart * z4;
    p->x = cosImuRollStart * x5 + sinImuRollStart * y5 + imuShiftFromStartXCur;
    p->y = -sinImuRollStart * x5 + cosImuRollStart * y5 + imuShiftFromStartYCur;
    p->z = z5 + imuShiftFromStartZCur;
  }

  // adjustDistortion :491-619
  void adjustDistortion() {
    bool halfPassed = false;
    const int n = (int)segmentedCloud.size();
    for (int i = 0; i < n; ++i) {
      Pt point;
      point.x = segmentedCloud[i].y;
      point.y = segmentedCloud[i].z;
      point.z = segmentedCloud[i].x;
      float ori = -lego_atan2f(point.x, point.z);
      if (!halfPassed) {
        if ((double)ori < (double)startOri - M_PI / 2) ori = (float)((double)ori + 2 * M_PI);
        else if ((double)ori > (double)startOri + M_PI * 3 / 2) ori = (float)((double)ori - 2 * M_PI);
        if ((double)(ori - startOri) > M_PI) halfPassed = true;
      } else {
        ori = (float)((double)ori + 2 * M_PI);
        if ((double)ori < (double)endOri - M_PI * 3 / 2) ori = (float)((double)ori + 2 * M_PI);
        else if ((double)ori > (double)endOri + M_PI / 2) ori = (float)((double)ori - 2 * M_PI);
      }
      float relTime = (ori - startOri) / oriDiff;
      point.intensity = (float)(int)segmentedCloud[i].intensity + c.scan_period * relTime;
      if (imuPointerLast >= 0) {
        const float pointTime = relTime * c.scan_period;
        imuPointerFront = imuPointerLastIteration;
        // imuPointerLastIteration is -1 when the previous scan saw no message:
        // the reference then reads imuTime[-1] (undefined; SURVEY.md §9.7
        // policy) — restated as a zero slot, which the scan time passes.
        if (imuPointerFront < 0) imuPointerFront = 0;
        while (imuPointerFront != imuPointerLast) {
          if (stamp + pointTime < imuTime[imuPointerFront]) break;
          imuPointerFront = (imuPointerFront + 1) % kImuQ;
        }
        const int f = imuPointerFront;
        if (stamp + pointTime > imuTime[f]) {
          imuRollCur = imuRoll[f]; imuPitchCur = imuPitch[f]; imuYawCur = imuYaw[f];
          imuVeloXCur = imuVeloX[f]; imuVeloYCur = imuVeloY[f]; imuVeloZCur = imuVeloZ[f];
          imuShiftXCur = imuShiftX[f]; imuShiftYCur = imuShiftY[f]; imuShiftZCur = imuShiftZ[f];
        } else {
          const int b = (f + kImuQ - 1) % kImuQ;
          const float ratioFront = (float)((stamp + pointTime - imuTime[b]) / (imuTime[f] - imuTime[b]));
          const float ratioBack = (float)((imuTime[f] - stamp - pointTime) / (imuTime[f] - imuTime[b]));
          imuRollCur = imuRoll[f] * ratioFront + imuRoll[b] * ratioBack;
          imuPitchCur = imuPitch[f] * ratioFront + imuPitch[b] * ratioBack;
          if ((double)(imuYaw[f] - imuYaw[b]) > M_PI)
            imuYawCur = (float)(imuYaw[f] * ratioFront + (imuYaw[b] + 2 * M_PI) * ratioBack);
          else if ((double)(imuYaw[f] - imuYaw[b]) < -M_PI)
            imuYawCur = (float)(imuYaw[f] * ratioFront + (imuYaw[b] - 2 * M_PI) * ratioBack);
          else
            imuYawCur = imuYaw[f] * ratioFront + imuYaw[b] * ratioBack;
          imuVeloXCur = imuVeloX[f] * ratioFront + imuVeloX[b] * ratioBack;
          imuVeloYCur = imuVeloY[f] * ratioFront + imuVeloY[b] * ratioBack;
          imuVeloZCur = imuVeloZ[f] * ratioFront + imuVeloZ[b] * ratioBack;
          imuShiftXCur = imuShiftX[f] * ratioFront + imuShiftX[b] * ratioBack;
          imuShiftYCur = imuShiftY[f] * ratioFront + imuShiftY[b] * ratioBack;
          imuShiftZCur = imuShiftZ[f] * ratioFront + imuShiftZ[b] * ratioBack;
        }
        if (i == 0) {
          imuRollStart = imuRollCur; imuPitchStart = imuPitchCur; imuYawStart = imuYawCur;
          imuVeloXStart = imuVeloXCur; imuVeloYStart = imuVeloYCur; imuVeloZStart = imuVeloZCur;
          imuShiftXStart = imuShiftXCur; imuShiftYStart = imuShiftYCur; imuShiftZStart = imuShiftZCur;
          if (stamp + pointTime > imuTime[f]) {
            imuAngularRotationXCur = imuAngularRotationX[f];
            imuAngularRotationYCur = imuAngularRotationY[f];
            imuAngularRotationZCur = imuAngularRotationZ[f];
          } else {
            const int b = (f + kImuQ - 1) % kImuQ;
            const float ratioFront = (float)((stamp + pointTime - imuTime[b]) / (imuTime[f] - imuTime[b]));
            const float ratioBack = (float)((imuTime[f] - stamp - pointTime) / (imuTime[f] - imuTime[b]));
            imuAngularRotationXCur = imuAngularRotationX[f] * ratioFront + imuAngularRotationX[b] * ratioBack;
            imuAngularRotationYCur = imuAngularRotationY[f] * ratioFront + imuAngularRotationY[b] * ratioBack;
            imuAngularRotationZCur = imuAngularRotationZ[f] * ratioFront + imuAngularRotationZ[b] * ratioBack;
          }
          imuAngularFromStartX = imuAngularRotationXCur - imuAngularRotationXLast;
          imuAngularFromStartY = imuAngularRotationYCur - imuAngularRotationYLast;
          imuAngularFromStartZ = imuAngularRotationZCur - imuAngularRotationZLast;
          imuAngularRotationXLast = imuAngularRotationXCur;
          imuAngularRotationYLast = imuAngularRotationYCur;
          imuAngularRotationZLast = imuAngularRotationZCur;
          updateImuStartSinCos();
        } else {
          veloToStartIMU();
          transformToStartIMU(&point);
        }
      }
      segmentedCloud[i] = point;
    }
    imuPointerLastIteration = imuPointerLast;
  }

  // updateInitialGuess :1639-1664
  void updateInitialGuess() {
    imuPitchLast = imuPitchCur; imuYawLast = imuYawCur; imuRollLast = imuRollCur;
    imuShiftFromStartX = imuShiftFromStartXCur;
    imuShiftFromStartY = imuShiftFromStartYCur;
    imuShiftFromStartZ = imuShiftFromStartZCur;
    imuVeloFromStartX = imuVeloFromStartXCur;
    imuVeloFromStartY = imuVeloFromStartYCur;
    imuVeloFromStartZ = imuVeloFromStartZCur;
    if (imuAngularFromStartX != 0 || imuAngularFromStartY != 0 || imuAngularFromStartZ != 0) {
      transformCur[0] = -imuAngularFromStartY;
      transformCur[1] = -imuAngularFromStartZ;
      transformCur[2] = -imuAngularFromStartX;
    }
    if (imuVeloFromStartX != 0 || imuVeloFromStartY != 0 || imuVeloFromStartZ != 0) {
      transformCur[3] -= imuVeloFromStartX * c.scan_period;
      transformCur[4] -= imuVeloFromStartY * c.scan_period;
      transformCur[5] -= imuVeloFromStartZ * c.scan_period;
    }
  }

  // calculateSmoothness :621-641
  void calculateSmoothness() {
    const int n = (int)segmentedCloud.size();
    const float* r = segRange.data();
    for (int i = 5; i < n - 5; ++i) {
      float d = r[i - 5] + r[i - 4] + r[i - 3] + r[i - 2] + r[i - 1] - r[i] * 10 + r[i + 1] +
                r[i + 2] + r[i + 3] + r[i + 4] + r[i + 5];
      cloudCurvature[i] = d * d;
      cloudNeighborPicked[i] = 0;
      cloudLabel[i] = 0;
      cloudSmoothness[i].value = cloudCurvature[i];
      cloudSmoothness[i].ind = i;
    }
  }

  // markOccludedPoints :643-678
  void markOccludedPoints() {
    const int n = (int)segmentedCloud.size();
    const float* r = segRange.data();
    for (int i = 5; i < n - 6; ++i) {
      float depth1 = r[i], depth2 = r[i + 1];
      int columnDiff = std::abs((int)(colInd[i + 1] - colInd[i]));
      if (columnDiff < 10) {
        if ((double)(depth1 - depth2) > 0.3) {
          for (int k = i - 5; k <= i; ++k) cloudNeighborPicked[k] = 1;
        } else if ((double)(depth2 - depth1) > 0.3) {
          for (int k = i + 1; k <= i + 6; ++k) cloudNeighborPicked[k] = 1;
        }
      }
      float diff1 = std::fabs(float(r[i - 1] - r[i]));
      float diff2 = std::fabs(float(r[i + 1] - r[i]));
      if ((double)diff1 > 0.02 * (double)r[i] && (double)diff2 > 0.02 * (double)r[i])
        cloudNeighborPicked[i] = 1;
    }
  }

  // neighbour suppression used by both picks (:720-732, :751-767).  A negative
  // index (the phantom entry) reads colInd[-1] in the
  // reference (UB); treated as a column break.
  void suppress(int ind) {
    cloudNeighborPicked[ind] = 1;
    for (int l = 1; l <= 5; l++) {
      int cd = std::abs((int)(colInd[ind + l] - colInd[ind + l - 1]));
      if (cd > 10) break;
      cloudNeighborPicked[ind + l] = 1;
    }
    for (int l = -1; l >= -5; l--) {
      if (ind + l < 0) break;
      int cd = std::abs((int)(colInd[ind + l] - colInd[ind + l + 1]));
      if (cd > 10) break;
      cloudNeighborPicked[ind + l] = 1;
    }
  }

  // extractFeatures :680-784
  void extractFeatures() {
    sharp.clear(); lessSharp.clear(); flat.clear(); lessFlat.clear();
    for (int i = 0; i < N; i++) {
      lessFlatScan.clear();
      for (int j = 0; j < 6; j++) {
        int sp = (sri[i] * (6 - j) + eri[i] * j) / 6;
        int ep = (sri[i] * (5 - j) + eri[i] * (j + 1)) / 6 - 1;
        if (sp >= ep) continue;
        std::sort(cloudSmoothness.begin() + sp, cloudSmoothness.begin() + ep, ByValue());
        int largestPickedNum = 0;
        for (int k = ep; k >= sp; k--) {
          int ind = (int)cloudSmoothness[k].ind;
          if (cloudNeighborPicked[ind] == 0 && cloudCurvature[ind] > c.edge_threshold &&
              gflag[ind] == 0) {
            largestPickedNum++;
            if (largestPickedNum <= 2) {
              cloudLabel[ind] = 2;
              sharp.push_back(segmentedCloud[ind]);
              lessSharp.push_back(segmentedCloud[ind]);
            } else if (largestPickedNum <= 20) {
              cloudLabel[ind] = 1;
              lessSharp.push_back(segmentedCloud[ind]);
            } else {
              break;
            }
            suppress(ind);
          }
        }
        int smallestPickedNum = 0;
        for (int k = sp; k <= ep; k++) {
          int ind = (int)cloudSmoothness[k].ind;
          if (cloudNeighborPicked[ind] == 0 && cloudCurvature[ind] < c.surf_threshold &&
              gflag[ind] == 1) {
            cloudLabel[ind] = -1;
            flat.push_back(segmentedCloud[ind]);
            smallestPickedNum++;
            if (smallestPickedNum >= 4) break;
            suppress(ind);
          }
        }
        for (int k = sp; k <= ep; k++)
          if (cloudLabel[k] <= 0) lessFlatScan.push_back(segmentedCloud[k]);
      }
      voxel_grid(lessFlatScan, 0.2f, pcl_sort, lessFlatScanDS);
      lessFlat.insert(lessFlat.end(), lessFlatScanDS.begin(), lessFlatScanDS.end());
    }
  }

  // TransformToStart :860-883
  void toStart(const Pt& pi, Pt& po) const {
    float s = 10 * (pi.intensity - int(pi.intensity));
    float rx = s * transformCur[0], ry = s * transformCur[1], rz = s * transformCur[2];
    float tx = s * transformCur[3], ty = s * transformCur[4], tz = s * transformCur[5];
    float x1 = lego_cosf(rz) * (pi.x - tx) + lego_sinf(rz) * (pi.y - ty);
    float y1 = -lego_sinf(rz) * (pi.x - tx) + lego_cosf(rz) * (pi.y - ty);
    float z1 = (pi.z - tz);
    float x2 = x1;
    float y2 = lego_cosf(rx) * y1 + lego_sinf(rx) * z1;
    float z2 = -lego_sinf(rx) * y1 + lego_cosf(rx) * z1;
    po.x = lego_cosf(ry) * x2 - lego_sinf(ry) * z2;
    po.y = y2;
    po.z = lego_sinf(ry) * x2 + lego_cosf(ry) * z2;
    po.intensity = pi.intensity;
  }

  // TransformToEnd :885-953
  void toEnd(const Pt& pi, Pt& po) const {
    float s = 10 * (pi.intensity - int(pi.intensity));
    float rx = s * transformCur[0], ry = s * transformCur[1], rz = s * transformCur[2];
    float tx = s * transformCur[3], ty = s * transformCur[4], tz = s * transformCur[5];
    float x1 = lego_cosf(rz) * (pi.x - tx) + lego_sinf(rz) * (pi.y - ty);
    float y1 = -lego_sinf(rz) * (pi.x - tx) + lego_cosf(rz) * (pi.y - ty);
    float z1 = (pi.z - tz);
    float x2 = x1;
    float y2 = lego_cosf(rx) * y1 + lego_sinf(rx) * z1;
    float z2 = -lego_sinf(rx) * y1 + lego_cosf(rx) * z1;
    float x3 = lego_cosf(ry) * x2 - lego_sinf(ry) * z2;
    float y3 = y2;
    float z3 = lego_sinf(ry) * x2 + lego_cosf(ry) * z2;
    rx = transformCur[0]; ry = transformCur[1]; rz = transformCur[2];
    tx = transformCur[3]; ty = transformCur[4]; tz = transformCur[5];
    float x4 = lego_cosf(ry) * x3 + lego_sinf(ry) * z3;
    float y4 = y3;
    float z4 = -lego_sinf(ry) * x3 + lego_cosf(ry) * z3;
    float x5 = x4;
    float y5 = lego_cosf(rx) * y4 - lego_sinf(rx) * z4;
    float z5 = lego_sinf(rx) * y4 + lego_cosf(rx) * z4;
    float x6 = lego_cosf(rz) * x5 - lego_sinf(rz) * y5 + tx;
    float y6 = lego_sinf(rz) * x5 + lego_cosf(rz) * y5 + ty;
    float z6 = z5 + tz;
    float x7 = cosImuRollStart * (x6 - imuShiftFromStartX) - sinImuRollStart * (y6 - imuShiftFromStartY);
    float y7 = sinImuRollStart * (x6 - imuShiftFromStartX) + cosImuRollStart * (y6 - imuShiftFromStartY);
    float z7 = z6 - imuShiftFromStartZ;
    float x8 = x7;
    float y8 = cosImuPitchStart * y7 - sinImuPitchStart * z7;
    float z8 = sinImuPitchStart * y7 + cosImuPitchStart * z7;
    float x9 = cosImuYawStart * x8 + sinImuYawStart * z8;
    float y9 = y8;
    float z9 = -sinImuYawStart * x8 + cosImuYawStart * z8;
    float x10 = lego_cosf(imuYawLast) * x9 - lego_sinf(imuYawLast) * z9;
    float y10 = y9;
    float z10 = lego_sinf(imuYawLast) * x9 + lego_cosf(imuYawLast) * z9;
    float x11 = x10;
    float y11 = lego_cosf(imuPitchLast) * y10 + lego_sinf(imuPitchLast) * z10;
    float z11 = -lego_sinf(imuPitchLast) * y10 + lego_cosf(imuPitchLast) * z10;
    po.x = lego_cosf(imuRollLast) * x11 + lego_sinf(imuRollLast) * y11;
    po.y = -lego_sinf(imuRollLast) * x11 + lego_cosf(imuRollLast) * y11;
    po.z = z11;
    po.intensity = (float)int(pi.intensity);
  }

  // PluginIMURotation :955-1013
  static void pluginIMURotation(float bcx, float bcy, float bcz, float blx, float bly, float blz,
                                float alx, float aly, float alz, float& acx, float& acy, float& acz) {
    float sbcx = lego_sinf(bcx), cbcx = lego_cosf(bcx), sbcy = lego_sinf(bcy), cbcy = lego_cosf(bcy);
    float sbcz = lego_sinf(bcz), cbcz = lego_cosf(bcz);
    float sblx = lego_sinf(blx), cblx = lego_cosf(blx), sbly = lego_sinf(bly), cbly = lego_cosf(bly);
    float sblz = lego_sinf(blz), cblz = lego_cosf(blz);
    float salx = lego_sinf(alx), calx = lego_cosf(alx), saly = lego_sinf(aly), caly = lego_cosf(aly);
    float salz = lego_sinf(alz), calz = lego_cosf(alz);
    float srx = -sbcx * (salx * sblx + calx * caly * cblx * cbly + calx * cblx * saly * sbly) -
                cbcx * cbcz * (calx * saly * (cbly * sblz - cblz * sblx * sbly) -
                               calx * caly * (sbly * sblz + cbly * cblz * sblx) + cblx * cblz * salx) -
                cbcx * sbcz * (calx * caly * (cblz * sbly - cbly * sblx * sblz) -
                               calx * saly * (cbly * cblz + sblx * sbly * sblz) + cblx * salx * sblz);
    acx = -lego_asinf(srx);
    float srycrx = (cbcy * sbcz - cbcz * sbcx * sbcy) *
                       (calx * saly * (cbly * sblz - cblz * sblx * sbly) -
                        calx * caly * (sbly * sblz + cbly * cblz * sblx) + cblx * cblz * salx) -
                   (cbcy * cbcz + sbcx * sbcy * sbcz) *
                       (calx * caly * (cblz * sbly - cbly * sblx * sblz) -
                        calx * saly * (cbly * cblz + sblx * sbly * sblz) + cblx * salx * sblz) +
                   cbcx * sbcy * (salx * sblx + calx * caly * cblx * cbly + calx * cblx * saly * sbly);
    float crycrx = (cbcz * sbcy - cbcy * sbcx * sbcz) *
                       (calx * caly * (cblz * sbly - cbly * sblx * sblz) -
                        calx * saly * (cbly * cblz + sblx * sbly * sblz) + cblx * salx * sblz) -
                   (sbcy * sbcz + cbcy * cbcz * sbcx) *
                       (calx * saly * (cbly * sblz - cblz * sblx * sbly) -
                        calx * caly * (sbly * sblz + cbly * cblz * sblx) + cblx * cblz * salx) +
                   cbcx * cbcy * (salx * sblx + calx * caly * cblx * cbly + calx * cblx * saly * sbly);
    acy = lego_atan2f(srycrx / lego_cosf(acx), crycrx / lego_cosf(acx));
    float srzcrx = sbcx * (cblx * cbly * (calz * saly - caly * salx * salz) -
                           cblx * sbly * (caly * calz + salx * saly * salz) + calx * salz * sblx) -
                   cbcx * cbcz * ((caly * calz + salx * saly * salz) * (cbly * sblz - cblz * sblx * sbly) +
                                  (calz * saly - caly * salx * salz) * (sbly * sblz + cbly * cblz * sblx) -
                                  calx * cblx * cblz * salz) +
                   cbcx * sbcz * ((caly * calz + salx * saly * salz) * (cbly * cblz + sblx * sbly * sblz) +
                                  (calz * saly - caly * salx * salz) * (cblz * sbly - cbly * sblx * sblz) +
                                  calx * cblx * salz * sblz);
    float crzcrx = sbcx * (cblx * sbly * (caly * salz - calz * salx * saly) -
                           cblx * cbly * (saly * salz + caly * calz * salx) + calx * calz * sblx) +
                   cbcx * cbcz * ((saly * salz + caly * calz * salx) * (sbly * sblz + cbly * cblz * sblx) +
                                  (caly * salz - calz * salx * saly) * (cbly * sblz - cblz * sblx * sbly) +
                                  calx * calz * cblx * cblz) -
                   cbcx * sbcz * ((saly * salz + caly * calz * salx) * (cblz * sbly - cbly * sblx * sblz) +
                                  (caly * salz - calz * salx * saly) * (cbly * cblz + sblx * sbly * sblz) -
                                  calx * calz * cblx * sblz);
    acz = lego_atan2f(srzcrx / lego_cosf(acx), crzcrx / lego_cosf(acx));
  }

  // AccumulateRotation :1015-1032
  static void accumulateRotation(float cx, float cy, float cz, float lx, float ly, float lz,
                                 float& ox, float& oy, float& oz) {
    float srx = lego_cosf(lx) * lego_cosf(cx) * lego_sinf(ly) * lego_sinf(cz) -
                lego_cosf(cx) * lego_cosf(cz) * lego_sinf(lx) -
                lego_cosf(lx) * lego_cosf(ly) * lego_sinf(cx);
    ox = -lego_asinf(srx);
    float srycrx = lego_sinf(lx) * (lego_cosf(cy) * lego_sinf(cz) - lego_cosf(cz) * lego_sinf(cx) * lego_sinf(cy)) +
                   lego_cosf(lx) * lego_sinf(ly) * (lego_cosf(cy) * lego_cosf(cz) + lego_sinf(cx) * lego_sinf(cy) * lego_sinf(cz)) +
                   lego_cosf(lx) * lego_cosf(ly) * lego_cosf(cx) * lego_sinf(cy);
    float crycrx = lego_cosf(lx) * lego_cosf(ly) * lego_cosf(cx) * lego_cosf(cy) -
                   lego_cosf(lx) * lego_sinf(ly) * (lego_cosf(cz) * lego_sinf(cy) - lego_cosf(cy) * lego_sinf(cx) * lego_sinf(cz)) -
                   lego_sinf(lx) * (lego_sinf(cy) * lego_sinf(cz) + lego_cosf(cy) * lego_cosf(cz) * lego_sinf(cx));
    oy = lego_atan2f(srycrx / lego_cosf(ox), crycrx / lego_cosf(ox));
    float srzcrx = lego_sinf(cx) * (lego_cosf(lz) * lego_sinf(ly) - lego_cosf(ly) * lego_sinf(lx) * lego_sinf(lz)) +
                   lego_cosf(cx) * lego_sinf(cz) * (lego_cosf(ly) * lego_cosf(lz) + lego_sinf(lx) * lego_sinf(ly) * lego_sinf(lz)) +
                   lego_cosf(lx) * lego_cosf(cx) * lego_cosf(cz) * lego_sinf(lz);
    float crzcrx = lego_cosf(lx) * lego_cosf(lz) * lego_cosf(cx) * lego_cosf(cz) -
                   lego_cosf(cx) * lego_sinf(cz) * (lego_cosf(ly) * lego_sinf(lz) - lego_cosf(lz) * lego_sinf(lx) * lego_sinf(ly)) -
                   lego_sinf(cx) * (lego_sinf(ly) * lego_sinf(lz) + lego_cosf(ly) * lego_cosf(lz) * lego_sinf(lx));
    oz = lego_atan2f(srzcrx / lego_cosf(ox), crzcrx / lego_cosf(ox));
  }

  static float sqd(const Pt& a, const Pt& b) {  // the scan-line search distance
    return (a.x - b.x) * (a.x - b.x) + (a.y - b.y) * (a.y - b.y) + (a.z - b.z) * (a.z - b.z);
  }

  // findCorrespondingCornerFeatures :1044-1153
  void findCorrespondingCorner(int iter) {
    const int num = (int)sharp.size();
    const int lastN = (int)cornerLast.size();
    for (int i = 0; i < num; i++) {
      Pt sel;
      toStart(sharp[i], sel);
      if (iter % 5 == 0) {
        int nnI; float nnD;
        int got = kdCorner.knn(sel, 1, &nnI, &nnD);
        int closest = -1, min2 = -1;
        if (got == 1 && nnD < c.nearest_feature_search_sq_dist && nnI < lastN) {
          closest = nnI;
          int cScan = int(cornerLast[closest].intensity);
          float minD2 = c.nearest_feature_search_sq_dist;
          // loop bound is the *current* sharp count (:1062), clamped to the
          // last cloud (the reference reads past its end otherwise)
          const int jend = std::min(num, lastN);
          for (int j = closest + 1; j < jend; j++) {
            if ((double)int(cornerLast[j].intensity) > cScan + 2.5) break;
            float d = sqd(cornerLast[j], sel);
            if (int(cornerLast[j].intensity) > cScan && d < minD2) { minD2 = d; min2 = j; }
          }
          for (int j = closest - 1; j >= 0; j--) {
            if ((double)int(cornerLast[j].intensity) < cScan - 2.5) break;
            float d = sqd(cornerLast[j], sel);
            if (int(cornerLast[j].intensity) < cScan && d < minD2) { minD2 = d; min2 = j; }
          }
        }
        ind1[i] = (float)closest;
        ind2[i] = (float)min2;
      }
      if (ind2[i] >= 0) {
        const Pt& t1 = cornerLast[(int)ind1[i]];
        const Pt& t2 = cornerLast[(int)ind2[i]];
        float x0 = sel.x, y0 = sel.y, z0 = sel.z;
        float x1 = t1.x, y1 = t1.y, z1 = t1.z, x2 = t2.x, y2 = t2.y, z2 = t2.z;
        float m11 = ((x0 - x1) * (y0 - y2) - (x0 - x2) * (y0 - y1));
        float m22 = ((x0 - x1) * (z0 - z2) - (x0 - x2) * (z0 - z1));
        float m33 = ((y0 - y1) * (z0 - z2) - (y0 - y2) * (z0 - z1));
        float a012 = std::sqrt(m11 * m11 + m22 * m22 + m33 * m33);
        float l12 = std::sqrt((x1 - x2) * (x1 - x2) + (y1 - y2) * (y1 - y2) + (z1 - z2) * (z1 - z2));
        float la = ((y1 - y2) * m11 + (z1 - z2) * m22) / a012 / l12;
        float lb = -((x1 - x2) * m11 - (z1 - z2) * m33) / a012 / l12;
        float lc = -((x1 - x2) * m22 + (y1 - y2) * m33) / a012 / l12;
        float ld2 = a012 / l12;
        float s = 1;
        if (iter >= 5) s = (float)(1 - 1.8 * (double)std::fabs(ld2));
        if ((double)s > 0.1 && ld2 != 0) {
          laserCloudOri.push_back(sharp[i]);
          coeffSel.push_back({s * la, s * lb, s * lc, s * ld2});
        }
      }
    }
  }

  // findCorrespondingSurfFeatures :1155-1268
  void findCorrespondingSurf(int iter) {
    const int num = (int)flat.size();
    const int lastN = (int)surfLast.size();
    for (int i = 0; i < num; i++) {
      Pt sel;
      toStart(flat[i], sel);
      if (iter % 5 == 0) {
        int nnI; float nnD;
        int got = kdSurf.knn(sel, 1, &nnI, &nnD);
        int closest = -1, min2 = -1, min3 = -1;
        if (got == 1 && nnD < c.nearest_feature_search_sq_dist && nnI < lastN) {
          closest = nnI;
          int cScan = int(surfLast[closest].intensity);
          float minD2 = c.nearest_feature_search_sq_dist, minD3 = c.nearest_feature_search_sq_dist;
          const int jend = std::min(num, lastN);  // bound bug :1173, clamped
          for (int j = closest + 1; j < jend; j++) {
            if ((double)int(surfLast[j].intensity) > cScan + 2.5) break;
            float d = sqd(surfLast[j], sel);
            if (int(surfLast[j].intensity) <= cScan) {
              if (d < minD2) { minD2 = d; min2 = j; }
            } else {
              if (d < minD3) { minD3 = d; min3 = j; }
            }
          }
          for (int j = closest - 1; j >= 0; j--) {
            if ((double)int(surfLast[j].intensity) < cScan - 2.5) break;
            float d = sqd(surfLast[j], sel);
            if (int(surfLast[j].intensity) >= cScan) {
              if (d < minD2) { minD2 = d; min2 = j; }
            } else {
              if (d < minD3) { minD3 = d; min3 = j; }
            }
          }
        }
        ind1[i] = (float)closest;
        ind2[i] = (float)min2;
        ind3[i] = (float)min3;
      }
      if (ind2[i] >= 0 && ind3[i] >= 0) {
        const Pt& t1 = surfLast[(int)ind1[i]];
        const Pt& t2 = surfLast[(int)ind2[i]];
        const Pt& t3 = surfLast[(int)ind3[i]];
        float pa = (t2.y - t1.y) * (t3.z - t1.z) - (t3.y - t1.y) * (t2.z - t1.z);
        float pb = (t2.z - t1.z) * (t3.x - t1.x) - (t3.z - t1.z) * (t2.x - t1.x);
        float pc = (t2.x - t1.x) * (t3.y - t1.y) - (t3.x - t1.x) * (t2.y - t1.y);
        float pd = -(pa * t1.x + pb * t1.y + pc * t1.z);
        float ps = std::sqrt(pa * pa + pb * pb + pc * pc);
        pa /= ps; pb /= ps; pc /= ps; pd /= ps;
        float pd2 = pa * sel.x + pb * sel.y + pc * sel.z + pd;
        float s = 1;
        if (iter >= 5)
          s = (float)(1 - 1.8 * (double)std::fabs(pd2) /
                              (double)std::sqrt(std::sqrt(sel.x * sel.x + sel.y * sel.y + sel.z * sel.z)));
        if ((double)s > 0.1 && pd2 != 0) {
          laserCloudOri.push_back(flat[i]);
          coeffSel.push_back({s * pa, s * pb, s * pc, s * pd2});
        }
      }
    }
  }

  // AtA / AtB as OpenCV's float gemm: double accumulation, float result.
  static void normal_eq3(const std::vector<float>& A, const std::vector<float>& B, int M,
                         float AtA[3][3], float AtB[3]) {
    for (int a = 0; a < 3; a++) {
      for (int b = 0; b < 3; b++) {
        double s = 0;
        for (int r = 0; r < M; r++) s += (double)A[r * 3 + a] * (double)A[r * 3 + b];
        AtA[a][b] = (float)s;
      }
      double s = 0;
      for (int r = 0; r < M; r++) s += (double)A[r * 3 + a] * (double)B[r];
      AtB[a] = (float)s;
    }
  }

  // the shared tail of calculateTransformationSurf/Corner (:1324-1356, :1425-1457)
  void solve3(float AtA[3][3], float AtB[3], int iter, float X[3]) {
    if (log) {
      float rec[12];
      std::memcpy(rec, AtA, 9 * sizeof(float));
      std::memcpy(rec + 9, AtB, 3 * sizeof(float));
      log->add(0, rec, 12);
    }
    float Acopy[3][3];
    std::memcpy(Acopy, AtA, sizeof(Acopy));
    lego::cv_solve_qr<3, 3>(Acopy, *reinterpret_cast<float(*)[3]>(AtB), *reinterpret_cast<float(*)[3]>(X));
    if (iter == 0) {
      float E[3], V[3][3], V2[3][3], Ae[3][3];
      std::memcpy(Ae, AtA, sizeof(Ae));
      lego::cv_eigen_sym<3>(Ae, E, V);
      std::memcpy(V2, V, sizeof(V2));
      isDegenerate = false;
      const float thr[3] = {10, 10, 10};
      for (int i = 2; i >= 0; i--) {
        if (E[i] < thr[i]) {
          for (int j = 0; j < 3; j++) V2[i][j] = 0;
          isDegenerate = true;
        } else {
          break;
        }
      }
      float Vi[3][3];
      lego::cv_inv3(V, Vi);
      lego::cv_matmul<3>(Vi, V2, matP);
    }
    if (isDegenerate) {
      float X2[3] = {X[0], X[1], X[2]};
      lego::cv_matvec<3>(matP, X2, *reinterpret_cast<float(*)[3]>(X));
    }
  }

  static double rad2deg(double r) { return r * 180.0 / M_PI; }

  // calculateTransformationSurf :1270-1377
  bool calcSurf(int iter) {
    const int M = (int)laserCloudOri.size();
    std::vector<float> A(M * 3), B(M);
    float srx = lego_sinf(transformCur[0]), crx = lego_cosf(transformCur[0]);
    float sry = lego_sinf(transformCur[1]), cry = lego_cosf(transformCur[1]);
    float srz = lego_sinf(transformCur[2]), crz = lego_cosf(transformCur[2]);
    float tx = transformCur[3], ty = transformCur[4], tz = transformCur[5];
    float a1 = crx * sry * srz; float a2 = crx * crz * sry; float a3 = srx * sry; float a4 = tx * a1 - ty * a2 - tz * a3;
    float a5 = srx * srz; float a6 = crz * srx; float a7 = ty * a6 - tz * crx - tx * a5;
    float a8 = crx * cry * srz; float a9 = crx * cry * crz; float a10 = cry * srx; float a11 = tz * a10 + ty * a9 - tx * a8;
    float b1 = -crz * sry - cry * srx * srz; float b2 = cry * crz * srx - sry * srz;
    float b5 = cry * crz - srx * sry * srz; float b6 = cry * srz + crz * srx * sry;
    float c1 = -b6; float c2 = b5; float c3 = tx * b6 - ty * b5; float c4 = -crx * crz; float c5 = crx * srz;
    float c6 = ty * c5 + tx * -c4;
    float c7 = b2; float c8 = -b1; float c9 = tx * -b2 - ty * -b1;
    (void)b1;
    for (int i = 0; i < M; i++) {
      const Pt& po = laserCloudOri[i];
      const Pt& cf = coeffSel[i];
      float arx = (-a1 * po.x + a2 * po.y + a3 * po.z + a4) * cf.x +
                  (a5 * po.x - a6 * po.y + crx * po.z + a7) * cf.y +
                  (a8 * po.x - a9 * po.y - a10 * po.z + a11) * cf.z;
      float arz = (c1 * po.x + c2 * po.y + c3) * cf.x + (c4 * po.x - c5 * po.y + c6) * cf.y +
                  (c7 * po.x + c8 * po.y + c9) * cf.z;
      float aty = -b6 * cf.x + c4 * cf.y + b2 * cf.z;
      A[i * 3 + 0] = arx; A[i * 3 + 1] = arz; A[i * 3 + 2] = aty;
      B[i] = (float)(-0.05 * (double)cf.intensity);
    }
    float AtA[3][3], AtB[3], X[3];
    normal_eq3(A, B, M, AtA, AtB);
    solve3(AtA, AtB, iter, X);
    transformCur[0] += X[0];
    transformCur[2] += X[1];
    transformCur[4] += X[2];
    for (int i = 0; i < 6; i++) if (std::isnan(transformCur[i])) transformCur[i] = 0;
    double r0 = rad2deg(X[0]), r1 = rad2deg(X[1]), t2 = (double)(X[2] * 100);
    float deltaR = (float)std::sqrt(r0 * r0 + r1 * r1);
    float deltaT = (float)std::sqrt(t2 * t2);
    return !((double)deltaR < 0.1 && (double)deltaT < 0.1);
  }

  // calculateTransformationCorner :1379-1478
  bool calcCorner(int iter) {
    const int M = (int)laserCloudOri.size();
    std::vector<float> A(M * 3), B(M);
    float srx = lego_sinf(transformCur[0]), crx = lego_cosf(transformCur[0]);
    float sry = lego_sinf(transformCur[1]), cry = lego_cosf(transformCur[1]);
    float srz = lego_sinf(transformCur[2]), crz = lego_cosf(transformCur[2]);
    float tx = transformCur[3], ty = transformCur[4], tz = transformCur[5];
    float b1 = -crz * sry - cry * srx * srz; float b2 = cry * crz * srx - sry * srz; float b3 = crx * cry;
    float b4 = tx * -b1 + ty * -b2 + tz * b3;
    float b5 = cry * crz - srx * sry * srz; float b6 = cry * srz + crz * srx * sry; float b7 = crx * sry;
    float b8 = tz * b7 - ty * b6 - tx * b5;
    float c5 = crx * srz;
    for (int i = 0; i < M; i++) {
      const Pt& po = laserCloudOri[i];
      const Pt& cf = coeffSel[i];
      float ary = (b1 * po.x + b2 * po.y - b3 * po.z + b4) * cf.x + (b5 * po.x + b6 * po.y - b7 * po.z + b8) * cf.z;
      float atx = -b5 * cf.x + c5 * cf.y + b1 * cf.z;
      float atz = b7 * cf.x - srx * cf.y - b3 * cf.z;
      A[i * 3 + 0] = ary; A[i * 3 + 1] = atx; A[i * 3 + 2] = atz;
      B[i] = (float)(-0.05 * (double)cf.intensity);
    }
    float AtA[3][3], AtB[3], X[3];
    normal_eq3(A, B, M, AtA, AtB);
    solve3(AtA, AtB, iter, X);
    transformCur[1] += X[0];
    transformCur[3] += X[1];
    transformCur[5] += X[2];
    for (int i = 0; i < 6; i++) if (std::isnan(transformCur[i])) transformCur[i] = 0;
    double r0 = rad2deg(X[0]), t1 = (double)(X[1] * 100), t2 = (double)(X[2] * 100);
    float deltaR = (float)std::sqrt(r0 * r0);
    float deltaT = (float)std::sqrt(t1 * t1 + t2 * t2);
    return !((double)deltaR < 0.1 && (double)deltaT < 0.1);
  }

  // updateTransformation :1666-1695
  void updateTransformation() {
    if (cornerLastNum < 10 || surfLastNum < 100) return;
    statScans++;
    for (int it = 0; it < 25; it++) {
      laserCloudOri.clear(); coeffSel.clear();
      statSurfIters++;
      if (it % 5 == 0) statNNRounds++;
      findCorrespondingSurf(it);
      statRows += (long)laserCloudOri.size();
      if (laserCloudOri.size() < 10) continue;
      if (!calcSurf(it)) break;
    }
    for (int it = 0; it < 25; it++) {
      laserCloudOri.clear(); coeffSel.clear();
      statCornerIters++;
      if (it % 5 == 0) statNNRounds++;
      findCorrespondingCorner(it);
      statRows += (long)laserCloudOri.size();
      if (laserCloudOri.size() < 10) continue;
      if (!calcCorner(it)) break;
    }
  }

  // integrateTransformation :1697-1725
  void integrateTransformation() {
    float rx, ry, rz, tx, ty, tz;
    accumulateRotation(transformSum[0], transformSum[1], transformSum[2], -transformCur[0],
                       -transformCur[1], -transformCur[2], rx, ry, rz);
    float x1 = lego_cosf(rz) * (transformCur[3] - imuShiftFromStartX) -
               lego_sinf(rz) * (transformCur[4] - imuShiftFromStartY);
    float y1 = lego_sinf(rz) * (transformCur[3] - imuShiftFromStartX) +
               lego_cosf(rz) * (transformCur[4] - imuShiftFromStartY);
    float z1 = transformCur[5] - imuShiftFromStartZ;
    float x2 = x1;
    float y2 = lego_cosf(rx) * y1 - lego_sinf(rx) * z1;
    float z2 = lego_sinf(rx) * y1 + lego_cosf(rx) * z1;
    tx = transformSum[3] - (lego_cosf(ry) * x2 + lego_sinf(ry) * z2);
    ty = transformSum[4] - y2;
    tz = transformSum[5] - (-lego_sinf(ry) * x2 + lego_cosf(ry) * z2);
    pluginIMURotation(rx, ry, rz, imuPitchStart, imuYawStart, imuRollStart, imuPitchLast, imuYawLast,
                      imuRollLast, rx, ry, rz);
    transformSum[0] = rx; transformSum[1] = ry; transformSum[2] = rz;
    transformSum[3] = tx; transformSum[4] = ty; transformSum[5] = tz;
  }

  // publishCloudsLast :1759-1815
  void publishCloudsLast() {
    updateImuStartSinCos();
    for (Pt& p : lessSharp) toEnd(p, p);
    for (Pt& p : lessFlat) toEnd(p, p);
    std::swap(lessSharp, cornerLast);
    std::swap(lessFlat, surfLast);
    cornerLastNum = (int)cornerLast.size();
    surfLastNum = (int)surfLast.size();
    if (cornerLastNum > 10 && surfLastNum > 100) {
      kdCorner.build(cornerLast);
      kdSurf.build(surfLast);
    }
    frameCount++;
    publishToMapping = false;
    if (frameCount >= c.skip_frame_num + 1) {
      frameCount = 0;
      publishToMapping = true;
      outOutlierLast.resize(outlierCloud.size());
      for (size_t i = 0; i < outlierCloud.size(); ++i)  // adjustOutlierCloud :1746-1757
        outOutlierLast[i] = {outlierCloud[i].y, outlierCloud[i].z, outlierCloud[i].x, outlierCloud[i].intensity};
      outCornerLast = cornerLast;
      outSurfLast = surfLast;
    }
  }

  // checkSystemInitialization :1605-1637
  void checkSystemInitialization() {
    std::swap(lessSharp, cornerLast);
    std::swap(lessFlat, surfLast);
    kdCorner.build(cornerLast);
    kdSurf.build(surfLast);
    cornerLastNum = (int)cornerLast.size();
    surfLastNum = (int)surfLast.size();
    transformSum[0] += imuPitchStart;
    transformSum[2] += imuRollStart;
    systemInitedLM = true;
  }

  int process(const lego_ip_out* in) {
    if (!in || in->n_segmented < 0) return LEGO_E_ARG;
    const int ns = in->n_segmented;
    segmentedCloud.assign(in->segmented_cloud, in->segmented_cloud + ns);
    outlierCloud.assign(in->outlier_cloud, in->outlier_cloud + in->n_outlier);
    sri.assign(in->info.start_ring_index, in->info.start_ring_index + N);
    eri.assign(in->info.end_ring_index, in->info.end_ring_index + N);
    gflag.assign(P, 0); colInd.assign(P, 0); segRange.assign(P, 0.f);
    std::copy(in->info.segmented_cloud_ground_flag, in->info.segmented_cloud_ground_flag + ns, gflag.begin());
    std::copy(in->info.segmented_cloud_col_ind, in->info.segmented_cloud_col_ind + ns, colInd.begin());
    std::copy(in->info.segmented_cloud_range, in->info.segmented_cloud_range + ns, segRange.begin());
    startOri = in->info.start_orientation; endOri = in->info.end_orientation;
    oriDiff = in->info.orientation_diff;
    stamp = in->info.stamp;
    adjustDistortion();
    calculateSmoothness();
    markOccludedPoints();
    extractFeatures();
    // copies of the published feature clouds (before the swap in the hand-off)
    pubSharp = sharp; pubLessSharp = lessSharp; pubFlat = flat; pubLessFlat = lessFlat;
    publishToMapping = false;
    if (!systemInitedLM) {
      checkSystemInitialization();
      odomValid = false;
      return LEGO_OK;
    }
    updateInitialGuess();
    updateTransformation();
    integrateTransformation();
    odomValid = true;
    publishCloudsLast();
    return LEGO_OK;
  }
  std::vector<Pt> pubSharp, pubLessSharp, pubFlat, pubLessFlat;
  long statSurfIters = 0, statCornerIters = 0, statNNRounds = 0, statScans = 0, statRows = 0;
};

#include "oracle_mo.inc"

}  // namespace oracle

// ============================================================ C ABI
struct lego_oracle {
  lego_sensor_cfg cfg;
  std::unique_ptr<oracle::ImageProjection> ip;
  std::unique_ptr<oracle::FeatureAssociation> fa;
  std::unique_ptr<oracle::MapOptimization> mo;
  oracle::TransformFusionNode fusion;
  double ip_stamp = 0;
  oracle::SysLog log;
};

extern "C" int lego_oracle_sensor_preset(const char* name, lego_sensor_cfg* out) {
  return oracle::sensor_preset(name, out);
}

extern "C" int lego_oracle_create(const lego_sensor_cfg* cfg, lego_oracle** out) {
  if (!cfg || !out || cfg->n_scan <= 0 || cfg->horizon_scan <= 0 || cfg->ground_scan_ind < 0 ||
      cfg->ground_scan_ind >= cfg->n_scan)
    return LEGO_E_ARG;
  lego_oracle* o = new lego_oracle;
  o->cfg = *cfg;
  o->ip.reset(new oracle::ImageProjection(*cfg));
  o->fa.reset(new oracle::FeatureAssociation(*cfg));
  o->mo.reset(new oracle::MapOptimization(*cfg));
  o->fa->log = &o->log;
  o->mo->log = &o->log;
  o->fa->pcl_sort = (LEGO_ORACLE_DEFAULT_OPTS & LEGO_ORACLE_VG_FA) != 0;
  o->mo->pcl_sort = (LEGO_ORACLE_DEFAULT_OPTS & LEGO_ORACLE_VG_MO) != 0;
  *out = o;
  return LEGO_OK;
}

extern "C" int lego_oracle_destroy(lego_oracle* o) {
  delete o;
  return LEGO_OK;
}

extern "C" int lego_oracle_set_options(lego_oracle* o, uint32_t opts) {
  if (!o) return LEGO_E_ARG;
  o->fa->pcl_sort = (opts & LEGO_ORACLE_VG_FA) != 0;
  o->mo->pcl_sort = (opts & LEGO_ORACLE_VG_MO) != 0;
  return LEGO_OK;
}

extern "C" int lego_oracle_ip_process(lego_oracle* o, const lego_point_xyzir* pts, int32_t n,
                                      double stamp, uint32_t flags, lego_ip_out* out) {
  if (!o || !out) return LEGO_E_ARG;
  auto& ip = *o->ip;
  int st = ip.process(pts, n, (flags & LEGO_IP_IMAGES) != 0, (flags & LEGO_IP_GATED) != 0);
  if (st != LEGO_OK) return st;
  std::memset(out, 0, sizeof(*out));
  out->info.stamp = stamp;
  out->info.start_ring_index = ip.startRingIndex.data();
  out->info.end_ring_index = ip.endRingIndex.data();
  out->info.start_orientation = ip.startOrientation;
  out->info.end_orientation = ip.endOrientation;
  out->info.orientation_diff = ip.orientationDiff;
  out->info.segmented_cloud_ground_flag = ip.groundFlag.data();
  out->info.segmented_cloud_col_ind = ip.colInd.data();
  out->info.segmented_cloud_range = ip.segRange.data();
  out->segmented_cloud = ip.segmentedCloud.data();
  out->n_segmented = (int32_t)ip.segmentedCloud.size();
  out->outlier_cloud = ip.outlierCloud.data();
  out->n_outlier = (int32_t)ip.outlierCloud.size();
  if (flags & LEGO_IP_IMAGES) {
    out->full_cloud = ip.fullCloud.data();
    out->range_image = ip.rangeMat.data();
    out->ground_image = ip.groundMat.data();
    out->label_image = ip.labelMat.data();
  }
  if (flags & LEGO_IP_GATED) {  // publishCloud :480-506
    out->full_info_cloud = ip.fullInfoCloud.data();
    out->ground_cloud = ip.groundCloud.data();
    out->n_ground = (int32_t)ip.groundCloud.size();
    out->segmented_cloud_pure = ip.segmentedCloudPure.data();
    out->n_segmented_pure = (int32_t)ip.segmentedCloudPure.size();
  }
  return LEGO_OK;
}

extern "C" int lego_oracle_fa_process(lego_oracle* o, const lego_ip_out* in, lego_fa_out* out) {
  if (!o || !in || !out) return LEGO_E_ARG;
  auto& fa = *o->fa;
  int st = fa.process(in);
  if (st != LEGO_OK) return st;
  std::memset(out, 0, sizeof(*out));
  out->stamp = in->info.stamp;
  out->sharp = fa.pubSharp.data(); out->n_sharp = (int32_t)fa.pubSharp.size();
  out->less_sharp = fa.pubLessSharp.data(); out->n_less_sharp = (int32_t)fa.pubLessSharp.size();
  out->flat = fa.pubFlat.data(); out->n_flat = (int32_t)fa.pubFlat.size();
  out->less_flat = fa.pubLessFlat.data(); out->n_less_flat = (int32_t)fa.pubLessFlat.size();
  out->odom_valid = fa.odomValid;
  for (int i = 0; i < 6; ++i) {
    out->transform_cur[i] = fa.transformCur[i];
    out->transform_sum[i] = fa.transformSum[i];
  }
  oracle::odom_quaternion(fa.transformSum, out->odom_quat, out->odom_pos);
  out->publish_to_mapping = fa.publishToMapping;
  if (fa.publishToMapping) {
    out->corner_last = fa.outCornerLast.data(); out->n_corner_last = (int32_t)fa.outCornerLast.size();
    out->surf_last = fa.outSurfLast.data(); out->n_surf_last = (int32_t)fa.outSurfLast.size();
    out->outlier_last = fa.outOutlierLast.data(); out->n_outlier_last = (int32_t)fa.outOutlierLast.size();
  }
  return LEGO_OK;
}

extern "C" int lego_oracle_fusion_odometry(lego_oracle* o, const lego_fa_out* odom, lego_fusion_out* out) {
  if (!o || !odom || !out) return LEGO_E_ARG;
  o->fusion.laserOdometryHandler(odom->odom_quat, odom->odom_pos);
  std::memset(out, 0, sizeof(*out));
  out->stamp = odom->stamp;
  for (int i = 0; i < 6; ++i) out->transform_mapped[i] = o->fusion.transformMapped[i];
  oracle::odom_quaternion(o->fusion.transformMapped, out->quat, out->pos);  // :187-196
  return LEGO_OK;
}

extern "C" int lego_oracle_fusion_aft_mapped(lego_oracle* o, const lego_mo_out* mo) {
  if (!o || !mo) return LEGO_E_ARG;
  if (!mo->processed) return LEGO_OK;
  double q[4], pos[3];
  oracle::odom_quaternion(mo->transform_aft_mapped, q, pos);  // publishTF, mapOptmization.cpp:656-665
  o->fusion.odomAftMappedHandler(q, pos, mo->transform_bef_mapped);
  return LEGO_OK;
}

extern "C" int lego_oracle_imu_push(lego_oracle* o, const lego_imu_msg* msgs, int32_t n) {
  if (!o || n < 0 || (n > 0 && !msgs)) return LEGO_E_ARG;
  for (int i = 0; i < n; ++i) {  // both nodes subscribe to /imu_raw
    o->fa->imuHandler(msgs[i]);
    o->mo->imuHandler(msgs[i]);
  }
  return LEGO_OK;
}

extern "C" int lego_oracle_voxel_grid(const lego_point_xyzi* in, int32_t n, float leaf,
                                      int32_t pcl_sort, lego_point_xyzi* out, int32_t* n_out) {
  if ((n && !in) || !out || !n_out || n < 0) return LEGO_E_ARG;
  std::vector<oracle::Pt> a(in, in + n), b;
  oracle::voxel_grid(a, leaf, pcl_sort != 0, b);
  std::copy(b.begin(), b.end(), out);
  *n_out = (int32_t)b.size();
  return LEGO_OK;
}

extern "C" int lego_oracle_sort_permutation(const uint32_t* keys, int32_t n, int32_t* perm) {
  if (n < 0 || (n && (!keys || !perm))) return LEGO_E_ARG;
  struct KI {  // voxel_grid.hpp's cloud_point_index_idx: compared by idx alone
    uint32_t idx;
    int32_t i;
    bool operator<(const KI& o) const { return idx < o.idx; }
  };
  std::vector<KI> a((size_t)n);
  for (int32_t i = 0; i < n; ++i) a[(size_t)i] = {keys[i], i};
  std::sort(a.begin(), a.end());
  for (int32_t i = 0; i < n; ++i) perm[i] = a[(size_t)i].i;
  return LEGO_OK;
}

extern "C" float lego_oracle_atan2f(float y, float x) { return lego_atan2f(y, x); }
extern "C" float lego_oracle_sinf(float x) { return lego_sinf(x); }
extern "C" float lego_oracle_cosf(float x) { return lego_cosf(x); }
extern "C" float lego_oracle_asinf(float x) { return lego_asinf(x); }

extern "C" int lego_oracle_mo_set_map(lego_oracle* o, const lego_point_xyzi* corner, int32_t n_corner,
                                      const lego_point_xyzi* surf, int32_t n_surf) {
  if (!o) return LEGO_E_ARG;
  auto& mo = *o->mo;
  if (!corner && !surf) {
    mo.fixedMap = false;
    mo.fixedCorner.clear(); mo.fixedSurf.clear();
    return LEGO_OK;
  }
  if (!corner || !surf || n_corner < 0 || n_surf < 0) return LEGO_E_ARG;
  mo.fixedMap = true;
  mo.fixedCorner.assign(corner, corner + n_corner);
  mo.fixedSurf.assign(surf, surf + n_surf);
  return LEGO_OK;
}

extern "C" int lego_oracle_mo_configure(lego_oracle* o, const lego_mo_opts* opts) {
  if (!o || !opts) return LEGO_E_ARG;
  if ((opts->loop_closure_enable != 0) != o->mo->loopClosureEnable && !o->mo->keyPoses3D.empty())
    return LEGO_E_STATE;
  o->mo->loopClosureEnable = opts->loop_closure_enable != 0;
  o->mo->keyframeSearchNum = opts->surrounding_keyframe_search_num > 0 ? opts->surrounding_keyframe_search_num : 50;
  return LEGO_OK;  // fixed_map_per_step: the oracle filters the map every step anyway
}

extern "C" int lego_oracle_mo_loop_closure(lego_oracle* o, lego_loop_out* out) {
  if (!o || !out) return LEGO_E_ARG;
  return o->mo->loopClosure(out);
}

extern "C" int lego_oracle_mo_process(lego_oracle* o, const lego_fa_out* in, lego_mo_out* out) {
  if (!o || !in || !out) return LEGO_E_ARG;
  auto& mo = *o->mo;
  int st = mo.process(in);
  if (st != LEGO_OK) return st;
  std::memset(out, 0, sizeof(*out));
  out->processed = mo.processed;
  if (!mo.processed) return LEGO_OK;  // nothing published this call (the product's ABI too)
  out->optimized = mo.processed && mo.optimized;
  out->iterations = mo.iterations;
  for (int i = 0; i < 6; ++i) {
    out->transform_tobe_mapped[i] = mo.transformTobeMapped[i];
    out->transform_aft_mapped[i] = mo.transformAftMapped[i];
    out->transform_bef_mapped[i] = mo.transformBefMapped[i];
  }
  out->n_corner_map_ds = mo.cornerFromMapDSNum;
  out->n_surf_map_ds = mo.surfFromMapDSNum;
  out->n_corner_scan_ds = (int32_t)mo.cornerLastDS.size();
  out->n_surf_scan_ds = (int32_t)mo.surfTotalLastDS.size();
  out->n_rows_last = mo.rowsLast;
  return LEGO_OK;
}

extern "C" int lego_oracle_log_systems(lego_oracle* o, int32_t enable) {
  if (!o) return LEGO_E_ARG;
  o->log = oracle::SysLog{};
  o->log.on = enable != 0;
  return LEGO_OK;
}

extern "C" int lego_oracle_systems(lego_oracle* o, int32_t kind, float* out, int32_t cap, int32_t* n) {
  if (!o || !n || kind < 0 || kind > 3) return LEGO_E_ARG;
  const auto& v = o->log.v[kind];
  *n = (int32_t)v.size();
  if (out) std::memcpy(out, v.data(), sizeof(float) * std::min<size_t>(v.size(), (size_t)std::max(cap, 0)));
  return LEGO_OK;
}

extern "C" int lego_oracle_stats(lego_oracle* o, long* out5) {
  if (!o || !out5) return LEGO_E_ARG;
  out5[0] = o->fa->statScans; out5[1] = o->fa->statSurfIters; out5[2] = o->fa->statCornerIters;
  out5[3] = o->fa->statNNRounds; out5[4] = o->fa->statRows;
  return LEGO_OK;
}
