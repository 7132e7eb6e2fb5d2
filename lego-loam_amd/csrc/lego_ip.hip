// lego_ip.hip — imageProjection hot path on gfx950.
//
//   k_project   1 lane / input point: ring -> row, atan2f -> column, range;
//               last-writer-wins through atomicMax on the point index
//               (imageProjection.cpp:219-256)
//   k_pixels    1 lane / pixel: rangeMat + fullCloud (:248-255)
//   k_ground    1 lane / column: the sequential ground-pair walk (:267-301)
//   k_seg_lds   VLP-16-class images: 1 workgroup / scan, BFS segmentation
//               as union-find in LDS + the ordered compaction (below)
//   k_ccl_*     larger images: BFS segmentation as connected components
//               (:312-317, 370-460): symmetric edge predicate -> union-find
//               with CAS on roots in HBM; the root is the component's minimum
//               raster index = the BFS seed
//   k_seg_flags / _scan / _write / _labels
//               their compaction, one 1024-pixel chunk per workgroup:
//               component validity, label ranking, row-major compaction into
//               segmented cloud + cloud_info, outlier cloud (:319-355)
//
// All float expressions mirror the reference's mixed float/double evaluation
// (SURVEY.md §9.2); compiled with -ffp-contract=off.
#include <cfloat>

#include <algorithm>
#include <cstdlib>

#include "lego_device.h"
#include "lego_kernels.h"
#include "lego_seg.h"
#include "lego_loam.h"

namespace lego {

// Diagnostic build (IP_PROF=1, scripts/ip_phase.sh): thread 0 of every
// k_ip_lds workgroup adds the clock64 ticks between its phase barriers to
// g_ipprof (lego_ip_profile reads and clears them).  No effect otherwise.
#ifndef IP_PROF
#define IP_PROF 0
#endif
#if IP_PROF
constexpr int kIpProf = 12;  // [0, 10): phases, 11: workgroups
__device__ unsigned long long g_ipprof[kIpProf];
#define IP_T0() unsigned long long ipt_ = threadIdx.x == 0 ? (unsigned long long)clock64() : 0ull
#define IP_STAMP(k)                                                      \
  do {                                                                   \
    if (threadIdx.x == 0) {                                              \
      const unsigned long long n_ = clock64();                           \
      atomicAdd(&g_ipprof[k], n_ - ipt_);                                \
      ipt_ = n_;                                                         \
    }                                                                    \
  } while (0)
#else
#define IP_T0() (void)0
#define IP_STAMP(k) (void)0
#endif

__device__ __forceinline__ bool xyz_finite(const float4& p) {
  return __builtin_isfinite(p.x) && __builtin_isfinite(p.y) && __builtin_isfinite(p.z);
}

// projectPointCloud for point i of scan b (:219-256): its pixel, or -1 when
// it is dropped; findStartEndAngle's two raw angles (:201-202) from the
// scan's first / last point, and the non-dense flag.  k_project (one lane per
// point, the owner image in HBM) and k_ip_lds (one workgroup per scan, the
// owner image in LDS) share it.
// Scan b's points: the caller's XYZIR records (32 B), or, with bit 0 of
// bb.pts set, the node call's packed form (16 B: x, y, z and the ring's bits
// in the fourth word; upload_checked in lego_api.hip).
struct PtsView {
  const unsigned char* base;
  bool packed;
  __device__ __forceinline__ float4 xyz(int i) const {
    return *(const float4*)(base + (size_t)i * (packed ? 16 : 32));
  }
};
__device__ __forceinline__ PtsView pts_view(const BatchBufs& bb, int b) {
  const uintptr_t a = (uintptr_t)bb.pts;
  const bool packed = (a & 1) != 0;
  return PtsView{(const unsigned char*)(a & ~(uintptr_t)1) + (size_t)bb.off[b] * (packed ? 16 : 32), packed};
}

__device__ __forceinline__ int project_point(const BatchBufs& bb, const DevCfg& c, int b, int n, int i) {
  const PtsView pv = pts_view(bb, b);
  const float4 xyz = pv.xyz(i);
  const uint16_t ring = pv.packed ? (uint16_t)__float_as_uint(xyz.w) : ((const lego_point_xyzir*)pv.base + i)->ring;
  const float x = xyz.x, y = xyz.y, z = xyz.z;
  if (!xyz_finite(xyz)) {
    if (c.ringRow) {
      bb.bad[b] = kBadNotDense;  // the host rejects the batch with LEGO_E_NOT_DENSE
      return -1;
    }
    // useCloudRing = false: removeNaNFromPointCloud (:170) drops the point,
    // and points[0] / points[size - 1] of findStartEndAngle (:201-202) are
    // the first / last finite ones.  One lane walks inwards from each end
    // (the walk is as long as the run of non-finite points at that end).
    if (i == 0) {
      int k = 1;
      while (k < n && !xyz_finite(pv.xyz(k))) ++k;
      if (k == n) {
        bb.bad[b] = kBadNotDense;  // no finite point: points[0] of an empty cloud (UB upstream)
        return -1;
      }
      const float4 q = pv.xyz(k);
      bb.rawang[2 * b] = -lego_atan2f(q.y, q.x);
    }
    if (i == n - 1) {
      int k = n - 2;
      while (k >= 0 && !xyz_finite(pv.xyz(k))) --k;
      if (k >= 0) {
        const float4 q = pv.xyz(k);
        bb.rawang[2 * b + 1] = -lego_atan2f(q.y, q.x);
      }
    }
    return -1;
  }
  if (i == 0) bb.rawang[2 * b] = -lego_atan2f(y, x);                   // :201
  if (i == n - 1) bb.rawang[2 * b + 1] = -lego_atan2f(y, x);           // :202
  int row;
  if (c.ringRow) {
    row = ring;  // :226
    if (row >= c.N) return -1;
  } else {
    // :229-230: float atan2 / sqrt (utility.h's `using namespace std`), the
    // product with 180 in float, the division by M_PI in double, stored to
    // the float verticalAngle; then (float + float) / float
    const float va = (float)((double)(lego_atan2f(z, __builtin_sqrtf(x * x + y * y)) * 180.0f) / M_PI);
    const float v = (va + c.ang_bottom) / c.ang_res_y;
    // rowIdn is size_t: x86-64 converts a float below 2^63 by truncation
    // toward zero through int64, so (-1, 0) gives row 0 and v <= -1 an index
    // past N_SCAN (skipped by :232, where `rowIdn < 0` is always false)
    if (!(v > -1.0f && v < (float)c.N)) return -1;
    row = (int)v;
  }
  const float h = (float)((double)(lego_atan2f(x, y) * 180.0f) / M_PI);  // :235
  const double cd = -round(((double)h - 90.0) / (double)c.ang_res_x) + (double)(c.H / 2);
  if (cd < 0) return -1;
  long col = (long)cd;
  if (col >= c.H) col -= c.H;
  if (col >= c.H) return -1;
  const float range = __builtin_sqrtf(x * x + y * y + z * z);          // :244
  if (range < c.min_range) return -1;
  return row * c.H + (int)col;
}

__global__ void k_project(BatchBufs bb, DevCfg c) {
  const int b = blockIdx.y;
  const int n = scan_npts(bb, b);
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int pix = project_point(bb, c, b, n, i);
  if (pix >= 0) atomicMax(&bb.owner[(size_t)b * c.P + pix], i);  // last writer wins (:248-255)
}

// A pixel of the range image and the full cloud (:248-255) from its owner
// point o (-1: none) and that point's coordinates.
__device__ __forceinline__ void pixel_store(const BatchBufs& bb, const DevCfg& c, int b, int row, int col, int o,
                                            float4 xyz) {
  const size_t gp = (size_t)b * c.P + row * c.H + col;
  if (o < 0) {
    bb.range[gp] = FLT_MAX;
    const float qn = __builtin_nanf("");
    bb.full[gp] = make_float4(qn, qn, qn, -1.0f);
    return;
  }
  const float range = __builtin_sqrtf(xyz.x * xyz.x + xyz.y * xyz.y + xyz.z * xyz.z);
  const float inten = (float)((double)(float)row + (double)(float)col / 10000.0);  // :250
  bb.range[gp] = range;
  bb.full[gp] = make_float4(xyz.x, xyz.y, xyz.z, inten);
}
__device__ __forceinline__ void pixel_out(const BatchBufs& bb, const DevCfg& c, int b, int row, int col, int o) {
  pixel_store(bb, c, b, row, col, o, o >= 0 ? pts_view(bb, b).xyz(o) : make_float4(0.f, 0.f, 0.f, 0.f));
}

// One workgroup per 4 rows x 64 columns (a wave per row): the stores stay
// row-contiguous, and the records a wave gathers (16 rings apart in firing
// order) share their 128-B lines with the other three waves' at the same
// columns, so each line is fetched once per workgroup instead of once per row
// (rocprofv3 FETCH_SIZE calibration: scripts/mb/mb_gather.hip).
__global__ void __launch_bounds__(256) k_pixels(BatchBufs bb, DevCfg c) {
  const int b = blockIdx.z;
  const int row = blockIdx.y * 4 + (threadIdx.x >> 6), col = blockIdx.x * 64 + (threadIdx.x & 63);
  if (row >= c.N || col >= c.H) return;
  const int p = row * c.H + col;
  const size_t gp = (size_t)b * c.P + p;
  const int o = bb.owner[gp];
  // the owner image is left all -1 for the slot's next batch (k_project's
  // atomicMax needs it so): the pixel that was written is cleared here, in
  // place of a separate fill of the whole image before every batch (a fleet
  // call's 590 MB fill took ~1.4 ms of a ~20 ms call)
  if (o >= 0) bb.owner[gp] = -1;
  pixel_out(bb, c, b, row, col, o);
}

// groundMat column walk.  Carry form of the overwrite semantics:
// G[i] is final once pair (i, i+1) has been examined.  Rows in chunks of
// kGroundRows: the chunk's points and ranges are loaded before any of its
// stores (one memory latency per chunk; the stores' possible aliasing kept
// the per-row form's loads behind the previous row's stores: ~13.5 us for a
// single VLP-16 scan, 16 dependent rows).
constexpr int kGroundRows = 8;
// Column j of scan b; par (k_ip_lds): the union-find's initial parents of
// the column's pixels in LDS as well (p for an unlabelled pixel, -2 for a
// ground one, else -1);
// labels: also the ground image and the label image's initial values (the
// HBM union-find and compaction read them; k_ip_lds needs them only when the
// images are outputs: its segmentation takes the ground from the parents).
__device__ __forceinline__ void ground_column(const BatchBufs& bb, const DevCfg& c, int b, int j, int* par,
                                              bool labels = true) {
  const size_t base = (size_t)b * c.P;
  int cur = 0;  // value G[i] holds before pair i is examined
  for (int i0 = 0; i0 < c.N; i0 += kGroundRows) {
    float4 pt[kGroundRows + 1];  // rows i0 .. i0 + kGroundRows, where a pair (i < g) reads them
    float rg[kGroundRows];
#pragma unroll
    for (int u = 0; u <= kGroundRows; ++u) {
      const int i = i0 + u;
      pt[u] = i <= c.g && i < c.N ? bb.full[base + i * c.H + j] : make_float4(0.f, 0.f, 0.f, 0.f);
      if (u < kGroundRows) rg[u] = i < c.N ? bb.range[base + i * c.H + j] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < kGroundRows; ++u) {
      const int i = i0 + u;
      if (i >= c.N) break;
      int G;
      int next = 0;
      if (i < c.g) {
        const float4 lo = pt[u], up = pt[u + 1];
        if (lo.w == -1.0f || up.w == -1.0f) {
          G = -1;
        } else {
          const float dX = up.x - lo.x, dY = up.y - lo.y, dZ = up.z - lo.z;
          const float angle =
              (float)((double)(lego_atan2f(dZ, __builtin_sqrtf(dX * dX + dY * dY)) * 180.0f) / M_PI);
          if (lfabsf(angle - c.mount_angle) <= 10) {
            G = 1;
            next = 1;
          } else {
            G = cur;
          }
        }
      } else {
        G = cur;
      }
      cur = next;
      const size_t gp = base + i * c.H + j;
      const bool lab = G == 1 || rg[u] == FLT_MAX;
      if (labels) {  // the images (k_ip_lds reads neither unless they are outputs)
        bb.ground[gp] = (int8_t)G;
        bb.label[gp] = lab ? -1 : 0;  // :295-301
      }
      // k_ip_lds's parents: -2 for a ground pixel (G == 1), -1 for another
      // labelled one, so the segmentation knows the ground without the image
      if (par) par[i * c.H + j] = lab ? (G == 1 ? -2 : -1) : i * c.H + j;
    }
  }
}

__global__ void k_ground(BatchBufs bb, DevCfg c) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j < c.H) ground_column(bb, c, blockIdx.y, j, nullptr);
}

__device__ __forceinline__ TanBand seg_tan_band(const DevCfg& c) {  // computed on the host
  return TanBand{c.tanLo, c.tanHi, c.quad1 != 0};
}

__global__ void k_ccl_init(BatchBufs bb, DevCfg c) {
  const int b = blockIdx.y;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= c.P) return;
  const size_t base = (size_t)b * c.P;
  const int L = bb.label[base + p];
  bb.parent[base + p] = (L == 0) ? p : -1;
  // the size and row counters k_ccl_root accumulates into (two launches later)
  bb.csize[base + p] = 0;
  bb.rowmask[(base + p) * 2] = 0ull;
  bb.rowmask[(base + p) * 2 + 1] = 0ull;
  uint8_t e = 0;
  if (L == 0) {
    const int row = p / c.H, col = p - row * c.H;
    const float r = bb.range[base + p];
    const int qr = row * c.H + (col + 1 == c.H ? 0 : col + 1);        // column wrap :403-406
    const TanBand tb = seg_tan_band(c);
    if (bb.label[base + qr] == 0 && seg_edge_fast(r, bb.range[base + qr], c.sinAX, c.cosAX, c.theta, tb)) e |= 1;
    if (row + 1 < c.N) {
      const int qd = p + c.H;
      if (bb.label[base + qd] == 0 && seg_edge_fast(r, bb.range[base + qd], c.sinAY, c.cosAY, c.theta, tb)) e |= 2;
    }
  }
  bb.edges[base + p] = e;
}

__device__ __forceinline__ int uf_load(int* a) {
  return __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int uf_find(int* par, int x) {
  while (true) {
    const int p = uf_load(&par[x]);
    if (p == x) return x;
    x = p;
  }
}
__device__ __forceinline__ void uf_unite(int* par, int a, int b) {
  while (true) {
    a = uf_find(par, a);
    b = uf_find(par, b);
    if (a == b) return;
    if (a < b) { const int t = a; a = b; b = t; }  // link the larger root under the smaller
    const int old = atomicCAS(&par[a], a, b);
    if (old == a) return;
  }
}

__device__ __forceinline__ int lds_find(volatile int* par, int x) {
  while (true) {
    const int p = par[x];
    if (p == x) return x;
    x = p;
  }
}
__device__ __forceinline__ void lds_unite(int* par, int a, int b) {
  while (true) {
    a = lds_find(par, a);
    b = lds_find(par, b);
    if (a == b) return;
    if (a < b) { const int t = a; a = b; b = t; }  // the larger root under the smaller
    if (atomicCAS(&par[a], a, b) == a) return;
  }
}

__global__ void k_ccl_union(BatchBufs bb, DevCfg c) {
  const int b = blockIdx.y;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= c.P) return;
  const size_t base = (size_t)b * c.P;
  const uint8_t e = bb.edges[base + p];
  if (!e) return;
  int* par = bb.parent + base;
  const int row = p / c.H, col = p - row * c.H;
  if (e & 1) uf_unite(par, p, row * c.H + (col + 1 == c.H ? 0 : col + 1));
  if (e & 2) uf_unite(par, p, p + c.H);
}

// Each pixel's root, and the roots' sizes and row masks.  The counts are
// aggregated per wave first (a wave's 64 consecutive pixels lie in one or two
// rows and mostly share their root): one atomic per distinct root of the
// wave, not one per pixel on the same word (a large segment's thousands of
// pixels had serialised on its root's counters).
__global__ void k_ccl_root(BatchBufs bb, DevCfg c) {
  const int b = blockIdx.y;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  const size_t base = (size_t)b * c.P;
  const bool cand = p < c.P && bb.parent[base + p] >= 0;
  int r = -1;
  if (cand) {
    r = uf_find(bb.parent + base, p);
    bb.root[base + p] = r;
  }
  const int row = p / c.H;
  // lineCountFlag is set only for pushed (non-seed) pixels (:431)
  const unsigned long long rbit = (cand && r != p) ? 1ull << (row & 63) : 0ull;
  const int lane = threadIdx.x & 63;
  for (unsigned long long act = __ballot(cand); act;) {
    const int lead = __ffsll((long long)act) - 1;
    const int r0 = __shfl(r, lead, 64);
    const bool mine = cand && r == r0;
    const unsigned long long same = __ballot(mine);
    unsigned long long lo = mine && row < 64 ? rbit : 0ull, hi = mine && row >= 64 ? rbit : 0ull;
    for (int o = 32; o > 0; o >>= 1) {
      lo |= __shfl_xor(lo, o, 64);
      hi |= __shfl_xor(hi, o, 64);
    }
    if (lane == lead) {
      atomicAdd(&bb.csize[base + r0], (int)__popcll(same));
      if (lo) atomicOr(&bb.rowmask[(base + r0) * 2], lo);
      if (hi) atomicOr(&bb.rowmask[(base + r0) * 2 + 1], hi);
    }
    act &= ~same;
  }
}

// The union-find in column tiles (images too large for k_seg_lds's one
// workgroup): a 1024-thread workgroup per (scan, tile of TW columns x all
// rows, <= kCclTilePx pixels) unites the tile's pixels over its own right and
// down edges in LDS (lds_unite: the larger root under the smaller, so a
// root is its component's smallest index, row-major within the tile as in
// the image), then writes every pixel's tile root as its parent (a forest of
// depth one) and zeroes the counters k_ccl_root accumulates.  k_ccl_seam then
// unites across the tiles' seams (the column wrap among them, :403-406) in
// HBM; the smallest tile root of a component becomes its root, the same
// index the HBM-only union-find (k_ccl_init / _union) gives.
constexpr int kCclTilePx = 32768;  // 128 KB of parents
// A launch of few scans takes narrower tiles, so that it still spreads over
// kCclMinTiles workgroups: one VLP-16 scan was one tile, one workgroup's
// serial unions (68 us in the node call's trace, gpurun_out r05p/node), now 64
// tiles of 29 columns and their seams.
constexpr int kCclMinTiles = 64, kCclMinWidth = 16;
int ccl_tile_width(const DevCfg& c, int B) {
  const int byLds = std::max(1, kCclTilePx / c.N);
  const int byGrid = std::max(kCclMinWidth, (c.H * B + kCclMinTiles - 1) / kCclMinTiles);
  const int tw = std::min(byLds, byGrid);
  return tw >= c.H ? c.H : tw;
}
__global__ void __launch_bounds__(1024) k_ccl_tile(BatchBufs bb, DevCfg c, int TW) {
  extern __shared__ int par[];  // [N * tw], index row * tw + (col - c0)
  volatile int* vpar = par;
  const int b = blockIdx.y, c0 = blockIdx.x * TW, tid = threadIdx.x;
  const int H = c.H, tw = min(TW, H - c0), n = c.N * tw;
  const bool whole = tw == H;  // one tile: the column wrap is inside it
  const size_t base = (size_t)b * c.P;
  const TanBand tb = seg_tan_band(c);
  for (int l = tid; l < n; l += blockDim.x) {
    const int row = l / tw, p = row * H + c0 + (l - row * tw);
    par[l] = bb.label[base + p] == 0 ? l : -1;
    bb.csize[base + p] = 0;
    bb.rowmask[(base + p) * 2] = 0ull;
    bb.rowmask[(base + p) * 2 + 1] = 0ull;
  }
  __syncthreads();
  for (int l0 = 0; l0 < n; l0 += 4 * (int)blockDim.x) {  // four pixels' ranges in flight per thread
    float rp[4], rr_[4], rd[4];
    int pp[4], qrl[4], qrp[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int l = l0 + u * (int)blockDim.x + tid;
      rp[u] = rr_[u] = rd[u] = 0.f;
      pp[u] = -1;
      qrl[u] = qrp[u] = -1;
      if (l < n) {
        const int row = l / tw, cc = l - row * tw, p = row * H + c0 + cc;
        pp[u] = p;
        if (cc + 1 < tw) { qrl[u] = l + 1; qrp[u] = p + 1; }
        else if (whole) { qrl[u] = row * tw; qrp[u] = row * H; }
        rp[u] = bb.range[base + p];
        if (qrp[u] >= 0) rr_[u] = bb.range[base + qrp[u]];
        if (row + 1 < c.N) rd[u] = bb.range[base + p + H];
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int l = l0 + u * (int)blockDim.x + tid;
      if (pp[u] < 0 || vpar[l] < 0) continue;  // candidates keep a parent >= 0 throughout
      if (qrl[u] >= 0 && vpar[qrl[u]] >= 0 && seg_edge_fast(rp[u], rr_[u], c.sinAX, c.cosAX, c.theta, tb))
        lds_unite(par, l, qrl[u]);
      if (l + tw < n && vpar[l + tw] >= 0 && seg_edge_fast(rp[u], rd[u], c.sinAY, c.cosAY, c.theta, tb))
        lds_unite(par, l, l + tw);
    }
  }
  __syncthreads();
  for (int l = tid; l < n; l += blockDim.x) {
    const int row = l / tw, p = row * H + c0 + (l - row * tw);
    int pr = -1;
    if (vpar[l] >= 0) {
      const int r = lds_find(vpar, l), rrow = r / tw;
      pr = rrow * H + c0 + (r - rrow * tw);
    }
    bb.parent[base + p] = pr;
  }
}
// The seams between column tiles, one thread per (scan, seam, row): tile t's
// last column against the next column (tile t + 1's first; the last tile's
// against column 0, the wrap).
__global__ void k_ccl_seam(BatchBufs bb, DevCfg c, int TW, int nTiles) {
  const int b = blockIdx.y;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nTiles * c.N) return;
  const int t = i / c.N, row = i - t * c.N, H = c.H;
  const int ce = min(H, (t + 1) * TW);  // the first column past tile t
  const size_t base = (size_t)b * c.P;
  const int p = row * H + ce - 1, q = row * H + (ce == H ? 0 : ce);
  int* par = bb.parent + base;
  if (uf_load(&par[p]) < 0 || uf_load(&par[q]) < 0) return;
  const TanBand tb = seg_tan_band(c);
  if (seg_edge_fast(bb.range[base + p], bb.range[base + q], c.sinAX, c.cosAX, c.theta, tb)) uf_unite(par, p, q);
}

// Block-wide exclusive scan of up to 3 counters for 1024-thread blocks.
struct Scan3 {
  int v[3];
};
__device__ __forceinline__ Scan3 block_scan3(Scan3 in, Scan3* total, int* lds /*3*16+3*/) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  Scan3 out;
  for (int k = 0; k < 3; ++k) {
    // inclusive wave scan
    int x = in.v[k];
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    if (lane == 63) lds[k * 16 + wave] = x;
    out.v[k] = x - in.v[k];
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    int s = 0;
    for (int w = 0; w < nw; ++w) {
      const int t = lds[threadIdx.x * 16 + w];
      lds[threadIdx.x * 16 + w] = s;
      s += t;
    }
    lds[48 + threadIdx.x] = s;
  }
  __syncthreads();
  for (int k = 0; k < 3; ++k) {
    out.v[k] += lds[k * 16 + wave];
    total->v[k] = lds[48 + k];
  }
  __syncthreads();
  return out;
}

// Exclusive block prefix of three 0/1 flags (any block size up to 16 waves):
// ballots within a wave, the wave totals through LDS (one barrier).  The
// caller separates two calls with a barrier (lds is reused).
__device__ __forceinline__ Scan3 block_scan3_bits(bool f0, bool f1, bool f2, Scan3* total, int* lds /*48*/) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const unsigned long long lt = (1ull << lane) - 1;
  const unsigned long long m0 = __ballot(f0), m1 = __ballot(f1), m2 = __ballot(f2);
  if (lane == 0) {
    lds[wave] = (int)__popcll(m0);
    lds[16 + wave] = (int)__popcll(m1);
    lds[32 + wave] = (int)__popcll(m2);
  }
  __syncthreads();
  Scan3 out{{(int)__popcll(m0 & lt), (int)__popcll(m1 & lt), (int)__popcll(m2 & lt)}};
  Scan3 t{{0, 0, 0}};
  for (int w = 0; w < nw; ++w) {
    const int a = lds[w], b = lds[16 + w], c = lds[32 + w];
    if (w < wave) { out.v[0] += a; out.v[1] += b; out.v[2] += c; }
    t.v[0] += a; t.v[1] += b; t.v[2] += c;
  }
  *total = t;
  return out;
}

// cloudSegmentation's compaction (:318-367) after the HBM union-find, over
// the whole batch at once: one 1024-pixel chunk per workgroup.
//  k_seg_flags  each pixel's flags (kept in the segmented cloud, outlier,
//               valid root, valid, in a segment) into edges[] (free after the
//               unions), and the chunk's three counts into parent[] (free
//               after the roots: 3 ints per chunk at the scan's base);
//  k_seg_write  each chunk's exclusive prefixes (wave 0 sums the earlier
//               chunks' counts: a few hundred L2-resident words at most, in
//               place of a per-scan scan launch), the chunk's outputs at their
//               ordered positions, a valid root's label, negated, into root[]
//               at the root; the last chunk the scan's totals (seg_totals);
//  k_seg_labels (labels wanted) the final labelMat.
// The results equal the single-workgroup walk of round 1 and k_seg_lds.
enum { SF_KEEP = 1, SF_OUTL = 2, SF_VROOT = 4, SF_VALID = 8, SF_INSEG = 16 };

__device__ __forceinline__ void block_counts3(bool f0, bool f1, bool f2, int* lds /*48*/, int* out3) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const unsigned long long m0 = __ballot(f0), m1 = __ballot(f1), m2 = __ballot(f2);
  if (lane == 0) {
    lds[wave] = (int)__popcll(m0);
    lds[16 + wave] = (int)__popcll(m1);
    lds[32 + wave] = (int)__popcll(m2);
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    int t = 0;
    for (int w = 0; w < nw; ++w) t += lds[16 * threadIdx.x + w];
    out3[threadIdx.x] = t;
  }
}

__global__ void __launch_bounds__(1024) k_seg_flags(BatchBufs bb, DevCfg c) {
  __shared__ int lds[48];
  const int b = blockIdx.y, ch = blockIdx.x;
  const int p = ch * blockDim.x + threadIdx.x;
  const size_t base = (size_t)b * c.P;
  bool keep = false, outl = false, vroot = false, valid = false, inseg = false;
  if (p < c.P) {
    const int row = p / c.H, col = p - row * c.H;
    const int L0 = bb.label[base + p];
    if (L0 == 0) {
      inseg = true;
      const int r = bb.root[base + p];
      const int sz = bb.csize[base + r];
      const unsigned long long* rm = &bb.rowmask[(base + r) * 2];
      const int lines = __popcll(rm[0]) + __popcll(rm[1]);
      valid = sz >= 30 || (sz >= c.valid_pt && lines >= c.valid_line);  // :441-451
      vroot = valid && r == p;
      keep = valid;
      outl = !valid && row > c.g && col % 5 == 0;                      // :328-334
    } else if (bb.ground[base + p] == 1) {
      keep = !(col % 5 != 0 && col > 5 && col < c.H - 5);              // :337-340
    }
    bb.edges[base + p] = (uint8_t)((keep ? SF_KEEP : 0) | (outl ? SF_OUTL : 0) | (vroot ? SF_VROOT : 0) |
                                   (valid ? SF_VALID : 0) | (inseg ? SF_INSEG : 0));
  }
  block_counts3(keep, outl, vroot, lds, bb.parent + base + 3 * ch);
}

// The scan's totals (segmented / outlier counts, the last ring's end) and
// findStartEndAngle (:199-209); k_seg_write's last chunk.
__device__ void seg_totals(const BatchBufs& bb, const DevCfg& c, int b, int segc, int outc) {
  bb.ns[b] = segc;
  bb.nout[b] = outc;
  bb.eri[b * c.N + c.N - 1] = segc - 1 - 5;
  const float so = bb.rawang[2 * b];
  float eo = (float)((double)bb.rawang[2 * b + 1] + 2 * M_PI);
  if ((double)(eo - so) > 3 * M_PI) eo = (float)((double)eo - 2 * M_PI);
  else if ((double)(eo - so) < M_PI) eo = (float)((double)eo + 2 * M_PI);
  bb.orient[3 * b] = so;
  bb.orient[3 * b + 1] = eo;
  bb.orient[3 * b + 2] = eo - so;
}

__global__ void __launch_bounds__(1024) k_seg_write(BatchBufs bb, DevCfg c) {
  __shared__ int lds[64];
  __shared__ int off[3];  // the kept / outlier / valid-root pixels of the chunks before this one
  const int b = blockIdx.y, ch = blockIdx.x;
  const int p = ch * blockDim.x + threadIdx.x;
  const size_t base = (size_t)b * c.P;
  if (threadIdx.x < 64) {  // the earlier chunks' counts (k_seg_flags), summed by wave 0
    const int* cnt = bb.parent + base;
    int s0 = 0, s1 = 0, s2 = 0;
    for (int q = threadIdx.x; q < ch; q += 64) {
      s0 += cnt[3 * q];
      s1 += cnt[3 * q + 1];
      s2 += cnt[3 * q + 2];
    }
    for (int o = 32; o > 0; o >>= 1) {
      s0 += __shfl_xor(s0, o, 64);
      s1 += __shfl_xor(s1, o, 64);
      s2 += __shfl_xor(s2, o, 64);
    }
    if (threadIdx.x == 0) {
      off[0] = s0;
      off[1] = s1;
      off[2] = s2;
    }
  }
  const int f = p < c.P ? bb.edges[base + p] : 0;
  const bool keep = f & SF_KEEP, outl = f & SF_OUTL, vroot = f & SF_VROOT;
  Scan3 tot;
  const Scan3 ex = block_scan3_bits(keep, outl, vroot, &tot, lds);  // its barriers publish off[]
  if (threadIdx.x == 0 && ch == (int)gridDim.x - 1) seg_totals(bb, c, b, off[0] + tot.v[0], off[1] + tot.v[1]);
  if (p >= c.P) return;
  const int row = p / c.H, col = p - row * c.H;
  const int pos = off[0] + ex.v[0];  // kept pixels before p
  if (col == 0) {  // ring boundaries (:323, :354)
    bb.sri[b * c.N + row] = pos - 1 + 5;
    if (row > 0) bb.eri[b * c.N + row - 1] = pos - 1 - 5;
  }
  if (vroot) bb.root[base + p] = -(off[2] + ex.v[2] + 1);  // a valid root's label, negated
  if (keep) {
    bb.seg[base + pos] = bb.full[base + p];
    bb.gflag[base + pos] = (bb.ground[base + p] == 1) ? 1 : 0;
    bb.col[base + pos] = (uint32_t)col;
    bb.srange[base + pos] = bb.range[base + p];
  }
  if (outl) bb.outl[base + off[1] + ex.v[1]] = bb.full[base + p];
}

__global__ void k_seg_labels(BatchBufs bb, DevCfg c) {
  const int b = blockIdx.y;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= c.P) return;
  const size_t base = (size_t)b * c.P;
  const int f = bb.edges[base + p];
  if (!(f & SF_INSEG)) return;
  const int v = bb.root[base + p];  // -(label) at a valid root, else the root index
  bb.label[base + p] = v < 0 ? -v : ((f & SF_VALID) ? -bb.root[base + v] : 999999);  // the final labelMat
}

// The gated topics of publishCloud (imageProjection.cpp:480-506) for scan 0 of
// the batch, one 1024-pixel chunk per workgroup in row-major order:
// /full_cloud_info (the full cloud with intensity = range, :252-254), the
// ground cloud (groundMat == 1 in rows <= groundScanInd, :301-308) and the
// pure segmented cloud (labels > 0 and != 999999, intensity = label,
// :357-367).  Needs the final label image (want_labels).  k_gated_flags
// writes the info cloud and each chunk's two counts (into parent[], free
// after the segmentation), k_gated_scan their exclusive prefixes and the
// totals, k_gated_write both clouds at their ordered positions.
__device__ __forceinline__ void gated_flags(const BatchBufs& bb, const DevCfg& c, int p, bool& gnd, bool& pure) {
  gnd = pure = false;
  if (p < c.P) {
    const int L = bb.label[p];
    gnd = p / c.H <= c.g && bb.ground[p] == 1;
    pure = L > 0 && L != 999999;
  }
}

__global__ void __launch_bounds__(1024) k_gated_flags(BatchBufs bb, DevCfg c, GatedBufs gb) {
  __shared__ int lds[48];
  const int ch = blockIdx.x, p = ch * blockDim.x + threadIdx.x;
  if (p < c.P) {
    const float4 f = bb.full[p];
    const float r = bb.range[p];
    gb.info[p] = r == FLT_MAX ? f : make_float4(f.x, f.y, f.z, r);
  }
  bool gnd, pure;
  gated_flags(bb, c, p, gnd, pure);
  block_counts3(gnd, pure, false, lds, bb.parent + 3 * ch);
}

__global__ void __launch_bounds__(1024) k_gated_scan(BatchBufs bb, DevCfg c, GatedBufs gb) {
  __shared__ int lds[64];
  const int nCh = (c.P + 1023) / 1024;
  int* cnt = bb.parent;
  int run[2] = {0, 0};
  for (int c0 = 0; c0 < nCh; c0 += blockDim.x) {
    const int ch = c0 + threadIdx.x;
    Scan3 in{{0, 0, 0}}, tot;
    if (ch < nCh) in = Scan3{{cnt[3 * ch], cnt[3 * ch + 1], 0}};
    const Scan3 ex = block_scan3(in, &tot, lds);
    if (ch < nCh) {
      cnt[3 * ch] = run[0] + ex.v[0];
      cnt[3 * ch + 1] = run[1] + ex.v[1];
    }
    run[0] += tot.v[0];
    run[1] += tot.v[1];
  }
  if (threadIdx.x == 0) {
    gb.n[0] = run[0];
    gb.n[1] = run[1];
  }
}

__global__ void __launch_bounds__(1024) k_gated_write(BatchBufs bb, DevCfg c, GatedBufs gb) {
  __shared__ int lds[64];
  const int ch = blockIdx.x, p = ch * blockDim.x + threadIdx.x;
  bool gnd, pure;
  gated_flags(bb, c, p, gnd, pure);
  Scan3 tot;
  const Scan3 ex = block_scan3_bits(gnd, pure, false, &tot, lds);
  if (!gnd && !pure) return;
  const int* off = bb.parent + 3 * ch;
  const float4 f = bb.full[p];
  if (gnd) gb.ground[off[0] + ex.v[0]] = f;
  if (pure) gb.pure[off[1] + ex.v[1]] = make_float4(f.x, f.y, f.z, (float)bb.label[p]);
}

// ---------------------------------------------------------------------------
// Segmentation of one scan in LDS (labelComponents + the cloudSegmentation
// compaction, imageProjection.cpp:300-460), one 1024-thread workgroup per
// scan, for images of at most kSegLdsMaxP pixels and 16 rows (VLP-16 class):
// the union-find parents live in LDS instead of HBM, so the unions are LDS
// compare-and-swaps, and the per-component size and rows are LDS words
// instead of HBM atomics read back through two dependent gathers per pixel.
//
//  1. parent[p] = p for the unlabelled pixels (labelMat 0), -1 otherwise;
//  2. unions over the right (wrapping) and down neighbours whose angle test
//     passes (:397-427), linking the larger root under the smaller, so every
//     component's root is its smallest pixel index — the BFS seed;
//  3. each pixel's root (path-compressed) to HBM (root[], read back by
//     step 5 in pixel order);
//  4. per root one LDS word: the component's size (bits 0-14) and the rows of
//     its pushed (non-seed) pixels (bits 15-30, lineCountFlag :431);
//  5. the ordered compaction pass, the validity test (:441-451) on the root's
//     word; a valid root's word becomes -(its label) when its chunk is
//     scanned, which its later pixels read (the root precedes them).
// Results equal the HBM kernels' (k_ccl_* + k_seg_flags/_scan/_write) bit for bit.
constexpr int kSegLdsMaxP = 32767;  // counts fit 15 bits; 128 KB of parents
constexpr int kSegLdsMaxN = 16;     // the row mask fits 16 bits
constexpr int kSegK = (kSegLdsMaxP + 1023) / 1024;  // 1024-pixel chunks per scan
constexpr int kSegOutU = 2;                          // chunks per round of the output pass
constexpr int kSegHbmMaxScans = 8;  // launches of up to this many scans segment in HBM (launch_ip)
bool seg_lds_ok(const DevCfg& c) { return c.N <= kSegLdsMaxN && c.P <= kSegLdsMaxP && !c.segHbm; }


// p / H for a pixel index p < 2^15 (kSegLdsMaxP): the float product with
// the reciprocal is within 2^-8 of the quotient, so one correction makes it
// exact.  A few instructions where the integer division by the runtime width
// is a ~25-instruction sequence (five per pixel in seg_lds).
struct RowDiv {
  int H;
  float inv;
  __device__ __forceinline__ int row(int p) const {
    int r = (int)((float)p * inv);
    const int m = r * H;
    if (m > p) --r;
    else if (m + H <= p) ++r;
    return r;
  }
};

// Scan b's segmentation and compaction by the calling 1024-thread workgroup,
// par[P] its LDS parents; parReady: par already holds the initial parents
// (k_ip_lds writes them with the ground image), else they come from bb.label.
__device__ __forceinline__ void seg_lds(const BatchBufs& bb, const DevCfg& c, int b, int want_labels, int* par,
                                        bool parReady) {
  __shared__ int wpre[kSegK][3][16];    // per chunk and flag: the waves' exclusive prefixes
  __shared__ int cpre[kSegK + 1][3];    // per chunk and flag: the chunks' exclusive prefixes
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const size_t base = (size_t)b * c.P;
  const int P = c.P, H = c.H, K = (P + 1023) >> 10;
  const RowDiv rdiv{H, 1.0f / (float)H};
  volatile int* vpar = par;
  const TanBand tb = seg_tan_band(c);
  IP_T0();
  // pixel k * 1024 + tid of chunk k: loads coalesced, chunk-ordered
  if (!parReady) {
#pragma unroll
    for (int k = 0; k < kSegK; ++k) {
      const int p = (k << 10) + tid;
      if (k < K && p < P) par[p] = bb.label[base + p] == 0 ? p : -1;
    }
  }
  __syncthreads();
  IP_STAMP(3);  // (k_ip_lds: the ground walk and the parents)
  // unions over the right (wrapping) and down neighbours, four chunks' ranges in flight
  for (int k0 = 0; k0 < K; k0 += 4) {
    float rp[4], rr_[4], rd[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int p = ((k0 + u) << 10) + tid;
      rp[u] = rr_[u] = rd[u] = 0.f;
      if (k0 + u < K && p < P) {
        const int row = rdiv.row(p), col = p - row * H;
        rp[u] = bb.range[base + p];
        rr_[u] = bb.range[base + row * H + (col + 1 == H ? 0 : col + 1)];
        if (row + 1 < c.N) rd[u] = bb.range[base + p + H];
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int p = ((k0 + u) << 10) + tid;
      if (k0 + u >= K || p >= P || vpar[p] < 0) continue;  // candidates keep a parent >= 0 throughout
      const int row = rdiv.row(p), col = p - row * H;
      const int qr = row * H + (col + 1 == H ? 0 : col + 1);  // column wrap :403-406
      if (vpar[qr] >= 0 && seg_edge_fast(rp[u], rr_[u], c.sinAX, c.cosAX, c.theta, tb)) lds_unite(par, p, qr);
      if (row + 1 < c.N) {
        const int qd = p + H;
        if (vpar[qd] >= 0 && seg_edge_fast(rp[u], rd[u], c.sinAY, c.cosAY, c.theta, tb)) lds_unite(par, p, qd);
      }
    }
  }
  __syncthreads();
  IP_STAMP(4);
  int rt[kSegK];  // each pixel's root (-1: not a candidate), in registers
#pragma unroll
  for (int k = 0; k < kSegK; ++k) {
    const int p = (k << 10) + tid;
    // parReady: a non-candidate keeps its mark (-2: ground, ground_column)
    const int v = (k < K && p < P) ? vpar[p] : -1;
    rt[k] = v >= 0 ? lds_find(vpar, p) : (parReady ? v : -1);
  }
  __syncthreads();  // every find done before the parents become words
#pragma unroll
  for (int k = 0; k < kSegK; ++k) {
    const int p = (k << 10) + tid;
    if (k < K && p < P) par[p] = 0;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kSegK; ++k) {
    const int p = (k << 10) + tid;
    if (rt[k] < 0) continue;
    atomicAdd(&par[rt[k]], 1);
    if (rt[k] != p) atomicOr(&par[rt[k]], 1 << (15 + rdiv.row(p)));
  }
  __syncthreads();
  IP_STAMP(5);
  // flags per chunk: kept in the segmented cloud, outlier, valid root; the
  // waves' counts per chunk into wpre
  unsigned mkeep = 0, mout = 0, mroot = 0, mgnd = 0;  // mgnd: kept for being ground (the segmented cloud's ground flag)
#pragma unroll
  for (int k0 = 0; k0 < kSegK; k0 += 8) {
    int8_t G[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int p = ((k0 + u) << 10) + tid;
      if (parReady) G[u] = (k0 + u < K && rt[k0 + u] == -2) ? (int8_t)1 : (int8_t)0;  // no image read
      else G[u] = (k0 + u < K && p < P) ? bb.ground[base + p] : (int8_t)0;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int k = k0 + u, p = (k << 10) + tid;
      if (k >= K) break;
      bool keep = false, outl = false, vroot = false;
      if (p < P) {
        const int row = rdiv.row(p), col = p - row * H;
        if (rt[k] >= 0) {
          const int w = vpar[rt[k]];
          const int sz = w & 0x7fff;
          const int lines = __popc((unsigned)w >> 15);
          const bool valid = sz >= 30 || (sz >= c.valid_pt && lines >= c.valid_line);  // :441-451
          vroot = valid && rt[k] == p;
          keep = valid;
          outl = !valid && row > c.g && col % 5 == 0;                                // :328-334
        } else if (G[u] == 1) {
          keep = !(col % 5 != 0 && col > 5 && col < H - 5);                          // :337-340
          mgnd |= (keep ? 1u : 0u) << k;
        }
      }
      mkeep |= (keep ? 1u : 0u) << k;
      mout |= (outl ? 1u : 0u) << k;
      mroot |= (vroot ? 1u : 0u) << k;
      const unsigned long long b0 = __ballot(keep), b1 = __ballot(outl), b2 = __ballot(vroot);
      if (lane == 0) {
        wpre[k][0][wave] = (int)__popcll(b0);
        wpre[k][1][wave] = (int)__popcll(b1);
        wpre[k][2][wave] = (int)__popcll(b2);
      }
    }
  }
  __syncthreads();
  IP_STAMP(6);
  const int nw = blockDim.x >> 6;
  if (tid < 3 * K) {  // per (chunk, flag): the waves' exclusive prefix, the chunk's total
    const int k = tid / 3, f = tid - 3 * k;
    int run = 0;
    for (int w = 0; w < nw; ++w) {
      const int v = wpre[k][f][w];
      wpre[k][f][w] = run;
      run += v;
    }
    cpre[k][f] = run;
  }
  __syncthreads();
  if (tid < 3) {  // the chunks' exclusive prefix (cpre[K]: the totals)
    int run = 0;
    for (int k = 0; k <= K; ++k) {
      const int v = k < K ? cpre[k][tid] : 0;
      cpre[k][tid] = run;
      run += v;
    }
  }
  __syncthreads();
  IP_STAMP(7);
  // outputs at their ordered positions (cloudSegmentation :318-357)
  // kSegOutU chunks per round: their pixels' loads (full cloud, range) all in
  // flight before the round's stores; the ground flag from the flags pass
  const unsigned long long lt = (1ull << lane) - 1;
  for (int k0 = 0; k0 < K; k0 += kSegOutU) {
    int pos[kSegOutU], opos[kSegOutU];
    unsigned fl[kSegOutU];  // bit 0 keep, 1 outlier, 2 ground flag
    float4 fv[kSegOutU];
    float rv[kSegOutU];
#pragma unroll
    for (int u = 0; u < kSegOutU; ++u) {
      const int k = k0 + u, p = (k << 10) + tid;
      const bool in = k < K && p < P;
      const bool keep = in && ((mkeep >> k) & 1u), outl = in && ((mout >> k) & 1u), vroot = in && ((mroot >> k) & 1u);
      const unsigned long long b0 = __ballot(keep), b1 = __ballot(outl), b2 = __ballot(vroot);
      pos[u] = k < K ? cpre[k][0] + wpre[k][0][wave] + (int)__popcll(b0 & lt) : 0;  // kept pixels before p
      opos[u] = outl ? cpre[k][1] + wpre[k][1][wave] + (int)__popcll(b1 & lt) : 0;
      if (vroot) par[p] = -(cpre[k][2] + wpre[k][2][wave] + (int)__popcll(b2 & lt) + 1);  // its label, negated
      fl[u] = (keep ? 1u : 0u) | (outl ? 2u : 0u) | (in && ((mgnd >> k) & 1u) ? 4u : 0u);
      fv[u] = keep || outl ? bb.full[base + p] : make_float4(0.f, 0.f, 0.f, 0.f);
      rv[u] = keep ? bb.range[base + p] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < kSegOutU; ++u) {
      const int k = k0 + u, p = (k << 10) + tid;
      if (k >= K || p >= P) continue;
      const int row = rdiv.row(p), col = p - row * H;
      if (col == 0) {  // ring boundaries (:323, :354)
        bb.sri[b * c.N + row] = pos[u] - 1 + 5;
        if (row > 0) bb.eri[b * c.N + row - 1] = pos[u] - 1 - 5;
      }
      if (fl[u] & 1u) {
        bb.seg[base + pos[u]] = fv[u];
        bb.gflag[base + pos[u]] = (fl[u] & 4u) ? 1 : 0;
        bb.col[base + pos[u]] = (uint32_t)col;
        bb.srange[base + pos[u]] = rv[u];
      }
      if (fl[u] & 2u) bb.outl[base + opos[u]] = fv[u];
    }
  }
  if (want_labels) {  // the final labelMat: a valid segment's label, 999999 for the rest
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kSegK; ++k) {
      const int p = (k << 10) + tid;
      if (rt[k] >= 0) bb.label[base + p] = ((mkeep >> k) & 1u) ? -vpar[rt[k]] : 999999;
    }
  }
  if (tid == 0) {
    const int segc = cpre[K][0], outc = cpre[K][1];
    bb.ns[b] = segc;
    bb.nout[b] = outc;
    bb.eri[b * c.N + c.N - 1] = segc - 1 - 5;
    // findStartEndAngle :199-209
    const float so = bb.rawang[2 * b];
    float eo = (float)((double)bb.rawang[2 * b + 1] + 2 * M_PI);
    if ((double)(eo - so) > 3 * M_PI) eo = (float)((double)eo - 2 * M_PI);
    else if ((double)(eo - so) < M_PI) eo = (float)((double)eo + 2 * M_PI);
    bb.orient[3 * b] = so;
    bb.orient[3 * b + 1] = eo;
    bb.orient[3 * b + 2] = eo - so;
  }
  IP_STAMP(8);
}

__global__ void __launch_bounds__(1024) k_seg_lds(BatchBufs bb, DevCfg c, int want_labels) {
  extern __shared__ int par[];  // [P]
  seg_lds(bb, c, blockIdx.x, want_labels, par, false);
}

// The whole projection of a VLP-16-class scan (P <= kSegLdsMaxP) by one
// 1024-thread workgroup, for batches (the launch's other workgroups fill the
// device): the owner image in LDS (last writer wins by LDS atomicMax, :248),
// the range image and full cloud (:248-255), the ground walk of each column
// with the union-find's initial parents (:260-301), then k_seg_lds's
// segmentation and compaction over the same LDS (:312-367).  Replaces
// k_project + k_pixels + k_ground + k_seg_lds: no owner image in HBM, three
// launches fewer, and the later phases read what the earlier ones wrote from
// the CU's caches.
constexpr int kIpLdsU = 4;  // points per thread in flight (the projection)
constexpr int kIpPixU = 4;  // pixels per thread in flight (the range image and full cloud)
__global__ void __launch_bounds__(1024) k_ip_lds(BatchBufs bb, DevCfg c, int want_labels) {
  extern __shared__ int par[];  // [P]: the owner image, then the parents
  const int b = blockIdx.x, tid = threadIdx.x;
  const int P = c.P, H = c.H, n = scan_npts(bb, b);
  if (tid == 0) bb.bad[b] = 0;  // before the barrier: the projection may set kBadNotDense (ip_clears_bad)
  IP_T0();
  for (int p = tid; p < P; p += 1024) par[p] = -1;
  __syncthreads();
  IP_STAMP(0);
  for (int i0 = tid; i0 < n; i0 += kIpLdsU * 1024) {
    int pix[kIpLdsU];
#pragma unroll
    for (int u = 0; u < kIpLdsU; ++u) {
      const int i = i0 + u * 1024;
      pix[u] = i < n ? project_point(bb, c, b, n, i) : -1;
    }
#pragma unroll
    for (int u = 0; u < kIpLdsU; ++u)
      if (pix[u] >= 0) atomicMax(&par[pix[u]], i0 + u * 1024);
  }
  __syncthreads();
  IP_STAMP(1);
  // the pixels by (64-column block, row), a wave per pair: the waves of rows
  // 4q .. 4q + 3 at the same columns gather the owners from the same 128-B
  // lines of the firing-ordered input (k_pixels' mapping), instead of a wave
  // per 64 row-major pixels touching 64 lines for one record each
  // kIpPixU pairs per wave and round: their owners and gathers are all in
  // flight before the first store (one memory latency per round)
  {
    const int N = c.N, nq = N * ((H + 63) >> 6);
    const PtsView pv = pts_view(bb, b);
    const RowDiv ndiv{N, 1.0f / (float)N};
    for (int q0 = tid >> 6; q0 < nq; q0 += 16 * kIpPixU) {
      int o[kIpPixU], row[kIpPixU], col[kIpPixU];
      float4 xyz[kIpPixU];
#pragma unroll
      for (int u = 0; u < kIpPixU; ++u) {
        const int q = q0 + 16 * u;
        const int qb = ndiv.row(q);  // q / N
        row[u] = q - qb * N;
        col[u] = q < nq ? qb * 64 + (tid & 63) : H;
        o[u] = col[u] < H ? par[row[u] * H + col[u]] : -1;
        xyz[u] = o[u] >= 0 ? pv.xyz(o[u]) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int u = 0; u < kIpPixU; ++u)
        if (col[u] < H) pixel_store(bb, c, b, row[u], col[u], o[u], xyz[u]);
    }
  }
  __syncthreads();  // the pixels' stores are visible to the workgroup: the ground walk reads them
  IP_STAMP(2);
#if IP_PROF
  if (tid == 0) atomicAdd(&g_ipprof[11], 1ull);
#endif
  for (int j = tid; j < H; j += 1024) ground_column(bb, c, b, j, par, want_labels != 0);
  seg_lds(bb, c, b, want_labels, par, true);  // (its first barrier orders the parents)
}

#if IP_PROF
}  // namespace lego
extern "C" int lego_ip_profile(unsigned long long* out) {  // diagnostic build only: read and clear
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(lego::g_ipprof), sizeof(unsigned long long) * lego::kIpProf) != hipSuccess)
    return -1;
  static const unsigned long long zero[lego::kIpProf] = {};
  return hipMemcpyToSymbol(HIP_SYMBOL(lego::g_ipprof), zero, sizeof(zero)) == hipSuccess ? 0 : -1;
}
namespace lego {
#endif

void launch_gated(const BatchBufs& bb, const DevCfg& c, const GatedBufs& gb, hipStream_t s) {
  const int nCh = (c.P + 1023) / 1024;
  k_gated_flags<<<nCh, 1024, 0, s>>>(bb, c, gb);
  k_gated_scan<<<1, 1024, 0, s>>>(bb, c, gb);
  k_gated_write<<<nCh, 1024, 0, s>>>(bb, c, gb);
}

bool ip_clears_bad(const DevCfg& c, int B, const LaunchOpts& lo) {
  return seg_lds_ok(c) && B > kSegHbmMaxScans && lo.ipFused;
}

void launch_ip(const BatchBufs& bb, const DevCfg& c, int B, int want_labels, hipStream_t s,
               StageTimer* tm, const LaunchOpts& lo) {
  const int P = c.P;
  tm->mark("ip.memset", s);
  // launch-path errors are sticky: the caller checks hipGetLastError() after the batch
  // A launch of a few scans takes the HBM union-find: its grid-wide kernels
  // finish sooner than k_seg_lds's one workgroup per scan (a node call: ip
  // 0.20 -> 0.16 ms, profiles/r04_ab_node_seg.txt; the same labels, pinned by
  // test_seg_lds_equals_hbm_union_find)
  const bool segLds = seg_lds_ok(c) && B > kSegHbmMaxScans;
  if (ip_clears_bad(c, B, lo)) {  // one workgroup per scan, everything in its LDS
    tm->mark("ip.fused", s);
    k_ip_lds<<<B, 1024, (size_t)P * sizeof(int), s>>>(bb, c, want_labels);
    return;
  }
  // bb.owner is all -1 here: filled at creation, and k_pixels clears what k_project set
  tm->mark("ip.project", s);
  dim3 gpts((bb.Nmax + 255) / 256, B), gpix((P + 255) / 256, B), gcol((c.H + 255) / 256, B);
  k_project<<<gpts, 256, 0, s>>>(bb, c);
  tm->mark("ip.pixels", s);
  k_pixels<<<dim3((c.H + 63) / 64, (c.N + 3) / 4, B), 256, 0, s>>>(bb, c);
  tm->mark("ip.ground", s);
  k_ground<<<gcol, 256, 0, s>>>(bb, c);
  if (segLds) {
    tm->mark("ip.seg_lds", s);
    k_seg_lds<<<B, 1024, (size_t)P * sizeof(int), s>>>(bb, c, want_labels);
    return;
  }
  tm->mark("ip.ccl", s);
  // the union-find: in LDS column tiles plus the seams (lego_ctx_opts::ccl_tiles
  // = 0, diagnostic: every edge in HBM, k_ccl_init / k_ccl_union)
  if (lo.cclTiles) {
    const int TW = ccl_tile_width(c, B), nT = (c.H + TW - 1) / TW;
    k_ccl_tile<<<dim3(nT, B), 1024, (size_t)c.N * TW * sizeof(int), s>>>(bb, c, TW);
    if (nT > 1) k_ccl_seam<<<dim3((nT * c.N + 255) / 256, B), 256, 0, s>>>(bb, c, TW, nT);
  } else {
    k_ccl_init<<<gpix, 256, 0, s>>>(bb, c);
    k_ccl_union<<<gpix, 256, 0, s>>>(bb, c);
  }
  k_ccl_root<<<gpix, 256, 0, s>>>(bb, c);
  tm->mark("ip.compact", s);
  const dim3 gch((P + 1023) / 1024, B);
  k_seg_flags<<<gch, 1024, 0, s>>>(bb, c);
  k_seg_write<<<gch, 1024, 0, s>>>(bb, c);
  if (want_labels) k_seg_labels<<<gpix, 256, 0, s>>>(bb, c);
}

}  // namespace lego
