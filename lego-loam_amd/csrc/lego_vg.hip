// lego_vg.hip — pcl::VoxelGrid and the mapping NN index on gfx950, with the
// device-wide scan and sorts they need written here (no library sorts).
//
// VoxelGrid (voxel_grid.hpp applyFilter, PCL 1.7/1.8; called at
// mapOptmization.cpp:1058-1064 on the surrounding map, :1067-1091 on the
// scan's clouds, :1363 on the surrounding key poses and by the loop closure,
// :905-913):
//   k_vg_minmax        getMinMax3D over the finite points
//   k_vg_keys          the voxel index of every point (idx, point index)
//   k_vg_plan0         drops non-finite points (PCL skips them), sizes the sort
//   sort               std::sort of (idx, point) by idx — PCL's call, unstable;
//                      its order of equal keys is the summation order, so the
//                      permutation is reproduced exactly (lego_vgsort.h):
//     per round        k_vg_count / k_vg_decide / k_vg_swap partition every
//                      segment larger than kVgSplit across many workgroups
//                      (tiles of kVgTile keys), k_vg_plan turns the cuts into
//                      the next level's segments
//     k_vg_local_small / k_vg_local  each remaining segment in one workgroup's LDS
//   k_vg_head_tiles, k_scan_top, k_vg_emit
//                      voxel heads, their ranks, one lane per voxel summing its
//                      points in sorted order (PCL's centroid)
// NN index (replaces KdTreeFLANN on the map, :1335-1336): 1 m cells hashed
// into T buckets by a counting sort — histogram, scan, scatter.  The searches
// take exact (distance, index) minima, so the order inside a bucket is free.
#include <algorithm>
#include <cfloat>
#include <climits>
#include <cstdlib>

#include "lego_device.h"
#include "lego_kernels.h"
#include "lego_mo.h"
#include "lego_vgsort.h"
#include "lego_vgsort_wave.h"

namespace lego {

constexpr unsigned kInvalidKey = 0xffffffffu;
constexpr int kScanThreads = 256, kScanPer = 16, kScanTile = kScanThreads * kScanPer;
constexpr int kVgTileThreads = 256, kVgTilePer = 16, kVgTile = kVgTileThreads * kVgTilePer;
// The rounds split segments down to kVgSplit keys; those sort in small
// workgroups (many per CU, so the sorts' latency overlaps).  Segments the
// rounds leave larger (their last round, or rounds forced off) go to the big
// local kernel: LDS up to kVgLocal, a global-memory partition above.
constexpr int kVgSplit = 1024, kVgSplitThreads = 256;    // vg_sort_max(256) = 2048 >= kVgSplit
constexpr int kVgLocal = 8192, kVgLocalThreads = 1024;  // vg_sort_max(1024) = 8192 >= kVgLocal (98 KB of LDS)
constexpr int kVgRoundsMax = 16;
constexpr int kVgPlanThreads = 1024;

// VgScratch::ctl words
enum { C_M = 0, C_D = 1, C_NB = 2, C_NT = 3, C_NLOC = 4, C_NONFIN = 5, C_NOUT = 6, C_SLOW = 7, C_HEAP = 8, C_NLOCB = 9,
       C_ERR = 10 };

// The local list: segments of <= kVgSplit keys from the front of loc
// (k_vg_local_small's, C_NLOC), larger ones from its back (k_vg_local's,
// C_NLOCB), so that k_vg_local's workgroups take one large segment each
// instead of striding over the small ones (a workgroup that drew two large
// segments set the kernel's time).
__device__ __forceinline__ void vg_push_local(const VgScratch& v, int s, int e, int depth) {
  if (e - s > kVgSplit) v.loc[v.capLoc - 1 - atomicAdd(&v.ctl[C_NLOCB], 1)] = make_int4(s, e, depth, 0);
  else v.loc[atomicAdd(&v.ctl[C_NLOC], 1)] = make_int4(s, e, depth, 0);
}

// ---------------------------------------------------------------- block scans
// Exclusive scan of one int per thread over the block (<= 1024 threads);
// tmp: >= 17 ints of LDS.  Ends with the block in sync.
__device__ __forceinline__ int block_excl_scan(int v, int* tmp, int* total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) tmp[wave] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    int a = 0;
    for (int w = 0; w < nw; ++w) {
      const int t = tmp[w];
      tmp[w] = a;
      a += t;
    }
    tmp[16] = a;
  }
  __syncthreads();
  const int r = tmp[wave] + x - v;
  *total = tmp[16];
  __syncthreads();
  return r;
}
__device__ __forceinline__ int block_sum(int v, int* tmp) {
  int t;
  (void)block_excl_scan(v, tmp, &t);
  return t;
}
__device__ __forceinline__ int block_min(int v, int* tmp) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
  if (lane == 0) tmp[wave] = v;
  __syncthreads();
  int r = tmp[0];
  for (int w = 1; w < nw; ++w) r = min(r, tmp[w]);
  __syncthreads();
  return r;
}

// K sums (or, with MIN, minima) over the block at once: one barrier pair for
// all of them.  tmp: >= 16 K ints of LDS.  Ends with the block in sync.
template <int K, bool MIN = false>
__device__ __forceinline__ void block_reduce_k(int (&v)[K], int* tmp) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
  for (int k = 0; k < K; ++k)
    for (int o = 32; o > 0; o >>= 1) {
      const int y = __shfl_xor(v[k], o, 64);
      v[k] = MIN ? min(v[k], y) : v[k] + y;
    }
  if (lane == 0)
#pragma unroll
    for (int k = 0; k < K; ++k) tmp[k * 16 + wave] = v[k];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < K; ++k) {
    int a = tmp[k * 16];
    for (int w = 1; w < nw; ++w) a = MIN ? min(a, tmp[k * 16 + w]) : a + tmp[k * 16 + w];
    v[k] = a;
  }
  __syncthreads();
}

// Per-tile sums of in[0, n) (kScanTile elements per block).
__global__ void __launch_bounds__(kScanThreads) k_scan_tiles(const int* in, int n, int* tiles) {
  __shared__ int tmp[20];
  const int base = blockIdx.x * kScanTile + threadIdx.x * kScanPer;
  int s = 0;
#pragma unroll
  for (int j = 0; j < kScanPer; ++j) s += base + j < n ? in[base + j] : 0;
  const int t = block_sum(s, tmp);
  if (threadIdx.x == 0) tiles[blockIdx.x] = t;
}
// Exclusive scan of tiles[0, *ntp or nt) in place, one block; the total to *total.
__global__ void __launch_bounds__(1024) k_scan_top(int* tiles, int nt, const int* ntp, int* total) {
  __shared__ int tmp[20];
  const int n = ntp ? *ntp : nt;
  int carry = 0;
  for (int c = 0; c < n; c += blockDim.x) {
    const int i = c + threadIdx.x;
    const int v = i < n ? tiles[i] : 0;
    int t;
    const int e = block_excl_scan(v, tmp, &t);
    if (i < n) tiles[i] = carry + e;
    carry += t;
  }
  if (threadIdx.x == 0 && total) *total = carry;
}
static int grid_for(int n, int bs = 256) {
  int g = (n + bs - 1) / bs;
  return g < 1 ? 1 : (g > 4096 ? 4096 : g);
}
static int tiles_for(int n, int tile) { return n <= 0 ? 1 : (n + tile - 1) / tile; }

// ---------------------------------------------------------------- VoxelGrid
__device__ __forceinline__ int ord_of(float f) {  // order-preserving float -> int
  const int o = __float_as_int(f);
  return o >= 0 ? o : o ^ 0x7fffffff;
}
__device__ __forceinline__ float of_ord(int o) { return __int_as_float(o >= 0 ? o : o ^ 0x7fffffff); }
__device__ __forceinline__ bool finite3(float4 p) {
  return __builtin_isfinite(p.x) && __builtin_isfinite(p.y) && __builtin_isfinite(p.z);
}

__global__ void k_vg_init(VgScratch v) {
  if (threadIdx.x < 3) { v.mm[threadIdx.x] = INT_MAX; v.mm[3 + threadIdx.x] = INT_MIN; }
  if (threadIdx.x < 16) v.ctl[threadIdx.x] = 0;
  if (threadIdx.x == 0) *v.overflow = 0;
}

// n: element count (host bound); nDev: actual count on the device, or null
__global__ void k_vg_minmax(const float4* in, int n, const int* nDev, VgScratch v) {
  const int nn = nDev ? min(n, *nDev) : n;
  int mn[3] = {INT_MAX, INT_MAX, INT_MAX}, mx[3] = {INT_MIN, INT_MIN, INT_MIN};
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < nn; i += gridDim.x * blockDim.x) {
    const float4 p = in[i];
    if (!finite3(p)) continue;
    const int o[3] = {ord_of(p.x), ord_of(p.y), ord_of(p.z)};
#pragma unroll
    for (int k = 0; k < 3; ++k) { mn[k] = min(mn[k], o[k]); mx[k] = max(mx[k], o[k]); }
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    for (int off = 32; off > 0; off >>= 1) {
      mn[k] = min(mn[k], __shfl_xor(mn[k], off, 64));
      mx[k] = max(mx[k], __shfl_xor(mx[k], off, 64));
    }
  }
  // the block's waves through LDS, then one atomic per block and component
  __shared__ int red[6][16];
  const int wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if ((threadIdx.x & 63) == 0)
#pragma unroll
    for (int k = 0; k < 3; ++k) { red[k][wave] = mn[k]; red[3 + k][wave] = mx[k]; }
  __syncthreads();
  if (threadIdx.x < 6) {
    const int k = threadIdx.x;
    int r = red[k][0];
    for (int w = 1; w < nw; ++w) r = k < 3 ? min(r, red[k][w]) : max(r, red[k][w]);
    if (k < 3) atomicMin(&v.mm[k], r);
    else atomicMax(&v.mm[k], r);
  }
}

struct VgGeom {
  float inv;
  int minb[3], divb0, divb1;
  bool overflow;
};
// pcl::VoxelGrid::applyFilter: leaf_size -> inverse, integer-overflow guard,
// min/max voxel, division multipliers (float arithmetic as PCL's Eigen arrays).
__device__ __forceinline__ VgGeom vg_geom(const VgScratch& v, float leaf) {
  VgGeom g;
  g.inv = 1.0f / leaf;
  float minp[3], maxp[3];
  for (int k = 0; k < 3; ++k) { minp[k] = of_ord(v.mm[k]); maxp[k] = of_ord(v.mm[3 + k]); }
  const long long dx = (long long)((maxp[0] - minp[0]) * g.inv) + 1;
  const long long dy = (long long)((maxp[1] - minp[1]) * g.inv) + 1;
  const long long dz = (long long)((maxp[2] - minp[2]) * g.inv) + 1;
  g.overflow = dx * dy * dz > (long long)INT_MAX;
  int maxb[3];
  for (int k = 0; k < 3; ++k) {
    g.minb[k] = (int)floorf(minp[k] * g.inv);
    maxb[k] = (int)floorf(maxp[k] * g.inv);
  }
  g.divb0 = maxb[0] - g.minb[0] + 1;
  g.divb1 = maxb[1] - g.minb[1] + 1;
  return g;
}

// (idx, point index) in input order; a non-finite point gets kInvalidKey and
// is counted (k_vg_plan0 removes it, as PCL's index vector never holds it)
__global__ void k_vg_keys(const float4* in, int n, const int* nDev, float leaf, VgScratch v) {
  const int nn = nDev ? min(n, *nDev) : n;
  const VgGeom g = vg_geom(v, leaf);
  if (blockIdx.x == 0 && threadIdx.x == 0 && g.overflow) *v.overflow = 1;
  int bad = 0;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < nn; i += gridDim.x * blockDim.x) {
    unsigned key = kInvalidKey;
    const float4 p = in[i];
    if (finite3(p)) {
      const int i0 = (int)(floorf(p.x * g.inv) - (float)g.minb[0]);
      const int i1 = (int)(floorf(p.y * g.inv) - (float)g.minb[1]);
      const int i2 = (int)(floorf(p.z * g.inv) - (float)g.minb[2]);
      key = (unsigned)(i0 + i1 * g.divb0 + i2 * g.divb0 * g.divb1);
    } else {
      ++bad;
    }
    v.keys[i] = key;
    v.vals[i] = i;
  }
  for (int o = 32; o > 0; o >>= 1) bad += __shfl_xor(bad, o, 64);
  if ((threadIdx.x & 63) == 0 && bad) atomicAdd(&v.ctl[C_NONFIN], bad);
}

__device__ __forceinline__ int lg2i(int n) { return 31 - __builtin_clz((unsigned)n); }

// The new big segments' median-to-first (std::__move_median_to_first in
// global memory, one thread each), their cut / swap-count slots and tiles.
// nb segments in big[]; all threads of the block.
__device__ void vg_plan_big(const VgScratch& v, const int2* big, int nb, int* tmp) {
  int carry = 0;
  for (int c = 0; c < nb; c += blockDim.x) {
    const int b = c + threadIdx.x;
    int nt = 0;
    if (b < nb) {
      const int s = big[b].x, e = big[b].y;
      vg_median_to_first(v.keys, v.vals, s, s + 1, s + (e - s) / 2, e - 1);
      v.cut[b] = e;
      v.kcnt[b] = 0;
      nt = (e - s - 1 + kVgTile - 1) / kVgTile;
    }
    int t;
    const int off = block_excl_scan(nt, tmp, &t);
    if (b < nb) {
      v.tileOff[b] = carry + off;
      for (int k = 0; k < nt; ++k) v.tileSeg[carry + off + k] = b | (k << 16);  // no search per tile
    }
    carry += t;
  }
  if (threadIdx.x == 0) {
    v.tileOff[nb] = carry;
    v.ctl[C_NT] = carry;
    v.ctl[C_NB] = nb;
  }
}

// Removes non-finite points (stable), then the first level: the whole array as
// one big segment (partitioned by the rounds) or one local segment.
__global__ void __launch_bounds__(kVgPlanThreads) k_vg_plan0(int n, const int* nDev, VgScratch v, int rounds, int split) {
  __shared__ int tmp[20];
  const int nn = nDev ? min(n, *nDev) : n;
  int m = nn;
  if (v.ctl[C_NONFIN] > 0) {  // rare: a block-wide ordered compaction in place
    int w = 0;
    for (int c = 0; c < nn; c += blockDim.x) {
      const int i = c + threadIdx.x;
      const unsigned k = i < nn ? v.keys[i] : kInvalidKey;
      const int val = i < nn ? v.vals[i] : 0;
      const int f = k != kInvalidKey ? 1 : 0;
      int t;
      const int r = block_excl_scan(f, tmp, &t);
      if (f) { v.keys[w + r] = k; v.vals[w + r] = val; }
      w += t;
      __syncthreads();
    }
    m = w;
  }
  if (threadIdx.x == 0) {
    v.ctl[C_M] = m;
    v.ctl[C_D] = m > 1 ? 2 * lg2i(m) : 0;
    v.ctl[C_NLOC] = 0;
    v.ctl[C_NLOCB] = 0;
  }
  __syncthreads();
  if (*v.overflow || m <= 1) {
    if (threadIdx.x == 0) { v.ctl[C_NB] = 0; v.ctl[C_NT] = 0; v.tileOff[0] = 0; }
    return;
  }
  if (m <= split || rounds == 0) {  // one workgroup (above kVgLocal: its global-memory partition)
    if (threadIdx.x == 0) {
      vg_push_local(v, 0, m, 2 * lg2i(m));
      v.ctl[C_NB] = 0; v.ctl[C_NT] = 0; v.tileOff[0] = 0;
    }
    return;
  }
  if (threadIdx.x == 0) v.big[0] = make_int2(0, m);
  __syncthreads();
  vg_plan_big(v, v.big, 1, tmp);
}

// After round r - 1 (big list in big[(r-1)&1]): the cuts make the children;
// children larger than split form the next round's big list (unless flush),
// the others (and, when flushing, all) go to the local list with their depth
// budget 2 lg m - r.
__global__ void __launch_bounds__(kVgPlanThreads) k_vg_plan(VgScratch v, int r, int flush, int split) {
  __shared__ int tmp[20];
  const int nbp = v.ctl[C_NB];
  if (nbp == 0) return;  // uniform: nothing was partitioned
  const int2* prev = v.big + ((r - 1) & 1) * v.capBig;
  int2* next = v.big + (r & 1) * v.capBig;
  const int depth = v.ctl[C_D] - r;
  int carry = 0;
  for (int c = 0; c < nbp; c += blockDim.x) {
    const int b = c + threadIdx.x;
    int2 ch[2] = {make_int2(0, 0), make_int2(0, 0)};
    int nbig = 0;
    if (b < nbp) {
      const int s = prev[b].x, e = prev[b].y, cut = v.cut[b];
      ch[0] = make_int2(s, cut);
      ch[1] = make_int2(cut, e);
      for (int q = 0; q < 2; ++q) {
        const int sz = ch[q].y - ch[q].x;
        if (!flush && sz > split) {
          ++nbig;
        } else if (sz > 1) {
          vg_push_local(v, ch[q].x, ch[q].y, depth);
        }
      }
    }
    int t;
    int at = carry + block_excl_scan(nbig, tmp, &t);
    if (b < nbp)
      for (int q = 0; q < 2; ++q)
        if (!flush && ch[q].y - ch[q].x > split) next[at++] = ch[q];
    carry += t;
  }
  __syncthreads();  // the cut / kcnt slots are reused below
  vg_plan_big(v, next, carry, tmp);
}

// left / right stops of one tile
__global__ void __launch_bounds__(kVgTileThreads) k_vg_count(VgScratch v, int r) {
  __shared__ int tmp[32];
  const int nt = v.ctl[C_NT];
  if ((int)blockIdx.x >= nt) return;
  const int2* big = v.big + (r & 1) * v.capBig;
  const int ts = v.tileSeg[blockIdx.x], sg = ts & 0xffff;
  const int s = big[sg].x, e = big[sg].y;
  const int base = s + 1 + (ts >> 16) * kVgTile;
  const unsigned p = v.keys[s];
  int cl = 0, cr = 0;
#pragma unroll
  for (int j = 0; j < kVgTilePer; ++j) {
    const int i = base + j * kVgTileThreads + threadIdx.x;
    if (i < e) {
      const unsigned k = v.keys[i];
      cl += !(k < p);
      cr += !(p < k);
    }
  }
  int lr[2] = {cl, cr};
  block_reduce_k<2>(lr, tmp);
  if (threadIdx.x == 0) { v.tileL[blockIdx.x] = lr[0]; v.tileR[blockIdx.x] = lr[1]; }
}

// Ranks every stop of one tile by the stops after it (tiles to the right from
// their counts, the tile's own rows by ballots), scatters the swapped right
// stops into pr by rank and the swapped left stops into pl by their partner's
// rank, and folds the tile's cut candidates and swap count into the segment.
__global__ void __launch_bounds__(kVgTileThreads) k_vg_decide(VgScratch v, int r) {
  __shared__ int tmp[48];
  __shared__ int rowL[kVgTilePer][4], rowR[kVgTilePer][4];
  const int nt = v.ctl[C_NT];
  if ((int)blockIdx.x >= nt) return;
  const int2* big = v.big + (r & 1) * v.capBig;
  const int ts = v.tileSeg[blockIdx.x], sg = ts & 0xffff, kt = ts >> 16;
  const int s = big[sg].x, e = big[sg].y;
  const int t0 = (int)blockIdx.x - kt, t1 = t0 + (e - s - 1 + kVgTile - 1) / kVgTile;
  const int base = s + 1 + kt * kVgTile;
  const unsigned p = v.keys[s];
  unsigned kv[kVgTilePer];
#pragma unroll
  for (int j = 0; j < kVgTilePer; ++j) {  // the tile's keys in flight with the counts below
    const int i = base + j * kVgTileThreads + threadIdx.x;
    kv[j] = i < e ? v.keys[i] : 0u;
  }
  int abr[3] = {0, 0, 0};  // the segment's left stops; the left / right stops of the tiles after this one
  for (int q = t0 + threadIdx.x; q < t1; q += blockDim.x) {
    const int l = v.tileL[q];
    abr[0] += l;
    if (q > (int)blockIdx.x) { abr[1] += l; abr[2] += v.tileR[q]; }
  }
  block_reduce_k<3>(abr, tmp);
  const int totL = abr[0], LabT = abr[1], RabT = abr[2];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < kVgTilePer; ++j) {
    const int i = base + j * kVgTileThreads + threadIdx.x;
    const bool in = i < e;
    const unsigned long long ml = __ballot(in && !(kv[j] < p)), mr = __ballot(in && !(p < kv[j]));
    if (lane == 0) { rowL[j][wave] = (int)__popcll(ml); rowR[j][wave] = (int)__popcll(mr); }
  }
  __syncthreads();
  const unsigned long long above = lane == 63 ? 0ull : (~0ull << (lane + 1));
  int afterL = LabT, afterR = RabT;  // stops in the rows after row j
#pragma unroll
  for (int j = kVgTilePer - 1; j >= 0; --j) {
    int rl = 0, rr = 0, wl = 0, wr = 0;
    for (int w = 0; w < 4; ++w) {
      rl += rowL[j][w]; rr += rowR[j][w];
      if (w > wave) { wl += rowL[j][w]; wr += rowR[j][w]; }
    }
    const int i = base + j * kVgTileThreads + threadIdx.x;
    const bool in = i < e;
    const bool lf = in && !(kv[j] < p), rf = in && !(p < kv[j]);
    const unsigned long long ml = __ballot(lf), mr = __ballot(rf);
    const int Lab = afterL + wl + (int)__popcll(ml & above);
    const int Rab = afterR + wr + (int)__popcll(mr & above);
    const bool rsw = rf && totL - Lab - (lf ? 1 : 0) >= Rab + 1;
    const bool lsw = lf && Rab >= totL - Lab;
    if (rsw) v.pr[s + Rab] = i;
    if (lsw) v.pl[s + (totL - Lab) - 1] = i;
    kv[j] = ((lf && !lsw) || rsw) ? 1u : 0u;  // reuse: cut candidate
    afterL += rl;
    afterR += rr;
    if (lsw) kv[j] |= 2u;
  }
  int cmin = INT_MAX, nsw = 0;
#pragma unroll
  for (int j = 0; j < kVgTilePer; ++j) {
    const int i = base + j * kVgTileThreads + threadIdx.x;
    if ((kv[j] & 1u) && i < cmin) cmin = i;
    nsw += (kv[j] >> 1) & 1u;
  }
  int mn[1] = {cmin}, sw[1] = {nsw};
  block_reduce_k<1, true>(mn, tmp);
  block_reduce_k<1>(sw, tmp + 16);
  if (threadIdx.x == 0) {
    if (mn[0] != INT_MAX) atomicMin(&v.cut[sg], mn[0]);
    if (sw[0]) atomicAdd(&v.kcnt[sg], sw[0]);
  }
}

// the swaps: pair q = (pl[s + q], pr[s + q]) for q < the segment's count
__global__ void __launch_bounds__(kVgTileThreads) k_vg_swap(VgScratch v, int r) {
  const int nt = v.ctl[C_NT];
  if ((int)blockIdx.x >= nt) return;
  const int2* big = v.big + (r & 1) * v.capBig;
  const int ts = v.tileSeg[blockIdx.x], sg = ts & 0xffff;
  const int s = big[sg].x;
  const int K = v.kcnt[sg];
  const int q0 = (ts >> 16) * kVgTile;
  // every pair's partners, then every key / value, then the stores (the
  // swaps touch disjoint positions): two dependent load rounds per thread
  int a[kVgTilePer], b[kVgTilePer];
#pragma unroll
  for (int j = 0; j < kVgTilePer; ++j) {
    const int q = q0 + j * kVgTileThreads + threadIdx.x;
    a[j] = q < K ? v.pl[s + q] : -1;
    b[j] = q < K ? v.pr[s + q] : -1;
  }
  unsigned ka[kVgTilePer], kb[kVgTilePer];
  int va[kVgTilePer], vb[kVgTilePer];
#pragma unroll
  for (int j = 0; j < kVgTilePer; ++j)
    if (a[j] >= 0) { ka[j] = v.keys[a[j]]; va[j] = v.vals[a[j]]; kb[j] = v.keys[b[j]]; vb[j] = v.vals[b[j]]; }
#pragma unroll
  for (int j = 0; j < kVgTilePer; ++j)
    if (a[j] >= 0) { v.keys[a[j]] = kb[j]; v.vals[a[j]] = vb[j]; v.keys[b[j]] = ka[j]; v.vals[b[j]] = va[j]; }
}

// One workgroup partitions [s, e) in global memory (a segment still larger
// than kVgLocal after the rounds; rare): the same rules tile by tile from the
// right.  Returns the cut.
__device__ int vg_block_partition_global(const VgScratch& v, int s, int e, int* tmp, int* rows /*[2][8][16]*/) {
  if (threadIdx.x == 0) vg_median_to_first(v.keys, v.vals, s, s + 1, s + (e - s) / 2, e - 1);
  __syncthreads();
  const unsigned p = v.keys[s];
  int a = 0;
  for (int i = s + 1 + (int)threadIdx.x; i < e; i += blockDim.x) a += !(v.keys[i] < p);
  const int totL = block_sum(a, tmp);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const unsigned long long above = lane == 63 ? 0ull : (~0ull << (lane + 1));
  const int T = blockDim.x;
  int afterL = 0, afterR = 0, cmin = INT_MAX, nsw = 0;
  for (int c = ((e - s - 2) / T) * T; c >= 0; c -= T) {  // rows of T positions from the right
    const int i = s + 1 + c + (int)threadIdx.x;
    const bool in = i < e;
    const unsigned k = in ? v.keys[i] : 0u;
    const bool lf = in && !(k < p), rf = in && !(p < k);
    const unsigned long long ml = __ballot(lf), mr = __ballot(rf);
    if (lane == 0) { rows[wave] = (int)__popcll(ml); rows[16 + wave] = (int)__popcll(mr); }
    __syncthreads();
    int rl = 0, rr = 0, wl = 0, wr = 0;
    for (int w = 0; w < nw; ++w) {
      rl += rows[w]; rr += rows[16 + w];
      if (w > wave) { wl += rows[w]; wr += rows[16 + w]; }
    }
    const int Lab = afterL + wl + (int)__popcll(ml & above);
    const int Rab = afterR + wr + (int)__popcll(mr & above);
    const bool rsw = rf && totL - Lab - (lf ? 1 : 0) >= Rab + 1;
    const bool lsw = lf && Rab >= totL - Lab;
    if (rsw) v.pr[s + Rab] = i;
    if (lsw) { v.pl[s + (totL - Lab) - 1] = i; ++nsw; }
    if (((lf && !lsw) || rsw) && i < cmin) cmin = i;
    afterL += rl;
    afterR += rr;
    __syncthreads();
  }
  const int K = block_sum(nsw, tmp);
  const int cut = min(block_min(cmin, tmp), e);
  __threadfence_block();
  __syncthreads();
  for (int q = threadIdx.x; q < K; q += blockDim.x) vg_swap(v.keys, v.vals, v.pl[s + q], v.pr[s + q]);
  __threadfence_block();
  __syncthreads();
  return cut;
}

template <int CAP, int T>
__host__ __device__ inline size_t vg_local_lds_bytes() {
  return (size_t)CAP * 6 + vg_sort_scratch_bytes(CAP, T);
}

// [s, s + m), m <= kVgLocal, through LDS: keys and local positions sorted,
// then the keys and the gathered point indices written back.  lv: the
// element's position in the segment before the sort.
__device__ void vg_local_sort(const VgScratch& v, uint32_t* key, uint16_t* lv, unsigned char* sc, int s, int m,
                              int depth) {
  for (int i = threadIdx.x; i < m; i += blockDim.x) {
    key[i] = v.keys[s + i];
    lv[i] = (uint16_t)i;
  }
  __syncthreads();
  vg_block_sort(vg_sort_carve(key, lv, sc, m, (int)blockDim.x), m, depth, v.ctl + C_HEAP, true);
  for (int i = threadIdx.x; i < m; i += blockDim.x) {
    v.keys[s + i] = key[i];
    const int li = (int)lv[i];
    if (li >= m) atomicOr(v.err, 1);  // cannot come out of the sort (VgScratch::err): reported, never read
    key[i] = (uint32_t)v.vals[s + (li < m ? li : i)];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < m; i += blockDim.x) v.vals[s + i] = (int)key[i];
  __threadfence_block();
  __syncthreads();
}

// The local segments (grid-stride over the list) of up to kVgSplit keys:
// LDS sorts in small workgroups.
__global__ void __launch_bounds__(kVgSplitThreads) k_vg_local_small(VgScratch v) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
  uint32_t* key = (uint32_t*)lds_raw;
  uint16_t* lv = (uint16_t*)(lds_raw + (size_t)kVgSplit * 4);
  unsigned char* sc = lds_raw + (size_t)kVgSplit * 6;
  const int nloc = v.ctl[C_NLOC];
  for (int t = blockIdx.x; t < nloc; t += gridDim.x) {
    const int4 g = v.loc[t];
    vg_local_sort(v, key, lv, sc, g.x, g.y - g.x, g.z);
  }
}

// The larger local segments: LDS sort up to kVgLocal, above it the block
// partition in global memory, depth first with an LDS stack, its pieces
// sorted in LDS.
__global__ void __launch_bounds__(kVgLocalThreads) k_vg_local(VgScratch v) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
  __shared__ int tmp[20];
  __shared__ int rows[32];
  __shared__ int4 stk[64];
  __shared__ int sp;
  uint32_t* key = (uint32_t*)lds_raw;
  uint16_t* lv = (uint16_t*)(lds_raw + (size_t)kVgLocal * 4);
  unsigned char* sc = lds_raw + (size_t)kVgLocal * 6;
  const int nlocb = v.ctl[C_NLOCB];
  for (int t = blockIdx.x; t < nlocb; t += gridDim.x) {
    const int4 g = v.loc[v.capLoc - 1 - t];
    // one call site of the LDS sort (two inlined copies spilled registers);
    // every thread has read sp's last value before it is set again
    __syncthreads();
    if (threadIdx.x == 0) {
      stk[0] = g;
      sp = 1;
      if (g.y - g.x > kVgLocal) atomicAdd(&v.ctl[C_SLOW], 1);
    }
    __syncthreads();
    while (sp > 0) {
      const int4 c = stk[sp - 1];
      __syncthreads();
      if (threadIdx.x == 0) --sp;
      const int m = c.y - c.x;
      if (m <= kVgLocal) {
        vg_local_sort(v, key, lv, sc, c.x, m, c.z);
      } else if (c.z == 0) {  // depth budget spent: std::__partial_sort
        if (threadIdx.x == 0) { VgHeap<int>{v.keys, v.vals}.sort(c.x, c.y); atomicAdd(&v.ctl[C_HEAP], 1); }
        __threadfence_block();
        __syncthreads();
      } else {
        const int cut = vg_block_partition_global(v, c.x, c.y, tmp, rows);
        if (threadIdx.x == 0) {
          stk[sp++] = make_int4(cut, c.y, c.z - 1, 0);
          stk[sp++] = make_int4(c.x, cut, c.z - 1, 0);
        }
      }
      __syncthreads();
    }
  }
}

// voxel heads per tile of kHeadTile sorted positions (one position per thread)
constexpr int kHeadTile = 256;
__device__ __forceinline__ bool vg_head(const VgScratch& v, int t, int m) {
  return t < m && (t == 0 || v.keys[t] != v.keys[t - 1]);
}
__global__ void __launch_bounds__(kHeadTile) k_vg_head_tiles(VgScratch v) {
  const int m = v.ctl[C_M];
  const int t = blockIdx.x * kHeadTile + threadIdx.x;
  const unsigned long long b = __ballot(vg_head(v, t, m));
  __shared__ int w[kHeadTile / 64];
  if ((threadIdx.x & 63) == 0) w[threadIdx.x >> 6] = (int)__popcll(b);
  __syncthreads();
  if (threadIdx.x == 0) {
    int a = 0;
    for (int i = 0; i < kHeadTile / 64; ++i) a += w[i];
    v.scanTiles[blockIdx.x] = a;
  }
}

// One lane per voxel: the centroid of its points summed in sorted order
// (PCL's), written at the voxel's rank.  Overflow: copy.
__global__ void __launch_bounds__(kHeadTile) k_vg_emit(const float4* in, int n, const int* nDev, VgScratch v,
                                                       float4* out, int* nOut) {
  const int nn = nDev ? min(n, *nDev) : n;
  if (*v.overflow) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < nn; i += gridDim.x * blockDim.x) out[i] = in[i];
    if (blockIdx.x == 0 && threadIdx.x == 0) *nOut = nn;
    return;
  }
  const int m = v.ctl[C_M];
  if (blockIdx.x == 0 && threadIdx.x == 0) *nOut = v.ctl[C_NOUT];
  const int t = blockIdx.x * kHeadTile + threadIdx.x;
  const bool hd = vg_head(v, t, m);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const unsigned long long b = __ballot(hd);
  __shared__ int w[kHeadTile / 64];
  if (lane == 0) w[wave] = (int)__popcll(b);
  __syncthreads();
  if (!hd) return;
  int r = v.scanTiles[blockIdx.x] + (int)__popcll(b & ((1ull << lane) - 1));
  for (int i = 0; i < wave; ++i) r += w[i];
  const unsigned k = v.keys[t];
  float c0 = 0.f, c1 = 0.f, c2 = 0.f, c3 = 0.f;
  int u = t;
  for (; u < m && v.keys[u] == k; ++u) {
    const int vi = v.vals[u];
    if ((unsigned)vi >= (unsigned)nn) {  // see vg_local_sort: reported, never read
      atomicOr(v.err, 1);
      continue;
    }
    const float4 p = in[vi];
    c0 += p.x; c1 += p.y; c2 += p.z; c3 += p.w;
  }
  const float cnt = (float)(u - t);
  out[r] = make_float4(c0 / cnt, c1 / cnt, c2 / cnt, c3 / cnt);
}

// The partition rounds split a cloud's segments down to vg_split_for(n) keys.
// Small clouds (the scan's, <= kVgSmallCloud) stop at kVgLocal: their few
// rounds are launch-bound (four launches each for a few tiles), while a
// level of the LDS sort costs a fraction of a round; the map's clouds stop at
// kVgSplit, so that their thousand leftovers sort in many small workgroups.
constexpr int kVgSmallCloud = 65536;
int vg_split_for(int n) { return n <= kVgSmallCloud ? kVgLocal : kVgSplit; }
int vg_rounds_for(int n, int forced) {
  if (forced >= 0) return std::min(forced, kVgRoundsMax);
  const int split = vg_split_for(n);
  if (n <= split) return 0;
  int r = 1;
  while (((long long)split << r) < n) ++r;
  // margins for unbalanced partitions: two rounds for a small cloud (C5's
  // outlier cloud needs four where two halve it), one, plus one above 256 k
  // keys, for a map cloud (the C5 map's leftovers then fit one workgroup's
  // LDS instead of its global-memory partition)
  if (split == kVgLocal) return std::min(r + 2, kVgRoundsMax);
  return std::min(r + 1 + (n > (1 << 18) ? 1 : 0), kVgRoundsMax);
}

// in[0 .. min(n, *nDev)) -> out[0 .. *nOut), all on stream s.  n is a host
// upper bound (the capacity the scratch was sized for).
int voxel_grid_device(const float4* in, int n, const int* nDev, float leaf, float4* out, int* nOut,
                      const VgScratch& v, hipStream_t s) {
  if (n <= 0) {
    if (hipMemsetAsync(nOut, 0, sizeof(int), s) != hipSuccess) return -1;
    return 0;
  }
  if (n > v.cap) return -1;
  k_vg_init<<<1, 64, 0, s>>>(v);
  k_vg_minmax<<<std::min(grid_for(n), 512), 256, 0, s>>>(in, n, nDev, v);
  k_vg_keys<<<grid_for(n), 256, 0, s>>>(in, n, nDev, leaf, v);
  const int R = vg_rounds_for(n, v.rounds), split = vg_split_for(n);
  k_vg_plan0<<<1, kVgPlanThreads, 0, s>>>(n, nDev, v, R, split);
  // grids sized by this cloud's bound n, not the scratch's capacity: a round's
  // tiles <= n / kVgTile + its segments (each > split keys)
  const int gt = tiles_for(n, kVgTile) + std::min(v.capBig, n / split + 2);
  for (int r = 0; r < R; ++r) {
    k_vg_count<<<gt, kVgTileThreads, 0, s>>>(v, r);
    k_vg_decide<<<gt, kVgTileThreads, 0, s>>>(v, r);
    k_vg_swap<<<gt, kVgTileThreads, 0, s>>>(v, r);
    k_vg_plan<<<1, kVgPlanThreads, 0, s>>>(v, r + 1, r + 1 == R ? 1 : 0, split);
  }
  const int gl = n <= kVgSplit ? 1 : std::min({v.capLoc, 2048, std::max(64, n / 256)});  // grid-stride over the list
  k_vg_local_small<<<gl, kVgSplitThreads, vg_local_lds_bytes<kVgSplit, kVgSplitThreads>(), s>>>(v);
  if (n > kVgSplit)
    k_vg_local<<<std::min({v.capLoc, 256, n / kVgSplit + 1}), kVgLocalThreads, vg_local_lds_bytes<kVgLocal, kVgLocalThreads>(),
                 s>>>(v);
  const int ht = tiles_for(n, kHeadTile);
  k_vg_head_tiles<<<ht, kHeadTile, 0, s>>>(v);
  k_scan_top<<<1, 1024, 0, s>>>(v.scanTiles, ht, nullptr, v.ctl + C_NOUT);
  k_vg_emit<<<ht, kHeadTile, 0, s>>>(in, n, nDev, v, out, nOut);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int vg_read_ctl(const VgScratch& v, int* ctl16, hipStream_t s) {
  if (hipMemcpyAsync(ctl16, v.ctl, sizeof(int) * 16, hipMemcpyDeviceToHost, s) != hipSuccess) return -1;
  return hipStreamSynchronize(s) == hipSuccess ? 0 : -1;
}

int vg_scratch_alloc(VgScratch& v, int cap, void* ctx, int (*alloc)(void* ctx, void** p, size_t bytes)) {
  v.cap = cap;
  v.capBig = cap / kVgSplit + 2;
  v.capTiles = tiles_for(cap, kVgTile) + v.capBig + 1;
  v.capLoc = 2 * (kVgRoundsMax + 1) * v.capBig + 4;
  v.capScanTiles = std::max(tiles_for(2 * cap + 64, kScanTile), tiles_for(cap, kHeadTile)) + 1;
  struct A { void** p; size_t b; } as[] = {
      {(void**)&v.keys, sizeof(unsigned) * (size_t)cap}, {(void**)&v.vals, sizeof(int) * (size_t)cap},
      {(void**)&v.pl, sizeof(int) * (size_t)cap},        {(void**)&v.pr, sizeof(int) * (size_t)cap},
      {(void**)&v.big, sizeof(int2) * 2 * (size_t)v.capBig},
      {(void**)&v.cut, sizeof(int) * (size_t)v.capBig},  {(void**)&v.kcnt, sizeof(int) * (size_t)v.capBig},
      {(void**)&v.tileOff, sizeof(int) * (size_t)(v.capBig + 1)},
      {(void**)&v.tileSeg, sizeof(int) * (size_t)v.capTiles},
      {(void**)&v.tileL, sizeof(int) * (size_t)v.capTiles}, {(void**)&v.tileR, sizeof(int) * (size_t)v.capTiles},
      {(void**)&v.loc, sizeof(int4) * (size_t)v.capLoc},
      {(void**)&v.scanTiles, sizeof(int) * (size_t)v.capScanTiles},
      {(void**)&v.ctl, sizeof(int) * 16}, {(void**)&v.mm, sizeof(int) * 8}, {(void**)&v.overflow, sizeof(int) * 4},
  };
  for (auto& a : as)
    if (alloc(ctx, a.p, a.b)) return -1;
  v.err = v.ctl + C_ERR;
  return 0;
}

// ---------------------------------------------------------------- sort permutation
// libstdc++'s std::sort permutation of (key, index) pairs compared by key
// (the VoxelGrid's sort) for one array: wave = 0 the block sort (one
// 1024-thread workgroup, n <= kSortPermBlockMax), wave = 1 one wave's sort
// (n <= kVgWaveMax).  perm[i] = the index of the pair at sorted position i.
constexpr int kSortPermBlockMax = 8192;  // vg_sort_max(1024)
__global__ void __launch_bounds__(1024) k_sort_perm(const uint32_t* keys, int n, int wave, int* perm, int* heap) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
  uint32_t* key = (uint32_t*)lds_raw;
  uint16_t* val = (uint16_t*)(lds_raw + (size_t)4 * kSortPermBlockMax);
  unsigned char* sc = lds_raw + (size_t)6 * kSortPermBlockMax;
  if (wave == 1) {
    if (threadIdx.x >= 64) return;
    for (int i = threadIdx.x; i < n; i += 64) { key[i] = keys[i]; val[i] = (uint16_t)i; }
    vg_wave_sync();
    vg_wave_sort(key, val, (uint32_t*)sc, n, -1, heap);
    for (int i = threadIdx.x; i < n; i += 64) perm[i] = val[i];
    return;
  }
  for (int i = threadIdx.x; i < n; i += blockDim.x) { key[i] = keys[i]; val[i] = (uint16_t)i; }
  __syncthreads();
  vg_block_sort(vg_sort_carve(key, val, sc, n, (int)blockDim.x), n, -1, heap, wave >= 2);
  for (int i = threadIdx.x; i < n; i += blockDim.x) perm[i] = val[i];
}
// Either block form at either block size (modes 2, 4-8), compiled under the
// register budget of the kernel that runs it in the product: 256 threads with
// k_lf_voxel's LFV_MINB workgroups per CU (the 128-VGPR build that spills),
// 1024 threads with one.  REG: segment ids in registers (vg_block_sort) or in
// LDS (vg_block_sort_sid).  One instance per kernel, so that no form's
// registers weigh on another's.
template <int T, bool REG, bool SUM>
__global__ void __launch_bounds__(T, T == 256 ? LFV_MINB : 1) k_sort_perm_form(const uint32_t* keys, int n, int* perm,
                                                                            int* heap) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
  uint32_t* key = (uint32_t*)lds_raw;
  uint16_t* val = (uint16_t*)(lds_raw + (size_t)4 * kSortPermBlockMax);
  unsigned char* sc = lds_raw + (size_t)6 * kSortPermBlockMax;
  for (int i = threadIdx.x; i < n; i += blockDim.x) { key[i] = keys[i]; val[i] = (uint16_t)i; }
  __syncthreads();
  if (REG) vg_block_sort(vg_sort_carve(key, val, sc, n, (int)blockDim.x), n, -1, heap, SUM);
  else vg_block_sort_sid(vg_sort_carve(key, val, sc, n, (int)blockDim.x), n, -1, heap, SUM);
  for (int i = threadIdx.x; i < n; i += blockDim.x) perm[i] = val[i];
}
size_t sort_perm_lds_bytes() { return (size_t)6 * kSortPermBlockMax + vg_sort_scratch_bytes(kSortPermBlockMax, 1024); }
// Modes (lego_sort_permutation):
//   0 register form, 1024 threads, exact      3 register form, 1024, sumOrder
//   1 one wave (n <= kVgWaveMax)               2 LDS-id form, 256, sumOrder (k_lf_voxel's)
//   4 register form, 256, exact                5 register form, 256, sumOrder
//   6 LDS-id form, 256, exact                  7 LDS-id form, 1024, exact
//   8 LDS-id form, 1024, sumOrder
// 256-thread forms hold n <= vg_sort_max(256) = 2048, 1024-thread ones 8192.
int sort_perm_cap(int mode) {
  switch (mode) {
    case 1: return kVgWaveMax;
    case 2: case 4: case 5: case 6: return vg_sort_max(256);
    case 0: case 3: case 7: case 8: return kSortPermBlockMax;
    default: return -1;
  }
}
int sort_perm_device(const uint32_t* keys, int n, int mode, int* perm, int* heap, hipStream_t s) {
  const int cap = sort_perm_cap(mode);
  if (cap < 0 || n < 0 || n > cap) return -1;
  if (n == 0) return 0;
  const size_t lds = sort_perm_lds_bytes();
  switch (mode) {
    case 0: case 1: case 3: k_sort_perm<<<1, 1024, lds, s>>>(keys, n, mode, perm, heap); break;
    case 2: k_sort_perm_form<256, false, true><<<1, 256, lds, s>>>(keys, n, perm, heap); break;
    case 4: k_sort_perm_form<256, true, false><<<1, 256, lds, s>>>(keys, n, perm, heap); break;
    case 5: k_sort_perm_form<256, true, true><<<1, 256, lds, s>>>(keys, n, perm, heap); break;
    case 6: k_sort_perm_form<256, false, false><<<1, 256, lds, s>>>(keys, n, perm, heap); break;
    case 7: k_sort_perm_form<1024, false, false><<<1, 1024, lds, s>>>(keys, n, perm, heap); break;
    case 8: k_sort_perm_form<1024, false, true><<<1, 1024, lds, s>>>(keys, n, perm, heap); break;
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ---------------------------------------------------------------- NN index
__global__ void k_idx_count(const float4* pts, const int* nDev, int n, MoIndex ix) {
  const int nn = min(n, *nDev);
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < nn; i += gridDim.x * blockDim.x) {
    const float4 p = pts[i];
    const unsigned b = mo_cell_hash(cell1(p.x), cell1(p.y), cell1(p.z)) & (unsigned)(ix.T - 1);
    atomicAdd(&ix.end[b], 1);
  }
}
// begin = exclusive scan of the counts in end; end = begin (the scatter's cursor)
__global__ void __launch_bounds__(kScanThreads) k_idx_begin(MoIndex ix, const int* tiles) {
  __shared__ int tmp[20];
  const int n = ix.T;
  const int base = blockIdx.x * kScanTile + threadIdx.x * kScanPer;
  int c[kScanPer];
  int s = 0;
#pragma unroll
  for (int j = 0; j < kScanPer; ++j) {
    c[j] = base + j < n ? ix.end[base + j] : 0;
    s += c[j];
  }
  int t;
  int a = tiles[blockIdx.x] + block_excl_scan(s, tmp, &t);
#pragma unroll
  for (int j = 0; j < kScanPer; ++j) {
    if (base + j < n) { ix.begin[base + j] = a; ix.end[base + j] = a; }
    a += c[j];
  }
}
__global__ void k_idx_scatter(const float4* pts, const int* nDev, int n, MoIndex ix) {
  const int nn = min(n, *nDev);
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < nn; i += gridDim.x * blockDim.x) {
    const float4 p = pts[i];
    const unsigned b = mo_cell_hash(cell1(p.x), cell1(p.y), cell1(p.z)) & (unsigned)(ix.T - 1);
    const int at = atomicAdd(&ix.end[b], 1);
    ix.sorted[at] = make_float4(p.x, p.y, p.z, __int_as_float(i));
  }
}

int index_build_device(const float4* pts, int n, const int* nDev, MoIndex& ix, const VgScratch& v, hipStream_t s) {
  if (n > v.cap || n > ix.cap) return -1;
  int T = 64;
  while (T < n) T <<= 1;
  ix.T = T;
  if (hipMemsetAsync(ix.end, 0, sizeof(int) * T, s) != hipSuccess) return -1;
  if (n <= 0) return hipMemsetAsync(ix.begin, 0, sizeof(int) * T, s) == hipSuccess ? 0 : -1;
  const int nt = tiles_for(T, kScanTile);
  if (nt > v.capScanTiles) return -1;
  k_idx_count<<<grid_for(n), 256, 0, s>>>(pts, nDev, n, ix);
  k_scan_tiles<<<nt, kScanThreads, 0, s>>>(ix.end, T, v.scanTiles);
  k_scan_top<<<1, 1024, 0, s>>>(v.scanTiles, nt, nullptr, nullptr);
  k_idx_begin<<<nt, kScanThreads, 0, s>>>(ix, v.scanTiles);
  k_idx_scatter<<<grid_for(n), 256, 0, s>>>(pts, nDev, n, ix);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace lego
