// lego_vgsort.h — the permutation libstdc++'s std::sort gives an array of
// (key, payload) pairs compared by key only, computed in parallel.
//
// pcl::VoxelGrid::applyFilter (voxel_grid.hpp, PCL 1.7/1.8) std::sorts its
// (voxel idx, point index) vector by idx alone and then sums each voxel's
// points in that order.  The sort is unstable, so the in-voxel summation
// order — and with it the centroid's float rounding — is whatever libstdc++'s
// introsort leaves (featureAssociation.cpp:778-780; mapOptmization.cpp:
// 1058-1091).  The oracle runs the real std::sort (oracle/lego_oracle.cpp
// voxel_grid); lego_introsort.h is the serial port.  This file reproduces the
// same final order without running the serial algorithm:
//
//  * std::sort = __introsort_loop (GCC 11 stl_algo.h:1925-1957), then
//    __final_insertion_sort (:1861-1871).  Insertion sort is stable and the
//    introsort loop leaves the array partitioned into blocks of <= 16 (or
//    heap-sorted blocks) with every key of an earlier block <= every key of a
//    later one, so the final order is a stable sort of each block.
//  * Each partition (__unguarded_partition_pivot, :1911-1921) is Hoare's scheme
//    on [first+1, last) around the median of three moved to *first.  Let
//    "left stops" be the positions whose key is >= the pivot and "right stops"
//    those whose key is <= it (both from the array as it is before the
//    partition).  The k-th left stop L_k is swapped with the k-th right stop
//    from the right R_k exactly while L_k < R_k (a swapped position is never
//    revisited: its new value stops the other scan), and the returned cut is
//    min(L_{K+1}, R_K) with K the number of swaps (R_0 = last; L_{K+1} absent
//    counts as +inf) = the lowest position among the unswapped left stops and
//    the swapped right stops.  Both tests are prefix counts, so one wave
//    partitions a segment in two passes of ballots: a count of the left stops,
//    then a pass from the right that ranks both kinds, scatters the swapped
//    right stops' positions by rank and lets each swapped left stop fetch its
//    partner.
//  * Segments are disjoint, so their order of processing does not matter: the
//    recursion runs level by level (a segment's depth budget is the same
//    2*lg(n) - level for every segment of a level), the segments of a level
//    spread over the waves; a segment left with no budget is heap-sorted by one
//    lane exactly as std::__partial_sort(first, last, last) does.
//
// tests/native/vgsort_check.cpp checks the pairing/cut rules against std::sort
// on adversarial inputs; the GPU tests compare the per-ring less-flat clouds
// (and everything after them) with the oracle's std::sort VoxelGrid.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lego {

__device__ __forceinline__ void vg_wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <typename V>
__device__ __forceinline__ void vg_swap(uint32_t* key, V* val, int i, int j) {
  const uint32_t k = key[i];
  const V v = val[i];
  key[i] = key[j]; val[i] = val[j];
  key[j] = k; val[j] = v;
}

// std::__move_median_to_first(result, a, b, c) (stl_algo.h:79-97)
template <typename V>
__device__ __forceinline__ void vg_median_to_first(uint32_t* key, V* val, int r, int a, int b, int c) {
  const uint32_t ka = key[a], kb = key[b], kc = key[c];
  int m;
  if (ka < kb) {
    if (kb < kc) m = b;
    else if (ka < kc) m = c;
    else m = a;
  } else if (ka < kc) m = a;
  else if (kb < kc) m = c;
  else m = b;
  vg_swap(key, val, r, m);
}

// std::__partial_sort(first, last, last) = make_heap + sort_heap (stl_heap.h),
// one lane.
template <typename V>
struct VgHeap {
  uint32_t* key;
  V* val;
  __device__ void push_heap(int first, int hole, int top, uint32_t vk, V vv) const {
    int parent = (hole - 1) / 2;
    while (hole > top && key[first + parent] < vk) {
      key[first + hole] = key[first + parent];
      val[first + hole] = val[first + parent];
      hole = parent;
      parent = (hole - 1) / 2;
    }
    key[first + hole] = vk;
    val[first + hole] = vv;
  }
  __device__ void adjust_heap(int first, int hole, int len, uint32_t vk, V vv) const {
    const int top = hole;
    int second = hole;
    while (second < (len - 1) / 2) {
      second = 2 * (second + 1);
      if (key[first + second] < key[first + (second - 1)]) second--;
      key[first + hole] = key[first + second];
      val[first + hole] = val[first + second];
      hole = second;
    }
    if ((len & 1) == 0 && second == (len - 2) / 2) {
      second = 2 * (second + 1);
      key[first + hole] = key[first + (second - 1)];
      val[first + hole] = val[first + (second - 1)];
      hole = second - 1;
    }
    push_heap(first, hole, top, vk, vv);
  }
  __device__ void sort(int first, int last) const {
    const int len = last - first;
    if (len >= 2) {
      int parent = (len - 2) / 2;
      while (true) {
        adjust_heap(first, parent, len, key[first + parent], val[first + parent]);
        if (parent == 0) break;
        parent--;
      }
    }
    while (last - first > 1) {
      --last;
      const uint32_t vk = key[last];
      const V vv = val[last];
      key[last] = key[first];
      val[last] = val[first];
      adjust_heap(first, 0, last - first, vk, vv);
    }
  }
};

// One wave partitions [s, e) (e - s > 16) as std::__unguarded_partition_pivot
// and returns the cut.  pr[s .. e) is the wave's scratch for the partners.
template <typename V, typename P>
__device__ __forceinline__ int vg_wave_partition(uint32_t* key, V* val, P* pr, int s, int e) {
  const int lane = threadIdx.x & 63;
  if (lane == 0) vg_median_to_first(key, val, s, s + 1, s + (e - s) / 2, e - 1);
  vg_wave_sync();
  const uint32_t p = key[s];
  const int b = s + 1;
  const int nch = (e - b + 63) >> 6;
  int totL = 0;
  for (int k = 0; k < nch; ++k) {
    const int i = b + (k << 6) + lane;
    totL += (int)__popcll(__ballot(i < e && !(key[i] < p)));
  }
  const unsigned long long above = lane == 63 ? 0ull : (~0ull << (lane + 1));
  int cLa = 0, cR = 0, cut = e;
  for (int k = nch - 1; k >= 0; --k) {
    const int c0 = b + (k << 6);
    const int i = c0 + lane;
    const bool in = i < e;
    const uint32_t kv = in ? key[i] : 0u;
    const bool lf = in && !(kv < p), rf = in && !(p < kv);
    const unsigned long long ml = __ballot(lf), mr = __ballot(rf);
    const int Lab = cLa + (int)__popcll(ml & above);  // left stops after i
    const int Rab = cR + (int)__popcll(mr & above);   // right stops after i
    // right stop of rank Rab + 1 (from the right): swapped iff at least that
    // many left stops precede it; left stop of rank totL - Lab: swapped iff at
    // least that many right stops follow it
    const bool rsw = rf && totL - Lab - (lf ? 1 : 0) >= Rab + 1;
    const bool lsw = lf && Rab >= totL - Lab;
    if (rsw) pr[s + Rab] = (P)i;
    const unsigned long long mc = __ballot((lf && !lsw) || rsw);
    if (mc) cut = c0 + (int)__ffsll((long long)mc) - 1;
    vg_wave_sync();
    if (lsw) {
      const int j = (int)pr[s + (totL - Lab) - 1];
      const V vv = val[i];
      key[i] = key[j]; val[i] = val[j];
      key[j] = kv; val[j] = vv;
    }
    cR += (int)__popcll(mr);
    cLa += (int)__popcll(ml);
  }
  vg_wave_sync();
  return cut;
}

// Stable sort of up to two blocks of <= 16 (lanes 0-15: [s0, s0 + m0), lanes
// 16-31: [s1, s1 + m1); m = 0 for none), i.e. the final insertion sort's
// effect on them.
template <typename V>
__device__ __forceinline__ void vg_wave_leaf_sort(uint32_t* key, V* val, int s0, int m0, int s1, int m1) {
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4, l = lane & 15;
  const int s = g == 0 ? s0 : s1, m = g == 0 ? m0 : (g == 1 ? m1 : 0);
  const bool act = l < m;
  const uint32_t kv = act ? key[s + l] : 0u;
  const V vv = act ? val[s + l] : (V)0;
  int rank = 0;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const uint32_t kj = __shfl(kv, (lane & ~15) + j, 64);
    if (j < m) rank += (kj < kv || (kj == kv && j < l)) ? 1 : 0;
  }
  vg_wave_sync();
  if (act && m > 1) {
    key[s + rank] = kv;
    val[s + rank] = vv;
  }
  vg_wave_sync();
}

constexpr int kVgLeaf = 16;  // _S_threshold

__host__ __device__ inline int vg_list_cap(int n) { return n / (kVgLeaf + 1) + 1; }

// std::sort of key[0, n) / val[0, n) by key, all threads of the block; depth:
// the introsort loop's budget (2 lg n for a whole array, less for a segment
// of one; -1 = 2 lg n).  pr: n entries of scratch; lists: 2 * vg_list_cap(n)
// words; ctl: 3 ints.  n < 65536.  Ends with a block barrier.
template <typename V, typename P>
__device__ void vg_block_sort(uint32_t* key, V* val, P* pr, uint32_t* lists, int* ctl, int n, int depth = -1) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = blockDim.x >> 6;
  if (n <= kVgLeaf) {
    if (wave == 0 && n > 1) vg_wave_leaf_sort(key, val, 0, n, 0, 0);
    __syncthreads();
    return;
  }
  const int cap = vg_list_cap(n);
  const int D = depth >= 0 ? depth : 2 * (31 - __builtin_clz((unsigned)n));
  if (tid == 0) {
    lists[0] = (uint32_t)n << 16;  // [0, n)
    ctl[0] = 1; ctl[1] = 0; ctl[2] = 0;
  }
  __syncthreads();
  for (int r = 0;; ++r) {
    const int ncur = ctl[r % 3];
    if (ncur == 0) break;
    const uint32_t* cur = lists + (r & 1) * cap;
    uint32_t* nxt = lists + ((r + 1) & 1) * cap;
    if (tid == 0) ctl[(r + 2) % 3] = 0;  // read in round r - 1 (before its barrier), appended in round r + 1
    for (int t = wave; t < ncur; t += nw) {
      const uint32_t sg = cur[t];
      const int s = (int)(sg & 0xffffu), e = (int)(sg >> 16);
      if (D - r == 0) {  // depth budget spent: __partial_sort
        if (lane == 0) VgHeap<V>{key, val}.sort(s, e);
        vg_wave_sync();
        continue;
      }
      const int cut = vg_wave_partition(key, val, pr, s, e);
      const int m0 = cut - s, m1 = e - cut;
      if (lane == 0) {
        if (m0 > kVgLeaf) nxt[atomicAdd(&ctl[(r + 1) % 3], 1)] = (uint32_t)s | ((uint32_t)cut << 16);
        if (m1 > kVgLeaf) nxt[atomicAdd(&ctl[(r + 1) % 3], 1)] = (uint32_t)cut | ((uint32_t)e << 16);
      }
      vg_wave_leaf_sort(key, val, s, m0 > kVgLeaf ? 0 : m0, cut, m1 > kVgLeaf ? 0 : m1);
    }
    __syncthreads();
  }
}

}  // namespace lego
