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
//    spread over the waves; a segment left with no budget is heap-sorted by a
//    wave (vg_heap_sort_wave) exactly as std::__partial_sort(first, last,
//    last) does.
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

// The same std::__partial_sort(first, last, last) by one wave (all 64 lanes,
// first / last uniform; the piece synced to the wave before the call), with
// exactly VgHeap::sort's element moves:
//  * make_heap's __adjust_heap calls (parents (len-2)/2 down to 0) each touch
//    only the parent's subtree, so the parents of one heap level are
//    independent: levels deepest first, a lane per parent (VgHeap's own
//    adjust_heap), the order inside a level immaterial;
//  * a sort_heap pop moves the hole from the root down the larger child (the
//    right one unless right < left, __adjust_heap's rule; the single left
//    child at (len-2)/2 of an even heap) to where it stops, then __push_heap
//    moves the popped value up while its parent is < it.  The walk only reads
//    keys below the hole, all as they were before the pop, so it runs in
//    chunks of six levels: lane l < 63 holds the chunk root's descendant l
//    (heap order) and loads its two children, the chunk's choices are two
//    ballots and the walk is scalar bit tests.  The path's shifted keys are
//    the walked children's, so the push stops below the deepest path node
//    whose key is not < the value (one ballot), and the pop's stores (the
//    path shifted up to the stop, the value there) go out together.
// One LDS round trip per chunk and pop instead of two dependent ones per
// level (VLS-128's per-ring pieces of ~600 keys: the serial form took most of
// k_lf_voxel's 0.8 ms).
constexpr int kVgHeapWaveMax = 1 << 13;  // two chunks: internal levels < 12 (vg_sort_max(1024) keys)
template <typename V>
__device__ void vg_heap_sort_wave(uint32_t* key, V* val, int first, int last) {
  int lane = threadIdx.x & 63;
  asm volatile("" : "+v"(lane));  // the lane terms are computed here, not hoisted over the caller's loops
  const int len = last - first;
  if (len < 2) return;
  if (len > kVgHeapWaveMax) {
    if (lane == 0) VgHeap<V>{key, val}.sort(first, last);
    vg_wave_sync();
    return;
  }
  uint32_t* K = key + first;
  V* W = val + first;
  const VgHeap<V> Hp{K, W};
  const int lastP = (len - 2) / 2;
  for (int d = 31 - __builtin_clz((unsigned)lastP + 1); d >= 0; --d) {
    const int hi = min(lastP + 1, (2 << d) - 1);
    for (int p = (1 << d) - 1 + lane; p < hi; p += 64) Hp.adjust_heap(0, p, len, K[p], W[p]);
    vg_wave_sync();
  }
  // lane l < 63 of a chunk: its level dl and offset jl under the chunk's
  // root, the bits of its ancestors (anc) and of those whose right child
  // leads to it (ancR): the walk reaches l exactly when every ancestor moves
  // (G) and chose (R) that way, two mask tests instead of a serial walk
  const int dl = 31 - __builtin_clz((unsigned)lane + 1);
  const int jl = lane + 1 - (1 << dl);
  unsigned long long anc = 0ull, ancR = 0ull;
  for (int i = 0; i < dl; ++i) {
    const int a = ((lane + 1) >> (dl - i)) - 1;
    anc |= 1ull << a;
    if (((lane + 1) >> (dl - i - 1)) & 1) ancR |= 1ull << a;
  }
  constexpr int NC = 2;
  for (int m = len - 1; m >= 1; --m) {
    const int lim = (m - 1) / 2, tnode = (m & 1) == 0 ? (m - 2) / 2 : -1;
    uint32_t ck[NC], cv[NC];
    int px[NC];       // the lane's path index << 16 | its node (-1: not moved), its chosen child's key / payload
    int h = 0, k = 0; // the chunk's root, the path's steps so far
    bool more = true;
    uint32_t vk = 0u, vv = 0u, rk = 0u, rv = 0u;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      ck[c] = 0u; cv[c] = 0u; px[c] = -1;
      if (!more) continue;
      const int x = c == 0 ? lane : (h + 1) * (1 << dl) - 1 + jl;
      const bool two = lane < 63 && x < lim, one = lane < 63 && x == tnode;
      const int il = two || one ? 2 * x + 1 : 0, ir = two ? 2 * x + 2 : 0;
      if (c == 0) {  // the popped value and the root with the first chunk's children: one round trip
        vk = K[m]; vv = (uint32_t)W[m]; rk = K[0]; rv = (uint32_t)W[0];
      }
      const uint32_t kl = K[il], kr = K[ir], vl = (uint32_t)W[il], vr = (uint32_t)W[ir];
      const bool right = two && !(kr < kl);
      ck[c] = right ? kr : kl;
      cv[c] = right ? vr : vl;
      const unsigned long long G = __ballot(two || one), R = __ballot(right);
      const bool on = lane < 63 && (G & anc) == anc && (R & anc) == ancR;
      const unsigned long long P = __ballot(on);  // the walk's nodes in this chunk, one per level
      if (on && (two || one)) px[c] = ((k + dl) << 16) | x;
      k += (int)__popcll(P & G);
      const int last = 63 - __builtin_clzll(P);
      const int dL = 31 - __builtin_clz((unsigned)last + 1);
      const int xl = (h + 1) * (1 << dL) - 1 + (last + 1 - (1 << dL));
      more = ((G >> last) & 1ull) != 0;  // the chunk's last level moves on: the next chunk starts at its child
      h = more ? 2 * xl + 1 + (int)((R >> last) & 1ull) : xl;
    }
    vk = __builtin_amdgcn_readfirstlane(vk);
    vv = __builtin_amdgcn_readfirstlane(vv);
    // the push: the hole stops at path node j = 1 + the deepest path index
    // whose chosen child's key is not < the value (0 if none)
    int j = 0;
    bool found = false;
#pragma unroll
    for (int c = NC - 1; c >= 0; --c) {
      const unsigned long long F = __ballot(px[c] >= 0 && !(ck[c] < vk));
      if (!found && F) {
        j = (__builtin_amdgcn_readlane(px[c], 63 - __builtin_clzll(F)) >> 16) + 1;
        found = true;
      }
    }
    if (lane == 0) { K[m] = rk; W[m] = (V)rv; }  // outside the heap [0, m)
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int pi = px[c] >> 16, x = px[c] & 0xffff;
      if (px[c] >= 0 && pi < j) { K[x] = ck[c]; W[x] = (V)cv[c]; }
      if (px[c] >= 0 && pi == j) { K[x] = vk; W[x] = (V)vv; }
    }
    if (j == k && lane == 0) { K[h] = vk; W[h] = (V)vv; }
    vg_wave_sync();
  }
}

constexpr int kVgLeaf = 16;  // _S_threshold

// k_lf_voxel's 256-thread workgroups are built for LFV_MINB workgroups per CU
// (a 128-VGPR budget); the permutation tests compile their 256-thread sorts
// under the same bound (lego_vg.hip k_sort_perm_form).
#ifndef LFV_MINB
#define LFV_MINB 4
#endif

// bits 0..b of a word
__device__ __forceinline__ uint32_t bi_mask_le(int b) { return b == 31 ? ~0u : ((2u << b) - 1); }

// One segment of the current level: [s, e); A / B = left / right stops up to
// and including e - 1 (block-wide inclusive counts); ck = the left stops up
// to s (low half) | the swaps (high half: atomicMax of the swapped left
// stops' ranks), then the children's first table slot | which children are
// segments of the next level (bits 16, 17); cut (atomicMin).  16 B: two
// 8-byte loads.
struct alignas(16) VgSeg {
  uint16_t s, e, A, B;
  uint32_t ck, cut;
};

__host__ __device__ inline int vg_list_cap(int n) { return n / (kVgLeaf + 1) + 1; }
constexpr int kVgRowsMax = 8;  // rows of 64 positions per wave
// the largest sort a block of T threads handles
__host__ __device__ inline int vg_sort_max(int T) { return (T / 64) * 64 * kVgRowsMax; }

// The LDS a block sort of up to n keys uses besides key / val: segment id and
// partner per position, two segment tables, the leaf-start bits, counters.
template <typename V>
struct VgSortLds {
  uint32_t* key;   // [n]
  V* val;          // [n]
  uint16_t* sid;   // [n] the position's segment at this level, 0xffff in a leaf
  uint16_t* pr;    // [n] partners: right stops from a segment's start, left stops from its middle
  VgSeg* tab;      // [2 * vg_list_cap(n)]
  uint32_t* head;  // [(n + 31) / 32 + 1] leaf starts
  int* ctl;        // [2 + 2 * 16] segments of the current / next level, the waves' stop counts
};
__host__ __device__ inline size_t vg_sort_scratch_bytes(int n, int T) {
  (void)T;
  const size_t a = (4 * (size_t)n + 15) & ~(size_t)15;                    // sid, pr
  const size_t b = 2 * (size_t)vg_list_cap(n) * sizeof(VgSeg);            // tab
  const size_t c = (4 * (size_t)((n + 31) / 32 + 1) + 15) & ~(size_t)15;  // head
  return a + b + c + 4 * (2 + 2 * 16);
}
// carves the scratch (16-B aligned base) for a sort of up to n keys
template <typename V>
__device__ __forceinline__ VgSortLds<V> vg_sort_carve(uint32_t* key, V* val, unsigned char* base, int n, int T) {
  (void)T;
  VgSortLds<V> S;
  S.key = key;
  S.val = val;
  S.sid = (uint16_t*)base;
  S.pr = S.sid + n;
  unsigned char* p = base + ((4 * (size_t)n + 15) & ~(size_t)15);
  S.tab = (VgSeg*)p;
  p += 2 * (size_t)vg_list_cap(n) * sizeof(VgSeg);
  S.head = (uint32_t*)p;
  p += (4 * (size_t)((n + 31) / 32 + 1) + 15) & ~(size_t)15;
  S.ctl = (int*)p;
  return S;
}

#ifndef VG_STAMP
#define VG_STAMP(k)
#endif

// std::sort of key[0, n) / val[0, n) by key, all threads of the block.
// depth: the introsort loop's budget (2 lg n for a whole array, less for a
// segment of one; -1 = 2 lg n).  n <= vg_sort_max(blockDim.x), blockDim.x <=
// 1024; S carved for at least n.  heapStat: a counter bumped per heap-sorted
// piece, or null.  Ends with a block barrier.
//
// Level by level, every segment (> 16 keys) of the level at once.  Wave w
// owns the positions [w * P, (w + 1) * P) (P a multiple of 64, <= 8 rows of
// 64), so its running stop counts are wave-uniform; each pass gathers its
// rows' operands together (a few LDS round trips per pass, not per row) and
// skips rows with no position in a segment.  Passes: the median of three, one
// thread per segment; the stop flags and each wave's totals; the block-wide
// counts at each segment's ends; each stop's ranks from them and its own
// counts, the swapped right stops scattered by rank to the head of the
// segment's partner scratch and the swapped left stops to its middle, the
// cut's candidates and the swap count (one LDS atomic per segment run of a
// row); the pairs swapped; the children (> 16 keys) numbered; the positions'
// new segments.  Pieces of <= 16 keys become leaves; at the end every
// position ranks itself within its leaf (stably: the final insertion sort's
// effect) and moves there.
//
// sumOrder: the caller only sums each key's payloads in the sorted order (a
// VoxelGrid centroid, summed from 0).  A heap-sorted piece whose keys each
// occur at most twice in it, and whose smallest key, if twice, does not also
// end the pieces before it, then yields the same sums from a stable order: a
// key's one or two points in the piece are its voxel's first addends, and
// 0 + a + b == 0 + b + a (IEEE addition commutes).  Such a piece is ranked in
// parallel like a leaf instead of heap-sorted; any other piece is
// still heap-sorted exactly.  Off, the permutation itself is std::sort's
// (lego_sort_permutation).
constexpr int kVgMoveRows = 4;  // the moves' batch: rows of blockDim.x positions
// The end of both block sorts: every position ranks itself within its leaf,
// the sum-order heap pieces, the moves.  All threads of the block.
template <typename V>
__device__ void vg_block_finish(const VgSortLds<V>& S, int n, bool sumOrder) {
  int tid = threadIdx.x;
  asm volatile("" : "+v"(tid));  // nothing of this pass hoisted over the levels
  const int T = blockDim.x;
  // leaves: every position ranks itself within its leaf (its start the
  // highest leaf-start bit at or below it, its end the next one; <= 16 keys,
  // or a heap piece of up to T * kVgMoveRows with sumOrder)
  if (tid == 0) S.ctl[0] = 0;  // the heap pieces' count (read last at the final level's top: 0 or behind a barrier)
  for (int i = tid; i < n; i += T) {
    const int wi = i >> 5, bi = i & 31;
    const uint32_t hw = S.head[wi];
    const uint32_t msk = bi == 31 ? ~0u : ((2u << bi) - 1);
    uint32_t lo = hw & msk, hi = hw & ~msk;
    int wl = wi, wh = wi;
    while (!lo) lo = S.head[--wl];  // position 0 is always a leaf start
    while (!hi && ((wh + 1) << 5) < n) hi = S.head[++wh];
    const int ls = (wl << 5) + 31 - __builtin_clz(lo);
    const int le = hi ? min(n, (wh << 5) + __builtin_ctz(hi)) : n;
    if (le - ls > kVgLeaf && S.pr[ls] == 2) {  // heap-sorted below
      S.sid[i] = (uint16_t)i;
      continue;
    }
    const uint32_t k = S.key[i];
    int lt = 0, eqb = 0, eq = 0;
    for (int u0 = 0; u0 < le - ls; u0 += 8) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int q = ls + u0 + u;
        const uint32_t kq = S.key[min(q, n - 1)];
        if (q < le) {
          lt += kq < k ? 1 : 0;
          eqb += (kq == k && q < i) ? 1 : 0;
          eq += kq == k ? 1 : 0;
        }
      }
    }
    if (sumOrder && le - ls > kVgLeaf) {
      // a key 3+ times, or the piece's smallest key twice when the pieces
      // before it end with that key too (its sum then starts before the
      // piece and the two addends no longer come first): exact heap sort.
      // Every key before the piece is <= every key in it, so only the
      // preceding leaf can hold it.
      bool exact = eq >= 3;
      if (!exact && eq == 2 && lt == 0 && eqb == 0 && ls > 0) {
        int w = (ls - 1) >> 5;
        uint32_t m = S.head[w] & bi_mask_le((ls - 1) & 31);
        while (!m) m = S.head[--w];
        const int pls = (w << 5) + 31 - __builtin_clz(m);
        for (int q = pls; q < ls && !exact; ++q) exact = S.key[q] == k;
      }
      if (exact) S.pr[ls] = 1;
    }
    S.sid[i] = (uint16_t)(ls + lt + eqb);
  }
  __syncthreads();
  {  // the heap pieces (pr = 2, or 1: holding a key 3+ times), std::__partial_sort
    // listed (the segment tables are free now; ctl[0] zeroed in the leaf
    // pass), then a wave per piece; each position becomes a leaf
    int2* hl = (int2*)S.tab;
    for (int i = tid; i < n; i += T) {
      if (!((S.head[i >> 5] >> (i & 31)) & 1u)) continue;
      int w = i >> 5;
      uint32_t hi = S.head[w] & ~(bi_mask_le(i & 31));
      while (!hi && ((w + 1) << 5) < n) hi = S.head[++w];
      const int le = hi ? min(n, (w << 5) + __builtin_ctz(hi)) : n;
      if (le - i <= kVgLeaf || !S.pr[i]) continue;
      hl[atomicAdd(&S.ctl[0], 1)] = make_int2(i, le);
    }
    __syncthreads();
    const int nh = S.ctl[0];
    for (int q = tid >> 6; q < nh; q += T >> 6) {
      const int2 pc = hl[q];
      vg_heap_sort_wave(S.key, S.val, pc.x, pc.y);
      for (int i = pc.x + (tid & 63); i < pc.y; i += 64) {
        S.sid[i] = (uint16_t)i;
        atomicOr(&S.head[i >> 5], 1u << (i & 31));
      }
    }
    __syncthreads();
  }
  // the moves, in batches of whole leaves (a batch ends at the highest leaf
  // start within kVgMoveRows rows; every leaf fits in them): each batch's
  // keys / vals / places to registers, then to their places
  constexpr int MB = kVgMoveRows;
  for (int b = 0; b < n;) {
    int bn = b + T * MB;
    if (bn >= n) {
      bn = n;
    } else {
      int w = bn >> 5;
      const int wb = b >> 5;
      uint32_t m = S.head[w] & bi_mask_le(bn & 31);
      if (w == wb) m &= ~bi_mask_le(b & 31);
      while (!m) {
        m = S.head[--w];
        if (w == wb) m &= ~bi_mask_le(b & 31);
      }
      bn = (w << 5) + 31 - __builtin_clz(m);
    }
    uint32_t kk[MB], vd[MB];
#pragma unroll
    for (int j = 0; j < MB; ++j) {
      const int i = b + j * T + tid;
      const bool in = i < bn;
      kk[j] = in ? S.key[i] : 0u;
      vd[j] = in ? ((uint32_t)S.val[i] | ((uint32_t)S.sid[i] << 16)) : 0xffffffffu;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < MB; ++j)
      if (vd[j] != 0xffffffffu) { S.key[vd[j] >> 16] = kk[j]; S.val[vd[j] >> 16] = (V)(vd[j] & 0xffffu); }
    __syncthreads();
    b = bn;
  }
  VG_STAMP(8);
}

template <typename V>
__device__ void vg_block_sort(const VgSortLds<V>& S, int n, int depth = -1, int* heapStat = nullptr,
                              bool sumOrder = false) {
  constexpr int RM = kVgRowsMax;
  int tid = threadIdx.x;
  asm volatile("" : "+v"(tid));  // the lane terms computed per call, not held across the caller's loops
  const int T = blockDim.x, lane = tid & 63, wave = tid >> 6, nw = T >> 6;
  const int cap = vg_list_cap(n);
  const int D = depth >= 0 ? depth : (n > 1 ? 2 * (31 - __builtin_clz((unsigned)n)) : 0);
  const int P = (((n + nw - 1) / nw) + 63) & ~63;  // positions per wave
  const int w0 = wave * P;
  const unsigned long long below = (1ull << lane) - 1;
  int* wt = S.ctl + 2;  // [nw][2] the waves' stop totals
  if (n <= 1) {
    __syncthreads();
    return;
  }
  for (int w = tid; w < (n + 31) / 32 + 1; w += T) S.head[w] = (w == 0 && n <= kVgLeaf) ? 1u : 0u;
  if (tid == 0) {
    S.ctl[0] = n > kVgLeaf ? 1 : 0;
    S.tab[0] = VgSeg{0, (uint16_t)n, 0, 0, 0u, (uint32_t)n};
    if (n > kVgLeaf && D > 0) vg_median_to_first(S.key, S.val, 0, 1, n / 2, n - 1);
  }
  // Per row j of this wave's positions, in registers for the whole loop: the
  // position's segment at this level (table index SD(j), 0xffff in a leaf;
  // two rows per word) and its bounds se[j] = s | e << 16.  Positions never
  // change threads.
  uint32_t rowact = 0;  // rows of this wave holding positions of a segment (wave-uniform)
  uint32_t sdp[RM / 2], se[RM];
#define SD(j) ((sdp[(j) >> 1] >> (((j) & 1) * 16)) & 0xffffu)
#define SD_SET(j, x) (sdp[(j) >> 1] = (sdp[(j) >> 1] & (0xffff0000u >> (((j) & 1) * 16))) | ((uint32_t)(x) << (((j) & 1) * 16)))
#pragma unroll
  for (int j = 0; j < RM; ++j) {
    const bool a = n > kVgLeaf && (j << 6) < P && w0 + (j << 6) + lane < n;
    if ((j & 1) == 0) sdp[j >> 1] = 0xffffffffu;
    SD_SET(j, a ? 0u : 0xffffu);
    se[j] = (uint32_t)n << 16;
    if (n > kVgLeaf && w0 + (j << 6) < n && (j << 6) < P) rowact |= 1u << j;
  }
  __syncthreads();
  constexpr int BR = 4;  // rows whose operands are gathered together (registers)
  // Five barriers per level: the stop flags and the waves' totals | the
  // counts at the segments' ends | ranks, pairing, partners, cut | the swaps
  // and the children | the positions' new segments and the children's
  // medians of three (std::__move_median_to_first, before the next level's
  // flags; not when the next level's depth budget is spent).
  for (int r = 0;; ++r) {
    const int nseg = S.ctl[r & 1];
    if (nseg == 0) break;
    VgSeg* cur = S.tab + (r & 1) * cap;
    VgSeg* nxt = S.tab + ((r + 1) & 1) * cap;
    if (D - r == 0) {  // depth budget spent: std::__partial_sort of every piece
      // pieces of > 16 keys, heap-sorted in vg_block_finish (pr[s] = 2),
      // or with sumOrder a leaf unless a key occurs 3+ times (pr[s] = 0, set
      // to 1 there if so)
      for (int j = tid; j < nseg; j += T) {
        const int s = cur[j].s, e = cur[j].e;
        atomicOr(&S.head[s >> 5], 1u << (s & 31));
        S.pr[s] = sumOrder && e - s <= T * kVgMoveRows ? 0 : 2;
        if (heapStat) atomicAdd(heapStat, 1);
      }
      __syncthreads();
      break;
    }
    if (tid == 0) S.ctl[(r + 1) & 1] = 0;  // last read at level r - 1's top; counted into below
    VG_STAMP(0);
    // stop flags (a bit per row) and the wave's totals
    uint32_t fl = 0, fr = 0;
    int totLw = 0, totRw = 0;
    for (int j0 = 0; j0 < RM; j0 += BR) {
      if (!((rowact >> j0) & ((1u << BR) - 1))) continue;
      uint32_t kp[BR], ki[BR];
#pragma unroll
      for (int u = 0; u < BR; ++u) {
        const int j = j0 + u, i = w0 + (j << 6) + lane, s = (int)(se[j] & 0xffffu);
        const bool in = SD(j) != 0xffffu && i > s;
        kp[u] = in ? S.key[s] : 0u;
        ki[u] = in ? S.key[i] : 0u;
      }
#pragma unroll
      for (int u = 0; u < BR; ++u) {
        const int j = j0 + u, i = w0 + (j << 6) + lane, s = (int)(se[j] & 0xffffu);
        const bool in = SD(j) != 0xffffu && i > s;
        const bool lf = in && !(ki[u] < kp[u]), rf = in && !(kp[u] < ki[u]);
        fl |= (lf ? 1u : 0u) << j;
        fr |= (rf ? 1u : 0u) << j;
        totLw += (int)__popcll(__ballot(lf));
        totRw += (int)__popcll(__ballot(rf));
      }
    }
    if (lane == 0) { wt[2 * wave] = totLw; wt[2 * wave + 1] = totRw; }
    __syncthreads();
    VG_STAMP(1);
    int baseL = 0, baseR = 0;
    for (int w = 0; w < wave; ++w) { baseL += wt[2 * w]; baseR += wt[2 * w + 1]; }
    {  // the block-wide inclusive counts at every segment's start and last position
      int aL = baseL, aR = baseR;
#pragma unroll
      for (int j = 0; j < RM; ++j) {
        const bool lf = (fl >> j) & 1u, rf = (fr >> j) & 1u;
        const unsigned long long ml = __ballot(lf), mr = __ballot(rf);
        const int SL = aL + (int)__popcll(ml & below) + (lf ? 1 : 0);
        const int SR = aR + (int)__popcll(mr & below) + (rf ? 1 : 0);
        aL += (int)__popcll(ml);
        aR += (int)__popcll(mr);
        const uint32_t id = SD(j);
        if (id == 0xffffu) continue;
        const int i = w0 + (j << 6) + lane, s = (int)(se[j] & 0xffffu), e = (int)(se[j] >> 16);
        if (i == s) *(uint16_t*)&cur[id].ck = (uint16_t)SL;
        if (i == e - 1) { cur[id].A = (uint16_t)SL; cur[id].B = (uint16_t)SR; }
      }
    }
    __syncthreads();
    VG_STAMP(2);
    {  // ranks, the pairing rule, partners, the cut's candidates, the swap count
      int aL = baseL, aR = baseR;
      for (int j0 = 0; j0 < RM; j0 += BR) {
        int SL[BR], SR[BR];
#pragma unroll
        for (int u = 0; u < BR; ++u) {
          const int j = j0 + u;
          const bool lf = (fl >> j) & 1u, rf = (fr >> j) & 1u;
          const unsigned long long ml = __ballot(lf), mr = __ballot(rf);
          SL[u] = aL + (int)__popcll(ml & below) + (lf ? 1 : 0);
          SR[u] = aR + (int)__popcll(mr & below) + (rf ? 1 : 0);
          aL += (int)__popcll(ml);
          aR += (int)__popcll(mr);
        }
        if (!((rowact >> j0) & ((1u << BR) - 1))) continue;
        uint2 g[BR];  // A | B << 16, ck
#pragma unroll
        for (int u = 0; u < BR; ++u) {
          const int j = j0 + u;
          g[u] = make_uint2(0u, 0u);
          if (((fl | fr) >> j) & 1u) {
            const uint32_t* c = (const uint32_t*)&cur[SD(j)];
            g[u] = make_uint2(c[1], c[2]);
          }
        }
#pragma unroll
        for (int u = 0; u < BR; ++u) {
          const int j = j0 + u;
          if (!((rowact >> j) & 1u)) continue;
          const bool lf = (fl >> j) & 1u, rf = (fr >> j) & 1u;
          const int i = w0 + (j << 6) + lane;
          const int s = (int)(se[j] & 0xffffu), e = (int)(se[j] >> 16);
          const int A = (int)(g[u].x & 0xffffu), B = (int)(g[u].x >> 16), Cc = (int)(g[u].y & 0xffffu);
          const int totL = A - Cc, Lab = A - SL[u], Rab = B - SR[u];  // left stops, stops after i
          // right stop of rank Rab + 1 (from the right): swapped iff at least
          // that many left stops precede it; left stop of rank totL - Lab:
          // swapped iff at least that many right stops follow it
          const bool rsw = rf && totL - Lab - (lf ? 1 : 0) >= Rab + 1;
          const bool lsw = lf && Rab >= totL - Lab;
          if (rsw) S.pr[s + Rab] = (uint16_t)i;
          if (lsw) S.pr[s + ((e - s + 1) >> 1) + (totL - Lab) - 1] = (uint16_t)i;
          const bool cand = (lf && !lsw) || rsw;
          // one atomic per segment run of the row: its lowest candidate, its
          // highest swapped left stop (ranks grow with the position)
          const unsigned long long mc = __ballot(cand), mw = __ballot(lsw);
          const int rb = i - lane;
          if (cand && !(mc & below & ~((1ull << max(0, s - rb)) - 1))) atomicMin(&cur[SD(j)].cut, (uint32_t)i);
          if (lsw) {
            const int hiL = min(64, e - rb);
            const unsigned long long abv = (hiL >= 64 ? ~0ull : ((1ull << hiL) - 1)) & ~below & ~(1ull << lane);
            if (!(mw & abv)) atomicMax(&cur[SD(j)].ck, (uint32_t)Cc | ((uint32_t)(totL - Lab) << 16));
          }
        }
      }
    }
    __syncthreads();
    VG_STAMP(3);
    for (int j0 = 0; j0 < RM; j0 += BR) {  // pair q of a segment, at the position s + q (its
      // partners read beside the swap count, used when q is below it)
      if (!((rowact >> j0) & ((1u << BR) - 1))) continue;
      int pa[BR], pb[BR];
      uint32_t K[BR];
#pragma unroll
      for (int u = 0; u < BR; ++u) {
        const int j = j0 + u;
        K[u] = 0u;
        pa[u] = pb[u] = 0;
        const uint32_t id = SD(j);
        if (id == 0xffffu) continue;
        const int x = w0 + (j << 6) + lane, s = (int)(se[j] & 0xffffu), e = (int)(se[j] >> 16), q = x - s;
        const int half = (e - s + 1) >> 1;
        if (q < half) {
          K[u] = cur[id].ck >> 16;
          pa[u] = (int)S.pr[s + half + q];
          pb[u] = (int)S.pr[x];
        }
      }
#pragma unroll
      for (int u = 0; u < BR; ++u) {
        const int j = j0 + u, x = w0 + (j << 6) + lane, s = (int)(se[j] & 0xffffu);
        if ((uint32_t)(x - s) < K[u]) vg_swap(S.key, S.val, pa[u], pb[u]);
      }
    }
    // the children: > 16 keys to the next level's table (its cut = its end
    // until the partition), else a leaf start; cur[j].A | B (free since the
    // ranks) takes the children's first slot | which are segments.  nseg <=
    // vg_list_cap(n) < T: a thread per segment.
    uint32_t cse0 = 0u, cse1 = 0u;  // this thread's segment's children (s | e << 16), 0: none / a leaf
    if (tid < nseg) {
      const uint4 g = *(const uint4*)&cur[tid];
      const int s = (int)(g.x & 0xffffu), e = (int)(g.x >> 16), cut = (int)g.w;
      const int aL = cut - s > kVgLeaf ? 1 : 0, aR = e - cut > kVgLeaf ? 1 : 0;
      const int base = (aL + aR) ? atomicAdd(&S.ctl[(r + 1) & 1], aL + aR) : 0;
      if (aL) {
        nxt[base] = VgSeg{(uint16_t)s, (uint16_t)cut, 0, 0, 0u, (uint32_t)cut};
        cse0 = (uint32_t)s | ((uint32_t)cut << 16);
      } else {
        atomicOr(&S.head[s >> 5], 1u << (s & 31));
      }
      if (aR) {
        nxt[base + aL] = VgSeg{(uint16_t)cut, (uint16_t)e, 0, 0, 0u, (uint32_t)e};
        cse1 = (uint32_t)cut | ((uint32_t)e << 16);
      } else {
        atomicOr(&S.head[cut >> 5], 1u << (cut & 31));
      }
      ((uint32_t*)&cur[tid])[1] = (uint32_t)base | ((uint32_t)(aL | (aR << 1)) << 16);
    }
    __syncthreads();
    VG_STAMP(4);
    {  // the positions' new segments
      uint32_t act = 0;
      for (int j0 = 0; j0 < RM; j0 += BR) {
        if (!((rowact >> j0) & ((1u << BR) - 1))) continue;
        uint2 g[BR];  // children's slot | which, cut
#pragma unroll
        for (int u = 0; u < BR; ++u) {
          const int j = j0 + u;
          g[u] = make_uint2(0u, 0u);
          const uint32_t id = SD(j);
          if (id != 0xffffu) {
            const uint32_t* c = (const uint32_t*)&cur[id];
            g[u] = make_uint2(c[1], c[3]);
          }
        }
#pragma unroll
        for (int u = 0; u < BR; ++u) {
          const int j = j0 + u;
          if (!((rowact >> j) & 1u)) continue;
          const int i = w0 + (j << 6) + lane;
          if (SD(j) != 0xffffu) {
            const int ch = (int)(g[u].x >> 16), base = (int)(g[u].x & 0xffffu), cut = (int)g[u].y;
            const uint32_t s = se[j] & 0xffffu, e = se[j] >> 16;
            uint32_t nid = 0xffffu;
            if (i < cut) {
              if (ch & 1) { nid = (uint32_t)base; se[j] = s | ((uint32_t)cut << 16); }
            } else if (ch & 2) {
              nid = (uint32_t)(base + (ch & 1));
              se[j] = (uint32_t)cut | (e << 16);
            }
            SD_SET(j, nid);
          }
          if (__ballot(SD(j) != 0xffffu)) act |= 1u << j;
        }
      }
      rowact = act;
    }
    if (D - (r + 1) != 0) {  // the children's medians (their keys are final since the swaps)
      if (cse0) {
        const int s = (int)(cse0 & 0xffffu), e = (int)(cse0 >> 16);
        vg_median_to_first(S.key, S.val, s, s + 1, s + (e - s) / 2, e - 1);
      }
      if (cse1) {
        const int s = (int)(cse1 & 0xffffu), e = (int)(cse1 >> 16);
        vg_median_to_first(S.key, S.val, s, s + 1, s + (e - s) / 2, e - 1);
      }
    }
    __syncthreads();
    VG_STAMP(6);
  }
#undef SD
#undef SD_SET
  VG_STAMP(7);
  vg_block_finish(S, n, sumOrder);
}

// The same sort with the positions' segment ids in LDS (S.sid) instead of
// registers: seven barriers per level and more LDS round trips, twelve
// fewer VGPRs.  k_lf_voxel keeps it: inside that kernel the register form
// spilled under the 128-VGPR cap at both block sizes, and both such builds
// faulted on the GPU, though the form itself is exact in
// kernels of its own (modes 0, 3, 4, 5 of lego_sort_permutation).
template <typename V>
__device__ void vg_block_sort_sid(const VgSortLds<V>& S, int n, int depth = -1, int* heapStat = nullptr,
                              bool sumOrder = false) {
  constexpr int RM = kVgRowsMax;
  int tid = threadIdx.x;
  asm volatile("" : "+v"(tid));  // the lane terms computed per call, not held across the caller's loops
  const int T = blockDim.x, lane = tid & 63, wave = tid >> 6, nw = T >> 6;
  const int cap = vg_list_cap(n);
  const int D = depth >= 0 ? depth : (n > 1 ? 2 * (31 - __builtin_clz((unsigned)n)) : 0);
  const int P = (((n + nw - 1) / nw) + 63) & ~63;  // positions per wave
  const int w0 = wave * P;
  const unsigned long long below = (1ull << lane) - 1;
  int* wt = S.ctl + 2;  // [nw][2] the waves' stop totals
  if (n <= 1) {
    __syncthreads();
    return;
  }
  for (int i = tid; i < n; i += T) S.sid[i] = n > kVgLeaf ? 0 : 0xffff;
  for (int w = tid; w < (n + 31) / 32 + 1; w += T) S.head[w] = (w == 0 && n <= kVgLeaf) ? 1u : 0u;
  if (tid == 0) {
    S.ctl[0] = n > kVgLeaf ? 1 : 0;
    S.tab[0] = VgSeg{0, (uint16_t)n, 0, 0, 0u, (uint32_t)n};
  }
  uint32_t rowact = 0;  // rows of this wave holding positions of a segment (wave-uniform)
  if (n > kVgLeaf)
#pragma unroll
    for (int j = 0; j < RM; ++j)
      if (w0 + (j << 6) < n && (j << 6) < P) rowact |= 1u << j;
  __syncthreads();
  constexpr int BR = 4;  // rows whose operands are gathered together (registers)
  for (int r = 0;; ++r) {
    const int nseg = S.ctl[r & 1];
    if (nseg == 0) break;
    VgSeg* cur = S.tab + (r & 1) * cap;
    VgSeg* nxt = S.tab + ((r + 1) & 1) * cap;
    if (D - r == 0) {  // depth budget spent: std::__partial_sort of every piece
      // pieces of > 16 keys, heap-sorted in vg_block_finish (pr[s] = 2),
      // or with sumOrder a leaf unless a key occurs 3+ times (pr[s] = 0, set
      // to 1 there if so)
      for (int j = tid; j < nseg; j += T) {
        const int s = cur[j].s, e = cur[j].e;
        atomicOr(&S.head[s >> 5], 1u << (s & 31));
        S.pr[s] = sumOrder && e - s <= T * kVgMoveRows ? 0 : 2;
        if (heapStat) atomicAdd(heapStat, 1);
      }
      __syncthreads();
      break;
    }
    for (int j = tid; j < nseg; j += T) {
      const int s = cur[j].s, e = cur[j].e;
      vg_median_to_first(S.key, S.val, s, s + 1, s + (e - s) / 2, e - 1);
      cur[j].cut = (uint32_t)e;
      cur[j].ck = 0u;
    }
    if (tid == 0) S.ctl[(r + 1) & 1] = 0;  // last read at round r - 1's top
    __syncthreads();
    VG_STAMP(0);
    // stop flags (a bit per row) and the wave's totals
    uint32_t fl = 0, fr = 0;
    int totLw = 0, totRw = 0;
    for (int j0 = 0; j0 < RM; j0 += BR) {
      if (!((rowact >> j0) & ((1u << BR) - 1))) continue;
      int id[BR], ss[BR];
      uint32_t kp[BR], ki[BR];
#pragma unroll
      for (int u = 0; u < BR; ++u) {
        const int i = w0 + ((j0 + u) << 6) + lane;
        id[u] = ((rowact >> (j0 + u)) & 1u) && i < n ? (int)S.sid[i] : 0xffff;
      }
#pragma unroll
      for (int u = 0; u < BR; ++u) ss[u] = id[u] != 0xffff ? (int)cur[id[u]].s : 0;
#pragma unroll
      for (int u = 0; u < BR; ++u) {
        const int i = w0 + ((j0 + u) << 6) + lane;
        const bool in = id[u] != 0xffff && i > ss[u];
        kp[u] = in ? S.key[ss[u]] : 0u;
        ki[u] = in ? S.key[i] : 0u;
      }
#pragma unroll
      for (int u = 0; u < BR; ++u) {
        const int i = w0 + ((j0 + u) << 6) + lane;
        const bool in = id[u] != 0xffff && i > ss[u];
        const bool lf = in && !(ki[u] < kp[u]), rf = in && !(kp[u] < ki[u]);
        fl |= (lf ? 1u : 0u) << (j0 + u);
        fr |= (rf ? 1u : 0u) << (j0 + u);
        totLw += (int)__popcll(__ballot(lf));
        totRw += (int)__popcll(__ballot(rf));
      }
    }
    if (lane == 0) { wt[2 * wave] = totLw; wt[2 * wave + 1] = totRw; }
    __syncthreads();
    VG_STAMP(1);
    int baseL = 0, baseR = 0;
    for (int w = 0; w < wave; ++w) { baseL += wt[2 * w]; baseR += wt[2 * w + 1]; }
    {  // the block-wide inclusive counts at every segment's start and last position
      int aL = baseL, aR = baseR;
      for (int j0 = 0; j0 < RM; j0 += BR) {
        int id[BR], ss[BR], ee[BR], SL[BR], SR[BR];
#pragma unroll
        for (int u = 0; u < BR; ++u) {
          const int j = j0 + u;
          const bool lf = (fl >> j) & 1u, rf = (fr >> j) & 1u;
          const unsigned long long ml = __ballot(lf), mr = __ballot(rf);
          SL[u] = aL + (int)__popcll(ml & below) + (lf ? 1 : 0);
          SR[u] = aR + (int)__popcll(mr & below) + (rf ? 1 : 0);
          aL += (int)__popcll(ml);
          aR += (int)__popcll(mr);
        }
        if (!((rowact >> j0) & ((1u << BR) - 1))) continue;
#pragma unroll
        for (int u = 0; u < BR; ++u) {
          const int i = w0 + ((j0 + u) << 6) + lane;
          id[u] = ((rowact >> (j0 + u)) & 1u) && i < n ? (int)S.sid[i] : 0xffff;
        }
#pragma unroll
        for (int u = 0; u < BR; ++u) {
          ss[u] = id[u] != 0xffff ? (int)cur[id[u]].s : -1;
          ee[u] = id[u] != 0xffff ? (int)cur[id[u]].e : -1;
        }
#pragma unroll
        for (int u = 0; u < BR; ++u) {
          const int i = w0 + ((j0 + u) << 6) + lane;
          if (id[u] == 0xffff) continue;
          if (i == ss[u]) *(uint16_t*)&cur[id[u]].ck = (uint16_t)SL[u];
          if (i == ee[u] - 1) { cur[id[u]].A = (uint16_t)SL[u]; cur[id[u]].B = (uint16_t)SR[u]; }
        }
      }
    }
    __syncthreads();
    VG_STAMP(2);
    {  // ranks, the pairing rule, partners, the cut's candidates, the swap count
      int aL = baseL, aR = baseR;
      for (int j0 = 0; j0 < RM; j0 += BR) {
        int SL[BR], SR[BR];
#pragma unroll
        for (int u = 0; u < BR; ++u) {
          const int j = j0 + u;
          const bool lf = (fl >> j) & 1u, rf = (fr >> j) & 1u;
          const unsigned long long ml = __ballot(lf), mr = __ballot(rf);
          SL[u] = aL + (int)__popcll(ml & below) + (lf ? 1 : 0);
          SR[u] = aR + (int)__popcll(mr & below) + (rf ? 1 : 0);
          aL += (int)__popcll(ml);
          aR += (int)__popcll(mr);
        }
        if (!((rowact >> j0) & ((1u << BR) - 1))) continue;
        int id[BR];
        uint4 g[BR];  // s | e << 16, A | B << 16, ck, cut
#pragma unroll
        for (int u = 0; u < BR; ++u) {
          const int i = w0 + ((j0 + u) << 6) + lane;
          id[u] = (((fl | fr) >> (j0 + u)) & 1u) ? (int)S.sid[i] : 0xffff;
        }
#pragma unroll
        for (int u = 0; u < BR; ++u) g[u] = id[u] != 0xffff ? *(const uint4*)&cur[id[u]] : make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int u = 0; u < BR; ++u) {
          const int j = j0 + u;
          if (!((rowact >> j) & 1u)) continue;
          const bool lf = (fl >> j) & 1u, rf = (fr >> j) & 1u;
          const int i = w0 + (j << 6) + lane;
          const int s = (int)(g[u].x & 0xffffu), e = (int)(g[u].x >> 16);
          const int A = (int)(g[u].y & 0xffffu), B = (int)(g[u].y >> 16), Cc = (int)(g[u].z & 0xffffu);
          const int totL = A - Cc, Lab = A - SL[u], Rab = B - SR[u];  // left stops, stops after i
          // right stop of rank Rab + 1 (from the right): swapped iff at least
          // that many left stops precede it; left stop of rank totL - Lab:
          // swapped iff at least that many right stops follow it
          const bool rsw = rf && totL - Lab - (lf ? 1 : 0) >= Rab + 1;
          const bool lsw = lf && Rab >= totL - Lab;
          if (rsw) S.pr[s + Rab] = (uint16_t)i;
          if (lsw) S.pr[s + ((e - s + 1) >> 1) + (totL - Lab) - 1] = (uint16_t)i;
          const bool cand = (lf && !lsw) || rsw;
          // one atomic per segment run of the row: its lowest candidate, its
          // highest swapped left stop (ranks grow with the position)
          const unsigned long long mc = __ballot(cand), mw = __ballot(lsw);
          const int rb = i - lane;
          if (cand && !(mc & below & ~((1ull << max(0, s - rb)) - 1))) atomicMin(&cur[id[u]].cut, (uint32_t)i);
          if (lsw) {
            const int hiL = min(64, e - rb);
            const unsigned long long abv = (hiL >= 64 ? ~0ull : ((1ull << hiL) - 1)) & ~below & ~(1ull << lane);
            if (!(mw & abv)) atomicMax(&cur[id[u]].ck, (uint32_t)Cc | ((uint32_t)(totL - Lab) << 16));
          }
        }
      }
    }
    __syncthreads();
    VG_STAMP(3);
    for (int j0 = 0; j0 < RM; j0 += BR) {  // pair q of a segment, at the position s + q
      if (!((rowact >> j0) & ((1u << BR) - 1))) continue;
      int id[BR], pa[BR], pb[BR];
      uint4 g[BR];
#pragma unroll
      for (int u = 0; u < BR; ++u) {
        const int x = w0 + ((j0 + u) << 6) + lane;
        id[u] = ((rowact >> (j0 + u)) & 1u) && x < n ? (int)S.sid[x] : 0xffff;
      }
#pragma unroll
      for (int u = 0; u < BR; ++u) g[u] = id[u] != 0xffff ? *(const uint4*)&cur[id[u]] : make_uint4(0, 0, 0, 0);
#pragma unroll
      for (int u = 0; u < BR; ++u) {
        const int x = w0 + ((j0 + u) << 6) + lane;
        const int s = (int)(g[u].x & 0xffffu), e = (int)(g[u].x >> 16), q = x - s;
        const bool sw = id[u] != 0xffff && q < (int)(g[u].z >> 16);
        pa[u] = sw ? (int)S.pr[s + ((e - s + 1) >> 1) + q] : -1;
        pb[u] = sw ? (int)S.pr[x] : -1;
      }
#pragma unroll
      for (int u = 0; u < BR; ++u)
        if (pa[u] >= 0) vg_swap(S.key, S.val, pa[u], pb[u]);
    }
    __syncthreads();
    VG_STAMP(4);
    for (int j = tid; j < nseg; j += T) {  // the children
      const int s = cur[j].s, e = cur[j].e, cut = (int)cur[j].cut;
      const int aL = cut - s > kVgLeaf ? 1 : 0, aR = e - cut > kVgLeaf ? 1 : 0;
      const int base = (aL + aR) ? atomicAdd(&S.ctl[(r + 1) & 1], aL + aR) : 0;
      if (aL) nxt[base] = VgSeg{(uint16_t)s, (uint16_t)cut, 0, 0, 0u, 0u};
      else atomicOr(&S.head[s >> 5], 1u << (s & 31));
      if (aR) nxt[base + aL] = VgSeg{(uint16_t)cut, (uint16_t)e, 0, 0, 0u, 0u};
      else atomicOr(&S.head[cut >> 5], 1u << (cut & 31));
      cur[j].ck = (uint32_t)base | ((uint32_t)(aL | (aR << 1)) << 16);
    }
    __syncthreads();
    VG_STAMP(5);
    {
      uint32_t act = 0;
      for (int j0 = 0; j0 < RM; j0 += BR) {
        if (!((rowact >> j0) & ((1u << BR) - 1))) continue;
        int id[BR];
        uint4 g[BR];
#pragma unroll
        for (int u = 0; u < BR; ++u) {
          const int i = w0 + ((j0 + u) << 6) + lane;
          id[u] = ((rowact >> (j0 + u)) & 1u) && i < n ? (int)S.sid[i] : 0xffff;
        }
#pragma unroll
        for (int u = 0; u < BR; ++u) g[u] = id[u] != 0xffff ? *(const uint4*)&cur[id[u]] : make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int u = 0; u < BR; ++u) {
          const int i = w0 + ((j0 + u) << 6) + lane;
          int nid = 0xffff;
          if (id[u] != 0xffff) {
            const int ch = (int)(g[u].z >> 16), base = (int)(g[u].z & 0xffffu);
            if (i < (int)g[u].w) { if (ch & 1) nid = base; }
            else if (ch & 2) nid = base + (ch & 1);
            S.sid[i] = (uint16_t)nid;
          }
          if ((rowact >> (j0 + u)) & 1u)
            if (__ballot(nid != 0xffff)) act |= 1u << (j0 + u);
        }
      }
      rowact = act;
    }
    __syncthreads();
    VG_STAMP(6);
  }
  VG_STAMP(7);
  vg_block_finish(S, n, sumOrder);
}

}  // namespace lego
