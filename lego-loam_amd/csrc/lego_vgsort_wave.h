// lego_vgsort_wave.h — libstdc++'s std::sort permutation of one small array
// (<= kVgWaveMax keys) by ONE wave, no workgroup barrier: the same rules as
// lego_vgsort.h's block sort (see there), every level of the segment's pieces
// at once.  Up to 64 keys in registers (shuffles and ballots); up to
// kVgWaveMax keys with a key per lane per row and an LDS word per position for
// the prefix counts and partners.
#pragma once
#include "lego_vgsort.h"

namespace lego {

#ifndef VG_WSTAMP
#define VG_WSTAMP(k, t0) (void)(t0)
#endif
#ifndef VG_CLOCK
#define VG_CLOCK() 0ull
#endif
#ifndef VG_WAVE_ROWS_W
#define VG_WAVE_ROWS_W 8
#endif
constexpr int kVgWaveRowsW = VG_WAVE_ROWS_W;
constexpr int kVgWaveMax = 64 * kVgWaveRowsW;

// index of the n-th (1-based) set bit of m (n <= popcount(m))
__device__ __forceinline__ int vg_nth_bit(unsigned long long m, int n) {
  int q = 0;
#pragma unroll
  for (int b = 32; b > 0; b >>= 1) {
    const unsigned long long low = q + b >= 64 ? m : (m & ((1ull << (q + b)) - 1));
    if ((int)__popcll(low) < n) q += b;
  }
  return q;
}
// bits [a, b) of a 64-bit mask (0 <= a, b <= 64)
__device__ __forceinline__ unsigned long long vg_range(int a, int b) {
  if (a >= b) return 0ull;
  const unsigned long long hi = b >= 64 ? ~0ull : ((1ull << b) - 1);
  const unsigned long long lo = a >= 64 ? ~0ull : ((1ull << a) - 1);
  return hi & ~lo;
}

// The whole introsort of a segment [s, s + m), m <= 64, in one wave's
// registers: lane l holds position s + l; every level partitions all of the
// segment's pieces larger than 16 at once (median of three, the pairing rule
// by popcounts of ballots, the partners as the n-th set bit, the swaps as lane
// permutations), the pieces of <= 16 are stable-sorted by rank, and each key
// lands at its final position.  depth: the segment's budget; when it runs out
// the pieces still larger than 16 are heap-sorted (the wave, in LDS).
template <typename V>
__device__ void vg_wave_sort64(uint32_t* key, V* val, int s, int m, int depth, int* heapStat) {
  const int lane = threadIdx.x & 63;
  const bool act = lane < m;
  uint32_t k = act ? key[s + lane] : 0xffffffffu;
  int v = act ? (int)val[s + lane] : 0;
  int lo = 0, hi = m;
  for (int r = 0;; ++r) {
    const bool big = act && hi - lo > kVgLeaf;
    if (!__ballot(big)) break;
    if (depth - r == 0) {  // std::__partial_sort of every piece still above 16
      if (act) { key[s + lane] = k; val[s + lane] = (V)v; }
      vg_wave_sync();
      unsigned long long starts = __ballot(big && lane == lo);
      while (starts) {
        const int st = (int)__ffsll((long long)starts) - 1;
        const int en = __builtin_amdgcn_readlane(hi, st);
        vg_heap_sort_wave(key, val, s + st, s + en);
        if (heapStat && lane == 0) atomicAdd(heapStat, 1);
        starts &= starts - 1;
      }
      vg_wave_sync();
      if (act) { k = key[s + lane]; v = (int)val[s + lane]; }
      if (big) { lo = lane; hi = lane + 1; }  // sorted: the leaf step leaves them
      continue;
    }
    // std::__move_median_to_first(lo, lo + 1, mid, hi - 1)
    const int mid = lo + (hi - lo) / 2;
    const uint32_t ka = __shfl(k, min(lo + 1, 63), 64), kb = __shfl(k, mid, 64), kc = __shfl(k, max(hi - 1, 0), 64);
    int med;
    if (ka < kb) med = kb < kc ? mid : (ka < kc ? hi - 1 : lo + 1);
    else med = ka < kc ? lo + 1 : (kb < kc ? hi - 1 : mid);
    int src = lane;
    if (big && lane == lo) src = med;
    else if (big && lane == med) src = lo;
    k = __shfl(k, src, 64);
    v = __shfl(v, src, 64);
    const uint32_t p = __shfl(k, lo, 64);
    const bool inr = big && lane > lo;
    const bool lf = inr && !(k < p), rf = inr && !(p < k);
    const unsigned long long ml = __ballot(lf), mr = __ballot(rf);
    const unsigned long long seg = vg_range(lo + 1, hi), aft = vg_range(lane + 1, hi);
    const int totL = (int)__popcll(ml & seg), totR = (int)__popcll(mr & seg);
    const int Lab = (int)__popcll(ml & aft), Rab = (int)__popcll(mr & aft);
    const bool rsw = rf && totL - Lab - (lf ? 1 : 0) >= Rab + 1;
    const bool lsw = lf && Rab >= totL - Lab;
    src = lane;
    if (lsw) src = vg_nth_bit(mr & seg, totR - (totL - Lab) + 1);  // the (totL - Lab)-th right stop from the right
    if (rsw) src = vg_nth_bit(ml & seg, Rab + 1);                  // the (Rab + 1)-th left stop
    k = __shfl(k, src, 64);
    v = __shfl(v, src, 64);
    const unsigned long long mc = __ballot((lf && !lsw) || rsw);
    if (big) {
      const unsigned long long cm = mc & seg;
      const int cut = cm ? (int)__ffsll((long long)cm) - 1 : hi;
      if (lane < cut) hi = cut;
      else lo = cut;
    }
  }
  // pieces of <= 16: stable rank within the piece, then the final positions
  int rank = 0;
#pragma unroll
  for (int j = 0; j < kVgLeaf; ++j) {
    const int q = lo + j;
    const uint32_t kj = __shfl(k, q < 64 ? q : 63, 64);
    if (q < hi) rank += (kj < k || (kj == k && q < lane)) ? 1 : 0;
  }
  vg_wave_sync();
  if (act) {
    key[s + lo + rank] = k;
    val[s + lo + rank] = (V)v;
  }
  vg_wave_sync();
}


// The introsort of a segment [s, s + m), 64 < m <= kVgWave, by one wave: slot
// (j, lane) holds the position s + 64 j + lane in registers (key, payload, its
// piece [lo, hi) in slot indices); every level partitions all of the
// segment's pieces larger than 16 at once.  Per level: the median of three
// (LDS reads of the synced key array) and its swap to the piece's start; the
// stop flags and their wave-wide prefix counts (ballots, row by row); the
// counts at each piece's ends through c[] (a word per position, the block's
// sid / pr scratch); the pairing rule; the partners' slot indices scattered
// into c[]'s low halves (right stops from the piece's start + 1, left stops
// from its middle), the cut by an LDS atomicMin at the piece's start; the
// swaps through the key array.  Then every slot ranks itself (stably) in its
// piece of <= 16 and moves there.  The depth budget runs out: every piece
// still above 16 is heap-sorted by the wave.
template <typename V>
__device__ void vg_wave_sortR(uint32_t* key, V* val, uint32_t* c, int s, int m, int depth, int* heapStat) {
  constexpr int RM = kVgWaveRowsW;
  const int lane = threadIdx.x & 63;
  const int R = (m + 63) >> 6;
  const unsigned long long below = (1ull << lane) - 1;
  uint16_t* c16 = (uint16_t*)c;
  uint32_t k[RM], v[RM], lh[RM];  // key, payload, piece lo | hi << 16
#pragma unroll
  for (int j = 0; j < RM; ++j) {
    const int x = (j << 6) + lane;
    const bool act = j < R && x < m;
    k[j] = act ? key[s + x] : 0u;
    v[j] = act ? (uint32_t)val[s + x] : 0u;
    lh[j] = act ? ((uint32_t)m << 16) : ((uint32_t)x | ((uint32_t)(x + 1) << 16));
  }
#define VG_LO(j) ((int)(lh[j] & 0xffffu))
#define VG_HI(j) ((int)(lh[j] >> 16))
  unsigned long long t0 = VG_CLOCK();
  for (int r = 0;; ++r) {
    uint32_t big = 0;  // bit j: this lane's slot of row j is in a piece > 16
#pragma unroll
    for (int j = 0; j < RM; ++j)
      if (j < R && VG_HI(j) - VG_LO(j) > kVgLeaf) big |= 1u << j;
    if (!__ballot(big != 0)) break;
    if (depth - r == 0) {  // std::__partial_sort of every piece still above 16
#pragma unroll
      for (int j = 0; j < RM; ++j) {  // the pieces' ends at their first slots, 0 elsewhere
        const int x = (j << 6) + lane;
        if (j < R && x < m) c[s + x] = (((big >> j) & 1u) && x == VG_LO(j)) ? (uint32_t)VG_HI(j) : 0u;
      }
      vg_wave_sync();
      for (int q0 = 0; q0 < m; q0 += 64) {  // the pieces row by row, the wave on each
        const int h = q0 + lane < m ? (int)c[s + q0 + lane] : 0;
        unsigned long long starts = __ballot(h != 0);
        while (starts) {
          const int st = (int)__ffsll((long long)starts) - 1;
          vg_heap_sort_wave(key, val, s + q0 + st, s + __builtin_amdgcn_readlane(h, st));
          if (heapStat && lane == 0) atomicAdd(heapStat, 1);
          starts &= starts - 1;
        }
      }
      vg_wave_sync();
#pragma unroll
      for (int j = 0; j < RM; ++j)
        if ((big >> j) & 1u) {
          const int x = (j << 6) + lane;
          k[j] = key[s + x];
          v[j] = (uint32_t)val[s + x];
          lh[j] = (uint32_t)x | ((uint32_t)(x + 1) << 16);
        }
      vg_wave_sync();
      break;
    }
    // std::__move_median_to_first(lo, lo + 1, mid, hi - 1); p = the median.
    // The piece's first slot takes the median's payload, the median's slot
    // the first's key and payload (read before either is written).
    uint32_t p[RM], tk[RM], tv[RM];
    uint32_t sw = 0;  // bit j: the slot changes in the median swap
#pragma unroll
    for (int j = 0; j < RM; ++j) {
      p[j] = 0u;
      if ((big >> j) & 1u) {
        const int lo = VG_LO(j), hi = VG_HI(j), x = (j << 6) + lane;
        const int mid = lo + ((hi - lo) >> 1);
        const uint32_t ka = key[s + lo + 1], kb = key[s + mid], kc = key[s + hi - 1];
        int md;
        if (ka < kb) md = kb < kc ? mid : (ka < kc ? hi - 1 : lo + 1);
        else md = ka < kc ? lo + 1 : (kb < kc ? hi - 1 : mid);
        p[j] = md == mid ? kb : (md == lo + 1 ? ka : kc);
        if (x == lo) { tk[j] = p[j]; tv[j] = (uint32_t)val[s + md]; sw |= 1u << j; }
        else if (x == md) { tk[j] = key[s + lo]; tv[j] = (uint32_t)val[s + lo]; sw |= 1u << j; }
      }
    }
    vg_wave_sync();
    VG_WSTAMP(9, t0); t0 = VG_CLOCK();
#pragma unroll
    for (int j = 0; j < RM; ++j)
      if ((sw >> j) & 1u) {
        const int x = (j << 6) + lane;
        k[j] = tk[j];
        v[j] = tv[j];
        key[s + x] = tk[j];
        val[s + x] = (V)tv[j];
      }
    // stop flags, their wave-wide inclusive prefix counts to c[]
    uint32_t fl = 0, fr = 0;
    {
      int aL = 0, aR = 0;
#pragma unroll
      for (int j = 0; j < RM; ++j) {
        if (j >= R) continue;
        const int x = (j << 6) + lane;
        const bool in = ((big >> j) & 1u) && x > VG_LO(j);
        const bool lf = in && !(k[j] < p[j]), rf = in && !(p[j] < k[j]);
        fl |= (lf ? 1u : 0u) << j;
        fr |= (rf ? 1u : 0u) << j;
        const unsigned long long ml = __ballot(lf), mr = __ballot(rf);
        const int PL = aL + (int)__popcll(ml & below) + (lf ? 1 : 0);
        const int PR = aR + (int)__popcll(mr & below) + (rf ? 1 : 0);
        aL += (int)__popcll(ml);
        aR += (int)__popcll(mr);
        if (x < m) c[s + x] = (uint32_t)PL | ((uint32_t)PR << 16);
      }
    }
    vg_wave_sync();
    VG_WSTAMP(10, t0); t0 = VG_CLOCK();
    // the pairing rule: rk = a swapped left stop's rank t (the t-th right
    // stop from the right is its partner) or a swapped right stop's rank
    // from the right - 1 (Rab; its partner the (Rab + 1)-th left stop)
    uint32_t lsw = 0, rsw = 0;
    int rk[RM];
#pragma unroll
    for (int j = 0; j < RM; ++j) {
      rk[j] = 0;
      if (((fl | fr) >> j) & 1u) {
        const int lo = VG_LO(j), hi = VG_HI(j), x = (j << 6) + lane;
        const uint32_t c0 = c[s + lo], c1 = c[s + hi - 1], cx = c[s + x];
        const int Al = (int)(c1 & 0xffffu), Ar = (int)(c1 >> 16);
        const int totL = Al - (int)(c0 & 0xffffu), Lab = Al - (int)(cx & 0xffffu), Rab = Ar - (int)(cx >> 16);
        const bool lf = (fl >> j) & 1u, rf = (fr >> j) & 1u;
        const bool rs = rf && totL - Lab - (lf ? 1 : 0) >= Rab + 1;
        const bool ls = lf && Rab >= totL - Lab;
        if (rs) { rsw |= 1u << j; rk[j] = Rab; }
        if (ls) { lsw |= 1u << j; rk[j] = totL - Lab; }
      }
    }
    vg_wave_sync();
#pragma unroll
    for (int j = 0; j < RM; ++j)
      if (((big >> j) & 1u) && (j << 6) + lane == VG_LO(j)) c[s + VG_LO(j)] = (uint32_t)VG_HI(j);
    vg_wave_sync();
    VG_WSTAMP(11, t0); t0 = VG_CLOCK();
#pragma unroll
    for (int j = 0; j < RM; ++j) {
      if (j >= R) continue;
      const int lo = VG_LO(j), x = (j << 6) + lane;
      const int half = (VG_HI(j) - lo - 1) >> 1;
      if ((rsw >> j) & 1u) c16[2 * (s + lo + 1 + rk[j])] = (uint16_t)x;
      if ((lsw >> j) & 1u) c16[2 * (s + lo + half + rk[j])] = (uint16_t)x;
      const bool cand = (((fl & ~lsw) | rsw) >> j) & 1u;
      const unsigned long long mc = __ballot(cand);
      if (cand && !(mc & below & ~((1ull << max(0, lo - (j << 6))) - 1)))  // the piece's lowest in this row
        atomicMin(&c[s + lo], (uint32_t)x);
    }
    vg_wave_sync();
    VG_WSTAMP(12, t0); t0 = VG_CLOCK();
#pragma unroll
    for (int j = 0; j < RM; ++j) {
      tk[j] = k[j];
      tv[j] = v[j];
      if ((big >> j) & 1u) {
        const int lo = VG_LO(j), x = (j << 6) + lane;
        const int half = (VG_HI(j) - lo - 1) >> 1;
        int pa = -1;
        if ((lsw >> j) & 1u) pa = (int)c16[2 * (s + lo + rk[j])];
        if ((rsw >> j) & 1u) pa = (int)c16[2 * (s + lo + 1 + half + rk[j])];
        if (pa >= 0) { tk[j] = key[s + pa]; tv[j] = (uint32_t)val[s + pa]; }
        const int cut = (int)c[s + lo];
        lh[j] = x < cut ? ((uint32_t)lo | ((uint32_t)cut << 16)) : ((uint32_t)cut | (lh[j] & 0xffff0000u));
      }
    }
    vg_wave_sync();
#pragma unroll
    for (int j = 0; j < RM; ++j)
      if (((lsw | rsw) >> j) & 1u) {
        const int x = (j << 6) + lane;
        k[j] = tk[j];
        v[j] = tv[j];
        key[s + x] = tk[j];
        val[s + x] = (V)tv[j];
      }
    vg_wave_sync();
    VG_WSTAMP(13, t0); t0 = VG_CLOCK();
  }
  // pieces of <= 16: stable rank within the piece (the key array is synced)
  int rk[RM];
#pragma unroll
  for (int j = 0; j < RM; ++j) {
    rk[j] = 0;
    const int x = (j << 6) + lane;
    if (j >= R || x >= m) continue;
    for (int q = VG_LO(j); q < VG_HI(j); ++q) {
      const uint32_t kq = key[s + q];
      rk[j] += (kq < k[j] || (kq == k[j] && q < x)) ? 1 : 0;
    }
  }
  vg_wave_sync();
#pragma unroll
  for (int j = 0; j < RM; ++j) {
    const int x = (j << 6) + lane;
    if (j < R && x < m) {
      key[s + VG_LO(j) + rk[j]] = k[j];
      val[s + VG_LO(j) + rk[j]] = (V)v[j];
    }
  }
  vg_wave_sync();
  VG_WSTAMP(14, t0);
#undef VG_LO
#undef VG_HI
}


// std::sort of key[0, n) / val[0, n), n <= kVgWaveMax, by the calling wave
// alone; c: an LDS scratch word per key.  Ends with the wave in sync.
// depth: the introsort loop's budget (2 lg n for a whole array, less for a
// segment of one; -1 = 2 lg n); heapStat: bumped per heap-sorted piece.
template <typename V>
__device__ void vg_wave_sort(uint32_t* key, V* val, uint32_t* c, int n, int depth = -1, int* heapStat = nullptr) {
  if (n <= 1) return;
  const int D = depth >= 0 ? depth : 2 * (31 - __builtin_clz((unsigned)n));
  if (n <= 64) vg_wave_sort64(key, val, 0, n, D, heapStat);
  else vg_wave_sortR(key, val, c, 0, n, D, heapStat);
}

}  // namespace lego
