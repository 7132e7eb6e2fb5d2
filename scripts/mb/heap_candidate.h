// Candidate pop loop for vg_heap_sort_wave (mb_heap.hip, -DMB_HEAP_CANDIDATE):
// every internal node's choice bit ("the walk goes right": !(K[2x+2] <
// K[2x+1]), __adjust_heap's rule) is kept across pops, nodes 0..63 in one
// SGPR pair, the rest at bit x >> 6 of lane x & 63, so a pop's walk from the
// root is scalar bit tests with no LDS access.  Lane i then loads the path's
// x_{i+1} (key, payload), its sibling's key and x_{i+2}'s key in one round
// trip; the push is one ballot; the pop's stores go out together; the
// choice bits of the parents whose child changed (x_0 .. x_{j-1}) are
// recomputed from those loads.  Same element moves as VgHeap::sort.
#pragma once

template <typename V>
__device__ void mb_heap_candidate(uint32_t* key, V* val, int first, int last) {
  int lane = threadIdx.x & 63;
  asm volatile("" : "+v"(lane));
  const int len = last - first;
  if (len < 2) return;
  if (len > lego::kVgHeapWaveMax) {
    if (lane == 0) lego::VgHeap<V>{key, val}.sort(first, last);
    lego::vg_wave_sync();
    return;
  }
  uint32_t* K = key + first;
  V* W = val + first;
  const lego::VgHeap<V> Hp{K, W};
  const int lastP = (len - 2) / 2;
  for (int d = 31 - __builtin_clz((unsigned)lastP + 1); d >= 0; --d) {
    const int hi = min(lastP + 1, (2 << d) - 1);
    for (int p = (1 << d) - 1 + lane; p < hi; p += 64) Hp.adjust_heap(0, p, len, K[p], W[p]);
    lego::vg_wave_sync();
  }
  // choice bits of the heap as built: node x at bit x >> 6 of lane x & 63
  uint32_t dlo = 0u, dhi = 0u;
  for (int b = 0; (b << 6) <= lastP; ++b) {
    const int x = (b << 6) + lane;
    const bool d = 2 * x + 2 < len && !(K[2 * x + 2] < K[2 * x + 1]);
    if (b < 32) dlo |= (uint32_t)d << b;
    else dhi |= (uint32_t)d << (b - 32);
  }
  unsigned long long top = __ballot(dlo & 1u);  // nodes 0..63
  for (int m = len - 1; m >= 1; --m) {
    const int lim = (m - 1) / 2, tnode = (m & 1) == 0 ? (m - 2) / 2 : -1;
    // the walk: x_0 = 0 .. x_k, the choices in `bits` (MSB first)
    int x = 0, k = 0;
    unsigned bits = 0u;
    while (true) {
      int c;
      if (x < lim) {
        if (x < 64) {
          c = (int)((top >> x) & 1ull);
        } else {
          const int b = x >> 6;
          const uint32_t w = b < 32 ? (uint32_t)__builtin_amdgcn_readlane(dlo, x & 63)
                                    : (uint32_t)__builtin_amdgcn_readlane(dhi, x & 63);
          c = (int)((w >> (b & 31)) & 1u);
        }
      } else if (x == tnode) {
        c = 0;
      } else {
        break;
      }
      x = 2 * x + 1 + c;
      bits = (bits << 1) | (unsigned)c;
      ++k;
    }
    // lane i: x_i, x_{i+1} (its key P and payload), x_{i+1}'s sibling's key, x_{i+2}'s key
    const int sh = max(k - lane, 0);
    const int xi = lane <= k ? (1 << lane) - 1 + (int)(bits >> sh) : 0;
    const bool hasC = lane < k, hasC2 = lane + 1 < k;
    const int xc = hasC ? 2 * xi + 1 + (int)((bits >> max(k - lane - 1, 0)) & 1u) : 0;
    const int xc2 = hasC2 ? 2 * xc + 1 + (int)((bits >> max(k - lane - 2, 0)) & 1u) : 0;
    const int sib = (xc & 1) ? xc + 1 : max(xc - 1, 0);
    const bool hasS = hasC && sib < m;
    const uint32_t vk0 = K[m], rk = K[0];
    const V vv0 = W[m], rv = W[0];
    const uint32_t P = K[xc], S = K[hasS ? sib : 0], P2 = K[xc2];
    const V Wp = W[xc];
    const uint32_t vk = __builtin_amdgcn_readfirstlane(vk0);
    // the push: the hole stops at x_j, j = 1 + the deepest i whose P_{i+1} is not < vk
    const unsigned long long F = __ballot(hasC && !(P < vk));
    const int j = F ? 64 - __builtin_clzll(F) : 0;
    if (lane == 0) { K[m] = rk; W[m] = rv; }
    if (lane < j) { K[xi] = P; W[xi] = Wp; }
    if (lane == j) { K[xi] = vk; W[xi] = vv0; }
    // choice bits of x_0 .. x_{j-1}: x_{i+1}'s new key against its sibling's
    const uint32_t nk = lane + 1 < j ? P2 : vk;
    const bool upd = lane < j && hasS;
    const bool nd = (xc & 1) ? !(S < nk) : !(nk < S);
    unsigned long long U = __ballot(upd);
    const unsigned long long D = __ballot(upd && nd);
    while (U) {
      const int i = __builtin_ctzll(U);
      U &= U - 1;
      const int xn = (1 << i) - 1 + (int)(bits >> (k - i));
      const bool bit = (D >> i) & 1ull;
      if (xn < 64) {
        top = bit ? (top | (1ull << xn)) : (top & ~(1ull << xn));
      } else {
        const int b = xn >> 6;
        if (lane == (xn & 63)) {
          if (b < 32) dlo = bit ? (dlo | (1u << b)) : (dlo & ~(1u << b));
          else dhi = bit ? (dhi | (1u << (b - 32))) : (dhi & ~(1u << (b - 32)));
        }
      }
    }
    lego::vg_wave_sync();
  }
}
