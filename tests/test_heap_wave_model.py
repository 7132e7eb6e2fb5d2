"""The wave heap sort's algorithm (lego_vgsort.h vg_heap_sort_wave), restated
lane by lane in Python, against std::__partial_sort(first, last, last) as
libstdc++ runs it (make_heap + sort_heap, stl_heap.h; VgHeap in lego_vgsort.h
is its device port).  The wave form runs make_heap a heap level at a time and
each sort_heap pop as a six-level chunked walk (the path's nodes found by
mask tests against the chunk's ballots), a ballot for the push and one
batch of stores; it must leave every (key, payload) pair where the serial form
does, duplicates included (a VoxelGrid sums a voxel's points in that order).
CPU model test; the device code itself is checked against std::sort by
tests/test_gpu_sort_perm.py (McIlroy adversaries: heap-sorted pieces)."""
import random

import pytest


def adjust_heap(K, W, hole, n, vk, vv):
    """std::__adjust_heap + __push_heap (stl_heap.h), as VgHeap::adjust_heap"""
    top = second = hole
    while second < (n - 1) // 2:
        second = 2 * (second + 1)
        if K[second] < K[second - 1]:
            second -= 1
        K[hole], W[hole] = K[second], W[second]
        hole = second
    if n % 2 == 0 and second == (n - 2) // 2:
        second = 2 * (second + 1)
        K[hole], W[hole] = K[second - 1], W[second - 1]
        hole = second - 1
    parent = (hole - 1) // 2
    while hole > top and K[parent] < vk:
        K[hole], W[hole] = K[parent], W[parent]
        hole = parent
        parent = (hole - 1) // 2
    K[hole], W[hole] = vk, vv


def serial_heap_sort(K, W):
    """VgHeap::sort: make_heap (parents (n-2)/2 .. 0), then sort_heap"""
    n = len(K)
    for p in range((n - 2) // 2, -1, -1):
        adjust_heap(K, W, p, n, K[p], W[p])
    for last in range(n - 1, 0, -1):
        vk, vv = K[last], W[last]
        K[last], W[last] = K[0], W[0]
        adjust_heap(K, W, 0, last, vk, vv)


def level(x):
    return x.bit_length() - 1  # 31 - clz(x)


def wave_heap_sort(K, W):
    """vg_heap_sort_wave, one iteration of the lane loops per lane"""
    n = len(K)
    if n < 2:
        return
    last_p = (n - 2) // 2
    for d in range(level(last_p + 1), -1, -1):  # make_heap, a level at a time
        for p in range((1 << d) - 1, min(last_p + 1, (2 << d) - 1)):
            adjust_heap(K, W, p, n, K[p], W[p])
    dl = [level(lane + 1) for lane in range(64)]
    jl = [lane + 1 - (1 << dl[lane]) for lane in range(64)]
    anc, anc_r = [0] * 64, [0] * 64  # the lane's ancestors in a chunk, and those that go right toward it
    for lane in range(64):
        for i in range(dl[lane]):
            a = ((lane + 1) >> (dl[lane] - i)) - 1
            anc[lane] |= 1 << a
            if ((lane + 1) >> (dl[lane] - i - 1)) & 1:
                anc_r[lane] |= 1 << a
    for m in range(n - 1, 0, -1):
        lim, tnode = (m - 1) // 2, ((m - 2) // 2 if m % 2 == 0 else -1)
        h = k = 0
        more = True
        vk, vv, rk, rv = K[m], W[m], K[0], W[0]
        chunks = []
        for _ in range(2):
            px, ck, cv = [-1] * 64, [0] * 64, [0] * 64
            if not more:
                chunks.append((px, ck, cv))
                continue
            G = R = 0
            xs = [(h + 1) * (1 << dl[lane]) - 1 + jl[lane] for lane in range(64)]
            go = [False] * 64
            for lane in range(64):
                x = xs[lane]
                two, one = lane < 63 and x < lim, lane < 63 and x == tnode
                il, ir = (2 * x + 1 if two or one else 0), (2 * x + 2 if two else 0)
                kl, kr, vl, vr = K[il], K[ir], W[il], W[ir]
                right = two and not kr < kl
                ck[lane], cv[lane] = (kr, vr) if right else (kl, vl)
                go[lane] = two or one
                G |= go[lane] << lane
                R |= right << lane
            on = [lane < 63 and (G & anc[lane]) == anc[lane] and (R & anc[lane]) == anc_r[lane]
                  for lane in range(64)]
            P = sum(1 << lane for lane in range(64) if on[lane])
            for lane in range(64):
                if on[lane] and go[lane]:
                    px[lane] = ((k + dl[lane]) << 16) | xs[lane]
            k += bin(P & G).count("1")
            last = P.bit_length() - 1
            dL = level(last + 1)
            xl = (h + 1) * (1 << dL) - 1 + (last + 1 - (1 << dL))
            more = bool((G >> last) & 1)
            h = 2 * xl + 1 + ((R >> last) & 1) if more else xl
            chunks.append((px, ck, cv))
        j = 0
        for px, ck, cv in reversed(chunks):  # the push: one ballot per chunk, deepest first
            F = [lane for lane in range(64) if px[lane] >= 0 and not ck[lane] < vk]
            if F:
                j = (px[max(F)] >> 16) + 1
                break
        K[m], W[m] = rk, rv
        for px, ck, cv in chunks:
            for lane in range(64):
                if px[lane] < 0:
                    continue
                pi, x = px[lane] >> 16, px[lane] & 0xFFFF
                if pi < j:
                    K[x], W[x] = ck[lane], cv[lane]
                elif pi == j:
                    K[x], W[x] = vk, vv
        if j == k:
            K[h], W[h] = vk, vv


@pytest.mark.parametrize("seed", range(4))
def test_wave_heap_model_matches_serial_heap(seed):
    rng = random.Random(seed)
    sizes = [2, 3, 4, 5, 17, 30, 63, 64, 65, 126, 127, 128, 129, 200, 255, 256, 600, 1023, 1024, 2047]
    for t in range(60):
        n = sizes[t % len(sizes)] if t < len(sizes) else rng.randint(2, 700)
        r = rng.choice([2, 5, 20, 1000, 10**9])
        K = [rng.randrange(r) for _ in range(n)]
        W = list(range(n))
        K1, W1, K2, W2 = K[:], W[:], K[:], W[:]
        serial_heap_sort(K1, W1)
        wave_heap_sort(K2, W2)
        assert K1 == sorted(K)
        assert (K1, W1) == (K2, W2), (n, r)
