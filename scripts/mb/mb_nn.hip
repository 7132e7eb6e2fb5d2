// Microbenchmark: the odometry's per-query NN search (nn_i1 + nn_lines) on
// real-shaped clouds (scripts/mb/nn_data.py), one workgroup, one wave per
// query, LDS-resident index exactly as k_odom builds it.  Prints per-pair the
// query-time distribution and the brute-force fallbacks, surf and corner.
#include <cstdio>
#include <vector>
#include <algorithm>
#include "../../lego-loam_amd/csrc/lego_odom.hip"
using namespace lego;
namespace lego {

// branch-free scan-line window: four loads in flight per lane, selects only
template <class Idx>
__device__ __forceinline__ bool nn_lines_v2(const NNView<Idx>& v, int ci, int jend, float4 sel, bool surf, float nn_sq,
                                            int g, int* o2, int* o3, unsigned long long* ts) {
  long long t0 = wall_clock64();
  if (v.irregular) return false;
  const int cScan = (int)v.pts[ci].w;
  const int F = (cScan + 3 <= v.NK) ? v.sufFirst[cScan + 3] : INT_MAX;
  const int B = (cScan - 3 >= 0) ? v.preLast[cScan - 3] : -1;
  if (F <= ci || B >= ci) return false;
  const int fwdEnd = min(F, jend);
  float m2 = nn_sq, m3 = nn_sq;
  int r2 = INT_MAX, r3 = INT_MAX;
  // forward part (ci, fwdEnd) then backward part (B, ci) as one range of
  // visit ranks: rank k < nf is j = ci + 1 + k, else j = B + 1 + (k - nf)
  const int nf = max(0, fwdEnd - ci - 1), nb = ci - B - 1, n = nf + nb;
  const int fwdSpan = jend - ci;
  long long t1 = wall_clock64();
  for (int k0 = 0; k0 < n; k0 += 4 * kGL) {
    float4 p[4];
    int jj[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int k = k0 + u * kGL + g;
      jj[u] = k < nf ? ci + 1 + k : B + 1 + (k - nf);
      p[u] = v.pts[k < n ? jj[u] : ci];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int k = k0 + u * kGL + g, j = jj[u];
      const bool fwd = k < nf;
      const int kj = (int)p[u].w;
      const bool side = fwd ? kj <= cScan : kj >= cScan;  // surf: class 2; corner: skipped
      const float d = line_d2(p[u], sel);
      const bool ok = (k < n) & (d < nn_sq) & (surf | !side);
      const bool c2 = surf ? side : true;
      const int rank = fwd ? j - ci : fwdSpan + (ci - j);
      const bool u2 = ok & c2 & ((d < m2) | ((d == m2) & (rank < r2)));
      const bool u3 = ok & !c2 & ((d < m3) | ((d == m3) & (rank < r3)));
      m2 = u2 ? d : m2; r2 = u2 ? rank : r2;
      m3 = u3 ? d : m3; r3 = u3 ? rank : r3;
    }
  }
  // the index from the rank
  long long t2 = wall_clock64();
  const float d2m = wave_min_f32(m2);
  const int r2m = wave_min_i32(m2 == d2m ? r2 : INT_MAX);
  *o2 = r2m == INT_MAX ? -1 : (r2m < fwdSpan ? ci + r2m : ci - (r2m - fwdSpan));
  if (surf) {
    const float d3m = wave_min_f32(m3);
    const int r3m = wave_min_i32(m3 == d3m ? r3 : INT_MAX);
    *o3 = r3m == INT_MAX ? -1 : (r3m < fwdSpan ? ci + r3m : ci - (r3m - fwdSpan));
  } else {
    *o3 = -1;
  }
  long long t3 = wall_clock64();
  if (g == 0) { ts[0] += t1 - t0; ts[1] += t2 - t1; ts[2] += t3 - t2; ts[3] += 1; ts[4] += n; }
  return true;
}

// u64-key scan-line window: (distance bits, visit rank) packed so that one
// unsigned 64-bit minimum is the lexicographic (distance, rank) minimum
template <class Idx>
__device__ __forceinline__ bool nn_lines_v3(const NNView<Idx>& v, int ci, int jend, float4 sel, bool surf, float nn_sq,
                                            int g, int* o2, int* o3) {
  if (v.irregular) return false;
  const int cScan = (int)v.pts[ci].w;
  const int F = (cScan + 3 <= v.NK) ? v.sufFirst[cScan + 3] : INT_MAX;
  const int B = (cScan - 3 >= 0) ? v.preLast[cScan - 3] : -1;
  if (F <= ci || B >= ci) return false;
  const int fwdEnd = min(F, jend);
  const int nf = max(0, fwdEnd - ci - 1), nb = ci - B - 1, n = nf + nb;
  const int fwdSpan = jend - ci;
  const unsigned long long kNone = ~0ull;
  unsigned long long k2 = kNone, k3 = kNone;
  for (int k0 = 0; k0 < n; k0 += 4 * kGL) {
    float4 p[4];
    int jj[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int k = k0 + u * kGL + g;
      jj[u] = k < nf ? ci + 1 + k : B + 1 + (k - nf);
      p[u] = v.pts[k < n ? jj[u] : ci];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int k = k0 + u * kGL + g, j = jj[u];
      const bool fwd = k < nf;
      const int kj = (int)p[u].w;
      const bool side = fwd ? kj <= cScan : kj >= cScan;  // surf: class 2; corner: skipped
      const float d = line_d2(p[u], sel);
      const bool ok = k < n && d < nn_sq;
      const unsigned rank = fwd ? (unsigned)(j - ci) : (unsigned)(fwdSpan + (ci - j));
      const unsigned long long key = ((unsigned long long)__float_as_uint(d) << 32) | rank;
      const bool to2 = ok && (surf ? side : !side);
      const bool to3 = ok && surf && !side;
      k2 = (to2 && key < k2) ? key : k2;
      k3 = (to3 && key < k3) ? key : k3;
    }
  }
  auto wave_min_u64 = [&](unsigned long long x) {
    x = min(x, (unsigned long long)(((unsigned long long)(unsigned)dpp_i32<0xB1>((int)(x >> 32)) << 32) | (unsigned)dpp_i32<0xB1>((int)x)));
    x = min(x, (unsigned long long)(((unsigned long long)(unsigned)dpp_i32<0x4E>((int)(x >> 32)) << 32) | (unsigned)dpp_i32<0x4E>((int)x)));
    x = min(x, (unsigned long long)(((unsigned long long)(unsigned)dpp_i32<0x141>((int)(x >> 32)) << 32) | (unsigned)dpp_i32<0x141>((int)x)));
    x = min(x, (unsigned long long)(((unsigned long long)(unsigned)dpp_i32<0x140>((int)(x >> 32)) << 32) | (unsigned)dpp_i32<0x140>((int)x)));
    unsigned long long r = kNone;
    for (int l = 0; l < 64; l += 16) {
      const unsigned long long y = ((unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)(x >> 32), l) << 32) |
                                   (unsigned)__builtin_amdgcn_readlane((int)x, l);
      r = min(r, y);
    }
    return r;
  };
  auto idx_of = [&](unsigned long long key) {
    if (key == kNone) return -1;
    const int r = (int)(unsigned)key;
    return r < fwdSpan ? ci + r : ci - (r - fwdSpan);
  };
  *o2 = idx_of(wave_min_u64(k2));
  *o3 = surf ? idx_of(wave_min_u64(k3)) : -1;
  return true;
}

template <int MODE, class Idx>
__device__ __forceinline__ bool nn_lines_dbg(const NNView<Idx>& v, int ci, int jend, float4 sel, bool surf, float nn_sq,
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
  if (MODE != 2) {
#pragma unroll 2
  for (int j = ci + 1 + g; j < fwdEnd; j += kGL) visit(j, true);
#pragma unroll 4
  for (int j = B + 1 + g; j < ci; j += kGL) visit(j, false);
  }
  if (MODE != 1) {
    group_lex_min3(m2, r2, i2);
    if (surf) group_lex_min3(m3, r3, i3);
  } else {
    i2 = i2 + (int)m2 + r2; i3 = i3 + (int)m3 + r3;
  }
  *o2 = i2;
  *o3 = surf ? i3 : -1;
  return true;
}

}

template <int MODE>
__global__ void __launch_bounds__(512) knn(const float4* lastS, int nLS, const float4* qS, int nQS, const float4* lastC,
                                           int nLC, const float4* qC, int nQC, long long* qt, int* qb, int nwk) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
  const OdomLds L = odom_carve(lds_raw);
  __shared__ unsigned long long wp[8][32];
  const int tid = threadIdx.x, g = tid & 63, w = tid >> 6;
  OdomState* st = L.st;
  DevCfg c = {};
  c.N = 16;
  c.nn_sq = 25.f;
  if (tid == 0) {
    st->surfLastNum = nLS; st->cornerLastNum = nLC; st->resident = 1; st->curBuf = st->snapBuf = 0;
  }
  if (tid < 256) ((unsigned long long*)wp)[tid] = 0;
  for (int i = tid; i < nLS; i += 512) L.lastS[i] = lastS[i];
  for (int i = tid; i < nLC; i += 512) L.lastC[i] = lastC[i];
  __syncthreads();
  nn_build2(lds_build_args(L, st, c, 0), nullptr);  // the grids (this benchmark times their searches)
  for (int side = 0; side < 2; ++side) {
    const bool surf = side == 0;
    const NNView<uint16_t> v = view_lds(surf, L, st, c, 0);
    const float4* qp = surf ? qS : qC;
    const int nQ = surf ? nQS : nQC, lastN = surf ? nLS : nLC, jend = min(nQ, lastN);
    for (int q = w; q < nQ && w < nwk; q += nwk) {
      const unsigned long long b0 = wp[w][P_NN_BRUTE];
      const long long t0 = wall_clock64();
      const float4 sel = qp[q];
      int i1 = nn_i1(v, sel, c.nn_sq, g, wp[w]);
      const long long tm = wall_clock64();
      int win = 0;
      if (i1 >= 0) {
        const int cScan = (int)v.pts[i1].w;
        const int F = (cScan + 3 <= v.NK) ? v.sufFirst[cScan + 3] : INT_MAX;
        const int B = (cScan - 3 >= 0) ? v.preLast[cScan - 3] : -1;
        win = (min(F, jend) > i1 ? min(F, jend) - i1 - 1 : 0) + (i1 - B - 1);
      }
      int i2 = -1, i3 = -1;
      if (i1 >= 0 && !(MODE == 4 ? nn_lines_v3(v, i1, jend, sel, surf, c.nn_sq, g, &i2, &i3) : MODE == 3 ? nn_lines_v2(v, i1, jend, sel, surf, c.nn_sq, g, &i2, &i3, wp[w] + 16 + 5 * side) : nn_lines_dbg<MODE>(v, i1, jend, sel, surf, c.nn_sq, g, &i2, &i3)))
        scanline_group(surf ? L.lastS : L.lastC, jend, i1, sel, surf, c.nn_sq, g, &i2, &i3);
      const long long t1 = wall_clock64();
      if (g == 0 && q + nwk >= nQ && side == 1 && MODE == 3) {
        for (int k = 0; k < 10; ++k) atomicAdd((unsigned long long*)&qt[1900 + k], wp[w][16 + k]);
      }
      if (g == 0) {
        qt[side * 512 + q] = t1 - t0 + (i1 + i2 + i3 == 12345678 ? 1 : 0);
        qb[side * 512 + q] = (int)(wp[w][P_NN_BRUTE] - b0);
        qt[1024 + side * 512 + q] = tm - t0 + (i1 == 12345678);
        qb[1024 + side * 512 + q] = win;
        qb[2048 + side * 512 + q] = i2;
        qb[3072 + side * 512 + q] = i3;
      }
    }
  }
}

int main(int argc, char** argv) {
  FILE* f = fopen("build/nn_data.bin", "rb");
  if (!f) { printf("run scripts/mb/nn_data.py first\n"); return 1; }
  int np = 0;
  if (fread(&np, 4, 1, f) != 1) return 1;
  (void)hipFuncSetAttribute((const void*)knn<0>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)odom_lds_bytes());
  (void)hipFuncSetAttribute((const void*)knn<1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)odom_lds_bytes());
  (void)hipFuncSetAttribute((const void*)knn<2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)odom_lds_bytes());
  (void)hipFuncSetAttribute((const void*)knn<4>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)odom_lds_bytes());
  (void)hipFuncSetAttribute((const void*)knn<3>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)odom_lds_bytes());
  const int MODE = argc > 1 ? atoi(argv[1]) : 0;
  const int nwk = argc > 2 ? atoi(argv[2]) : 8;
  long long* dqt; int* dqb;
  (void)hipMalloc(&dqt, 2048 * 8); (void)hipMalloc(&dqb, 4096 * 4);
  double sumMaxS = 0, sumMaxC = 0, sumMeanS = 0, sumMeanC = 0; int brS = 0, brC = 0, nS = 0, nC = 0;
  for (int p = 0; p < np; ++p) {
    int n[4];
    if (fread(n, 4, 4, f) != 4) return 1;
    std::vector<float4> a[4];
    float4* d[4];
    for (int k = 0; k < 4; ++k) {
      a[k].resize(n[k]);
      if (fread(a[k].data(), 16, n[k], f) != (size_t)n[k]) return 1;
      (void)hipMalloc(&d[k], 16 * (n[k] + 1));
      (void)hipMemcpy(d[k], a[k].data(), 16 * n[k], hipMemcpyHostToDevice);
    }
    if (n[0] > kLdsSurf || n[2] > kLdsCorner || n[1] > 384 || n[3] > 192) { printf("pair %d too large\n", p); continue; }
    (void)hipMemset(dqt, 0, 2048 * 8);
    for (int rep = 0; rep < 1; ++rep)
      if (MODE == 0) knn<0><<<1, 512, odom_lds_bytes()>>>(d[0], n[0], d[1], n[1], d[2], n[2], d[3], n[3], dqt, dqb, nwk);
      else if (MODE == 1) knn<1><<<1, 512, odom_lds_bytes()>>>(d[0], n[0], d[1], n[1], d[2], n[2], d[3], n[3], dqt, dqb, nwk);
      else if (MODE == 4) knn<4><<<1, 512, odom_lds_bytes()>>>(d[0], n[0], d[1], n[1], d[2], n[2], d[3], n[3], dqt, dqb, nwk);
      else if (MODE == 3) knn<3><<<1, 512, odom_lds_bytes()>>>(d[0], n[0], d[1], n[1], d[2], n[2], d[3], n[3], dqt, dqb, nwk);
      else knn<2><<<1, 512, odom_lds_bytes()>>>(d[0], n[0], d[1], n[1], d[2], n[2], d[3], n[3], dqt, dqb, nwk);
    (void)hipDeviceSynchronize();
    std::vector<long long> qt(2048); std::vector<int> qb(4096);
    (void)hipMemcpy(qt.data(), dqt, 2048 * 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(qb.data(), dqb, 4096 * 4, hipMemcpyDeviceToHost);
    if (MODE == 3 && p == np - 1) { for (int sd = 0; sd < 2; ++sd) printf("%s: pre %.2f loop %.2f red %.2f us per call, %.0f pts\n", sd ? "corner" : "surf", qt[1900+5*sd]/100.0/qt[1903+5*sd], qt[1901+5*sd]/100.0/qt[1903+5*sd], qt[1902+5*sd]/100.0/qt[1903+5*sd], (double)qt[1904+5*sd]/qt[1903+5*sd]); }
    static long long ck = 0; for (int t = 2048; t < 4096; ++t) ck = ck * 31 + qb[t]; if (p == np - 1) printf("checksum %lld\n", ck);
    for (int side = 0; side < 2; ++side) {
      const int nq = side ? n[3] : n[1];
      double mx = 0, sm = 0, mxb = 0, si1 = 0, sw = 0; int br = 0;
      for (int q = 0; q < nq; ++q) {
        si1 += qt[1024 + side * 512 + q] / 100.0;
        sw += qb[1024 + side * 512 + q];
        const double us = qt[side * 512 + q] / 100.0;
        mx = std::max(mx, us); sm += us; br += qb[side * 512 + q];
        if (qb[side * 512 + q]) mxb = std::max(mxb, us);
      }
      if (p < 4) printf("pair %2d %s: %3d queries, mean %.2f us (nn_i1 %.2f), max %.2f us, brute %d (max %.2f us), window %.0f pts\n", p,
                        side ? "corner" : "surf  ", nq, sm / nq, si1 / nq, mx, br, mxb, sw / nq);
      if (side) { sumMaxC += mx; sumMeanC += sm / nq; brC += br; nC += nq; }
      else { sumMaxS += mx; sumMeanS += sm / nq; brS += br; nS += nq; }
    }
    for (auto* x : d) (void)hipFree(x);
  }
  printf("ALL %d pairs: surf mean %.2f max %.2f us, brute %d/%d; corner mean %.2f max %.2f us, brute %d/%d\n", np,
         sumMeanS / np, sumMaxS / np, brS, nS, sumMeanC / np, sumMaxC / np, brC, nC);
  return 0;
}
