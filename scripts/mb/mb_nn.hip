// Microbenchmark: the odometry's per-query NN search (nn_i1 + nn_lines) on
// real-shaped clouds (scripts/mb/nn_data.py), one workgroup, one wave per
// query, LDS-resident index exactly as k_odom builds it.  Prints per-pair the
// query-time distribution and the brute-force fallbacks, surf and corner.
#include <cstdio>
#include <vector>
#include <algorithm>
#include "../../lego-loam_amd/csrc/lego_odom.hip"
using namespace lego;

__global__ void __launch_bounds__(512) knn(const float4* lastS, int nLS, const float4* qS, int nQS, const float4* lastC,
                                           int nLC, const float4* qC, int nQC, long long* qt, int* qb) {
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
  nn_build2(lds_build_args(L, st, c), nullptr);
  for (int side = 0; side < 2; ++side) {
    const bool surf = side == 0;
    const NNView<uint16_t> v = view_lds(surf, L, st, c);
    const float4* qp = surf ? qS : qC;
    const int nQ = surf ? nQS : nQC, lastN = surf ? nLS : nLC, jend = min(nQ, lastN);
    for (int q = w; q < nQ; q += 8) {
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
      if (i1 >= 0 && !nn_lines(v, i1, jend, sel, surf, c.nn_sq, g, &i2, &i3))
        scanline_group(surf ? L.lastS : L.lastC, jend, i1, sel, surf, c.nn_sq, g, &i2, &i3);
      const long long t1 = wall_clock64();
      if (g == 0) {
        qt[side * 512 + q] = t1 - t0 + (i1 + i2 + i3 == 12345678 ? 1 : 0);
        qb[side * 512 + q] = (int)(wp[w][P_NN_BRUTE] - b0);
        qt[1024 + side * 512 + q] = tm - t0 + (i1 == 12345678);
        qb[1024 + side * 512 + q] = win;
      }
    }
  }
}

int main() {
  FILE* f = fopen("build/nn_data.bin", "rb");
  if (!f) { printf("run scripts/mb/nn_data.py first\n"); return 1; }
  int np = 0;
  if (fread(&np, 4, 1, f) != 1) return 1;
  (void)hipFuncSetAttribute((const void*)knn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)odom_lds_bytes());
  long long* dqt; int* dqb;
  (void)hipMalloc(&dqt, 2048 * 8); (void)hipMalloc(&dqb, 2048 * 4);
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
    for (int rep = 0; rep < 2; ++rep)
      knn<<<1, 512, odom_lds_bytes()>>>(d[0], n[0], d[1], n[1], d[2], n[2], d[3], n[3], dqt, dqb);
    (void)hipDeviceSynchronize();
    std::vector<long long> qt(2048); std::vector<int> qb(2048);
    (void)hipMemcpy(qt.data(), dqt, 2048 * 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(qb.data(), dqb, 2048 * 4, hipMemcpyDeviceToHost);
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
