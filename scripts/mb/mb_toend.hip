// microbenchmark: the odometry hand-off (TransformToEnd of the less-flat and
// less-sharp clouds on waves 1-7, stores, counting into the next index) with
// pieces switched off, to see which part its ~8 us per scan goes to.
#include "../../lego-loam_amd/csrc/lego_odom.hip"
using namespace lego;
// MODE bits: 1 = to_end, 2 = global stores, 4 = build_count, 8 = bucket
// atomics only (64-bit hash), 16 = bucket atomics only (24-bit multiply hash)
__device__ __forceinline__ int bucket24(int ix, int iy, int iz, int T) {
  return (int)(((unsigned)__mul24(ix, 0x9E3779) ^ (unsigned)__mul24(iy, 0x85EBCB) ^ (unsigned)__mul24(iz, 0xC2B2AE)) & (unsigned)(T - 1));
}
template <int MODE>
__global__ void __launch_bounds__(512) kend(const float4* lf, const float4* ls, float4* gS, float4* gC, float4* sE,
                                            float4* cE, long long* t, int reps, int nLF, int nLS) {
  __shared__ float4 lastS[4096], lastC[2048];
  __shared__ unsigned cnt[kLdsCnt];
  __shared__ int kfirst[2 * kKeyTab], klast[2 * kKeyTab], irr[2];
  const int tid = threadIdx.x;
  float tcur[6] = {0.01f, 0.02f, -0.015f, 0.1f, 0.05f, 0.2f};
  const ImuEnd im{1.f, 1.f, 1.f, 0.f, 0.f, 0.f, 1.f, 0.f, 1.f, 0.f, 1.f, 0.f};
  NNStore<uint16_t> nsS{nullptr, nullptr, nullptr, nullptr, nullptr, &irr[0], kLdsGridS};
  NNStore<uint16_t> nsC{nullptr, nullptr, nullptr, nullptr, nullptr, &irr[1], kLdsGridC};
  long long t0 = 0;
  for (int r = 0; r < reps; ++r) {
    tcur[0] += 1e-6f;
    const EndTrig et = end_trig(tcur);
    const BuildArgs<uint16_t> B = build_args<uint16_t>(lastS, nLF, nsS, lastC, nLS, nsC, 16, cnt, nullptr, kfirst,
                                                       klast);
    build_zero(B);
    __syncthreads();
    if (r == 1) t0 = wall_clock64();
    const int t0i = tid - 64, tstep = 448;
    if (t0i >= 0) {
      const int nS = nLF, n = nLF + nLS, lane = tid & 63;
      for (int i0 = t0i - lane; i0 < n; i0 += tstep) {
        const int i = i0 + lane;
        float4 p = make_float4(0.f, 0.f, 0.f, 0.f);
        if (i < nS) {
          p = (MODE & 1) ? to_end(lf[i], tcur, et, im, false) : lf[i];
          if (MODE & 2) { gS[i] = p; sE[i] = p; }
          lastS[i] = p;
        } else if (i < n) {
          const int j = i - nS;
          p = (MODE & 1) ? to_end(ls[j], tcur, et, im, false) : ls[j];
          if (MODE & 2) { gC[j] = p; cE[j] = p; }
          lastC[j] = p;
        }
        if (MODE & 4) {
          auto w_at = [&](int j) { return j < nS ? lf[j].w : ls[j - nS].w; };
          int kp = 0, kn = 0;
          if (i < n) nbr_keys(i, nS, n, w_at(max(i - 1, 0)), w_at(min(i + 1, n - 1)), kp, kn);
          build_count(B, i0, p, kp, kn);
        }
        if ((MODE & 24) && i < n) {
          const bool corner = i >= nS;
          const int T = corner ? B.TC : B.TS;
          const int ix = cell_of(p.x), iy = cell_of(p.y), iz = cell_of(p.z);
          atomicAdd(&cnt[(corner ? B.TS : 0) + ((MODE & 8) ? fine_bucket(ix, iy, iz, T) : bucket24(ix, iy, iz, T))], 1u);
        }
      }
    }
    __syncthreads();
  }
  const long long t1 = wall_clock64();
  if (tid == 0) *t = t1 - t0;
  if (tid == 0) gS[0].w += (float)cnt[5] + lastS[7].x + lastC[3].y;
}
int main() {
  const int nLF = 3480, nLS = 270;
  static float4 hf[4096], hs[2048];
  srand(1);
  auto R = [] { return (float)rand() / RAND_MAX * 20.f - 10.f; };
  // points in ring order, relative time growing along the ring (as the extraction emits them)
  for (int i = 0; i < nLF; ++i) {
    const int ring = i * 16 / nLF;
    hf[i] = make_float4(R(), R(), R() * 0.2f, ring + 0.0999f * (float)(i % (nLF / 16)) / (nLF / 16));
  }
  for (int i = 0; i < nLS; ++i) {
    const int ring = i * 16 / nLS;
    hs[i] = make_float4(R(), R(), R() * 0.2f, ring + 0.0999f * (float)(i % (nLS / 16)) / (nLS / 16));
  }
  float4 *df, *ds, *gS, *gC, *sE, *cE;
  long long* t;
  (void)hipMalloc(&df, sizeof hf); (void)hipMalloc(&ds, sizeof hs);
  (void)hipMalloc(&gS, sizeof hf); (void)hipMalloc(&gC, sizeof hs);
  (void)hipMalloc(&sE, sizeof hf); (void)hipMalloc(&cE, sizeof hs);
  (void)hipMalloc(&t, 8);
  (void)hipMemcpy(df, hf, sizeof hf, hipMemcpyHostToDevice);
  (void)hipMemcpy(ds, hs, sizeof hs, hipMemcpyHostToDevice);
  const int modes[] = {0, 1, 4, 8, 16, 5, 7};
  const char* nm[] = {"loads + LDS only", "to_end", "count", "bucket atomics", "bucket atomics mul24", "to_end+count",
                      "full hand-off"};
  for (int m = 0; m < 7; ++m) {
    long long ht = 0;
    const int reps = 201;
    for (int rep = 0; rep < 2; ++rep) {
      switch (modes[m]) {
#define L_(M) case M: kend<M><<<1, 512>>>(df, ds, gS, gC, sE, cE, t, reps, nLF, nLS); break;
        L_(0) L_(1) L_(4) L_(8) L_(16) L_(5) L_(7)
      }
      (void)hipDeviceSynchronize();
      (void)hipMemcpy(&ht, t, 8, hipMemcpyDeviceToHost);
    }
    printf("%-22s: %.3f us per hand-off (%d + %d points, 7 waves)\n", nm[m], ht / 100.0 / (reps - 1), nLF, nLS);
  }
  return 0;
}
