// Microbenchmark of the heap-sort fallback of the VoxelGrid sorts
// (lego_vgsort.h: std::__partial_sort by one wave, vg_heap_sort_wave): one
// 64-thread workgroup per piece, the piece in LDS, clock64 around the call;
// keys with ~14 repeats per value, as VLS-128's dense rings leave them
// (DESIGN §4a).  Every output permutation is checked against the one-lane
// VgHeap::sort of the same piece.  Prints cycles per pop.
//   ./build/mb_heap [n=700] [pieces=256] [distinct=50]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "lego_vgsort.h"
#ifdef MB_HEAP_CANDIDATE
#include MB_HEAP_CANDIDATE
#endif

using namespace lego;

#define CK(x)                                                                                  \
  do {                                                                                         \
    hipError_t e = (x);                                                                        \
    if (e != hipSuccess) {                                                                     \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));            \
      std::exit(1);                                                                            \
    }                                                                                          \
  } while (0)

constexpr int kMaxN = 4096;

// form 0: one lane (VgHeap), 1: vg_heap_sort_wave, 2: the candidate (if built)
template <int F>
__global__ void __launch_bounds__(64) k_heap(const uint32_t* keys, int n, uint32_t* perm, unsigned long long* cyc) {
  __shared__ uint32_t K[kMaxN], W[kMaxN];
  const uint32_t* src = keys + (size_t)blockIdx.x * n;
  for (int i = threadIdx.x; i < n; i += 64) {
    K[i] = src[i];
    W[i] = (uint32_t)i;
  }
  __syncthreads();
  const unsigned long long t0 = clock64();
  if constexpr (F == 0) {
    if (threadIdx.x == 0) VgHeap<uint32_t>{K, W}.sort(0, n);
  } else if constexpr (F == 1) {
    vg_heap_sort_wave(K, W, 0, n);
  } else {
#ifdef MB_HEAP_CANDIDATE
    mb_heap_candidate(K, W, 0, n);
#endif
  }
  __syncthreads();
  const unsigned long long t1 = clock64();
  for (int i = threadIdx.x; i < n; i += 64) perm[(size_t)blockIdx.x * n + i] = W[i];
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? std::atoi(argv[1]) : 700;
  const int G = argc > 2 ? std::atoi(argv[2]) : 256;
  const int D = argc > 3 ? std::atoi(argv[3]) : 50;
  if (n < 2 || n > kMaxN) return 1;
  std::vector<uint32_t> keys((size_t)n * G);
  unsigned s = 12345u;
  for (auto& k : keys) {
    s = s * 1664525u + 1013904223u;
    k = (s >> 8) % (unsigned)D * 7919u;
  }
  uint32_t *dk, *dp;
  unsigned long long* dc;
  CK(hipMalloc(&dk, keys.size() * 4));
  CK(hipMalloc(&dp, keys.size() * 4));
  CK(hipMalloc(&dc, G * 8));
  CK(hipMemcpy(dk, keys.data(), keys.size() * 4, hipMemcpyHostToDevice));
  std::vector<uint32_t> ref(keys.size()), got(keys.size());
  std::vector<unsigned long long> cyc(G);
  auto run = [&](auto kern, const char* name, std::vector<uint32_t>& out) {
    double best = 1e30;
    for (int r = 0; r < 3; ++r) {
      kern<<<G, 64>>>(dk, n, dp, dc);
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(cyc.data(), dc, G * 8, hipMemcpyDeviceToHost));
      double m = 0;
      for (auto c : cyc) m += (double)c;
      best = std::min(best, m / G);
    }
    CK(hipMemcpy(out.data(), dp, out.size() * 4, hipMemcpyDeviceToHost));
    std::printf("%-10s n %d: %10.0f cycles per piece, %7.1f per pop\n", name, n, best, best / (n - 1));
  };
  run(k_heap<0>, "one-lane", ref);
  run(k_heap<1>, "wave", got);
  size_t bad = 0;
  for (size_t i = 0; i < ref.size(); ++i) bad += ref[i] != got[i];
  std::printf("wave vs one-lane: %zu mismatches\n", bad);
#ifdef MB_HEAP_CANDIDATE
  run(k_heap<2>, "candidate", got);
  bad = 0;
  for (size_t i = 0; i < ref.size(); ++i) bad += ref[i] != got[i];
  std::printf("candidate vs one-lane: %zu mismatches\n", bad);
#endif
  return bad != 0;
}
