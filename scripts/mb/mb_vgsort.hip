// Microbenchmark of the per-ring VoxelGrid sort (k_extract's phase 3): the
// bitonic sort of unique (idx, t) keys that rounds 1-2 used, against the
// std::sort permutation of lego_vgsort.h (vg_block_sort).  One
// 256-thread workgroup per ring, G rings per launch; ring-shaped voxel keys
// (points around a wavy circle, 0.2 m voxels) and random keys with ties.  The
// output of vg_block_sort is checked against std::sort on the host.
//   ./build/mb_vgsort [n=1800] [G=1536]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

__device__ unsigned long long g_stamp[16];
__device__ unsigned long long g_levels;
#define VG_STAMP(k)                                                   \
  do {                                                                \
    if (blockIdx.x == 0 && threadIdx.x == 0) {                        \
      const unsigned long long now_ = clock64();                      \
      g_stamp[k] += now_ - t_prev_;                                   \
      t_prev_ = now_;                                                 \
      if ((k) == 6) ++g_levels;                                       \
    }                                                                 \
  } while (0)
__device__ unsigned long long t_prev_;
__device__ unsigned long long g_wst[16], g_wcnt[16];
#define VG_WSTAMP(k, t0)                                                         \
  do {                                                                           \
    if (blockIdx.x == 0 && (threadIdx.x & 63) == 0) {                            \
      atomicAdd(&g_wst[k], clock64() - (t0));                                    \
      atomicAdd(&g_wcnt[k], 1ull);                                               \
    }                                                                            \
  } while (0)
#define VG_CLOCK() clock64()
#include "lego_vgsort.h"
#include "lego_vgsort_wave.h"

using namespace lego;

__device__ __forceinline__ void bitonic_u64(unsigned long long* a, int m) {
  const int nw = blockDim.x >> 6, wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int C = m / nw;
  unsigned long long* w = a + wave * C;
  const int base = wave * C;
  for (int k = 2; k <= m; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      if (j >= C || C < 128) {
        __syncthreads();
        for (int t = threadIdx.x; t < m / 2; t += blockDim.x) {
          const int i = (t / j) * 2 * j + (t % j), l = i + j;
          const bool up = (i & k) == 0;
          const unsigned long long x = a[i], y = a[l];
          if ((x > y) == up) { a[i] = y; a[l] = x; }
        }
        __syncthreads();
      } else {
        for (int t = lane; t < C / 2; t += 64) {
          const int i = (t / j) * 2 * j + (t % j), l = i + j;
          const bool up = ((base + i) & k) == 0;
          const unsigned long long x = w[i], y = w[l];
          if ((x > y) == up) { w[i] = y; w[l] = x; }
        }
        vg_wave_sync();
      }
    }
  }
  __syncthreads();
}

__global__ void __launch_bounds__(256) k_bitonic(const uint32_t* keys, int n, uint32_t* out, uint16_t* outv) {
  __shared__ unsigned long long a[4096];
  const uint32_t* k = keys + (size_t)blockIdx.x * n;
  int m = 1;
  while (m < n) m <<= 1;
  for (int t = threadIdx.x; t < m; t += blockDim.x) a[t] = t < n ? ((unsigned long long)k[t] << 32) | t : ~0ull;
  __syncthreads();
  bitonic_u64(a, m);
  for (int t = threadIdx.x; t < n; t += blockDim.x) {
    out[(size_t)blockIdx.x * n + t] = (uint32_t)(a[t] >> 32);
    outv[(size_t)blockIdx.x * n + t] = (uint16_t)a[t];
  }
}

__global__ void __launch_bounds__(256) k_vgsort(const uint32_t* keys, int n, uint32_t* out, uint16_t* outv) {
  __shared__ uint32_t key[4096];
  __shared__ uint16_t val[4096];
  __shared__ __attribute__((aligned(16))) unsigned char sc[24 * 1024];
  const uint32_t* k = keys + (size_t)blockIdx.x * n;
  for (int t = threadIdx.x; t < n; t += blockDim.x) { key[t] = k[t]; val[t] = (uint16_t)t; }
  __syncthreads();
  if (blockIdx.x == 0 && threadIdx.x == 0) t_prev_ = clock64();
  vg_block_sort(vg_sort_carve(key, val, sc, n, (int)blockDim.x), n);
  for (int t = threadIdx.x; t < n; t += blockDim.x) {
    out[(size_t)blockIdx.x * n + t] = key[t];
    outv[(size_t)blockIdx.x * n + t] = val[t];
  }
}

// one ring per wave (n <= kVgWaveMax): four rings per workgroup, no barrier
__global__ void __launch_bounds__(256) k_vgsort_wave(const uint32_t* keys, int n, uint32_t* out, uint16_t* outv,
                                                     int G) {
  __shared__ uint32_t key[4][kVgWaveMax];
  __shared__ uint16_t val[4][kVgWaveMax];
  __shared__ uint32_t cw[4][kVgWaveMax];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int ring = blockIdx.x * 4 + wave;
  if (ring >= G) return;
  const uint32_t* k = keys + (size_t)ring * n;
  for (int t = lane; t < n; t += 64) { key[wave][t] = k[t]; val[wave][t] = (uint16_t)t; }
  vg_wave_sync();
  vg_wave_sort(key[wave], val[wave], cw[wave], n);
  for (int t = lane; t < n; t += 64) {
    out[(size_t)ring * n + t] = key[wave][t];
    outv[(size_t)ring * n + t] = val[wave][t];
  }
}

struct Idx {
  uint32_t idx;
  uint32_t t;
  bool operator<(const Idx& o) const { return idx < o.idx; }
};

__global__ void __launch_bounds__(256) k_vgsort_var(const uint32_t* keys, const int* off, uint32_t* out, uint16_t* outv,
                                                    int garbage) {
  __shared__ uint32_t key[4096];
  __shared__ uint16_t val[4096];
  __shared__ __attribute__((aligned(16))) unsigned char sc[24 * 1024];
  const int b0 = off[blockIdx.x], n = off[blockIdx.x + 1] - b0;
  if (garbage)
    for (int t = threadIdx.x; t < 24 * 1024 / 4; t += blockDim.x) ((uint32_t*)sc)[t] = 0xABCD1234u * (t + 1);
  for (int t = threadIdx.x; t < n; t += blockDim.x) { key[t] = keys[b0 + t]; val[t] = (uint16_t)t; }
  __syncthreads();
  vg_block_sort(vg_sort_carve(key, val, sc, n, (int)blockDim.x), n);
  for (int t = threadIdx.x; t < n; t += blockDim.x) { out[b0 + t] = key[t]; outv[b0 + t] = val[t]; }
}

// The mapping VoxelGrid's local sorts (k_vg_local / k_vg_local_small shape):
// one segment per workgroup of T threads, dynamic LDS for CAP keys, sumOrder,
// the segment's depth budget as given.
template <int CAP, int T>
__global__ void __launch_bounds__(T) k_vgsort_seg(const uint32_t* keys, const int* off, uint32_t* out, uint16_t* outv,
                                                  int depth, int* heap) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
  uint32_t* key = (uint32_t*)lds_raw;
  uint16_t* lv = (uint16_t*)(lds_raw + (size_t)CAP * 4);
  unsigned char* sc = lds_raw + (size_t)CAP * 6;
  const int b0 = off[blockIdx.x], n = off[blockIdx.x + 1] - b0;
  for (int t = threadIdx.x; t < n; t += T) { key[t] = keys[b0 + t]; lv[t] = (uint16_t)t; }
  __syncthreads();
  if (blockIdx.x == 0 && threadIdx.x == 0) t_prev_ = clock64();
  vg_block_sort(vg_sort_carve(key, lv, sc, n, T), n, depth, heap, true);
  for (int t = threadIdx.x; t < n; t += T) { out[b0 + t] = key[t]; outv[b0 + t] = lv[t]; }
}

// ./mb_vgsort seg <file> <depth> [one=0]: the segments of a file written by
// the C5 dump replay (deepest first), all at once (one per workgroup) and,
// with one = 1, the deepest alone; block 0's phase stamps.
static int run_seg(const char* path, int depth, int one) {
  FILE* f = fopen(path, "rb");
  if (!f) return 1;
  int R;
  if (fread(&R, 4, 1, f) != 1) return 1;
  std::vector<int> off{0};
  std::vector<uint32_t> keys;
  int nmax = 0;
  for (int r = 0; r < R; ++r) {
    int n;
    if (fread(&n, 4, 1, f) != 1) return 1;
    const size_t b = keys.size();
    keys.resize(b + n);
    if (fread(keys.data() + b, 4, n, f) != (size_t)n) return 1;
    off.push_back((int)keys.size());
    nmax = std::max(nmax, n);
  }
  fclose(f);
  uint32_t *dk, *dout;
  uint16_t* dv;
  int *doff, *dheap;
  hipMalloc(&dk, keys.size() * 4); hipMalloc(&dout, keys.size() * 4); hipMalloc(&dv, keys.size() * 2);
  hipMalloc(&doff, off.size() * 4); hipMalloc(&dheap, 4);
  hipMemcpy(dk, keys.data(), keys.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(doff, off.data(), off.size() * 4, hipMemcpyHostToDevice);
  const bool big = nmax > 1024;
  const size_t lds = big ? 8192 * 6 + vg_sort_scratch_bytes(8192, 1024) : 1024 * 6 + vg_sort_scratch_bytes(1024, 256);
  const int G = one ? 1 : R;
  auto launch = [&] {
    if (big) k_vgsort_seg<8192, 1024><<<G, 1024, lds>>>(dk, doff, dout, dv, depth, dheap);
    else k_vgsort_seg<1024, 256><<<G, 256, lds>>>(dk, doff, dout, dv, depth, dheap);
  };
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  launch();
  hipDeviceSynchronize();
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) launch();
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  unsigned long long z[16] = {}, zl = 0;
  hipMemcpyToSymbol(HIP_SYMBOL(g_stamp), z, sizeof(z));
  hipMemcpyToSymbol(HIP_SYMBOL(g_levels), &zl, sizeof(zl));
  launch();
  hipDeviceSynchronize();
  hipMemcpyFromSymbol(z, HIP_SYMBOL(g_stamp), sizeof(z));
  hipMemcpyFromSymbol(&zl, HIP_SYMBOL(g_levels), sizeof(zl));
  std::vector<uint32_t> hk(keys.size());
  hipMemcpy(hk.data(), dout, hk.size() * 4, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int r = 0; r < G; ++r)
    for (int i = off[r] + 1; i < off[r + 1]; ++i)
      if (hk[i] < hk[i - 1]) { ++bad; break; }
  printf("%s: %d segments (n max %d, %d threads), %d launched: %.1f us/launch, %d unsorted\n", path, R, nmax,
         big ? 1024 : 256, G, 1000 * ms / 5, bad);
  printf("  segment 0 (n=%d) phases (kcycles): median %.1f flags %.1f counts %.1f ranks %.1f swaps %.1f children %.1f "
         "sid %.1f | loop-exit %.1f leaves %.1f  levels %llu\n",
         off[1], z[0] / 1e3, z[1] / 1e3, z[2] / 1e3, z[3] / 1e3, z[4] / 1e3, z[5] / 1e3, z[6] / 1e3, z[7] / 1e3,
         z[8] / 1e3, zl);
  return 0;
}

static int run_file(const char* path, int reps) {
  FILE* f = fopen(path, "rb");
  if (!f) return 1;
  int R;
  if (fread(&R, 4, 1, f) != 1) return 1;
  std::vector<int> off{0};
  std::vector<uint32_t> keys;
  for (int r = 0; r < R; ++r) {
    int n;
    if (fread(&n, 4, 1, f) != 1) return 1;
    const size_t b = keys.size();
    keys.resize(b + n);
    if (fread(keys.data() + b, 4, n, f) != (size_t)n) return 1;
    off.push_back((int)keys.size());
  }
  fclose(f);
  uint32_t *dk, *dout;
  uint16_t* dv;
  int* doff;
  hipMalloc(&dk, keys.size() * 4); hipMalloc(&dout, keys.size() * 4); hipMalloc(&dv, keys.size() * 2);
  hipMalloc(&doff, off.size() * 4);
  hipMemcpy(dk, keys.data(), keys.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(doff, off.data(), off.size() * 4, hipMemcpyHostToDevice);
  for (int rep = 0; rep < reps; ++rep) {
    k_vgsort_var<<<R, 256>>>(dk, doff, dout, dv, rep & 1);
    std::vector<uint16_t> hv(keys.size());
    hipMemcpy(hv.data(), dv, hv.size() * 2, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int r = 0; r < R; ++r) {
      const int n = off[r + 1] - off[r];
      std::vector<Idx> a(n);
      for (int i = 0; i < n; ++i) a[i] = {keys[off[r] + i], (uint32_t)i};
      std::sort(a.begin(), a.end());
      for (int i = 0; i < n; ++i)
        if (a[i].t != hv[off[r] + i]) {
          if (rep == 0) printf("  ring %d (n=%d) differs at %d\n", r, n, i);
          ++bad;
          break;
        }
    }
    printf("file rep %d (garbage LDS %d): %d of %d rings differ\n", rep, rep & 1, bad, R);
  }
  return 0;
}

static int run_wave(int n, int G) {
  for (int shape = 0; shape < 4; ++shape) {
    std::vector<uint32_t> h((size_t)G * n);
    for (int g = 0; g < G; ++g) {
      uint64_t s = 88172645463325252ull + g;
      for (int i = 0; i < n; ++i) {
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        uint32_t key;
        if (shape == 3) {  // a whole ring (the main mode's shape 0)
          const double th = 2 * M_PI * i / n + 0.001 * g;
          const double r = 12 + 3 * std::sin(3 * th + g) + 0.05 * (double)(s % 100) / 100;
          const float x = (float)(r * std::cos(th)), y = (float)(r * std::sin(th)), z = -1.2f;
          key = (uint32_t)((int)(std::floor(x * 5.0f) + 80) + (int)(std::floor(y * 5.0f) + 80) * 161 +
                           (int)(std::floor(z * 5.0f) + 7) * 161 * 161);
        } else if (shape == 0) {  // a ring's arc, 0.2 m voxels, a few points per voxel
          const double th = 0.6 * M_PI * i / n + 0.01 * g;
          const double r = 8 + 2 * std::sin(3 * th + g) + 0.05 * (double)(s % 100) / 100;
          const float x = (float)(r * std::cos(th)), y = (float)(r * std::sin(th));
          key = (uint32_t)((int)(std::floor(x * 5.0f) + 80) + (int)(std::floor(y * 5.0f) + 80) * 161);
        } else if (shape == 1) {
          key = (uint32_t)(s % (uint64_t)(n / 2 + 1));
        } else {
          key = (uint32_t)(s % 100000u);
        }
        h[(size_t)g * n + i] = key;
      }
    }
    uint32_t *dk, *dout;
    uint16_t* dv;
    hipMalloc(&dk, h.size() * 4);
    hipMalloc(&dout, h.size() * 4);
    hipMalloc(&dv, h.size() * 2);
    hipMemcpy(dk, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto timeit = [&](const char* name, auto&& launch) {
      launch();
      hipDeviceSynchronize();
      hipEventRecord(e0);
      for (int r = 0; r < 5; ++r) launch();
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      printf("  %-22s %9.2f us/launch  %7.4f us/ring\n", name, 1000 * ms / 5, 1000 * ms / 5 / G);
    };
    printf("%s keys, n=%d, %d rings\n", shape == 0 ? "arc" : (shape == 1 ? "dup" : (shape == 2 ? "random" : "ring")), n,
           G);
    timeit("block (ring per WG)", [&] { k_vgsort<<<G, 256>>>(dk, n, dout, dv); });
    timeit("block, 128 threads", [&] { k_vgsort<<<G, 128>>>(dk, n, dout, dv); });
    if (n <= kVgWaveMax) timeit("wave (ring per wave)", [&] { k_vgsort_wave<<<(G + 3) / 4, 256>>>(dk, n, dout, dv, G); });
    std::vector<uint16_t> hv(h.size());
    hipMemcpy(hv.data(), dv, hv.size() * 2, hipMemcpyDeviceToHost);
    long bad = 0;
    for (int g = 0; g < G; ++g) {
      std::vector<Idx> a(n);
      for (int i = 0; i < n; ++i) a[i] = {h[(size_t)g * n + i], (uint32_t)i};
      std::sort(a.begin(), a.end());
      for (int i = 0; i < n; ++i)
        if (a[i].t != hv[(size_t)g * n + i]) { ++bad; break; }
    }
    printf("  wave sort vs std::sort: %ld of %d rings differ\n", bad, G);
    hipFree(dk); hipFree(dout); hipFree(dv);
  }
  return 0;
}

int main(int argc, char** argv) {
  if (argc > 2 && std::string(argv[1]) == "file") return run_file(argv[2], argc > 3 ? atoi(argv[3]) : 3);
  if (argc > 3 && std::string(argv[1]) == "seg") return run_seg(argv[2], atoi(argv[3]), argc > 4 ? atoi(argv[4]) : 0);
  if (argc > 3 && std::string(argv[1]) == "wave") return run_wave(atoi(argv[2]), atoi(argv[3]));
  const int n = argc > 1 ? atoi(argv[1]) : 1800;
  const int G = argc > 2 ? atoi(argv[2]) : 1536;
  const int shapes = argc > 3 ? atoi(argv[3]) : 2;
  for (int shape = 0; shape < shapes; ++shape) {
    std::vector<uint32_t> h((size_t)G * n);
    for (int g = 0; g < G; ++g) {
      uint64_t s = 88172645463325252ull + g;
      for (int i = 0; i < n; ++i) {
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        uint32_t key;
        if (shape >= 2) {  // rings of other radii / heights, partial arcs, 0.2 m voxels in a larger grid
          const double R0 = 3.0 + 4.0 * (shape - 2) + 0.7 * (g % 5);
          const double th = (0.3 + 1.7 * (g % 3) / 2.0) * M_PI * i / n + 0.01 * g;
          const double r = R0 * (1 + 0.2 * std::sin(5 * th + g)) + 0.02 * (double)(s % 100) / 100;
          const float x = (float)(r * std::cos(th)), y = (float)(r * std::sin(th)), z = (float)(-1.7 + 0.3 * std::sin(th * 7));
          const int i0 = (int)(std::floor(x * 5.0f) + 400), i1 = (int)(std::floor(y * 5.0f) + 400),
                    i2 = (int)(std::floor(z * 5.0f) + 20);
          key = (uint32_t)(i0 + i1 * 801 + i2 * 801 * 801);
        } else if (shape == 0) {  // a ring: points around a wavy circle, 0.2 m voxels
          const double th = 2 * M_PI * i / n + 0.001 * g;
          const double r = 12 + 3 * std::sin(3 * th + g) + 0.05 * (double)(s % 100) / 100;
          const float x = (float)(r * std::cos(th)), y = (float)(r * std::sin(th)), z = -1.2f;
          const int i0 = (int)(std::floor(x * 5.0f) + 80), i1 = (int)(std::floor(y * 5.0f) + 80),
                    i2 = (int)(std::floor(z * 5.0f) + 7);
          key = (uint32_t)(i0 + i1 * 161 + i2 * 161 * 161);
        } else {
          key = (uint32_t)(s % (uint64_t)(n / 2 + 1));
        }
        h[(size_t)g * n + i] = key;
      }
    }
    uint32_t *dk, *dout;
    uint16_t* dv;
    hipMalloc(&dk, h.size() * 4);
    hipMalloc(&dout, h.size() * 4);
    hipMalloc(&dv, h.size() * 2);
    hipMemcpy(dk, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto timeit = [&](const char* name, int G2, auto&& launch) {
      launch(G2);
      hipDeviceSynchronize();
      hipEventRecord(e0);
      const int reps = 5;
      for (int r = 0; r < reps; ++r) launch(G2);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      printf("  %-28s G=%5d  %9.2f us/launch  %7.3f us/ring\n", name, G2, 1000 * ms / reps, 1000 * ms / reps / G2);
    };
    printf("%s keys (shape %d), n=%d\n", shape == 0 ? "ring" : (shape == 1 ? "random" : "arc"), shape, n);
    for (int G2 : {1, G}) {
      timeit("bitonic (rounds 1-2)", G2, [&](int g) { k_bitonic<<<g, 256>>>(dk, n, dout, dv); });
      timeit("vg_block_sort", G2, [&](int g) { k_vgsort<<<g, 256>>>(dk, n, dout, dv); });
    }
    {
      unsigned long long z[16] = {}, zl = 0;
      hipMemcpyToSymbol(HIP_SYMBOL(g_stamp), z, sizeof(z));
      hipMemcpyToSymbol(HIP_SYMBOL(g_levels), &zl, sizeof(zl));
      hipMemcpyToSymbol(HIP_SYMBOL(g_wst), z, sizeof(z));
      hipMemcpyToSymbol(HIP_SYMBOL(g_wcnt), z, sizeof(z));
      k_vgsort<<<1, 256>>>(dk, n, dout, dv);
      hipDeviceSynchronize();
      hipMemcpyFromSymbol(z, HIP_SYMBOL(g_stamp), sizeof(z));
      hipMemcpyFromSymbol(&zl, HIP_SYMBOL(g_levels), sizeof(zl));
      unsigned long long ws[16], wc[16];
      hipMemcpyFromSymbol(ws, HIP_SYMBOL(g_wst), sizeof(ws));
      hipMemcpyFromSymbol(wc, HIP_SYMBOL(g_wcnt), sizeof(wc));
      printf("  wave sort (kcycles, calls): median %.1f/%llu flags %.1f/%llu pairing %.1f/%llu scatter %.1f/%llu swaps %.1f/%llu final %.1f/%llu\n",
             ws[9] / 1e3, wc[9], ws[10] / 1e3, wc[10], ws[11] / 1e3, wc[11], ws[12] / 1e3, wc[12], ws[13] / 1e3, wc[13], ws[14] / 1e3, wc[14]);
      printf("  ring 0 phases (kcycles): median %.1f flags %.1f counts %.1f ranks %.1f swaps %.1f children %.1f sid %.1f | loop-exit %.1f leaves %.1f  levels %llu\n",
             z[0] / 1e3, z[1] / 1e3, z[2] / 1e3, z[3] / 1e3, z[4] / 1e3, z[5] / 1e3, z[6] / 1e3, z[7] / 1e3, z[8] / 1e3, zl);
    }
    k_vgsort<<<G, 256>>>(dk, n, dout, dv);
    std::vector<uint16_t> hv(h.size());
    hipMemcpy(hv.data(), dv, hv.size() * 2, hipMemcpyDeviceToHost);
    long bad = 0;
    for (int g = 0; g < G; ++g) {
      std::vector<Idx> a(n);
      for (int i = 0; i < n; ++i) a[i] = {h[(size_t)g * n + i], (uint32_t)i};
      std::sort(a.begin(), a.end());
      for (int i = 0; i < n; ++i)
        if (a[i].t != hv[(size_t)g * n + i]) { ++bad; break; }
    }
    printf("  vg_block_sort vs std::sort: %ld of %d rings differ\n", bad, G);
    hipFree(dk); hipFree(dout); hipFree(dv);
  }
  return 0;
}
