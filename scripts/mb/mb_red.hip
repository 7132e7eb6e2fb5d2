#include <hip/hip_runtime.h>
#include <cstdio>
template <int kCtrl>
__device__ __forceinline__ double dpp_f64(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp((int)b, kCtrl, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), kCtrl, 0xf, 0xf, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double rdlane_f64(double v, int l) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)b, l), hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double wave_sum_f64(double v) {
  v += dpp_f64<0xB1>(v); v += dpp_f64<0x4E>(v); v += dpp_f64<0x141>(v); v += dpp_f64<0x140>(v);
  return (rdlane_f64(v, 0) + rdlane_f64(v, 16)) + (rdlane_f64(v, 32) + rdlane_f64(v, 48));
}
__device__ __forceinline__ void block_sum9(double v[9], int m, double* red, double out[9], int* mt, int nQ) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  double r[10];
  if (wave * 64 < nQ) {
    for (int k = 0; k < 9; ++k) r[k] = wave_sum_f64(v[k]);
    r[9] = wave_sum_f64((double)m);
  } else for (int k = 0; k < 10; ++k) r[k] = 0.0;
  if (lane == 0) for (int k = 0; k < 10; ++k) red[wave * 10 + k] = r[k];
  __syncthreads();
  double sum = 0;
  if (lane < 10) for (int w = 0; w < 8; ++w) sum += red[w * 10 + lane];
  for (int k = 0; k < 9; ++k) out[k] = rdlane_f64(sum, k);
  *mt = (int)rdlane_f64(sum, 9);
}

// v2: row sums by DPP (4 steps), row leaders to LDS, lanes (row + 4k) sum the
// waves in order, quad DPP adds the 4 rows, 10 readlanes
__device__ __forceinline__ double row_sum_f64(double v) {
  v += dpp_f64<0xB1>(v); v += dpp_f64<0x4E>(v); v += dpp_f64<0x141>(v); v += dpp_f64<0x140>(v);
  return v;
}
__device__ __forceinline__ void block_sum9_v2(double v[9], int m, double* red, double out[9], int* mt, int nQ) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nw = (nQ + 63) >> 6;
  if (wave < nw) {
    double r[10];
    for (int k = 0; k < 9; ++k) r[k] = row_sum_f64(v[k]);
    r[9] = row_sum_f64((double)m);
    if ((lane & 15) == 0) {
      const int row = lane >> 4;
      for (int k = 0; k < 10; ++k) red[(wave * 4 + row) * 10 + k] = r[k];
    }
  }
  __syncthreads();
  double s = 0;
  if (lane < 40) {
    const int row = lane & 3, k = lane >> 2;
    for (int w = 0; w < nw; ++w) s += red[(w * 4 + row) * 10 + k];
  }
  s += dpp_f64<0xB1>(s);
  s += dpp_f64<0x4E>(s);
  for (int k = 0; k < 9; ++k) out[k] = rdlane_f64(s, 4 * k);
  *mt = (int)rdlane_f64(s, 36);
}
__global__ void __launch_bounds__(512) k(double* o, long long* t, int iters, int mode, int nQ) {
  __shared__ double red[2][320];
  double v[9];
  for (int k = 0; k < 9; ++k) v[k] = threadIdx.x * 0.001 + k;
  double acc = 0;
  long long t0 = wall_clock64();
  for (int it = 0; it < iters; ++it) {
    double out[9]; int mt;
    if (mode == 0) block_sum9(v, 1, red[it & 1], out, &mt, nQ);
    else if (mode == 1) { __syncthreads(); out[0] = v[0]; mt = 1; }
    else if (mode == 3) block_sum9_v2(v, 1, red[it & 1], out, &mt, nQ);
    else { for (int k = 0; k < 9; ++k) out[k] = wave_sum_f64(v[k]); mt = 1; }
    acc += out[0] + mt;
    v[0] += out[1] * 1e-30;
  }
  long long t1 = wall_clock64();
  if (threadIdx.x == 0) { *o = acc; *t = t1 - t0; }
}
int main() {
  double* o; long long* t; hipMalloc(&o, 8); hipMalloc(&t, 8);
  const char* nm[4] = {"block_sum9", "barrier only", "wave DPP x9 only", "block_sum9_v2"};
  for (int mode = 0; mode < 4; ++mode) for (int nQ : {192, 512}) {
    const int iters = 10000;
    k<<<1, 512>>>(o, t, iters, mode, nQ); hipDeviceSynchronize();
    k<<<1, 512>>>(o, t, iters, mode, nQ); long long ht; hipMemcpy(&ht, t, 8, hipMemcpyDeviceToHost);
    printf("%-18s nQ=%3d: %.3f us per call\n", nm[mode], nQ, ht / 100.0 / iters);
  }
  return 0;
}
