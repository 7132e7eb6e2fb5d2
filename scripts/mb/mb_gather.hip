// Calibration of FETCH_SIZE for k_pixels' access pattern:
// 100 VLP-16-shaped scans of 32-B XYZIR records (28,800 per scan, firing order
// = column-major, ring inner, as lego_synth emits).  Three kernels with known
// useful bytes, run under `rocprofv3 --pmc FETCH_SIZE`:
//   k_stream  every record's first 16 B, coalesced in storage order
//             (the guide's calibrated case: FETCH_SIZE = half the bytes);
//   k_gather  the first 16 B of every record in pixel (row-major) order, the
//             k_pixels gather: consecutive lanes 16 records = 512 B apart;
//   k_owner   4-B coalesced loads of an int array of the same pixel count
//             (k_pixels' owner read).
// Each kernel writes one float per thread to a sink so nothing is elided.
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kScans = 100, kRings = 16, kCols = 1800, kP = kRings * kCols;

__global__ void k_stream(const float4* rec2, float* sink) {  // rec2: 2 float4 per record
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (size_t)kScans * kP) return;
  const float4 v = rec2[2 * i];
  sink[i] = v.x + v.y + v.z;
}
__global__ void k_gather(const float4* rec2, float* sink) {
  const size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= (size_t)kScans * kP) return;
  const size_t b = g / kP, p = g % kP;
  const size_t row = p / kCols, col = p % kCols;
  const size_t o = b * kP + col * kRings + row;  // firing order
  const float4 v = rec2[2 * o];
  sink[g] = v.x + v.y + v.z;
}
__global__ void k_owner(const int* own, float* sink) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (size_t)kScans * kP) return;
  sink[i] = (float)own[i];
}

int main() {
  const size_t n = (size_t)kScans * kP;
  float4* rec = nullptr;
  int* own = nullptr;
  float* sink = nullptr;
  if (hipMalloc(&rec, n * 32) != hipSuccess || hipMalloc(&own, n * 4) != hipSuccess ||
      hipMalloc(&sink, n * 4) != hipSuccess)
    return 1;
  (void)hipMemset(rec, 0, n * 32);
  (void)hipMemset(own, 0, n * 4);
  // a 512 MB scrub between runs so nothing is served from the 256 MB Infinity Cache
  void* scrub = nullptr;
  if (hipMalloc(&scrub, 512u << 20) != hipSuccess) return 1;
  const int blocks = (int)((n + 255) / 256);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const char* names[3] = {"k_stream", "k_gather", "k_owner"};
  const double useful[3] = {16.0 * n, 16.0 * n, 4.0 * n};
  for (int k = 0; k < 3; ++k)
    for (int rep = 0; rep < 3; ++rep) {
      (void)hipMemset(scrub, rep, 512u << 20);
      (void)hipEventRecord(a);
      if (k == 0) k_stream<<<blocks, 256>>>(rec, sink);
      if (k == 1) k_gather<<<blocks, 256>>>(rec, sink);
      if (k == 2) k_owner<<<blocks, 256>>>(own, sink);
      (void)hipEventRecord(b);
      (void)hipEventSynchronize(b);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, a, b);
      printf("%s rep %d: %.3f ms, useful %.1f MB, %.0f GB/s useful\n", names[k], rep, ms, useful[k] / 1e6,
             useful[k] / (ms * 1e-3) / 1e9);
    }
  return 0;
}
