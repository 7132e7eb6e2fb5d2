// Does a hipGraph with two independent branches run them concurrently, and
// what does a captured chain of short dependent kernels cost against the
// same chain launched eagerly?  (C5 mapping step: three VoxelGrid chains on
// three streams, ~250 launches.)  Prints microseconds.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void spin(long long cycles, int* sink) {
  const long long t0 = clock64();
  while (clock64() - t0 < cycles) {}
  if (threadIdx.x == 0 && blockIdx.x == 0) atomicAdd(sink, 1);
}
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

int main() {
  int* sink;
  CK(hipMalloc(&sink, 4));
  hipStream_t s0, s1, s2;
  CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t f, j1, j2, a, b;
  CK(hipEventCreateWithFlags(&f, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&j1, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&j2, hipEventDisableTiming));
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const long long LONG = 200000;  // ~100 us at ~2 GHz
  const int NCHAIN = 60;          // short kernels per chain
  auto enqueue = [&](bool shortk) {
    (void)hipEventRecord(f, s0);
    (void)hipStreamWaitEvent(s1, f, 0);
    (void)hipStreamWaitEvent(s2, f, 0);
    for (hipStream_t st : {s0, s1, s2}) {
      if (shortk) for (int i = 0; i < NCHAIN; ++i) spin<<<64, 64, 0, st>>>(2000, sink);
      else spin<<<1, 64, 0, st>>>(LONG, sink);
    }
    (void)hipEventRecord(j1, s1);
    (void)hipEventRecord(j2, s2);
    (void)hipStreamWaitEvent(s0, j1, 0);
    (void)hipStreamWaitEvent(s0, j2, 0);
  };
  for (int shortk = 0; shortk < 2; ++shortk) {
    // eager
    for (int w = 0; w < 3; ++w) enqueue(shortk);
    CK(hipStreamSynchronize(s0));
    float ms = 0;
    CK(hipEventRecord(a, s0));
    for (int r = 0; r < 20; ++r) enqueue(shortk);
    CK(hipEventRecord(b, s0));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms, a, b));
    printf("%s eager: %.1f us per step\n", shortk ? "3 chains x 60 short kernels" : "3 x 100us kernels", ms * 1e3 / 20);
    // graph
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s0, hipStreamCaptureModeGlobal));
    enqueue(shortk);
    CK(hipStreamEndCapture(s0, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int w = 0; w < 3; ++w) CK(hipGraphLaunch(ge, s0));
    CK(hipStreamSynchronize(s0));
    CK(hipEventRecord(a, s0));
    for (int r = 0; r < 20; ++r) CK(hipGraphLaunch(ge, s0));
    CK(hipEventRecord(b, s0));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms, a, b));
    printf("%s graph: %.1f us per step\n", shortk ? "3 chains x 60 short kernels" : "3 x 100us kernels", ms * 1e3 / 20);
    // single chain (one stream) for reference
    CK(hipStreamSynchronize(s0));
    CK(hipEventRecord(a, s0));
    for (int r = 0; r < 20; ++r) {
      if (shortk) for (int i = 0; i < NCHAIN; ++i) spin<<<64, 64, 0, s0>>>(2000, sink);
      else spin<<<1, 64, 0, s0>>>(LONG, sink);
    }
    CK(hipEventRecord(b, s0));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms, a, b));
    printf("%s one chain eager: %.1f us per step\n", shortk ? "60 short kernels" : "1 x 100us kernel", ms * 1e3 / 20);
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
  }
  return 0;
}
