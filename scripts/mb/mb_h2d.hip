// Host -> device copy of one scan's points from a pageable caller buffer
// (the node API's lego_ip_process input), four ways:
//   pageable   hipMemcpyAsync straight from the pageable buffer (the runtime's
//              staged copy; what stage_inputs does)
//   register   hipHostRegister of the caller's buffer, one DMA, unregister
//   pin1       memcpy into a pinned staging buffer, then one DMA
//   pinT/C     T threads memcpy chunks of C bytes into pinned staging, each
//              chunk's DMA issued as soon as it is copied (copy/DMA overlap)
// Sizes: VLP-16 (28.8k points x 32 B) and VLS-128 (230k x 32 B).  Median of
// 50 after 5 warm-ups, host wall clock to the end of the last DMA.  Diagnostic.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e = (x);                                                     \
    if (e != hipSuccess) {                                                  \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      std::exit(1);                                                         \
    }                                                                       \
  } while (0)

using clk = std::chrono::steady_clock;

static double median(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main() {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const size_t sizes[2] = {28800ull * 32, 230400ull * 32};
  const size_t cap = sizes[1];
  char* src = (char*)std::malloc(cap);
  for (size_t i = 0; i < cap; ++i) src[i] = (char)(i * 131u);
  char *pin, *dev;
  CK(hipHostMalloc((void**)&pin, cap, hipHostMallocDefault));
  CK(hipMalloc((void**)&dev, cap));
  for (size_t bytes : sizes) {
    auto run = [&](const char* name, auto&& body) {
      std::vector<double> t;
      for (int r = 0; r < 55; ++r) {
        // evict the source from the caches between runs? The caller's buffer
        // was just written by its producer: keep it warm, as in the node call.
        const auto a = clk::now();
        body();
        CK(hipStreamSynchronize(s));
        const auto b = clk::now();
        if (r >= 5) t.push_back(std::chrono::duration<double, std::micro>(b - a).count());
      }
      std::printf("%8zu B  %-14s median %8.1f us  (%.1f GB/s)\n", bytes, name, median(t),
                  bytes / median(t) / 1e3);
    };
    run("pageable", [&] { CK(hipMemcpyAsync(dev, src, bytes, hipMemcpyHostToDevice, s)); });
    run("register", [&] {  // pin the caller's buffer for the one copy
      CK(hipHostRegister(src, bytes, hipHostRegisterDefault));
      CK(hipMemcpyAsync(dev, src, bytes, hipMemcpyHostToDevice, s));
      CK(hipStreamSynchronize(s));
      CK(hipHostUnregister(src));
    });
    run("pin1", [&] {
      std::memcpy(pin, src, bytes);
      CK(hipMemcpyAsync(dev, pin, bytes, hipMemcpyHostToDevice, s));
    });
    for (int T : {2, 4, 8}) {
      for (size_t C : {size_t(256) << 10, size_t(1) << 20}) {
        char name[32];
        std::snprintf(name, sizeof name, "pin%d/%zuK", T, C >> 10);
        run(name, [&] {
          const size_t nc = (bytes + C - 1) / C;
          std::atomic<size_t> next{0};
          std::vector<std::atomic<int>> done(nc);
          for (auto& d : done) d.store(0);
          auto worker = [&] {
            for (size_t k; (k = next.fetch_add(1)) < nc;) {
              const size_t o = k * C, n = std::min(C, bytes - o);
              std::memcpy(pin + o, src + o, n);
              done[k].store(1, std::memory_order_release);
            }
          };
          std::vector<std::thread> th;
          for (int i = 1; i < T; ++i) th.emplace_back(worker);
          worker();
          for (size_t k = 0; k < nc; ++k) {  // DMAs in chunk order as the chunks land
            while (!done[k].load(std::memory_order_acquire)) {
            }
            const size_t o = k * C, n = std::min(C, bytes - o);
            CK(hipMemcpyAsync(dev + o, pin + o, n, hipMemcpyHostToDevice, s));
          }
          for (auto& x : th) x.join();
        });
      }
    }
  }
  CK(hipFree(dev));
  CK(hipHostFree(pin));
  std::free(src);
  return 0;
}
