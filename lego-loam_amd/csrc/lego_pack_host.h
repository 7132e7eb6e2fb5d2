// lego_pack_host.h — the node call's upload pass (lego_ip_process ->
// upload_checked, lego_api.hip) on a few host threads.  A VLS-128 cloud is
// 7.4 MB of caller records: one core reads and packs it at memory speed in
// ~0.2 ms while the copy engine waits; the pool's workers and the caller
// pack chunks side by side, and the caller queues each run of packed chunks'
// DMA as soon as it is complete, in order.
//
// Jobs never overlap (one context, one call at a time).  Chunks are claimed
// through one 64-bit word, generation | chunk count | next index, so a worker
// that wakes after its job has ended (or sees an old generation) claims
// nothing; a chunk is done when its flag holds the job's generation.
#pragma once
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "lego_loam.h"

namespace lego {

// Records [c0, c1) of src as (x, y, z, ring) words into dst[4 * i ..]; the
// non-finite flag of their xyz (an all-ones exponent is inf / nan).
inline uint32_t pack_points(const lego_point_xyzir* src, uint32_t* dst, int c0, int c1) {
  uint32_t nonfinite = 0;
  for (int i = c0; i < c1; ++i) {
    uint32_t u[3];
    std::memcpy(u, &src[i].x, sizeof(u));
    nonfinite |= (uint32_t)((u[0] & 0x7f800000u) == 0x7f800000u) | (uint32_t)((u[1] & 0x7f800000u) == 0x7f800000u) |
                 (uint32_t)((u[2] & 0x7f800000u) == 0x7f800000u);
    uint32_t* w = dst + (size_t)4 * i;
    w[0] = u[0];
    w[1] = u[1];
    w[2] = u[2];
    w[3] = (uint32_t)src[i].ring;
  }
  return nonfinite;
}

class PackPool {
 public:
  static constexpr int kChunk = 16384;  // points per chunk (256 KB packed)

  PackPool(int workers, int maxPoints)
      : maxChunks_((maxPoints + kChunk - 1) / kChunk + 1), done_(new std::atomic<uint32_t>[maxChunks_]) {
    for (int k = 0; k < maxChunks_; ++k) done_[k].store(0u, std::memory_order_relaxed);
    for (int i = 0; i < workers; ++i) th_.emplace_back([this] { loop(); });
  }
  ~PackPool() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  PackPool(const PackPool&) = delete;
  PackPool& operator=(const PackPool&) = delete;

  // Packs src[0, n) into dst; ready(c0, c1) is called by the caller, in
  // order, for every run of packed points [c0, c1).  Returns the non-finite
  // flag.  n <= the pool's maxPoints.
  template <class F>
  uint32_t run(const lego_point_xyzir* src, uint32_t* dst, int n, F&& ready) {
    const int nch = (n + kChunk - 1) / kChunk;
    uint32_t g;
    {
      std::lock_guard<std::mutex> lk(m_);
      src_ = src;
      dst_ = dst;
      n_ = n;
      g = ++gen_;
      if (g == 0) g = ++gen_;  // 0 marks "never done"
      nonfinite_.store(0u, std::memory_order_relaxed);
      next_.store(((uint64_t)g << 32) | ((uint64_t)nch << 16), std::memory_order_release);
    }
    cv_.notify_all();
    int issued = 0;
    while (issued < nch) {
      const int k = claim(g);
      if (k >= 0) finish(g, src, dst, n, k);
      int e = issued;
      while (e < nch && done_[e].load(std::memory_order_acquire) == g) ++e;
      if (e > issued) {
        ready(issued * kChunk, std::min(n, e * kChunk));
        issued = e;
      } else if (k < 0) {
        std::this_thread::yield();  // the workers hold the remaining chunks
      }
    }
    return nonfinite_.load(std::memory_order_acquire);
  }

 private:
  int claim(uint32_t g) {
    uint64_t v = next_.load(std::memory_order_acquire);
    for (;;) {
      if ((uint32_t)(v >> 32) != g) return -1;
      const int idx = (int)(v & 0xffffu), nch = (int)((v >> 16) & 0xffffu);
      if (idx >= nch) return -1;
      if (next_.compare_exchange_weak(v, v + 1, std::memory_order_acq_rel, std::memory_order_acquire)) return idx;
    }
  }
  void finish(uint32_t g, const lego_point_xyzir* src, uint32_t* dst, int n, int k) {
    const uint32_t f = pack_points(src, dst, k * kChunk, std::min(n, (k + 1) * kChunk));
    if (f) nonfinite_.fetch_or(f, std::memory_order_relaxed);
    done_[k].store(g, std::memory_order_release);
  }
  void loop() {
    uint32_t seen = 0;
    for (;;) {
      const lego_point_xyzir* src;
      uint32_t* dst;
      int n;
      uint32_t g;
      {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = g = gen_;
        src = src_;
        dst = dst_;
        n = n_;
      }
      for (int k; (k = claim(g)) >= 0;) finish(g, src, dst, n, k);
    }
  }

  const int maxChunks_;
  std::unique_ptr<std::atomic<uint32_t>[]> done_;
  std::vector<std::thread> th_;
  std::mutex m_;
  std::condition_variable cv_;
  bool stop_ = false;
  uint32_t gen_ = 0;
  const lego_point_xyzir* src_ = nullptr;
  uint32_t* dst_ = nullptr;
  int n_ = 0;
  std::atomic<uint64_t> next_{0};
  std::atomic<uint32_t> nonfinite_{0};
};

}  // namespace lego
