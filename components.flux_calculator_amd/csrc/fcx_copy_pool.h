// fcx_copy_pool.h -- host memcpy batches spread over a process-wide pool of worker threads
// (the staging arena's gather and scatter, fcx_engine.hip).  Header-only so that the CPU test
// (tests/cpp/copy_pool_stress.cpp) exercises the same code.
#pragma once
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>
#if defined(__x86_64__)
#include <emmintrin.h>
#endif

namespace fcx {

inline void cpu_relax() {
#if defined(__x86_64__) || defined(__i386__)
  __builtin_ia32_pause();
#else
  std::this_thread::yield();
#endif
}

// memcpy with non-temporal stores (x86-64: 16-B streaming stores once the destination is
// aligned): the destination is not read back by this CPU soon (the arena is read by the DMA
// engine, the caller's arrays by the host program later), so the stores skip the
// read-for-ownership of every line and leave the caches alone
inline void copy_nt(char *dst, const char *src, size_t n) {
#if defined(__x86_64__)
  const size_t head = std::min(n, (size_t)((16 - (reinterpret_cast<uintptr_t>(dst) & 15)) & 15));
  std::memcpy(dst, src, head);
  dst += head;
  src += head;
  n -= head;
  size_t i = 0;
  for (; i + 64 <= n; i += 64) {
    const __m128i a = _mm_loadu_si128(reinterpret_cast<const __m128i *>(src + i));
    const __m128i b = _mm_loadu_si128(reinterpret_cast<const __m128i *>(src + i + 16));
    const __m128i c = _mm_loadu_si128(reinterpret_cast<const __m128i *>(src + i + 32));
    const __m128i d = _mm_loadu_si128(reinterpret_cast<const __m128i *>(src + i + 48));
    _mm_stream_si128(reinterpret_cast<__m128i *>(dst + i), a);
    _mm_stream_si128(reinterpret_cast<__m128i *>(dst + i + 16), b);
    _mm_stream_si128(reinterpret_cast<__m128i *>(dst + i + 32), c);
    _mm_stream_si128(reinterpret_cast<__m128i *>(dst + i + 48), d);
  }
  std::memcpy(dst + i, src + i, n - i);
  _mm_sfence();  // the streamed lines are globally visible before the batch is reported done
#else
  std::memcpy(dst, src, n);
#endif
}

// Host copies of the staging arena (gather of the caller's arrays into it, scatter out of
// it), spread over a process-wide pool of worker threads.  The calling thread takes part;
// workers spin ~100 us after a batch before sleeping, so the scatter that follows a step's
// gather finds them awake.  One batch at a time (engines on several host threads queue).
struct CopyJob {
  char *dst;
  const char *src;
  size_t bytes;
};

class CopyPool {
 public:
  static CopyPool &get() {
    static CopyPool *p = new CopyPool();  // never destroyed: workers may outlive static dtors
    return *p;
  }
  // every job done when this returns; `threads` counts the caller; nt: non-temporal stores
  void run(const std::vector<CopyJob> &jobs, int threads, bool nt = false) {
    if (jobs.empty()) return;
    std::lock_guard<std::mutex> one(batch_mu_);
    const int helpers = std::max(0, std::min<int>({threads - 1, (int)jobs.size() - 1, 63}));
    if (helpers == 0) {
      for (const auto &j : jobs) nt ? copy_nt(j.dst, j.src, j.bytes) : (void)std::memcpy(j.dst, j.src, j.bytes);
      return;
    }
    nt_ = nt;
    grow(helpers);
    jobs_ = jobs.data();
    njobs_ = jobs.size();
    next_.store(0, std::memory_order_relaxed);
    busy_.store(helpers, std::memory_order_relaxed);
    // one word: batch counter and the number of helpers, so a worker reads both at once
    count_ += 1;
    gen_.store((count_ << 8) | (uint64_t)helpers, std::memory_order_seq_cst);
    if (sleepers_.load(std::memory_order_seq_cst) > 0) {
      std::lock_guard<std::mutex> lk(mu_);
      cv_.notify_all();
    }
    work();
    while (busy_.load(std::memory_order_acquire) > 0) cpu_relax();
    jobs_ = nullptr;
  }

 private:
  void work() {
    for (size_t i; (i = next_.fetch_add(1, std::memory_order_relaxed)) < njobs_;) {
      if (nt_)
        copy_nt(jobs_[i].dst, jobs_[i].src, jobs_[i].bytes);
      else
        std::memcpy(jobs_[i].dst, jobs_[i].src, jobs_[i].bytes);
    }
  }
  // new workers start from the generation before the batch about to be published, so a
  // worker created for a batch always takes part in it
  void grow(int n) {
    const uint64_t before = gen_.load(std::memory_order_relaxed);
    while ((int)workers_.size() < n) {
      const int id = (int)workers_.size();
      workers_.emplace_back([this, id, before] { loop(id, before); });
      workers_.back().detach();
    }
  }
  void loop(int id, uint64_t seen) {
    for (;;) {
      // spin for a while, then sleep until the next batch
      auto t0 = std::chrono::steady_clock::now();
      uint64_t g;
      while ((g = gen_.load(std::memory_order_acquire)) == seen) {
        cpu_relax();
        if (std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(100)) {
          std::unique_lock<std::mutex> lk(mu_);
          sleepers_.fetch_add(1, std::memory_order_seq_cst);
          cv_.wait(lk, [&] { return gen_.load(std::memory_order_seq_cst) != seen; });
          sleepers_.fetch_sub(1, std::memory_order_seq_cst);
          t0 = std::chrono::steady_clock::now();
        }
      }
      seen = g;
      if (id < (int)(g & 0xff)) {  // a helper of this batch: the caller waits for it
        work();
        busy_.fetch_sub(1, std::memory_order_acq_rel);
      }
    }
  }
  std::mutex batch_mu_, mu_;
  std::condition_variable cv_;
  std::vector<std::thread> workers_;
  const CopyJob *jobs_ = nullptr;
  size_t njobs_ = 0;
  bool nt_ = false;
  std::atomic<size_t> next_{0};
  std::atomic<int> busy_{0}, sleepers_{0};
  std::atomic<uint64_t> gen_{0};  // (batch counter << 8) | helpers of the batch
  uint64_t count_ = 0;
};

}  // namespace fcx
