#include "runtime/thread_pool.h"

#if defined(__x86_64__) || defined(__i386__)
#include <immintrin.h>
#endif

namespace oap {

namespace {
// ~50-100 us of spinning before a thread blocks (pause is 40-140 cycles on current x86)
constexpr int kSpin = 2000;
inline void cpu_relax() {
#if defined(__x86_64__) || defined(__i386__)
  _mm_pause();
#endif
}
}  // namespace

ThreadPool::ThreadPool(int nthreads) {
  if (nthreads < 1) nthreads = 1;
  for (int i = 1; i < nthreads; ++i) workers_.emplace_back([this, i] { worker(i); });
}

ThreadPool::~ThreadPool() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_.store(true, std::memory_order_release);
  }
  cv_.notify_all();
  for (auto& t : workers_) t.join();
}

void ThreadPool::worker(int idx) {
  int64_t seen = 0;
  for (;;) {
    int64_t g = generation_.load(std::memory_order_acquire);
    for (int spin = 0; g == seen && spin < kSpin && !stop_.load(std::memory_order_relaxed);
         ++spin) {
      cpu_relax();
      g = generation_.load(std::memory_order_acquire);
    }
    if (g == seen) {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] {
        return stop_.load(std::memory_order_relaxed) ||
               generation_.load(std::memory_order_relaxed) != seen;
      });
      g = generation_.load(std::memory_order_acquire);
    }
    if (stop_.load(std::memory_order_acquire)) return;
    seen = g;
    // job_ / job_n_ were written before the generation bump (release) and stay untouched until
    // every worker has decremented pending_
    const std::function<void(int, int64_t, int64_t)>* job = job_;
    const int64_t n = job_n_;
    const int parts = size();
    const int64_t b = n * idx / parts, e = n * (idx + 1) / parts;
    std::exception_ptr err;
    if (b < e) {
      try {
        (*job)(idx, b, e);
      } catch (...) {
        err = std::current_exception();
      }
    }
    if (err) {
      std::lock_guard<std::mutex> lk(mu_);
      if (!error_) error_ = err;
    }
    if (pending_.fetch_sub(1, std::memory_order_acq_rel) == 1) {
      std::lock_guard<std::mutex> lk(mu_);  // pairs with the caller's predicate check
      done_cv_.notify_all();
    }
  }
}

void ThreadPool::parallel_for(int64_t n, const std::function<void(int, int64_t, int64_t)>& fn) {
  const int parts = size();
  if (parts == 1 || n < 2) {
    if (n > 0) fn(0, 0, n);
    return;
  }
  job_ = &fn;
  job_n_ = n;
  pending_.store(parts - 1, std::memory_order_relaxed);
  {
    std::lock_guard<std::mutex> lk(mu_);
    error_ = nullptr;
    generation_.fetch_add(1, std::memory_order_release);
  }
  cv_.notify_all();
  std::exception_ptr mine;
  const int64_t e = n / parts;
  if (e > 0) {
    try {
      fn(0, 0, e);
    } catch (...) {
      mine = std::current_exception();
    }
  }
  for (int spin = 0; spin < kSpin && pending_.load(std::memory_order_acquire) != 0; ++spin)
    cpu_relax();
  std::exception_ptr theirs;
  {
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [&] { return pending_.load(std::memory_order_acquire) == 0; });
    job_ = nullptr;
    theirs = error_;
    error_ = nullptr;
  }
  if (mine) std::rethrow_exception(mine);
  if (theirs) std::rethrow_exception(theirs);
}

}  // namespace oap
