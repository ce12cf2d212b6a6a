// Static-partition thread pool for the CPU engine and host-side phases (ingest, CSR build,
// eigensolver): deterministic chunking, so results do not depend on scheduling.  Pure C++ (no
// HIP), so it is also built into the sanitizer test binary (tests/native).
// Hand-off is hybrid: workers and the caller spin on atomics for a bounded time (~tens of µs)
// before blocking on condition variables, so back-to-back parallel_for calls (the eigensolver
// issues two per Householder step, ~2000 for d = 1000) do not pay a futex wake-up each.
#pragma once

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <exception>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace oap {

class ThreadPool {
 public:
  explicit ThreadPool(int nthreads);
  ~ThreadPool();
  ThreadPool(const ThreadPool&) = delete;
  ThreadPool& operator=(const ThreadPool&) = delete;
  int size() const { return static_cast<int>(workers_.size()) + 1; }
  // Runs fn(chunk_index, begin, end) over [0, n) split into size() contiguous chunks (chunk i
  // covers [n*i/size, n*(i+1)/size)).  The first exception thrown by any chunk is rethrown
  // after every chunk has finished.
  void parallel_for(int64_t n, const std::function<void(int, int64_t, int64_t)>& fn);

 private:
  void worker(int idx);
  std::vector<std::thread> workers_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(int, int64_t, int64_t)>* job_ = nullptr;
  int64_t job_n_ = 0;
  std::atomic<int64_t> generation_{0};
  std::atomic<int> pending_{0};
  std::atomic<bool> stop_{false};
  std::exception_ptr error_;
};

}  // namespace oap
