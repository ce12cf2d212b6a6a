#include "runtime/thread_pool.h"

namespace oap {

ThreadPool::ThreadPool(int nthreads) {
  if (nthreads < 1) nthreads = 1;
  for (int i = 1; i < nthreads; ++i) workers_.emplace_back([this, i] { worker(i); });
}

ThreadPool::~ThreadPool() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  for (auto& t : workers_) t.join();
}

void ThreadPool::worker(int idx) {
  int64_t seen = 0;
  for (;;) {
    const std::function<void(int, int64_t, int64_t)>* job;
    int64_t n;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] { return stop_ || generation_ != seen; });
      if (stop_) return;
      seen = generation_;
      job = job_;
      n = job_n_;
    }
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
    {
      std::lock_guard<std::mutex> g(mu_);
      if (err && !error_) error_ = err;
      if (--pending_ == 0) done_cv_.notify_all();
    }
  }
}

void ThreadPool::parallel_for(int64_t n, const std::function<void(int, int64_t, int64_t)>& fn) {
  const int parts = size();
  if (parts == 1 || n < 2) {
    if (n > 0) fn(0, 0, n);
    return;
  }
  {
    std::lock_guard<std::mutex> g(mu_);
    job_ = &fn;
    job_n_ = n;
    pending_ = parts - 1;
    error_ = nullptr;
    ++generation_;
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
  std::exception_ptr theirs;
  {
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [&] { return pending_ == 0; });
    job_ = nullptr;
    theirs = error_;
    error_ = nullptr;
  }
  if (mine) std::rethrow_exception(mine);
  if (theirs) std::rethrow_exception(theirs);
}

}  // namespace oap
