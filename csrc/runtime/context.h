// Per-process execution context: backend (GPU or CPU), device pinning, HBM arena, HIP streams,
// host thread pool and metrics.  One Context per (process, device); it replaces the
// reference's process-global oneDAL/oneCCL state (mllib-dal/src/main/native/OneCCL.cpp:35-38,
// ALSDALImpl.cpp:37-51) with an explicit, reentrant object.
#pragma once

#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "runtime/common.h"
#include "runtime/log.h"
#include "runtime/memory.h"
#include "runtime/thread_pool.h"

namespace oap {

// RAII HIP stream.
class Stream {
 public:
  Stream() = default;
  explicit Stream(int device, int priority = 0);
  ~Stream();
  Stream(const Stream&) = delete;
  Stream& operator=(const Stream&) = delete;
  hipStream_t get() const { return s_; }
  void sync() const;

 private:
  hipStream_t s_ = nullptr;
  int device_ = -1;
};

// RAII HIP event (timing-enabled by default).
class Event {
 public:
  explicit Event(bool timing = true);
  ~Event();
  Event(const Event&) = delete;
  Event& operator=(const Event&) = delete;
  hipEvent_t get() const { return e_; }
  void record(hipStream_t s);
  void wait_on(hipStream_t s) const;  // make stream s wait for this event
  void sync() const;
  static float elapsed_ms(const Event& a, const Event& b);

 private:
  hipEvent_t e_ = nullptr;
};

struct DeviceInfo {
  int id = -1;
  std::string name;
  std::string arch;
  int cu_count = 0;
  size_t total_mem = 0;
  size_t free_mem = 0;
  int lds_per_block = 0;
  int warp_size = 64;
};

class Context {
 public:
  // device < 0 => CPU backend.  hbm_fraction: share of currently-free HBM the arena may use.
  Context(int device, double hbm_fraction, int cpu_threads);
  ~Context();

  Backend backend() const { return backend_; }
  bool is_gpu() const { return backend_ == Backend::GPU; }
  int device() const { return device_; }
  const DeviceInfo& info() const { return info_; }
  DeviceArena* arena() { return arena_.get(); }
  ThreadPool& pool() { return *pool_; }
  Metrics& metrics() { return metrics_; }

  hipStream_t compute() const { return compute_ ? compute_->get() : nullptr; }
  hipStream_t comm_stream() const { return comm_ ? comm_->get() : nullptr; }
  hipStream_t h2d() const { return h2d_ ? h2d_->get() : nullptr; }
  void sync_all() const;
  void activate() const;  // hipSetDevice(device_) for the calling thread

  // Allocate on this context's backend (device arena for GPU, aligned host memory for CPU).
  Buffer alloc(size_t bytes);
  Buffer alloc_pinned(size_t bytes);

  // Generic copies; kinds inferred from the context's backend.
  void copy_to_backend(void* dst, const void* host_src, size_t bytes, hipStream_t s = nullptr);
  void copy_to_host(void* host_dst, const void* src, size_t bytes, hipStream_t s = nullptr);
  void memset(void* dst, int value, size_t bytes, hipStream_t s = nullptr);
  // Row-pitched download of `rows` rows of `width` bytes (device pitch src_pitch, host pitch
  // dst_pitch) into pageable host memory: 2D copies into two pinned staging buffers on stream s,
  // each drained by the thread pool while the next one transfers (padding dropped on the GPU
  // side; no pageable DMA, no single-threaded copy).  Blocks until done.
  void download_rows(void* dst, size_t dst_pitch, const void* src, size_t src_pitch, size_t width,
                     int64_t rows, hipStream_t s = nullptr);

 private:
  Backend backend_;
  int device_;
  DeviceInfo info_;
  std::shared_ptr<DeviceArena> arena_;
  std::unique_ptr<Stream> compute_, comm_, h2d_;
  std::unique_ptr<ThreadPool> pool_;
  Metrics metrics_;
  Buffer stage_[2];  // download_rows staging (allocated on first use, regrown for wider rows)
  std::mutex stage_mu_;
};

// Number of visible HIP devices (0 when no GPU / no driver).
int visible_device_count();
DeviceInfo query_device(int device);

}  // namespace oap
