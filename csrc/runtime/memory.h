// Memory management: an HBM arena sized against a per-GPU budget (288 GB HBM3E on MI355X),
// pinned host staging buffers for ingestion, and an owning Buffer handle that is either host-
// or device-resident.
//
// The reference allocates one oneDAL HomogenNumericTable per Spark partition and copies rows
// into it with one JNI call per row (mllib-dal/src/main/scala/org/apache/spark/ml/util/
// OneDAL.scala:116-142 -> native/OneDAL.cpp:50-60), and never frees the result tables
// (KMeansDALImpl.cpp:245).  Here every allocation is an RAII Buffer carved out of a
// DeviceArena: one hipMalloc per large segment, first-fit free list with coalescing, a hard
// budget that turns into OutOfMemoryError instead of a driver OOM, and peak/used statistics
// for the partition planner (runtime/planner.h).
#pragma once

#include <cstddef>
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <vector>

#include "runtime/common.h"

namespace oap {

class DeviceArena {
 public:
  DeviceArena(int device, size_t budget_bytes, size_t segment_bytes);
  ~DeviceArena();
  DeviceArena(const DeviceArena&) = delete;
  DeviceArena& operator=(const DeviceArena&) = delete;

  void* allocate(size_t bytes);
  void release(void* p);

  size_t used() const;
  size_t peak() const;
  size_t reserved() const;
  size_t budget() const { return budget_; }
  void set_budget(size_t b) { budget_ = b; }
  int device() const { return device_; }
  // Returns every fully-free segment to the driver.
  void trim();

 private:
  struct Segment {
    char* base;
    size_t size;
  };
  struct Block {
    size_t seg;
    size_t off;
    size_t size;
  };
  mutable std::mutex mu_;
  int device_;
  size_t budget_;
  size_t segment_bytes_;
  size_t used_ = 0;
  size_t peak_ = 0;
  size_t reserved_ = 0;
  std::vector<Segment> segments_;
  // free blocks per segment keyed by offset (for coalescing)
  std::vector<std::map<size_t, size_t>> free_;
  std::map<void*, Block> live_;
};

enum class MemKind : int { Host = 0, Device = 1, Pinned = 2, View = 3, PinnedPooled = 4 };

// Owning, typed-agnostic buffer.  Device buffers come from an arena; host buffers are 64-byte
// aligned malloc; pinned buffers are hipHostMalloc (for async H2D/D2H) — small ones (<= 1 MiB:
// flags, counters, per-fit read-backs) from a process-wide pool of power-of-two blocks, since a
// hipHostMalloc / hipHostFree pair costs far more than the copies such a buffer serves (a fit
// allocated six of them: ~0.2 ms of host time on every call).
// Contract of a pooled pinned buffer: no async copy into or out of it may still be in flight when
// it is destroyed (hipHostFree used to wait for the device; the pool does not) — the owner drains
// the stream first, on the exception path too (kmeans.cpp StreamDrainOnUnwind).
class Buffer {
 public:
  Buffer() = default;
  static Buffer host(size_t bytes);
  static Buffer pinned(size_t bytes);
  static Buffer device(const std::shared_ptr<DeviceArena>& arena, size_t bytes);
  // Non-owning view of memory someone else manages (e.g. a torch tensor's device storage);
  // the owner must outlive the view.
  static Buffer view(void* p, size_t bytes);
  ~Buffer();
  Buffer(Buffer&& o) noexcept;
  Buffer& operator=(Buffer&& o) noexcept;
  Buffer(const Buffer&) = delete;
  Buffer& operator=(const Buffer&) = delete;

  void* data() const { return ptr_; }
  template <typename T>
  T* as() const {
    return static_cast<T*>(ptr_);
  }
  size_t bytes() const { return bytes_; }
  MemKind kind() const { return kind_; }
  bool empty() const { return ptr_ == nullptr; }
  void reset();

 private:
  void* ptr_ = nullptr;
  size_t bytes_ = 0;
  MemKind kind_ = MemKind::Host;
  // Shared ownership: a buffer keeps its arena alive, so Python may destroy a Context before
  // the tables allocated from it (interpreter-shutdown order is arbitrary).
  std::shared_ptr<DeviceArena> arena_;
};

// Large host result array (model factors, labels): uninitialised (no zero pass over GBs),
// 2 MiB-aligned with transparent huge pages requested (few first-touch faults when the download
// threads fill it), and shared so a binding can hand it to numpy without a copy.
void* host_alloc_large(size_t bytes);
void host_free_large(void* p);

template <typename T>
class HostArray {
 public:
  HostArray() = default;
  static HostArray alloc(size_t n) {
    HostArray a;
    a.n_ = n;
    a.p_ = std::shared_ptr<T>(static_cast<T*>(host_alloc_large(n * sizeof(T))),
                              [](T* q) { host_free_large(q); });
    return a;
  }
  T* data() const { return p_.get(); }
  size_t size() const { return n_; }
  bool empty() const { return n_ == 0; }
  T& operator[](size_t i) const { return p_.get()[i]; }
  const std::shared_ptr<T>& owner() const { return p_; }

 private:
  std::shared_ptr<T> p_;
  size_t n_ = 0;
};

}  // namespace oap
