#include "runtime/memory.h"

#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include <sys/mman.h>

#include "runtime/log.h"

namespace oap {

namespace {
constexpr size_t kAlign = 256;  // keeps every carve 256-B aligned (dwordx4 / LDS-DMA friendly)

// Small pinned blocks, by power-of-two class (64 B .. 1 MiB).  Blocks are never returned to the
// driver: the pool only holds what the process's peak of simultaneously live small pinned
// buffers needed.  A block goes back on its list when its Buffer is destroyed — by then the
// owner has synchronised whatever copy used it (as it had to before hipHostFree).
constexpr int kPoolMinLog = 6, kPoolMaxLog = 20;
struct PinnedPool {
  std::mutex mu;
  std::vector<void*> free_[kPoolMaxLog + 1];
};
PinnedPool& pinned_pool() {
  static PinnedPool* p = new PinnedPool();  // (leaked on purpose: no teardown-order hazards)
  return *p;
}
int pool_class(size_t bytes) {
  int c = kPoolMinLog;
  while ((size_t(1) << c) < bytes) ++c;
  return c;
}
}  // namespace

DeviceArena::DeviceArena(int device, size_t budget_bytes, size_t segment_bytes)
    : device_(device), budget_(budget_bytes), segment_bytes_(segment_bytes) {}

DeviceArena::~DeviceArena() {
  std::lock_guard<std::mutex> g(mu_);
  if (!segments_.empty()) {
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(device_);
    for (auto& s : segments_)
      if (s.base) (void)hipFree(s.base);
    (void)hipSetDevice(prev);
  }
}

void* DeviceArena::allocate(size_t bytes) {
  if (bytes == 0) bytes = kAlign;
  bytes = round_up(bytes, kAlign);
  std::lock_guard<std::mutex> g(mu_);
  // first fit over existing segments
  for (size_t s = 0; s < segments_.size(); ++s) {
    if (!segments_[s].base) continue;
    auto& fl = free_[s];
    for (auto it = fl.begin(); it != fl.end(); ++it) {
      if (it->second >= bytes) {
        size_t off = it->first, sz = it->second;
        fl.erase(it);
        if (sz > bytes) fl.emplace(off + bytes, sz - bytes);
        void* p = segments_[s].base + off;
        live_[p] = Block{s, off, bytes};
        used_ += bytes;
        if (used_ > peak_) peak_ = used_;
        return p;
      }
    }
  }
  // new segment
  size_t seg = bytes > segment_bytes_ ? bytes : segment_bytes_;
  if (reserved_ + seg > budget_) {
    // try an exact-size segment before giving up
    seg = bytes;
    if (reserved_ + seg > budget_)
      OAP_THROW(OutOfMemoryError, "HBM arena budget exceeded on device "
                                      << device_ << ": request " << bytes << " B, reserved "
                                      << reserved_ << " B, budget " << budget_ << " B");
  }
  int prev = 0;
  OAP_HIP_CHECK(hipGetDevice(&prev));
  OAP_HIP_CHECK(hipSetDevice(device_));
  void* base = nullptr;
  hipError_t e = hipMalloc(&base, seg);
  (void)hipSetDevice(prev);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    OAP_THROW(OutOfMemoryError, "hipMalloc(" << seg << ") failed on device " << device_ << ": "
                                             << hipGetErrorString(e));
  }
  segments_.push_back(Segment{static_cast<char*>(base), seg});
  free_.emplace_back();
  size_t s = segments_.size() - 1;
  if (seg > bytes) free_[s].emplace(bytes, seg - bytes);
  reserved_ += seg;
  live_[base] = Block{s, 0, bytes};
  used_ += bytes;
  if (used_ > peak_) peak_ = used_;
  return base;
}

void DeviceArena::release(void* p) {
  if (!p) return;
  std::lock_guard<std::mutex> g(mu_);
  auto it = live_.find(p);
  if (it == live_.end()) return;
  Block b = it->second;
  live_.erase(it);
  used_ -= b.size;
  auto& fl = free_[b.seg];
  auto ins = fl.emplace(b.off, b.size).first;
  // coalesce with successor
  auto nx = std::next(ins);
  if (nx != fl.end() && ins->first + ins->second == nx->first) {
    ins->second += nx->second;
    fl.erase(nx);
  }
  // coalesce with predecessor
  if (ins != fl.begin()) {
    auto pv = std::prev(ins);
    if (pv->first + pv->second == ins->first) {
      pv->second += ins->second;
      fl.erase(ins);
    }
  }
}

void DeviceArena::trim() {
  std::lock_guard<std::mutex> g(mu_);
  for (size_t s = 0; s < segments_.size(); ++s) {
    auto& seg = segments_[s];
    if (!seg.base) continue;
    auto& fl = free_[s];
    if (fl.size() == 1 && fl.begin()->first == 0 && fl.begin()->second == seg.size) {
      int prev = 0;
      (void)hipGetDevice(&prev);
      (void)hipSetDevice(device_);
      (void)hipFree(seg.base);
      (void)hipSetDevice(prev);
      reserved_ -= seg.size;
      seg.base = nullptr;
      seg.size = 0;
      fl.clear();
    }
  }
}

size_t DeviceArena::used() const {
  std::lock_guard<std::mutex> g(mu_);
  return used_;
}
size_t DeviceArena::peak() const {
  std::lock_guard<std::mutex> g(mu_);
  return peak_;
}
size_t DeviceArena::reserved() const {
  std::lock_guard<std::mutex> g(mu_);
  return reserved_;
}

// ------------------------------------------------------------------------------------ Buffer
void* host_alloc_large(size_t bytes) {
  constexpr size_t kHuge = size_t(2) << 20;
  const size_t sz = round_up(bytes == 0 ? 64 : bytes, bytes >= kHuge ? kHuge : 64);
  void* p = std::aligned_alloc(bytes >= kHuge ? kHuge : 64, sz);
  if (!p) OAP_THROW(OutOfMemoryError, "host allocation of " << bytes << " B failed");
  if (bytes >= kHuge) madvise(p, sz, MADV_HUGEPAGE);  // (advice only)
  return p;
}

void host_free_large(void* p) { std::free(p); }

Buffer Buffer::host(size_t bytes) {
  Buffer b;
  size_t sz = round_up(bytes == 0 ? 64 : bytes, 64);
  b.ptr_ = std::aligned_alloc(64, sz);
  if (!b.ptr_) OAP_THROW(OutOfMemoryError, "host allocation of " << bytes << " B failed");
  std::memset(b.ptr_, 0, sz);
  b.bytes_ = bytes;
  b.kind_ = MemKind::Host;
  return b;
}

Buffer Buffer::pinned(size_t bytes) {
  Buffer b;
  void* p = nullptr;
  if (bytes <= (size_t(1) << kPoolMaxLog)) {
    const int c = pool_class(bytes == 0 ? 1 : bytes);
    PinnedPool& pool = pinned_pool();
    {
      std::lock_guard<std::mutex> g(pool.mu);
      if (!pool.free_[c].empty()) {
        p = pool.free_[c].back();
        pool.free_[c].pop_back();
      }
    }
    if (!p) OAP_HIP_CHECK(hipHostMalloc(&p, size_t(1) << c, hipHostMallocDefault));
    b.ptr_ = p;
    b.bytes_ = bytes;
    b.kind_ = MemKind::PinnedPooled;
    return b;
  }
  OAP_HIP_CHECK(hipHostMalloc(&p, bytes, hipHostMallocDefault));
  b.ptr_ = p;
  b.bytes_ = bytes;
  b.kind_ = MemKind::Pinned;
  return b;
}

Buffer Buffer::device(const std::shared_ptr<DeviceArena>& arena, size_t bytes) {
  Buffer b;
  b.ptr_ = arena->allocate(bytes);
  b.bytes_ = bytes;
  b.kind_ = MemKind::Device;
  b.arena_ = arena;
  return b;
}

Buffer Buffer::view(void* p, size_t bytes) {
  Buffer b;
  b.ptr_ = p;
  b.bytes_ = bytes;
  b.kind_ = MemKind::View;
  return b;
}

void Buffer::reset() {
  if (!ptr_) return;
  switch (kind_) {
    case MemKind::View: break;
    case MemKind::Host: std::free(ptr_); break;
    case MemKind::Pinned: (void)hipHostFree(ptr_); break;
    case MemKind::PinnedPooled: {
      PinnedPool& pool = pinned_pool();
      std::lock_guard<std::mutex> g(pool.mu);
      pool.free_[pool_class(bytes_ == 0 ? 1 : bytes_)].push_back(ptr_);
      break;
    }
    case MemKind::Device:
      if (arena_) arena_->release(ptr_);
      break;
  }
  ptr_ = nullptr;
  bytes_ = 0;
  arena_.reset();
}

Buffer::~Buffer() { reset(); }

Buffer::Buffer(Buffer&& o) noexcept
    : ptr_(o.ptr_), bytes_(o.bytes_), kind_(o.kind_), arena_(std::move(o.arena_)) {
  o.ptr_ = nullptr;
  o.bytes_ = 0;
}

Buffer& Buffer::operator=(Buffer&& o) noexcept {
  if (this != &o) {
    reset();
    ptr_ = o.ptr_;
    bytes_ = o.bytes_;
    kind_ = o.kind_;
    arena_ = std::move(o.arena_);
    o.ptr_ = nullptr;
    o.bytes_ = 0;
  }
  return *this;
}

}  // namespace oap
