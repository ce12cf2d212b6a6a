#include "runtime/context.h"

#include <algorithm>
#include <cstring>

namespace oap {

// -------------------------------------------------------------------------------- Stream/Event
Stream::Stream(int device, int priority) : device_(device) {
  OAP_HIP_CHECK(hipSetDevice(device));
  OAP_HIP_CHECK(hipStreamCreateWithPriority(&s_, hipStreamNonBlocking, priority));
}
Stream::~Stream() {
  if (s_) (void)hipStreamDestroy(s_);
}
void Stream::sync() const { OAP_HIP_CHECK(hipStreamSynchronize(s_)); }

Event::Event(bool timing) {
  OAP_HIP_CHECK(hipEventCreateWithFlags(&e_, timing ? hipEventDefault : hipEventDisableTiming));
}
Event::~Event() {
  if (e_) (void)hipEventDestroy(e_);
}
void Event::record(hipStream_t s) { OAP_HIP_CHECK(hipEventRecord(e_, s)); }
void Event::wait_on(hipStream_t s) const { OAP_HIP_CHECK(hipStreamWaitEvent(s, e_, 0)); }
void Event::sync() const { OAP_HIP_CHECK(hipEventSynchronize(e_)); }
float Event::elapsed_ms(const Event& a, const Event& b) {
  float ms = 0.f;
  OAP_HIP_CHECK(hipEventElapsedTime(&ms, a.e_, b.e_));
  return ms;
}

// -------------------------------------------------------------------------------- devices
int visible_device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return n;
}

DeviceInfo query_device(int device) {
  DeviceInfo d;
  hipDeviceProp_t p;
  OAP_HIP_CHECK(hipGetDeviceProperties(&p, device));
  d.id = device;
  d.name = p.name;
  d.arch = p.gcnArchName;
  d.cu_count = p.multiProcessorCount;
  d.total_mem = p.totalGlobalMem;
  d.lds_per_block = static_cast<int>(p.sharedMemPerBlock);
  d.warp_size = p.warpSize;
  int prev = 0;
  OAP_HIP_CHECK(hipGetDevice(&prev));
  OAP_HIP_CHECK(hipSetDevice(device));
  size_t fr = 0, tot = 0;
  OAP_HIP_CHECK(hipMemGetInfo(&fr, &tot));
  OAP_HIP_CHECK(hipSetDevice(prev));
  d.free_mem = fr;
  return d;
}

// -------------------------------------------------------------------------------- Context
Context::Context(int device, double hbm_fraction, int cpu_threads)
    : backend_(device >= 0 ? Backend::GPU : Backend::CPU), device_(device) {
  if (cpu_threads <= 0) {
    unsigned hc = std::thread::hardware_concurrency();
    cpu_threads = static_cast<int>(std::min<unsigned>(hc == 0 ? 1 : hc, 16));
  }
  pool_ = std::make_unique<ThreadPool>(cpu_threads);
  if (backend_ == Backend::GPU) {
    int n = visible_device_count();
    OAP_CHECK(device < n, "device " << device << " requested but only " << n << " visible");
    info_ = query_device(device);
    OAP_HIP_CHECK(hipSetDevice(device));
    if (hbm_fraction <= 0.0 || hbm_fraction > 1.0) hbm_fraction = 0.9;
    size_t budget = static_cast<size_t>(static_cast<double>(info_.free_mem) * hbm_fraction);
    // 1 GiB segments: few hipMallocs for 288 GB-class devices, little waste for small fits.
    arena_ = std::make_shared<DeviceArena>(device, budget, size_t(1) << 30);
    int lo = 0, hi = 0;
    OAP_HIP_CHECK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    compute_ = std::make_unique<Stream>(device, 0);
    comm_ = std::make_unique<Stream>(device, hi);  // collectives get the higher priority
    h2d_ = std::make_unique<Stream>(device, 0);
  } else {
    info_.id = -1;
    info_.name = "cpu";
    info_.arch = "x86_64";
    info_.cu_count = pool_->size();
  }
}

Context::~Context() {
  if (backend_ == Backend::GPU) {
    (void)hipSetDevice(device_);
    (void)hipDeviceSynchronize();
  }
}

void Context::activate() const {
  if (backend_ == Backend::GPU) OAP_HIP_CHECK(hipSetDevice(device_));
}

void Context::sync_all() const {
  if (backend_ != Backend::GPU) return;
  OAP_HIP_CHECK(hipSetDevice(device_));
  compute_->sync();
  comm_->sync();
  h2d_->sync();
}

Buffer Context::alloc(size_t bytes) {
  if (backend_ == Backend::GPU) return Buffer::device(arena_, bytes);
  return Buffer::host(bytes);
}

Buffer Context::alloc_pinned(size_t bytes) {
  if (backend_ == Backend::GPU) return Buffer::pinned(bytes);
  return Buffer::host(bytes);
}

void Context::copy_to_backend(void* dst, const void* src, size_t bytes, hipStream_t s) {
  if (bytes == 0) return;
  if (backend_ == Backend::GPU) {
    OAP_HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s ? s : compute()));
  } else {
    std::memcpy(dst, src, bytes);
  }
}

void Context::copy_to_host(void* dst, const void* src, size_t bytes, hipStream_t s) {
  if (bytes == 0) return;
  if (backend_ == Backend::GPU) {
    hipStream_t st = s ? s : compute();
    OAP_HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, st));
    OAP_HIP_CHECK(hipStreamSynchronize(st));
  } else {
    std::memcpy(dst, src, bytes);
  }
}

void Context::download_rows(void* dst, size_t dst_pitch, const void* src, size_t src_pitch,
                            size_t width, int64_t rows, hipStream_t s) {
  if (rows <= 0 || width == 0) return;
  OAP_CHECK(width <= dst_pitch && width <= src_pitch, "download_rows: width exceeds a pitch");
  if (backend_ != Backend::GPU) {
    pool_->parallel_for(rows, [&](int, int64_t b, int64_t e) {
      for (int64_t i = b; i < e; ++i)
        std::memcpy(static_cast<char*>(dst) + size_t(i) * dst_pitch,
                    static_cast<const char*>(src) + size_t(i) * src_pitch, width);
    });
    return;
  }
  hipStream_t st = s ? s : compute();
  constexpr size_t kStage = size_t(64) << 20;
  const int64_t per = std::max<int64_t>(1, int64_t(kStage / width));
  // (one Context's staging pair: download_rows is not thread-safe per Context — callers
  // serialise on the Context, as every driver does on its compute stream)
  std::lock_guard<std::mutex> lk(stage_mu_);
  if (stage_[0].empty() || stage_[0].bytes() < std::max(kStage, width)) {
    stage_[0] = Buffer::pinned(std::max(kStage, width));  // (regrown for a wider row)
    stage_[1] = Buffer::pinned(std::max(kStage, width));
  }
  const int64_t nch = (rows + per - 1) / per;
  Event done[2];
  auto issue = [&](int64_t c) {
    const int64_t r0 = c * per, nr = std::min(per, rows - r0);
    OAP_HIP_CHECK(hipMemcpy2DAsync(stage_[c & 1].data(), width,
                                   static_cast<const char*>(src) + size_t(r0) * src_pitch,
                                   src_pitch, width, size_t(nr), hipMemcpyDeviceToHost, st));
    done[c & 1].record(st);
  };
  issue(0);
  if (nch > 1) issue(1);
  for (int64_t c = 0; c < nch; ++c) {
    done[c & 1].sync();
    const int64_t r0 = c * per, nr = std::min(per, rows - r0);
    const char* from = stage_[c & 1].as<char>();
    char* to = static_cast<char*>(dst) + size_t(r0) * dst_pitch;
    if (dst_pitch == width) {
      const size_t bytes = size_t(nr) * width;
      const int64_t parts = std::min<int64_t>(int64_t(pool_->size()) * 4, int64_t(bytes >> 20) + 1);
      pool_->parallel_for(parts, [&](int, int64_t b, int64_t e) {
        const size_t lo = bytes * size_t(b) / size_t(parts), hi = bytes * size_t(e) / size_t(parts);
        std::memcpy(to + lo, from + lo, hi - lo);
      });
    } else {
      pool_->parallel_for(nr, [&](int, int64_t b, int64_t e) {
        for (int64_t i = b; i < e; ++i)
          std::memcpy(to + size_t(i) * dst_pitch, from + size_t(i) * width, width);
      });
    }
    if (c + 2 < nch) issue(c + 2);  // (this stage is drained)
  }
}

void Context::memset(void* dst, int value, size_t bytes, hipStream_t s) {
  if (bytes == 0) return;
  if (backend_ == Backend::GPU) {
    OAP_HIP_CHECK(hipMemsetAsync(dst, value, bytes, s ? s : compute()));
  } else {
    std::memset(dst, value, bytes);
  }
}

}  // namespace oap
