#include "comm/comm.h"
#include "runtime/knobs.h"

#include <rccl/rccl.h>
#include <unistd.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <sstream>
#include <thread>

namespace oap {

// ------------------------------------------------------------------------------------ Comm
void Comm::wait(hipStream_t s) {
  if (s) OAP_HIP_CHECK(hipStreamSynchronize(s));
}

// ------------------------------------------------------------------------------- LocalComm
void LocalComm::allgather(const void* send, void* recv, size_t count, DType dt, hipStream_t s) {
  size_t bytes = count * dtype_size(dt);
  if (send == recv || bytes == 0) return;
  if (device_) {
    OAP_HIP_CHECK(hipMemcpyAsync(recv, send, bytes, hipMemcpyDeviceToDevice, s));
  } else {
    std::memmove(recv, send, bytes);
  }
}

void LocalComm::alltoallv(const void* send, const std::vector<size_t>& send_counts, void* recv,
                          const std::vector<size_t>& recv_counts, DType dt, hipStream_t s) {
  OAP_CHECK(send_counts.size() == 1 && recv_counts.size() == 1 &&
                send_counts[0] == recv_counts[0],
            "LocalComm::alltoallv: inconsistent counts");
  allgather(send, recv, send_counts[0], dt, s);
}

// -------------------------------------------------------------------------------- RCCL
namespace {
ncclDataType_t to_nccl(DType t) {
  switch (t) {
    case DType::F32: return ncclFloat32;
    case DType::F64: return ncclFloat64;
    case DType::BF16: return ncclBfloat16;
    case DType::I32: return ncclInt32;
    case DType::I64: return ncclInt64;
    case DType::U8: return ncclUint8;
  }
  return ncclUint8;
}
ncclRedOp_t to_nccl(ReduceOp op) {
  switch (op) {
    case ReduceOp::Sum: return ncclSum;
    case ReduceOp::Max: return ncclMax;
    case ReduceOp::Min: return ncclMin;
  }
  return ncclSum;
}
#define OAP_NCCL_CHECK(expr)                                                                   \
  do {                                                                                         \
    ncclResult_t _r = (expr);                                                                  \
    if (_r != ncclSuccess)                                                                     \
      ::oap::detail::raise<::oap::CommError>(__FILE__, __LINE__,                               \
                                             std::string(#expr) + ": " +                       \
                                                 ncclGetErrorString(_r));                      \
  } while (0)
}  // namespace

bool rccl_available() {
  int v = 0;
  return ncclGetVersion(&v) == ncclSuccess && v > 0;
}

std::string rccl_unique_id() {
  ncclUniqueId id;
  OAP_NCCL_CHECK(ncclGetUniqueId(&id));
  return std::string(id.internal, sizeof(id.internal));
}

RcclComm::RcclComm(const std::string& unique_id, int world, int rank, int device,
                   double timeout_s)
    : world_(world), rank_(rank), device_(device), timeout_s_(timeout_s) {
  OAP_CHECK(unique_id.size() == sizeof(ncclUniqueId),
            "RCCL unique id must be " << sizeof(ncclUniqueId) << " bytes, got "
                                      << unique_id.size());
  OAP_CHECK(rank >= 0 && rank < world, "bad rank " << rank << " for world " << world);
  ncclUniqueId id;
  std::memcpy(id.internal, unique_id.data(), sizeof(id.internal));
  OAP_HIP_CHECK(hipSetDevice(device));
  ncclComm_t c = nullptr;
  OAP_NCCL_CHECK(ncclCommInitRank(&c, world, id, rank));
  comm_ = c;
  OAP_HIP_CHECK(hipMalloc(&barrier_buf_, 64));
  OAP_HIP_CHECK(hipStreamCreateWithFlags(&barrier_stream_, hipStreamNonBlocking));
  std::ostringstream os;
  os << "\"world\":" << world << ",\"device\":" << device;
  Logger::instance().log(LogLevel::Info, "comm/rccl_init", os.str());
}

RcclComm::~RcclComm() {
  if (comm_ && !aborted_) (void)ncclCommDestroy(static_cast<ncclComm_t>(comm_));
  if (barrier_buf_) (void)hipFree(barrier_buf_);
  if (barrier_stream_) (void)hipStreamDestroy(barrier_stream_);
}

void RcclComm::check_async() {
  if (aborted_) OAP_THROW(CommError, "RCCL communicator was aborted");
  ncclResult_t r = ncclSuccess;
  OAP_NCCL_CHECK(ncclCommGetAsyncError(static_cast<ncclComm_t>(comm_), &r));
  if (r != ncclSuccess && r != ncclInProgress)
    OAP_THROW(CommError, "RCCL async error: " << ncclGetErrorString(r));
}

void Comm::allreduce_oop(const void* send, void* recv, size_t count, DType dt, ReduceOp op,
                         hipStream_t s) {
  const size_t bytes = count * dtype_size(dt);
  if (bytes && send != recv) {
    if (on_device())
      OAP_HIP_CHECK(hipMemcpyAsync(recv, send, bytes, hipMemcpyDeviceToDevice, s));
    else
      std::memcpy(recv, send, bytes);
  }
  allreduce(recv, count, dt, op, s);
}

void RcclComm::allreduce_oop(const void* send, void* recv, size_t count, DType dt, ReduceOp op,
                             hipStream_t s) {
  check_async();
  if (count == 0) return;
  OAP_NCCL_CHECK(ncclAllReduce(send, recv, count, to_nccl(dt), to_nccl(op),
                               static_cast<ncclComm_t>(comm_), s));
}

void RcclComm::allreduce(void* buf, size_t count, DType dt, ReduceOp op, hipStream_t s) {
  check_async();
  if (count == 0) return;
  OAP_NCCL_CHECK(ncclAllReduce(buf, buf, count, to_nccl(dt), to_nccl(op),
                               static_cast<ncclComm_t>(comm_), s));
}

void RcclComm::allgather(const void* send, void* recv, size_t count, DType dt, hipStream_t s) {
  check_async();
  if (count == 0) return;
  OAP_NCCL_CHECK(
      ncclAllGather(send, recv, count, to_nccl(dt), static_cast<ncclComm_t>(comm_), s));
}

void RcclComm::alltoallv(const void* send, const std::vector<size_t>& send_counts, void* recv,
                         const std::vector<size_t>& recv_counts, DType dt, hipStream_t s) {
  check_async();
  OAP_CHECK(static_cast<int>(send_counts.size()) == world_ &&
                static_cast<int>(recv_counts.size()) == world_,
            "alltoallv: counts must have one entry per rank");
  const size_t es = dtype_size(dt);
  auto c = static_cast<ncclComm_t>(comm_);
  // Segments move in rounds of at most kChunk bytes per peer (a 1B-rating shuffle sends GBs
  // per peer): bounded transfers per send/recv pair and per group.  Both sides of a pair agree
  // on the counts, hence on the number of rounds; p2p ops match in order per pair, so ranks may
  // run different numbers of rounds.
  // (OAP_RCCL_A2A_CHUNK_BYTES overrides the 256 MiB round size: tests drive several rounds
  // with small uneven counts)
  const size_t kChunk = [] {  // (read per call: tests set it mid-process)
    const int64_t v = knob_int("OAP_RCCL_A2A_CHUNK_BYTES");
    return v > 0 ? size_t(v) : size_t(1) << 28;
  }();
  const size_t chunk = std::max<size_t>(1, kChunk / es);
  size_t most = 0;
  for (int p = 0; p < world_; ++p) most = std::max({most, send_counts[p], recv_counts[p]});
  for (size_t done = 0; done < most; done += chunk) {
    OAP_NCCL_CHECK(ncclGroupStart());
    size_t soff = 0, roff = 0;
    for (int p = 0; p < world_; ++p) {
      if (send_counts[p] > done)
        OAP_NCCL_CHECK(ncclSend(static_cast<const char*>(send) + (soff + done) * es,
                                std::min(chunk, send_counts[p] - done), to_nccl(dt), p, c, s));
      if (recv_counts[p] > done)
        OAP_NCCL_CHECK(ncclRecv(static_cast<char*>(recv) + (roff + done) * es,
                                std::min(chunk, recv_counts[p] - done), to_nccl(dt), p, c, s));
      soff += send_counts[p];
      roff += recv_counts[p];
    }
    OAP_NCCL_CHECK(ncclGroupEnd());
  }
}

void RcclComm::bcast(void* buf, size_t count, DType dt, int root, hipStream_t s) {
  check_async();
  if (count == 0) return;
  OAP_NCCL_CHECK(
      ncclBroadcast(buf, buf, count, to_nccl(dt), root, static_cast<ncclComm_t>(comm_), s));
}

void RcclComm::group_start() { OAP_NCCL_CHECK(ncclGroupStart()); }
void RcclComm::group_end() { OAP_NCCL_CHECK(ncclGroupEnd()); }

void RcclComm::barrier() {
  OAP_HIP_CHECK(hipSetDevice(device_));
  allreduce(barrier_buf_, 1, DType::I32, ReduceOp::Sum, barrier_stream_);
  wait(barrier_stream_);
}

void RcclComm::wait(hipStream_t s) {
  if (timeout_s_ <= 0) {
    OAP_HIP_CHECK(hipStreamSynchronize(s));
    check_async();
    return;
  }
  auto t0 = std::chrono::steady_clock::now();
  int spins = 0;
  for (;;) {
    hipError_t q = hipStreamQuery(s);
    if (q == hipSuccess) break;
    if (q != hipErrorNotReady) OAP_HIP_CHECK(q);
    check_async();
    double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (el > timeout_s_) {
      std::ostringstream os;
      os << "\"timeout_s\":" << timeout_s_;
      Logger::instance().log(LogLevel::Error, "comm/watchdog_timeout", os.str());
      abort();
      OAP_THROW(CommError, "collective watchdog: stream not finished after "
                               << timeout_s_ << " s (rank " << rank_
                               << "); communicator aborted");
    }
    // Spin briefly (collectives are usually µs), then back off to keep a core free.
    if (++spins > 2000) std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
}

void RcclComm::abort() {
  if (comm_ && !aborted_) {
    (void)ncclCommAbort(static_cast<ncclComm_t>(comm_));
    aborted_ = true;
  }
}

// -------------------------------------------------------------------------------- helpers
namespace {
bool need_stage(Context& ctx, Comm& comm) { return ctx.is_gpu() && !comm.on_device(); }
}  // namespace

void comm_allreduce(Context& ctx, Comm& comm, void* buf, size_t count, DType dt, ReduceOp op,
                    hipStream_t s) {
  if (comm.trivial() || count == 0) return;
  if (!need_stage(ctx, comm)) {
    comm.allreduce(buf, count, dt, op, s);
    return;
  }
  size_t bytes = count * dtype_size(dt);
  Buffer h = Buffer::pinned(bytes);
  OAP_HIP_CHECK(hipMemcpyAsync(h.data(), buf, bytes, hipMemcpyDeviceToHost, s));
  OAP_HIP_CHECK(hipStreamSynchronize(s));
  comm.allreduce(h.data(), count, dt, op, nullptr);
  OAP_HIP_CHECK(hipMemcpyAsync(buf, h.data(), bytes, hipMemcpyHostToDevice, s));
  OAP_HIP_CHECK(hipStreamSynchronize(s));
}

void comm_allgather(Context& ctx, Comm& comm, const void* send, void* recv, size_t count,
                    DType dt, hipStream_t s) {
  size_t bytes = count * dtype_size(dt);
  if (!need_stage(ctx, comm)) {
    comm.allgather(send, recv, count, dt, s);
    return;
  }
  Buffer hs = Buffer::pinned(bytes), hr = Buffer::pinned(bytes * comm.size());
  OAP_HIP_CHECK(hipMemcpyAsync(hs.data(), send, bytes, hipMemcpyDeviceToHost, s));
  OAP_HIP_CHECK(hipStreamSynchronize(s));
  comm.allgather(hs.data(), hr.data(), count, dt, nullptr);
  OAP_HIP_CHECK(
      hipMemcpyAsync(recv, hr.data(), bytes * comm.size(), hipMemcpyHostToDevice, s));
  OAP_HIP_CHECK(hipStreamSynchronize(s));
}

void comm_alltoallv(Context& ctx, Comm& comm, const void* send,
                    const std::vector<size_t>& send_counts, void* recv,
                    const std::vector<size_t>& recv_counts, DType dt, hipStream_t s) {
  if (!need_stage(ctx, comm)) {
    comm.alltoallv(send, send_counts, recv, recv_counts, dt, s);
    return;
  }
  size_t es = dtype_size(dt), sn = 0, rn = 0;
  for (auto c : send_counts) sn += c;
  for (auto c : recv_counts) rn += c;
  Buffer hs = Buffer::pinned(sn * es), hr = Buffer::pinned(rn * es);
  OAP_HIP_CHECK(hipMemcpyAsync(hs.data(), send, sn * es, hipMemcpyDeviceToHost, s));
  OAP_HIP_CHECK(hipStreamSynchronize(s));
  comm.alltoallv(hs.data(), send_counts, hr.data(), recv_counts, dt, nullptr);
  OAP_HIP_CHECK(hipMemcpyAsync(recv, hr.data(), rn * es, hipMemcpyHostToDevice, s));
  OAP_HIP_CHECK(hipStreamSynchronize(s));
}

void comm_bcast(Context& ctx, Comm& comm, void* buf, size_t count, DType dt, int root,
                hipStream_t s) {
  if (comm.trivial() || count == 0) return;
  if (!need_stage(ctx, comm)) {
    comm.bcast(buf, count, dt, root, s);
    return;
  }
  size_t bytes = count * dtype_size(dt);
  Buffer h = Buffer::pinned(bytes);
  OAP_HIP_CHECK(hipMemcpyAsync(h.data(), buf, bytes, hipMemcpyDeviceToHost, s));
  OAP_HIP_CHECK(hipStreamSynchronize(s));
  comm.bcast(h.data(), count, dt, root, nullptr);
  OAP_HIP_CHECK(hipMemcpyAsync(buf, h.data(), bytes, hipMemcpyHostToDevice, s));
  OAP_HIP_CHECK(hipStreamSynchronize(s));
}

void comm_allreduce_host(Context& ctx, Comm& comm, void* host, size_t count, DType dt,
                         ReduceOp op) {
  if (comm.trivial() || count == 0) return;
  if (!comm.on_device()) {
    comm.allreduce(host, count, dt, op, nullptr);
    return;
  }
  const size_t bytes = count * dtype_size(dt);
  Buffer d = ctx.alloc(bytes);
  hipStream_t s = ctx.comm_stream();
  OAP_HIP_CHECK(hipMemcpyAsync(d.data(), host, bytes, hipMemcpyHostToDevice, s));
  comm.allreduce(d.data(), count, dt, op, s);
  OAP_HIP_CHECK(hipMemcpyAsync(host, d.data(), bytes, hipMemcpyDeviceToHost, s));
  comm.wait(s);
}

void comm_allgather_host(Context& ctx, Comm& comm, const void* send, void* recv, size_t count,
                         DType dt) {
  const size_t bytes = count * dtype_size(dt);
  if (comm.trivial()) {
    if (bytes) std::memmove(recv, send, bytes);
    return;
  }
  if (!comm.on_device()) {
    comm.allgather(send, recv, count, dt, nullptr);
    return;
  }
  Buffer ds = ctx.alloc(bytes), dr = ctx.alloc(bytes * comm.size());
  hipStream_t s = ctx.comm_stream();
  OAP_HIP_CHECK(hipMemcpyAsync(ds.data(), send, bytes, hipMemcpyHostToDevice, s));
  comm.allgather(ds.data(), dr.data(), count, dt, s);
  OAP_HIP_CHECK(hipMemcpyAsync(recv, dr.data(), bytes * comm.size(), hipMemcpyDeviceToHost, s));
  comm.wait(s);
}

void comm_alltoallv_host(Context& ctx, Comm& comm, const void* send,
                         const std::vector<size_t>& send_counts, void* recv,
                         const std::vector<size_t>& recv_counts, DType dt) {
  const size_t es = dtype_size(dt);
  size_t sn = 0, rn = 0;
  for (auto c : send_counts) sn += c;
  for (auto c : recv_counts) rn += c;
  if (comm.trivial()) {
    OAP_CHECK(sn == rn, "alltoallv: world of one with mismatched counts");
    if (sn) std::memmove(recv, send, sn * es);
    return;
  }
  if (!comm.on_device()) {
    comm.alltoallv(send, send_counts, recv, recv_counts, dt, nullptr);
    return;
  }
  Buffer ds = ctx.alloc(std::max<size_t>(sn * es, 16));
  Buffer dr = ctx.alloc(std::max<size_t>(rn * es, 16));
  hipStream_t s = ctx.comm_stream();
  if (sn) OAP_HIP_CHECK(hipMemcpyAsync(ds.data(), send, sn * es, hipMemcpyHostToDevice, s));
  comm.alltoallv(ds.data(), send_counts, dr.data(), recv_counts, dt, s);
  if (rn) OAP_HIP_CHECK(hipMemcpyAsync(recv, dr.data(), rn * es, hipMemcpyDeviceToHost, s));
  comm.wait(s);
}

double comm_allreduce_scalar(Context& ctx, Comm& comm, double v, ReduceOp op) {
  if (comm.trivial()) return v;
  if (comm.on_device()) {
    Buffer d = ctx.alloc(sizeof(double));
    hipStream_t s = ctx.comm_stream();
    OAP_HIP_CHECK(hipMemcpyAsync(d.data(), &v, sizeof(double), hipMemcpyHostToDevice, s));
    comm.allreduce(d.data(), 1, DType::F64, op, s);
    OAP_HIP_CHECK(hipMemcpyAsync(&v, d.data(), sizeof(double), hipMemcpyDeviceToHost, s));
    comm.wait(s);
    return v;
  }
  comm.allreduce(&v, 1, DType::F64, op, nullptr);
  return v;
}

std::vector<int64_t> comm_allgather_i64(Context& ctx, Comm& comm, int64_t v) {
  std::vector<int64_t> out(comm.size(), v);
  if (comm.trivial()) return out;
  if (comm.on_device()) {
    Buffer d = ctx.alloc(sizeof(int64_t) * (comm.size() + 1));
    hipStream_t s = ctx.comm_stream();
    int64_t* dp = d.as<int64_t>();
    OAP_HIP_CHECK(hipMemcpyAsync(dp, &v, sizeof(int64_t), hipMemcpyHostToDevice, s));
    comm.allgather(dp, dp + 1, 1, DType::I64, s);
    OAP_HIP_CHECK(hipMemcpyAsync(out.data(), dp + 1, sizeof(int64_t) * comm.size(),
                                 hipMemcpyDeviceToHost, s));
    comm.wait(s);
    return out;
  }
  comm.allgather(&v, out.data(), 1, DType::I64, nullptr);
  return out;
}

// ------------------------------------------------------------------------- fault injection
void maybe_inject_fault(int rank, const char* phase, int iteration) {
  const std::string spec_s = knob_str("OAP_MLLIB_FAULT");
  if (spec_s.empty()) return;
  const char* spec = spec_s.c_str();
  int r = -1, it = -1;
  char ph[64] = {0};
  if (std::sscanf(spec, "%d:%63[^:]:%d", &r, ph, &it) != 3) return;
  if (r != rank || it != iteration || std::strcmp(ph, phase) != 0) return;
  const std::string mode = knob_str("OAP_MLLIB_FAULT_MODE");
  std::ostringstream os;
  os << "\"iteration\":" << iteration << ",\"mode\":\"" << mode << "\"";
  Logger::instance().log(LogLevel::Error, std::string("fault/") + phase, os.str());
  if (mode == "exit") _exit(17);
  OAP_THROW(CommError, "injected fault at rank " << rank << " phase " << phase << " iteration "
                                                   << iteration);
}

}  // namespace oap
