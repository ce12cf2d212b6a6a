// Collective-communication layer.
//
// Replaces the reference's oneCCL usage (mllib-dal/src/main/native/OneCCL.cpp:47-99 for
// communicator setup; the per-iteration byte-archive collectives listed in SURVEY.md §2.7,
// e.g. KMeansDALImpl.cpp:49-59,97-99,213-214 and ALSDALImpl.cpp:53-151) with typed, rootless,
// stream-ordered collectives:
//   * RcclComm   — RCCL over xGMI on device buffers (one communicator per process, reused
//                  across fits instead of being built and torn down per fit).
//   * LocalComm  — world of one (no-op collectives).
//   * host comms — implemented by the bindings (a Python object, e.g. torch.distributed/gloo),
//                  used on CPU and as a fallback when RCCL is unavailable.
// A Comm that works on host buffers can still serve a GPU engine: comm_* helpers below stage
// through pinned memory.
#pragma once

#include <chrono>
#include <memory>
#include <string>
#include <vector>

#include "runtime/common.h"
#include "runtime/context.h"

namespace oap {

class Comm {
 public:
  virtual ~Comm() = default;
  virtual int rank() const = 0;
  virtual int size() const = 0;
  virtual bool on_device() const = 0;  // true => buffers must be device pointers
  virtual const char* name() const = 0;
  // True when every collective is a no-op (a world of one without a real communicator): the
  // drivers then skip their exchange steps.  An RCCL communicator of one rank is NOT trivial —
  // it runs every collective (send/recv to self, 1-rank allreduce / broadcast), which is how a
  // 1-GPU box exercises the device-collective code paths of the multi-GPU drivers.
  virtual bool trivial() const { return size() == 1; }

  // In-place allreduce.
  virtual void allreduce(void* buf, size_t count, DType dt, ReduceOp op, hipStream_t s) = 0;
  // Out-of-place allreduce (send and recv distinct); the default copies send into recv (on the
  // device when on_device(), else on the host) and reduces in place.
  virtual void allreduce_oop(const void* send, void* recv, size_t count, DType dt, ReduceOp op,
                             hipStream_t s);
  // recv holds size()*count elements, rank-major.
  virtual void allgather(const void* send, void* recv, size_t count, DType dt, hipStream_t s) = 0;
  // Variable-size exchange; counts are in elements, displacements are packed (prefix sums).
  virtual void alltoallv(const void* send, const std::vector<size_t>& send_counts, void* recv,
                         const std::vector<size_t>& recv_counts, DType dt, hipStream_t s) = 0;
  virtual void bcast(void* buf, size_t count, DType dt, int root, hipStream_t s) = 0;
  virtual void barrier() = 0;
  // Block until everything enqueued on `s` (including collectives) has finished; RcclComm
  // enforces the watchdog timeout here and aborts the communicator on expiry.
  virtual void wait(hipStream_t s);
  virtual void abort() {}
};

class LocalComm final : public Comm {
 public:
  explicit LocalComm(bool device) : device_(device) {}
  int rank() const override { return 0; }
  int size() const override { return 1; }
  bool on_device() const override { return device_; }
  const char* name() const override { return "local"; }
  void allreduce(void*, size_t, DType, ReduceOp, hipStream_t) override {}
  void allgather(const void* send, void* recv, size_t count, DType dt, hipStream_t s) override;
  void alltoallv(const void* send, const std::vector<size_t>& send_counts, void* recv,
                 const std::vector<size_t>& recv_counts, DType dt, hipStream_t s) override;
  void bcast(void*, size_t, DType, int, hipStream_t) override {}
  void barrier() override {}

 private:
  bool device_;
};

// 128-byte opaque unique id (ncclUniqueId).
std::string rccl_unique_id();
bool rccl_available();

class RcclComm final : public Comm {
 public:
  // timeout_s <= 0 disables the watchdog.
  RcclComm(const std::string& unique_id, int world, int rank, int device, double timeout_s);
  ~RcclComm() override;
  int rank() const override { return rank_; }
  int size() const override { return world_; }
  bool on_device() const override { return true; }
  const char* name() const override { return "rccl"; }
  bool trivial() const override { return false; }
  void allreduce(void* buf, size_t count, DType dt, ReduceOp op, hipStream_t s) override;
  void allreduce_oop(const void* send, void* recv, size_t count, DType dt, ReduceOp op,
                     hipStream_t s) override;
  void allgather(const void* send, void* recv, size_t count, DType dt, hipStream_t s) override;
  void alltoallv(const void* send, const std::vector<size_t>& send_counts, void* recv,
                 const std::vector<size_t>& recv_counts, DType dt, hipStream_t s) override;
  void bcast(void* buf, size_t count, DType dt, int root, hipStream_t s) override;
  void barrier() override;
  void wait(hipStream_t s) override;
  void abort() override;
  // Group several collectives into one RCCL launch (ncclGroupStart/End).
  void group_start();
  void group_end();

 private:
  void check_async();
  void* comm_ = nullptr;  // ncclComm_t
  int world_, rank_, device_;
  double timeout_s_;
  bool aborted_ = false;
  void* barrier_buf_ = nullptr;
  hipStream_t barrier_stream_ = nullptr;
};

// Helpers that make any Comm usable from any Context: when the context is a GPU and the comm
// wants host buffers, the payload is staged through a pinned buffer.
void comm_allreduce(Context& ctx, Comm& comm, void* buf, size_t count, DType dt, ReduceOp op,
                    hipStream_t s);
void comm_allgather(Context& ctx, Comm& comm, const void* send, void* recv, size_t count,
                    DType dt, hipStream_t s);
void comm_alltoallv(Context& ctx, Comm& comm, const void* send,
                    const std::vector<size_t>& send_counts, void* recv,
                    const std::vector<size_t>& recv_counts, DType dt, hipStream_t s);
void comm_bcast(Context& ctx, Comm& comm, void* buf, size_t count, DType dt, int root,
                hipStream_t s);
// Host memory in, host memory out, whatever memory the comm works on.
void comm_allreduce_host(Context& ctx, Comm& comm, void* host, size_t count, DType dt,
                         ReduceOp op);
// allgather of HOST buffers over any comm (device comms stage through HBM).
void comm_allgather_host(Context& ctx, Comm& comm, const void* send, void* recv, size_t count,
                         DType dt);
// Variable-size exchange of HOST buffers over any comm (device comms stage through HBM).
void comm_alltoallv_host(Context& ctx, Comm& comm, const void* send,
                         const std::vector<size_t>& send_counts, void* recv,
                         const std::vector<size_t>& recv_counts, DType dt);
// Host-side scalar convenience (always host memory in, host memory out).
double comm_allreduce_scalar(Context& ctx, Comm& comm, double v, ReduceOp op);
std::vector<int64_t> comm_allgather_i64(Context& ctx, Comm& comm, int64_t v);

// Fault injection (SURVEY.md §5 "failure detection"): OAP_MLLIB_FAULT="<rank>:<phase>:<iter>"
// makes that rank throw CommError (mode "raise") or _exit (OAP_MLLIB_FAULT_MODE=exit) when it
// reaches the named phase at the given iteration, so tests can check that no peer hangs.
void maybe_inject_fault(int rank, const char* phase, int iteration);

}  // namespace oap
