// TCP rendezvous and host collectives: the reference's KVS bootstrap contract
// (OneCCL.init(size, rank, "ip_port") -> ccl::create_main_kvs / create_communicator,
// mllib-dal/src/main/native/OneCCL.cpp:47-86; the port comes from the executors' bind scan,
// OneCCL.cpp:207-247) without oneCCL:
//   * TcpStore: rank 0 listens on ip:port, every other rank connects to it (retrying until the
//     timeout) and identifies itself; afterwards rank 0 holds one socket per peer.  GPU worlds
//     use it once, to hand rank 0's RCCL unique id to everyone (then RCCL takes over).
//   * TcpComm: a host-memory Comm over those sockets for CPU-engine worlds (the reference's
//     host-byte collectives over OFI sockets), star-routed through rank 0.  Reductions run in
//     rank order on rank 0 and the result is sent back, so every rank holds bitwise the same
//     value.  Every socket carries a receive / send timeout: a dead peer raises CommError
//     instead of hanging the world (the reference has no collective timeout).
#pragma once

#include <memory>
#include <string>
#include <vector>

#include "comm/comm.h"

namespace oap {

// "ip_port" (the reference's KVS string, KMeansDALImpl.scala:46) or "ip:port" -> (ip, port);
// false when `s` is neither.
bool parse_kvs_address(const std::string& s, std::string* ip, int* port);

class TcpStore {
 public:
  TcpStore(const std::string& ip, int port, int world, int rank, double timeout_s);
  ~TcpStore();
  TcpStore(const TcpStore&) = delete;
  TcpStore& operator=(const TcpStore&) = delete;
  int rank() const { return rank_; }
  int world() const { return world_; }
  // Blocking exact-size transfers between rank 0 and peer p (rank 0 side) / rank 0 (peer side).
  void send_to(int peer, const void* data, size_t bytes);
  void recv_from(int peer, void* data, size_t bytes);
  // rank 0's `bytes` -> every rank
  void broadcast(void* data, size_t bytes);

 private:
  int fd_for(int peer) const;
  int world_, rank_;
  double timeout_s_;
  int listen_fd_ = -1;
  std::vector<int> peers_;  // rank 0: socket per rank (index 0 unused); others: [0] = to rank 0
};

class TcpComm final : public Comm {
 public:
  explicit TcpComm(std::shared_ptr<TcpStore> store) : store_(std::move(store)) {}
  int rank() const override { return store_->rank(); }
  int size() const override { return store_->world(); }
  bool on_device() const override { return false; }
  const char* name() const override { return "tcp"; }
  void allreduce(void* buf, size_t count, DType dt, ReduceOp op, hipStream_t s) override;
  void allgather(const void* send, void* recv, size_t count, DType dt, hipStream_t s) override;
  void alltoallv(const void* send, const std::vector<size_t>& send_counts, void* recv,
                 const std::vector<size_t>& recv_counts, DType dt, hipStream_t s) override;
  void bcast(void* buf, size_t count, DType dt, int root, hipStream_t s) override;
  void barrier() override;

 private:
  std::shared_ptr<TcpStore> store_;
};

}  // namespace oap
