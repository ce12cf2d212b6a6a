#include "comm/tcp_comm.h"

#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <thread>

#include "runtime/log.h"
#include "runtime/knobs.h"

namespace oap {

namespace {

constexpr uint32_t kHello = 0x4f415031;  // "OAP1"

void set_timeouts(int fd, double timeout_s) {
  if (timeout_s <= 0) return;
  struct timeval tv;
  tv.tv_sec = static_cast<time_t>(timeout_s);
  tv.tv_usec = static_cast<suseconds_t>((timeout_s - double(tv.tv_sec)) * 1e6);
  setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
  setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof(tv));
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
}

void send_all(int fd, const void* data, size_t bytes) {
  const char* p = static_cast<const char*>(data);
  while (bytes > 0) {
    const ssize_t n = ::send(fd, p, bytes, MSG_NOSIGNAL);
    if (n < 0 && errno == EINTR) continue;
    if (n <= 0)
      OAP_THROW(CommError, "tcp comm: send failed (" << (n < 0 ? std::strerror(errno) : "closed")
                                                     << ")");
    p += n;
    bytes -= size_t(n);
  }
}

void recv_all(int fd, void* data, size_t bytes) {
  char* p = static_cast<char*>(data);
  while (bytes > 0) {
    const ssize_t n = ::recv(fd, p, bytes, 0);
    if (n < 0 && errno == EINTR) continue;
    if (n == 0) OAP_THROW(CommError, "tcp comm: peer closed the connection");
    if (n < 0)
      OAP_THROW(CommError, "tcp comm: receive failed ("
                               << (errno == EAGAIN || errno == EWOULDBLOCK ? "timeout"
                                                                           : std::strerror(errno))
                               << ")");
    p += n;
    bytes -= size_t(n);
  }
}

template <typename T>
void reduce_into(T* dst, const T* src, size_t n, ReduceOp op) {
  switch (op) {
    case ReduceOp::Sum:
      for (size_t i = 0; i < n; ++i) dst[i] = dst[i] + src[i];
      break;
    case ReduceOp::Max:
      for (size_t i = 0; i < n; ++i) dst[i] = std::max(dst[i], src[i]);
      break;
    case ReduceOp::Min:
      for (size_t i = 0; i < n; ++i) dst[i] = std::min(dst[i], src[i]);
      break;
  }
}

void reduce_any(void* dst, const void* src, size_t n, DType dt, ReduceOp op) {
  switch (dt) {
    case DType::F32:
      reduce_into(static_cast<float*>(dst), static_cast<const float*>(src), n, op);
      return;
    case DType::F64:
      reduce_into(static_cast<double*>(dst), static_cast<const double*>(src), n, op);
      return;
    case DType::I32:
      reduce_into(static_cast<int32_t*>(dst), static_cast<const int32_t*>(src), n, op);
      return;
    case DType::I64:
      reduce_into(static_cast<int64_t*>(dst), static_cast<const int64_t*>(src), n, op);
      return;
    case DType::U8:
      reduce_into(static_cast<uint8_t*>(dst), static_cast<const uint8_t*>(src), n, op);
      return;
    case DType::BF16:
      break;
  }
  OAP_THROW(CommError, "tcp comm: no host reduction for bf16");
}

}  // namespace

bool parse_kvs_address(const std::string& s, std::string* ip, int* port) {
  const size_t cut = s.find_last_of("_:");
  if (cut == std::string::npos || cut == 0 || cut + 1 >= s.size()) return false;
  const std::string host = s.substr(0, cut), p = s.substr(cut + 1);
  if (p.find_first_not_of("0123456789") != std::string::npos || p.size() > 5) return false;
  struct in_addr a;
  if (inet_pton(AF_INET, host.c_str(), &a) != 1) return false;
  const int v = std::stoi(p);
  if (v <= 0 || v > 65535) return false;
  *ip = host;
  *port = v;
  return true;
}

TcpStore::TcpStore(const std::string& ip, int port, int world, int rank, double timeout_s)
    : world_(world), rank_(rank), timeout_s_(timeout_s) {
  OAP_CHECK(world >= 1 && rank >= 0 && rank < world, "bad world/rank " << world << "/" << rank);
  struct sockaddr_in sa;
  std::memset(&sa, 0, sizeof(sa));
  sa.sin_family = AF_INET;
  sa.sin_port = htons(static_cast<uint16_t>(port));
  OAP_CHECK(inet_pton(AF_INET, ip.c_str(), &sa.sin_addr) == 1, "bad rendezvous ip " << ip);
  const auto t0 = std::chrono::steady_clock::now();
  auto elapsed = [&] {
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  };
  if (rank == 0) {
    peers_.assign(world, -1);
    listen_fd_ = ::socket(AF_INET, SOCK_STREAM, 0);
    OAP_CHECK(listen_fd_ >= 0, "tcp store: socket()");
    int one = 1;
    setsockopt(listen_fd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    if (::bind(listen_fd_, reinterpret_cast<struct sockaddr*>(&sa), sizeof(sa)) != 0 ||
        ::listen(listen_fd_, std::max(world, 16)) != 0) {
      const std::string err = std::strerror(errno);
      ::close(listen_fd_);
      listen_fd_ = -1;
      OAP_THROW(CommError, "tcp store: cannot listen on " << ip << ":" << port << " (" << err
                                                          << ")");
    }
    set_timeouts(listen_fd_, timeout_s);  // (accept honours SO_RCVTIMEO)
    for (int got = 1; got < world;) {
      const int fd = ::accept(listen_fd_, nullptr, nullptr);
      if (fd < 0) {
        if (errno == EINTR) continue;
        OAP_THROW(CommError, "tcp store: " << got - 1 << " of " << world - 1
                                           << " ranks joined before the timeout");
      }
      set_timeouts(fd, timeout_s);
      uint32_t hello[2] = {0, 0};
      try {
        recv_all(fd, hello, sizeof(hello));
      } catch (...) {
        ::close(fd);
        throw;
      }
      const int r = int(hello[1]);
      if (hello[0] != kHello || r <= 0 || r >= world || peers_[r] >= 0) {
        ::close(fd);
        OAP_THROW(CommError, "tcp store: bad or duplicate hello (rank " << r << ")");
      }
      peers_[r] = fd;
      ++got;
    }
  } else {
    peers_.assign(1, -1);
    for (;;) {  // rank 0 may not be listening yet: retry until the timeout
      const int fd = ::socket(AF_INET, SOCK_STREAM, 0);
      OAP_CHECK(fd >= 0, "tcp store: socket()");
      if (::connect(fd, reinterpret_cast<struct sockaddr*>(&sa), sizeof(sa)) == 0) {
        set_timeouts(fd, timeout_s);
        peers_[0] = fd;
        break;
      }
      ::close(fd);
      if (timeout_s > 0 && elapsed() > timeout_s)
        OAP_THROW(CommError, "tcp store: rank 0 at " << ip << ":" << port << " not reachable");
      std::this_thread::sleep_for(std::chrono::milliseconds(20));
    }
    const uint32_t hello[2] = {kHello, uint32_t(rank)};
    send_all(peers_[0], hello, sizeof(hello));
  }
  // every rank has joined once rank 0 releases them
  uint32_t go = kHello;
  broadcast(&go, sizeof(go));
  OAP_CHECK(go == kHello, "tcp store: bad release");
  Logger::instance().log(LogLevel::Info, "comm/tcp_store",
                         "\"world\":" + std::to_string(world) + ",\"port\":" +
                             std::to_string(port));
}

TcpStore::~TcpStore() {
  for (int fd : peers_)
    if (fd >= 0) ::close(fd);
  if (listen_fd_ >= 0) ::close(listen_fd_);
}

int TcpStore::fd_for(int peer) const {
  if (rank_ == 0) {
    OAP_CHECK(peer > 0 && peer < world_, "tcp store: bad peer " << peer);
    return peers_[peer];
  }
  OAP_CHECK(peer == 0, "tcp store: star topology (peers talk to rank 0 only)");
  return peers_[0];
}

void TcpStore::send_to(int peer, const void* data, size_t bytes) {
  send_all(fd_for(peer), data, bytes);
}

void TcpStore::recv_from(int peer, void* data, size_t bytes) {
  recv_all(fd_for(peer), data, bytes);
}

void TcpStore::broadcast(void* data, size_t bytes) {
  if (world_ == 1 || bytes == 0) return;
  if (rank_ == 0) {
    for (int p = 1; p < world_; ++p) send_to(p, data, bytes);
  } else {
    recv_from(0, data, bytes);
  }
}

// ------------------------------------------------------------------------------- TcpComm
void TcpComm::allreduce(void* buf, size_t count, DType dt, ReduceOp op, hipStream_t) {
  const size_t bytes = count * dtype_size(dt);
  if (size() == 1 || bytes == 0) return;
  if (rank() == 0) {
    std::vector<char> tmp(bytes);
    for (int p = 1; p < size(); ++p) {  // rank order: the same sum on every run
      store_->recv_from(p, tmp.data(), bytes);
      reduce_any(buf, tmp.data(), count, dt, op);
    }
  } else {
    store_->send_to(0, buf, bytes);
  }
  store_->broadcast(buf, bytes);
}

void TcpComm::allgather(const void* send, void* recv, size_t count, DType dt, hipStream_t) {
  const size_t bytes = count * dtype_size(dt);
  char* out = static_cast<char*>(recv);
  if (send != out + size_t(rank()) * bytes && bytes)
    std::memmove(out + size_t(rank()) * bytes, send, bytes);
  if (size() == 1 || bytes == 0) return;
  if (rank() == 0) {
    for (int p = 1; p < size(); ++p) store_->recv_from(p, out + size_t(p) * bytes, bytes);
  } else {
    store_->send_to(0, out + size_t(rank()) * bytes, bytes);
  }
  store_->broadcast(out, bytes * size());
}

void TcpComm::bcast(void* buf, size_t count, DType dt, int root, hipStream_t) {
  const size_t bytes = count * dtype_size(dt);
  if (size() == 1 || bytes == 0) return;
  OAP_CHECK(root >= 0 && root < size(), "bcast: bad root " << root);
  if (root != 0) {  // root -> 0, then 0 -> everyone
    if (rank() == root) store_->send_to(0, buf, bytes);
    if (rank() == 0) store_->recv_from(root, buf, bytes);
  }
  store_->broadcast(buf, bytes);
}

void TcpComm::alltoallv(const void* send, const std::vector<size_t>& send_counts, void* recv,
                        const std::vector<size_t>& recv_counts, DType dt, hipStream_t) {
  // Star-routed, but streamed: for each source rank in order, rank 0 receives that source's
  // segment for one destination at a time, in pieces of at most kPiece bytes, and forwards
  // each piece before reading the next — rank 0 holds one piece, never the world's exchange.
  // Every rank follows the same (source, destination) order, so the blocking sockets cannot
  // deadlock; a rank's segment to itself never leaves the rank.
  const int P = size(), me = rank();
  OAP_CHECK(int(send_counts.size()) == P && int(recv_counts.size()) == P,
            "alltoallv: counts must have one entry per rank");
  const size_t es = dtype_size(dt);
  // (OAP_TCP_PIECE_BYTES overrides the 64 MiB forwarding piece: tests drive several pieces)
  const size_t kPiece = [] {  // (read per call: tests set it mid-process)
    const int64_t v = knob_int("OAP_TCP_PIECE_BYTES");
    return v > 0 ? size_t(v) : size_t(64) << 20;
  }();
  std::vector<size_t> soff(P + 1, 0), roff(P + 1, 0);
  for (int q = 0; q < P; ++q) {
    soff[q + 1] = soff[q] + send_counts[q];
    roff[q + 1] = roff[q] + recv_counts[q];
  }
  const char* sb = static_cast<const char*>(send);
  char* rb = static_cast<char*>(recv);
  OAP_CHECK(send_counts[me] == recv_counts[me], "alltoallv: own segment counts disagree");
  if (send_counts[me]) std::memmove(rb + roff[me] * es, sb + soff[me] * es, send_counts[me] * es);
  if (P == 1) return;
  // rank 0 learns every (source, destination) count (one small gather)
  std::vector<uint64_t> mine(send_counts.begin(), send_counts.end());
  std::vector<uint64_t> all;
  if (me == 0) {
    all.resize(size_t(P) * P);
    std::copy(mine.begin(), mine.end(), all.begin());
    for (int p = 1; p < P; ++p) store_->recv_from(p, all.data() + size_t(p) * P, size_t(P) * 8);
  } else {
    store_->send_to(0, mine.data(), size_t(P) * 8);
  }
  std::vector<char> piece;
  for (int src = 0; src < P; ++src) {
    if (me == 0) {
      for (int q = 0; q < P; ++q) {
        if (q == src) continue;
        const size_t n = size_t(all[size_t(src) * P + q]) * es;
        if (q == 0) {  // a peer's segment to rank 0
          OAP_CHECK(n == recv_counts[src] * es, "alltoallv: receive counts disagree");
          if (n) store_->recv_from(src, rb + roff[src] * es, n);
          continue;
        }
        if (src == 0) {  // rank 0's own segment to a peer
          if (n) store_->send_to(q, sb + soff[q] * es, n);
          continue;
        }
        for (size_t done = 0; done < n;) {  // peer -> peer, piece by piece
          const size_t m = std::min(kPiece, n - done);
          piece.resize(m);
          store_->recv_from(src, piece.data(), m);
          store_->send_to(q, piece.data(), m);
          done += m;
        }
      }
    } else if (src == me) {  // my segments to every other rank, in destination order
      for (int q = 0; q < P; ++q)
        if (q != me && send_counts[q]) store_->send_to(0, sb + soff[q] * es, send_counts[q] * es);
    } else if (recv_counts[src]) {  // the segment from src, through rank 0
      store_->recv_from(0, rb + roff[src] * es, recv_counts[src] * es);
    }
  }
}

void TcpComm::barrier() {
  int32_t v = 1;
  allreduce(&v, 1, DType::I32, ReduceOp::Sum, nullptr);
}

}  // namespace oap
