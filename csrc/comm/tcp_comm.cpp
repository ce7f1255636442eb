// Star-topology TCP communicator.
//
// The reference's only inter-node channel is a one-shot TCP command socket bound to a
// hard-coded 127.0.0.1:1337 with a bare `except:` and a blind "ACK"
// (/root/reference/Distributor/slave.py:5-24).  This communicator is the
// framework's control plane: framed messages, timeouts on every socket, connection
// retries during bootstrap, and errors that name the peer.  Rank 0 relays (star), which
// is fine for control messages and for the CPU backend's test-sized data plane; the GPU
// data plane is RCCL (rccl_comm.hip).
#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <cstring>
#include <thread>

#include "locust/dist.hpp"
#include "locust/shm.hpp"

namespace locust {

int Communicator::agree(int local_error) {
  std::vector<int> all((size_t)size());
  int mine = local_error ? 1 : 0;
  allgather_host(&mine, all.data(), sizeof(int));
  for (int r = 0; r < size(); ++r)
    if (all[(size_t)r]) return r;
  return -1;
}

void Communicator::allgather_device(const void*, void*, u64, void*) {
  throw Error(std::string("allgather_device: the ") + name() +
              " communicator has no device data plane");
}

void Communicator::alltoall_device(const void*, void*, u64, void*) {
  throw Error(std::string("alltoall_device: the ") + name() +
              " communicator has no device data plane");
}

void Communicator::gather_device(const void*, void*, u64, int, void*) {
  throw Error(std::string("gather_device: the ") + name() +
              " communicator has no device data plane");
}

void Communicator::alltoallv_device(const void*, const u64*, const u64*, void*, const u64*,
                                    const u64*, void*) {
  throw Error(std::string("alltoallv_device: the ") + name() +
              " communicator has no device data plane");
}

void Communicator::sync_stream(void*) {
  throw Error(std::string("sync_stream: the ") + name() + " communicator has no device streams");
}

void Communicator::gatherv_known(const void* send, u64 bytes, const u64* sizes,
                                 void* recv_at_root, int root) {
  std::vector<char> buf;
  gatherv_host(send, bytes, &buf, nullptr, root);
  u64 total = 0;
  for (int r = 0; r < size(); ++r) total += sizes[r];
  if (rank() == root && total) {
    if (buf.size() != total) throw Error("gatherv_known: size mismatch");
    std::memcpy(recv_at_root, buf.data(), total);
  }
}

namespace {

void set_timeouts(int fd, double timeout_s) {
  timeval tv;
  tv.tv_sec = (time_t)timeout_s;
  tv.tv_usec = (suseconds_t)((timeout_s - (double)tv.tv_sec) * 1e6);
  setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
  setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof(tv));
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
}

void send_all(int fd, const void* data, u64 n, int peer) {
  const char* p = static_cast<const char*>(data);
  while (n) {
    ssize_t k = ::send(fd, p, (size_t)std::min<u64>(n, 1u << 30), MSG_NOSIGNAL);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0)
      throw Error("tcp comm: send to rank " + std::to_string(peer) + " failed: " +
                  std::strerror(errno));
    p += k;
    n -= (u64)k;
  }
}

void recv_all(int fd, void* data, u64 n, int peer) {
  char* p = static_cast<char*>(data);
  while (n) {
    ssize_t k = ::recv(fd, p, (size_t)std::min<u64>(n, 1u << 30), 0);
    if (k < 0 && errno == EINTR) continue;
    if (k == 0) throw Error("tcp comm: rank " + std::to_string(peer) + " closed the connection");
    if (k < 0)
      throw Error("tcp comm: receive from rank " + std::to_string(peer) + " failed: " +
                  std::strerror(errno) + (errno == EAGAIN ? " (timeout)" : ""));
    p += k;
    n -= (u64)k;
  }
}

sockaddr_in resolve(const std::string& host, int port) {
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons((uint16_t)port);
  if (inet_pton(AF_INET, host.c_str(), &a.sin_addr) != 1) {
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_INET;
    if (getaddrinfo(host.c_str(), nullptr, &hints, &res) != 0 || !res)
      throw Error("tcp comm: cannot resolve " + host);
    a.sin_addr = reinterpret_cast<sockaddr_in*>(res->ai_addr)->sin_addr;
    freeaddrinfo(res);
  }
  return a;
}

class TcpComm final : public Communicator {
 public:
  TcpComm(int rank, int world, const std::string& host, int port, double timeout_s,
          int listen_fd)
      : rank_(rank), world_(world), fds_((size_t)world, -1) {
    LOCUST_CHECK_ARG(world >= 1 && rank >= 0 && rank < world, "bad rank/world");
    if (rank == 0 && listen_fd >= 0) listen_fd_ = listen_fd;  // owned from here on
    group_ = new_group_token();  // rank 0's is sent to every peer with the handshake
    if (world == 1) return;
    // A throwing constructor runs no destructor: close what the handshake opened (and the
    // inherited listener) before rethrowing, so a failed bootstrap holds no port.
    try {
      handshake(host, port, timeout_s);
    } catch (...) {
      close_all();
      throw;
    }
  }

  ~TcpComm() override { close_all(); }

 private:
  void close_all() {
    for (int& fd : fds_)
      if (fd >= 0) {
        ::close(fd);
        fd = -1;
      }
    if (listen_fd_ >= 0) {
      ::close(listen_fd_);
      listen_fd_ = -1;
    }
  }
  void handshake(const std::string& host, int port, double timeout_s) {
    const int rank = rank_, world = world_;
    if (rank == 0 && listen_fd_ >= 0) {
      // inherited: already bound to `port` and listening (no window for another process)
    } else if (rank == 0) {
      sockaddr_in addr = resolve(host, port);
      listen_fd_ = ::socket(AF_INET, SOCK_STREAM, 0);
      int one = 1;
      setsockopt(listen_fd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
      if (::bind(listen_fd_, reinterpret_cast<sockaddr*>(&addr), sizeof(addr)) != 0)
        throw Error("tcp comm: bind " + host + ":" + std::to_string(port) + " failed: " +
                    std::strerror(errno));
      ::listen(listen_fd_, world);
    }
    if (rank == 0) {
      set_timeouts(listen_fd_, timeout_s);
      for (int i = 1; i < world; ++i) {
        int fd = ::accept(listen_fd_, nullptr, nullptr);
        if (fd < 0)
          throw Error("tcp comm: accept failed (" + std::to_string(i - 1) + " of " +
                      std::to_string(world - 1) + " peers joined): " + std::strerror(errno));
        set_timeouts(fd, timeout_s);
        int r = -1;
        recv_all(fd, &r, sizeof(r), -1);
        if (r <= 0 || r >= world || fds_[(size_t)r] >= 0) {
          ::close(fd);
          throw Error("tcp comm: bad hello from rank " + std::to_string(r));
        }
        fds_[(size_t)r] = fd;
      }
      for (int r = 1; r < world; ++r) send_all(fds_[(size_t)r], &group_, sizeof(group_), r);
    } else {
      sockaddr_in addr = resolve(host, port);
      const u64 deadline = now_ns() + (u64)(timeout_s * 1e9);
      int fd = -1;
      for (;;) {
        fd = ::socket(AF_INET, SOCK_STREAM, 0);
        if (::connect(fd, reinterpret_cast<sockaddr*>(&addr), sizeof(addr)) == 0) break;
        ::close(fd);
        if (now_ns() > deadline)
          throw Error("tcp comm: rank " + std::to_string(rank) + " could not connect to " + host +
                      ":" + std::to_string(port));
        std::this_thread::sleep_for(std::chrono::milliseconds(20));
      }
      fds_[0] = fd;  // owned (closed by close_all on a failed handshake)
      set_timeouts(fd, timeout_s);
      send_all(fd, &rank_, sizeof(rank_), 0);
      recv_all(fd, &group_, sizeof(group_), 0);
    }
  }

 public:
  int rank() const override { return rank_; }
  int size() const override { return world_; }
  const char* name() const override { return "tcp"; }
  bool device_buffers() const override { return false; }
  u64 group_id() const override { return group_; }

  void allgather_host(const void* send, void* recv, u64 bytes) override {
    char* out = static_cast<char*>(recv);
    std::memcpy(out + (u64)rank_ * bytes, send, bytes);
    if (world_ == 1) return;
    if (rank_ == 0) {
      for (int r = 1; r < world_; ++r) recv_all(fds_[(size_t)r], out + (u64)r * bytes, bytes, r);
      for (int r = 1; r < world_; ++r) send_all(fds_[(size_t)r], out, bytes * (u64)world_, r);
    } else {
      send_all(fds_[0], send, bytes, 0);
      recv_all(fds_[0], out, bytes * (u64)world_, 0);
    }
  }

  void gatherv_host(const void* send, u64 bytes, std::vector<char>* recv_at_root,
                    std::vector<u64>* sizes_at_root, int root) override {
    LOCUST_CHECK_ARG(root == 0, "tcp comm gathers to rank 0 only");
    if (rank_ == 0) {
      std::vector<u64> sizes((size_t)world_);
      sizes[0] = bytes;
      for (int r = 1; r < world_; ++r) recv_all(fds_[(size_t)r], &sizes[(size_t)r], 8, r);
      u64 total = 0;
      for (u64 s : sizes) total += s;
      recv_at_root->resize(total);
      u64 off = 0;
      if (bytes) std::memcpy(recv_at_root->data(), send, bytes);
      off += bytes;
      for (int r = 1; r < world_; ++r) {
        recv_all(fds_[(size_t)r], recv_at_root->data() + off, sizes[(size_t)r], r);
        off += sizes[(size_t)r];
      }
      if (sizes_at_root) *sizes_at_root = sizes;
    } else {
      send_all(fds_[0], &bytes, 8, 0);
      send_all(fds_[0], send, bytes, 0);
    }
  }

  void barrier() override {
    char c = 0;
    std::vector<char> all((size_t)world_);
    allgather_host(&c, all.data(), 1);
  }

  void alltoallv(const void* send, const u64* send_bytes, const u64* send_off, void* recv,
                 const u64* recv_bytes, const u64* recv_off, void*) override {
    const char* s = static_cast<const char*>(send);
    char* out = static_cast<char*>(recv);
    const int P = world_;
    if (P == 1) {
      if (send_bytes[0]) std::memcpy(out + recv_off[0], s + send_off[0], send_bytes[0]);
      return;
    }
    if (rank_ != 0) {
      send_all(fds_[0], send_bytes, 8 * (u64)P, 0);
      for (int d = 0; d < P; ++d) send_all(fds_[0], s + send_off[d], send_bytes[d], 0);
      for (int src = 0; src < P; ++src) recv_all(fds_[0], out + recv_off[src], recv_bytes[src], 0);
      return;
    }
    // root: collect every rank's buckets, then route.
    std::vector<std::vector<u64>> sb((size_t)P, std::vector<u64>((size_t)P));
    std::vector<std::vector<std::vector<char>>> data((size_t)P);
    for (int d = 0; d < P; ++d) sb[0][(size_t)d] = send_bytes[d];
    for (int src = 1; src < P; ++src) {
      recv_all(fds_[(size_t)src], sb[(size_t)src].data(), 8 * (u64)P, src);
      data[(size_t)src].resize((size_t)P);
      for (int d = 0; d < P; ++d) {
        data[(size_t)src][(size_t)d].resize(sb[(size_t)src][(size_t)d]);
        recv_all(fds_[(size_t)src], data[(size_t)src][(size_t)d].data(), sb[(size_t)src][(size_t)d],
                 src);
      }
    }
    for (int src = 0; src < P; ++src) {
      const char* chunk = src == 0 ? s + send_off[0] : data[(size_t)src][0].data();
      const u64 n = sb[(size_t)src][0];
      if (n) std::memcpy(out + recv_off[src], chunk, n);
    }
    for (int d = 1; d < P; ++d) {
      for (int src = 0; src < P; ++src) {
        const char* chunk = src == 0 ? s + send_off[d] : data[(size_t)src][(size_t)d].data();
        send_all(fds_[(size_t)d], chunk, sb[(size_t)src][(size_t)d], d);
      }
    }
  }

 private:
  int rank_, world_;
  u64 group_ = 0;
  int listen_fd_ = -1;
  std::vector<int> fds_;
};

}  // namespace

std::unique_ptr<Communicator> make_tcp_comm(int rank, int world, const std::string& host, int port,
                                            double timeout_s, int listen_fd) {
  return std::unique_ptr<Communicator>(new TcpComm(rank, world, host, port, timeout_s, listen_fd));
}

}  // namespace locust
