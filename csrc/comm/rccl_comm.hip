// RCCL communicator: one rank per GPU, collectives over xGMI.
//
// Bootstrap: the ncclUniqueId is created by rank 0 and shared over the TCP control channel
// (the MI355X-native replacement of the reference's TCP command socket, slave.py:5-16).
// Data plane: the shuffle is ONE grouped ncclSend/ncclRecv per peer (an all-to-all-v), so
// every point-to-point xGMI link of the node carries 1/P of each rank's records at once
// -- unlike a ring, which would serialise on one link per step.  The self bucket is a
// device-to-device copy.  Small control collectives (samples, counts, totals) are
// ncclAllGather on a device staging buffer.  The gather strategy's slots are one
// ncclAllGather enqueued on the engine's own stream right behind the map (no host round
// trip; allgather_device).  Every wait polls ncclCommGetAsyncError with a timeout and
// aborts the communicator instead of hanging.
//
// RCCL is loaded on first use (dlopen), not linked: a single-GPU job -- the CLI's default,
// the headline bench -- never maps librccl.so and its code objects.
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <atomic>
#include <cstdlib>
#include <memory>
#include <cstring>
#include <mutex>
#include <thread>

#include "locust/dist.hpp"
#include "locust/hip_check.hpp"
#include "locust/shm.hpp"

#define LOCUST_RCCL_CHECK(expr)                                                        \
  do {                                                                                 \
    ncclResult_t _r = (expr);                                                          \
    if (_r != ncclSuccess)                                                             \
      ::locust::throw_error(__FILE__, __LINE__,                                        \
                            std::string("RCCL error: ") + rccl().GetErrorString(_r) +  \
                                " in `" #expr "`");                                    \
  } while (0)

namespace locust {
namespace {

// The RCCL entry points this communicator uses, resolved from librccl on first use.
struct RcclApi {
#define LOCUST_RCCL_FNS(X)                                                            \
  X(GetErrorString) X(GetUniqueId) X(CommInitRank) X(CommInitAll) X(CommAbort)         \
  X(CommDestroy) X(CommCount) X(CommGetAsyncError) X(AllGather) X(AllToAll)           \
  X(Send) X(Recv) X(GroupStart) X(GroupEnd)
#define LOCUST_RCCL_PTR(name) decltype(&nccl##name) name = nullptr;
  LOCUST_RCCL_FNS(LOCUST_RCCL_PTR)
#undef LOCUST_RCCL_PTR
  void* lib = nullptr;
};

const RcclApi& rccl() {
  static RcclApi api;
  static std::once_flag once;
  static std::string err;
  std::call_once(once, [] {
    // the soname first (ld.so.cache / LD_LIBRARY_PATH), then the ROCm install itself
    for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
      api.lib = dlopen(name, RTLD_NOW | RTLD_LOCAL);
      if (api.lib) break;
    }
    if (!api.lib) {
      const char* e = dlerror();
      err = std::string("cannot load librccl.so: ") + (e ? e : "not found");
      return;
    }
#define LOCUST_RCCL_SYM(name)                                                          \
  api.name = reinterpret_cast<decltype(api.name)>(dlsym(api.lib, "nccl" #name));        \
  if (!api.name && err.empty()) err = "librccl.so lacks nccl" #name;
    LOCUST_RCCL_FNS(LOCUST_RCCL_SYM)
#undef LOCUST_RCCL_SYM
    if (err.empty()) LOCUST_LOG_DEBUG("RCCL loaded on first use");
  });
  if (!err.empty()) throw Error(err);
  return api;
}

class RcclComm final : public Communicator {
 public:
  RcclComm(int rank, int world, int device, const std::string& host, int port, double timeout_s,
           int listen_fd)
      : rank_(rank), world_(world), timeout_s_(timeout_s) {
    tcp_ = make_tcp_comm(rank, world, host, port, timeout_s, listen_fd);
    group_ = tcp_->group_id();
    ncclUniqueId id;
    if (rank == 0) LOCUST_RCCL_CHECK(rccl().GetUniqueId(&id));
    std::vector<ncclUniqueId> ids((size_t)world);
    tcp_->allgather_host(&id, ids.data(), sizeof(id));
    id = ids[0];
    LOCUST_HIP_CHECK(hipSetDevice(device));
    LOCUST_HIP_CHECK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    // The slot job captures its all-gather into a hipGraph (graph_capturable).  The
    // package sets NCCL_GRAPH_REGISTER=0 at import / CLI start (before any thread or RCCL
    // use; a user's setting wins) so captured collectives stay on RCCL's own connection
    // buffers instead of IPC-registering our slot buffers; log what is in effect.
    LOCUST_LOG_DEBUG("rccl rank %d/%d on device %d, NCCL_GRAPH_REGISTER=%s", rank, world,
        device, std::getenv("NCCL_GRAPH_REGISTER") ? std::getenv("NCCL_GRAPH_REGISTER") : "(unset)");
    LOCUST_RCCL_CHECK(rccl().CommInitRank(&comm_, world, id, rank));
    stage_cap_ = 1 << 20;
    LOCUST_HIP_CHECK(hipMalloc(&d_stage_, stage_cap_ * (u64)(world + 1)));
    LOCUST_HIP_CHECK(hipHostMalloc(&h_stage_, stage_cap_ * (u64)(world + 1), hipHostMallocDefault));
  }

  // One rank of a single-process clique (ncclCommInitAll): no TCP bootstrap.  The calling
  // thread drives `device`; every rank of the clique runs on its own thread.
  RcclComm(ncclComm_t comm, int rank, int world, int device, double timeout_s,
           std::shared_ptr<std::atomic<bool>> group_abort, u64 group)
      : rank_(rank), world_(world), timeout_s_(timeout_s), group_abort_(std::move(group_abort)),
        comm_(comm), group_(group) {
    LOCUST_HIP_CHECK(hipSetDevice(device));
    LOCUST_HIP_CHECK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    stage_cap_ = 1 << 20;
    LOCUST_HIP_CHECK(hipMalloc(&d_stage_, stage_cap_ * (u64)(world + 1)));
    LOCUST_HIP_CHECK(hipHostMalloc(&h_stage_, stage_cap_ * (u64)(world + 1), hipHostMallocDefault));
  }

  ~RcclComm() override {
    if (comm_) {
      if (aborted_)
        (void)rccl().CommAbort(comm_);
      else
        (void)rccl().CommDestroy(comm_);
    }
    if (d_stage_) (void)hipFree(d_stage_);
    if (h_stage_) (void)hipHostFree(h_stage_);
    if (d_gsend_) (void)hipFree(d_gsend_);
    if (d_grecv_) (void)hipFree(d_grecv_);
    if (stream_) (void)hipStreamDestroy(stream_);
  }

  int rank() const override { return rank_; }
  int size() const override { return world_; }
  const char* name() const override { return "rccl"; }
  int comm_count() const override {
    int n = -1;
    return rccl().CommCount(comm_, &n) == ncclSuccess ? n : -1;
  }
  bool device_buffers() const override { return true; }
  u64 group_id() const override { return group_; }
  bool in_process() const override { return !tcp_; }  // a clique member (no TCP bootstrap)

  void allgather_host(const void* send, void* recv, u64 bytes) override {
    ensure_stage(bytes);
    char* dsend = d_stage_ + (u64)world_ * stage_cap_;
    // through the pinned slot: a pageable H2D would be a synchronous staged copy
    char* hsend = h_stage_ + (u64)world_ * stage_cap_;
    std::memcpy(hsend, send, bytes);
    LOCUST_HIP_CHECK(hipMemcpyAsync(dsend, hsend, bytes, hipMemcpyHostToDevice, stream_));
    LOCUST_RCCL_CHECK(rccl().AllGather(dsend, d_stage_, bytes, ncclUint8, comm_, stream_));
    LOCUST_HIP_CHECK(hipMemcpyAsync(h_stage_, d_stage_, bytes * (u64)world_,
                                    hipMemcpyDeviceToHost, stream_));
    wait(stream_);
    std::memcpy(recv, h_stage_, bytes * (u64)world_);
  }

  void gatherv_host(const void* send, u64 bytes, std::vector<char>* recv_at_root,
                    std::vector<u64>* sizes_at_root, int root) override {
    std::vector<u64> sizes((size_t)world_);
    allgather_host(&bytes, sizes.data(), sizeof(u64));
    u64 total = 0;
    for (u64 s : sizes) total += s;
    if (rank_ == root) recv_at_root->resize(total);
    gatherv_known(send, bytes, sizes.data(), rank_ == root ? recv_at_root->data() : nullptr, root);
    if (rank_ == root && sizes_at_root) *sizes_at_root = sizes;
  }

  // Payload over grouped send/recv through persistent device staging buffers.
  void gatherv_known(const void* send, u64 bytes, const u64* sizes, void* recv_at_root,
                     int root) override {
    u64 total = 0;
    for (int r = 0; r < world_; ++r) total += sizes[r];
    ensure_gather(std::max<u64>(bytes, 1), rank_ == root ? std::max<u64>(total, 1) : 1);
    if (bytes) LOCUST_HIP_CHECK(hipMemcpyAsync(d_gsend_, send, bytes, hipMemcpyHostToDevice, stream_));
    if (rank_ == root && bytes) {
      u64 off = 0;
      for (int r = 0; r < root; ++r) off += sizes[r];
      LOCUST_HIP_CHECK(hipMemcpyAsync(d_grecv_ + off, d_gsend_, bytes, hipMemcpyDeviceToDevice, stream_));
    }
    LOCUST_RCCL_CHECK(rccl().GroupStart());
    if (rank_ == root) {
      u64 off = 0;
      for (int r = 0; r < world_; ++r) {
        if (r != root && sizes[r])
          LOCUST_RCCL_CHECK(rccl().Recv(d_grecv_ + off, sizes[r], ncclUint8, r, comm_, stream_));
        off += sizes[r];
      }
    } else if (bytes) {
      LOCUST_RCCL_CHECK(rccl().Send(d_gsend_, bytes, ncclUint8, root, comm_, stream_));
    }
    LOCUST_RCCL_CHECK(rccl().GroupEnd());
    if (rank_ == root && total)
      LOCUST_HIP_CHECK(hipMemcpyAsync(recv_at_root, d_grecv_, total, hipMemcpyDeviceToHost, stream_));
    wait(stream_);
  }

  void barrier() override {
    int v = 0;
    std::vector<int> all((size_t)world_);
    allgather_host(&v, all.data(), sizeof(int));
  }

  void allgather_device(const void* send, void* recv, u64 bytes, void* stream) override {
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : stream_;
    LOCUST_RCCL_CHECK(rccl().AllGather(send, recv, bytes, ncclUint8, comm_, s));
  }

  // ncclAllToAll: every peer's chunk over its own xGMI link at once (no ring).
  void alltoall_device(const void* send, void* recv, u64 bytes, void* stream) override {
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : stream_;
    LOCUST_RCCL_CHECK(rccl().AllToAll(send, recv, bytes, ncclUint8, comm_, s));
  }

  // Root receives every other rank's chunk (grouped point-to-point: P-1 links in
  // parallel into the root); only the root needs the data, so no all-gather.
  void gather_device(const void* send, void* recv, u64 bytes, int root, void* stream) override {
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : stream_;
    if (world_ == 1 || !bytes) return;
    LOCUST_RCCL_CHECK(rccl().GroupStart());
    if (rank_ == root) {
      for (int r = 0; r < world_; ++r)
        if (r != root)
          LOCUST_RCCL_CHECK(rccl().Recv(static_cast<char*>(recv) + (u64)r * bytes, bytes, ncclUint8,
                                     r, comm_, s));
    } else {
      LOCUST_RCCL_CHECK(rccl().Send(send, bytes, ncclUint8, root, comm_, s));
    }
    LOCUST_RCCL_CHECK(rccl().GroupEnd());
  }

  void sync_stream(void* stream) override {
    wait(stream ? static_cast<hipStream_t>(stream) : stream_);
  }

  bool graph_capturable() const override { return true; }

  void alltoallv(const void* send, const u64* send_bytes, const u64* send_off, void* recv,
                 const u64* recv_bytes, const u64* recv_off, void* stream) override {
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : stream_;
    const char* sb = static_cast<const char*>(send);
    char* rb = static_cast<char*>(recv);
    if (send_bytes[rank_])
      LOCUST_HIP_CHECK(hipMemcpyAsync(rb + recv_off[rank_], sb + send_off[rank_], send_bytes[rank_],
                                      hipMemcpyDeviceToDevice, s));
    LOCUST_RCCL_CHECK(rccl().GroupStart());
    for (int p = 0; p < world_; ++p) {
      if (p == rank_) continue;
      if (send_bytes[p])
        LOCUST_RCCL_CHECK(rccl().Send(sb + send_off[p], send_bytes[p], ncclUint8, p, comm_, s));
      if (recv_bytes[p])
        LOCUST_RCCL_CHECK(rccl().Recv(rb + recv_off[p], recv_bytes[p], ncclUint8, p, comm_, s));
    }
    LOCUST_RCCL_CHECK(rccl().GroupEnd());
    wait(s);
  }

  // The same, stream-ordered: the sizes come from a count matrix every rank holds.
  void alltoallv_device(const void* send, const u64* send_bytes, const u64* send_off, void* recv,
                        const u64* recv_bytes, const u64* recv_off, void* stream) override {
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : stream_;
    const char* sb = static_cast<const char*>(send);
    char* rb = static_cast<char*>(recv);
    if (send_bytes[rank_])
      LOCUST_HIP_CHECK(hipMemcpyAsync(rb + recv_off[rank_], sb + send_off[rank_], send_bytes[rank_],
                                      hipMemcpyDeviceToDevice, s));
    if (world_ == 1) return;
    LOCUST_RCCL_CHECK(rccl().GroupStart());
    for (int p = 0; p < world_; ++p) {
      if (p == rank_) continue;
      if (send_bytes[p])
        LOCUST_RCCL_CHECK(rccl().Send(sb + send_off[p], send_bytes[p], ncclUint8, p, comm_, s));
      if (recv_bytes[p])
        LOCUST_RCCL_CHECK(rccl().Recv(rb + recv_off[p], recv_bytes[p], ncclUint8, p, comm_, s));
    }
    LOCUST_RCCL_CHECK(rccl().GroupEnd());
  }

 private:
  void ensure_gather(u64 send_bytes, u64 recv_bytes) {
    if (send_bytes > gsend_cap_) {
      wait(stream_);
      if (d_gsend_) (void)hipFree(d_gsend_);
      gsend_cap_ = align_up(send_bytes * 2, 1 << 16);
      LOCUST_HIP_CHECK(hipMalloc(&d_gsend_, gsend_cap_));
    }
    if (recv_bytes > grecv_cap_) {
      wait(stream_);
      if (d_grecv_) (void)hipFree(d_grecv_);
      grecv_cap_ = align_up(recv_bytes * 2, 1 << 16);
      LOCUST_HIP_CHECK(hipMalloc(&d_grecv_, grecv_cap_));
    }
  }

  void ensure_stage(u64 bytes) {
    if (bytes <= stage_cap_) return;
    wait(stream_);
    (void)hipFree(d_stage_);
    (void)hipHostFree(h_stage_);
    stage_cap_ = align_up(bytes, 4096);
    LOCUST_HIP_CHECK(hipMalloc(&d_stage_, stage_cap_ * (u64)(world_ + 1)));
    LOCUST_HIP_CHECK(hipHostMalloc(&h_stage_, stage_cap_ * (u64)(world_ + 1), hipHostMallocDefault));
  }

  // Wait for the stream while watching for asynchronous RCCL errors and a timeout.
  void wait(hipStream_t s) {
    const u64 deadline = now_ns() + (u64)(timeout_s_ * 1e9);
    u64 spins = 0;
    for (;;) {
      hipError_t e = hipStreamQuery(s);
      if (e == hipSuccess) return;
      if (e != hipErrorNotReady) LOCUST_HIP_CHECK(e);
      ncclResult_t ae = ncclSuccess;
      LOCUST_RCCL_CHECK(rccl().CommGetAsyncError(comm_, &ae));
      if (ae != ncclSuccess && ae != ncclInProgress) {
        aborted_ = true;
        throw Error(std::string("RCCL async error: ") + rccl().GetErrorString(ae));
      }
      if (now_ns() > deadline) {
        aborted_ = true;
        throw Error("RCCL operation timed out after " + std::to_string(timeout_s_) + " s");
      }
      if (group_abort_ && group_abort_->load(std::memory_order_relaxed)) {
        aborted_ = true;  // another rank of the clique failed: do not wait for it
        throw Error("RCCL clique aborted: another rank failed");
      }
      if (++spins > 1000) std::this_thread::yield();
    }
  }

  int rank_, world_;
  double timeout_s_;
  bool aborted_ = false;
  std::shared_ptr<std::atomic<bool>> group_abort_;
  std::unique_ptr<Communicator> tcp_;
  ncclComm_t comm_ = nullptr;
  u64 group_ = 0;
  hipStream_t stream_ = nullptr;
  char* d_stage_ = nullptr;
  char* h_stage_ = nullptr;
  u64 stage_cap_ = 0;
  char* d_gsend_ = nullptr;
  char* d_grecv_ = nullptr;
  u64 gsend_cap_ = 0, grecv_cap_ = 0;
};

}  // namespace

std::unique_ptr<Communicator> make_rccl_comm(int rank, int world, int device,
                                             const std::string& host, int port, double timeout_s,
                                             int listen_fd) {
  return std::unique_ptr<Communicator>(
      new RcclComm(rank, world, device, host, port, timeout_s, listen_fd));
}

std::vector<RcclCliqueMember> make_rccl_clique(const std::vector<int>& devices) {
  const int n = (int)devices.size();
  LOCUST_CHECK_ARG(n >= 1, "empty device list");
  std::vector<ncclComm_t> comms((size_t)n, nullptr);
  // one process, one communicator per device: RCCL wires the clique over xGMI itself
  LOCUST_RCCL_CHECK(rccl().CommInitAll(comms.data(), n, devices.data()));
  std::vector<RcclCliqueMember> out((size_t)n);
  auto abort = std::make_shared<std::atomic<bool>>(false);
  const u64 group = new_group_token();
  for (int r = 0; r < n; ++r) {
    out[(size_t)r].abort = abort;
    out[(size_t)r].group = group;
    out[(size_t)r].handle = comms[(size_t)r];
    out[(size_t)r].rank = r;
    out[(size_t)r].world = n;
    out[(size_t)r].device = devices[(size_t)r];
  }
  return out;
}

std::unique_ptr<Communicator> make_rccl_clique_comm(const RcclCliqueMember& m, double timeout_s) {
  return std::unique_ptr<Communicator>(
      new RcclComm(static_cast<ncclComm_t>(m.handle), m.rank, m.world, m.device, timeout_s, m.abort,
                   m.group));
}

void release_rccl_clique_member(RcclCliqueMember& m) {
  if (!m.handle) return;
  (void)rccl().CommAbort(static_cast<ncclComm_t>(m.handle));
  m.handle = nullptr;
}

}  // namespace locust
