// Loopback communicator: N virtual ranks (threads) in one process.
//
// RCCL refuses two ranks on one device, and the gpurun box has one GPU, so the
// splitter / partition / all-to-all-v / global-offset logic of the multi-GPU pipeline is
// rehearsed with this communicator: each rank has its own stream and buffers, collectives
// rendezvous through a generation barrier, and the all-to-all-v is a set of
// hipMemcpyAsync pulls from the peers' send buffers (device or host memory alike).
#include <condition_variable>
#include <cstring>
#include <mutex>

#include "locust/dist.hpp"
#include "locust/hip_check.hpp"
#include "locust/shm.hpp"

namespace locust {

struct LoopbackGroup::State {
  int world;
  bool device;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  u64 generation = 0;
  bool failed = false;
  // rendezvous slots
  std::vector<const void*> ptr;
  std::vector<u64> bytes;
  std::vector<const u64*> sb, so;
  std::vector<char> gather_buf;

  u64 group = new_group_token();

  State(int w, bool d) : world(w), device(d), ptr((size_t)w), bytes((size_t)w), sb((size_t)w), so((size_t)w) {}

  void barrier() {
    std::unique_lock<std::mutex> lk(mu);
    const u64 gen = generation;
    if (++arrived == world) {
      arrived = 0;
      ++generation;
      cv.notify_all();
      return;
    }
    const bool ok = cv.wait_for(lk, std::chrono::seconds(300),
                                [&] { return generation != gen || failed; });
    if (failed) throw Error("loopback comm: another rank failed");
    if (!ok) throw Error("loopback comm: barrier timed out (a rank died?)");
  }
  // A rank failed outside a collective: wake every waiter so the group fails fast.
  void abort() {
    std::lock_guard<std::mutex> lk(mu);
    failed = true;
    cv.notify_all();
  }
};

namespace {

class LoopbackComm final : public Communicator {
 public:
  LoopbackComm(std::shared_ptr<LoopbackGroup::State> st, int rank) : st_(std::move(st)), rank_(rank) {}
  int rank() const override { return rank_; }
  int size() const override { return st_->world; }
  const char* name() const override { return "loopback"; }
  bool device_buffers() const override { return st_->device; }
  u64 group_id() const override { return st_->group; }
  bool in_process() const override { return true; }

  void allgather_host(const void* send, void* recv, u64 bytes) override {
    st_->ptr[(size_t)rank_] = send;
    st_->barrier();
    for (int r = 0; r < size(); ++r)
      std::memcpy(static_cast<char*>(recv) + (u64)r * bytes, st_->ptr[(size_t)r], bytes);
    st_->barrier();
  }

  void gatherv_host(const void* send, u64 bytes, std::vector<char>* recv_at_root,
                    std::vector<u64>* sizes_at_root, int root) override {
    st_->ptr[(size_t)rank_] = send;
    st_->bytes[(size_t)rank_] = bytes;
    st_->barrier();
    if (rank_ == root) {
      u64 total = 0;
      for (int r = 0; r < size(); ++r) total += st_->bytes[(size_t)r];
      recv_at_root->resize(total);
      u64 off = 0;
      for (int r = 0; r < size(); ++r) {
        if (st_->bytes[(size_t)r])
          std::memcpy(recv_at_root->data() + off, st_->ptr[(size_t)r], st_->bytes[(size_t)r]);
        off += st_->bytes[(size_t)r];
      }
      if (sizes_at_root) sizes_at_root->assign(st_->bytes.begin(), st_->bytes.end());
    }
    st_->barrier();
  }

  void barrier() override { st_->barrier(); }

  // Blocking rehearsal of the stream-ordered all-gather: the send data must be complete
  // before a peer pulls it, and no rank may overwrite its send buffer before every pull
  // finished -- hence a stream sync before and a barrier after.
  void allgather_device(const void* send, void* recv, u64 bytes, void* stream) override {
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (st_->device) LOCUST_HIP_CHECK(hipStreamSynchronize(s));
    st_->ptr[(size_t)rank_] = send;
    st_->barrier();
    char* out = static_cast<char*>(recv);
    for (int r = 0; r < size(); ++r) {
      if (!bytes) break;
      if (st_->device)
        LOCUST_HIP_CHECK(hipMemcpyAsync(out + (u64)r * bytes, st_->ptr[(size_t)r], bytes,
                                        hipMemcpyDefault, s));
      else
        std::memcpy(out + (u64)r * bytes, st_->ptr[(size_t)r], bytes);
    }
    if (st_->device) LOCUST_HIP_CHECK(hipStreamSynchronize(s));
    st_->barrier();
  }

  // Blocking rehearsals of the stream-ordered all-to-all / gather (see allgather_device).
  void alltoall_device(const void* send, void* recv, u64 bytes, void* stream) override {
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (st_->device) LOCUST_HIP_CHECK(hipStreamSynchronize(s));
    st_->ptr[(size_t)rank_] = send;
    st_->barrier();
    char* out = static_cast<char*>(recv);
    for (int r = 0; r < size() && bytes; ++r) {
      const char* from = static_cast<const char*>(st_->ptr[(size_t)r]) + (u64)rank_ * bytes;
      if (st_->device)
        LOCUST_HIP_CHECK(hipMemcpyAsync(out + (u64)r * bytes, from, bytes, hipMemcpyDefault, s));
      else
        std::memcpy(out + (u64)r * bytes, from, bytes);
    }
    if (st_->device) LOCUST_HIP_CHECK(hipStreamSynchronize(s));
    st_->barrier();
  }

  void gather_device(const void* send, void* recv, u64 bytes, int root, void* stream) override {
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (st_->device) LOCUST_HIP_CHECK(hipStreamSynchronize(s));
    st_->ptr[(size_t)rank_] = send;
    st_->barrier();
    if (rank_ == root) {
      char* out = static_cast<char*>(recv);
      for (int r = 0; r < size() && bytes; ++r) {
        if (r == root) continue;
        if (st_->device)
          LOCUST_HIP_CHECK(hipMemcpyAsync(out + (u64)r * bytes, st_->ptr[(size_t)r], bytes,
                                          hipMemcpyDefault, s));
        else
          std::memcpy(out + (u64)r * bytes, st_->ptr[(size_t)r], bytes);
      }
      if (st_->device) LOCUST_HIP_CHECK(hipStreamSynchronize(s));
    }
    st_->barrier();
  }

  void sync_stream(void* stream) override {
    if (st_->device) LOCUST_HIP_CHECK(hipStreamSynchronize(static_cast<hipStream_t>(stream)));
  }

  // Blocking rehearsal of the stream-ordered all-to-all-v: the send buffers must be
  // complete before a peer pulls from them.
  void alltoallv_device(const void* send, const u64* send_bytes, const u64* send_off, void* recv,
                        const u64* recv_bytes, const u64* recv_off, void* stream) override {
    if (st_->device) LOCUST_HIP_CHECK(hipStreamSynchronize(static_cast<hipStream_t>(stream)));
    alltoallv(send, send_bytes, send_off, recv, recv_bytes, recv_off, stream);
  }

  void alltoallv(const void* send, const u64* send_bytes, const u64* send_off, void* recv,
                 const u64* recv_bytes, const u64* recv_off, void* stream) override {
    st_->ptr[(size_t)rank_] = send;
    st_->sb[(size_t)rank_] = send_bytes;
    st_->so[(size_t)rank_] = send_off;
    st_->barrier();
    char* out = static_cast<char*>(recv);
    for (int src = 0; src < size(); ++src) {
      const u64 n = st_->sb[(size_t)src][rank_];
      if (n != recv_bytes[src])
        throw Error("loopback comm: recv size mismatch from rank " + std::to_string(src));
      if (!n) continue;
      const char* from = static_cast<const char*>(st_->ptr[(size_t)src]) + st_->so[(size_t)src][rank_];
      if (st_->device) {
        LOCUST_HIP_CHECK(hipMemcpyAsync(out + recv_off[src], from, n, hipMemcpyDefault,
                                        static_cast<hipStream_t>(stream)));
      } else {
        std::memcpy(out + recv_off[src], from, n);
      }
    }
    if (st_->device) LOCUST_HIP_CHECK(hipStreamSynchronize(static_cast<hipStream_t>(stream)));
    st_->barrier();  // senders may reuse their buffers only after every pull finished
  }

 private:
  std::shared_ptr<LoopbackGroup::State> st_;
  int rank_;
};

}  // namespace

LoopbackGroup::LoopbackGroup(int world, bool device_buffers)
    : state_(std::make_shared<State>(world, device_buffers)) {
  LOCUST_CHECK_ARG(world >= 1, "loopback world must be >= 1");
}
LoopbackGroup::~LoopbackGroup() = default;
void LoopbackGroup::abort() { state_->abort(); }

std::unique_ptr<Communicator> LoopbackGroup::comm(int rank) {
  LOCUST_CHECK_ARG(rank >= 0 && rank < state_->world, "bad loopback rank");
  return std::unique_ptr<Communicator>(new LoopbackComm(state_, rank));
}

}  // namespace locust
