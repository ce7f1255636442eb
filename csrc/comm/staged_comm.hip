// Device data plane staged through a host communicator ("tcpdev"): every rank a process,
// several processes sharing one GPU.
//
// RCCL refuses two ranks on one device, and the pool's boxes have one GPU, so the
// multi-process device paths -- the device exchange with every rank writing into the
// shared host output (a POSIX shm segment each process maps and registers itself), the
// completion stamps the root polls, the output regions -- would otherwise only ever run
// with one rank before a real multi-GPU node runs them.  This wrapper gives a host-only
// communicator (TCP) the device operations of the Communicator interface as blocking
// rehearsals: wait for the stream, copy the device buffers to host memory, run the host
// collective, copy back.  Same bytes, same order of collectives as RCCL; not fast.
#include <cstring>
#include <vector>

#include "locust/dist.hpp"
#include "locust/hip_check.hpp"

namespace locust {
namespace {

class StagedDeviceComm final : public Communicator {
 public:
  explicit StagedDeviceComm(std::unique_ptr<Communicator> host) : h_(std::move(host)) {}

  int rank() const override { return h_->rank(); }
  int size() const override { return h_->size(); }
  const char* name() const override { return "tcpdev"; }
  bool device_buffers() const override { return true; }
  u64 group_id() const override { return h_->group_id(); }

  void allgather_host(const void* send, void* recv, u64 bytes) override {
    h_->allgather_host(send, recv, bytes);
  }
  void gatherv_host(const void* send, u64 bytes, std::vector<char>* recv_at_root,
                    std::vector<u64>* sizes_at_root, int root) override {
    h_->gatherv_host(send, bytes, recv_at_root, sizes_at_root, root);
  }
  void gatherv_known(const void* send, u64 bytes, const u64* sizes, void* recv_at_root,
                     int root) override {
    h_->gatherv_known(send, bytes, sizes, recv_at_root, root);
  }
  void barrier() override { h_->barrier(); }

  // Engine buffers are device memory here: staged both ways.
  void alltoallv(const void* send, const u64* send_bytes, const u64* send_off, void* recv,
                 const u64* recv_bytes, const u64* recv_off, void* stream) override {
    stage_alltoallv(send, send_bytes, send_off, recv, recv_bytes, recv_off, stream);
  }
  void alltoallv_device(const void* send, const u64* send_bytes, const u64* send_off, void* recv,
                        const u64* recv_bytes, const u64* recv_off, void* stream) override {
    stage_alltoallv(send, send_bytes, send_off, recv, recv_bytes, recv_off, stream);
  }

  void allgather_device(const void* send, void* recv, u64 bytes, void* stream) override {
    hipStream_t s = static_cast<hipStream_t>(stream);
    const u64 P = (u64)size();
    out_.resize(std::max<u64>(bytes, 1));
    in_.resize(std::max<u64>(bytes * P, 1));
    to_host(out_.data(), send, bytes, s);
    h_->allgather_host(out_.data(), in_.data(), bytes);
    to_device(recv, in_.data(), bytes * P, s);
  }

  void alltoall_device(const void* send, void* recv, u64 bytes, void* stream) override {
    const int P = size();
    std::vector<u64> cnt((size_t)P, bytes), off((size_t)P);
    for (int p = 0; p < P; ++p) off[(size_t)p] = (u64)p * bytes;
    stage_alltoallv(send, cnt.data(), off.data(), recv, cnt.data(), off.data(), stream);
  }

  void gather_device(const void* send, void* recv, u64 bytes, int root, void* stream) override {
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int P = size();
    out_.resize(std::max<u64>(bytes, 1));
    to_host(out_.data(), send, bytes, s);
    std::vector<char> all;
    h_->gatherv_host(out_.data(), bytes, &all, nullptr, root);
    if (rank() == root)
      for (int r = 0; r < P; ++r)
        if (r != root && bytes)
          to_device(static_cast<char*>(recv) + (u64)r * bytes, all.data() + (u64)r * bytes, bytes, s);
  }

  void sync_stream(void* stream) override {
    LOCUST_HIP_CHECK(hipStreamSynchronize(static_cast<hipStream_t>(stream)));
  }

 private:
  void to_host(void* dst, const void* src, u64 bytes, hipStream_t s) {
    LOCUST_HIP_CHECK(hipStreamSynchronize(s));  // the producer of `src` has finished
    if (bytes) LOCUST_HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, s));
    LOCUST_HIP_CHECK(hipStreamSynchronize(s));
  }
  void to_device(void* dst, const void* src, u64 bytes, hipStream_t s) {
    if (bytes) LOCUST_HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s));
    LOCUST_HIP_CHECK(hipStreamSynchronize(s));  // `src` is reused by the next collective
  }
  void stage_alltoallv(const void* send, const u64* sb, const u64* so, void* recv, const u64* rb,
                       const u64* ro, void* stream) {
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int P = size();
    u64 send_end = 0, recv_end = 0;
    for (int p = 0; p < P; ++p) {
      send_end = std::max(send_end, so[p] + sb[p]);
      recv_end = std::max(recv_end, ro[p] + rb[p]);
    }
    out_.resize(std::max<u64>(send_end, 1));
    in_.resize(std::max<u64>(recv_end, 1));
    LOCUST_HIP_CHECK(hipStreamSynchronize(s));
    for (int p = 0; p < P; ++p)
      if (sb[p])
        LOCUST_HIP_CHECK(hipMemcpyAsync(out_.data() + so[p], static_cast<const char*>(send) + so[p],
                                        sb[p], hipMemcpyDeviceToHost, s));
    LOCUST_HIP_CHECK(hipStreamSynchronize(s));
    h_->alltoallv(out_.data(), sb, so, in_.data(), rb, ro, nullptr);
    for (int p = 0; p < P; ++p)
      if (rb[p])
        LOCUST_HIP_CHECK(hipMemcpyAsync(static_cast<char*>(recv) + ro[p], in_.data() + ro[p], rb[p],
                                        hipMemcpyHostToDevice, s));
    LOCUST_HIP_CHECK(hipStreamSynchronize(s));
  }

  std::unique_ptr<Communicator> h_;
  std::vector<char> out_, in_;
};

}  // namespace

std::unique_ptr<Communicator> make_staged_device_comm(std::unique_ptr<Communicator> host) {
  return std::unique_ptr<Communicator>(new StagedDeviceComm(std::move(host)));
}

}  // namespace locust
