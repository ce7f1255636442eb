// Single-process multi-rank driver: one thread per rank.  With a GPU per rank the ranks
// form an RCCL clique (ncclCommInitAll over xGMI) -- `MapReduce --gpus N`;
// with fewer GPUs than ranks (tests rehearsing 2/4/8 ranks on the one GPU of a test box)
// the loopback communicator moves data with device copies; the CPU engine uses loopback.
#include <atomic>
#include <exception>
#include <thread>

#include "locust/dist.hpp"
#include "locust/hip_check.hpp"

namespace locust {

void copy_device(void* dst, const void* src, u64 bytes, bool to_host, void* stream) {
  if (!bytes) return;
  hipStream_t s = static_cast<hipStream_t>(stream);
  LOCUST_HIP_CHECK(hipMemcpyAsync(dst, src, bytes,
                                  to_host ? hipMemcpyDeviceToHost : hipMemcpyHostToDevice, s));
  LOCUST_HIP_CHECK(hipStreamSynchronize(s));
}

int visible_device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
  return n;
}

LocalComm resolve_local_comm(const DistConfig& cfg, LocalComm comm) {
  if (cfg.job.backend != Backend::kGpu) return LocalComm::kLoopback;
  if (comm != LocalComm::kAuto) return comm;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess) return LocalComm::kLoopback;
  return cfg.job.device + cfg.world <= ndev ? LocalComm::kRccl : LocalComm::kLoopback;
}

std::vector<DistResult> run_single_process_schedule(const std::vector<DistConfig>& schedule,
                                                    const TextInput& whole, LocalComm comm_kind) {
  LOCUST_CHECK_ARG(!schedule.empty(), "empty job schedule");
  const DistConfig& cfg = schedule[0];
  const int P = cfg.world;
  LOCUST_CHECK_ARG(P >= 1, "world must be >= 1");
  for (const auto& c : schedule)
    LOCUST_CHECK_ARG(c.world == P && c.job.backend == cfg.job.backend,
                     "every job of a schedule runs on the same ranks");
  const bool gpu = cfg.job.backend == Backend::kGpu;
  int ndev = 1;
  if (gpu) {
    LOCUST_HIP_CHECK(hipGetDeviceCount(&ndev));
    LOCUST_CHECK_ARG(ndev >= 1, "no GPU visible");
  }
  std::vector<TextInput> shards = shard_text(whole, P);
  const bool rccl = resolve_local_comm(cfg, comm_kind) == LocalComm::kRccl;
  if (rccl)
    LOCUST_CHECK_ARG(cfg.job.device + P <= ndev,
                     "an RCCL clique needs one GPU per rank (RCCL refuses two ranks per "
                     "device); use the loopback communicator to rehearse more ranks");
  // RCCL clique: rank r on device (device + r), communicators created together up front
  // (ncclCommInitAll), one thread per rank drives its GPU.  Loopback: ranks round-robin
  // on the visible GPUs, collectives as device copies between the ranks' buffers.
  std::vector<RcclCliqueMember> clique;
  if (rccl) {
    std::vector<int> devs((size_t)P);
    for (int r = 0; r < P; ++r) devs[(size_t)r] = cfg.job.device + r;
    clique = make_rccl_clique(devs);
  }
  LoopbackGroup group(P, gpu);
  std::vector<DistResult> results(schedule.size());
  std::vector<std::exception_ptr> errors((size_t)P);
  std::vector<int> error_order((size_t)P, 0);
  std::atomic<int> error_seq{0};
  std::vector<std::thread> threads;
  for (int r = 0; r < P; ++r) {
    threads.emplace_back([&, r] {
      try {
        JobConfig job = cfg.job;
        job.device = gpu ? (cfg.job.device + r) % ndev : 0;
        if (rccl) LOCUST_HIP_CHECK(hipSetDevice(job.device));
        // Ranks are threads of one process here: no stream capture while other ranks may
        // allocate or copy (hipGraph replay is for one-process-per-GPU runs).
        if (P > 1) job.graph = 0;
        std::unique_ptr<ShardEngine> eng =
            gpu ? make_gpu_shard_engine(job, shards[(size_t)r].bytes, shards[(size_t)r].num_lines)
                : make_cpu_shard_engine(job);
        std::unique_ptr<Communicator> comm =
            rccl ? make_rccl_clique_comm(clique[(size_t)r]) : group.comm(r);
        // the same engines and communicators across jobs, like a long-lived rank
        for (size_t j = 0; j < schedule.size(); ++j) {
          DistResult d = run_distributed(schedule[j], *comm, *eng, shards[(size_t)r]);
          if (r == 0) results[j] = std::move(d);
        }
      } catch (...) {
        errors[(size_t)r] = std::current_exception();
        error_order[(size_t)r] = ++error_seq;
        group.abort();  // ranks waiting in a collective fail now instead of timing out
        // (RCCL ranks: their waits poll ncclCommGetAsyncError and time out)
      }
    });
  }
  for (auto& t : threads) t.join();
  // report the root cause: the first rank that failed, not the ones that were woken up
  int first = -1;
  for (int r = 0; r < P; ++r)
    if (errors[(size_t)r] && (first < 0 || error_order[(size_t)r] < error_order[(size_t)first]))
      first = r;
  if (first >= 0) std::rethrow_exception(errors[(size_t)first]);
  return results;
}

DistResult run_single_process_multi_gpu(const DistConfig& cfg, const TextInput& whole,
                                        LocalComm comm) {
  return run_single_process_schedule({cfg}, whole, comm)[0];
}

}  // namespace locust
