// Single-process multi-rank driver: one thread per rank.  With a GPU per rank the ranks
// form an RCCL clique (ncclCommInitAll over xGMI) -- `MapReduce --gpus N`;
// with fewer GPUs than ranks (tests rehearsing 2/4/8 ranks on the one GPU of a test box)
// the loopback communicator moves data with device copies; the CPU engine uses loopback.
#include <atomic>
#include <cstring>
#include <exception>
#include <thread>

#include "locust/dist.hpp"
#include "locust/hip_check.hpp"
#include "locust/numa.hpp"

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

// kAuto is the loopback communicator: with a GPU per rank its collectives are peer copies
// between the ranks' devices over xGMI.  The RCCL clique is opt-in (`--comm rccl`) until a
// run with real RCCL peers has been recorded on this pool (one-GPU boxes only so far).
LocalComm resolve_local_comm(const DistConfig& cfg, LocalComm comm) {
  if (cfg.job.backend != Backend::kGpu) return LocalComm::kLoopback;
  return comm == LocalComm::kAuto ? LocalComm::kLoopback : comm;
}

std::vector<DistResult> run_single_process_schedule(const std::vector<DistConfig>& schedule,
                                                    const TextInput& whole, LocalComm comm_kind,
                                                    std::vector<DistResult>* per_rank) {
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
  // clique members whose handle a rank has wrapped (the wrapper owns it from then on)
  std::vector<char> wrapped((size_t)P, 0);
  std::vector<DistResult> results(schedule.size());
  if (per_rank) per_rank->assign((size_t)P, DistResult{});
  std::vector<std::exception_ptr> errors((size_t)P);
  std::vector<int> error_order((size_t)P, 0);
  std::atomic<int> error_seq{0};
  std::vector<std::thread> threads;
  for (int r = 0; r < P; ++r) {
    threads.emplace_back([&, r] {
      try {
        JobConfig job = cfg.job;
        job.device = gpu ? (cfg.job.device + r) % ndev : 0;
        if (gpu && numa_enabled()) {
          // this rank's thread on its GPU's NUMA node before anything is allocated: the
          // engine's pinned buffers (its copy of the shard below) are first touched there
          char bdf[64] = {0};
          if (hipDeviceGetPCIBusId(bdf, (int)sizeof(bdf), job.device) == hipSuccess) {
            const GpuPlacement pl = placement_for_bdf(bdf);
            const bool bound = bind_thread_to(pl);
            LOCUST_LOG_INFO("rank %d on GPU %d (%s): NUMA node %d, %s", r, job.device, bdf,
                            pl.numa_node, bound ? "thread bound to its CPUs" : "not bound");
          } else {
            (void)hipGetLastError();
          }
        }
        std::unique_ptr<Communicator> comm;
        if (rccl) {
          LOCUST_HIP_CHECK(hipSetDevice(job.device));
          comm = make_rccl_clique_comm(clique[(size_t)r]);  // owns the handle from here on
          wrapped[(size_t)r] = 1;
        } else {
          comm = group.comm(r);
        }
        // Ranks are threads of one process here: no stream capture while other ranks may
        // allocate or copy (hipGraph replay is for one-process-per-GPU runs).
        if (P > 1) job.graph = 0;
        std::unique_ptr<ShardEngine> eng =
            gpu ? make_gpu_shard_engine(job, shards[(size_t)r].bytes, shards[(size_t)r].num_lines)
                : make_cpu_shard_engine(job);
        // the rank's own pinned copy of its shard (not a slice of one shared host buffer):
        // written by this thread, so on its NUMA node, and uploaded without staging
        TextInput shard = shards[(size_t)r];
        if (char* buf = eng->input_buffer()) {
          if (shard.bytes && (!job.chunk_bytes || shard.bytes <= job.chunk_bytes)) {
            std::memcpy(buf, shard.data, shard.bytes);
            shard.data = buf;
          }
        }
        // the same engines and communicators across jobs, like a long-lived rank
        for (size_t j = 0; j < schedule.size(); ++j) {
          DistResult d = run_distributed(schedule[j], *comm, *eng, shard);
          if (per_rank && j + 1 == schedule.size()) {  // the last job's stats (no entries)
            DistResult& pr = (*per_rank)[(size_t)r];
            pr = d;
            if (r == 0) pr.result.entries = EntryList{};
          }
          if (r == 0) results[j] = std::move(d);
        }
      } catch (...) {
        errors[(size_t)r] = std::current_exception();
        error_order[(size_t)r] = ++error_seq;
        group.abort();  // ranks waiting in a collective fail now instead of timing out
        // RCCL clique: every member's wait sees the flag and aborts its communicator
        if (rccl) clique[(size_t)r].abort->store(true);
      }
    });
  }
  for (auto& t : threads) t.join();
  for (int r = 0; r < P && rccl; ++r)
    if (!wrapped[(size_t)r]) release_rccl_clique_member(clique[(size_t)r]);
  // report the root cause: the first rank that failed, not the ones that were woken up
  int first = -1;
  for (int r = 0; r < P; ++r)
    if (errors[(size_t)r] && (first < 0 || error_order[(size_t)r] < error_order[(size_t)first]))
      first = r;
  if (first >= 0) std::rethrow_exception(errors[(size_t)first]);
  return results;
}

DistResult run_single_process_multi_gpu(const DistConfig& cfg, const TextInput& whole,
                                        LocalComm comm, std::vector<DistResult>* per_rank) {
  return run_single_process_schedule({cfg}, whole, comm, per_rank)[0];
}

}  // namespace locust
