// Single-process multi-rank driver: one thread per rank (`MapReduce --gpus N`,
// `locust_amd.run_multi`).  With a GPU per rank the ranks form an RCCL clique
// (ncclCommInitAll over xGMI); with fewer GPUs than ranks (tests
// rehearsing 2/4/8 ranks on the one GPU of a test box) the loopback communicator moves
// data with device copies; the CPU engine uses loopback.
//
// Inputs: an in-memory text (split by shard_text) or a file, of which every rank reads only
// its own line-aligned byte range (file_shards) -- the reference's per-node line ranges
// (/root/reference/MapReduce/src/main.cu:40-64, 369-374) without any rank holding the
// whole file.
#include <algorithm>
#include <atomic>
#include <cstring>
#include <exception>
#include <functional>
#include <thread>

#include "locust/dist.hpp"
#include "locust/hip_check.hpp"
#include "locust/io.hpp"
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

// auto = loopback: ranks in one process exchange by peer-to-peer device copies over xGMI.
// The RCCL clique (ncclCommInitAll + a driving thread per GPU) stays opt-in (--comm rccl)
// until a run with real RCCL peers has been recorded; the benchmark's ranks are
// separate processes on RCCL either way.
LocalComm resolve_local_comm(const DistConfig& cfg, LocalComm comm) {
  if (cfg.job.backend != Backend::kGpu) return LocalComm::kLoopback;
  return comm == LocalComm::kAuto ? LocalComm::kLoopback : comm;
}

std::vector<int> peer_access_row(int device) {
  const int n = visible_device_count();
  std::vector<int> row((size_t)std::max(n, 0), 0);
  for (int d = 0; d < n; ++d)
    if (d != device) LOCUST_HIP_CHECK(hipDeviceCanAccessPeer(&row[(size_t)d], device, d));
  return row;
}

// Which ordered pairs of `devices` can access each other directly (queried, not enabled).
static std::vector<int> query_peer_access(const std::vector<int>& devices) {
  const size_t n = devices.size();
  std::vector<int> m(n * n, 0);
  for (size_t i = 0; i < n; ++i)
    for (size_t j = 0; j < n; ++j)
      if (i != j && devices[i] != devices[j])
        LOCUST_HIP_CHECK(hipDeviceCanAccessPeer(&m[i * n + j], devices[i], devices[j]));
  return m;
}

std::vector<int> enable_peer_access(const std::vector<int>& devices) {
  const size_t n = devices.size();
  std::vector<int> m(n * n, 0);
  int cur = 0;
  LOCUST_HIP_CHECK(hipGetDevice(&cur));
  for (size_t i = 0; i < n; ++i)
    for (size_t j = 0; j < n; ++j) {
      if (i == j || devices[i] == devices[j]) continue;
      int can = 0;
      LOCUST_HIP_CHECK(hipDeviceCanAccessPeer(&can, devices[i], devices[j]));
      if (can) {
        LOCUST_HIP_CHECK(hipSetDevice(devices[i]));
        const hipError_t e = hipDeviceEnablePeerAccess(devices[j], 0);
        if (e == hipErrorPeerAccessAlreadyEnabled)
          (void)hipGetLastError();
        else
          LOCUST_HIP_CHECK(e);
      }
      m[i * n + j] = can ? 1 : 0;
      LOCUST_LOG_INFO("GPU %d -> GPU %d: %s", devices[i], devices[j],
                      can ? "peer access enabled (direct xGMI copies)"
                          : "no peer access (the runtime stages copies through host memory)");
    }
  LOCUST_HIP_CHECK(hipSetDevice(cur));
  return m;
}

namespace {

// What a rank thread needs to know about its input before and after its engine exists.
struct RankInput {
  u64 bytes = 0, lines = 0;  // engine sizing (lines: an upper bound)
  bool stream = false;       // larger than one pass: the engine streams it
  // Fills the rank's shard (called on the rank's thread, after its engine is built);
  // `keep` owns a source the shard points to for as long as the jobs run.
  std::function<TextInput(ShardEngine&, std::unique_ptr<TextSource>* keep)> load;
};

std::vector<DistResult> run_ranks(const std::vector<DistConfig>& schedule,
                                  const std::vector<RankInput>& inputs, LocalComm comm_kind,
                                  std::vector<DistResult>* per_rank) {
  LOCUST_CHECK_ARG(!schedule.empty(), "empty job schedule");
  const DistConfig& cfg = schedule[0];
  const int P = cfg.world;
  LOCUST_CHECK_ARG(P >= 1 && (int)inputs.size() == P, "world must be >= 1, one input per rank");
  for (const auto& c : schedule)
    LOCUST_CHECK_ARG(c.world == P && c.job.backend == cfg.job.backend,
                     "every job of a schedule runs on the same ranks");
  const bool gpu = cfg.job.backend == Backend::kGpu;
  int ndev = 1;
  if (gpu) {
    LOCUST_HIP_CHECK(hipGetDeviceCount(&ndev));
    LOCUST_CHECK_ARG(ndev >= 1, "no GPU visible");
  }
  bool rccl = resolve_local_comm(cfg, comm_kind) == LocalComm::kRccl;
  if (rccl)
    LOCUST_CHECK_ARG(cfg.job.device + P <= ndev,
                     "an RCCL clique needs one GPU per rank (RCCL refuses two ranks per "
                     "device); use the loopback communicator to rehearse more ranks");
  // RCCL clique: rank r on device (device + r), communicators created together up front
  // (ncclCommInitAll), one thread per rank drives its GPU.  Loopback: ranks round-robin
  // on the visible GPUs, collectives as device copies between the ranks' buffers.
  std::vector<RcclCliqueMember> clique;
  std::vector<int> devs;
  if (gpu)
    for (int r = 0; r < P; ++r) {
      const int d = rccl ? cfg.job.device + r : (cfg.job.device + r) % ndev;
      if (std::find(devs.begin(), devs.end(), d) == devs.end()) devs.push_back(d);
    }
  if (rccl) {
    std::vector<int> cd((size_t)P);
    for (int r = 0; r < P; ++r) cd[(size_t)r] = cfg.job.device + r;
    try {
      clique = make_rccl_clique(cd);
    } catch (const std::exception& e) {
      if (comm_kind == LocalComm::kRccl) throw;
      LOCUST_LOG_WARN("RCCL clique over %d GPUs failed (%s): loopback ranks instead", P, e.what());
      rccl = false;
    }
  }
  // Peer access for the loopback data plane's device-to-device copies (RCCL sets up its own
  // transports): one enable per ordered pair of distinct devices, logged per pair.
  // An RCCL clique reports the pairs that could access each other directly (its own
  // transports decide what it uses).
  std::vector<int> p2p;
  if (gpu && devs.size() > 1) p2p = rccl ? query_peer_access(devs) : enable_peer_access(devs);
  auto peers_of = [&](int dev) -> int {
    if (devs.size() < 2 || p2p.empty()) return -1;
    const size_t n = devs.size();
    const size_t i = (size_t)(std::find(devs.begin(), devs.end(), dev) - devs.begin());
    int k = 0;
    for (size_t j = 0; j < n; ++j) k += p2p[i * n + j];
    return k;
  };
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
        const RankInput& in = inputs[(size_t)r];
        JobConfig job = cfg.job;
        job.device = gpu ? (rccl ? cfg.job.device + r : (cfg.job.device + r) % ndev) : 0;
        if (gpu && numa_enabled()) {
          // this rank's thread on its GPU's NUMA node before anything is allocated: the
          // engine's pinned buffers (its shard below) are first touched there
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
        // the ranks on this rank's GPU share its HBM: each plans against its share
        if (gpu) {
          int share = 0;
          for (int q = 0; q < P; ++q)
            share += (rccl ? cfg.job.device + q : (cfg.job.device + q) % ndev) == job.device;
          job.hbm_share = std::max(share, 1);
        }
        std::unique_ptr<ShardEngine> eng =
            gpu ? make_gpu_shard_engine(job, std::max<u64>(in.bytes, 1), std::max<u64>(in.lines, 1))
                : make_cpu_shard_engine(job);
        LOCUST_LOG_DEBUG("rank %d: engine built, process %s", r, process_rss_breakdown().c_str());
        if (schedule.size() == 1) eng->out_regions = 1;  // one job: one output region
        std::unique_ptr<TextSource> keep;
        const TextInput shard = in.load(*eng, &keep);
        LOCUST_LOG_DEBUG("rank %d: shard ready (%s), process %s", r,
                         shard.source ? "streamed" : "in memory", process_rss_breakdown().c_str());
        // the same engines and communicators across jobs, like a long-lived rank
        for (size_t j = 0; j < schedule.size(); ++j) {
          LOCUST_CHECK_ARG(!shard.source || schedule.size() == 1,
                           "a streamed file shard is read once: one job per run");
          DistResult d = run_distributed(schedule[j], *comm, *eng, shard);
          LOCUST_LOG_DEBUG("rank %d: job %zu done, process %s", r, j,
                           process_rss_breakdown().c_str());
          d.input_bytes = shard.bytes;
          d.input_streamed = shard.source != nullptr;
          d.peer_p2p = gpu ? peers_of(job.device) : -1;
          d.rccl_clique = rccl;
          d.pinned_bytes = eng->host_pinned_bytes();
          d.shared_pinned_bytes = eng->shared_pinned_bytes();
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

// Stream threshold of a rank's file range (the single-GPU CLI's default pass, main.cpp).
constexpr u64 kDefaultRankChunk = 256ull << 20;

}  // namespace

std::vector<DistResult> run_single_process_schedule(const std::vector<DistConfig>& schedule,
                                                    const TextInput& whole, LocalComm comm_kind,
                                                    std::vector<DistResult>* per_rank) {
  LOCUST_CHECK_ARG(!schedule.empty() && schedule[0].world >= 1, "world must be >= 1");
  const int P = schedule[0].world;
  const std::vector<TextInput> shards = shard_text(whole, P);
  std::vector<RankInput> inputs((size_t)P);
  for (int r = 0; r < P; ++r) {
    const TextInput s = shards[(size_t)r];
    RankInput& ri = inputs[(size_t)r];
    ri.bytes = s.bytes;
    ri.lines = s.num_lines;
    const u64 chunk = schedule[0].job.chunk_bytes;
    ri.load = [s, chunk](ShardEngine& eng, std::unique_ptr<TextSource>*) {
      // the rank's own pinned copy of its shard (not a slice of one shared host buffer):
      // written by this thread, so on its NUMA node, and uploaded without staging
      TextInput shard = s;
      if (char* buf = eng.input_buffer())
        if (shard.bytes && (!chunk || shard.bytes <= chunk)) {
          std::memcpy(buf, shard.data, shard.bytes);
          shard.data = buf;
        }
      return shard;
    };
  }
  return run_ranks(schedule, inputs, comm_kind, per_rank);
}

DistResult run_single_process_multi_gpu(const DistConfig& cfg, const TextInput& whole,
                                        LocalComm comm, std::vector<DistResult>* per_rank) {
  return run_single_process_schedule({cfg}, whole, comm, per_rank)[0];
}

DistResult run_single_process_file(const DistConfig& cfg_in, const std::string& path,
                                   LocalComm comm, std::vector<DistResult>* per_rank) {
  DistConfig cfg = cfg_in;
  const int P = cfg.world;
  LOCUST_CHECK_ARG(P >= 1, "world must be >= 1");
  const bool gpu = cfg.job.backend == Backend::kGpu;
  const u64 chunk = cfg.job.chunk_bytes ? cfg.job.chunk_bytes : kDefaultRankChunk;
  const std::vector<FileRange> ranges = file_shards(path, P);
  bool any_stream = false;
  std::vector<RankInput> inputs((size_t)P);
  for (int r = 0; r < P; ++r) {
    const FileRange fr = ranges[(size_t)r];
    RankInput& ri = inputs[(size_t)r];
    ri.bytes = fr.bytes;
    ri.lines = fr.bytes + 1;  // unknown before reading: bounded by the bytes
    ri.stream = gpu && fr.bytes > chunk;
    any_stream |= ri.stream;
    const bool stream = ri.stream;
    ri.load = [path, fr, stream, gpu, r](ShardEngine& eng, std::unique_ptr<TextSource>* keep) {
      TextInput shard;
      shard.bytes = fr.bytes;
      if (stream) {
        // a range past one pass: line-aligned pieces of it stream through the engine's
        // pinned ring into device chunks (host memory: the ring, not the range)
        *keep = open_file_range_source(path, fr.offset, fr.offset + fr.bytes);
        shard.source = keep->get();
        LOCUST_LOG_INFO("rank %d: bytes [%llu, %llu) of %s streamed", r,
                        (unsigned long long)fr.offset, (unsigned long long)(fr.offset + fr.bytes),
                        path.c_str());
        return shard;
      }
      // one pass: parallel preads straight into the engine's pinned buffer (this thread
      // first touches it, on the rank's NUMA node); the CPU engine reads into its own
      char* buf = gpu ? eng.input_buffer() : nullptr;
      static thread_local std::vector<char> host;  // CPU ranks: their own host copy
      if (!buf) {
        host.assign(fr.bytes + 64, 0);
        buf = host.data();
      }
      read_file_range_into(path, buf, fr.offset, fr.bytes, &shard.num_lines);
      shard.data = buf;
      LOCUST_LOG_INFO("rank %d: bytes [%llu, %llu) of %s read (%llu lines)", r,
                      (unsigned long long)fr.offset, (unsigned long long)(fr.offset + fr.bytes),
                      path.c_str(), (unsigned long long)shard.num_lines);
      return shard;
    };
  }
  // streamed ranges need streaming engines (a pass of `chunk` bytes); one-pass ranges are
  // sized by their own bytes (chunk_bytes = 0 keeps them one pass)
  cfg.job.chunk_bytes = any_stream ? chunk : 0;
  // every streaming rank keeps a pinned read ring of 4 pieces: 16 MiB pieces for one rank,
  // 16 / P MiB (>= 2) for P ranks of this process -- they share the host's memory
  // bandwidth anyway, and 8 rings of 64 MiB were a fifth of the process's RSS
  if (!cfg.job.ring_piece_bytes && P > 1)
    cfg.job.ring_piece_bytes = std::max<u64>(2ull << 20, (16ull << 20) / (u64)P);
  return run_ranks({cfg}, inputs, comm, per_rank)[0];
}

}  // namespace locust
