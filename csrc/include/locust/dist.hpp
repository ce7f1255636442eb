// Distributed (multi-GPU / multi-process) WordCount.
//
// Replaces the reference's distribution layer: a TCP
// "slave" that runs shell commands (/root/reference/Distributor/slave.py:1-38), a missing
// master, and a shuffle that is a local file (/tmp/out.txt, main.cu:428-441) with the
// network hop missing.  Here every rank (one process or thread per GPU) runs:
//
//   map_local      tokenize its byte-range shard, sort, optionally combine (sum counts)
//   sample         S evenly spaced local keys -> allgather -> P-1 splitters (sample sort)
//   partition      lower_bound of each splitter in the sorted local records
//   shuffle        40-B KeyCount records over xGMI, every link busy at once: grouped
//                  ncclSend/ncclRecv with exact bucket sizes, or (steady state, see
//                  locust/exch.hpp) ONE fixed-slot ncclAllToAll padded to the previous
//                  job's largest bucket
//   reduce         sort received records, weighted head-mark + adjacent difference
//   offsets        allgather of per-rank token totals -> global `val` = exclusive prefix
//   gather         rank 0 receives every rank's entries in rank order (== key order)
//
// Output is byte-identical to the single-GPU run, including the global `val` indices.
// Every stage boundary runs an agreement collective on a status word, so a rank that
// fails (or is told to fail via LOCUST_FAULT) turns into a clean error on all ranks.
//
// Two strategies follow the map stage (DistStrategy):
//   shuffle   the sample-sort all-to-all above: every rank reduces 1/P of the key space.
//             Scales with the number of distinct keys; costs 3 more collectives.
//   gather    every rank's combined (key, count) records go straight to rank 0 over
//             point-to-point xGMI (one grouped send/recv) and rank 0 merges them.  When
//             the combined records are few (Hamlet-sized shards: ~5.6K distinct keys per
//             rank) the job is latency-bound and one collective beats four; rank 0 has
//             to receive the whole result anyway.
//   auto      gather when the total combined records <= gather_max_records, else shuffle.
//             Decided from the first allgather, so every rank takes the same branch.
#pragma once

#include <atomic>
#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "locust/engine.hpp"
#include "locust/exch.hpp"
#include "locust/slot.hpp"

namespace locust {

class Communicator {
 public:
  virtual ~Communicator() = default;
  virtual int rank() const = 0;
  virtual int size() const = 0;
  virtual const char* name() const = 0;
  // true: data-plane buffers are device pointers (RCCL, GPU loopback).
  virtual bool device_buffers() const = 0;

  // ---- control plane: host buffers, blocking ----
  // recv gets size() * bytes, rank r's contribution at offset r * bytes.
  virtual void allgather_host(const void* send, void* recv, u64 bytes) = 0;
  // Rank `root` receives every rank's variable-length blob, concatenated in rank order.
  virtual void gatherv_host(const void* send, u64 bytes, std::vector<char>* recv_at_root,
                            std::vector<u64>* sizes_at_root, int root) = 0;
  virtual void barrier() = 0;
  // gatherv when every rank already knows all sizes (host buffers; recv only at root).
  virtual void gatherv_known(const void* send, u64 bytes, const u64* sizes, void* recv_at_root,
                             int root);

  // ---- data plane: engine buffers, byte counts/offsets per peer (host arrays) ----
  // Blocking: returns when this rank's receives are complete and its sends may be reused.
  virtual void alltoallv(const void* send, const u64* send_bytes, const u64* send_off, void* recv,
                         const u64* recv_bytes, const u64* recv_off, void* stream) = 0;

  // Stream-ordered all-gather of device buffers (device_buffers() communicators): rank
  // r's `bytes` land at recv + r * bytes.  Enqueued on `stream` behind the work that
  // produces `send`, so no host synchronisation is needed first; complete after
  // sync_stream(stream).  Host-only communicators throw.
  virtual void allgather_device(const void* send, void* recv, u64 bytes, void* stream);
  // Stream-ordered all-to-all of fixed-size chunks (device_buffers() communicators): chunk
  // d of `send` goes to rank d, rank s's chunk for this rank lands at recv + s * bytes.
  virtual void alltoall_device(const void* send, void* recv, u64 bytes, void* stream);
  // Stream-ordered gather of fixed-size chunks to `root`: rank r's `bytes` land at
  // recv + r * bytes on the root; the root's own chunk must already be in place there
  // (recv is only used on the root).
  virtual void gather_device(const void* send, void* recv, u64 bytes, int root, void* stream);
  // Wait for `stream`, watching for communicator errors (timeouts abort the communicator).
  virtual void sync_stream(void* stream);
  // true: allgather_device only enqueues stream work (no host waits), so it can be
  // captured into a hipGraph together with the kernels around it.
  virtual bool graph_capturable() const { return false; }

  // Status agreement: every rank contributes `local_error` (0 = ok); returns the lowest
  // failing rank or -1.  One allgather of 4 bytes per rank.
  int agree(int local_error);
  // Ranks the data-plane library itself reports (RCCL: ncclCommCount), else size().
  virtual int comm_count() const { return size(); }
  // Stream-ordered all-to-all-v of device buffers with exact per-peer byte counts (host
  // arrays every rank derived from the same all-gathered count matrix): grouped
  // point-to-point sends/receives, no host wait.  Complete after sync_stream(stream).
  virtual void alltoallv_device(const void* send, const u64* send_bytes, const u64* send_off,
                                void* recv, const u64* recv_bytes, const u64* recv_off,
                                void* stream);
  // A 64-bit id every rank of this communicator agrees on (fixed at construction, distinct
  // between groups): names the group's shared output segment (locust/shm.hpp).
  virtual u64 group_id() const = 0;
  // true: every rank of the group is a thread of this process (loopback, RCCL clique)
  virtual bool in_process() const { return false; }
};

// Star-topology TCP communicator (rank 0 relays).  Control plane for everything and the
// data plane of the CPU backend; also the bootstrap channel for RCCL unique ids.
// listen_fd (rank 0, optional): a socket already bound to `port` and listening -- handed
// over by the launcher so no other process can take the port between its choice and the
// bind (the communicator owns and closes it).
std::unique_ptr<Communicator> make_tcp_comm(int rank, int world, const std::string& host, int port,
                                            double timeout_s = 120.0, int listen_fd = -1);
// RCCL communicator for one GPU per rank; bootstraps its ncclUniqueId over TCP.
std::unique_ptr<Communicator> make_rccl_comm(int rank, int world, int device,
                                             const std::string& host, int port,
                                             double timeout_s = 300.0, int listen_fd = -1);

// A host communicator (TCP) with the device data plane staged through host memory
// ("tcpdev", comm/staged_comm.hip): the multi-process device paths rehearsed with several
// processes sharing one GPU (RCCL refuses two ranks per device).  Blocking; tests only.
std::unique_ptr<Communicator> make_staged_device_comm(std::unique_ptr<Communicator> host);

// Single-process RCCL clique (`ncclCommInitAll` over the node's GPUs):
// make_rccl_clique creates one communicator per device from the calling thread; each
// rank's thread then wraps its member (make_rccl_clique_comm sets that thread's device).
// `abort` (shared by the clique): set when any rank fails; every member's wait then
// throws at once and its communicator is aborted (ncclCommAbort) instead of destroyed, so
// peers blocked on the failed rank fail fast rather than after the timeout.
struct RcclCliqueMember {
  void* handle = nullptr;  // ncclComm_t
  int rank = 0, world = 1, device = 0;
  u64 group = 0;  // the clique's group id (Communicator::group_id)
  std::shared_ptr<std::atomic<bool>> abort;
};
std::vector<RcclCliqueMember> make_rccl_clique(const std::vector<int>& devices);
std::unique_ptr<Communicator> make_rccl_clique_comm(const RcclCliqueMember& m,
                                                    double timeout_s = 300.0);
// A member whose handle was never wrapped (its rank failed first): abort it.
void release_rccl_clique_member(RcclCliqueMember& m);

// N virtual ranks inside one process (threads).  With device buffers the all-to-all is
// done with hipMemcpyAsync between the ranks' buffers, so a single GPU can rehearse the
// 2/4/8-rank shuffle (RCCL refuses two ranks on one device).
class LoopbackGroup {
 public:
  LoopbackGroup(int world, bool device_buffers);
  ~LoopbackGroup();
  std::unique_ptr<Communicator> comm(int rank);
  // A rank failed: collectives still waiting on it throw instead of timing out.
  void abort();
  struct State;

 private:
  std::shared_ptr<State> state_;
};

// kLocal: a one-rank job under kAuto -- there is no peer to exchange with, so the job is
// the local device pipeline end to end (result straight into host memory), the way a
// one-rank collective is a local copy.  Forcing kShuffle / kGather still runs the full
// exchange machinery with one rank (the tests and the overhead measurement do).
enum class DistStrategy : int { kAuto = 0, kShuffle = 1, kGather = 2, kLocal = 3 };

// Per-rank local engine used by the distributed driver.
class ShardEngine {
 public:
  virtual ~ShardEngine() = default;
  virtual bool device_buffers() const = 0;
  virtual void* stream() = 0;
  // One rank (DistStrategy::kLocal): the whole job on the local engine; false when the
  // engine has no such path (the driver then runs the exchange with itself).
  virtual bool run_whole(const TextInput& /*shard*/, WordCountResult* /*r*/) { return false; }
  // Pinned host staging buffer for the shard text (nullptr if the engine has none).  A
  // shard whose data already points here is uploaded without a host copy.
  virtual char* input_buffer() { return nullptr; }
  // Page-locked host memory this rank's engine holds (0: a CPU engine); the shared output
  // block of ranks in one process is counted apart (shared_pinned_bytes, once per process).
  virtual u64 host_pinned_bytes() const { return 0; }
  // HBM: the engine's device allocations, and its GPU's free / total memory before them
  virtual u64 device_bytes() const { return 0; }
  virtual u64 hbm_free() const { return 0; }
  virtual u64 hbm_total() const { return 0; }
  // device memory in use on its GPU now (every engine and process on it)
  virtual u64 hbm_used_now() const { return 0; }
  virtual u64 shared_pinned_bytes() const { return 0; }
  // Map + sort (+ combine) this rank's shard.  Returns the number of local records.
  // `plan` is the strategy the driver expects to take: kGather lets an engine skip the
  // local sort (records may be unsorted); prepare_shuffle() must then be called before
  // sample()/bucket_offsets() if the driver switches to the shuffle after all.
  virtual u64 map_local(const TextInput& shard, bool combine,
                        DistStrategy plan = DistStrategy::kShuffle) = 0;
  virtual void prepare_shuffle() {}
  virtual std::vector<PackedKey> sample(u32 num_samples) = 0;
  // Record offsets [0 .. P] of the P buckets defined by P-1 sorted splitters.
  virtual std::vector<u64> bucket_offsets(const std::vector<PackedKey>& splitters) = 0;
  virtual const void* send_records() = 0;      // KeyCount[num local records], sorted
  virtual void* recv_records(u64 n) = 0;       // room for n incoming KeyCount records
  // Sort + weighted reduce of the n received records; returns {total_count, num_unique}.
  virtual void reduce_received(u64 n, u64* total_count, u64* num_unique) = 0;
  // Same, knowing the layout: run_lens[p] records from rank p, back to back in rank
  // order, each run a slice of that rank's sorted records (run_flags: the AND of every
  // rank's record_flags(); total_tokens bounds the runs' summed counts).  Sorted runs of
  // distinct keys are merged instead of re-aggregated.
  virtual void reduce_received_runs(const std::vector<u64>& run_lens, u64 total_tokens,
                                    u32 run_flags, u64* total_count, u64* num_unique) {
    u64 n = 0;
    for (u64 l : run_lens) n += l;
    reduce_received(n, total_count, num_unique);
  }
  // Gather strategy, root only: reduce this rank's own records together with the records
  // the other ranks sent (already in recv_records(), which holds room for both), back to
  // back in rank order; run_lens[i] = records from rank i+1 (each such run is sorted).
  // total_tokens: the sum of every run's counts (known from the map statistics);
  // run_flags: the AND of every rank's record_flags().
  virtual void reduce_gathered(const std::vector<u64>& run_lens, u64 total_tokens,
                               u32 run_flags, u64* total_count, u64* num_unique) = 0;
  // What this rank's send_records() are after map_local: kRecordsSorted | kRecordsDistinct.
  virtual u32 record_flags() const { return 0; }
  static constexpr u32 kRecordsSorted = 1, kRecordsDistinct = 2;
  // Strategy of the previous job (the driver's prediction for the next one under kAuto).
  DistStrategy last_strategy = DistStrategy::kShuffle;

  // ---- gather strategy in ONE all-gather of fixed-size slots (device engines) ----
  // Slot = SlotHeader (two records) + slot_records KeyCount records.  The map writes the
  // header on the device, the slots are all-gathered right behind it on the engine's
  // stream, and the root merges them straight from the receive buffer: one host
  // synchronisation per job.  Every slot_* call is made by every rank in the same order.
  // Enqueue this rank's map and its slot; returns the device send slot.  A shard the fast
  // path cannot take is mapped synchronously and its header written from the host.
  virtual void* enqueue_map_slot(const TextInput& shard, u32 slot_records) { return nullptr; }
  // The whole slot job as ONE hipGraph per shape: [upload + map + ordered build into the
  // slot] -> `allgather(send, recv, bytes)` (a capturable collective on stream()) ->
  // [root: merge | others: header copy].  Replaces enqueue_map_slot + the all-gather +
  // enqueue_merge_slots + enqueue_slot_headers; returns false (nothing enqueued) when the
  // shard needs the synchronous map, so the caller takes that sequence instead.  Saves the
  // graph -> collective -> graph transitions (~9 us per job measured at one rank).
  // `allgather` is issued directly at most once per job (`capturing` = false) and may
  // also be recorded into a capture (`capturing` = true; a refused capture then issues it
  // directly).  The caller tracks whether it entered the collective, so an exception after
  // that never makes it enter the all-gather a second time (see run_distributed).
  using SlotAllgather =
      std::function<void(const void* send, void* recv, u64 bytes, bool capturing)>;
  virtual bool enqueue_slot_job(const TextInput& shard, u32 slot_records, u32 nslots,
                                bool root, const SlotAllgather& allgather) {
    return false;
  }
  // After a host-side failure: this rank's slot says so (status kSlotFailed, no records);
  // returns the send slot.
  virtual void* write_slot_failure() { return nullptr; }
  // Device receive buffer for `nslots` slots.
  virtual void* slot_buffer(u32 nslots, u32 slot_records) { return nullptr; }
  // Root: enqueue the merge of the received slots (output lands in host memory).
  virtual void enqueue_merge_slots(u32 nslots, u32 slot_records) {}
  // Enqueue the copy of every slot's header to host memory; read after the sync.
  virtual void enqueue_slot_headers(u32 nslots, u32 slot_records) {}
  virtual const SlotHeader* slot_headers() const { return nullptr; }
  // After the sync: finish this rank's map (local redo after an LDS overflow); returns the
  // number of local records (as map_local does).
  virtual u64 complete_map_slot(const TextInput& shard) { return 0; }
  // Root, after the sync: the merged output (as reduce_gathered).
  virtual void finish_merge_slots(u64* total_count, u64* num_unique) {}
  // Records a slot can hold on this rank (the all-gather uses the minimum over ranks).
  virtual u64 slot_capacity() const { return 0; }
  u32 slot_records = 0;  // agreed slot size for the next job (0: kSlotRecordsMin)
  // Regions of a new shared host output (the device exchange): 2 lets jobs whose results
  // stay alive in turn write without growing it; a one-job run (the CLI on a file) sets 1.
  // Every rank of a group must set the same value.
  u32 out_regions = 2;

  // ---- shuffle strategy on the device (locust/exch.hpp) ----
  // Every rank's key range ends in ONE shared host output (locust/shm.hpp), written by
  // each rank at its global offset; the root adopts it.  Each collective callback is
  // called in the documented order on every rank.
  struct ExchCollectives {
    std::function<void(const void* send, void* recv, u64 bytes)> allgather;
    std::function<void(const void* send, void* recv, u64 bytes)> alltoall;
    std::function<void(const void* send, const u64* send_bytes, const u64* send_off, void* recv,
                       const u64* recv_bytes, const u64* recv_off)>
        alltoallv;
  };
  // ONE host synchronisation (slot sizes exch_slot_records / exch_gather_records agreed
  // by an earlier job): enqueue the whole exchange of this rank's sorted, distinct records
  // on stream() -- allgather (headers + samples), alltoall (fixed-pitch slots), allgather
  // (reports), then this rank's range into the shared output.  `hdr` + `samples` are this
  // rank's ExchMsg1 (the root's out_region is filled in here).  map_shard
  // (exch_map_async_ok): this rank has NOT mapped yet -- the map is enqueued first and
  // hdr's counts and the samples are built on the device; afterwards exch_map_complete()
  // (or, if any header says kExchMapRedo, every rank maps again synchronously).
  virtual void enqueue_exchange(const ExchMsg1& hdr, const std::vector<PackedKey>& samples,
                                u32 P, int me, const ExchCollectives& coll,
                                const TextInput* map_shard = nullptr) {
    throw Error("this engine has no device exchange");
  }
  // TWO host synchronisations, no sizes needed (the first job, or one whose data outgrew
  // the agreed slots).  Phase 1: [map] + allgather (headers + samples) + plan + allgather
  // of every rank's bucket offsets (ExchCtl) -- after its sync exch_headers() and
  // exch_plans() hold the P x P count matrix.  Phase 2: pack + all-to-all-v with exact
  // per-peer sizes + merge + allgather (reports) + this rank's range into the shared output.
  virtual void enqueue_exchange_plan(const ExchMsg1& hdr, const std::vector<PackedKey>& samples,
                                     u32 P, int me, const ExchCollectives& coll,
                                     const TextInput* map_shard = nullptr) {
    throw Error("this engine has no device exchange");
  }
  // to_root: the gather strategy on the same machinery -- every record goes to rank 0,
  // which merges the P runs and writes the whole output.
  virtual const ExchCtl* exch_plans() const { return nullptr; }  // P plans after phase 1
  virtual void enqueue_exchange_sized(u32 P, int me, const ExchCollectives& coll, bool to_root) {
    throw Error("this engine has no device exchange");
  }
  // The one-sync exchange found no free output region at the root (every region held by
  // a live result): after growing the output, write this rank's range again.
  virtual void enqueue_exchange_emit(u32 P, int me) {}
  virtual bool exch_map_async_ok(const TextInput& /*shard*/) const { return false; }
  // The map half of an asynchronous-map exchange (before enqueue_exchange*, P ranks, S
  // samples); a throw here becomes the header's failure status.
  virtual void exch_map_enqueue(const TextInput& /*shard*/, u32 /*P*/, u32 /*S*/) {
    throw Error("this engine has no asynchronous-map exchange");
  }
  // After the first sync of an asynchronous-map exchange: this rank's record count; the
  // local statistics are then available from map_stats().
  virtual u64 exch_map_complete(const TextInput& /*shard*/) { return 0; }
  virtual const ExchMsg1* exch_headers() const { return nullptr; }  // P ExchMsg1 headers
  virtual const ExchMsg3* exch_reports() const { return nullptr; }  // P reports
  // Root, after the last sync: wait until every rank's range is in the shared output
  // (completion stamps), then adopt it as the result (finalize() hands it over).
  virtual void exch_finish_root(u32 P, u64* total_count, u64* num_unique) {}
  // Every rank, after the last sync of an exchange job: drop the names of shared output
  // segments mapped during it (every rank has mapped them by then).
  virtual void exch_job_done() {}
  // Agreed exchange slot sizes (every rank computes the same from collective data; 0 =
  // not known yet: the job takes the two-sync sized exchange, which then sets them).
  u32 exch_slot_records = 0, exch_gather_records = 0;
  u64 exch_last_sum = 0;  // all ranks' records of the last job (auto: gather or shuffle)
  u64 exch_group = 0;     // the communicator's group id (names the shared output)
  int exch_rank = 0;      // this rank in that group
  bool exch_in_process = false;  // every rank of the group is a thread of this process
  // NUMA node of every rank's GPU (all-gathered once per engine; -1: unknown): places the
  // shared output's pages (locust/numa.hpp plan_rank_slices)
  std::vector<int> exch_numa_nodes;
  virtual int numa_node() { return -1; }  // this engine's GPU's node
  // Hands this rank's entries over (the caller sets the result's val_base).
  virtual void finalize(EntryList* out) = 0;
  // Map-stage counters of the last map_local.
  virtual void map_stats(WordCountResult* r) = 0;
};

std::unique_ptr<ShardEngine> make_gpu_shard_engine(const JobConfig& cfg, u64 max_bytes,
                                                   u64 max_lines);
std::unique_ptr<ShardEngine> make_cpu_shard_engine(const JobConfig& cfg);

struct DistConfig {
  JobConfig job;
  int world = 1;
  u32 samples_per_rank = 64;
  bool gather = true;   // rank 0 receives the whole output
  DistStrategy strategy = DistStrategy::kAuto;
  // auto: gather-to-root when the combined records of all ranks fit this bound.  The root
  // merge is one dictionary pass over them (~1 record/ns), the shuffle costs three extra
  // collective round trips (~15-25 us each over xGMI), so the break-even is ~10^5.
  u64 gather_max_records = 1u << 17;
};

struct DistResult {
  WordCountResult result;  // rank 0 (gather=true): global output; otherwise this rank's range
  double map_ms = 0, shuffle_ms = 0, reduce_ms = 0, gather_ms = 0, total_ms = 0;
  u64 local_records = 0;   // records this rank sent into the shuffle
  u64 sent_bytes = 0, recv_bytes = 0;
  u64 output_bytes = 0;    // output records this rank wrote to host memory over its own link
  // the same per peer (this rank's link to rank p; [me] = 0): what each xGMI link carried
  std::vector<u64> sent_to, recv_from;
  u64 range_tokens = 0, range_unique = 0;  // this rank's key range after the shuffle
  DistStrategy strategy = DistStrategy::kShuffle;  // the one this job took
  bool device_exchange = false;  // the shuffle ran as the device exchange (locust/exch.hpp)
  int host_syncs = 0;            // ... with this many host synchronisations
  // single-process runs (run_single_process_*): this rank's input and its GPU's peers
  u64 input_bytes = 0;           // bytes of its shard it read / mapped
  bool input_streamed = false;   // ... streamed from its file range (larger than one pass)
  int peer_p2p = -1;             // peers of its GPU with direct (xGMI) access; -1: no peers
  bool rccl_clique = false;      // ... exchanged over an RCCL clique (else loopback copies)
  u64 pinned_bytes = 0;          // page-locked host memory of its engine (its GPU's share)
  u64 shared_pinned_bytes = 0;   // the shared output block the ranks of a process write
  u64 hbm_device_bytes = 0;      // device memory of its engine (the HBM plan, engine.hpp)
  u64 hbm_free_bytes = 0;        // its GPU's free memory when the engine was built
  u64 hbm_total_bytes = 0;
  u64 hbm_used_bytes = 0;        // its GPU's memory in use after the job (all engines on it)
};

DistResult run_distributed(const DistConfig& cfg, Communicator& comm, ShardEngine& eng,
                           const TextInput& shard);

// Synchronous device<->host copy on `stream` (implemented in the HIP part of the library).
void copy_device(void* dst, const void* src, u64 bytes, bool to_host, void* stream);

// Split a line-aligned text into `parts` line-aligned shards of ~equal bytes.
std::vector<TextInput> shard_text(const TextInput& in, int parts);

// One process drives `cfg.world` ranks (threads) over the visible GPUs (round robin);
// rank 0's result is returned.  With Backend::kCpu the ranks use the CPU shard engine.
// comm: kAuto = kLoopback (device-to-device copies between the ranks' buffers); kRccl =
// an RCCL clique (ncclCommInitAll over xGMI; every rank needs a GPU of its own: RCCL
// refuses two ranks per device).  Loopback ranks on distinct GPUs get peer access
// enabled pairwise first, so their device copies go GPU to GPU.
// Ranks in one process never share host memory for their input: each rank thread copies
// (or reads) its own shard into its engine's pinned buffer, first touched on its NUMA node.
enum class LocalComm : int { kAuto = 0, kLoopback = 1, kRccl = 2 };
// hipDeviceCanAccessPeer(device, d) for every visible d (1 = direct xGMI access; the
// device's own entry is 0).  Empty without a GPU runtime.
std::vector<int> peer_access_row(int device);
DistResult run_single_process_multi_gpu(const DistConfig& cfg, const TextInput& whole,
                                        LocalComm comm = LocalComm::kAuto,
                                        std::vector<DistResult>* per_rank = nullptr);
// Several jobs back to back on the same ranks (engines and communicators persist, as in a
// long-lived multi-process job); rank 0's result of every job.
// per_rank (optional): every rank's result of the last job, in rank order.
std::vector<DistResult> run_single_process_schedule(const std::vector<DistConfig>& schedule,
                                                    const TextInput& whole,
                                                    LocalComm comm = LocalComm::kAuto,
                                                    std::vector<DistResult>* per_rank = nullptr);
// The same over a FILE: rank r reads only its own line-aligned byte range (file_shards)
// -- straight into its engine's pinned buffer with parallel preads when the range fits
// one device pass (cfg.job.chunk_bytes, default 256 MiB), else streamed through a small
// pinned ring chunk by chunk (enqueue_stream_source).  The whole file is never held in
// host memory.
DistResult run_single_process_file(const DistConfig& cfg, const std::string& path,
                                   LocalComm comm = LocalComm::kAuto,
                                   std::vector<DistResult>* per_rank = nullptr);
// Visible GPUs (0 if none or the runtime fails).
int visible_device_count();
// Which communicator run_single_process_* would use for `world` ranks (for logging).
LocalComm resolve_local_comm(const DistConfig& cfg, LocalComm comm);
// Peer access between every pair of `devices` (distinct ordinals): enabled where the
// runtime reports it possible; m[i * n + j] = 1 when device i can access device j
// directly.  Logged per pair at LOCUST_LOG=info.
std::vector<int> enable_peer_access(const std::vector<int>& devices);

}  // namespace locust
