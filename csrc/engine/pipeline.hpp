// Device pipeline: the buffers, streams and stage enqueuers of one GPU engine instance
// (internal to csrc/engine: used by the single-GPU engine, gpu_wordcount.hip, and by the
// per-rank shard engine, shard_engine.hip).
//
// Reference orchestration: /root/reference/MapReduce/src/main.cu:388-487 (cudaMalloc per
// run, synchronous cudaMemcpy of fixed 5,800/116,000-slot arrays, thrust calls that block,
// no error checks).  Here: one device arena allocated at construction, pinned host staging,
// a single stream, hipEvents at every stage boundary, exact-size transfers, look-back
// scratch zeroed by one memset per run, and captured hipGraphs for the repeated sequences.
//
// This header declares the struct (its state, sizing constants and the short accessors);
// the members with real logic are defined once, out of line, in pipeline.hip.
#pragma once

#include <algorithm>
#include <atomic>
#include <chrono>
#include <future>
#include <memory>
#include <mutex>
#include <array>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "locust/devcache.hpp"
#include "locust/dist.hpp"
#include "locust/engine.hpp"
#include "locust/hip_check.hpp"
#include "locust/kernels.hpp"
#include "locust/partmap.hpp"
#include "locust/trace.hpp"
#include "locust/worker.hpp"

namespace locust {

void validate_result(const WordCountResult& r);  // engine/common.cpp

namespace detail {

struct Arena {
  char* base = nullptr;
  u64 size = 0, used = 0;
  template <typename T>
  T* take(u64 count) {
    used = align_up(used, 256);
    T* p = reinterpret_cast<T*>(base + used);
    used += count * sizeof(T);
    if (used > size) throw Error("device arena overflow (internal sizing bug)");
    return p;
  }
};

struct SizingPlan {
  u64 bytes = 0;
  template <typename T>
  void add(u64 count) {
    bytes = align_up(bytes, 256) + count * sizeof(T);
  }
};

constexpr u32 kMaxSamples = 4096;
constexpr u32 kMaxRanks = 1024;

// Device pipeline: every buffer of one engine instance.  cap_records is the number of
// records (tokens or received KeyCount records) the sort/reduce side can hold.
struct DevicePipeline {
  JobConfig cfg;
  u64 cap_bytes = 0, cap_lines = 0, cap = 0;
  // ---- HBM plan (plan_device_pass, locust/engine.hpp) ----
  // pass_bytes: the largest input one pass takes (== cap_bytes, except in a streaming
  // engine, whose chunks of cap_bytes are mapped in windows of map_window bytes, so its
  // token buffers hold one window's tokens, not one chunk's).  rcap: the records the
  // sort / reduce buffers hold -- every token on the radix path, the distinct keys (ucap)
  // on the dictionary path until a general radix pass needs every token
  // (ensure_radix_full grows them on first use).
  u64 pass_bytes = 0, map_window = 0, rcap = 0;
  bool streaming = false;
  u64 layout_gen = 0;  // bumped when buffers move: captured sequences are keyed by it
  char* radix_base = nullptr;
  size_t radix_block = 0;
  u64 hbm_free = 0, hbm_total = 0;  // the device's memory before this engine's allocations
  // The arena's layout for a planned pass (shape_arena: the constructor's sizing, also
  // what plan_device_pass prices before an engine exists).
  struct ArenaShape {
    u64 slot_cap = 0, t_line = 0, t_compact = 0, t_map = 0, t_heads = 0, t_scan = 0;
    u64 rx_zero_words = 0, rx_part_words = 0, dict_slots = 0, dict_zero_bytes = 0;
    u64 sync_bytes = 0, part_off_tiles = 0, arena_bytes = 0;
    u32 partial_slots_cap = 0;
    bool small_pass = false, large_ordered = false;
  };
  static ArenaShape shape_arena(const JobConfig& cfg, const DevicePassPlan& p,
                                u64 small_pass_bytes);
  // Grows the sort / reduce buffers to every token (cap) -- a dictionary engine entering
  // the reference algorithm (its table overflowed, an uncombined shuffle, a reducer); it
  // drops the captured graphs, whose pointers change.  No-op when rcap == cap.
  void ensure_radix_full();
  // Device memory this engine holds (arena, radix growth, the second stream chunk, plan).
  u64 device_bytes() const;
  hipStream_t stream = nullptr;
  hipEvent_t ev[6] = {};
  Arena arena;
  size_t arena_block = 0;  // the arena's block size (devcache)

  char* d_text = nullptr;
  u64* d_nl = nullptr;
  char* d_delims = nullptr;
  KeysSoA slots{}, tokens{}, sorted{}, heads{};
  u32* d_line_counts = nullptr;
  u64* d_counts = nullptr;         // per-record counts of received records
  u64* d_sorted_counts = nullptr;  // counts in sorted order
  u64* d_prefix = nullptr;         // exclusive scan of sorted counts
  u64* d_head_val = nullptr;
  u64* d_head_count = nullptr;
  u32* d_perm = nullptr;
  u8* d_parts = nullptr;           // hash partition tag per token (partitioned dict build)
  bool parts_ready = false;        // d_parts describes the current `tokens`
  // Per-tile partition table of the small-input fast map (launch_map_fast part_off), for
  // engines whose passes can take the ordered kernel; part_tiles > 0: it describes the
  // current `tokens`.
  u32* d_part_off = nullptr;
  u32* d_part_occ = nullptr;  // the small map's per-tile partition occupancy (the plan's input)
  u64 part_off_tiles = 0;  // capacity in tiles
  u32 part_tiles = 0;
  // Large single passes: the two-kernel ordered build's partial slots (dict.hip).
  bool large_ordered = false;
  // LOCUST_SMALL_PASS_KB (construction, default 1024; 0: off): an engine for at most this
  // many bytes keeps the one-kernel ordered build (and its in-job plan) even when its
  // worst-case token count passes kPartBuildMaxTokens
  static u64 small_pass_limit() {
    const char* e = std::getenv("LOCUST_SMALL_PASS_KB");
    return (u64)(e ? std::max(0, std::atoi(e)) : 1024) << 10;
  }
  const u64 small_pass_bytes = small_pass_limit();
  bool small_pass = false;
  KeyCount* d_partials = nullptr;
  u32* d_partial_n = nullptr;
  u32 partial_slots_cap = 0;  // slots per partition d_partials holds
  // Slots per partition of the current pass's partials; nonzero: the piecewise map
  // already aggregated each piece into its own slot (enqueue_partials adds nothing).
  u32 partial_nslots = 0;
  // Large single-pass inputs travel in line-aligned pieces on the copy stream, each mapped
  // and aggregated as soon as it lands (the H2D overlaps map + partials); set by
  // prepare_upload.  At least kPieceBytes each (inputs from 2 x kPieceBytes on), middle
  // pieces min(piece_target(), bytes / 4) (LOCUST_PIECE_MB, default 10: fewer copies run
  // the link closer to a single DMA's rate -- synth1m with 4 / 8 / 12 / 16 MiB targets:
  // 1.24 / 1.21 / 1.185 / 1.19 ms in round 3; with round 4's shorter ordered kernel 10 MiB
  // beats 12 (median 1.047 vs 1.060 ms over five alternating rounds,
  // profiles/r4/piece_ab.txt)), at most partial_slots_cap of them.
  static constexpr u64 kPieceBytes = 4ull << 20;
  static constexpr u64 kDevPageBytes = 2ull << 20;  // device allocations: whole 2 MiB pages
  static u64 piece_target();
  // Page-locked host memory this engine holds now (its buffers; not the HIP runtime's own
  // per-device memory): the input text, the output pool, the stream staging / read ring,
  // the key staging and the small control blocks.
  u64 pinned_bytes() const;
  static constexpr u64 kMaxPieces = kMaxPartialSlots;
  std::vector<std::pair<u64, u64>> pieces;
  // run() opts a large dictionary pass into the combining map (records + d_counts);
  // map_combined: the current `tokens` came from it (consumers must weigh by d_counts).
  bool combine_map = false;
  bool map_combined = false;
  std::vector<hipEvent_t> ev_piece;
  hipEvent_t ev_fork = nullptr;
  OutRecord* d_out = nullptr;
  KeyCount* d_records = nullptr;   // shuffle payload (send on the map side, recv on reduce)
  // Records d_records holds (>= cap; at least one minimum-size gather slot).
  u64 slot_records_cap() const { return std::max<u64>(cap, kSlotRecordsMin); }
  PackedKey* d_samples = nullptr;
  PackedKey* d_splitters = nullptr;
  u64* d_offsets = nullptr;
  u64* d_offset = nullptr;

  // zeroed once per run: counters + every look-back region
  char* d_sync = nullptr;
  u64 sync_bytes = 0;
  MapCounters* d_ctr = nullptr;
  LookbackScratch lb_line{}, lb_compact{}, lb_map{}, lb_heads{}, lb_scan{}, lb_dict{};
  // LOCUST_VPLAN=0 (read at construction): the ordered kernel keeps one workgroup per map
  // partition (A/B of the in-job plan)
  const bool vplan = [] {
    const char* e = std::getenv("LOCUST_VPLAN");
    return !e || e[0] != '0';
  }();
  // LOCUST_VPLAN_MIN_KB: the smallest pass that plans (default 0: every untuned small
  // pass).  Whole Hamlet with the letters map ran 0.0436 ms unplanned vs 0.0455 planned,
  // but a size threshold cannot tell Hamlet from a pass of the same size whose keys crowd
  // one partition (30,000 'w0...' keys: the unplanned job overflowed its LDS table and
  // redid the exchange) -- the plan's split is what keeps such a first job on the LDS
  // path (profiles/r3_s4/default_map/split_ab.txt).
  const u64 vplan_min_bytes = [] {
    const char* e = std::getenv("LOCUST_VPLAN_MIN_KB");
    return (u64)(e ? std::max(0, std::atoi(e)) : 0) << 10;
  }();
  bool plan_pass = false;  // this pass's map writes occupancy and its ordered kernel plans
  // LOCUST_PLAN_TRIGGER=0 (read at construction): a planned pass plans in every job instead
  // of only when the map saw kPlanTrigger tokens of one partition in a tile (plan_flag)
  const bool plan_trigger = [] {
    const char* e = std::getenv("LOCUST_PLAN_TRIGGER");
    return !(e && e[0] == '0');
  }();
  u32* d_plan_flag = nullptr;
  bool plan_small() const { return plan_pass; }
  void decide_plan(u64 pass_bytes) {
    plan_pass = vplan && pm_retunes == 0 && pass_bytes >= vplan_min_bytes;
  }
  // LOCUST_SPLIT_MIN (read at construction): tokens per extra sibling workgroup of a
  // planned partition (0: the kernel's default, kSplitMinTokens)
  const u32 split_min = [] {
    const char* e = std::getenv("LOCUST_SPLIT_MIN");
    return e ? (u32)std::max(0, std::atoi(e)) : 0u;
  }();
  // Scratch of the merge kernels (launch_merge_*: they reset it themselves): the heads and
  // scan regions, which lie back to back -- 2 * (cap / kReduceTile + 1) status words.
  LookbackScratch lb_merge(u64 n) const {
    LOCUST_CHECK_ARG(merge_scratch_words(n) <= 2 * (div_up(cap, kReduceTile) + 1),
                     "merge larger than the engine's look-back scratch");
    return lb_heads;
  }
  RadixWorkspace rx{};

  // dictionary path: [table | ucount | rank] is one zeroed block
  DictWorkspace dict{};
  u64 dict_slots = 0;
  u64 ucap = 0;       // dense distinct-key capacity of the dictionary
  u64 h_out_cap = 0;  // records h_out holds
  u64 h_keys_cap = 0;
  u32* d_rank = nullptr;
  u64 dict_zero_bytes = 0;

  // streaming (inputs larger than one chunk), allocated on first use
  char* d_text_alt = nullptr;        // second device text buffer (double buffering)
  size_t d_text_alt_block = 0;       // its block size (devcache)
  char* h_stage[2] = {nullptr, nullptr};  // pinned staging halves for pageable inputs
  // a TextSource's pinned read ring: kRingPieces pieces of ring_piece bytes, whatever the
  // chunk size (host memory of a streamed file stays kRingPieces x ring_piece)
  static constexpr int kRingPieces = 4;
  static constexpr u64 kRingPieceMax = 16ull << 20;
  char* h_ring[kRingPieces] = {};
  hipEvent_t ev_ring[kRingPieces] = {};
  u64 ring_piece = 0;
  hipStream_t cstream = nullptr;     // H2D copy stream
  // Second copy stream for upload pieces: back-to-back copies on one stream leave the link
  // idle between commands (measured 43 GB/s for 4 MiB pieces on one stream, 52 GB/s
  // alternating over two -- the single-copy rate)
  hipStream_t cstream2 = nullptr;
  // Piece copies: issued at the very start of the job's enqueue, ahead of the compute
  // stream's resets (their fills delayed the first copy by ~20 us, profiles/r3_s4/), and
  // alternated over the two copy streams (one or three measured slower, copy_ab.txt).
  bool pieces_issued = false;  // this job's piece copies are already on the copy streams
  hipStream_t piece_stream(size_t k) const { return (k & 1) ? cstream2 : cstream; }
  void issue_piece_copies(const char* src);
  hipEvent_t ev_copied[2] = {}, ev_consumed[2] = {};
  MapCounters* d_dctr = nullptr;     // dictionary counters that persist across chunks
  MapCounters* h_chunk_ctr = nullptr;  // pinned per-window map counter snapshots
  u64 h_chunk_cap = 0;
  // Streamed maps (one per window): snapshots pending in h_chunk_ctr, and the sum of the
  // ones folded when it filled up (stream_stats adds both).
  u64 win_pending = 0;
  MapCounters win_acc{};
  void reset_window_counters() {
    win_pending = 0;
    win_acc = MapCounters{};
  }
  // Queues the snapshot of d_ctr after a window's map (folding the full array first).
  void snapshot_window_counters();
  // Map + dictionary insert of one window [dtext, dtext + len) of a streamed chunk.
  void enqueue_map_window(const char* dtext, u64 len, const DelimMask& dm);
  // Bytes of the next map window of host text [p, p + n): at most map_window bytes cut
  // after a '\n', or one line longer than that (<= emits_per_line tokens).
  u64 window_len(const char* p, u64 n) const;

  char* h_text = nullptr;
  char* d_h_text = nullptr;    // device view of the pinned h_text (zero-copy map input)
  const char* map_text = nullptr;  // what the map kernel reads this run
  MapCounters* h_ctr = nullptr;
  SortPlan* h_plan = nullptr;
  OutRecord* h_out = nullptr;         // host-mapped output records
  OutRecord* d_out_mapped = nullptr;  // device view of h_out
  u64* h_ctab = nullptr;              // its compact-output table (OrderedExtra::ctab)
  u64* d_ctab_mapped = nullptr;
  bool ord_compact = false;           // the last ordered launch wrote compact records
  MapCounters* h_ctr_mapped = nullptr;
  MapCounters* d_ctr_mapped = nullptr;
  // Lean jobs: completion word the last kernel publishes (host-mapped) and its sequence.
  u32* h_done = nullptr;
  u32* d_done = nullptr;
  u32 done_seq = 0;
  // set before enqueue_dict_job: a self-cleaning ordered kernel publishes this value
  // itself (and clears it); still set afterwards -> publish_done() behind the job
  u32 done_pending = 0;
  bool split_stages = false;  // run(): this job records per-stage events
  // Partition map of the ordered dictionary build (PartMap / locust/partmap.hpp): device
  // tables (persist across jobs), a pinned staging image, and the per-partition work the
  // ordered kernel reports each run (host-mapped) from which the host decides to retune.
  PartMapTables* d_pmap = nullptr;
  PartMapTables* h_pmap = nullptr;
  u32* h_pw = nullptr;
  u32* d_pw = nullptr;
  u64 pm_predicted_max = 0;  // predicted max partition work of the current map (0: default)
  u32 pm_retunes = 0;
  // ---- in-job partition plan of a large piecewise pass (partplan.hip) ----
  // Before piece 0 is mapped: a <= 1 MiB line-aligned prefix of it is mapped into scratch,
  // its distinct keys collected in a small HBM table, and launch_part_plan cuts the key
  // space at equal counts of them into d_pmap -- the pass's partitions come from its own
  // text, not from the previous job's output.  LOCUST_DEVPLAN=0 (read at construction):
  // the host-tuned map instead.  A planned pass that overflows an LDS table falls back as
  // before and hands this engine to the host-tuned map (devplan_failed).
  const bool devplan_env = [] {
    const char* e = std::getenv("LOCUST_DEVPLAN");
    return !e || e[0] != '0';
  }();
  bool devplan_failed = false;
  bool devplan_used = false;  // the current pass's map was planned on the device
  // d_pmap was tuned from a large pass's exact output (retune_with): later passes of the
  // engine take it (the plan costs ~0.1-0.2 ms of the pass; the tuned map is exact).
  // LOCUST_PART_TUNE=0 never tunes: every pass plans itself.
  bool pm_tuned = false;
  u32 fallbacks = 0, planned_passes = 0;  // diagnostics (GpuWordCount::stats)
  static constexpr u64 kPlanSampleBytes = 1ull << 20;
  static constexpr u64 kPlanCap = 1ull << 19;  // sample tokens kept
  char* d_plan = nullptr;                      // one allocation, made on first use
  u64 plan_zero_bytes = 0;                     // [MapCounters | table | ucount], zeroed per pass
  MapCounters* d_plan_ctr = nullptr;
  KeysSoA plan_keys{};
  DictWorkspace plan_dict{};
  void ensure_plan();
  // The plan's kernels, on `stream` once piece 0 (`len0` bytes at d_text; host copy at
  // `host`) has landed; the scratch was zeroed at the start of the pass.
  void enqueue_devplan(const char* host, u64 len0, const DelimMask& dm,
                       const char* dev_text = nullptr);
  u64* h_keys = nullptr;  // staging for key up/downloads (4 words x cap)
  PackedKey* h_small = nullptr;
  u64* h_u64 = nullptr;

  // This library's code objects on `device`, once per process (kernels.hpp).
  static void warm_modules_once(int device);

  DevicePipeline(const JobConfig& c, u64 max_bytes, u64 max_lines, u64 cap_records = 0);

  // The copy streams' first use (queue bring-up, the runtime's copy and fill kernels) in the
  // constructor, not in the first job: one piece-sized copy, a fill at an unaligned address
  // and a short read-back on each, as a piecewise upload issues them.
  void warm_copy_streams();

  ~DevicePipeline();

  // ---- host-mapped output buffers (zero-copy emit target AND zero-copy results) ----
  // A result adopts the buffer its job wrote (EntryList keeps it alive); the next job
  // takes a buffer no result holds any more, so jobs whose results are dropped in turn
  // alternate between two buffers and nothing is ever copied out.
  static constexpr u64 kMappedOutMax =
      kPartBuildMaxTokens > (u64)kRankSortMax ? kPartBuildMaxTokens : (u64)kRankSortMax;
  struct HostOut {
    OutRecord* h = nullptr;
    OutRecord* d = nullptr;
    u64 cap = 0;
    u64* ctab_h = nullptr;  // kDictParts words after the records: the compact table
    u64* ctab_d = nullptr;
    // fine-grained: the kernels write it straight over PCIe (coarse-grained buffers
    // measured no faster, profiles/r1_s3/out_coherence_ab.txt)
    explicit HostOut(u64 n) : cap(std::max<u64>(n, 1)) {
      h = static_cast<OutRecord*>(pinned_alloc(cap * sizeof(OutRecord) + kDictParts * sizeof(u64),
                                               hipHostMallocMapped | hipHostMallocCoherent,
                                               "mapped result buffer"));
      LOCUST_HIP_CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&d), h, 0));
      ctab_h = reinterpret_cast<u64*>(h + cap);
      ctab_d = reinterpret_cast<u64*>(d + cap);
    }
    ~HostOut() { pinned_free(h); }
    HostOut(const HostOut&) = delete;
    HostOut& operator=(const HostOut&) = delete;
  };
  std::vector<std::shared_ptr<HostOut>> out_pool;
  size_t out_idx = 0;
  void use_out(size_t i);
  // Before a job writes the mapped output: a buffer no earlier result still holds.
  void select_out();
  // ... with room for n records (grown when a radix-path result has more distinct keys
  // than the dictionary's capacity).
  void grow_host_out(u64 n);
  // Pinned staging for key up/downloads (stage-split paths only), allocated on demand.
  void grow_host_keys(u64 n);

  void check_input(const TextInput& in) const {
    if (in.bytes > pass_bytes || in.num_lines > cap_lines)
      throw Error("input (" + std::to_string(in.bytes) + " B, " + std::to_string(in.num_lines) +
                  " lines) exceeds engine capacity (" + std::to_string(cap_bytes) + " B, " +
                  std::to_string(cap_lines) + " lines)");
  }

  // (Spinning on hipStreamQuery instead measured no faster, profiles/r3_s4/spin_sync_ab.txt.)
  void sync() { LOCUST_HIP_CHECK(hipStreamSynchronize(stream)); }
  // Lean jobs: the stream's last kernel publishes `seq` to h_done; poll it (bounded, then
  // a real synchronisation -- a long job does not burn the core, a failed one reports).
  void publish_done(u32 seq) { launch_signal_host(d_done, seq, stream); }
  // bounded_sync=false: just return after the bound (the caller synchronises itself).
  void wait_done(u32 seq, bool bounded_sync = true);

  // H2D of the text; zero counters and look-back scratch.
  //  * zero-copy (small inputs, fast map): no copy at all -- the map kernel's 16-byte
  //    staging loads read the pinned host buffer over PCIe, which for a ~200 KB text is
  //    cheaper than an SDMA transfer's fixed latency.
  //  * pinned input elsewhere (HostText): DMA straight from it.
  //  * otherwise: host copy into the pinned buffer, then DMA.
  void enqueue_upload(const TextInput& in);
  // Host half: stage the text where the device half expects it and pick the map's source.
  enum class Upload { kZeroCopy, kDirect, kStaged };
  Upload upload_mode = Upload::kStaged;
  void prepare_upload(const TextInput& in);
  // Line-aligned pieces of a large single-pass input (none: one copy, one map launch).
  void plan_pieces(const TextInput& in);
  u32 piece_tiles() const {
    u64 t = 0;
    for (const auto& pc : pieces) t += div_up(pc.second, kMapTileBytesLarge);
    return t <= part_off_tiles ? (u32)t : 0u;
  }
  void ensure_piece_events(size_t n);
  // Device half (capturable): the DMA if any, then the per-run reset of counters and
  // look-back scratch.
  void enqueue_upload_device(const TextInput& in);
  // d_sync is all zero: the last job was a self-cleaning ordered run (see OrderedExtra).
  // Only run() sets it; every other entry point must clear it before touching d_sync.
  bool sync_clean = false;
  bool skip_sync_reset = false;  // enqueue_upload_device leaves out the reset (run() only)

  // ---- captured launch sequences (hipGraph), keyed by call site and shape ----
  using GraphKeyArr = std::array<u64, 6>;
  struct CachedGraph {
    GraphKeyArr key;
    hipGraphExec_t exec;
  };
  std::vector<CachedGraph> graph_cache;
  // Replays the sequence `enqueue` captured for `key`, capturing it on first use.  The
  // sequence may only enqueue work on `stream` (kernels, memsets, async copies).
  template <class F>
  void launch_cached(const GraphKeyArr& key, F&& enqueue) {
    for (auto& g : graph_cache)
      if (g.key == key) {
        LOCUST_HIP_CHECK(hipGraphLaunch(g.exec, stream));
        return;
      }
    if (graph_cache.size() >= 8) {  // shapes changed a lot: drop the oldest
      LOCUST_HIP_CHECK(hipGraphExecDestroy(graph_cache.front().exec));
      graph_cache.erase(graph_cache.begin());
    }
    hipGraph_t g = nullptr;
    LOCUST_HIP_CHECK(hipStreamBeginCapture(stream, hipStreamCaptureModeRelaxed));
    enqueue();
    LOCUST_HIP_CHECK(hipStreamEndCapture(stream, &g));
    hipGraphExec_t exec = nullptr;
    LOCUST_HIP_CHECK(hipGraphInstantiate(&exec, g, nullptr, nullptr, 0));
    LOCUST_HIP_CHECK(hipGraphDestroy(g));
    graph_cache.push_back({key, exec});
    LOCUST_HIP_CHECK(hipGraphLaunch(exec, stream));
  }

  // ---- hipGraph replay of the dictionary job ----
  struct GraphKey {
    u64 bytes = ~0ull;
    u64 lines = 0;
    const char* src = nullptr;
    const char* map_text = nullptr;
    Upload mode = Upload::kStaged;
    const OutRecord* out = nullptr;  // the host-mapped output buffer the graph writes
    bool no_reset = false;           // captured without the d_sync reset (clean start)
    u64 pieces_sig = 0;              // the upload pieces (line-aligned: content dependent)
    bool operator==(const GraphKey& o) const {
      return bytes == o.bytes && lines == o.lines && src == o.src && map_text == o.map_text &&
             mode == o.mode && out == o.out && no_reset == o.no_reset && pieces_sig == o.pieces_sig;
    }
  };
  struct DictGraph {
    GraphKey key;
    hipGraphExec_t exec;
    bool ordered;  // the captured job uses the ordered kernel
    bool clean;    // ... and re-zeroes its scratch (job_self_cleaned)
    bool compact;  // ... writing compact records (ord_compact)
  };
  std::vector<DictGraph> dict_graphs;  // one per (input shape, output buffer)
  bool graph_ordered = false;          // the last launched graph uses the ordered kernel
  // Dictionary jobs, and radix jobs that stay on the device end to end (partitioned sort
  // from the fast map's table, records straight into the mapped output: no host sync).
  // (A piecewise upload is never captured: its copy/map fork-join replayed from a graph
  // lost the overlap -- measured 1.91 vs 1.52 ms on 1M synthetic lines.)
  bool use_graph() const {  // dictionary jobs (the shard engine's entry points)
    if (cfg.graph >= 0) return cfg.graph > 0 && cfg.sort_path == SortPath::kDict;
    return cfg.sort_path == SortPath::kDict && cfg.map_path == MapPath::kFast;
  }
  bool use_job_graph(const TextInput& in) const;
  // Lean jobs: what auto mode used to replay as a graph (small single-pass dictionary jobs,
  // device-resident radix jobs) launched directly and completed by polling a host word.
  // Measured on the box: a 3-node graph replay + sync costs ~20 us of launch/wake-up per
  // job, 3 direct launches + a polled completion word ~11 us (tools/micro/launch_lat.hip).
  // LOCUST_LEAN=0: the graph replay (cfg.graph < 0) / event-timed path instead.
  static bool lean_enabled();
  // The shard engine's cached sequences (small pass, merge tails): replayed graphs only
  // when asked for (graph=1); in auto mode direct launches are cheaper (see lean_job).
  bool graph_launches() const { return use_graph() && !(cfg.graph < 0 && lean_enabled()); }
  bool lean_job(const TextInput& in) const {
    if (!lean_enabled() || cfg.graph >= 0 || cfg.map_path != MapPath::kFast) return false;
    if (large_ordered && in.bytes >= 2 * kPieceBytes) return false;
    if (cfg.sort_path == SortPath::kDict) return true;
    return table_tiles(in.bytes) > 0 && radix_mapped() && psort_enabled();
  }
  // Capture [upload DMA + reset, map, dictionary build, rank, emit] once per input shape
  // and source; later runs replay it with one hipGraphLaunch.
  void launch_dict_graph(const TextInput& in, bool compat);
  bool use_zero_copy(const TextInput& in) const {
    if (cfg.map_path != MapPath::kFast || !d_h_text) return false;
    if (cfg.zero_copy_text >= 0) return cfg.zero_copy_text > 0;
    return in.bytes <= kZeroCopyMaxBytes;
  }

  void enqueue_map(const TextInput& in);

  // Compaction (compat path) + radix sort of `tokens` into `sorted` (and counts).
  // host_n: record count when the host already knows it.  With sync_plan the count is
  // read back (one 4-byte D2H) so the sort can pick its regime and exact grids; without
  // it everything stays on the device (graph-capturable).
  // allow_psort: the caller checks kCtrSortOverflow afterwards (psort_overflow_redo).
  void enqueue_process(u32 num_lines, bool compat, bool with_counts, u64 host_n = kUnknownCount,
                       bool allow_psort = false);

  // The unweighted tokens of the small-input fast map (per-tile partition table present)
  // take the partitioned LDS sort; everything else the device-wide LSD sort.
  static bool psort_enabled() {  // LOCUST_PSORT=0: A/B against the device-wide sort
    const char* v = std::getenv("LOCUST_PSORT");
    return !(v && v[0] == '0');
  }
  bool psort_ok(bool compat, bool with_counts) const {
    return psort_enabled() && !compat && !with_counts && parts_ready && part_tiles > 0 &&
           cap <= kPartBuildMaxTokens;
  }
  bool psort_used = false;  // the last enqueue_process took the partitioned sort

  // Process + Reduce of the reference algorithm (sort every token, boundary mark + head
  // compaction + adjacent difference), records packed into the host-mapped output with a
  // counter snapshot when every possible key fits it (then the host needs no D2H), else
  // into d_out.  Events (optional; not while capturing) mark the stage ends.
  bool radix_mapped() const { return h_out_cap >= cap; }
  bool radix_fused = false;  // the last radix job took the fused sort + reduce kernel
  void enqueue_radix_job(u32 num_lines, bool compat, hipEvent_t after_process,
                         hipEvent_t after_reduce);
  // After a psort partition overflowed (kCtrSortOverflow): sort the same tokens with the
  // device-wide LSD sort and reduce again (the map output is still in `tokens`).
  void redo_radix_general(u32 num_lines);
  // The Process stage alone, again, on the device-wide sort (flags cleared).
  void redo_process_general(u32 num_lines) {
    LOCUST_HIP_CHECK(hipMemsetAsync(&d_ctr->flags, 0, sizeof(u32), stream));
    enqueue_process(num_lines, false, false, h_ctr->num_records);
  }

  // Head mark + compaction + adjacent difference over `sorted` (weighted when counts).
  void enqueue_reduce_core(bool with_counts);

  void enqueue_pack_output() {
    ensure_radix_full();
    launch_pack_output(heads, d_head_val, d_head_count, cap, d_ctr, d_out, stream);
  }

  // ---- dictionary path (SortPath::kDict): no host synchronisation inside ----
  void enqueue_process_dict(u32 num_lines, bool compat, bool with_counts = false) {
    enqueue_dict_insert(num_lines, compat, with_counts);
    enqueue_rank();
  }
  // Every token (or weighted record) into a fresh dictionary: the partitioned LDS build
  // when the tokens carry partition tags and the pass is small, else the HBM table.
  void enqueue_dict_insert(u32 num_lines, bool compat, bool with_counts);
  // Ranks of the distinct keys (rank and uval must be zero): the weighted rank -- the
  // all-pairs pass also sums the counts of the smaller keys, which IS the output's val,
  // and rank_emit writes the records straight from it.  (Ranks only + a look-back scan of
  // the counts in rank order measured slower; git history keeps it.)
  void enqueue_rank() {
    launch_rank_sort(dict.ukeys, dict.ucount, &d_ctr->num_unique, ucap, d_rank, dict.uval,
                     stream);
  }
  // Process + Reduce of the dictionary path in ONE kernel (ordered partitions, see
  // launch_dict_ordered) when the tokens carry partition tags and the pass is small.
  bool ordered_ok() const { return parts_ready && (cap <= kPartBuildMaxTokens || small_pass); }
  // Two-kernel ordered build of a large pass (the map wrote its partition table).
  bool large_ordered_ok() const {
    return large_ordered && parts_ready && part_tiles > 0 && cap > kPartBuildMaxTokens;
  }
  // Its first kernel: the partials of kOrdWorkers tile slices, unless the piecewise map
  // already wrote one slot per piece (partial_nslots).
  void enqueue_partials();
  // Tiles of the per-tile partition table the fast map writes for an input of `bytes`
  // (0: no table for this input).
  u32 table_tiles(u64 bytes) const {
    const u64 t = div_up(bytes, map_tile_bytes(bytes));
    return d_part_off && t <= part_off_tiles ? (u32)t : 0u;
  }
  // The ordered kernel reads partition runs from the map's per-tile table when the current
  // tokens came from the small-input fast map (unweighted).
  void set_tile_source(OrderedExtra& ex, bool with_counts) const;
  // Fills the self-clean fields of an OrderedExtra (see OrderedExtra::self_clean).
  void set_self_clean(OrderedExtra& ex) const {
    ex.self_clean = true;
    ex.map_lb = lb_map;
    ex.map_words = (u32)(div_up(pass_bytes, kMapTileBytesMin) + 1);
    ex.done_counter = lb_dict.tile_counter + 1;  // the sync block's spare counter word
  }
  // Device view of this pipeline's partition map (tables live at fixed addresses, so
  // captured graphs stay valid when the host retunes the contents).
  PartMap part_map() const {
    PartMap pm;
    pm.lo = d_pmap->lo;
    return pm;
  }
  // After a successful ordered run (ordered kernel wrote h_pw and the sorted output
  // `e[0..n)`): if its partitions were badly unbalanced, rebuild the map from this output
  // for the next job.  Cheap to check (256 words); a rebuild is one pass over the output.
  // Largest reported partition work when a rebuild looks worthwhile, else 0.
  u64 retune_wanted() const;
  // After an ordered run overflowed a partition (or the output): rebuild the map from the
  // fallback's output so the next job's partitions fit (kept if it would not help).
  void force_retune(const EntryList& e);
  void upload_pmap(const PartMapTables& t, u64 pred) {
    *h_pmap = t;
    LOCUST_HIP_CHECK(hipMemcpyAsync(d_pmap, h_pmap, sizeof(PartMapTables), hipMemcpyHostToDevice,
                                    stream));
    pm_predicted_max = pred;
  }
  // The map is built on the engine's worker thread (part_map_from_entries took ~0.15 ms of
  // a small first job's wall time inline, ~2 ms over 200K entries); the next job takes it
  // if it is ready and otherwise runs on what it has (the in-job plan, or the current map).
  // The task holds the output buffer, which the pool then skips.
  void maybe_retune(const EntryList& e);
  // One two-byte job at construction (GpuWordCount engines that run lean jobs): the map and
  // the ordered build launched once on this engine's stream with their own argument
  // blocks, so a fresh engine's first real job does not enqueue them for the first time
  // (~15-20 us more than later jobs, tools/cold_probe.py).  No retune, no trace output.
  void warm_first_job();
  bool warming = false;
  struct RetuneTask {
    u64 mx = 0, pred = 0;
    PartMapTables t;
    std::shared_ptr<HostOut> hold;
    EntryList entries;
    std::vector<PartGroup> groups;
    std::atomic<bool> released{true};  // the worker has let go of the output buffer
    u64 t_submit = 0, t_start = 0, t_released = 0, t_done = 0;  // (debug log)
  };
  RetuneTask retune_task;
  bool retune_pending = false;  // a task was handed to the worker and not adopted yet
  TaskWorker retune_worker;
  // Before a job: adopt a finished background retune (never waits).
  void poll_retune();
  // The same when the sorted output is device KeyCount records (the distributed map): one
  // D2H of them, only when a rebuild is due.
  void maybe_retune_records(const KeyCount* d_recs, u64 n, bool force = false);
  void retune_with(u64 mx, u64 pred, const PartMapTables& t);
  void enqueue_dict_ordered(bool with_counts, bool mapped, bool self_clean = false);
  // Diagnostics: LOCUST_ORD_TRACE=1 prints the ordered kernel's per-partition phase times
  // (shader clock ticks) after each run.
  u64* d_ord_trace = nullptr;
  u64* ord_trace();
  // Diagnostics: LOCUST_MAP_TRACE=1 prints the fast map kernel's per-tile timeline (us,
  // device-wide real-time clock) after each run.
  u64* d_map_trace = nullptr;
  u64* map_trace();
  void print_map_trace();
  // LOCUST_ORD_TRACE=1 on a large pass: the partials kernel's per-workgroup timeline.
  u64* d_partials_trace = nullptr;
  u64* partials_trace();
  void print_partials_trace();
  // LOCUST_ORD_TRACE=1 on the radix path: the partitioned sort's per-partition phases.
  void print_psort_trace();
  void print_ord_trace();
  // The last enqueue_dict_job's kernels re-zero the scratch they dirty (small ordered
  // build with self_clean): the next run() may skip the reset.
  bool job_self_cleaned = false;
  // Process + emit of a dictionary run; returns true if the ordered kernel was used.
  bool enqueue_dict_job(u32 num_lines, bool compat, bool with_counts, hipEvent_t after_process,
                        bool self_clean = false);
  // After an ordered run reported a partition overflow: redo Process + emit through the
  // HBM table (the map output is still in `tokens`).
  void redo_dict_on_table(u32 num_lines, bool with_counts);
  // Sorted distinct keys + counts (for the shuffle's range partition).
  void enqueue_sorted_from_dict() {
    launch_rank_scatter(dict.ukeys, dict.ucount, d_rank, &d_ctr->num_unique, ucap, sorted,
                        d_sorted_counts, stream);
  }
  // Output records in key order; `mapped` writes them (and the counters) straight into
  // host memory (zero-copy: the host needs no D2H).
  void enqueue_emit_dict(bool mapped) {
    launch_rank_emit(dict.ukeys, dict.ucount, d_rank, dict.uval, ucap, d_ctr,
                     mapped ? d_out_mapped : d_out, mapped ? d_ctr_mapped : nullptr, stream);
  }
  // Radix-fallback reduce: scan of the sorted counts -> records in d_out.
  void enqueue_reduce_dict() {
    launch_scan_pack(sorted, d_sorted_counts, rcap, d_ctr, d_out, lb_scan, stream);
  }
  // After the counters are read: a dictionary run whose distinct-key count exceeded the
  // rank sort's range (or whose table overflowed) is finished on the radix path.
  bool dict_fallback_needed() const {
    return (h_ctr->flags & (kCtrDictOverflow | kCtrNotEmitted)) ||
           h_ctr->num_unique > (u32)kRankSortMax;
  }
  void finish_dict_with_radix(u32 num_lines, bool with_counts = false);

  void read_counters() {
    LOCUST_HIP_CHECK(
        hipMemcpyAsync(h_ctr, d_ctr, sizeof(MapCounters), hipMemcpyDeviceToHost, stream));
    sync();
  }

  void download_output(WordCountResult& r, hipEvent_t done);

  // An ordered launch writing the mapped output writes compact records (kv.hpp): the
  // drain across PCIe shrinks from 40 B per entry to ~16-24 B.
  void set_compact_out(OrderedExtra& ex, bool mapped);

  // Host output records -> result entries: the result simply adopts the buffer the device
  // wrote (no copy; see select_out) -- 40-B records (the same layout as WordCountEntry),
  // or with `compact` the ordered kernel's compact segments, one per virtual partition,
  // listed in its table.
  void copy_out(EntryList& e, u64 u, bool compact = false);

  void fill_counters(WordCountResult& r) const;

  static double ms_between(hipEvent_t a, hipEvent_t b) {
    float ms = 0;
    LOCUST_HIP_CHECK(hipEventElapsedTime(&ms, a, b));
    return ms;
  }

  // Reference-semantics timing (JobConfig.ref_timers): the same device work, with host
  // timestamps where main.cu:405-468 took them.  The H2D happens before the first timer,
  // as main.cu:403 does.
  WordCountResult run_ref_timed(const TextInput& in);

  WordCountResult run(const TextInput& in);

  // ---------------------------------------------------------------------------------
  // Streaming: an input larger than the engine's text capacity is processed in
  // line-aligned chunks of <= cap_bytes.  Chunk k+1's H2D runs on the copy
  // stream while chunk k is mapped and folded into ONE dictionary that persists across
  // chunks; the distinct keys are ranked and emitted once at the end.  Device memory is
  // therefore bounded by the chunk size plus the dictionary, not by the input size.
  // ---------------------------------------------------------------------------------
  static bool host_pinned(const void* p);

  void ensure_stream_buffers(bool staging, u64 nchunks);
  // the read ring's piece size for a TextSource stream, and its (re)allocation
  u64 stream_ring_piece() const;
  void ensure_read_ring(u64 piece);

  char* ensure_h_text();

  // Line-aligned chunk boundaries, each <= cap_bytes.
  std::vector<std::pair<u64, u64>> plan_chunks(const TextInput& in) const;

  // Streams every chunk of `in` through map + dictionary insert (the table is reset
  // first).  When the stream has drained, d_ctr->num_unique / flags describe the whole
  // dictionary and h_chunk_ctr[0 .. chunks) holds each chunk's map counters.
  size_t enqueue_stream_insert(const TextInput& in);
  // The same from a TextSource (a file): line-aligned pieces are read into a small ring of
  // pinned buffers and copied into the current device chunk while the device maps the
  // previous chunk -- host memory stays kRingPieces x ring_piece (64 MiB), independent of
  // the chunk size.  A chunk closes when the next piece would not fit.
  size_t enqueue_stream_source(TextSource& src_text);
  // produce(b, &src): the next chunk's bytes at *src (pinned) -- when `staging`, into
  // h_stage[b], whose previous H2D has drained by then; returns its length, 0 at the end.
  template <class Produce>
  size_t enqueue_stream_chunks(bool staging, u64 max_chunks, Produce&& produce) {
    LOCUST_CHECK_ARG(cfg.sort_path == SortPath::kDict && cfg.map_path == MapPath::kFast,
                     "inputs larger than the engine capacity stream through the dictionary "
                     "path with the fast map (sort=dict, map=fast)");
    LOCUST_CHECK_ARG(cap >= map_window / 2 + 1,
                     "a streaming engine must be sized by bytes (max_lines >= max_bytes / 40)");
    ensure_stream_buffers(staging, max_chunks * (div_up(cap_bytes, map_window) + 1));
    reset_window_counters();
    const DelimMask dm = make_delim_mask(cfg.delimiters.c_str());
    LOCUST_HIP_CHECK(hipMemsetAsync(dict.table, 0, dict_zero_bytes, stream));
    LOCUST_HIP_CHECK(hipMemsetAsync(d_dctr, 0, sizeof(MapCounters), stream));
    // the copy stream must not overwrite a text buffer before the reset is queued
    LOCUST_HIP_CHECK(hipEventRecord(ev_copied[1], stream));
    LOCUST_HIP_CHECK(hipStreamWaitEvent(cstream, ev_copied[1], 0));
    size_t k = 0;
    for (;; ++k) {
      const int b = (int)(k & 1);
      char* dtext = b ? d_text_alt : d_text;
      // the staging half's previous H2D must have drained before it is refilled
      if (staging && k >= 2) LOCUST_HIP_CHECK(hipEventSynchronize(ev_copied[b]));
      const char* src = nullptr;
      const u64 len = produce(b, &src);
      if (!len) break;
      if (k >= 2) LOCUST_HIP_CHECK(hipStreamWaitEvent(cstream, ev_consumed[b], 0));
      LOCUST_HIP_CHECK(hipMemcpyAsync(dtext, src, len, hipMemcpyHostToDevice, cstream));
      LOCUST_HIP_CHECK(hipMemsetAsync(dtext + len, 0, 16, cstream));
      LOCUST_HIP_CHECK(hipEventRecord(ev_copied[b], cstream));

      LOCUST_HIP_CHECK(hipStreamWaitEvent(stream, ev_copied[b], 0));
      // the chunk in windows of <= map_window bytes (cut after a newline, found in the
      // host copy): the token buffers hold one window
      for (u64 off = 0; off < len;) {
        const u64 wl = window_len(src + off, len - off);
        enqueue_map_window(dtext + off, wl, dm);
        off += wl;
      }
      LOCUST_HIP_CHECK(hipEventRecord(ev_consumed[b], stream));
    }
    // hand the dictionary's counters to the single-pass stages that follow
    LOCUST_HIP_CHECK(hipMemcpyAsync(&d_ctr->num_unique, &d_dctr->num_unique, sizeof(u32),
                                    hipMemcpyDeviceToDevice, stream));
    LOCUST_HIP_CHECK(hipMemcpyAsync(&d_ctr->flags, &d_dctr->flags, sizeof(u32),
                                    hipMemcpyDeviceToDevice, stream));
    return k;
  }

  // After the stream has drained: whole-input map statistics from the chunk snapshots.
  void stream_stats(size_t nchunks, WordCountResult& r) const;

  WordCountResult run_stream(const TextInput& in) {
    return finish_stream(in.num_lines, [&] { return enqueue_stream_insert(in); });
  }
  WordCountResult run_source(TextSource& src);
  template <class Enqueue>
  WordCountResult finish_stream(u64 num_lines, Enqueue&& enqueue_chunks) {
    WordCountResult r;
    r.num_lines = num_lines;
    const u64 t0 = now_ns();
    LOCUST_HIP_CHECK(hipEventRecord(ev[0], stream));
    LOCUST_HIP_CHECK(hipEventRecord(ev[1], stream));
    const size_t nchunks = enqueue_chunks();
    LOCUST_HIP_CHECK(hipEventRecord(ev[2], stream));
    enqueue_rank();
    LOCUST_HIP_CHECK(hipEventRecord(ev[3], stream));
    enqueue_emit_dict(/*mapped=*/true);
    LOCUST_HIP_CHECK(hipEventRecord(ev[4], stream));
    LOCUST_HIP_CHECK(hipEventRecord(ev[5], stream));
    sync();
    *h_ctr = *h_ctr_mapped;
    if (h_ctr->flags & kCtrDictOverflow)
      throw Error("streaming dictionary overflow: more than " + std::to_string(ucap) +
                  " distinct keys; use a larger chunk size");
    if (dict_fallback_needed()) {
      // more distinct keys than the rank sort takes: LSD radix sort of the dictionary
      finish_dict_with_radix(0);
      LOCUST_HIP_CHECK(hipEventRecord(ev[4], stream));
      download_output(r, ev[5]);
    } else {
      copy_out(r.entries, h_ctr->num_unique);
    }
    stream_stats(nchunks, r);
    r.num_unique = r.entries.size();
    r.times.wall_ms = (now_ns() - t0) * 1e-6;
    r.times.h2d_ms = 0;  // overlapped with the map: included in map_ms
    r.times.map_ms = ms_between(ev[1], ev[2]);
    r.times.process_ms = ms_between(ev[2], ev[3]);
    r.times.reduce_ms = ms_between(ev[3], ev[4]);
    r.times.d2h_ms = ms_between(ev[4], ev[5]);
    if (cfg.check) validate_result(r);
    return r;
  }

  void download_keys(const KeysSoA& src, u64 n, std::vector<PackedKey>* out);

  void set_num_records(u64 n);

  void upload_tokens(const PackedKey* keys, u64 n) {
    parts_ready = false;
    part_tiles = 0;
    set_num_records(n);
    upload_keys(tokens, keys, n);
  }
  // Host keys (AoS) into device SoA words through the pinned key staging.
  void upload_keys(const KeysSoA& dst, const PackedKey* keys, u64 n);
};


}  // namespace detail
}  // namespace locust
