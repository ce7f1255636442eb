// Out-of-line members of DevicePipeline (csrc/engine/pipeline.hpp): the engine's host-side
// job logic -- construction and sizing, uploads, the map / Process / Reduce enqueue paths,
// partition-map retuning, graph capture, streaming and the result hand-over -- compiled once
// here instead of in every translation unit that includes the header.
#include "pipeline.hpp"

namespace locust {
namespace detail {

u64 DevicePipeline::piece_target() {
  static const u64 b = [] {
    const char* e = std::getenv("LOCUST_PIECE_MB");
    const long mb = e ? std::atol(e) : 10;
    return (u64)std::max<long>(mb, 4) << 20;
  }();
  return b;
}

u64 DevicePipeline::pinned_bytes() const {
  u64 b = 0;
  if (h_text) b += cap_bytes + 64;
  for (const auto& o : out_pool) b += o->cap * sizeof(OutRecord) + kDictParts * sizeof(u64);
  for (int k = 0; k < 2; ++k)
    if (h_stage[k]) b += cap_bytes + 64;
  for (int i = 0; i < kRingPieces; ++i)
    if (h_ring[i]) b += ring_piece + 64;
  b += h_keys_cap * kKeyWords * sizeof(u64);
  b += h_chunk_cap * sizeof(MapCounters);
  b += 2 * sizeof(MapCounters) + sizeof(SortPlan) + 2 * sizeof(PartMapTables) +
       kMaxSamples * sizeof(PackedKey) + (kMaxRanks + 8) * sizeof(u64) + 64 +
       kDictParts * sizeof(u32);
  return b;
}

void DevicePipeline::issue_piece_copies(const char* src) {
  ensure_piece_events(pieces.size());
  for (size_t k = 0; k < pieces.size(); ++k) {
    const u64 off = pieces[k].first, len = pieces[k].second;
    hipStream_t cs = piece_stream(k);
    LOCUST_HIP_CHECK(hipMemcpyAsync(d_text + off, src + off, len, hipMemcpyHostToDevice, cs));
    LOCUST_HIP_CHECK(hipEventRecord(ev_piece[k], cs));
  }
  pieces_issued = true;
}

void DevicePipeline::ensure_plan() {
  if (d_plan) return;
  const u64 slots = 2 * kPlanCap;  // load factor <= 0.5
  const u64 ctr_b = align_up(sizeof(MapCounters), 256), tab_b = align_up(slots * sizeof(DictSlot), 256);
  plan_zero_bytes = ctr_b + tab_b + kPlanCap * 8;
  const u64 total = plan_zero_bytes + 256 + (4 + 4 + 1) * kPlanCap * 8 + kPlanCap * 4 + 4096;
  LOCUST_HIP_CHECK(hipMalloc(&d_plan, total));
  char* c = d_plan;
  d_plan_ctr = reinterpret_cast<MapCounters*>(c);
  plan_dict.table = reinterpret_cast<DictSlot*>(c + ctr_b);
  plan_dict.ucount = reinterpret_cast<u64*>(c + ctr_b + tab_b);
  c = d_plan + align_up(plan_zero_bytes, 256);
  for (int j = 0; j < kKeyWords; ++j, c += kPlanCap * 8) plan_dict.ukeys.w[j] = reinterpret_cast<u64*>(c);
  for (int j = 0; j < kKeyWords; ++j, c += kPlanCap * 8) plan_keys.w[j] = reinterpret_cast<u64*>(c);
  plan_dict.uval = reinterpret_cast<u64*>(c);
  c += kPlanCap * 8;
  plan_dict.urank = reinterpret_cast<u32*>(c);
  plan_dict.mask = (u32)(slots - 1);
  plan_dict.ucap = (u32)kPlanCap;
}

void DevicePipeline::enqueue_devplan(const char* host, u64 len0, const DelimMask& dm,
                       const char* dev_text) {
  u64 n = std::min<u64>(len0, kPlanSampleBytes);
  if (n < len0) {
    const void* nl = memrchr(host, '\n', (size_t)n);
    if (nl) n = (u64)(static_cast<const char*>(nl) - host) + 1;
  }
  launch_map_fast(dev_text ? dev_text : d_text, n, dm, cfg.emits_per_line, cfg.max_key_len,
                  plan_keys, nullptr, kPlanCap, d_plan_ctr, lb_map, stream);
  launch_dict_insert(plan_keys, nullptr, &d_plan_ctr->num_records, kPlanCap, plan_dict,
                     d_plan_ctr, stream);
  launch_part_plan(plan_dict.ukeys.w[0], plan_dict.ucount, &d_plan_ctr->num_unique,
                   plan_dict.ucap, d_pmap, stream);
}

void DevicePipeline::warm_modules_once(int device) {
  static std::mutex mu;
  static u64 warmed = 0;  // bit per device
  std::lock_guard<std::mutex> lk(mu);
  const u64 bit = 1ull << (device & 63);
  if (warmed & bit) return;
  warm_kernel_modules();
  // the first roctx range of a process initialises the library (~0.12 ms, measured inside
  // a fresh engine's first job): pay it here
  { TraceRange warm("locust:warm"); }
  warmed |= bit;
}

// The arena's layout for a planned pass: the same sequence of buffers the constructor
// takes, so plan_device_pass prices an engine exactly before it exists.
DevicePipeline::ArenaShape DevicePipeline::shape_arena(const JobConfig& cfg, const DevicePassPlan& p,
                                                       u64 small_pass_bytes) {
  ArenaShape sh;
  const bool compat = cfg.map_path == MapPath::kCompat;
  const u64 cap_bytes = p.chunk_bytes, pass_bytes = p.pass_bytes, cap_lines = p.cap_lines;
  const u64 cap = p.cap, ucap = p.ucap, rcap = p.rcap;
  const bool streaming = p.streaming;
  // the reference algorithm's head buffers (boundary mark, prefix, adjacent difference):
  // a dictionary engine whose sort buffers hold its distinct keys only never reduces
  // that way until ensure_radix_full makes them
  const u64 hcap = rcap < cap ? 1 : rcap;
  sh.slot_cap = compat ? cap_lines * (u64)cfg.emits_per_line : 1;
  sh.t_line = div_up(pass_bytes, kLineIdxTile) + 1;
  sh.t_compact = div_up(cap_lines, 256) + 1;
  sh.t_map = div_up(pass_bytes, kMapTileBytesMin) + 1;
  sh.t_heads = div_up(cap, kReduceTile) + 1;
  sh.t_scan = div_up(cap, kReduceTile) + 1;
  sh.rx_zero_words = radix_zero_bytes(rcap) / 4;
  // Hash table: >= 2x the distinct keys it can see (load factor <= 0.5), capped at
  // 2^25 slots (16M distinct keys per call; beyond that the radix path takes over).
  sh.dict_slots = 1024;
  while (sh.dict_slots < 2 * ucap) sh.dict_slots <<= 1;
  // [table | ucount | uval | rank]
  sh.dict_zero_bytes = align_up(sh.dict_slots * sizeof(DictSlot), 256) +
                       2 * align_up(ucap * 8, 256) + ucap * 4;
  sh.rx_part_words = (u64)radix_hist_blocks(rcap) * kNumPositions * 256;
  sh.sync_bytes = 256 + 8 * (sh.t_line + sh.t_compact + sh.t_map + sh.t_heads + sh.t_scan +
                             kDictParts + 1);

  SizingPlan sz;
  sz.add<char>(cap_bytes + 64);
  sz.add<u64>(compat ? cap_lines + 1 : 1);  // the line index: compat map only
  sz.add<char>(64);
  for (int j = 0; j < kKeyWords; ++j) {
    sz.add<u64>(sh.slot_cap);
    sz.add<u64>(cap);   // tokens
    sz.add<u64>(rcap);  // sorted
    sz.add<u64>(hcap);  // heads
  }
  sz.add<u32>(compat ? cap_lines : 1);
  sz.add<u64>(cap);   // d_counts (per token)
  sz.add<u64>(rcap);  // d_sorted_counts
  for (int k = 0; k < 3; ++k) sz.add<u64>(hcap);  // d_prefix, d_head_val, d_head_count
  sz.add<u32>(rcap);
  sz.add<u8>(align_up(cap, 16) + 16);
  // A pass of at most small_pass_bytes (1 KiB tiles <= kPartBlock: the in-job plan's
  // range) takes the one-kernel ordered build whatever its worst-case token count: natural
  // text has a third of the tokens the capacity allows, and the large build's device plan
  // cost ~0.2 ms of a 0.3 ms untuned job at 3-5x Hamlet (docs/PERFORMANCE.md round 5).
  sh.small_pass = cap > kPartBuildMaxTokens && cap_bytes <= small_pass_bytes && !streaming &&
                  cfg.map_path == MapPath::kFast && cfg.sort_path == SortPath::kDict;
  if ((cap <= kPartBuildMaxTokens || sh.small_pass) && cap_bytes < kMapLargeInput) {
    sh.part_off_tiles = div_up(cap_bytes, kMapTileBytesMin);
  } else if (!streaming && cfg.map_path == MapPath::kFast && cfg.sort_path == SortPath::kDict) {
    // large single passes (the two-kernel ordered build): 1 KiB tiles below
    // kMapLargeInput, 4 KiB tiles (whole inputs or upload pieces) above
    sh.part_off_tiles =
        std::max<u64>(div_up(std::min<u64>(cap_bytes, kMapLargeInput), kMapTileBytesMin),
                      div_up(cap_bytes, kMapTileBytesLarge) + kMaxPieces);
    sh.large_ordered = cap > kPartBuildMaxTokens;
  }
  if (sh.part_off_tiles) sz.add<u32>(sh.part_off_tiles * kPartTable);
  if (sh.part_off_tiles) sz.add<u32>(sh.part_off_tiles * kPartOccWords);
  sh.partial_slots_cap = sh.large_ordered
                             ? (u32)std::clamp<u64>(div_up(cap_bytes, kPieceBytes) + 3,
                                                    kOrdWorkers, kMaxPartialSlots)
                             : 0u;
  const u64 partial_slots = (u64)kDictParts * sh.partial_slots_cap;
  if (partial_slots) {
    sz.add<KeyCount>(partial_slots * kPartSlotsHost);
    sz.add<u32>(partial_slots);
  }
  sz.add<OutRecord>(rcap);
  sz.add<KeyCount>(std::max<u64>(cap, kSlotRecordsMin) + kSlotHeaderRecords);  // d_records
  sz.add<PackedKey>(kMaxSamples);
  sz.add<PackedKey>(kMaxRanks);
  sz.add<u64>(kMaxRanks + 1);
  sz.add<u64>(1);
  sz.add<char>(sh.sync_bytes);
  sz.add<u32>(sh.rx_zero_words);
  sz.add<u32>(sh.rx_part_words);
  sz.add<SortPlan>(1);
  for (int b = 0; b < 2; ++b) {
    sz.add<u64>(rcap);
    sz.add<u32>(rcap);
  }
  for (int j = 0; j < kKeyWords; ++j) sz.add<u64>(ucap);
  sz.add<char>(sh.dict_zero_bytes);
  sh.arena_bytes = align_up(sz.bytes + 4096, kDevPageBytes);
  return sh;
}

// The every-token sort / reduce buffers a dictionary engine leaves out of its arena
// (rcap == ucap): sorted and head keys, sorted counts, prefix, head val / count, the
// permutation, the output records and the radix scratch, at cap.
static u64 radix_full_bytes(u64 cap) {
  SizingPlan sz;
  for (int j = 0; j < kKeyWords; ++j) {
    sz.add<u64>(cap);
    sz.add<u64>(cap);
  }
  for (int k = 0; k < 4; ++k) sz.add<u64>(cap);
  sz.add<u32>(cap);
  sz.add<OutRecord>(cap);
  sz.add<u32>(radix_zero_bytes(cap) / 4);
  sz.add<u32>((u64)radix_hist_blocks(cap) * kNumPositions * 256);
  for (int b = 0; b < 2; ++b) {
    sz.add<u64>(cap);
    sz.add<u32>(cap);
  }
  return align_up(sz.bytes + 4096, DevicePipeline::kDevPageBytes);
}

void DevicePipeline::ensure_radix_full() {
  if (rcap >= cap) return;
  hipStreamCaptureStatus cst = hipStreamCaptureStatusNone;
  LOCUST_HIP_CHECK(hipStreamIsCapturing(stream, &cst));
  LOCUST_CHECK_ARG(cst == hipStreamCaptureStatusNone,
                   "internal: the every-token sort buffers must exist before a capture");
  const u64 bytes = radix_full_bytes(cap);
  LOCUST_LOG_INFO("dictionary engine enters the every-token sort: +%.1f MiB of device memory",
                  bytes / 1048576.0);
  sync();  // nothing in flight may still use the buffers being replaced
  for (auto& g : dict_graphs) LOCUST_HIP_CHECK(hipGraphExecDestroy(g.exec));
  dict_graphs.clear();
  for (auto& g : graph_cache) LOCUST_HIP_CHECK(hipGraphExecDestroy(g.exec));
  graph_cache.clear();
  size_t got = 0;
  radix_base = static_cast<char*>(dev_block_alloc(bytes, &got));
  radix_block = got;
  Arena a;
  a.base = radix_base;
  a.size = bytes;
  for (int j = 0; j < kKeyWords; ++j) {
    sorted.w[j] = a.take<u64>(cap);
    heads.w[j] = a.take<u64>(cap);
  }
  d_sorted_counts = a.take<u64>(cap);
  d_prefix = a.take<u64>(cap);
  d_head_val = a.take<u64>(cap);
  d_head_count = a.take<u64>(cap);
  d_perm = a.take<u32>(cap);
  d_out = a.take<OutRecord>(cap);
  const u64 zw = radix_zero_bytes(cap) / 4;
  rx.cap = cap;
  rx.tile_counters = a.take<u32>(zw);
  rx.status = rx.tile_counters + kNumPositions;
  rx.hist_part = a.take<u32>((u64)radix_hist_blocks(cap) * kNumPositions * 256);
  for (int b = 0; b < 2; ++b) {
    rx.keys[b] = a.take<u64>(cap);
    rx.vals[b] = a.take<u32>(cap);
  }
  LOCUST_HIP_CHECK(hipMemsetAsync(rx.tile_counters, 0, zw * 4, stream));
  rcap = cap;
  ++layout_gen;
}

u64 DevicePipeline::device_bytes() const {
  u64 b = arena.size + (radix_base ? radix_full_bytes(cap) : 0);
  if (d_text_alt) b += cap_bytes + 64;
  if (d_plan) b += plan_zero_bytes;  // (+ the plan's key arrays: small)
  return b;
}

DevicePipeline::DevicePipeline(const JobConfig& c, u64 max_bytes, u64 max_lines, u64 cap_records)
    : cfg(c) {
  LOCUST_CHECK_ARG(cfg.emits_per_line > 0, "emits_per_line must be > 0");
  LOCUST_CHECK_ARG(cfg.max_key_len > 0 && cfg.max_key_len <= kKeyBytes - 1,
                   "max_key_len must be in [1, 31]");
  // construction phases, logged at LOCUST_LOG=debug (the cold CLI breakdown's engine_ms)
  u64 tc[6] = {now_ns(), 0, 0, 0, 0, 0};
  LOCUST_HIP_CHECK(hipSetDevice(cfg.device));
  {  // the device pass, planned against the HBM this engine may use (engine.hpp)
    size_t fr = 0, tot = 0;
    LOCUST_HIP_CHECK(hipMemGetInfo(&fr, &tot));
    hbm_free = fr;
    hbm_total = tot;
    const DevicePassPlan plan = plan_device_pass(cfg, max_bytes, max_lines, cap_records, fr);
    cap_bytes = plan.chunk_bytes;
    cap_lines = plan.cap_lines;
    cap = plan.cap;
    ucap = plan.ucap;
    rcap = plan.rcap;
    map_window = plan.map_window;
    pass_bytes = plan.pass_bytes;
    streaming = plan.streaming;
    if (plan.streaming && !(cfg.chunk_bytes && max_bytes > cfg.chunk_bytes))
      LOCUST_LOG_INFO("device pass: %llu B input planned as a stream of %llu B chunks (%s)",
                      (unsigned long long)max_bytes, (unsigned long long)cap_bytes,
                      plan.why.c_str());
  }
  warm_modules_once(cfg.device);
  tc[1] = now_ns();
  LOCUST_HIP_CHECK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
  for (auto& e : ev) LOCUST_HIP_CHECK(hipEventCreate(&e));
  tc[2] = now_ns();

  const bool compat = cfg.map_path == MapPath::kCompat;
  const u64 hcap = rcap < cap ? 1 : rcap;  // (shape_arena)
  DevicePassPlan plan;
  plan.streaming = streaming;
  plan.chunk_bytes = cap_bytes;
  plan.pass_bytes = pass_bytes;
  plan.map_window = map_window;
  plan.cap_lines = cap_lines;
  plan.cap = cap;
  plan.ucap = ucap;
  plan.rcap = rcap;
  const ArenaShape sh = shape_arena(cfg, plan, small_pass_bytes);
  const u64 slot_cap = sh.slot_cap;
  const u64 t_line = sh.t_line, t_compact = sh.t_compact, t_map = sh.t_map;
  const u64 t_heads = sh.t_heads, t_scan = sh.t_scan;
  const u64 rx_zero_words = sh.rx_zero_words, rx_part_words = sh.rx_part_words;
  dict_slots = sh.dict_slots;
  dict_zero_bytes = sh.dict_zero_bytes;
  sync_bytes = sh.sync_bytes;
  small_pass = sh.small_pass;
  part_off_tiles = sh.part_off_tiles;
  large_ordered = sh.large_ordered;
  partial_slots_cap = sh.partial_slots_cap;
  const u64 partial_slots = (u64)kDictParts * partial_slots_cap;
  arena.size = sh.arena_bytes;
  {
    size_t got = 0;  // the process-wide block cache (locust/devcache.hpp)
    arena.base = static_cast<char*>(dev_block_alloc(arena.size, &got));
    arena_block = got;
  }

  d_text = arena.take<char>(cap_bytes + 64);
  d_nl = arena.take<u64>(compat ? cap_lines + 1 : 1);
  d_delims = arena.take<char>(64);
  for (int j = 0; j < kKeyWords; ++j) {
    slots.w[j] = arena.take<u64>(slot_cap);
    tokens.w[j] = arena.take<u64>(cap);
    sorted.w[j] = arena.take<u64>(rcap);
    heads.w[j] = arena.take<u64>(hcap);
  }
  d_line_counts = arena.take<u32>(compat ? cap_lines : 1);
  d_counts = arena.take<u64>(cap);
  d_sorted_counts = arena.take<u64>(rcap);
  d_prefix = arena.take<u64>(hcap);
  d_head_val = arena.take<u64>(hcap);
  d_head_count = arena.take<u64>(hcap);
  d_perm = arena.take<u32>(rcap);
  d_parts = arena.take<u8>(align_up(cap, 16) + 16);
  if (part_off_tiles) d_part_off = arena.take<u32>(part_off_tiles * kPartTable);
  if (part_off_tiles) d_part_occ = arena.take<u32>(part_off_tiles * kPartOccWords);
  if (partial_slots) {
    d_partials = arena.take<KeyCount>(partial_slots * kPartSlotsHost);
    d_partial_n = arena.take<u32>(partial_slots);
  }
  d_out = arena.take<OutRecord>(rcap);
  // room for a gather slot header in front: d_records - kSlotHeaderRecords is the slot
  d_records = arena.take<KeyCount>(slot_records_cap() + kSlotHeaderRecords) + kSlotHeaderRecords;
  d_samples = arena.take<PackedKey>(kMaxSamples);
  d_splitters = arena.take<PackedKey>(kMaxRanks);
  d_offsets = arena.take<u64>(kMaxRanks + 1);
  d_offset = arena.take<u64>(1);

  // sync block: [MapCounters | tile counters | status regions]
  d_sync = arena.take<char>(sync_bytes);
  d_ctr = reinterpret_cast<MapCounters*>(d_sync);
  u32* counters = reinterpret_cast<u32*>(d_sync + 128);
  u64* st = reinterpret_cast<u64*>(d_sync + 256);
  lb_line = {st, counters + 0};
  st += t_line;
  lb_compact = {st, counters + 1};
  st += t_compact;
  lb_map = {st, counters + 2};
  st += t_map;
  lb_heads = {st, counters + 3};
  st += t_heads;
  lb_scan = {st, counters + 4};
  st += t_scan;
  lb_dict = {st, counters + 5};
  // counters[6] is the ordered kernels' done counter (lb_dict.tile_counter + 1);
  d_plan_flag = counters + 7;  // OrderedExtra::plan_flag

  rx.cap = rcap;
  rx.tile_counters = arena.take<u32>(rx_zero_words);
  rx.status = rx.tile_counters + kNumPositions;
  rx.hist_part = arena.take<u32>(rx_part_words);
  rx.plan = arena.take<SortPlan>(1);
  for (int b = 0; b < 2; ++b) {
    rx.keys[b] = arena.take<u64>(rcap);
    rx.vals[b] = arena.take<u32>(rcap);
  }
  for (int j = 0; j < kKeyWords; ++j) dict.ukeys.w[j] = arena.take<u64>(ucap);
  {
    char* z = arena.take<char>(dict_zero_bytes);
    dict.table = reinterpret_cast<DictSlot*>(z);
    dict.ucount = reinterpret_cast<u64*>(z + align_up(dict_slots * sizeof(DictSlot), 256));
    dict.uval = reinterpret_cast<u64*>(reinterpret_cast<char*>(dict.ucount) + align_up(ucap * 8, 256));
    d_rank = reinterpret_cast<u32*>(reinterpret_cast<char*>(dict.uval) + align_up(ucap * 8, 256));
    dict.mask = (u32)(dict_slots - 1);
    dict.ucap = (u32)ucap;
    dict.urank = d_rank;
  }

  char delim_buf[64] = {0};
  LOCUST_CHECK_ARG(cfg.delimiters.size() < sizeof(delim_buf), "too many delimiters");
  std::memcpy(delim_buf, cfg.delimiters.data(), cfg.delimiters.size());
  // on this pipeline's own stream: a legacy-stream copy would conflict with another
  // thread's graph capture (loopback ranks share the process)
  LOCUST_HIP_CHECK(
      hipMemcpyAsync(d_delims, delim_buf, sizeof(delim_buf), hipMemcpyHostToDevice, stream));
  // the counters and look-back words start zeroed, as a self-cleaning job leaves them: the
  // first job skips its reset memset (a fill kernel, and ~13 us of a first enqueue)
  LOCUST_HIP_CHECK(hipMemsetAsync(d_sync, 0, sync_bytes, stream));
  LOCUST_HIP_CHECK(hipStreamSynchronize(stream));
  sync_clean = true;

  tc[3] = now_ns();
  // A streaming engine reads files through its two staging halves; its one-pass buffer
  // is pinned only when a caller stages text there (input_buffer(), a one-pass job).
  if (!streaming && !cfg.records_only) ensure_h_text();
  LOCUST_HIP_CHECK(hipHostMalloc(&h_ctr, sizeof(MapCounters), hipHostMallocDefault));
  LOCUST_HIP_CHECK(hipHostMalloc(&h_plan, sizeof(SortPlan), hipHostMallocDefault));
  // Output records and the counter snapshot are host-mapped: the emit kernel writes them
  // over PCIe directly (zero-copy), so a dictionary run needs no D2H copy at all.  The
  // kernels that write it directly emit at most kMappedOutMax records (larger results
  // take the radix path, whose download grows the buffer), so a streaming engine with a
  // 16M-key dictionary does not pin 800 MB per output buffer.
  out_pool.push_back(std::make_shared<HostOut>(std::min<u64>(ucap, kMappedOutMax)));
  use_out(0);
  // and a second one: a job's result holds its buffer while the next job runs, so jobs
  // alternate between two -- allocated here, not inside the second job (pinning a
  // 12 MiB mapped buffer took ~1 ms of a cold CLI-style job).  A streaming engine's jobs
  // take hundreds of ms: its second buffer is pinned when a second job needs it (host
  // memory of `--gpus N` file ranks, one streaming engine each).
  if (!streaming && !cfg.records_only) out_pool.push_back(std::make_shared<HostOut>(h_out_cap));
  // and a third for small engines: the partition map's retune reads the first job's
  // output on the worker thread, so a caller holding each job's result (the CLI, a
  // Python loop) found both buffers taken at its third job and waited ~0.2 ms for the
  // worker (measured); pinning it here costs well under a millisecond of construction
  if (!streaming && !cfg.records_only && h_out_cap * sizeof(OutRecord) <= (8ull << 20))
    out_pool.push_back(std::make_shared<HostOut>(h_out_cap));
  use_out(0);
  LOCUST_HIP_CHECK(hipHostMalloc(&h_ctr_mapped, sizeof(MapCounters),
                                 hipHostMallocMapped | hipHostMallocCoherent));
  LOCUST_HIP_CHECK(hipHostMalloc(&h_done, 64, hipHostMallocMapped | hipHostMallocCoherent));
  *h_done = 0;
  LOCUST_HIP_CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&d_done), h_done, 0));
  LOCUST_HIP_CHECK(
      hipHostGetDevicePointer(reinterpret_cast<void**>(&d_ctr_mapped), h_ctr_mapped, 0));
  LOCUST_HIP_CHECK(hipMalloc(&d_pmap, sizeof(PartMapTables)));
  LOCUST_HIP_CHECK(hipHostMalloc(&h_pmap, sizeof(PartMapTables), hipHostMallocDefault));
  part_map_default(h_pmap);
  LOCUST_HIP_CHECK(hipMemcpyAsync(d_pmap, h_pmap, sizeof(PartMapTables), hipMemcpyHostToDevice,
                                  stream));
  LOCUST_HIP_CHECK(hipHostMalloc(&h_pw, kDictParts * sizeof(u32),
                                 hipHostMallocMapped | hipHostMallocCoherent));
  std::memset(h_pw, 0, kDictParts * sizeof(u32));
  LOCUST_HIP_CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&d_pw), h_pw, 0));
  LOCUST_HIP_CHECK(hipStreamSynchronize(stream));
  LOCUST_HIP_CHECK(hipHostMalloc(&h_small, kMaxSamples * sizeof(PackedKey), hipHostMallocDefault));
  LOCUST_HIP_CHECK(hipHostMalloc(&h_u64, (kMaxRanks + 8) * sizeof(u64), hipHostMallocDefault));
  std::memset(h_ctr, 0, sizeof(MapCounters));
  tc[4] = now_ns();
  if (large_ordered && cfg.map_path == MapPath::kFast && !cfg.records_only) {
    // what a piecewise pass needs, made here and not inside the first job: the copy
    // streams and piece events, and the plan's scratch
    ensure_piece_events(partial_slots_cap);
    if (devplan_env) ensure_plan();
    warm_copy_streams();
  }
  // the retune worker of a small engine is made here, not inside its first job (a
  // streaming engine's jobs take hundreds of ms: it makes it when first needed)
  if (!streaming) {
    retune_worker.start();
    // a first kernel launch on this engine's stream (its hardware queue's first dispatch,
    // kernel-argument space): here, not inside the first job -- a fresh engine's first job
    // spent ~35 us more than later ones enqueuing its launches (measured, bench cold_start)
    launch_signal_host(d_done, 0, stream);
    LOCUST_HIP_CHECK(hipStreamSynchronize(stream));
  }
  tc[5] = now_ns();
  LOCUST_LOG_DEBUG("engine (%llu B text, %llu tokens, %llu records%s): modules %.2f ms, stream "
                   "%.2f ms, device arena %.2f ms (%.1f MiB of %.1f GiB free), pinned host "
                   "buffers %.2f ms, copy streams %.2f ms",
                   (unsigned long long)cap_bytes, (unsigned long long)cap,
                   (unsigned long long)rcap, streaming ? ", streaming" : "",
                   (tc[1] - tc[0]) * 1e-6, (tc[2] - tc[1]) * 1e-6, (tc[3] - tc[2]) * 1e-6,
                   arena.size / 1048576.0, hbm_free / 1073741824.0, (tc[4] - tc[3]) * 1e-6,
                   (tc[5] - tc[4]) * 1e-6);
}

void DevicePipeline::warm_copy_streams() {
  if (!h_text || !cstream || !cstream2) return;
  const u64 n = std::min<u64>(cap_bytes, kPieceBytes);
  for (hipStream_t s : {cstream, cstream2, stream}) {
    LOCUST_HIP_CHECK(hipMemcpyAsync(d_text, h_text, n, hipMemcpyHostToDevice, s));
    LOCUST_HIP_CHECK(hipMemsetAsync(d_text + 1, 0, 16, s));
    LOCUST_HIP_CHECK(hipMemcpyAsync(h_u64, d_text, 8, hipMemcpyDeviceToHost, s));
    LOCUST_HIP_CHECK(hipStreamSynchronize(s));
  }
}

DevicePipeline::~DevicePipeline() {
  retune_worker.stop();  // its task may hold an output buffer
  if (stream) (void)hipStreamSynchronize(stream);
  for (auto& g : dict_graphs) (void)hipGraphExecDestroy(g.exec);
  for (auto& g : graph_cache) (void)hipGraphExecDestroy(g.exec);
  if (d_ord_trace) (void)hipFree(d_ord_trace);
  if (d_partials_trace) (void)hipFree(d_partials_trace);
  if (d_map_trace) (void)hipFree(d_map_trace);
  if (cstream) (void)hipStreamSynchronize(cstream);
  if (cstream2) (void)hipStreamSynchronize(cstream2);

  for (auto& e : ev)
    if (e) (void)hipEventDestroy(e);
  for (int b = 0; b < 2; ++b) {
    if (ev_copied[b]) (void)hipEventDestroy(ev_copied[b]);
    if (ev_consumed[b]) (void)hipEventDestroy(ev_consumed[b]);
    pinned_free(h_stage[b]);
  }
  for (int i = 0; i < kRingPieces; ++i) {
    pinned_free(h_ring[i]);
    if (ev_ring[i]) (void)hipEventDestroy(ev_ring[i]);
  }
  for (auto e : ev_piece) (void)hipEventDestroy(e);
  if (ev_fork) (void)hipEventDestroy(ev_fork);
  if (cstream) (void)hipStreamDestroy(cstream);
  if (cstream2) (void)hipStreamDestroy(cstream2);

  if (d_text_alt) dev_block_free(d_text_alt, d_text_alt_block);
  if (radix_base) dev_block_free(radix_base, radix_block);
  if (d_dctr) (void)hipFree(d_dctr);
  if (h_chunk_ctr) (void)hipHostFree(h_chunk_ctr);
  if (stream) (void)hipStreamDestroy(stream);
  if (arena.base) dev_block_free(arena.base, arena_block);  // every stream synchronised above
  pinned_free(h_text);
  pinned_free(h_keys);
  for (void* p : {(void*)h_ctr, (void*)h_plan, (void*)h_small, (void*)h_u64,
                  (void*)h_ctr_mapped, (void*)h_pmap, (void*)h_pw, (void*)h_done})
    if (p) (void)hipHostFree(p);
  if (d_pmap) (void)hipFree(d_pmap);
  if (d_plan) (void)hipFree(d_plan);
}

void DevicePipeline::use_out(size_t i) {
  out_idx = i;
  h_out = out_pool[i]->h;
  d_out_mapped = out_pool[i]->d;
  h_out_cap = out_pool[i]->cap;
  h_ctab = out_pool[i]->ctab_h;
  d_ctab_mapped = out_pool[i]->ctab_d;
}

void DevicePipeline::select_out() {
  if (!out_pool.empty() && out_pool[out_idx].use_count() == 1) return;
  for (size_t i = 0; i < out_pool.size(); ++i)
    if (out_pool[i].use_count() == 1) return use_out(i);
  if (retune_pending) {
    // a background retune reads a buffer a result no longer needs: wait until it has let
    // go of it (one pass over the output) rather than pin a new buffer (~2 ms for a large
    // engine's)
    while (!retune_task.released.load(std::memory_order_acquire)) std::this_thread::yield();
    poll_retune();
    for (size_t i = 0; i < out_pool.size(); ++i)
      if (out_pool[i].use_count() == 1) return use_out(i);
  }
  const u64 t0 = now_ns();
  out_pool.push_back(std::make_shared<HostOut>(h_out_cap));
  use_out(out_pool.size() - 1);
  LOCUST_LOG_DEBUG("output buffer #%zu: %llu records, %.2f ms", out_pool.size(),
                   (unsigned long long)h_out_cap, (now_ns() - t0) * 1e-6);
}

void DevicePipeline::grow_host_out(u64 n) {
  select_out();
  if (n <= h_out_cap) return;
  sync();  // the device may still write the buffer being replaced
  out_pool[out_idx] = std::make_shared<HostOut>(n);
  use_out(out_idx);
}

void DevicePipeline::grow_host_keys(u64 n) {
  if (n <= h_keys_cap) return;
  pinned_free(h_keys);
  h_keys_cap = std::max<u64>(n, 1);
  h_keys = static_cast<u64*>(pinned_alloc(h_keys_cap * kKeyWords * sizeof(u64), hipHostMallocDefault,
                                          "key staging"));
}

void DevicePipeline::wait_done(u32 seq, bool bounded_sync) {
  const u64 t0 = now_ns();
  while (__atomic_load_n(h_done, __ATOMIC_ACQUIRE) != seq) {
    if (now_ns() - t0 > 2000000) {  // 2 ms
      if (bounded_sync) sync();
      break;
    }
    __builtin_ia32_pause();
  }
  std::atomic_thread_fence(std::memory_order_acquire);
}

void DevicePipeline::enqueue_upload(const TextInput& in) {
  const u64 t0 = now_ns();
  prepare_upload(in);
  const u64 t1 = now_ns();
  enqueue_upload_device(in);
  if ((int)log_level() >= (int)LogLevel::kDebug)
    LOCUST_LOG_DEBUG("upload: mode %d, %zu pieces, host %.3f ms, enqueue %.3f ms",
                     (int)upload_mode, pieces.size(), (t1 - t0) * 1e-6, (now_ns() - t1) * 1e-6);
}

void DevicePipeline::prepare_upload(const TextInput& in) {
  ensure_h_text();
  map_text = d_text;
  pieces.clear();
  if (use_zero_copy(in)) {
    upload_mode = Upload::kZeroCopy;
    map_text = d_h_text;
  } else if (in.data != h_text && in.bytes && host_pinned(in.data)) {
    upload_mode = Upload::kDirect;
    plan_pieces(in);
    return;
  } else {
    upload_mode = Upload::kStaged;
  }
  if (in.data != h_text && in.bytes) std::memcpy(h_text, in.data, in.bytes);
  std::memset(h_text + in.bytes, 0, 16);
  plan_pieces(in);
}

void DevicePipeline::plan_pieces(const TextInput& in) {
  if (cfg.map_path != MapPath::kFast || !large_ordered || in.bytes < 2 * kPieceBytes) return;
  const u64 npieces = std::min<u64>(partial_slots_cap, kMaxPieces);
  const u64 piece = std::max<u64>({kPieceBytes, std::min<u64>(piece_target(), in.bytes / 4),
                                   div_up(in.bytes, npieces > 3 ? npieces - 3 : 1)});
  u64 pos = 0;
  while (pos < in.bytes && pieces.size() < npieces) {
    // Short first pieces start the map early, a short last piece keeps the work after
    // the final copy small: P/4, P/2, P, ..., P, (rest - P/4), P/4 (a P/8 tail measured
    // no better).  The last piece allowed takes the rest (line alignment shortens the
    // others).
    const u64 rest = in.bytes - pos, tail = piece / 4;
    u64 want = piece;
    if (pieces.size() == 0) want = piece / 4;
    else if (pieces.size() == 1) want = piece / 2;
    else if (rest <= tail + tail / 2) want = rest;
    else if (rest <= piece + tail) want = rest - tail;
    want = std::min(want, rest);
    u64 end = pieces.size() + 1 == npieces ? in.bytes : pos + want;
    if (end < in.bytes) {
      const void* nl = memrchr(in.data + pos, '\n', (size_t)(end - pos));
      if (!nl) {  // a line longer than a piece: no pieces at all
        pieces.clear();
        return;
      }
      end = (u64)(static_cast<const char*>(nl) - in.data) + 1;
    }
    pieces.emplace_back(pos, end - pos);
    pos = end;
  }
  if (pos < in.bytes) pieces.clear();
}

void DevicePipeline::ensure_piece_events(size_t n) {
  if (!cstream) LOCUST_HIP_CHECK(hipStreamCreateWithFlags(&cstream, hipStreamNonBlocking));
  if (!cstream2) LOCUST_HIP_CHECK(hipStreamCreateWithFlags(&cstream2, hipStreamNonBlocking));
  if (!ev_fork) LOCUST_HIP_CHECK(hipEventCreateWithFlags(&ev_fork, hipEventDisableTiming));
  while (ev_piece.size() < n) {
    hipEvent_t e;
    LOCUST_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    ev_piece.push_back(e);
  }
}

void DevicePipeline::enqueue_upload_device(const TextInput& in) {
  if (!pieces.empty()) {
    // the pieces' copies go out first (outside a graph capture: there they need the fork
    // from `stream`, made in enqueue_map); their maps follow in enqueue_map
    hipStreamCaptureStatus cst = hipStreamCaptureStatusNone;
    LOCUST_HIP_CHECK(hipStreamIsCapturing(stream, &cst));
    if (cst == hipStreamCaptureStatusNone)
      issue_piece_copies(upload_mode == Upload::kDirect ? in.data : h_text);
  } else if (upload_mode == Upload::kDirect) {
    LOCUST_HIP_CHECK(hipMemcpyAsync(d_text, in.data, in.bytes, hipMemcpyHostToDevice, stream));
    LOCUST_HIP_CHECK(hipMemsetAsync(d_text + in.bytes, 0, 16, stream));
  } else if (upload_mode == Upload::kStaged) {
    LOCUST_HIP_CHECK(hipMemcpyAsync(d_text, h_text, in.bytes + 16, hipMemcpyHostToDevice, stream));
  }
  if (!skip_sync_reset) LOCUST_HIP_CHECK(hipMemsetAsync(d_sync, 0, sync_bytes, stream));
}

bool DevicePipeline::use_job_graph(const TextInput& in) const {
  if (cfg.map_path == MapPath::kFast && large_ordered && in.bytes >= 2 * kPieceBytes) return false;
  if (cfg.graph < 0 && lean_job(in)) return false;  // auto: lean direct launches instead
  const bool radix_ok = cfg.sort_path == SortPath::kRadix && cfg.map_path == MapPath::kFast &&
                        table_tiles(in.bytes) > 0 && radix_mapped() && psort_enabled();
  if (cfg.graph >= 0) return cfg.graph > 0 && (cfg.sort_path == SortPath::kDict || radix_ok);
  return (cfg.sort_path == SortPath::kDict && cfg.map_path == MapPath::kFast) || radix_ok;
}

bool DevicePipeline::lean_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("LOCUST_LEAN");
    return !e || e[0] != '0';
  }();
  return on;
}

void DevicePipeline::launch_dict_graph(const TextInput& in, bool compat) {
  u64 sig = 0;
  for (const auto& pc : pieces) sig = (sig ^ pc.first) * 0x100000001b3ull;
  if (!pieces.empty()) sig |= 1;
  const GraphKey key{in.bytes, in.num_lines, upload_mode == Upload::kDirect ? in.data : nullptr,
                     map_text, upload_mode, d_out_mapped, skip_sync_reset, sig};
  const DictGraph* hit = nullptr;
  for (const auto& g : dict_graphs)
    if (g.key == key) hit = &g;
  if (!hit) {
    if (dict_graphs.size() >= 6) {  // shapes or buffers changed a lot: drop the oldest
      LOCUST_HIP_CHECK(hipGraphExecDestroy(dict_graphs.front().exec));
      dict_graphs.erase(dict_graphs.begin());
    }
    hipGraph_t g = nullptr;
    LOCUST_HIP_CHECK(hipStreamBeginCapture(stream, hipStreamCaptureModeRelaxed));
    enqueue_upload_device(in);
    enqueue_map(in);
    bool ordered;  // dictionary: the ordered kernel; radix: the partitioned sort
    if (cfg.sort_path == SortPath::kDict) {
      ordered = enqueue_dict_job((u32)in.num_lines, compat, false, nullptr, /*self_clean=*/true);
    } else {
      enqueue_radix_job((u32)in.num_lines, compat, nullptr, nullptr);
      ordered = psort_used;
      job_self_cleaned = false;
    }
    LOCUST_HIP_CHECK(hipStreamEndCapture(stream, &g));
    hipGraphExec_t exec = nullptr;
    LOCUST_HIP_CHECK(hipGraphInstantiate(&exec, g, nullptr, nullptr, 0));
    LOCUST_HIP_CHECK(hipGraphDestroy(g));
    dict_graphs.push_back({key, exec, ordered, job_self_cleaned, ordered && ord_compact});
    hit = &dict_graphs.back();
  }
  graph_ordered = hit->ordered;
  job_self_cleaned = hit->clean;
  ord_compact = hit->compact;
  if (cfg.sort_path == SortPath::kRadix) psort_used = hit->ordered;
  parts_ready = cfg.map_path == MapPath::kFast;  // what enqueue_map sets when not replaying
  part_tiles = cfg.map_path != MapPath::kFast ? 0u : pieces.empty() ? table_tiles(in.bytes)
                                                                       : piece_tiles();
  LOCUST_HIP_CHECK(hipGraphLaunch(hit->exec, stream));
}

void DevicePipeline::enqueue_map(const TextInput& in) {
  plan_pass = false;  // decided per pass (decide_plan) where the map can write occupancy
  parts_ready = cfg.map_path == MapPath::kFast;
  devplan_used = false;
  partial_nslots = 0;
  // combining needs the 4 KiB grouped map: upload pieces, or one launch past kMapLargeInput
  map_combined = combine_map && large_ordered && cfg.map_path == MapPath::kFast &&
                 (!pieces.empty() ? piece_tiles() > 0
                                  : in.bytes >= kMapLargeInput && table_tiles(in.bytes) > 0);
  if (cfg.map_path == MapPath::kCompat) {
    launch_line_index(d_text, in.bytes, d_nl, d_ctr, lb_line, stream);
    launch_map_compat(d_text, in.bytes, d_nl, (u32)in.num_lines, d_delims, cfg.emits_per_line,
                      cfg.max_key_len, slots, d_line_counts, d_ctr, stream);
  } else if (!pieces.empty()) {
    // piece k: H2D on the copy stream, then its map on the compute stream once it landed
    // (4 KiB tiles; the table rows of the pieces follow each other)
    ensure_piece_events(pieces.size());
    part_tiles = piece_tiles();
    const char* src = upload_mode == Upload::kDirect ? in.data : h_text;
    const DelimMask dm = make_delim_mask(cfg.delimiters.c_str());
    // The copies need no fork from `stream` outside a graph capture (nothing earlier in
    // the job touches d_text, and the previous job ended with a host sync).  A fork made
    // the first copy on a copy stream wait on the host for the compute queue's marker:
    // one job in ~8 stalled 8-9 ms inside hipMemcpyAsync (measured; none without it).
    hipStreamCaptureStatus cst = hipStreamCaptureStatusNone;
    LOCUST_HIP_CHECK(hipStreamIsCapturing(stream, &cst));
    if (cst != hipStreamCaptureStatusNone) {
      LOCUST_HIP_CHECK(hipEventRecord(ev_fork, stream));
      LOCUST_HIP_CHECK(hipStreamWaitEvent(cstream, ev_fork, 0));
      LOCUST_HIP_CHECK(hipStreamWaitEvent(cstream2, ev_fork, 0));
    }
    // a combining large pass (run() / the shard engine take the two-kernel ordered build
    // next): aggregate each piece right after its map, into slot k -- on the same stream:
    // beside the next map on a third stream both kernels ran ~1.6x slower and every
    // cross-queue hand-off cost ~20 us (measured), while the copies leave room for both
    const bool agg = map_combined && large_ordered_ok() && pieces.size() <= partial_slots_cap;
    devplan_used = agg && devplan_env && !devplan_failed && !pm_tuned;
    if (devplan_used) {  // zeroed while piece 0 is on its way
      ensure_plan();
      LOCUST_HIP_CHECK(hipMemsetAsync(d_plan, 0, plan_zero_bytes, stream));
    }
    const u64 t_enq = now_ns();
    // the padding after the text: off the copy streams (a 16-byte fill at an unaligned
    // address is two blit kernels there, ~15 us in front of the last piece's event)
    LOCUST_HIP_CHECK(hipMemsetAsync(d_text + in.bytes, 0, 16, stream));
    u64 tile_off = 0;
    const bool issued = pieces_issued;
    pieces_issued = false;
    for (size_t k = 0; k < pieces.size(); ++k) {
      const u64 off = pieces[k].first, len = pieces[k].second;
      if (!issued) {
        hipStream_t cs = piece_stream(k);
        LOCUST_HIP_CHECK(hipMemcpyAsync(d_text + off, src + off, len, hipMemcpyHostToDevice, cs));
        LOCUST_HIP_CHECK(hipEventRecord(ev_piece[k], cs));
      }
      LOCUST_HIP_CHECK(hipStreamWaitEvent(stream, ev_piece[k], 0));
      if (k == 0 && devplan_used) enqueue_devplan(src, len, dm);
      launch_map_fast(d_text + off, len, dm, cfg.emits_per_line, cfg.max_key_len, tokens, d_parts,
                      cap, d_ctr, lb_map, stream, map_trace(),
                      part_tiles ? d_part_off + tile_off * kPartTable : nullptr, part_map(),
                      /*large_tiles=*/true, map_combined ? d_counts : nullptr);
      const u64 t1 = tile_off + div_up(len, kMapTileBytesLarge);
      if (agg)
        launch_dict_partials(tokens, d_counts, d_part_off, (u32)tile_off, (u32)t1, 1, (u32)k,
                             (u32)pieces.size(), cap, d_partials, d_partial_n, stream,
                             partials_trace());
      tile_off = t1;
    }
    if ((int)log_level() >= (int)LogLevel::kDebug)
      LOCUST_LOG_DEBUG("piecewise map enqueued in %.3f ms", (now_ns() - t_enq) * 1e-6);
    if (agg) partial_nslots = (u32)pieces.size();
  } else {
    part_tiles = table_tiles(in.bytes);
    // A large pass in one launch (below the piecewise size): the same in-job plan as the
    // piecewise pass, from the first MiB of the text, before the map tags the tokens --
    // a first-letter map overflows the ordered kernel's LDS tables on ~80K distinct keys
    // (measured: 1/8 of synth1m, 5.7 ms first job with the HBM-table fallback).
    devplan_used = large_ordered && part_tiles && cfg.sort_path == SortPath::kDict &&
                   devplan_env && !devplan_failed && !pm_tuned;
    if (devplan_used) {
      ensure_plan();
      LOCUST_HIP_CHECK(hipMemsetAsync(d_plan, 0, plan_zero_bytes, stream));
      enqueue_devplan(upload_mode == Upload::kDirect || upload_mode == Upload::kZeroCopy ? in.data
                                                                                       : h_text,
                      in.bytes, make_delim_mask(cfg.delimiters.c_str()), map_text);
    }
    decide_plan(in.bytes);
    launch_map_fast(map_text, in.bytes, make_delim_mask(cfg.delimiters.c_str()),
                    cfg.emits_per_line, cfg.max_key_len, tokens, d_parts, cap, d_ctr, lb_map,
                    stream, map_trace(), part_tiles ? d_part_off : nullptr, part_map(), false,
                    map_combined ? d_counts : nullptr, plan_small() ? d_part_occ : nullptr,
                    plan_small() && plan_trigger ? d_plan_flag : nullptr);
  }
}

void DevicePipeline::enqueue_process(u32 num_lines, bool compat, bool with_counts, u64 host_n,
                       bool allow_psort) {
  ensure_radix_full();  // every token is sorted: a dictionary engine grows its buffers
  if (allow_psort && psort_ok(compat, with_counts)) {
    // one kernel, one workgroup per key range of the map's partition table (psort.hip)
    launch_psort(tokens, d_part_off, part_tiles, cap, sorted, d_ctr, d_pw, stream, ord_trace());
    psort_used = true;
    return;
  }
  psort_used = false;
  if (compat)
    launch_compact_slots(d_line_counts, num_lines, cfg.emits_per_line, slots, tokens, d_ctr,
                         lb_compact, stream);
  if (!cfg.sync_plan) {
    host_n = kUnknownCount;
  } else if (host_n == kUnknownCount) {
    LOCUST_HIP_CHECK(hipMemcpyAsync(h_u64, &d_ctr->num_records, sizeof(u32),
                                    hipMemcpyDeviceToHost, stream));
    sync();
    host_n = *reinterpret_cast<const u32*>(h_u64);
  }
  radix_sort(tokens, &d_ctr->num_records, host_n, rx, with_counts ? d_counts : nullptr, sorted,
             with_counts ? d_sorted_counts : nullptr, d_perm, h_plan, stream);
}

void DevicePipeline::enqueue_radix_job(u32 num_lines, bool compat, hipEvent_t after_process,
                         hipEvent_t after_reduce) {
  ensure_radix_full();
  radix_fused = cfg.reduce_path == ReducePath::kLds &&
                radix_mapped() && psort_ok(compat, false);
  if (radix_fused) {
    // Process + Reduce in one kernel, records straight into the mapped output; it
    // re-zeroes its scratch and, in a lean job, tells the host itself (psort.hip)
    PsortReduceArgs ra;
    ra.out = d_out_mapped;
    ra.out_cap = h_out_cap;
    ra.ctr_out = d_ctr_mapped;
    ra.status = lb_dict.status;
    ra.done_counter = lb_dict.tile_counter + 1;  // the sync block's spare counter word
    ra.map_lb = lb_map;
    ra.map_words = (u32)(div_up(pass_bytes, kMapTileBytesMin) + 1);
    if (done_pending) {
      ra.host_done = d_done;
      ra.host_done_value = done_pending;
      done_pending = 0;
    }
    launch_psort_reduce(tokens, d_part_off, part_tiles, cap, d_ctr, d_pw, ra, stream, ord_trace());
    psort_used = true;
    if (after_process) LOCUST_HIP_CHECK(hipEventRecord(after_process, stream));
    if (after_reduce) LOCUST_HIP_CHECK(hipEventRecord(after_reduce, stream));
    return;
  }
  enqueue_process(num_lines, compat, false, kUnknownCount, /*allow_psort=*/true);
  if (after_process) LOCUST_HIP_CHECK(hipEventRecord(after_process, stream));
  const bool mapped = radix_mapped();
  if (cfg.reduce_path == ReducePath::kLds) {
    // LDS path: mark + compact + adjacent difference + records in one kernel
    launch_reduce_fused(sorted, cap, d_ctr, mapped ? d_out_mapped : d_out, mapped ? h_out_cap : cap,
                        mapped ? d_ctr_mapped : nullptr, lb_heads, stream);
  } else {
    // global path: the reference's kernel sequence (kernFindUniqBool, partition,
    // kernGetCount) as separate launches
    enqueue_reduce_core(false);
    if (mapped)
      launch_pack_output(heads, d_head_val, d_head_count, cap, d_ctr, d_out_mapped, stream,
                         d_ctr_mapped);
    else
      enqueue_pack_output();
  }
  if (after_reduce) LOCUST_HIP_CHECK(hipEventRecord(after_reduce, stream));
}

void DevicePipeline::redo_radix_general(u32 num_lines) {
  redo_process_general(num_lines);
  LOCUST_HIP_CHECK(hipMemsetAsync(lb_heads.status, 0, 8 * (div_up(cap, kReduceTile) + 1), stream));
  LOCUST_HIP_CHECK(hipMemsetAsync(lb_heads.tile_counter, 0, 4, stream));
  enqueue_reduce_core(false);
  enqueue_pack_output();
}

void DevicePipeline::enqueue_reduce_core(bool with_counts) {
  ensure_radix_full();
  const u64* prefix = nullptr;
  if (with_counts) {
    launch_scan_counts(d_sorted_counts, cap, d_prefix, d_ctr, lb_scan, stream);
    prefix = d_prefix;
  }
  launch_mark_compact_heads(sorted, prefix, cap, cfg.reduce_path, heads, d_head_val, d_ctr,
                            lb_heads, stream);
  launch_adjacent_diff(d_head_val, cap, cfg.reduce_path, d_head_count, d_ctr, stream);
}

void DevicePipeline::enqueue_dict_insert(u32 num_lines, bool compat, bool with_counts) {
  if (compat)
    launch_compact_slots(d_line_counts, num_lines, cfg.emits_per_line, slots, tokens, d_ctr,
                         lb_compact, stream);
  if (!compat && parts_ready && cap <= kPartBuildMaxTokens) {
    launch_dict_part_build(tokens, with_counts ? d_counts : nullptr, d_parts,
                           &d_ctr->num_records, cap, dict, d_ctr, stream);
    return;
  }
  LOCUST_HIP_CHECK(hipMemsetAsync(dict.table, 0, dict_zero_bytes, stream));
  launch_dict_insert(tokens, with_counts ? d_counts : nullptr, &d_ctr->num_records, cap, dict,
                     d_ctr, stream);
}

void DevicePipeline::enqueue_partials() {
  if (partial_nslots) return;
  partial_nslots = kOrdWorkers;
  launch_dict_partials(tokens, map_combined ? d_counts : nullptr, d_part_off, 0, part_tiles,
                       kOrdWorkers, 0, kOrdWorkers, cap, d_partials, d_partial_n, stream,
                       partials_trace());
}

void DevicePipeline::set_tile_source(OrderedExtra& ex, bool with_counts) const {
  if (part_tiles && parts_ready && !with_counts) {
    ex.part_off = d_part_off;
    ex.part_tiles = part_tiles;
    // the in-job plan while the map is untuned (a retuned map is already balanced: the
    // plan would only add its ~2 us)
    if (plan_small()) ex.part_occ = d_part_occ;
    // ... and only when the map saw a crowded partition (plan_trigger)
    if (plan_small() && plan_trigger) ex.plan_flag = d_plan_flag;
  }
}

u64 DevicePipeline::retune_wanted() const {
  if (devplan_used && !pm_tuned) {  // a planned pass: hand over to the exact map
    if (const char* v = std::getenv("LOCUST_PART_TUNE"))
      if (v[0] == '0') return 0;
    return ~0ull / 8;
  }
  if (const char* v = std::getenv("LOCUST_PART_TUNE"))
    if (v[0] == '0') return 0;
  u64 sum = 0, mx = 0;
  for (int p = 0; p < kDictParts; ++p) {
    sum += h_pw[p];
    mx = std::max<u64>(mx, h_pw[p]);
  }
  if (sum < (1u << 13) || mx * kDictParts <= 2 * sum) return 0;  // small or balanced
  if (pm_predicted_max && mx * 4 <= pm_predicted_max * 5) return 0;  // as good as it gets
  return mx;
}

void DevicePipeline::force_retune(const EntryList& e) {
  if (warming) return;
  const u64 n = e.size();
  // a device-planned map overflowed: this engine keeps the host-side map from now on
  // (tuned from this output, or the default with tuning off) -- d_pmap holds the plan
  const bool planned = devplan_used;
  if (planned) {
    devplan_failed = true;
    devplan_used = false;
  }
  const char* v = std::getenv("LOCUST_PART_TUNE");
  const bool tune = n && !(v && v[0] == '0');
  PartMapTables t;
  u64 pred = 0;
  if (tune)
    pred = part_map_from_entries(e, &t);
  else
    part_map_default(&t);
  // The same map again (e.g. one first word with more distinct keys than an LDS table:
  // no cut can split it): a new upload would change nothing, so keep it.
  if (!planned && (!tune || std::memcmp(&t, h_pmap, sizeof(t)) == 0)) return;
  if (planned && !pred) return upload_pmap(t, 0);
  retune_with(~0ull / 8, pred, t);
}

void DevicePipeline::warm_first_job() {
  // small single-pass engines only: there the two-byte job launches the real job's kernels
  // (a large pass plans, pieces and aggregates differently)
  if (streaming || large_ordered || cfg.records_only || cfg.sort_path != SortPath::kDict ||
      cfg.map_path != MapPath::kFast || cap_bytes < 2)
    return;
  TextInput in;
  in.data = ensure_h_text();
  in.bytes = 2;
  in.num_lines = 1;
  if (!lean_job(in)) return;
  // one token: a byte outside the job's delimiter set
  char c = 0;
  for (const char* q = "aZ7xq"; *q && !c; ++q)
    if (cfg.delimiters.find(*q) == std::string::npos) c = *q;
  if (!c) return;
  h_text[0] = c;
  h_text[1] = '\n';
  // the engine's statistics describe the caller's jobs only
  const u64 fb = fallbacks, pp = planned_passes;
  warming = true;
  struct Reset {
    bool& w;
    ~Reset() { w = false; }
  } reset{warming};
  const WordCountResult r = run(in);
  if (r.num_unique != 1)
    LOCUST_LOG_INFO("engine warm-up job: %llu keys, expected 1", (unsigned long long)r.num_unique);
  fallbacks = fb;
  planned_passes = pp;
}

void DevicePipeline::maybe_retune(const EntryList& e) {
  if (warming) return;
  const u64 mx = retune_wanted();
  if (!mx || retune_pending) return;  // one at a time
  retune_pending = true;
  retune_task.mx = mx;
  retune_task.pred = 0;
  // a borrowed list: the copy shares the buffer (and its segments), not the entries
  retune_task.hold = out_pool[out_idx];
  retune_task.entries = e;
  retune_task.released.store(false, std::memory_order_relaxed);
  retune_task.t_submit = now_ns();
  retune_worker.submit([this] {
    RetuneTask& r = retune_task;
    r.t_start = now_ns();
    // the one pass over the output first, then the buffer is free for the next jobs
    part_map_groups(r.entries, &r.groups);
    r.entries = EntryList();
    r.hold.reset();
    r.t_released = now_ns();
    r.released.store(true, std::memory_order_release);
    r.pred = part_map_from_groups(r.groups, &r.t);
    r.t_done = now_ns();
  });
}

void DevicePipeline::poll_retune() {
  if (!retune_pending || !retune_worker.idle()) return;
  retune_pending = false;
  retune_worker.rethrow_error();  // a failed retune surfaces here, on the job's thread
  const RetuneTask& r = retune_task;
  LOCUST_LOG_DEBUG("retune on the worker: started %.3f ms after the job, output read in %.3f "
                   "ms, map built in %.3f ms (%zu first-word groups)",
                   (r.t_start - r.t_submit) * 1e-6, (r.t_released - r.t_start) * 1e-6,
                   (r.t_done - r.t_released) * 1e-6, r.groups.size());
  retune_with(retune_task.mx, retune_task.pred, retune_task.t);
}

void DevicePipeline::maybe_retune_records(const KeyCount* d_recs, u64 n, bool force) {
  const bool planned = force && devplan_used;
  if (planned) {  // as force_retune
    devplan_failed = true;
    devplan_used = false;
  }
  const u64 mx = force ? ~0ull / 8 : retune_wanted();
  if (planned && (!n || [] {
        const char* v = std::getenv("LOCUST_PART_TUNE");
        return v && v[0] == '0';
      }())) {
    PartMapTables t;
    part_map_default(&t);
    return upload_pmap(t, 0);
  }
  if (!mx || !n) return;
  std::vector<KeyCount> h(n);
  LOCUST_HIP_CHECK(hipMemcpyAsync(h.data(), d_recs, n * sizeof(KeyCount), hipMemcpyDeviceToHost,
                                  stream));
  sync();
  std::vector<WordCountEntry> e(n);
  for (u64 i = 0; i < n; ++i) {
    for (int w = 0; w < kKeyWords; ++w) e[i].key.w[w] = h[i].w[w];
    e[i].count = h[i].count;
  }
  PartMapTables t;
  const u64 pred = part_map_from_entries(EntryList(std::move(e)), &t);
  if (force && !planned && std::memcmp(&t, h_pmap, sizeof(t)) == 0) return;  // as force_retune
  retune_with(mx, pred, t);
}

void DevicePipeline::retune_with(u64 mx, u64 pred, const PartMapTables& t) {
  if (!pred || pred * 5 >= mx * 4) {  // < 20 % better: keep the map, stop asking
    pm_predicted_max = mx;
    return;
  }
  upload_pmap(t, pred);
  ++pm_retunes;
  if (large_ordered) pm_tuned = true;
  LOCUST_LOG_DEBUG("partition map retuned (#%u): max partition work %llu -> %llu",
                   pm_retunes, (unsigned long long)mx, (unsigned long long)pred);
}

void DevicePipeline::enqueue_dict_ordered(bool with_counts, bool mapped, bool self_clean) {
  OrderedExtra ex;
  ex.pm = part_map();
  ex.part_w = d_pw;
  ex.split_min = split_min;
  if (self_clean) set_self_clean(ex);
  if (self_clean && done_pending) {  // the kernel itself tells the host it is done
    ex.host_done = d_done;
    ex.host_done_value = done_pending;
    done_pending = 0;
  }
  set_tile_source(ex, with_counts);
  set_compact_out(ex, mapped);
  launch_dict_ordered(tokens, with_counts ? d_counts : nullptr, d_parts, &d_ctr->num_records,
                      cap, d_ctr, mapped ? d_out_mapped : d_out, mapped ? d_ctr_mapped : nullptr,
                      lb_dict, stream, ord_trace(), ex);
}

u64* DevicePipeline::ord_trace() {
  static const bool on = std::getenv("LOCUST_ORD_TRACE") != nullptr;
  if (!on) return nullptr;
  if (!d_ord_trace) {
    LOCUST_HIP_CHECK(hipMalloc(&d_ord_trace, kDictParts * 32 * sizeof(u64)));
    LOCUST_HIP_CHECK(hipMemset(d_ord_trace, 0, kDictParts * 32 * sizeof(u64)));
  }
  return d_ord_trace;
}

u64* DevicePipeline::map_trace() {
  static const bool on = std::getenv("LOCUST_MAP_TRACE") != nullptr;
  if (!on) return nullptr;
  if (!d_map_trace) {
    LOCUST_HIP_CHECK(hipMalloc(&d_map_trace, 4096 * 8 * sizeof(u64)));
    LOCUST_HIP_CHECK(hipMemset(d_map_trace, 0, 4096 * 8 * sizeof(u64)));
  }
  return d_map_trace;
}

void DevicePipeline::print_map_trace() {
  if (!d_map_trace || warming) return;
  std::vector<u64> t(4096 * 8);
  LOCUST_HIP_CHECK(hipMemcpy(t.data(), d_map_trace, t.size() * 8, hipMemcpyDeviceToHost));
  u64 t0 = ~0ull;
  for (int i = 0; i < 4096; ++i)
    if (t[i * 8]) t0 = std::min(t0, t[i * 8]);
  for (int i = 0; i < 4096; ++i) {
    const u64* x = &t[i * 8];
    if (!x[0] || !x[5]) continue;
    // (small grouped tiles: 6 = wave 0's masks done, 7 = its keys packed and ranked, 3 =
    // the barrier after; large grouped tiles: 6 = records reserved)
    std::fprintf(stderr, "map tile=%4d entry=%6.2f acquired=%6.2f staged=%6.2f masks=%6.2f "
                 "prefix=%6.2f reserved=%6.2f done=%6.2f w0masks=%6.2f w0packed=%6.2f us\n", i,
                 (x[0] - t0) * 0.01, (x[1] - t0) * 0.01, (x[2] - t0) * 0.01, (x[3] - t0) * 0.01,
                 (x[4] - t0) * 0.01, x[6] ? (x[6] - t0) * 0.01 : 0.0, (x[5] - t0) * 0.01,
                 x[6] ? (x[6] - t0) * 0.01 : 0.0, x[7] ? (x[7] - t0) * 0.01 : 0.0);
  }
}

u64* DevicePipeline::partials_trace() {
  static const bool on = std::getenv("LOCUST_ORD_TRACE") != nullptr;
  if (!on) return nullptr;
  if (!d_partials_trace) {
    LOCUST_HIP_CHECK(hipMalloc(&d_partials_trace, (u64)kDictParts * kMaxPartialSlots * 8 * sizeof(u64)));
    LOCUST_HIP_CHECK(hipMemset(d_partials_trace, 0, (u64)kDictParts * kMaxPartialSlots * 8 * sizeof(u64)));
  }
  return d_partials_trace;
}

void DevicePipeline::print_partials_trace() {
  if (!d_partials_trace || warming) return;
  const u64 ns = std::max<u32>(partial_nslots, 1), nb = (u64)kDictParts * ns;
  std::vector<u64> t(nb * 8);  // slot b = p * ns + k
  LOCUST_HIP_CHECK(hipMemcpy(t.data(), d_partials_trace, t.size() * 8, hipMemcpyDeviceToHost));
  LOCUST_HIP_CHECK(hipMemset(d_partials_trace, 0, t.size() * 8));
  u64 t0 = ~0ull, t1 = 0, tok = 0;
  for (u64 b = 0; b < nb; ++b) {
    if (!t[b * 8]) continue;
    t0 = std::min(t0, t[b * 8]);
    t1 = std::max(t1, t[b * 8 + 3]);
    tok += t[b * 8 + 4];
  }
  std::fprintf(stderr, "partials span=%.2f us, tokens=%llu\n", (t1 - t0) * 0.01,
               (unsigned long long)tok);
  for (u64 b = 0; b < nb; ++b) {
    const u64* x = &t[b * 8];
    if (!x[0]) continue;
    std::fprintf(stderr, "partials b=%4llu p=%3llu k=%llu in=%7.2f clear=%6.2f insert=%7.2f "
                 "out=%7.2f tok=%7llu distinct=%5llu\n", (unsigned long long)b,
                 (unsigned long long)(b / ns), (unsigned long long)(b % ns),
                 (x[0] - t0) * 0.01, (x[1] - x[0]) * 0.01, (x[2] - x[1]) * 0.01,
                 (x[3] - t0) * 0.01, (unsigned long long)x[4], (unsigned long long)x[5]);
  }
}

void DevicePipeline::print_psort_trace() {
  if (!d_ord_trace) return;
  std::vector<u64> t(kDictParts * 16);
  LOCUST_HIP_CHECK(hipMemcpy(t.data(), d_ord_trace, t.size() * 8, hipMemcpyDeviceToHost));
  u64 first_in = ~0ull, last_out = 0;
  int last_p = -1;
  for (int p = 0; p < kDictParts; ++p) {
    const u64* x = &t[p * 16];
    if (!x[10]) continue;
    first_in = std::min(first_in, x[10]);
    if (x[11] > last_out) {
      last_out = x[11];
      last_p = p;
    }
  }
  if (last_p >= 0)
    std::fprintf(stderr, "psort span=%.2f us (first entry -> last exit), last p=%d m=%llu\n",
                 (last_out - first_in) * 0.01, last_p, (unsigned long long)t[last_p * 16 + 5]);
  for (int p = 0; p < kDictParts; ++p) {
    const u64* x = &t[p * 16];
    if (!x[0] || !x[4]) continue;
    auto d = [&](int a, int b) { return (unsigned long long)(x[a] && x[b] ? x[b] - x[a] : 0); };
    std::fprintf(stderr, "psort p=%3d m=%5llu passes=%2llu list=%6llu keys=%6llu sort=%6llu "
                 "write=%6llu | in=%6.2f out=%6.2f us\n", p, (unsigned long long)x[5],
                 (unsigned long long)x[6], d(0, 1), d(1, 2), d(2, 3), d(3, 4),
                 (x[10] - first_in) * 0.01, (x[11] - first_in) * 0.01);
  }
}

void DevicePipeline::print_ord_trace() {
  if (!d_ord_trace || warming) return;
  std::vector<u64> t(kDictParts * 32);
  LOCUST_HIP_CHECK(hipMemcpy(t.data(), d_ord_trace, t.size() * 8, hipMemcpyDeviceToHost));
  // stamps: 0 start, 1 built, 2 published, 8 histogram, 7 bucketed, 9 ranked, 3 sorted,
  // 4 prefix known, 5 written; 6 = distinct keys; 10 / 11 = entry / exit on the 100 MHz
  // device-wide clock (the kernel's critical path across workgroups)
  u64 first_in = ~0ull, last_out = 0;
  int last_p = -1;
  for (int p = 0; p < kDictParts; ++p) {
    const u64* x = &t[p * 32];
    if (!x[10]) continue;
    first_in = std::min(first_in, x[10]);
    if (x[11] > last_out) {
      last_out = x[11];
      last_p = p;
    }
  }
  if (last_p >= 0)
    std::fprintf(stderr, "ord span=%.2f us (first entry -> last exit), last p=%d m=%llu\n",
                 (last_out - first_in) * 0.01, last_p, (unsigned long long)t[last_p * 32 + 6]);
  {  // self-clean handshake: each workgroup's release + done count (25), the last one's
     // re-zeroing done (24; stale values from earlier jobs are older than this job's exits)
    u64 done_max = 0, clean = 0;
    for (int p = 0; p < kDictParts; ++p) {
      done_max = std::max(done_max, t[p * 32 + 25]);
      clean = std::max(clean, t[p * 32 + 24]);
    }
    if (last_p >= 0 && done_max >= last_out)
      std::fprintf(stderr, "ord tail: last exit -> last done count %.2f us, -> self-clean done %.2f us\n",
                   (done_max - last_out) * 0.01, clean >= last_out ? (clean - last_out) * 0.01 : -1.0);
  }

  for (int p = 0; p < kDictParts; ++p) {
    const u64* x = &t[p * 32];
    if (!x[0] || !x[6]) continue;
    auto d = [&](int a, int b) { return (unsigned long long)(x[a] && x[b] ? x[b] - x[a] : 0); };
    std::fprintf(stderr,
                 "ord p=%3d m=%5llu build=%6llu publish=%5llu sort=%6llu wait=%6llu write=%6llu"
                 " | hist=%5llu bucket=%5llu rank=%6llu scatter=%5llu | in=%6.2f out=%6.2f us"
                 " | clear=%5llu scan=%5llu fill=%5llu ld=%5llu srt=%5llu list=%5llu gather=%5llu lbk=%6llu rank0=%6llu cand=%6llu tie=%6llu ranks=%6llu"
                 " | waited=%6.2f us | counted=%6.2f us after exit\n",
                 p, (unsigned long long)x[6], d(0, 1), d(1, 2), d(2, 3), d(3, 4), d(4, 5),
                 d(2, 8), d(8, 7), d(7, 9), d(9, 3), (x[10] - first_in) * 0.01,
                 (x[11] - first_in) * 0.01, d(0, 14), d(14, 28), d(28, 26), d(26, 27), d(27, 12), d(14, 12), d(12, 13), d(2, 15), x[17] != ~0ull ? d(2, 17) : 0ull, d(2, 18), d(2, 19), d(2, 16),
                 x[20] ? (x[20] - x[10]) * 0.01 : 0.0,
                 x[25] >= x[11] ? (x[25] - x[11]) * 0.01 : -1.0);
  }
}

bool DevicePipeline::enqueue_dict_job(u32 num_lines, bool compat, bool with_counts, hipEvent_t after_process,
                        bool self_clean) {
  job_self_cleaned = false;
  if (!compat && ordered_ok()) {
    job_self_cleaned = self_clean && cfg.map_path == MapPath::kFast;
    enqueue_dict_ordered(with_counts, /*mapped=*/true, job_self_cleaned);
    if (after_process) LOCUST_HIP_CHECK(hipEventRecord(after_process, stream));
    return true;
  }
  if (!compat && !with_counts && large_ordered_ok()) {
    // large pass: per-slice partials (Process), then merge + sort + records (Reduce)
    enqueue_partials();
    if (after_process) LOCUST_HIP_CHECK(hipEventRecord(after_process, stream));
    OrderedExtra ex;
    ex.pm = part_map();
    ex.part_w = d_pw;
    ex.out_cap = h_out_cap;
    set_compact_out(ex, true);
    launch_dict_ordered_partials(d_partials, d_partial_n, partial_nslots, d_ctr, d_out_mapped,
                                 d_ctr_mapped,
                                 lb_dict, stream, ord_trace(), ex);
    return true;
  }
  enqueue_process_dict(num_lines, compat, with_counts);
  if (after_process) LOCUST_HIP_CHECK(hipEventRecord(after_process, stream));
  enqueue_emit_dict(/*mapped=*/true);
  return false;
}

void DevicePipeline::redo_dict_on_table(u32 num_lines, bool with_counts) {
  LOCUST_HIP_CHECK(hipMemsetAsync(&d_ctr->num_unique, 0, sizeof(u32), stream));
  LOCUST_HIP_CHECK(hipMemsetAsync(&d_ctr->flags, 0, sizeof(u32), stream));
  LOCUST_HIP_CHECK(hipMemsetAsync(dict.table, 0, dict_zero_bytes, stream));
  launch_dict_insert(tokens, with_counts ? d_counts : nullptr, &d_ctr->num_records, cap, dict,
                     d_ctr, stream);
  enqueue_rank();
  enqueue_emit_dict(/*mapped=*/true);
  sync();
  *h_ctr = *h_ctr_mapped;
}

void DevicePipeline::finish_dict_with_radix(u32 num_lines, bool with_counts) {
  if (h_ctr->flags & kCtrDictOverflow) {
    // table overflow: sort every record and reduce the reference way
    LOCUST_HIP_CHECK(hipMemsetAsync(lb_heads.status, 0, 8 * (div_up(cap, kReduceTile) + 1), stream));
    LOCUST_HIP_CHECK(hipMemsetAsync(lb_heads.tile_counter, 0, 4, stream));
    LOCUST_HIP_CHECK(hipMemsetAsync(lb_scan.status, 0, 8 * (div_up(cap, kReduceTile) + 1), stream));
    LOCUST_HIP_CHECK(hipMemsetAsync(lb_scan.tile_counter, 0, 4, stream));
    enqueue_process(num_lines, false, with_counts, h_ctr->num_records);
    enqueue_reduce_core(with_counts);
    enqueue_pack_output();
    return;
  }
  LOCUST_HIP_CHECK(hipMemsetAsync(lb_scan.status, 0, 8 * (div_up(cap, kReduceTile) + 1), stream));
  LOCUST_HIP_CHECK(hipMemsetAsync(lb_scan.tile_counter, 0, 4, stream));
  radix_sort(dict.ukeys, &d_ctr->num_unique, h_ctr->num_unique, rx, dict.ucount, sorted,
             d_sorted_counts, d_perm, h_plan, stream);
  enqueue_reduce_dict();
}

void DevicePipeline::download_output(WordCountResult& r, hipEvent_t done) {
  read_counters();
  const u64 u = h_ctr->num_unique;
  grow_host_out(u);
  if (u)
    launch_copy_to_mapped(d_out_mapped, d_out, u * sizeof(OutRecord), stream);
  if (done) LOCUST_HIP_CHECK(hipEventRecord(done, stream));
  sync();
  fill_counters(r);
  copy_out(r.entries, u);
}

void DevicePipeline::set_compact_out(OrderedExtra& ex, bool mapped) {
  ord_compact = mapped;
  if (!ord_compact) return;
  ex.cout = reinterpret_cast<u64*>(d_out_mapped);
  ex.ctab = d_ctab_mapped;
  ex.out_cap = std::min<u64>(ex.out_cap, h_out_cap);
}

void DevicePipeline::copy_out(EntryList& e, u64 u, bool compact) {
  static_assert(sizeof(WordCountEntry) == sizeof(OutRecord), "entry layout");
  static_assert(offsetof(WordCountEntry, count) == offsetof(OutRecord, count), "entry layout");
  LOCUST_CHECK_ARG(u <= h_out_cap, "output larger than its buffer");
  if (!compact) return e.adopt(out_pool[out_idx], reinterpret_cast<WordCountEntry*>(h_out), u);
  std::vector<EntrySegment> segs;
  segs.reserve(64);
  const u64* words = reinterpret_cast<const u64*>(h_out);
  u64 at = 0;  // entries so far
  for (int v = 0; v < kDictParts; ++v) {
    const u64 t = h_ctab[v];
    LOCUST_CHECK_ARG(t != ~0ull, "compact output: partition " + std::to_string(v) + " not written");
    const u64 m = t & 0xffffull, first = t >> 32;  // first: where its entries start
    LOCUST_CHECK_ARG(first + m <= h_out_cap, "compact output: partition " + std::to_string(v) +
                                                 " past the buffer");
    if (m) segs.push_back({words + kOutWords * first, m});
    at += m;
  }
  LOCUST_CHECK_ARG(at == u, "compact output: " + std::to_string(at) + " entries, expected " +
                                std::to_string(u));
  e.adopt_compact(out_pool[out_idx], std::move(segs), u);
}

void DevicePipeline::fill_counters(WordCountResult& r) const {
  r.num_tokens = h_ctr->total_count ? h_ctr->total_count : h_ctr->num_records;
  r.num_unique = h_ctr->num_unique;
  r.overflow_lines = h_ctr->overflow_lines;
  r.truncated = h_ctr->truncated;
  r.max_key_len = h_ctr->max_key_len;
}

WordCountResult DevicePipeline::run_ref_timed(const TextInput& in) {
  check_input(in);
  WordCountResult r;
  r.num_lines = in.num_lines;
  const bool compat = cfg.map_path == MapPath::kCompat;
  const bool dict_path = cfg.sort_path == SortPath::kDict;
  const u64 w0 = now_ns();
  enqueue_upload(in);
  sync();
  const u64 t0 = now_ns();
  enqueue_map(in);  // map timer: the launch only (main.cu:405-407)
  const u64 t1 = now_ns();
  if (dict_path) {
    enqueue_process_dict((u32)in.num_lines, compat);
  } else {
    enqueue_process((u32)in.num_lines, compat, false, kUnknownCount, /*allow_psort=*/true);
  }
  sync();  // process timer ends once the sort is done (thrust::sort returns)
  if (!dict_path && psort_used) {
    read_counters();
    if (h_ctr->flags & kCtrSortOverflow) {  // a partition outgrew the LDS sort
      redo_process_general((u32)in.num_lines);
      sync();
    }
  }
  const u64 t2 = now_ns();
  if (dict_path) {
    enqueue_emit_dict(/*mapped=*/true);  // the last reduce kernel: launch only (B4)
  } else {
    enqueue_reduce_core(false);
    enqueue_pack_output();
  }
  const u64 t3 = now_ns();
  if (dict_path) {
    sync();
    *h_ctr = *h_ctr_mapped;
    if (dict_fallback_needed()) {
      finish_dict_with_radix((u32)in.num_lines);
      download_output(r, nullptr);
    } else {
      fill_counters(r);
      copy_out(r.entries, h_ctr->num_unique);
    }
  } else {
    download_output(r, nullptr);
  }
  r.times.ref_map_ms = (t1 - t0) * 1e-6;
  r.times.ref_process_ms = (t2 - t1) * 1e-6;
  r.times.ref_reduce_ms = (t3 - t2) * 1e-6;
  r.times.wall_ms = (now_ns() - w0) * 1e-6;
  if (cfg.check) validate_result(r);
  return r;
}

WordCountResult DevicePipeline::run(const TextInput& in) {
  TraceRange tr("locust:job");
  const u64 tp = now_ns();
  poll_retune();
  const u64 tq = now_ns();
  select_out();  // the previous result may still hold the last output buffer
  if ((int)log_level() >= (int)LogLevel::kDebug)
    LOCUST_LOG_DEBUG("job prologue: retune adoption %.3f ms, output buffer %.3f ms",
                     (tq - tp) * 1e-6, (now_ns() - tq) * 1e-6);
  // The previous job left d_sync zeroed (self-cleaning ordered run): no reset this time.
  const bool clean_start = sync_clean;
  sync_clean = false;
  if (in.bytes > pass_bytes && cfg.sort_path == SortPath::kDict &&
      cfg.map_path == MapPath::kFast)
    return run_stream(in);
  if (cfg.ref_timers) return run_ref_timed(in);
  check_input(in);
  WordCountResult r;
  r.num_lines = in.num_lines;
  const u64 t0 = now_ns();
  const bool compat = cfg.map_path == MapPath::kCompat;
  const bool dict_path = cfg.sort_path == SortPath::kDict;
  struct ClearOnExit {  // only this entry point's dictionary pass combines in the map
    bool& f;
    ~ClearOnExit() { f = false; }
  } clear_combine{combine_map};
  combine_map = dict_path && !compat && large_ordered;
  const bool graphed = use_job_graph(in);
  // lean: a small single-pass job launched directly, no stage events, completion polled
  const bool lean = !graphed && lean_job(in);
  split_stages = !lean && !graphed;
  skip_sync_reset = clean_start && !compat;
  if (!lean) LOCUST_HIP_CHECK(hipEventRecord(ev[0], stream));
  const bool dbg = (int)log_level() >= (int)LogLevel::kDebug;
  u64 t_map = 0;
  if (lean) {
    enqueue_upload(in);
    enqueue_map(in);
    if (dbg) t_map = now_ns();
  } else if (graphed) {
    prepare_upload(in);
    launch_dict_graph(in, compat);
    LOCUST_HIP_CHECK(hipEventRecord(ev[5], stream));  // a replay has no stage split
    r.times.graph = true;
  } else {
    enqueue_upload(in);
    // Auto mode, piecewise pass: no stage markers between the kernels (the pass
    // interleaves Map and Process anyway); graph=0 keeps the split
    split_stages = pieces.empty() || cfg.graph == 0;
    if (split_stages) LOCUST_HIP_CHECK(hipEventRecord(ev[1], stream));
    enqueue_map(in);
    if (split_stages) {
      LOCUST_HIP_CHECK(hipEventRecord(ev[2], stream));
      // a piecewise pass interleaves Process (the per-piece partials) with Map: one
      // boundary, and no marker between the last partials and the ordered kernel
      if (!pieces.empty()) LOCUST_HIP_CHECK(hipEventRecord(ev[3], stream));
    }
  }
  if (dict_path) {
    bool ordered = graph_ordered;
    if (lean) {
      done_pending = ++done_seq;
      ordered = enqueue_dict_job((u32)in.num_lines, compat, false, nullptr,
                                 /*self_clean=*/true);
      if (done_pending) publish_done(done_seq);
      done_pending = 0;
    } else if (!graphed) {
      ordered = enqueue_dict_job((u32)in.num_lines, compat, false,
                                 split_stages && pieces.empty() ? ev[3] : nullptr,
                                 /*self_clean=*/true);
      if (split_stages) LOCUST_HIP_CHECK(hipEventRecord(ev[4], stream));
      LOCUST_HIP_CHECK(hipEventRecord(ev[5], stream));
    }
    skip_sync_reset = false;
    const u64 t_launched = now_ns();
    if (dbg && lean)
      LOCUST_LOG_DEBUG("lean job: map launched +%.4f ms, ordered launched +%.4f ms",
                       (t_map - t0) * 1e-6, (t_launched - t0) * 1e-6);
    if (lean)
      wait_done(done_seq);
    else
      sync();  // the one host synchronisation of a dictionary run
    const u64 t_synced = now_ns();
    r.times.host_launch_ms = (t_launched - t0) * 1e-6;
    r.times.host_wait_ms = (t_synced - t_launched) * 1e-6;
    *h_ctr = *h_ctr_mapped;
    if (ordered && h_ctr->num_unique > h_out_cap) h_ctr->flags |= kCtrDictOverflow;  // no records
    const bool ordered_done = ordered && !(h_ctr->flags & kCtrDictOverflow);
    sync_clean = ordered_done && !compat && job_self_cleaned;  // the kernel re-zeroed its scratch
    if (ordered) print_ord_trace();
    print_partials_trace();
    print_map_trace();
    if (ordered && !ordered_done) ++fallbacks;
    if (devplan_used) ++planned_passes;
    if (ordered && !ordered_done) redo_dict_on_table((u32)in.num_lines, map_combined);
    if (!ordered_done && dict_fallback_needed()) {
      finish_dict_with_radix((u32)in.num_lines, map_combined);
      LOCUST_HIP_CHECK(hipEventRecord(ev[4], stream));
      download_output(r, ev[5]);
      if (ordered) force_retune(r.entries);
    } else {
      fill_counters(r);
      copy_out(r.entries, h_ctr->num_unique, ordered_done && ord_compact);
      r.times.host_copy_ms = (now_ns() - t_synced) * 1e-6;
      if (ordered_done) maybe_retune(r.entries);
      else if (ordered) force_retune(r.entries);
    }
  } else {
    if (lean) {
      done_pending = ++done_seq;  // the fused kernel publishes it itself
      enqueue_radix_job((u32)in.num_lines, compat, nullptr, nullptr);
      if (done_pending) publish_done(done_seq);
      done_pending = 0;
    } else if (!graphed) {
      enqueue_radix_job((u32)in.num_lines, compat, ev[3], ev[4]);
    }
    skip_sync_reset = false;
    bool overflow;
    if (radix_mapped()) {  // records and counters already in host memory
      if (lean) {
        wait_done(done_seq);
      } else {
        if (!graphed) LOCUST_HIP_CHECK(hipEventRecord(ev[5], stream));
        sync();  // the one host synchronisation of a radix run
      }
      *h_ctr = *h_ctr_mapped;
      overflow = (h_ctr->flags & kCtrSortOverflow) != 0;
      // a fused run re-zeroed its scratch (not replayed from a graph: those reset it)
      sync_clean = lean && radix_fused && !overflow && !compat;
      if (psort_used) print_psort_trace();
      if (!overflow) {
        fill_counters(r);
        copy_out(r.entries, h_ctr->num_unique);
        if (psort_used) maybe_retune(r.entries);
      }
    } else {
      download_output(r, ev[5]);
      overflow = (h_ctr->flags & kCtrSortOverflow) != 0;
    }
    if (overflow) {  // a partition outgrew the LDS sort: the device-wide sort instead
      redo_radix_general((u32)in.num_lines);
      LOCUST_HIP_CHECK(hipEventRecord(ev[4], stream));
      download_output(r, ev[5]);
    }
  }
  r.times.wall_ms = (now_ns() - t0) * 1e-6;
  r.times.lean = lean;
  if (lean) {  // no device timestamps: the job's wall time
    r.times.gpu_ms = r.times.wall_ms;
  } else {
    if (!graphed && split_stages) {
      r.times.h2d_ms = ms_between(ev[0], ev[1]);
      r.times.map_ms = ms_between(ev[1], ev[2]);
      r.times.process_ms = ms_between(ev[2], ev[3]);
      r.times.reduce_ms = ms_between(ev[3], ev[4]);
      r.times.d2h_ms = ms_between(ev[4], ev[5]);
    }
    r.times.gpu_ms = ms_between(ev[0], ev[5]);
  }
  if (cfg.check) validate_result(r);
  return r;
}

bool DevicePipeline::host_pinned(const void* p) {
  hipPointerAttribute_t a{};
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();  // pageable memory: clear the sticky error
    return false;
  }
  return a.type == hipMemoryTypeHost;
}

void DevicePipeline::ensure_stream_buffers(bool staging, u64 nchunks) {
  if (!cstream) {
    LOCUST_HIP_CHECK(hipStreamCreateWithFlags(&cstream, hipStreamNonBlocking));
    for (int b = 0; b < 2; ++b) {
      LOCUST_HIP_CHECK(hipEventCreateWithFlags(&ev_copied[b], hipEventDisableTiming));
      LOCUST_HIP_CHECK(hipEventCreateWithFlags(&ev_consumed[b], hipEventDisableTiming));
    }
    size_t got = 0;  // the process-wide block cache, like the arena
    d_text_alt = static_cast<char*>(dev_block_alloc(cap_bytes + 64, &got));
    d_text_alt_block = got;
    LOCUST_HIP_CHECK(hipMalloc(&d_dctr, sizeof(MapCounters)));
  }
  if (staging && !h_stage[0])
    for (int b = 0; b < 2; ++b)
      h_stage[b] = static_cast<char*>(pinned_alloc(cap_bytes + 64, hipHostMallocDefault, "chunk staging"));
  // per-window counter snapshots (folded when full: at most 4096 pinned)
  nchunks = std::min<u64>(std::max<u64>(nchunks, 64), 4096);
  if (nchunks > h_chunk_cap) {
    if (h_chunk_ctr) LOCUST_HIP_CHECK(hipHostFree(h_chunk_ctr));
    h_chunk_cap = nchunks;
    LOCUST_HIP_CHECK(hipHostMalloc(&h_chunk_ctr, h_chunk_cap * sizeof(MapCounters),
                                   hipHostMallocDefault));
  }
}

u64 DevicePipeline::stream_ring_piece() const {
  return std::min<u64>(cap_bytes, cfg.ring_piece_bytes ? cfg.ring_piece_bytes : kRingPieceMax);
}

void DevicePipeline::ensure_read_ring(u64 piece) {
  if (ring_piece == piece) return;
  for (int i = 0; i < kRingPieces; ++i) {
    pinned_free(h_ring[i]);
    h_ring[i] = static_cast<char*>(pinned_alloc(piece + 64, hipHostMallocDefault, "read ring piece"));
    if (!ev_ring[i]) LOCUST_HIP_CHECK(hipEventCreateWithFlags(&ev_ring[i], hipEventDisableTiming));
  }
  ring_piece = piece;
}

char* DevicePipeline::ensure_h_text() {
  if (h_text) return h_text;
  h_text = static_cast<char*>(pinned_alloc(cap_bytes + 64, hipHostMallocDefault, "input text buffer"));
  if (hipHostGetDevicePointer(reinterpret_cast<void**>(&d_h_text), h_text, 0) != hipSuccess) {
    (void)hipGetLastError();
    d_h_text = nullptr;  // not device-visible: always DMA
  }
  return h_text;
}

std::vector<std::pair<u64, u64>> DevicePipeline::plan_chunks(const TextInput& in) const {
  std::vector<std::pair<u64, u64>> out;
  u64 pos = 0;
  while (pos < in.bytes) {
    u64 end = std::min<u64>(pos + cap_bytes, in.bytes);
    if (end < in.bytes) {
      const void* nl = memrchr(in.data + pos, '\n', (size_t)(end - pos));
      if (!nl)
        throw Error("a line longer than the engine's chunk size (" + std::to_string(cap_bytes) +
                    " B) at byte " + std::to_string(pos));
      end = (u64)(static_cast<const char*>(nl) - in.data) + 1;
    }
    out.emplace_back(pos, end - pos);
    pos = end;
  }
  return out;
}

size_t DevicePipeline::enqueue_stream_insert(const TextInput& in) {
  const auto chunks = plan_chunks(in);
  const bool pinned = host_pinned(in.data);
  size_t k = 0;
  return enqueue_stream_chunks(!pinned, chunks.size(), [&](int b, const char** src) -> u64 {
    if (k >= chunks.size()) return 0;
    const u64 off = chunks[k].first, len = chunks[k].second;
    ++k;
    *src = in.data + off;
    if (!pinned) {  // pageable input: host copy into the pinned half
      std::memcpy(h_stage[b], in.data + off, len);
      *src = h_stage[b];
    }
    return len;
  });
}

void DevicePipeline::snapshot_window_counters() {
  if (win_pending == h_chunk_cap) {  // full: fold the snapshots so far (one host sync)
    sync();
    for (u64 k = 0; k < win_pending; ++k) {
      const MapCounters& c = h_chunk_ctr[k];
      win_acc.num_records += c.num_records;
      win_acc.overflow_lines += c.overflow_lines;
      win_acc.truncated += c.truncated;
      win_acc.max_key_len = std::max(win_acc.max_key_len, c.max_key_len);
    }
    win_pending = 0;
  }
  LOCUST_HIP_CHECK(hipMemcpyAsync(&h_chunk_ctr[win_pending], d_ctr, sizeof(MapCounters),
                                  hipMemcpyDeviceToHost, stream));
  ++win_pending;
}

void DevicePipeline::enqueue_map_window(const char* dtext, u64 len, const DelimMask& dm) {
  LOCUST_HIP_CHECK(hipMemsetAsync(d_sync, 0, sync_bytes, stream));
  launch_map_fast(dtext, len, dm, cfg.emits_per_line, cfg.max_key_len, tokens, nullptr, cap,
                  d_ctr, lb_map, stream);
  snapshot_window_counters();
  launch_dict_insert(tokens, nullptr, &d_ctr->num_records, cap, dict, d_dctr, stream);
}

u64 DevicePipeline::window_len(const char* p, u64 n) const {
  if (n <= map_window) return n;
  const void* nl = memrchr(p, '\n', (size_t)map_window);
  if (nl) return (u64)(static_cast<const char*>(nl) - p) + 1;
  // one line longer than a window: it alone (its tokens are capped at emits_per_line)
  nl = std::memchr(p + map_window, '\n', (size_t)(n - map_window));
  return nl ? (u64)(static_cast<const char*>(nl) - p) + 1 : n;
}

size_t DevicePipeline::enqueue_stream_source(TextSource& src_text) {
  LOCUST_CHECK_ARG(cfg.sort_path == SortPath::kDict && cfg.map_path == MapPath::kFast,
                   "inputs larger than the engine capacity stream through the dictionary "
                   "path with the fast map (sort=dict, map=fast)");
  const u64 piece = stream_ring_piece();
  // a map window closes before a piece would overflow it: windows >= map_window - piece
  const u64 min_window = map_window > piece ? map_window - piece : std::max<u64>(map_window / 2, 1);
  const u64 t_setup = now_ns();
  ensure_stream_buffers(false, div_up(std::max<u64>(src_text.size(), 1), min_window) + 2);
  const u64 t_bufs = now_ns();
  reset_window_counters();
  ensure_read_ring(piece);
  if ((int)log_level() >= (int)LogLevel::kDebug)
    LOCUST_LOG_DEBUG("stream setup: copy stream / second chunk / counters %.2f ms, read ring %.2f ms",
                     (t_bufs - t_setup) * 1e-6, (now_ns() - t_bufs) * 1e-6);
  const DelimMask dm = make_delim_mask(cfg.delimiters.c_str());
  LOCUST_HIP_CHECK(hipMemsetAsync(dict.table, 0, dict_zero_bytes, stream));
  LOCUST_HIP_CHECK(hipMemsetAsync(d_dctr, 0, sizeof(MapCounters), stream));
  // the copy stream must not overwrite a text buffer before the reset is queued
  LOCUST_HIP_CHECK(hipEventRecord(ev_copied[1], stream));
  LOCUST_HIP_CHECK(hipStreamWaitEvent(cstream, ev_copied[1], 0));
  size_t k = 0;     // chunks closed
  u64 fill = 0;     // bytes in chunk k
  u64 mapped = 0;   // bytes of chunk k already mapped (the windows so far)
  int last_slot = -1;  // the ring slot of the last piece copied into chunk k
  auto chunk_text = [&](size_t c) { return (c & 1) ? d_text_alt : d_text; };
  // Map + insert chunk k's bytes [mapped, fill) as one window, once their copies landed.
  auto map_pending = [&] {
    if (fill == mapped) return;
    LOCUST_HIP_CHECK(hipStreamWaitEvent(stream, ev_ring[last_slot], 0));
    enqueue_map_window(chunk_text(k) + mapped, fill - mapped, dm);
    mapped = fill;
  };
  auto close_chunk = [&] {
    const int b = (int)(k & 1);
    map_pending();
    // the chunk buffer is free for its refill two chunks on once its last map ran
    LOCUST_HIP_CHECK(hipEventRecord(ev_consumed[b], stream));
    ++k;
    fill = mapped = 0;
  };
  for (u64 r = 0;; ++r) {
    const int slot = (int)(r % kRingPieces);
    // the slot's previous H2D must have drained before the source refills it
    if (r >= (u64)kRingPieces) LOCUST_HIP_CHECK(hipEventSynchronize(ev_ring[slot]));
    const u64 n = src_text.next(h_ring[slot], piece);
    if (!n) break;
    if (fill + n > cap_bytes)
      close_chunk();
    else if (fill - mapped + n > map_window)
      map_pending();  // the window so far, before this piece would overflow it
    // a chunk buffer is refilled only after the maps two chunks back consumed it
    if (fill == 0 && k >= 2)
      LOCUST_HIP_CHECK(hipStreamWaitEvent(cstream, ev_consumed[k & 1], 0));
    LOCUST_HIP_CHECK(hipMemcpyAsync(chunk_text(k) + fill, h_ring[slot], n, hipMemcpyHostToDevice,
                                    cstream));
    LOCUST_HIP_CHECK(hipEventRecord(ev_ring[slot], cstream));
    last_slot = slot;
    fill += n;
  }
  if (fill) close_chunk();
  // hand the dictionary's counters to the single-pass stages that follow
  LOCUST_HIP_CHECK(hipMemcpyAsync(&d_ctr->num_unique, &d_dctr->num_unique, sizeof(u32),
                                  hipMemcpyDeviceToDevice, stream));
  LOCUST_HIP_CHECK(hipMemcpyAsync(&d_ctr->flags, &d_dctr->flags, sizeof(u32),
                                  hipMemcpyDeviceToDevice, stream));
  return k;
}

void DevicePipeline::stream_stats(size_t nchunks, WordCountResult& r) const {
  r.num_tokens = win_acc.num_records;
  r.overflow_lines = win_acc.overflow_lines;
  r.truncated = win_acc.truncated;
  r.max_key_len = win_acc.max_key_len;
  for (u64 k = 0; k < win_pending; ++k) {
    const MapCounters& c = h_chunk_ctr[k];
    r.num_tokens += c.num_records;
    r.overflow_lines += c.overflow_lines;
    r.truncated += c.truncated;
    r.max_key_len = std::max<u64>(r.max_key_len, c.max_key_len);
  }
  r.chunks = nchunks;
}

WordCountResult DevicePipeline::run_source(TextSource& src) {
  sync_clean = false;
  select_out();
  WordCountResult r = finish_stream(0, [&] { return enqueue_stream_source(src); });
  r.num_lines = src.lines();
  return r;
}

void DevicePipeline::download_keys(const KeysSoA& src, u64 n, std::vector<PackedKey>* out) {
  out->resize(n);
  if (!n) return;
  grow_host_keys(n);
  for (int w = 0; w < kKeyWords; ++w)
    LOCUST_HIP_CHECK(hipMemcpyAsync(h_keys + (u64)w * n, src.w[w], n * sizeof(u64),
                                    hipMemcpyDeviceToHost, stream));
  sync();
  for (u64 i = 0; i < n; ++i)
    for (int w = 0; w < kKeyWords; ++w) (*out)[i].w[w] = h_keys[(u64)w * n + i];
}

void DevicePipeline::set_num_records(u64 n) {
  LOCUST_CHECK_ARG(n <= cap, "too many records for engine capacity");
  LOCUST_HIP_CHECK(hipMemsetAsync(d_sync, 0, sync_bytes, stream));
  h_u64[0] = n;  // little endian: low 32 bits == num_records
  LOCUST_HIP_CHECK(hipMemcpyAsync(&d_ctr->num_records, h_u64, sizeof(u32),
                                  hipMemcpyHostToDevice, stream));
}

void DevicePipeline::upload_keys(const KeysSoA& dst, const PackedKey* keys, u64 n) {
  grow_host_keys(n);
  for (u64 i = 0; i < n; ++i)
    for (int w = 0; w < kKeyWords; ++w) h_keys[(u64)w * n + i] = keys[i].w[w];
  if (n)
    for (int w = 0; w < kKeyWords; ++w)
      LOCUST_HIP_CHECK(hipMemcpyAsync(dst.w[w], h_keys + (u64)w * n, n * sizeof(u64),
                                      hipMemcpyHostToDevice, stream));
}

}  // namespace detail

DevicePassPlan plan_device_pass(const JobConfig& cfg, u64 max_bytes, u64 max_lines,
                                u64 cap_records, u64 free_bytes) {
  using detail::DevicePipeline;
  const u64 E = (u64)std::max(cfg.emits_per_line, 1);
  const u64 share = (u64)std::max(cfg.hbm_share, 1);
  const u64 budget = (u64)((long double)free_bytes * kHbmUsable) / share;
  auto make = [&](bool stream, u64 chunk) {
    DevicePassPlan p;
    p.streaming = stream;
    if (stream) {
      p.chunk_bytes = std::max<u64>(chunk, 1);
      p.map_window = std::min<u64>(p.chunk_bytes, kStreamMapWindow);
      p.pass_bytes = p.map_window;
      p.cap_lines = p.map_window;
      // a window's tokens (a byte in two); the dictionary of a streamed input collects
      // the distinct keys of ALL windows: room for 2^20 of them even in small windows
      p.cap = std::max<u64>(p.map_window / 2 + 1, 1ull << 20);
    } else {
      p.chunk_bytes = std::max<u64>(max_bytes, 1);
      p.pass_bytes = p.chunk_bytes;
      p.map_window = p.chunk_bytes;  // (an input streamed through it anyway: chunk-sized maps)
      p.cap_lines = std::max<u64>(max_lines, 1);
      p.cap = cap_records ? cap_records : std::min<u64>(p.cap_lines * E, p.chunk_bytes / 2 + 1);
    }
    p.cap = std::max<u64>(p.cap, 1);
    // dense distinct-key capacity: every key of a pass, at most 16M (a 2^25-slot table)
    p.ucap = std::min<u64>(p.cap, 1ull << 24);
    // a dictionary engine's sort / reduce buffers hold its distinct keys (every ordered and
    // table path emits <= ucap of them); a receiver (cap_records) or a radix engine sorts
    // every record
    p.rcap = cfg.sort_path == SortPath::kDict && !cap_records ? p.ucap : p.cap;
    p.device_bytes = DevicePipeline::shape_arena(cfg, p, DevicePipeline::small_pass_limit()).arena_bytes;
    if (stream) p.device_bytes += p.chunk_bytes + 64;  // the second chunk buffer
    p.budget_bytes = budget;
    return p;
  };
  const bool streamable = !cap_records && cfg.sort_path == SortPath::kDict &&
                          cfg.map_path == MapPath::kFast;
  const bool asked = cfg.chunk_bytes && max_bytes > cfg.chunk_bytes && !cap_records;
  DevicePassPlan p = make(asked, cfg.chunk_bytes);
  if (!asked && streamable) {
    std::string why;
    if (p.cap >= (1ull << 30))
      why = "more than 2^30 tokens in one pass";
    else if (free_bytes && p.device_bytes > budget)
      why = "one pass would need " + std::to_string(p.device_bytes >> 20) + " MiB of the " +
            std::to_string(budget >> 20) + " MiB of HBM this engine may use";
    if (!why.empty()) {
      // the chunk asked for covers the whole input, and one pass of it does not fit
      LOCUST_CHECK_ARG(!cfg.chunk_bytes,
                       "--chunk-mb " + std::to_string(cfg.chunk_bytes >> 20) +
                           " asks for one device pass of the whole " +
                           std::to_string(max_bytes) + " B input: " + why +
                           "; use a smaller --chunk-mb (LOCUST_CHUNK_MB)");
      if (max_bytes > kDefaultStreamChunk) {
        p = make(true, kDefaultStreamChunk);
        p.why = why;
      }
    }
  }
  LOCUST_CHECK_ARG(p.cap < (1ull << 30),
                   "more than 2^30 records per GPU call (" + std::to_string(p.cap) +
                       "); inputs this large stream on the dictionary path with the fast map");
  if (free_bytes && p.device_bytes > budget) {
    char msg[512];
    std::snprintf(msg, sizeof(msg),
                  "device pass of %llu B needs %.2f GiB of HBM but this engine may use %.2f GiB "
                  "(%.2f GiB free x %.2f / %d engine(s) on the GPU)%s",
                  (unsigned long long)p.chunk_bytes, p.device_bytes / 1073741824.0,
                  budget / 1073741824.0, free_bytes / 1073741824.0, kHbmUsable,
                  std::max(cfg.hbm_share, 1),
                  p.streaming ? ": use a smaller --chunk-mb (LOCUST_CHUNK_MB)"
                              : ": stream it with --chunk-mb (dictionary path, fast map)");
    throw Error(msg);
  }
  return p;
}

}  // namespace locust
