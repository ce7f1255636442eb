// Per-rank GPU shard engine of the distributed driver (csrc/engine/dist.cpp): map +
// combine of this rank's shard, shuffle records and splitter samples, reduce of the
// received records, and the root's merge of the gather strategy.
#include <map>
#include <mutex>
#include <thread>

#include <sys/mman.h>

#include "locust/numa.hpp"
#include "locust/shm.hpp"
#include "pipeline.hpp"

namespace locust {

using detail::DevicePipeline;
using detail::kMaxRanks;
using detail::kMaxSamples;

// =====================================================================================
// GPU shard engine (one rank of the distributed job)
// =====================================================================================
namespace {

class GpuShardEngine final : public ShardEngine {
 public:
  GpuShardEngine(const JobConfig& cfg, u64 max_bytes, u64 max_lines)
      : cfg_(cfg), mp_(new DevicePipeline(cfg, max_bytes, max_lines)) {}

  ~GpuShardEngine() override {
    if (mp_) (void)hipStreamSynchronize(mp_->stream);  // pending copies from the pinned headers
    for (auto& g : slot_graphs_) (void)hipGraphExecDestroy(g.exec);
    if (h_headers_) (void)hipHostFree(h_headers_);
    if (h_send_header_) (void)hipHostFree(h_send_header_);
    free_exch();
  }

  bool device_buffers() const override { return true; }
  void* stream() override { return mp_->stream; }
  bool run_whole(const TextInput& shard, WordCountResult* r) override {
    // a shard read from a source (a file range larger than one pass) streams through
    // map_local's chunked path; the single-engine run() takes text in memory only
    if (shard.source) return false;
    *r = mp_->run(shard);
    mp_->sync_clean = false;  // the shard entry points reset the scratch themselves
    return true;
  }
  char* input_buffer() override { return mp_->ensure_h_text(); }
  u64 host_pinned_bytes() const override { return mp_->pinned_bytes(); }
  u64 device_bytes() const override {
    return mp_->device_bytes() + (rp_ ? rp_->device_bytes() : 0);
  }
  u64 hbm_free() const override { return mp_->hbm_free; }
  u64 hbm_total() const override { return mp_->hbm_total; }
  u64 hbm_used_now() const override {
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) != hipSuccess) {
      (void)hipGetLastError();
      return 0;
    }
    return (u64)(tot - fr);
  }
  u64 shared_pinned_bytes() const override {
    return out_ ? shm_segment_bytes(out_->region_records * out_->regions, sizeof(OutRecord)) : 0;
  }

  u64 map_local(const TextInput& shard, bool combine, DistStrategy plan) override {
    DevicePipeline& m = *mp_;
    const bool compat = cfg_.map_path == MapPath::kCompat;
    samples_valid_ = false;
    sorted_local_ = true;
    distinct_local_ = true;  // every path below yields distinct keys except combine=false
    stream_chunks_ = 0;
    const bool streamed = shard.bytes > m.pass_bytes;
    LOCUST_CHECK_ARG(!shard.source || streamed,
                     "a shard read from a source must be larger than one device pass");
    const bool small_ordered = combine && cfg_.sort_path == SortPath::kDict && !streamed &&
                               cfg_.map_path == MapPath::kFast &&
                               (m.cap <= kPartBuildMaxTokens || m.small_pass);
    if (streamed) {
      // a shard larger than one device pass: chunked H2D + map into one dictionary
      LOCUST_CHECK_ARG(combine && cfg_.sort_path == SortPath::kDict,
                       "streaming shards need the map-side combine of the dictionary path");
      stream_chunks_ = shard.source ? m.enqueue_stream_source(*shard.source)
                                    : m.enqueue_stream_insert(shard);
    } else if (!small_ordered) {
      m.check_input(shard);
      // a large dictionary pass maps in upload pieces with per-tile combining
      m.combine_map = combine && cfg_.sort_path == SortPath::kDict && m.large_ordered;
      m.enqueue_upload(shard);
      m.enqueue_map(shard);
      m.combine_map = false;
    }
    if (small_ordered) {
      enqueue_small_ordered(shard, plan != DistStrategy::kGather, nullptr, 0);
      m.sync();
      return complete_small_ordered(shard);
    }
    if (combine && cfg_.sort_path == SortPath::kDict && !streamed && m.large_ordered_ok())
      return large_ordered_map(shard, plan);
    m.sync_clean = false;  // the paths below dirty the scratch without re-zeroing it
    if (combine && cfg_.sort_path == SortPath::kDict) {
      if (plan == DistStrategy::kGather) {
        // Gather plan: the combined records go to rank 0 unsorted, straight from the
        // dictionary's dense arrays; no local sort at all.
        if (!streamed) m.enqueue_dict_insert((u32)shard.num_lines, compat, false);
        launch_pack_records(m.dict.ukeys, m.dict.ucount, &m.d_ctr->num_unique, m.ucap,
                            m.d_records, m.stream);
        m.read_counters();
        if (!(m.h_ctr->flags & kCtrDictOverflow)) {
          set_local(m.dict.ukeys, m.dict.ucount, &m.d_ctr->num_unique);
          sorted_local_ = false;
          return finish_map_stats(shard, m.h_ctr->num_unique);
        }
        return map_overflow_fallback(shard);
      }
      // Map-side combine through the dictionary: sorted distinct keys + counts.  The
      // shuffle records and the splitter samples are produced speculatively in the same
      // stream, so the common case costs ONE host synchronisation.
      if (streamed)
        m.enqueue_rank();
      else
        m.enqueue_process_dict((u32)shard.num_lines, compat);
      m.enqueue_sorted_from_dict();
      set_local(m.sorted, m.d_sorted_counts, &m.d_ctr->num_unique);
      launch_pack_records(local_keys_, local_counts_, local_n_, m.cap, m.d_records, m.stream);
      launch_sample_keys(local_keys_, local_n_, kSpecSamples, m.d_samples, m.stream);
      LOCUST_HIP_CHECK(hipMemcpyAsync(m.h_small, m.d_samples, kSpecSamples * sizeof(PackedKey),
                                      hipMemcpyDeviceToHost, m.stream));
      m.read_counters();
      if (!m.dict_fallback_needed()) {
        samples_.assign(m.h_small, m.h_small + kSpecSamples);
        samples_valid_ = true;
        return finish_map_stats(shard, m.h_ctr->num_unique);
      }
      if (m.h_ctr->flags & kCtrDictOverflow) return map_overflow_fallback(shard);
      // more distinct keys than the rank sort takes: radix-sort the dictionary's keys
      radix_sort(m.dict.ukeys, &m.d_ctr->num_unique, m.h_ctr->num_unique, m.rx, m.dict.ucount,
                 m.sorted, m.d_sorted_counts, m.d_perm, m.h_plan, m.stream);
      set_local(m.sorted, m.d_sorted_counts, &m.d_ctr->num_unique);
    } else {
      m.enqueue_process((u32)shard.num_lines, compat, false);
      if (combine) {
        // Map-side combine: local (key, count) runs become the shuffle records.
        m.enqueue_reduce_core(false);
        set_local(m.heads, m.d_head_count, &m.d_ctr->num_unique);
      } else {
        set_local(m.sorted, nullptr, &m.d_ctr->num_records);
        distinct_local_ = false;
      }
    }
    launch_pack_records(local_keys_, local_counts_, local_n_, m.cap, m.d_records, m.stream);
    m.read_counters();
    return finish_map_stats(shard, combine ? m.h_ctr->num_unique : m.h_ctr->num_records);
  }

  // Large pass (past kPartBuildMaxTokens, mapped above with the partition table): the
  // two-kernel ordered build writes this rank's sorted distinct keys straight into the
  // shuffle records and the SoA keys + counts the exchange reads; ONE host sync.  A table
  // overflow (e.g. the first job, on the first-byte map) redoes the pass on the HBM table
  // and retunes the map from its output.
  u64 large_ordered_map(const TextInput& shard, DistStrategy plan) {
    DevicePipeline& m = *mp_;
    const bool weighted = m.map_combined;
    m.enqueue_partials();
    OrderedExtra ex;
    ex.pm = m.part_map();
    ex.part_w = m.d_pw;
    ex.recs = m.d_records;
    ex.sorted = m.sorted;
    ex.counts = m.d_sorted_counts;
    launch_dict_ordered_partials(m.d_partials, m.d_partial_n, m.partial_nslots, m.d_ctr, nullptr,
                                 m.d_ctr_mapped,
                                 m.lb_dict, m.stream, nullptr, ex);
    set_local(m.sorted, m.d_sorted_counts, &m.d_ctr->num_unique);
    const bool spec = plan != DistStrategy::kGather;
    if (spec) {
      launch_sample_keys(local_keys_, local_n_, kSpecSamples, m.d_samples, m.stream);
      LOCUST_HIP_CHECK(hipMemcpyAsync(m.h_small, m.d_samples, kSpecSamples * sizeof(PackedKey),
                                      hipMemcpyDeviceToHost, m.stream));
    }
    m.sync();
    *m.h_ctr = *m.h_ctr_mapped;
    if (!(m.h_ctr->flags & kCtrDictOverflow)) {
      m.maybe_retune_records(m.d_records, m.h_ctr->num_unique);
      if (spec) {
        samples_.assign(m.h_small, m.h_small + kSpecSamples);
        samples_valid_ = true;
      }
      return finish_map_stats(shard, m.h_ctr->num_unique);
    }
    LOCUST_HIP_CHECK(hipMemsetAsync(&m.d_ctr->num_unique, 0, sizeof(u32), m.stream));
    LOCUST_HIP_CHECK(hipMemsetAsync(&m.d_ctr->flags, 0, sizeof(u32), m.stream));
    LOCUST_HIP_CHECK(hipMemsetAsync(m.dict.table, 0, m.dict_zero_bytes, m.stream));
    launch_dict_insert(m.tokens, weighted ? m.d_counts : nullptr, &m.d_ctr->num_records, m.cap,
                       m.dict, m.d_ctr, m.stream);
    m.read_counters();
    if (m.h_ctr->flags & kCtrDictOverflow)
      throw Error("large map pass: more distinct keys than the dictionary holds");
    if (m.h_ctr->num_unique <= (u32)kRankSortMax) {
      m.enqueue_rank();
      m.enqueue_sorted_from_dict();
    } else {
      radix_sort(m.dict.ukeys, &m.d_ctr->num_unique, m.h_ctr->num_unique, m.rx, m.dict.ucount,
                 m.sorted, m.d_sorted_counts, m.d_perm, m.h_plan, m.stream);
    }
    set_local(m.sorted, m.d_sorted_counts, &m.d_ctr->num_unique);
    launch_pack_records(local_keys_, local_counts_, local_n_, m.cap, m.d_records, m.stream);
    m.read_counters();
    m.maybe_retune_records(m.d_records, m.h_ctr->num_unique, /*force=*/true);
    return finish_map_stats(shard, m.h_ctr->num_unique);
  }

  // Small pass: upload, map and the ordered kernel give this rank's distinct keys sorted,
  // with counts; one more kernel lays them out as shuffle records + SoA keys (and, with
  // `hdr`, the gather slot's header), optionally the splitter samples, and the counters
  // come back -- one captured graph.  The gather plan needs no samples (a mispredict
  // samples late).
  bool small_ordered_ok(const TextInput& shard, bool combine) const {
    const DevicePipeline& m = *mp_;
    return combine && cfg_.sort_path == SortPath::kDict && shard.bytes <= m.pass_bytes &&
           cfg_.map_path == MapPath::kFast && (m.cap <= kPartBuildMaxTokens || m.small_pass);
  }
  // Host half of a small ordered pass (run for every job): returns the graph key of the
  // device half and the device half itself, which captures everything it needs by value
  // (so it can be captured later, inside a larger graph).
  using DeviceHalf = std::function<void()>;
  std::pair<DevicePipeline::GraphKeyArr, DeviceHalf> prepare_small_ordered(
      const TextInput& shard, bool spec_samples, SlotHeader* hdr, u32 slot_recs) {
    DevicePipeline& m = *mp_;
    m.check_input(shard);
    m.prepare_upload(shard);
    set_local(m.sorted, m.d_sorted_counts, &m.d_ctr->num_unique);
    spec_samples_ = spec_samples;
    SlotHeader tmpl{};
    tmpl.status = kSlotOk;
    tmpl.record_flags = kRecordsSorted | kRecordsDistinct;
    tmpl.lines = shard.num_lines;
    tmpl.slot_cap = slot_capacity();
    // The ordered kernel writes the records, the SoA keys + counts, the slot header and the
    // host-mapped counters itself: no conversion kernel, no counter copy.
    OrderedExtra ex;
    ex.pm = m.part_map();
    ex.part_w = m.d_pw;
    ex.recs = m.d_records;
    ex.sorted = m.sorted;
    ex.counts = m.d_sorted_counts;
    ex.hdr = hdr;
    ex.tmpl = tmpl;
    // Back-to-back small passes: the ordered kernel re-zeroes the scratch it and the map
    // dirtied, so the next pass skips the reset memset (m.sync_clean; any other use of this
    // pipeline clears it).
    m.set_self_clean(ex);
    const bool no_reset = m.sync_clean;
    m.sync_clean = false;
    m.parts_ready = true;  // set before enqueue: ordered_ok() is consulted while capturing
    const DevicePipeline::GraphKeyArr key{
        (spec_samples ? 2u : 3u) | (hdr ? 0x100u : 0u) | (no_reset ? 0x200u : 0u) |
            ((u64)slot_recs << 32),
        shard.bytes, shard.num_lines, reinterpret_cast<u64>(m.map_text), (u64)m.upload_mode,
        m.upload_mode == DevicePipeline::Upload::kDirect ? reinterpret_cast<u64>(shard.data) : 0};
    DeviceHalf enqueue = [this, shard, spec_samples, ex, no_reset]() mutable {
      DevicePipeline& m = *mp_;
      m.skip_sync_reset = no_reset;
      m.enqueue_upload_device(shard);
      m.skip_sync_reset = false;
      m.enqueue_map(shard);
      m.set_tile_source(ex, false);
      launch_dict_ordered(m.tokens, nullptr, m.d_parts, &m.d_ctr->num_records, m.cap, m.d_ctr,
                          nullptr, m.d_ctr_mapped, m.lb_dict, m.stream, m.ord_trace(), ex);
      if (spec_samples) {
        launch_sample_keys(local_keys_, local_n_, kSpecSamples, m.d_samples, m.stream);
        LOCUST_HIP_CHECK(hipMemcpyAsync(m.h_small, m.d_samples, kSpecSamples * sizeof(PackedKey),
                                        hipMemcpyDeviceToHost, m.stream));
      }
    };
    return {key, std::move(enqueue)};
  }
  void enqueue_small_ordered(const TextInput& shard, bool spec_samples, SlotHeader* hdr,
                             u32 slot_recs) {
    DevicePipeline& m = *mp_;
    auto half = prepare_small_ordered(shard, spec_samples, hdr, slot_recs);
    if (m.graph_launches())
      m.launch_cached(half.first, half.second);
    else
      half.second();
  }
  // After the sync of an enqueue_small_ordered: the map statistics, or the local redo on
  // the HBM table when a partition overflowed its LDS table.
  u64 complete_small_ordered(const TextInput& shard) {
    DevicePipeline& m = *mp_;
    *m.h_ctr = *m.h_ctr_mapped;
    if (!(m.h_ctr->flags & kCtrDictOverflow)) {
      m.sync_clean = true;  // the kernel re-zeroed the scratch (see enqueue_small_ordered)
      m.maybe_retune_records(m.d_records, m.h_ctr->num_unique);
      if (spec_samples_) {
        samples_.assign(m.h_small, m.h_small + kSpecSamples);
        samples_valid_ = true;
      }
      return finish_map_stats(shard, m.h_ctr->num_unique);
    }
    LOCUST_HIP_CHECK(hipMemsetAsync(&m.d_ctr->num_unique, 0, sizeof(u32), m.stream));
    LOCUST_HIP_CHECK(hipMemsetAsync(&m.d_ctr->flags, 0, sizeof(u32), m.stream));
    LOCUST_HIP_CHECK(hipMemsetAsync(m.dict.table, 0, m.dict_zero_bytes, m.stream));
    launch_dict_insert(m.tokens, nullptr, &m.d_ctr->num_records, m.cap, m.dict, m.d_ctr,
                       m.stream);
    m.read_counters();
    if (m.h_ctr->flags & kCtrDictOverflow) return map_overflow_fallback(shard);
    if (m.h_ctr->num_unique <= (u32)kRankSortMax) {
      m.enqueue_rank();
      m.enqueue_sorted_from_dict();
    } else {
      radix_sort(m.dict.ukeys, &m.d_ctr->num_unique, m.h_ctr->num_unique, m.rx, m.dict.ucount,
                 m.sorted, m.d_sorted_counts, m.d_perm, m.h_plan, m.stream);
    }
    set_local(m.sorted, m.d_sorted_counts, &m.d_ctr->num_unique);
    launch_pack_records(local_keys_, local_counts_, local_n_, m.cap, m.d_records, m.stream);
    m.read_counters();
    // the next pass should fit: rebuild the partition map from this one's keys
    m.maybe_retune_records(m.d_records, m.h_ctr->num_unique, /*force=*/true);
    return finish_map_stats(shard, m.h_ctr->num_unique);
  }

  // ---- gather strategy in one all-gather (ShardEngine::enqueue_map_slot and friends) ----
  u64 slot_capacity() const override { return mp_->slot_records_cap(); }

  void* enqueue_map_slot(const TextInput& shard, u32 slot_recs) override {
    DevicePipeline& m = *mp_;
    LOCUST_CHECK_ARG(slot_recs <= m.slot_records_cap(), "slot larger than the send buffer");
    SlotHeader* hdr = reinterpret_cast<SlotHeader*>(m.d_records - kSlotHeaderRecords);
    slot_fast_ = small_ordered_ok(shard, true);
    if (slot_fast_) {
      samples_valid_ = false;
      sorted_local_ = true;
      distinct_local_ = true;
      stream_chunks_ = 0;
      enqueue_small_ordered(shard, false, hdr, slot_recs);
      return hdr;
    }
    // Not a small pass: map synchronously (sorted, combined records), header from the host.
    const u64 n = map_local(shard, true, DistStrategy::kShuffle);
    SlotHeader* h = slot_host_header();
    *h = SlotHeader{};
    h->status = (sorted_local_ && distinct_local_ && n <= slot_recs) ? kSlotOk : kSlotRedo;
    h->record_flags = record_flags();
    h->n = n;
    h->lines = local_stats_.num_lines;
    h->tokens = local_stats_.num_tokens;
    h->overflow_lines = local_stats_.overflow_lines;
    h->truncated = local_stats_.truncated;
    h->max_key_len = local_stats_.max_key_len;
    h->slot_cap = slot_capacity();
    LOCUST_HIP_CHECK(hipMemcpyAsync(hdr, h, sizeof(SlotHeader), hipMemcpyHostToDevice, m.stream));
    return hdr;
  }

  void* write_slot_failure() override {
    DevicePipeline& m = *mp_;
    SlotHeader* h = slot_host_header();
    *h = SlotHeader{};
    h->status = kSlotFailed;
    h->slot_cap = slot_capacity();
    LOCUST_HIP_CHECK(hipMemcpyAsync(m.d_records - kSlotHeaderRecords, h, sizeof(SlotHeader),
                                    hipMemcpyHostToDevice, m.stream));
    slot_fast_ = false;
    local_count_ = 0;
    return m.d_records - kSlotHeaderRecords;
  }

  void* slot_buffer(u32 nslots, u32 slot_recs) override {
    // rp_ holds the slots in d_records; its d_out (40-B records) is the merge scratch.
    return recv_records((u64)nslots * (kSlotHeaderRecords + slot_recs));
  }

  // Host half of the root merge (buffers grown for this shape) + its device half.
  std::pair<DevicePipeline::GraphKeyArr, DeviceHalf> prepare_merge_slots(u32 nslots,
                                                                         u32 slot_recs) {
    DevicePipeline& r = *rp_;
    LOCUST_CHECK_ARG(nslots <= (u32)kMaxMergeRunsHost, "too many slots to merge");
    r.grow_host_out((u64)nslots * slot_recs);
    grow_headers(nslots);
    merge_copied_headers_ = true;
    // rp_gen_: graphs bake in rp_'s buffers beyond the ones in the key (d_out, d_ctr, the
    // look-back scratch); a reallocated rp_ may reuse d_records' address, so its
    // generation is part of every key that captures rp_ buffers.
    const DevicePipeline::GraphKeyArr key{
        6 | (rp_gen_ << 8), ((u64)nslots << 32) | slot_recs, reinterpret_cast<u64>(r.d_records),
        reinterpret_cast<u64>(r.d_out_mapped), reinterpret_cast<u64>(r.d_ctr_mapped),
        reinterpret_cast<u64>(d_headers_)};
    DeviceHalf enqueue = [this, nslots, slot_recs]() {
      DevicePipeline& m = *mp_;
      DevicePipeline& r = *rp_;
      // on the engine's stream, behind the all-gather
      launch_merge_slots(r.d_records, nslots, slot_recs, reinterpret_cast<KeyCount*>(r.d_out),
                         r.d_ctr, r.d_out_mapped, r.d_ctr_mapped,
                         r.lb_merge((u64)nslots * slot_recs), d_headers_, m.stream);
    };
    return {key, std::move(enqueue)};
  }
  void enqueue_merge_slots(u32 nslots, u32 slot_recs) override {
    DevicePipeline& m = *mp_;
    auto half = prepare_merge_slots(nslots, slot_recs);
    if (m.graph_launches())
      m.launch_cached(half.first, half.second);
    else
      half.second();
  }

  // Device half of the header copy (non-root ranks; the root's merge copies them).
  DeviceHalf header_copy(u32 nslots, u32 slot_recs) {
    grow_headers(nslots);
    merge_copied_headers_ = false;
    return [this, nslots, slot_recs]() {
      const u64 pitch = ((u64)kSlotHeaderRecords + slot_recs) * sizeof(KeyCount);
      LOCUST_HIP_CHECK(hipMemcpy2DAsync(h_headers_, sizeof(SlotHeader), rp_->d_records, pitch,
                                        sizeof(SlotHeader), nslots, hipMemcpyDeviceToHost,
                                        mp_->stream));
    };
  }
  void enqueue_slot_headers(u32 nslots, u32 slot_recs) override {
    if (merge_copied_headers_) {  // the root's merge kernel wrote them already
      grow_headers(nslots);
      merge_copied_headers_ = false;
      return;
    }
    header_copy(nslots, slot_recs)();
  }

  bool enqueue_slot_job(const TextInput& shard, u32 slot_recs, u32 nslots, bool root,
                        const SlotAllgather& allgather) override {
    DevicePipeline& m = *mp_;
    if (!m.use_graph() || !small_ordered_ok(shard, true) || nslots > (u32)kMaxMergeRunsHost)
      return false;
    LOCUST_CHECK_ARG(slot_recs <= m.slot_records_cap(), "slot larger than the send buffer");
    SlotHeader* hdr = reinterpret_cast<SlotHeader*>(m.d_records - kSlotHeaderRecords);
    slot_fast_ = true;
    samples_valid_ = false;
    sorted_local_ = true;
    distinct_local_ = true;
    stream_chunks_ = 0;
    // host halves first (they may grow buffers: the key records the pointers)
    auto map_half = prepare_small_ordered(shard, false, hdr, slot_recs);
    void* recv = slot_buffer(nslots, slot_recs);
    std::pair<DevicePipeline::GraphKeyArr, DeviceHalf> tail;
    if (root) {
      tail = prepare_merge_slots(nslots, slot_recs);
    } else {
      tail.second = header_copy(nslots, slot_recs);
      tail.first = {7, ((u64)nslots << 32) | slot_recs, reinterpret_cast<u64>(h_headers_), 0, 0,
                    0};
    }
    merge_copied_headers_ = false;  // this job's graph already holds the header copy
    const u64 slot_bytes = ((u64)kSlotHeaderRecords + slot_recs) * sizeof(KeyCount);
    SlotJobKey key;
    std::copy(map_half.first.begin(), map_half.first.end(), key.begin());
    std::copy(tail.first.begin(), tail.first.end(), key.begin() + 6);
    key[12] = reinterpret_cast<u64>(recv);
    key[13] = (root ? 1 : 0) | (rp_gen_ << 1) | (m.layout_gen << 32) |
              ((rp_ ? rp_->layout_gen : 0) << 48);
    for (auto& g : slot_graphs_)
      if (g.key == key) {
        LOCUST_HIP_CHECK(hipGraphLaunch(g.exec, m.stream));
        return true;
      }
    // A new shape runs once without capture: the collective's first call with these
    // buffers and this size (lazy connection / buffer setup inside the communicator)
    // happens outside a capture; the next job with the same shape captures and replays.
    // After a failed capture every job runs this way (same order, same single sync).
    auto run_uncaptured = [&](bool capturing) {
      map_half.second();
      allgather(hdr, recv, slot_bytes, capturing);
      tail.second();
    };
    if (slot_capture_failed_ ||
        std::find(slot_seen_.begin(), slot_seen_.end(), key) == slot_seen_.end()) {
      if (slot_seen_.size() >= 16) slot_seen_.erase(slot_seen_.begin());
      slot_seen_.push_back(key);
      run_uncaptured(false);
      return true;
    }
    if (slot_graphs_.size() >= 4) {
      LOCUST_HIP_CHECK(hipGraphExecDestroy(slot_graphs_.front().exec));
      slot_graphs_.erase(slot_graphs_.begin());
    }
    // Nothing captured has run, so a capture the runtime or the communicator refuses is
    // not a job failure: discard it and run the same work uncaptured.
    hipGraph_t g = nullptr;
    hipGraphExec_t exec = nullptr;
    std::string why;
    if (hipStreamBeginCapture(m.stream, hipStreamCaptureModeRelaxed) != hipSuccess) {
      why = "begin capture";
    } else {
      try {
        // test hooks: LOCUST_FAULT=<rank>:slot_capture fails the capture before anything
        // is recorded, <rank>:slot_capture_late after the all-gather was recorded (the
        // work then runs uncaptured: the recorded collective never ran)
        if (fault_injected(log_rank(), "slot_capture"))
          throw Error("injected fault (LOCUST_FAULT) in the slot job capture");
        run_uncaptured(true);  // recorded, not run
        if (fault_injected(log_rank(), "slot_capture_late"))
          throw Error("injected fault (LOCUST_FAULT) late in the slot job capture");
      } catch (const std::exception& e) {
        why = e.what();
      }
      const hipError_t ec = hipStreamEndCapture(m.stream, &g);
      if (why.empty() && ec != hipSuccess) why = hipGetErrorString(ec);
      if (why.empty() && hipGraphInstantiate(&exec, g, nullptr, nullptr, 0) != hipSuccess)
        why = "instantiate";
      if (g) (void)hipGraphDestroy(g);
    }
    if (!why.empty()) {
      (void)hipGetLastError();
      if (exec) (void)hipGraphExecDestroy(exec);
      slot_capture_failed_ = true;
      std::fprintf(stderr, "locust: slot job capture failed (%s); running it uncaptured\n",
                   why.c_str());
      run_uncaptured(false);
      return true;
    }
    slot_graphs_.push_back({key, exec});
    LOCUST_HIP_CHECK(hipGraphLaunch(exec, m.stream));
    return true;
  }
  const SlotHeader* slot_headers() const override { return h_headers_; }

  // ---- device-resident shuffle (locust/exch.hpp) ----
  // ---- one-sync shuffle: the map runs inside the exchange's enqueue ----
  // Small ordered passes (one kernel writes the sorted records) and large piecewise passes
  // (map + per-piece partials + merge) leave everything the exchange reads on the device.
  bool exch_map_async_ok(const TextInput& shard) const override {
    const DevicePipeline& m = *mp_;
    if (cfg_.sort_path != SortPath::kDict || cfg_.map_path != MapPath::kFast) return false;
    if (shard.bytes > m.pass_bytes || shard.num_lines > m.cap_lines) return false;
    if (small_ordered_ok(shard, true)) return true;
    return m.large_ordered && m.cap > kPartBuildMaxTokens && m.table_tiles(shard.bytes) > 0;
  }
  // Enqueues this rank's map (the sorted distinct records end in d_records / sorted keys)
  // and its S samples into the exchange's all-gather send slot.
  void exch_map_enqueue(const TextInput& shard, u32 P, u32 S) override {
    ensure_exch_ctl(P, S);
    async_combined_ = enqueue_async_map(shard);
    // the samples go out with the header (enqueue_msg1_plan): one launch for both
  }
  // Returns whether the token count is the combining map's (map_tokens).
  bool enqueue_async_map(const TextInput& shard) {
    DevicePipeline& m = *mp_;
    stream_chunks_ = 0;
    sorted_local_ = distinct_local_ = true;
    async_small_ = small_ordered_ok(shard, true);
    if (async_small_) {
      enqueue_small_ordered(shard, /*spec_samples=*/false, nullptr, 0);
      return false;
    }
    m.check_input(shard);
    m.combine_map = true;
    m.enqueue_upload(shard);
    m.enqueue_map(shard);
    m.combine_map = false;
    LOCUST_CHECK_ARG(m.large_ordered_ok(), "asynchronous map: no partition table for this pass");
    m.sync_clean = false;
    m.enqueue_partials();
    OrderedExtra ex;
    ex.pm = m.part_map();
    ex.part_w = m.d_pw;
    ex.recs = m.d_records;
    ex.sorted = m.sorted;
    ex.counts = m.d_sorted_counts;
    launch_dict_ordered_partials(m.d_partials, m.d_partial_n, m.partial_nslots, m.d_ctr, nullptr,
                                 m.d_ctr_mapped, m.lb_dict, m.stream, nullptr, ex);
    set_local(m.sorted, m.d_sorted_counts, &m.d_ctr->num_unique);
    return m.map_combined;
  }
  u64 exch_map_complete(const TextInput& shard) override {
    DevicePipeline& m = *mp_;
    *m.h_ctr = *m.h_ctr_mapped;
    LOCUST_CHECK_ARG(!(m.h_ctr->flags & kCtrDictOverflow), "asynchronous map needs a redo");
    if (async_small_) m.sync_clean = true;  // the ordered kernel re-zeroed its scratch
    samples_valid_ = false;  // the samples went to the device only
    m.maybe_retune_records(m.d_records, m.h_ctr->num_unique);
    return finish_map_stats(shard, m.h_ctr->num_unique);
  }

  // This rank's ExchMsg1 (+ samples) -> C1 -> plan.  slot_limit: the fixed slot pitch of
  // the one-sync schedule (larger buckets are flagged), ~0u for the sized one.
  void enqueue_msg1_plan(const ExchMsg1& h, const std::vector<PackedKey>& samples, u32 P,
                         u32 slot_limit, const ExchCollectives& coll, const TextInput* map_shard) {
    DevicePipeline& m = *mp_;
    const u32 S = (u32)samples.size();
    const u64 mb = exch_msg1_bytes(S);
    if (map_shard) {
      // exch_map_enqueue ran the map and wrote the samples; the header from the counters
      // (from the ordered kernel's counter snapshot: a small pass re-zeroes d_ctr itself)
      launch_exch_header(m.d_ctr_mapped, h, async_combined_,
                         reinterpret_cast<ExchMsg1*>(xb_.msg1_send), m.stream, local_keys_,
                         local_n_, S);
    } else {
      std::memcpy(xb_.h_msg1, &h, sizeof(ExchMsg1));
      if (S) std::memcpy(xb_.h_msg1 + sizeof(ExchMsg1), samples.data(), (u64)S * sizeof(PackedKey));
      LOCUST_HIP_CHECK(hipMemcpyAsync(xb_.msg1_send, xb_.h_msg1, mb, hipMemcpyHostToDevice, m.stream));
    }
    coll.allgather(xb_.msg1_send, xb_.msg1_all, mb);
    // a failed map has no valid records: the planner sees the status and every rank's
    // kernels turn into no-ops, but the collectives still run
    launch_exch_plan(xb_.msg1_all, P, S, local_keys(), exch_n(h), slot_limit, xb_.ctl, m.stream,
                     exch_trace());
  }
  const u32* exch_n(const ExchMsg1& h) const { return h.status ? xb_.zero_n : local_n(); }

  // merge -> report -> C3 -> emit -> the headers and reports to the host.  region: the
  // shared output region, or kExchNoRegion to take the root's from its all-gathered header.
  // The merge counts its range (n_out, tokens) without emitting it; the report and C3 then
  // give every rank its offset, and ONE emit writes the range from the merge slots straight
  // into the shared host output as compact records (no device range buffer, no second pass
  // over it).
  void enqueue_range_tail(u32 P, int me, u32 C, u32 G, u64 region, const ExchCollectives& coll) {
    DevicePipeline& m = *mp_;
    launch_merge_rank_slots(reinterpret_cast<const KeyCount*>(xb_.a2a_recv), P, C, xb_.merged,
                            xb_.acc, LookbackScratch{xb_.lb_status, xb_.lb_tile}, m.stream);
    launch_exch_report(xb_.a2a_recv, P, C, xb_.ctl, xb_.acc, G, xb_.msg3_send, m.stream);
    coll.allgather(xb_.msg3_send, xb_.msg3_all, sizeof(ExchMsg3));
    enqueue_emit(P, me, G, region);
    LOCUST_HIP_CHECK(hipMemcpy2DAsync(xb_.h_hdrs, sizeof(ExchMsg1), xb_.msg1_all,
                                      exch_msg1_bytes(xb_.S_job), sizeof(ExchMsg1), P,
                                      hipMemcpyDeviceToHost, m.stream));
    LOCUST_HIP_CHECK(hipMemcpyAsync(xb_.h_msg3, xb_.msg3_all, (u64)P * sizeof(ExchMsg3),
                                    hipMemcpyDeviceToHost, m.stream));
  }
  void enqueue_emit(u32 P, int me, u32 G, u64 region) {
    ++out_seq_;
    launch_merge_emit_compact(reinterpret_cast<const KeyCount*>(xb_.a2a_recv), P, xb_.C,
                              xb_.merged, xb_.msg3_all,
                              region == kExchNoRegion
                                  ? reinterpret_cast<const ExchMsg1*>(xb_.msg1_all)
                                  : nullptr,
                              region, out_->regions, out_->region_records, P, (u32)me, G,
                              reinterpret_cast<u64*>(out_->d_records), out_->d_stamps, out_seq_,
                              xb_.done, LookbackScratch{xb_.lb_status, xb_.lb_tile}, mp_->stream);
  }

  void enqueue_exchange(const ExchMsg1& hdr, const std::vector<PackedKey>& samples, u32 P,
                        int me, const ExchCollectives& coll,
                        const TextInput* map_shard) override {
    DevicePipeline& m = *mp_;
    const u32 S = (u32)samples.size();
    const u32 C = exch_slot_records, G = exch_gather_records;
    LOCUST_CHECK_ARG(P >= 1 && P <= kExchMaxRanks && C && G, "exchange: bad shape");
    // everything that can allocate or synchronise happens before the first collective
    if (!hdr.status && !map_shard) prepare_shuffle();
    ensure_exch_ctl(P, S);
    ensure_exch_data(P, C, G);
    ensure_out((u64)P * G, 0);
    ExchMsg1 h = hdr;
    h.out_region = me == 0 ? pick_region() : 0;
    job_region_ = h.out_region;
    enqueue_msg1_plan(h, samples, P, C, coll, map_shard);
    launch_exch_pack(m.d_records, exch_n(h), m.cap, xb_.ctl, P, C, xb_.a2a_send, m.stream);
    coll.alltoall(xb_.a2a_send, xb_.a2a_recv, exch_slot_bytes(C));
    enqueue_range_tail(P, me, C, G, kExchNoRegion, coll);
  }

  void enqueue_exchange_plan(const ExchMsg1& hdr, const std::vector<PackedKey>& samples, u32 P,
                             int me, const ExchCollectives& coll,
                             const TextInput* map_shard) override {
    DevicePipeline& m = *mp_;
    const u32 S = (u32)samples.size();
    LOCUST_CHECK_ARG(P >= 1 && P <= kExchMaxRanks, "exchange: bad shape");
    if (!hdr.status && !map_shard) prepare_shuffle();
    ensure_exch_ctl(P, S);
    ExchMsg1 h = hdr;
    h.out_region = me == 0 ? pick_region() : 0;
    enqueue_msg1_plan(h, samples, P, ~0u, coll, map_shard);
    coll.allgather(xb_.ctl, xb_.ctl_all, sizeof(ExchCtl));
    LOCUST_HIP_CHECK(hipMemcpy2DAsync(xb_.h_hdrs, sizeof(ExchMsg1), xb_.msg1_all,
                                      exch_msg1_bytes(S), sizeof(ExchMsg1), P,
                                      hipMemcpyDeviceToHost, m.stream));
    LOCUST_HIP_CHECK(hipMemcpyAsync(xb_.h_ctl_all, xb_.ctl_all, (u64)P * sizeof(ExchCtl),
                                    hipMemcpyDeviceToHost, m.stream));
  }
  const ExchCtl* exch_plans() const override { return xb_.h_ctl_all; }

  void enqueue_exchange_sized(u32 P, int me, const ExchCollectives& coll, bool to_root) override {
    DevicePipeline& m = *mp_;
    ExchCtl* pl = xb_.h_ctl_all;
    const ExchMsg1* H = xb_.h_hdrs;
    LOCUST_CHECK_ARG(P == xb_.P, "sized exchange: plan of another shape");
    if (to_root) {
      // the gather strategy: every rank's records form one bucket, the root's
      for (u32 p = 0; p < P; ++p) {
        const u64 n = pl[p].off[P];
        for (u32 d = 1; d <= P; ++d) pl[p].off[d] = n;
        pl[p].max_bucket = n;
      }
      LOCUST_HIP_CHECK(hipMemcpyAsync(xb_.ctl, pl + me, sizeof(ExchCtl), hipMemcpyHostToDevice,
                                      m.stream));
    }
    // the count matrix: rank p sends cnt(p, d) records to rank d
    auto cnt = [&](u32 p, u32 d) { return pl[p].off[d + 1] - pl[p].off[d]; };
    u64 C = 1, G = 1, total = 0;
    std::vector<u64> recv(P, 0);
    for (u32 p = 0; p < P; ++p)
      for (u32 d = 0; d < P; ++d) {
        const u64 c = cnt(p, d);
        C = std::max(C, c);
        recv[d] += c;
        total += c;
      }
    for (u32 d = 0; d < P; ++d) G = std::max(G, recv[d]);
    LOCUST_CHECK_ARG(C < (1ull << 31) && G < (1ull << 31), "sized exchange: buckets too large");
    ensure_exch_data(P, (u32)C, (u32)G);
    // the root's region, or region 0 of a grown output (every rank decides the same)
    const bool none = H[0].out_region == kExchNoRegion;
    const bool fresh = ensure_out(std::max<u64>(total, 1), none && out_ ? out_->regions + 1 : 0);
    job_region_ = fresh ? 0 : H[0].out_region;
    LOCUST_CHECK_ARG(job_region_ < out_->regions, "sized exchange: bad output region");
    launch_exch_pack(m.d_records, local_n(), m.cap, xb_.ctl, P, (u32)C, xb_.a2a_send, m.stream);
    // exact sizes: each slot's header + its records (the pitch stays C)
    const u64 pitch = exch_slot_bytes((u32)C);
    std::vector<u64> sb(P), so(P), rb(P), ro(P);
    for (u32 q = 0; q < P; ++q) {
      sb[q] = exch_slot_bytes((u32)cnt((u32)me, q));
      so[q] = q * pitch;
      rb[q] = exch_slot_bytes((u32)cnt(q, (u32)me));
      ro[q] = q * pitch;
    }
    exch_sent_ = sb;
    coll.alltoallv(xb_.a2a_send, sb.data(), so.data(), xb_.a2a_recv, rb.data(), ro.data());
    enqueue_range_tail(P, me, (u32)C, (u32)G, job_region_, coll);
  }
  // bytes this rank sent to each peer in the last sized exchange (accounting)
  std::vector<u64> exch_sent_;

  void enqueue_exchange_emit(u32 P, int me) override {
    ensure_out(out_->region_records, out_->regions + 1);
    job_region_ = 0;
    // the same merge emitted again: its look-back scratch and ticket from zero
    LOCUST_HIP_CHECK(hipMemsetAsync(xb_.lb_status, 0, merge_scratch_words((u64)P * xb_.C) * 8,
                                    mp_->stream));
    LOCUST_HIP_CHECK(hipMemsetAsync(xb_.lb_tile, 0, sizeof(u32), mp_->stream));
    enqueue_emit(P, me, xb_.G, 0);
  }

  // LOCUST_EXCH_TRACE=1: the plan kernel's phase stamps, printed after each exchange.
  u64* h_exch_trace_ = nullptr;  // host-mapped (leaked with the engine: diagnostics only)
  u64* exch_trace() {
    static const bool on = std::getenv("LOCUST_EXCH_TRACE") != nullptr;
    if (!on) return nullptr;
    if (!h_exch_trace_)
      LOCUST_HIP_CHECK(hipHostMalloc(&h_exch_trace_, 16 * sizeof(u64),
                                     hipHostMallocMapped | hipHostMallocCoherent));
    u64* d = nullptr;
    LOCUST_HIP_CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&d), h_exch_trace_, 0));
    return d;
  }
  void print_exch_trace() const {
    if (!h_exch_trace_) return;
    const u64* t = h_exch_trace_;
    std::fprintf(stderr, "exch_plan us: status %.2f load %.2f sort %.2f split %.2f search %.2f "
                 "out %.2f | shader clock %.0f MHz\n", (t[1] - t[0]) * 0.01,
                 (t[2] - t[1]) * 0.01, (t[3] - t[2]) * 0.01, (t[4] - t[3]) * 0.01,
                 (t[5] - t[4]) * 0.01, (t[6] - t[5]) * 0.01,
                 t[6] > t[0] ? (double)(t[8] - t[7]) / ((t[6] - t[0]) * 0.01) : 0.0);
  }
  const ExchMsg1* exch_headers() const override {
    print_exch_trace();
    return xb_.h_hdrs;
  }
  const ExchMsg3* exch_reports() const override { return xb_.h_msg3; }

  void exch_finish_root(u32 P, u64* total_count, u64* num_unique) override {
    const ExchMsg3* R = xb_.h_msg3;
    const u64 G = xb_.G;
    u64 n = 0, t = 0;
    for (u32 p = 0; p < P; ++p) {
      n += std::min<u64>(R[p].n_out, G);
      t += R[p].total;
    }
    LOCUST_CHECK_ARG(n <= out_->region_records, "shared output: range larger than its region");
    // every rank's range landed when its stamp says this job (its emit fenced its writes
    // at system scope before the stamp's release store)
    const u64* stamps = out_->stamps();
    const u64 deadline = now_ns() + (u64)(out_wait_s() * 1e9);
    for (u32 p = 0; p < P; ++p) {
      u64 spins = 0;
      while (__atomic_load_n(stamps + p, __ATOMIC_ACQUIRE) != out_seq_) {
        if (now_ns() > deadline)
          throw Error("shared output: rank " + std::to_string(p) + " did not finish writing its "
                      "key range within " + std::to_string(out_wait_s()) + " s");
        if (++spins > 64) std::this_thread::yield();
      }
    }
    // rank p's compact segment starts at word kOutWords x (region start + lower ranks' n_out)
    std::vector<EntrySegment> segs;
    const u64* words = reinterpret_cast<const u64*>(out_->records());
    u64 at = job_region_ * out_->region_records;
    for (u32 p = 0; p < P; ++p) {
      const u64 np = std::min<u64>(R[p].n_out, G);
      if (np) segs.push_back({words + (u64)kOutWords * at, np});
      at += np;
    }
    range_entries_.adopt_compact(leases_[job_region_], std::move(segs), n);
    *total_count = t;
    *num_unique = n;
  }
  static double out_wait_s() {
    static const double s = [] {
      const char* e = std::getenv("LOCUST_OUT_WAIT_S");
      return e ? std::atof(e) : 120.0;
    }();
    return s;
  }
  void exch_job_done() override {
    if (out_) out_->seg.unlink();
  }

  u64 complete_map_slot(const TextInput& shard) override {
    if (!slot_fast_) return local_count_;  // mapped synchronously (or failed) already
    return complete_small_ordered(shard);
  }

  void finish_merge_slots(u64* total_count, u64* num_unique) override {
    DevicePipeline& r = *rp_;
    *r.h_ctr = *r.h_ctr_mapped;
    WordCountResult tmp;
    r.fill_counters(tmp);
    r.copy_out(tmp.entries, r.h_ctr->num_unique);
    *total_count = r.h_ctr->total_count;
    *num_unique = r.h_ctr->num_unique;
    range_entries_ = std::move(tmp.entries);
  }

  // Shuffle after a gather-planned map: sort the dictionary's keys, repack, resample.
  void prepare_shuffle() override {
    if (sorted_local_) return;
    DevicePipeline& m = *mp_;
    m.sync_clean = false;
    if (m.h_ctr->num_unique <= (u32)kRankSortMax) {
      m.enqueue_rank();  // ranks are zero: reset with the table / written by the build
      m.enqueue_sorted_from_dict();
    } else {
      radix_sort(m.dict.ukeys, &m.d_ctr->num_unique, m.h_ctr->num_unique, m.rx, m.dict.ucount,
                 m.sorted, m.d_sorted_counts, m.d_perm, m.h_plan, m.stream);
    }
    set_local(m.sorted, m.d_sorted_counts, &m.d_ctr->num_unique);
    launch_pack_records(local_keys_, local_counts_, local_n_, m.cap, m.d_records, m.stream);
    m.sync();
    sorted_local_ = true;
  }

  std::vector<PackedKey> sample(u32 s) override {
    DevicePipeline& m = *mp_;
    prepare_shuffle();
    if (samples_valid_ && s == kSpecSamples) return samples_;
    LOCUST_CHECK_ARG(s <= kMaxSamples, "too many samples");
    launch_sample_keys(local_keys(), local_n(), s, m.d_samples, m.stream);
    LOCUST_HIP_CHECK(hipMemcpyAsync(m.h_small, m.d_samples, s * sizeof(PackedKey),
                                    hipMemcpyDeviceToHost, m.stream));
    m.sync();
    return std::vector<PackedKey>(m.h_small, m.h_small + s);
  }

  std::vector<u64> bucket_offsets(const std::vector<PackedKey>& splitters) override {
    DevicePipeline& m = *mp_;
    const u32 P = (u32)splitters.size() + 1;
    LOCUST_CHECK_ARG(P <= kMaxRanks, "too many ranks");
    prepare_shuffle();
    if (!splitters.empty()) {
      std::memcpy(m.h_small, splitters.data(), splitters.size() * sizeof(PackedKey));
      LOCUST_HIP_CHECK(hipMemcpyAsync(m.d_splitters, m.h_small,
                                      splitters.size() * sizeof(PackedKey), hipMemcpyHostToDevice,
                                      m.stream));
    }
    launch_bucket_offsets(local_keys(), local_n(), m.d_splitters, P, m.d_offsets, m.stream);
    LOCUST_HIP_CHECK(hipMemcpyAsync(m.h_u64, m.d_offsets, (P + 1) * sizeof(u64),
                                    hipMemcpyDeviceToHost, m.stream));
    m.sync();
    return std::vector<u64>(m.h_u64, m.h_u64 + P + 1);
  }

  const void* send_records() override { return mp_->d_records; }

  void* recv_records(u64 n) override {
    if (!rp_ || rp_->cap < n) {
      const u64 want = std::max<u64>(std::max<u64>(n + n / 4, 4096), rp_ ? rp_->cap * 2 : 0);
      if (rp_) (void)hipStreamSynchronize(mp_->stream);  // graphs may still read rp_
      rp_.reset();
      rp_.reset(new DevicePipeline(cfg_, 1, 1, want));
      ++rp_gen_;  // graphs keyed on the old rp_ can never match again
      for (auto& g : slot_graphs_) (void)hipGraphExecDestroy(g.exec);
      slot_graphs_.clear();
      slot_seen_.clear();
    }
    return rp_->d_records;
  }

  void reduce_received_runs(const std::vector<u64>& run_lens, u64 total_tokens, u32 run_flags,
                            u64* total_count, u64* num_unique) override {
    u64 n = 0;
    for (u64 l : run_lens) n += l;
    const bool mergeable = (run_flags & kRecordsSorted) && (run_flags & kRecordsDistinct) &&
                           run_lens.size() <= (size_t)kMaxMergeRunsHost && n &&
                           n <= kMergeMaxRecords && total_tokens <= kMergeMaxCount;
    if (!mergeable) return reduce_received(n, total_count, num_unique);
    // The shuffle delivered one sorted slice of distinct keys per rank, back to back in
    // rank order: merge them (binary-search positions + one look-back scan) straight
    // into host-mapped output -- no dictionary rebuild, no sort.
    DevicePipeline& r = *rp_;
    r.select_out();
    r.grow_host_out(n);
    u32* meta = reinterpret_cast<u32*>(r.h_u64);  // pinned; read by the copy below
    meta[0] = (u32)run_lens.size();
    for (size_t q = 0; q < run_lens.size(); ++q) meta[1 + q] = (u32)run_lens[q];
    u32* d_meta = reinterpret_cast<u32*>(r.d_offsets);
    LOCUST_HIP_CHECK(hipMemcpyAsync(d_meta, meta, (1 + run_lens.size()) * sizeof(u32),
                                    hipMemcpyHostToDevice, r.stream));
    launch_merge_sorted_runs(r.d_records, r.d_records + run_lens[0], d_meta, n,
                             reinterpret_cast<KeyCount*>(r.d_out), r.d_ctr, r.d_out_mapped,
                             r.d_ctr_mapped, r.lb_merge(n), r.stream);
    r.sync();
    *r.h_ctr = *r.h_ctr_mapped;
    WordCountResult tmp;
    r.fill_counters(tmp);
    r.copy_out(tmp.entries, r.h_ctr->num_unique);
    *total_count = r.h_ctr->total_count;
    *num_unique = r.h_ctr->num_unique;
    range_entries_ = std::move(tmp.entries);
  }

  void reduce_received(u64 n, u64* total_count, u64* num_unique) override {
    DevicePipeline& r = *rp_;
    r.select_out();  // the previous job's entries may still hold the last output buffer
    // The all-to-all finished on mp_'s stream (blocking), so rp_'s stream may start.
    r.set_num_records(n);
    launch_unpack_records(r.d_records, n, r.tokens, r.d_counts, r.d_parts, r.stream,
                          r.part_map());
    r.parts_ready = true;
    r.part_tiles = 0;  // tokens from records: partition tags only
    WordCountResult tmp;
    bool downloaded = false;
    if (cfg_.sort_path == SortPath::kDict) {
      const bool ordered = r.enqueue_dict_job(0, false, true, nullptr);
      r.sync();
      *r.h_ctr = *r.h_ctr_mapped;
      const bool ordered_done = ordered && !(r.h_ctr->flags & kCtrDictOverflow);
      if (ordered && !ordered_done) r.redo_dict_on_table(0, true);
      if (!ordered_done && r.dict_fallback_needed()) {
        r.finish_dict_with_radix(0, true);
      } else {
        r.fill_counters(tmp);
        r.copy_out(tmp.entries, r.h_ctr->num_unique);
        downloaded = true;
      }
    } else {
      r.enqueue_process(0, false, true, n);
      r.enqueue_reduce_core(true);
      r.enqueue_pack_output();
    }
    if (!downloaded) r.download_output(tmp, nullptr);
    *total_count = r.h_ctr->total_count;
    *num_unique = r.h_ctr->num_unique;
    range_entries_ = std::move(tmp.entries);
  }

  // The root's own combined records go behind the received ones; one dictionary pass over
  // all of them (partition tags come from the unpack) yields the merged, ranked output.
  u32 record_flags() const override {
    return (sorted_local_ ? kRecordsSorted : 0u) | (distinct_local_ ? kRecordsDistinct : 0u);
  }

  void reduce_gathered(const std::vector<u64>& run_lens, u64 total_tokens, u32 run_flags,
                       u64* total_count, u64* num_unique) override {
    DevicePipeline& m = *mp_;
    DevicePipeline& r = *rp_;  // recv_records() created it; holds the other ranks' records
    r.select_out();
    u64 n_other = 0;
    for (u64 l : run_lens) n_other += l;
    LOCUST_CHECK_ARG(n_other + local_count_ <= r.cap, "gather buffer too small");
    const int nruns = (int)run_lens.size() + 1;
    const u64 n_all = n_other + local_count_;
    const bool runs_sorted = (run_flags & kRecordsSorted) && sorted_local_;
    if (runs_sorted && (run_flags & kRecordsDistinct) && nruns <= kMaxMergeRunsHost &&
        n_all <= kMergeMaxRecords && total_tokens <= kMergeMaxCount) {
      // Every run is sorted with distinct keys: merge by binary search (position in the
      // merged order, first copy of each key sums the others) + one look-back scan that
      // writes the final records into host-mapped memory -- two kernels, one graph.
      u32* meta = reinterpret_cast<u32*>(r.h_u64);  // pinned; read at replay time
      meta[0] = (u32)nruns;
      meta[1] = (u32)local_count_;
      for (int q = 1; q < nruns; ++q) meta[1 + q] = (u32)run_lens[(size_t)q - 1];
      u32* d_meta = reinterpret_cast<u32*>(r.d_offsets);
      KeyCount* merged = reinterpret_cast<KeyCount*>(r.d_out);  // >= cap records of scratch
      r.grow_host_out(n_all);
      auto enqueue = [&] {
        LOCUST_HIP_CHECK(hipMemcpyAsync(d_meta, meta, (1 + (u64)nruns) * sizeof(u32),
                                        hipMemcpyHostToDevice, r.stream));
        launch_merge_sorted_runs(m.d_records, r.d_records, d_meta, r.cap, merged, r.d_ctr,
                                 r.d_out_mapped, r.d_ctr_mapped, r.lb_merge(r.cap), r.stream);
      };
      if (r.graph_launches())
        r.launch_cached({5 | (rp_gen_ << 8), (u64)nruns, reinterpret_cast<u64>(m.d_records),
                         reinterpret_cast<u64>(r.d_records),
                         reinterpret_cast<u64>(r.d_out_mapped), 0},
                        enqueue);
      else
        enqueue();
      r.sync();
      *r.h_ctr = *r.h_ctr_mapped;
      WordCountResult tmp;
      r.fill_counters(tmp);
      r.copy_out(tmp.entries, r.h_ctr->num_unique);
      *total_count = r.h_ctr->total_count;
      *num_unique = r.h_ctr->num_unique;
      range_entries_ = std::move(tmp.entries);
      return;
    }
    if (cfg_.sort_path == SortPath::kDict && runs_sorted && nruns <= kMaxMergeRunsHost &&
        n_all <= kPartBuildMaxTokens) {
      // Sorted runs that may repeat a key (no map-side combine): the ordered dictionary
      // kernel finds each partition's range in every run by binary search and aggregates
      // it in LDS -- one kernel (plus the counter reset and the run table), one graph.
      u32* meta = reinterpret_cast<u32*>(r.h_u64);  // pinned; read at replay time
      meta[0] = (u32)nruns;
      meta[1] = (u32)local_count_;
      for (int q = 1; q < nruns; ++q) meta[1 + q] = (u32)run_lens[(size_t)q - 1];
      u32* d_meta = reinterpret_cast<u32*>(r.d_offsets);
      auto enqueue = [&] {
        LOCUST_HIP_CHECK(hipMemsetAsync(r.d_sync, 0, r.sync_bytes, r.stream));
        LOCUST_HIP_CHECK(hipMemcpyAsync(d_meta, meta, (1 + (u64)nruns) * sizeof(u32),
                                        hipMemcpyHostToDevice, r.stream));
        launch_dict_merge_runs(m.d_records, r.d_records, d_meta, r.d_ctr, r.d_out_mapped,
                               r.d_ctr_mapped, r.lb_dict, r.stream, r.part_map());
      };
      if (r.graph_launches())
        r.launch_cached({4 | (rp_gen_ << 8), (u64)nruns, reinterpret_cast<u64>(m.d_records),
                         reinterpret_cast<u64>(r.d_records), 0, 0},
                        enqueue);
      else
        enqueue();
      r.sync();
      *r.h_ctr = *r.h_ctr_mapped;
      if (!(r.h_ctr->flags & kCtrDictOverflow)) {
        WordCountResult tmp;
        r.fill_counters(tmp);
        r.copy_out(tmp.entries, r.h_ctr->num_unique);
        *total_count = r.h_ctr->total_count;
        *num_unique = r.h_ctr->num_unique;
        range_entries_ = std::move(tmp.entries);
        return;
      }
      // a partition overflowed its LDS table: the general path below redoes the merge
    }
    // General path: this rank's records behind the received ones, then the usual reduce.
    if (local_count_)
      LOCUST_HIP_CHECK(hipMemcpyAsync(r.d_records + n_other, m.d_records,
                                      local_count_ * sizeof(KeyCount), hipMemcpyDeviceToDevice,
                                      m.stream));
    m.sync();
    reduce_received(n_other + local_count_, total_count, num_unique);
  }

  void finalize(EntryList* out) override { *out = std::move(range_entries_); }

  void map_stats(WordCountResult* r) override { *r = local_stats_; }

 private:
  u64 finish_map_stats(const TextInput& shard, u64 n_records) {
    DevicePipeline& m = *mp_;
    local_stats_ = WordCountResult();
    local_stats_.num_lines = shard.lines();
    m.fill_counters(local_stats_);
    local_stats_.num_tokens = m.map_combined ? m.h_ctr->map_tokens : m.h_ctr->num_records;
    if (stream_chunks_) m.stream_stats(stream_chunks_, local_stats_);
    local_count_ = n_records;
    return n_records;
  }
  // Dictionary table overflow: sort every token and combine the reference way.
  u64 map_overflow_fallback(const TextInput& shard) {
    DevicePipeline& m = *mp_;
    if (stream_chunks_)
      throw Error("streaming dictionary overflow: more than " + std::to_string(m.ucap) +
                  " distinct keys in one shard; use a larger chunk size");
    m.enqueue_process(0, false, false, m.h_ctr->num_records);
    m.enqueue_reduce_core(false);
    set_local(m.heads, m.d_head_count, &m.d_ctr->num_unique);
    launch_pack_records(local_keys_, local_counts_, local_n_, m.cap, m.d_records, m.stream);
    m.read_counters();
    return finish_map_stats(shard, m.h_ctr->num_unique);
  }
  void set_local(ConstKeysSoA k, const u64* c, const u32* n) {
    local_keys_ = k;
    local_counts_ = c;
    local_n_ = n;
  }
  ConstKeysSoA local_keys() const { return local_keys_; }
  const u32* local_n() const { return local_n_; }

  JobConfig cfg_;
  std::unique_ptr<DevicePipeline> mp_, rp_;
  u64 rp_gen_ = 0;  // bumped whenever rp_ is reallocated (graph keys)
  static constexpr u32 kSpecSamples = 64;  // DistConfig::samples_per_rank default
  ConstKeysSoA local_keys_{};
  bool async_small_ = false;     // the last asynchronous map was a small ordered pass
  bool async_combined_ = false;  // ... and its token count is the combining map's
  std::vector<PackedKey> samples_;
  bool samples_valid_ = false;
  EntryList range_entries_;
  const u64* local_counts_ = nullptr;
  const u32* local_n_ = nullptr;
  WordCountResult local_stats_;
  u64 local_count_ = 0;
  size_t stream_chunks_ = 0;  // > 0: the last shard streamed through in this many chunks
  bool sorted_local_ = true;  // d_records are sorted (shuffle-ready)
  bool distinct_local_ = true;  // d_records hold every key once (map-side combine)
  bool spec_samples_ = false;   // the last small pass produced splitter samples
  bool slot_fast_ = false;      // enqueue_map_slot took the one-graph small pass
  // whole-job graphs of enqueue_slot_job, keyed by [map half | tail half | recv | root]
  using SlotJobKey = std::array<u64, 14>;
  struct SlotJobGraph {
    SlotJobKey key;
    hipGraphExec_t exec;
  };
  std::vector<SlotJobGraph> slot_graphs_;
  std::vector<SlotJobKey> slot_seen_;  // shapes run once uncaptured (see enqueue_slot_job)
  bool slot_capture_failed_ = false;   // a capture was refused: slot jobs stay uncaptured
  SlotHeader* h_headers_ = nullptr;  // host-mapped copies of the all-gathered slot headers
  SlotHeader* d_headers_ = nullptr;  // device view of h_headers_
  u32 h_headers_cap_ = 0;
  bool merge_copied_headers_ = false;  // this job's merge kernel copies the headers
  void grow_headers(u32 nslots) {
    if (h_headers_cap_ >= nslots) return;
    if (h_headers_) {
      LOCUST_HIP_CHECK(hipStreamSynchronize(mp_->stream));
      LOCUST_HIP_CHECK(hipHostFree(h_headers_));
    }
    h_headers_cap_ = std::max<u32>(nslots, 64);
    LOCUST_HIP_CHECK(hipHostMalloc(&h_headers_, h_headers_cap_ * sizeof(SlotHeader),
                                   hipHostMallocMapped | hipHostMallocCoherent));
    LOCUST_HIP_CHECK(
        hipHostGetDevicePointer(reinterpret_cast<void**>(&d_headers_), h_headers_, 0));
  }
  // Buffers of the device exchange: control (sized by P, S) and data (by P x C and G, grown
  // geometrically: the sized schedule's exact C and G change from job to job).
  struct ExchBufs {
    u32 P = 0, S = 0, S_job = 0;  // S_job: the samples of the current job's messages
    u32 C = 0, G = 0;             // the current job's slot pitch and range buffer
    u64 cap_pc = 0, cap_g = 0;    // data capacities (P x C records, G records)
    char* ctl_dev = nullptr;
    char* data_dev = nullptr;
    char* msg1_send = nullptr;
    char* msg1_all = nullptr;
    ExchCtl* ctl = nullptr;
    ExchCtl* ctl_all = nullptr;
    ExchMsg3* msg3_send = nullptr;
    ExchMsg3* msg3_all = nullptr;
    u32* zero_n = nullptr;
    u32* done = nullptr;
    u64* acc = nullptr;  // the merge's (firsts, tokens, words) accumulators (kMergeAccSpread triples)
    char* a2a_send = nullptr;
    char* a2a_recv = nullptr;
    KeyCount* merged = nullptr;
    u64* lb_status = nullptr;
    u32* lb_tile = nullptr;
    char* h_msg1 = nullptr;        // pinned staging of this rank's message
    ExchMsg1* h_hdrs = nullptr;    // pinned: every rank's header after the job
    ExchMsg3* h_msg3 = nullptr;    // pinned: every rank's report after the job
    ExchCtl* h_ctl_all = nullptr;  // pinned: every rank's plan (sized schedule, phase 1)
  } xb_;
  void free_exch() {
    if (xb_.ctl_dev) (void)hipFree(xb_.ctl_dev);
    if (xb_.data_dev) (void)hipFree(xb_.data_dev);
    for (void* p : {(void*)xb_.h_msg1, (void*)xb_.h_hdrs, (void*)xb_.h_msg3, (void*)xb_.h_ctl_all})
      if (p) (void)hipHostFree(p);
    xb_ = ExchBufs{};
  }
  void ensure_exch_ctl(u32 P, u32 S) {
    xb_.S_job = S;
    if (xb_.ctl_dev && P == xb_.P && S <= xb_.S) return;
    LOCUST_HIP_CHECK(hipStreamSynchronize(mp_->stream));  // nothing may still use the old ones
    free_exch();  // the data buffers are sized for P too
    auto al = [](u64 x) { return align_up(x, (u64)256); };
    const u64 mb = exch_msg1_bytes(S);
    u64 off = 0;
    auto take = [&](u64 bytes) { const u64 o = off; off += al(bytes); return o; };
    const u64 o_m1 = take(mb), o_m1a = take(mb * P), o_ctl = take(sizeof(ExchCtl)),
              o_cta = take(sizeof(ExchCtl) * P), o_m3 = take(sizeof(ExchMsg3)),
              o_m3a = take(sizeof(ExchMsg3) * P), o_zn = take(8), o_dn = take(8),
              o_rc = take(kMergeAccSpread * 3 * sizeof(u64));
    LOCUST_HIP_CHECK(hipMalloc(&xb_.ctl_dev, off));
    // zeroed in stream order: a null-stream hipMemset is not ordered with the engine's
    // non-blocking stream, and with four ranks sharing a GPU it landed after this job's
    // header upload now and then (a rank's header all-gathered as zeros: wrong token sum)
    LOCUST_HIP_CHECK(hipMemsetAsync(xb_.ctl_dev, 0, off, mp_->stream));
    char* b = xb_.ctl_dev;
    xb_.P = P;
    xb_.S = S;
    xb_.S_job = S;
    xb_.msg1_send = b + o_m1;
    xb_.msg1_all = b + o_m1a;
    xb_.ctl = reinterpret_cast<ExchCtl*>(b + o_ctl);
    xb_.ctl_all = reinterpret_cast<ExchCtl*>(b + o_cta);
    xb_.msg3_send = reinterpret_cast<ExchMsg3*>(b + o_m3);
    xb_.msg3_all = reinterpret_cast<ExchMsg3*>(b + o_m3a);
    xb_.zero_n = reinterpret_cast<u32*>(b + o_zn);
    xb_.done = reinterpret_cast<u32*>(b + o_dn);
    xb_.acc = reinterpret_cast<u64*>(b + o_rc);
    LOCUST_HIP_CHECK(hipHostMalloc(&xb_.h_msg1, mb, hipHostMallocDefault));
    LOCUST_HIP_CHECK(hipHostMalloc(&xb_.h_hdrs, sizeof(ExchMsg1) * P, hipHostMallocDefault));
    LOCUST_HIP_CHECK(hipHostMalloc(&xb_.h_msg3, sizeof(ExchMsg3) * P, hipHostMallocDefault));
    LOCUST_HIP_CHECK(hipHostMalloc(&xb_.h_ctl_all, sizeof(ExchCtl) * P, hipHostMallocDefault));
  }
  void ensure_exch_data(u32 P, u32 C, u32 G) {
    LOCUST_CHECK_ARG(xb_.ctl_dev && P == xb_.P, "exchange: control buffers of another shape");
    xb_.C = C;
    xb_.G = G;
    const u64 pc = (u64)P * C;
    if (xb_.data_dev && pc <= xb_.cap_pc && G <= xb_.cap_g) return;
    LOCUST_HIP_CHECK(hipStreamSynchronize(mp_->stream));
    if (xb_.data_dev) (void)hipFree(xb_.data_dev);
    xb_.cap_pc = std::max<u64>(pc, xb_.cap_pc + xb_.cap_pc / 4);
    xb_.cap_g = std::max<u64>(G, xb_.cap_g + xb_.cap_g / 4);
    auto al = [](u64 x) { return align_up(x, (u64)256); };
    // slots: a header (2 records) per rank + the records
    const u64 slots_bytes = ((u64)2 * P + xb_.cap_pc) * sizeof(KeyCount);
    u64 off = 0;
    auto take = [&](u64 bytes) { const u64 o = off; off += al(bytes); return o; };
    const u64 o_as = take(slots_bytes), o_ar = take(slots_bytes),
              o_mg = take(xb_.cap_pc * sizeof(KeyCount)),
              o_lb = take(merge_scratch_words(xb_.cap_pc) * 8 + 8), o_lt = take(8);
    LOCUST_HIP_CHECK(hipMalloc(&xb_.data_dev, off));
    LOCUST_HIP_CHECK(hipMemsetAsync(xb_.data_dev, 0, off, mp_->stream));
    char* b = xb_.data_dev;
    xb_.a2a_send = b + o_as;
    xb_.a2a_recv = b + o_ar;
    xb_.merged = reinterpret_cast<KeyCount*>(b + o_mg);
    xb_.lb_status = reinterpret_cast<u64*>(b + o_lb);
    xb_.lb_tile = reinterpret_cast<u32*>(b + o_lt);
  }

  // ---- the shared host output (locust/shm.hpp) ----
  // One generation of it: `regions` regions of `region_records` records each.  The root
  // lends a region to each result (EntryList::adopt); a region a live result still holds
  // is not written again -- with none free the output grows by one region.
  // Ranks that are processes share a POSIX shm segment each maps and registers; ranks
  // that are threads of one process (the CLI's clique, loopback rehearsals) share one
  // pinned allocation instead (hipHostMalloc Portable | Mapped: GPU writes to it ran at
  // ~48 GB/s where the registered 4 KiB shm pages gave ~35).
  // Ranks spanning NUMA nodes: the block is mapped memory whose slices are bound to their
  // ranks' nodes before the first touch (plan_rank_slices), then registered.
  struct PinnedBlock {
    char* p = nullptr;
    u64 mapped = 0;  // > 0: mmap'ed + hipHostRegister'ed (NUMA-placed), else hipHostMalloc
    ~PinnedBlock() {
      if (!p) return;
      if (mapped) {
        (void)hipHostUnregister(p);
        ::munmap(p, mapped);
      } else {
        pinned_free(p);
      }
    }
  };
  static std::shared_ptr<PinnedBlock> shared_block(const std::string& name, u64 bytes,
                                                   const std::vector<NumaSlice>& plan) {
    static std::mutex mu;
    static std::map<std::string, std::weak_ptr<PinnedBlock>> reg;
    std::lock_guard<std::mutex> lk(mu);
    for (auto it = reg.begin(); it != reg.end();)  // forget the released ones
      it = it->second.expired() ? reg.erase(it) : std::next(it);
    if (auto b = reg[name].lock()) return b;
    auto b = std::make_shared<PinnedBlock>();
    if (!plan.empty()) {
      void* p = ::mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
      if (p == MAP_FAILED) throw Error("shared output: mmap of " + std::to_string(bytes) + " B failed");
      b->p = static_cast<char*>(p);
      b->mapped = bytes;
      (void)::madvise(p, bytes, MADV_HUGEPAGE);  // fewer GPU-side translations
      (void)::madvise(p, bytes, MADV_DONTFORK);  // registered below: no copy-on-write children
      place_slices(p, plan);
      std::memset(p, 0, bytes);  // first touch: every page on its slice's node
      LOCUST_HIP_CHECK(hipHostRegister(p, bytes, hipHostRegisterMapped | hipHostRegisterPortable));
    } else {
      b->p = static_cast<char*>(pinned_alloc(
          bytes, hipHostMallocPortable | hipHostMallocMapped | hipHostMallocCoherent,
          "shared output (ranks in one process)"));
      std::memset(b->p, 0, kShmHeaderBytes);  // the stamps
    }
    reg[name] = b;
    return b;
  }
  int numa_node_ = -2;
  int numa_node() override {
    if (numa_node_ == -2) {
      char bdf[64] = {0};
      numa_node_ = hipDeviceGetPCIBusId(bdf, (int)sizeof(bdf), cfg_.device) == hipSuccess
                       ? placement_for_bdf(bdf).numa_node
                       : -1;
    }
    return numa_node_;
  }
  struct OutSegment {
    ShmSegment seg;                       // processes
    std::shared_ptr<PinnedBlock> block;   // threads of one process
    char* base = nullptr;                 // host view: [stamps | records]
    u64 region_records = 0;
    u32 regions = 0;
    bool registered = false;
    OutRecord* d_records = nullptr;  // device view of the records
    u64* d_stamps = nullptr;         // device view of the stamps
    u64* stamps() const { return reinterpret_cast<u64*>(base); }
    char* records() const { return base + kShmHeaderBytes; }
    ~OutSegment() {
      if (registered) (void)hipHostUnregister(seg.data());
    }
  };
  struct RegionLease {
    std::shared_ptr<OutSegment> seg;  // keeps the mapping alive while a result holds it
  };
  std::shared_ptr<OutSegment> out_;
  std::vector<std::shared_ptr<RegionLease>> leases_;  // root: one per region
  u64 out_group_ = 0, out_seq_ = 0, job_region_ = 0;
  // Room for `records` per region and at least `regions` regions (0: as now, out_regions
  // for a new output); returns whether a new generation was mapped.  Every rank calls it with the
  // same arguments at the same point of the job sequence.
  bool ensure_out(u64 records, u32 regions) {
    LOCUST_CHECK_ARG(exch_group != 0, "device exchange: the communicator has no group id");
    if (exch_group != out_group_) {
      out_.reset();
      leases_.clear();
      out_group_ = exch_group;
      out_seq_ = 0;
    }
    const u32 K = std::max<u32>(regions, out_ ? out_->regions : std::max<u32>(out_regions, 1u));
    if (out_ && records <= out_->region_records && K <= out_->regions) return false;
    u64 R = std::max<u64>(records, 4096);
    if (out_ && records > out_->region_records)
      R = std::max<u64>(R, out_->region_records + out_->region_records / 2);
    if (out_) R = std::max<u64>(R, out_->region_records);
    R = align_up(R, (u64)1024);
    LOCUST_HIP_CHECK(hipStreamSynchronize(mp_->stream));  // our writes into the old one
    auto o = std::make_shared<OutSegment>();
    const std::string name = shm_segment_name(out_group_, next_segment_gen(out_group_, exch_rank));
    const u64 bytes = shm_segment_bytes(R * K, sizeof(OutRecord));
    // pages on the node of the rank whose key range lands there (locust/numa.hpp)
    std::vector<NumaSlice> plan;
    if (spans_numa_nodes(exch_numa_nodes))
      plan = plan_rank_slices(kShmHeaderBytes, R * sizeof(OutRecord), K, exch_numa_nodes);
    char* d = nullptr;
    if (exch_in_process) {
      o->block = shared_block(name, bytes, plan);
      o->base = o->block->p;
      LOCUST_HIP_CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&d), o->base, 0));
    } else {
      o->seg.open(name, bytes, plan.empty() ? nullptr : &plan);
      LOCUST_HIP_CHECK(hipHostRegister(o->seg.data(), o->seg.bytes(),
                                       hipHostRegisterMapped | hipHostRegisterPortable));
      o->registered = true;
      o->base = o->seg.data();
      LOCUST_HIP_CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&d), o->seg.data(), 0));
    }
    o->d_stamps = reinterpret_cast<u64*>(d);
    o->d_records = reinterpret_cast<OutRecord*>(d + kShmHeaderBytes);
    o->region_records = R;
    o->regions = K;
    out_ = o;
    leases_.clear();
    for (u32 i = 0; i < K; ++i) leases_.push_back(std::make_shared<RegionLease>(RegionLease{o}));
    LOCUST_LOG_DEBUG("shared output %s (%s): %u regions x %llu records", name.c_str(),
                     exch_in_process ? "pinned, in-process" : "shm", K,
                     (unsigned long long)R);
    return true;
  }
  // Root: a region no live result holds (the one after the last used first), else
  // kExchNoRegion; region 0 before the output exists.
  u64 pick_region() const {
    if (!out_) return 0;
    const u32 K = out_->regions;
    for (u32 k = 1; k <= K; ++k) {
      const u32 i = (u32)((job_region_ + k) % K);
      if (leases_[i].use_count() == 1) return i;
    }
    return kExchNoRegion;
  }

  SlotHeader* h_send_header_ = nullptr;  // pinned staging for a host-written header
  SlotHeader* slot_host_header() {
    if (!h_send_header_)
      LOCUST_HIP_CHECK(hipHostMalloc(&h_send_header_, sizeof(SlotHeader), hipHostMallocDefault));
    return h_send_header_;
  }
};

}  // namespace

std::unique_ptr<ShardEngine> make_gpu_shard_engine(const JobConfig& cfg, u64 max_bytes,
                                                   u64 max_lines) {
  return std::unique_ptr<ShardEngine>(new GpuShardEngine(cfg, max_bytes, max_lines));
}

}  // namespace locust
