// Single-GPU WordCount engine (GpuWordCount): the public API over the device pipeline
// (csrc/engine/pipeline.hpp).
#include "pipeline.hpp"
#include "locust/stage.hpp"

namespace locust {

using detail::DevicePipeline;

// =====================================================================================
// GpuWordCount
// =====================================================================================
struct GpuWordCount::Impl : DevicePipeline {
  using DevicePipeline::DevicePipeline;
};

GpuWordCount::GpuWordCount(const JobConfig& cfg, u64 max_text_bytes, u64 max_lines)
    : impl_(new Impl(cfg, max_text_bytes, max_lines)) {
  impl_->warm_first_job();
}
GpuWordCount::~GpuWordCount() = default;

const JobConfig& GpuWordCount::config() const { return impl_->cfg; }
u64 GpuWordCount::token_capacity() const { return impl_->cap; }
char* GpuWordCount::input_buffer() { return impl_->ensure_h_text(); }
u64 GpuWordCount::text_capacity() const { return impl_->cap_bytes; }

WordCountResult GpuWordCount::run(const TextInput& in) { return impl_->run(in); }
WordCountResult GpuWordCount::run_source(TextSource& src) {
  LOCUST_CHECK_ARG(impl_->streaming, "run_source needs a streaming engine (chunk_bytes set)");
  return impl_->run_source(src);
}
GpuWordCount::Stats GpuWordCount::stats() const {
  Stats s;
  s.retunes = impl_->pm_retunes;
  s.fallbacks = impl_->fallbacks;
  s.planned_passes = impl_->planned_passes;
  s.devplan_failed = impl_->devplan_failed;
  s.device_bytes = impl_->device_bytes();
  s.hbm_free = impl_->hbm_free;
  s.hbm_total = impl_->hbm_total;
  s.streaming = impl_->streaming;
  s.chunk_bytes = impl_->cap_bytes;
  s.map_window = impl_->map_window;
  return s;
}

bool GpuWordCount::partition_map(std::vector<u64>* lo) {
  Impl& m = *impl_;
  if (m.retune_pending) {  // the last job's retune: let it finish and adopt it
    m.retune_worker.wait_idle();
    m.poll_retune();
  }
  lo->assign(m.h_pmap->lo, m.h_pmap->lo + kDictParts + 1);
  return m.pm_retunes > 0;
}

bool GpuWordCount::set_partition_map(const std::vector<u64>& lo) {
  Impl& m = *impl_;
  if (lo.size() != (size_t)kDictParts + 1 || lo[0] != 0) return false;
  for (size_t i = 1; i < lo.size(); ++i)
    if (lo[i] < lo[i - 1]) return false;
  PartMapTables t;
  for (size_t i = 0; i < lo.size(); ++i) t.lo[i] = lo[i];
  t.lo[kDictParts] = ~0ull;
  m.sync();  // no job may still read the old tables (they are uploaded in stream order anyway)
  m.upload_pmap(t, 0);
  ++m.pm_retunes;  // a tuned map: no in-job plan (decide_plan), retunes only on imbalance
  if (m.large_ordered) m.pm_tuned = true;  // (large passes: no device plan either)
  return true;
}

std::vector<PackedKey> GpuWordCount::run_map_stage(const TextInput& in, WordCountResult* stats) {
  Impl& m = *impl_;
  m.sync_clean = false;  // this entry point dirties d_sync
  m.check_input(in);
  const u64 t0 = now_ns();
  LOCUST_HIP_CHECK(hipEventRecord(m.ev[0], m.stream));
  m.enqueue_upload(in);
  LOCUST_HIP_CHECK(hipEventRecord(m.ev[1], m.stream));
  m.enqueue_map(in);
  LOCUST_HIP_CHECK(hipEventRecord(m.ev[2], m.stream));
  m.enqueue_process((u32)in.num_lines, m.cfg.map_path == MapPath::kCompat, false, kUnknownCount,
                    /*allow_psort=*/true);
  LOCUST_HIP_CHECK(hipEventRecord(m.ev[3], m.stream));
  m.read_counters();
  StageTimes tm;
  tm.h2d_ms = DevicePipeline::ms_between(m.ev[0], m.ev[1]);
  tm.map_ms = DevicePipeline::ms_between(m.ev[1], m.ev[2]);
  tm.process_ms = DevicePipeline::ms_between(m.ev[2], m.ev[3]);
  if (m.h_ctr->flags & kCtrSortOverflow) {  // a partition outgrew the LDS sort
    LOCUST_HIP_CHECK(hipEventRecord(m.ev[2], m.stream));
    m.redo_process_general((u32)in.num_lines);
    LOCUST_HIP_CHECK(hipEventRecord(m.ev[3], m.stream));
    m.read_counters();
    tm.process_ms = DevicePipeline::ms_between(m.ev[2], m.ev[3]);
  }
  std::vector<PackedKey> out;
  m.download_keys(m.sorted, m.h_ctr->num_records, &out);
  tm.wall_ms = (now_ns() - t0) * 1e-6;
  if (stats) {
    stats->num_lines = in.num_lines;
    m.fill_counters(*stats);
    stats->times = tm;
  }
  return out;
}

WordCountResult GpuWordCount::run_reduce_stage(const PackedKey* keys, u64 n) {
  Impl& m = *impl_;
  m.sync_clean = false;  // this entry point dirties d_sync
  WordCountResult r;
  const u64 t0 = now_ns();
  LOCUST_HIP_CHECK(hipEventRecord(m.ev[0], m.stream));
  m.upload_tokens(keys, n);
  LOCUST_HIP_CHECK(hipEventRecord(m.ev[1], m.stream));
  LOCUST_HIP_CHECK(hipEventRecord(m.ev[2], m.stream));
  m.enqueue_process(0, false, false, n);  // B7 fix: the reducer always sorts its input
  LOCUST_HIP_CHECK(hipEventRecord(m.ev[3], m.stream));
  m.enqueue_reduce_core(false);
  m.enqueue_pack_output();
  LOCUST_HIP_CHECK(hipEventRecord(m.ev[4], m.stream));
  m.download_output(r, m.ev[5]);
  r.times.wall_ms = (now_ns() - t0) * 1e-6;
  r.times.h2d_ms = DevicePipeline::ms_between(m.ev[0], m.ev[1]);
  r.times.process_ms = DevicePipeline::ms_between(m.ev[2], m.ev[3]);
  r.times.reduce_ms = DevicePipeline::ms_between(m.ev[3], m.ev[4]);
  r.times.d2h_ms = DevicePipeline::ms_between(m.ev[4], m.ev[5]);
  if (m.cfg.check) validate_result(r);
  return r;
}

std::vector<u32> GpuWordCount::sort_keys(const PackedKey* keys, u64 n,
                                         std::vector<PackedKey>* sorted) {
  Impl& m = *impl_;
  m.sync_clean = false;  // this entry point dirties d_sync
  m.upload_tokens(keys, n);
  m.enqueue_process(0, false, false, n);
  std::vector<u32> perm(n);
  if (n)
    LOCUST_HIP_CHECK(hipMemcpyAsync(perm.data(), m.d_perm, n * sizeof(u32),
                                    hipMemcpyDeviceToHost, m.stream));
  m.sync();
  if (sorted) m.download_keys(m.sorted, n, sorted);
  return perm;
}

std::vector<PackedKey> GpuWordCount::compact_slots(const u32* line_counts, u32 num_lines,
                                                   const PackedKey* slot_keys) {
  Impl& m = *impl_;
  m.sync_clean = false;  // this entry point dirties d_sync
  LOCUST_CHECK_ARG(m.cfg.map_path == MapPath::kCompat, "compact_slots needs a compat engine");
  LOCUST_CHECK_ARG(num_lines <= m.cap_lines, "too many lines for engine capacity");
  const u64 E = (u64)m.cfg.emits_per_line;
  u64 live = 0;
  for (u32 l = 0; l < num_lines; ++l) {
    LOCUST_CHECK_ARG(line_counts[l] <= E, "line count above emits_per_line");
    live += line_counts[l];
  }
  LOCUST_CHECK_ARG(live <= m.cap, "too many live slots for engine capacity");
  m.set_num_records(0);
  m.upload_keys(m.slots, slot_keys, (u64)num_lines * E);
  m.sync();  // the key staging is reused below
  if (num_lines)
    LOCUST_HIP_CHECK(hipMemcpy(m.d_line_counts, line_counts, num_lines * sizeof(u32),
                               hipMemcpyHostToDevice));
  launch_compact_slots(m.d_line_counts, num_lines, (int)E, m.slots, m.tokens, m.d_ctr,
                       m.lb_compact, m.stream);
  LOCUST_HIP_CHECK(
      hipMemcpyAsync(m.h_ctr, m.d_ctr, sizeof(MapCounters), hipMemcpyDeviceToHost, m.stream));
  m.sync();
  std::vector<PackedKey> out;
  m.download_keys(m.tokens, m.h_ctr->num_records, &out);
  return out;
}

WordCountResult GpuWordCount::reduce_sorted(const PackedKey* sorted, u64 n) {
  Impl& m = *impl_;
  m.sync_clean = false;  // this entry point dirties d_sync
  WordCountResult r;
  m.ensure_radix_full();
  m.set_num_records(n);
  m.upload_keys(m.sorted, sorted, n);
  m.enqueue_reduce_core(false);
  m.enqueue_pack_output();
  m.download_output(r, m.ev[5]);
  return r;
}

WordCountResult GpuWordCount::merge_runs(const std::vector<std::vector<KeyCount>>& runs) {
  Impl& m = *impl_;
  m.sync_clean = false;  // this entry point dirties d_sync
  LOCUST_CHECK_ARG(!runs.empty() && runs.size() <= (size_t)kMaxMergeRunsHost,
                   "need 1..64 runs");
  u64 n = 0;
  for (const auto& r : runs) n += r.size();
  LOCUST_CHECK_ARG(n <= m.cap && n <= kMergeMaxRecords, "too many records for engine capacity");
  m.set_num_records(0);
  u32* meta = reinterpret_cast<u32*>(m.h_u64);
  meta[0] = (u32)runs.size();
  u64 off = 0;
  for (size_t q = 0; q < runs.size(); ++q) {
    meta[1 + q] = (u32)runs[q].size();
    if (!runs[q].empty())
      LOCUST_HIP_CHECK(hipMemcpyAsync(m.d_records + off, runs[q].data(),
                                      runs[q].size() * sizeof(KeyCount), hipMemcpyHostToDevice,
                                      m.stream));
    off += runs[q].size();
  }
  u32* d_meta = reinterpret_cast<u32*>(m.d_offsets);
  LOCUST_HIP_CHECK(hipMemcpyAsync(d_meta, meta, (1 + runs.size()) * sizeof(u32),
                                  hipMemcpyHostToDevice, m.stream));
  m.grow_host_out(n);
  launch_merge_sorted_runs(m.d_records, m.d_records + runs[0].size(), d_meta, n,
                           reinterpret_cast<KeyCount*>(m.d_out), m.d_ctr, m.d_out_mapped,
                           m.d_ctr_mapped, m.lb_merge(n), m.stream);
  m.sync();
  *m.h_ctr = *m.h_ctr_mapped;
  WordCountResult r;
  m.fill_counters(r);
  m.copy_out(r.entries, m.h_ctr->num_unique);
  return r;
}

namespace {

struct RunSlice {
  const KeyCount* p;
  u64 n;
};

// Merges the slices (each sorted, distinct keys) into `out` (appended, key order) on
// `eng`, whose capacity is `limit` records: one launch_merge_sorted_runs per group of
// <= 64 runs holding <= limit records and a total count below the kernel's 2^40; more
// runs merge in rounds, more records split at the median key of the largest run.
void merge_slices(GpuWordCount& eng, u64 limit, std::vector<RunSlice> runs,
                  std::vector<WordCountEntry>* out) {
  runs.erase(std::remove_if(runs.begin(), runs.end(), [](const RunSlice& r) { return r.n == 0; }),
             runs.end());
  if (runs.empty()) return;
  u64 total = 0, count = 0;
  for (const RunSlice& r : runs) {
    total += r.n;
    for (u64 i = 0; i < r.n; ++i) count += r.p[i].count;
  }
  if (runs.size() == 1) {
    for (u64 i = 0; i < runs[0].n; ++i) {
      WordCountEntry e;
      for (int w = 0; w < kKeyWords; ++w) e.key.w[w] = runs[0].p[i].w[w];
      e.count = runs[0].p[i].count;
      out->push_back(e);
    }
    return;
  }
  if (total <= limit && count <= kMergeMaxCount) {
    if (runs.size() <= (size_t)kMaxMergeRunsHost) {
      std::vector<std::vector<KeyCount>> v(runs.size());
      for (size_t q = 0; q < runs.size(); ++q) v[q].assign(runs[q].p, runs[q].p + runs[q].n);
      WordCountResult r = eng.merge_runs(v);
      for (const WordCountEntry e : r.entries) out->push_back(e);
      return;
    }
    // rounds: every group of 64 runs becomes one run
    std::vector<std::vector<KeyCount>> level;
    for (size_t g = 0; g < runs.size(); g += kMaxMergeRunsHost) {
      std::vector<RunSlice> grp(runs.begin() + (long)g,
                                runs.begin() + (long)std::min(runs.size(), g + kMaxMergeRunsHost));
      std::vector<WordCountEntry> e;
      merge_slices(eng, limit, grp, &e);
      std::vector<KeyCount> run(e.size());
      for (size_t i = 0; i < e.size(); ++i) {
        for (int w = 0; w < kKeyWords; ++w) run[i].w[w] = e[i].key.w[w];
        run[i].count = e[i].count;
      }
      level.push_back(std::move(run));
    }
    std::vector<RunSlice> next;
    for (const auto& r : level) next.push_back({r.data(), r.size()});
    return merge_slices(eng, limit, next, out);
  }
  if (total <= runs.size()) {  // one record per run left and still too much count: host
    std::vector<std::vector<KeyCount>> v(runs.size());
    for (size_t q = 0; q < runs.size(); ++q) v[q].assign(runs[q].p, runs[q].p + runs[q].n);
    for (const WordCountEntry e : merge_runs_host(v)) out->push_back(e);
    return;
  }
  // split by key range at the median of the largest run: both halves shrink
  size_t big = 0;
  for (size_t q = 1; q < runs.size(); ++q)
    if (runs[q].n > runs[big].n) big = q;
  const KeyCount pivot = runs[big].p[runs[big].n / 2];
  std::vector<RunSlice> left, right;
  for (const RunSlice& r : runs) {
    const KeyCount* m = std::lower_bound(r.p, r.p + r.n, pivot, record_less);
    left.push_back({r.p, (u64)(m - r.p)});
    right.push_back({m, r.n - (u64)(m - r.p)});
  }
  merge_slices(eng, limit, left, out);
  merge_slices(eng, limit, right, out);
}

}  // namespace

std::vector<WordCountEntry> merge_runs_device(const JobConfig& cfg,
                                              const std::vector<std::vector<KeyCount>>& runs,
                                              double* setup_ms) {
  u64 total = 0;
  for (const auto& r : runs) total += r.size();
  std::vector<WordCountEntry> out;
  if (!total) return out;
  out.reserve(total);
  JobConfig c = cfg;
  c.chunk_bytes = 0;  // one pass: the engine holds a merge's records
  c.records_only = true;
  u64 limit = std::min<u64>(total, kMergeMaxRecords);
  // LOCUST_MERGE_MAX_RECORDS: a lower per-launch record limit (tests of the key-range split)
  if (const char* e = std::getenv("LOCUST_MERGE_MAX_RECORDS"))
    limit = std::max<u64>(2, std::min<u64>(limit, (u64)std::atoll(e)));
  // capacity = min(lines x emits, bytes / 2 + 1) >= limit
  const u64 t0 = now_ns();
  GpuWordCount eng(c, 2 * limit + 2, limit + 1);
  if (setup_ms) *setup_ms = (now_ns() - t0) * 1e-6;
  std::vector<RunSlice> slices;
  for (const auto& r : runs) slices.push_back({r.data(), r.size()});
  merge_slices(eng, limit, slices, &out);
  return out;
}

}  // namespace locust
