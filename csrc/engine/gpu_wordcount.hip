// Single-GPU WordCount engine (GpuWordCount): the public API over the device pipeline
// (csrc/engine/pipeline.hpp).
#include "pipeline.hpp"

namespace locust {

using detail::DevicePipeline;

// =====================================================================================
// GpuWordCount
// =====================================================================================
struct GpuWordCount::Impl : DevicePipeline {
  using DevicePipeline::DevicePipeline;
};

GpuWordCount::GpuWordCount(const JobConfig& cfg, u64 max_text_bytes, u64 max_lines)
    : impl_(new Impl(cfg, max_text_bytes, max_lines)) {}
GpuWordCount::~GpuWordCount() = default;

const JobConfig& GpuWordCount::config() const { return impl_->cfg; }
u64 GpuWordCount::token_capacity() const { return impl_->cap; }
char* GpuWordCount::input_buffer() { return impl_->ensure_h_text(); }
u64 GpuWordCount::text_capacity() const { return impl_->cap_bytes; }

WordCountResult GpuWordCount::run(const TextInput& in) { return impl_->run(in); }
WordCountResult GpuWordCount::run_source(TextSource& src) {
  LOCUST_CHECK_ARG(impl_->cfg.chunk_bytes && impl_->cap_bytes <= impl_->cfg.chunk_bytes,
                   "run_source needs a streaming engine (chunk_bytes set)");
  return impl_->run_source(src);
}
GpuWordCount::Stats GpuWordCount::stats() const {
  Stats s;
  s.retunes = impl_->pm_retunes;
  s.fallbacks = impl_->fallbacks;
  s.planned_passes = impl_->planned_passes;
  s.devplan_failed = impl_->devplan_failed;
  return s;
}

std::vector<PackedKey> GpuWordCount::run_map_stage(const TextInput& in, WordCountResult* stats) {
  Impl& m = *impl_;
  m.sync_clean = false;  // this entry point dirties d_sync
  m.check_input(in);
  m.enqueue_upload(in);
  m.enqueue_map(in);
  m.enqueue_process((u32)in.num_lines, m.cfg.map_path == MapPath::kCompat, false, kUnknownCount,
                    /*allow_psort=*/true);
  m.read_counters();
  if (m.h_ctr->flags & kCtrSortOverflow) {  // a partition outgrew the LDS sort
    m.redo_process_general((u32)in.num_lines);
    m.read_counters();
  }
  std::vector<PackedKey> out;
  m.download_keys(m.sorted, m.h_ctr->num_records, &out);
  if (stats) {
    stats->num_lines = in.num_lines;
    m.fill_counters(*stats);
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

}  // namespace locust
