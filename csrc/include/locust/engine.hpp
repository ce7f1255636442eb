// WordCount engines: the single-GPU HIP pipeline and the CPU reference pipeline.
//
// GpuWordCount reproduces the reference's GPU path (/root/reference/
// MapReduce/src/main.cu:388-487) stage for stage -- Map (tokenize/emit), Process
// (stream compaction + key sort), Reduce (boundary mark + head compaction + adjacent
// difference) -- with every buffer preallocated at construction so a run performs no
// allocation and, apart from reading back result sizes, no host synchronisation.
// CpuWordCount is the golden oracle and the `--backend cpu` path (main.cu:489-527).
#pragma once

#include <cstddef>
#include <iterator>
#include <memory>
#include <string>
#include <vector>

#include "locust/common.hpp"
#include "locust/config.hpp"
#include "locust/kv.hpp"

namespace locust {

// A window of input lines: `bytes` bytes of text, lines separated by '\n' (the last line
// may lack one).  `first_line` is the global index of the first line (the reference's
// KeyValuePair.key, main.cu:58).
class TextSource;
struct TextInput {
  const char* data = nullptr;
  u64 bytes = 0;
  u64 num_lines = 0;
  u64 first_line = 0;
  // Distributed shards only: a shard larger than one device pass may be streamed from a
  // source (a rank's byte range of a file) instead of held in memory -- data is then null,
  // bytes the range's size, and num_lines unknown until the source is drained.
  TextSource* source = nullptr;
  u64 lines() const;  // num_lines, or the lines the source has handed out
};

struct StageTimes {
  // Honest device time from hipEvents on the compute stream (ms).
  double h2d_ms = 0, map_ms = 0, process_ms = 0, reduce_ms = 0, d2h_ms = 0;
  // Host wall clock of the whole run() call (ms).
  double wall_ms = 0;
  // Device time of the whole job (first to last enqueued operation, hipEvents).
  double gpu_ms = 0;
  // Host-side split of wall_ms (single-GPU runs): enqueue/launch, waiting for the device,
  // and copying the results out of the host-mapped output.
  double host_launch_ms = 0, host_wait_ms = 0, host_copy_ms = 0;
  bool graph = false;  // replayed as one hipGraph: the stage fields above are not split
  bool lean = false;   // direct launches, polled completion: no device stage timestamps
  // Host timers placed where the reference placed them (launch-only map etc., BASELINE.md
  // "How the reference measured these"), filled when JobConfig.ref_timers is set.
  double ref_map_ms = 0, ref_process_ms = 0, ref_reduce_ms = 0;
};

// One output entry: a unique key and the length of its run in the globally sorted token
// array (`count`); 40 B, the layout of KeyCount and of the device's output records.  The
// reference's `val` (start index of the run, KeyValue.h:13-18 / main.cu:181-206) is the
// exclusive prefix of the counts in key order: it is not stored per entry (it would be 8 B
// of every record crossing PCIe) but rebuilt on the host from WordCountResult::val_base --
// see EntryVals.
struct WordCountEntry {
  PackedKey key;
  u64 count;
};
static_assert(sizeof(WordCountEntry) == 40, "WordCountEntry 40 B");

// One segment of compact records (kv.hpp CompactRecord: a header word, then the key's
// non-zero words) holding `n` entries in key order.
struct EntrySegment {
  const u64* words = nullptr;
  u64 n = 0;
};

// The entries of a result: an owned vector, or -- zero-copy -- the engine's host-mapped
// output buffer itself, which the device wrote and which this list keeps alive (`owner`)
// until it is dropped; the engine then reuses the buffer for a later job.  The device may
// have written that buffer as 40-B records (adopt) or as compact records (adopt_compact:
// segments in key order, ~16-24 B per entry).  Iteration decodes
// compact records on the fly; data() / operator[] turn a compact list into an owned
// vector first (once).  Vector-like.
class EntryList {
 public:
  EntryList() = default;
  EntryList(std::vector<WordCountEntry>&& v) : vec_(std::move(v)) {}  // NOLINT: implicit
  EntryList& operator=(std::vector<WordCountEntry>&& v) {
    release();
    vec_ = std::move(v);
    return *this;
  }
  // Borrow n entries at p, kept valid by `owner`.
  void adopt(std::shared_ptr<void> owner, WordCountEntry* p, size_t n) {
    release();
    vec_.clear();
    vec_.shrink_to_fit();
    owner_ = std::move(owner);
    view_ = p;
    n_ = n;
  }
  // Borrow compact segments (n entries in all), kept valid by `owner`.
  void adopt_compact(std::shared_ptr<void> owner, std::vector<EntrySegment> segs, size_t n) {
    adopt(std::move(owner), nullptr, n);
    segs_ = std::move(segs);
    compact_ = true;
  }
  bool borrowed() const { return owner_ != nullptr; }
  bool compact() const { return compact_; }
  size_t size() const { return owner_ ? n_ : vec_.size(); }
  bool empty() const { return size() == 0; }
  // Bytes the device wrote for these entries (compact: the segments' words).
  u64 wire_bytes() const;
  WordCountEntry* data() {
    materialize();
    return owner_ ? view_ : vec_.data();
  }
  const WordCountEntry* data() const {
    materialize();
    return owner_ ? view_ : vec_.data();
  }
  WordCountEntry& operator[](size_t i) { return data()[i]; }
  const WordCountEntry& operator[](size_t i) const { return data()[i]; }
  WordCountEntry front() const { return *begin(); }

  // Forward iteration over either form; yields entries by value.
  class const_iterator {
   public:
    using iterator_category = std::forward_iterator_tag;
    using value_type = WordCountEntry;
    using difference_type = std::ptrdiff_t;
    using pointer = const WordCountEntry*;
    using reference = WordCountEntry;
    const_iterator() = default;
    WordCountEntry operator*() const {
      if (flat_) return *flat_;
      WordCountEntry e;
      decode_compact(w_, &e.key, &e.count);
      return e;
    }
    const_iterator& operator++() {
      if (flat_) {
        ++flat_;
        return *this;
      }
      w_ += compact_record_words(w_[0]);
      if (--left_ == 0) next_segment();
      return *this;
    }
    const_iterator operator++(int) {
      const_iterator t = *this;
      ++*this;
      return t;
    }
    bool operator==(const const_iterator& o) const { return flat_ == o.flat_ && w_ == o.w_; }
    bool operator!=(const const_iterator& o) const { return !(*this == o); }

   private:
    friend class EntryList;
    void next_segment() {
      w_ = nullptr;
      while (seg_ != seg_end_) {
        const EntrySegment& s = *seg_++;
        if (s.n) {
          w_ = s.words;
          left_ = s.n;
          return;
        }
      }
    }
    const WordCountEntry* flat_ = nullptr;
    const u64* w_ = nullptr;
    u64 left_ = 0;
    const EntrySegment* seg_ = nullptr;
    const EntrySegment* seg_end_ = nullptr;
  };
  const_iterator begin() const {
    const_iterator it;
    if (compact_) {
      it.seg_ = segs_.data();
      it.seg_end_ = segs_.data() + segs_.size();
      it.next_segment();
    } else if (size()) {
      it.flat_ = owner_ ? view_ : vec_.data();
    }
    return it;
  }
  const_iterator end() const {
    const_iterator it;
    if (!compact_ && size()) it.flat_ = (owner_ ? view_ : vec_.data()) + size();
    return it;
  }
  // Owned storage of n entries (a borrowed prefix is copied over).
  void resize(size_t n) {
    if (owner_) {
      std::vector<WordCountEntry> v;
      v.reserve(n);
      for (auto it = begin(); it != end() && v.size() < n; ++it) v.push_back(*it);
      release();
      vec_ = std::move(v);
    }
    vec_.resize(n);
  }
  void assign(const WordCountEntry* b, const WordCountEntry* e) {
    release();
    vec_.assign(b, e);
  }

 private:
  void release() const {
    owner_.reset();
    view_ = nullptr;
    n_ = 0;
    segs_.clear();
    compact_ = false;
  }
  // compact -> an owned vector (the buffer is released)
  void materialize() const {
    if (!compact_) return;
    std::vector<WordCountEntry> v;
    v.reserve(n_);
    for (auto it = begin(); it != end(); ++it) v.push_back(*it);
    release();
    vec_ = std::move(v);
  }
  mutable std::vector<WordCountEntry> vec_;
  mutable std::shared_ptr<void> owner_;
  mutable WordCountEntry* view_ = nullptr;
  mutable size_t n_ = 0;
  mutable std::vector<EntrySegment> segs_;
  mutable bool compact_ = false;
};

struct WordCountResult {
  EntryList entries;  // sorted by key
  // val of entries[0]: 0 for a whole result, the token total of the lower ranks' key
  // ranges for one rank's range of a distributed job.
  u64 val_base = 0;
  u64 num_lines = 0;
  u64 num_tokens = 0;       // kv_num_map
  u64 num_unique = 0;       // kv_num_reduce
  u64 overflow_lines = 0;   // lines that printed "WARN: Exceeded emit limit"
  u64 truncated = 0;        // tokens longer than max_key_len
  u64 max_key_len = 0;
  u64 chunks = 1;           // > 1: the input streamed through the engine in chunks
  StageTimes times;
};

// The reference's val of each entry in order: val(i) = val_base + sum of counts before i.
//   EntryVals v(res); for (auto& e : res.entries) { u64 val = v.next(e); ... }
class EntryVals {
 public:
  explicit EntryVals(const WordCountResult& r) : at_(r.val_base) {}
  explicit EntryVals(u64 base) : at_(base) {}
  u64 next(const WordCountEntry& e) {
    const u64 v = at_;
    at_ += e.count;
    return v;
  }

 private:
  u64 at_;
};

// Text read piece by piece (a file too large to hold): whole lines go straight into the
// engine's pinned staging, so host memory stays bounded by two chunks whatever the input.
class TextSource {
 public:
  virtual ~TextSource() = default;
  virtual u64 size() const = 0;  // total bytes (sizes the chunk bookkeeping)
  // Fills dst (room for cap bytes) with the next whole lines (the last line of the input
  // may lack its '\n'); returns the bytes written, 0 at the end.
  virtual u64 next(char* dst, u64 cap) = 0;
  virtual u64 lines() const = 0;  // lines handed out so far
};
// A file read with `threads` concurrent preads per chunk (0: up to 8); see io.cpp.
std::unique_ptr<TextSource> open_file_source(const std::string& path, u32 threads = 0);
// The same over the byte range [begin, end) of the file (begin at a line start).
std::unique_ptr<TextSource> open_file_range_source(const std::string& path, u64 begin, u64 end,
                                                   u32 threads = 0);

// ---- HBM budget planning (SURVEY.md §5.7 "HBM budget accounting per GPU") ----
// The reference sizes everything by compile-time constants (main.cu:18-20: 5,800 lines,
// 116,000 emits; three cudaMallocs at :393,402,451).  Here an engine's device pass is
// planned from its input size and the GPU's free memory before anything is allocated:
//  * the token buffers hold one map launch's worst case (a byte in two a token); a
//    streaming engine maps each chunk in windows of <= kStreamMapWindow bytes, so its
//    token buffers do not grow with --chunk-mb;
//  * the sort / reduce buffers of a dictionary engine hold the distinct keys only (ucap);
//    the reference algorithm's every-token buffers are made on first use
//    (DevicePipeline::ensure_radix_full);
//  * a one-pass input whose engine would not fit its share of HBM (free / hbm_share, at
//    most kHbmUsable of it), or that exceeds 2^30 tokens, is planned as a stream of
//    chunk_bytes chunks (default kDefaultStreamChunk) on the dictionary path; a plan that
//    still does not fit is refused with the sizes in the message.
struct DevicePassPlan {
  bool streaming = false;
  u64 chunk_bytes = 0;   // device text buffer: the one pass, or one stream chunk
  u64 pass_bytes = 0;    // largest input one pass takes (a streaming engine: map_window)
  u64 map_window = 0;    // a streamed chunk's map windows (0: not streaming)
  u64 cap_lines = 0;
  u64 cap = 0;           // tokens one map launch may emit
  u64 ucap = 0;          // distinct keys of the dictionary
  u64 rcap = 0;          // records the sort / reduce buffers hold
  u64 device_bytes = 0;  // the engine's planned device allocations
  u64 budget_bytes = 0;  // the HBM it may use
  std::string why;       // why the input was planned as a stream ("" if asked for)
};
constexpr u64 kStreamMapWindow = 32ull << 20;
constexpr u64 kDefaultStreamChunk = 256ull << 20;
constexpr double kHbmUsable = 0.9;
// free_bytes: the device's free memory (hipMemGetInfo).  Throws when no plan fits.
DevicePassPlan plan_device_pass(const JobConfig& cfg, u64 max_bytes, u64 max_lines,
                                u64 cap_records, u64 free_bytes);

class GpuWordCount {
 public:
  // Capacity is fixed at construction: max_text_bytes / max_lines per device pass.  With
  // the dictionary path and the fast map, larger inputs stream through in line-aligned
  // chunks of max_text_bytes (double-buffered H2D; one dictionary across chunks).
  GpuWordCount(const JobConfig& cfg, u64 max_text_bytes, u64 max_lines);
  ~GpuWordCount();
  GpuWordCount(const GpuWordCount&) = delete;
  GpuWordCount& operator=(const GpuWordCount&) = delete;

  WordCountResult run(const TextInput& in);
  // A streamed input (a streaming engine: JobConfig.chunk_bytes set, max_text_bytes larger
  // than it): chunks of chunk_bytes read from `src` into pinned staging, overlapped with
  // the H2D and the map of the previous chunk.
  WordCountResult run_source(TextSource& src);

  // How the engine's partition map has fared (diagnostics, tests): retunes of the map from
  // a job's output, jobs whose ordered build overflowed an LDS table and fell back to the
  // HBM table, and whether the in-job plan of large passes was given up.
  struct Stats {
    u32 retunes = 0, fallbacks = 0, planned_passes = 0;
    bool devplan_failed = false;
    // HBM: this engine's device allocations, and the GPU's free / total memory before them
    u64 device_bytes = 0, hbm_free = 0, hbm_total = 0;
    bool streaming = false;
    u64 chunk_bytes = 0, map_window = 0;
  };
  Stats stats() const;

  // The partition map (kDictParts + 1 ascending range starts, partmap.hpp) -- a
  // load-balancing hint only: any ascending map gives the same results.  partition_map()
  // finishes a background retune first and returns false while the map is still the data-
  // independent default; set_partition_map() starts this engine on a map tuned earlier (the
  // CLI's per-file cache), returning false (map unchanged) for a malformed one.
  bool partition_map(std::vector<u64>* lo);
  bool set_partition_map(const std::vector<u64>& lo);

  // Stage split: map + process only, returning the sorted tokens of
  // this input; and reduce-only over (possibly unsorted) tokens.
  std::vector<PackedKey> run_map_stage(const TextInput& in, WordCountResult* stats);
  WordCountResult run_reduce_stage(const PackedKey* keys, u64 n);

  // Sort arbitrary packed keys on the device (used by tests and the shuffle receiver).
  std::vector<u32> sort_keys(const PackedKey* keys, u64 n, std::vector<PackedKey>* sorted);

  // Single-stage entry points for the kernel unit tests.
  // Stable compaction of the compat map's fixed slots (main.cu:411): slot_keys holds
  // num_lines * emits_per_line keys, the first line_counts[l] slots of line l are live.
  // Needs a MapPath::kCompat engine with capacity for num_lines lines.
  std::vector<PackedKey> compact_slots(const u32* line_counts, u32 num_lines,
                                       const PackedKey* slot_keys);
  // Reduce steps over keys that are already sorted: boundary mark + head compaction +
  // adjacent difference (main.cu:161-238, 462) on the configured reduce path.
  WordCountResult reduce_sorted(const PackedKey* sorted, u64 n);
  // Root merge of the gather strategy (launch_merge_sorted_runs) over host-made runs, each
  // sorted with distinct keys: the merged (key, val, count) entries.
  WordCountResult merge_runs(const std::vector<std::vector<KeyCount>>& runs);

  const JobConfig& config() const;
  u64 token_capacity() const;
  u64 text_capacity() const;  // bytes per device pass (input_buffer() size)
  // Pinned host staging buffer of the text (capacity max_text_bytes + 64).  A TextInput
  // whose data points here is uploaded without the host-side staging copy -- the
  // analogue of the reference loading the file into its host array before any timer.
  char* input_buffer();

 private:
  struct Impl;
  std::unique_ptr<Impl> impl_;
};

// Input text in page-locked host memory: the GPU engine DMAs it (whole, or chunk by chunk
// when streaming) without a staging copy.  Falls back to ordinary memory when no GPU
// runtime is present (CPU engine, build machine).
class HostText {
 public:
  explicit HostText(u64 capacity);
  ~HostText();
  HostText(const HostText&) = delete;
  HostText& operator=(const HostText&) = delete;
  char* data() { return data_; }
  const char* data() const { return data_; }
  u64 size() const { return size_; }
  u64 lines() const { return lines_; }
  u64 capacity() const { return cap_; }
  bool pinned() const { return pinned_; }
  void set_size(u64 bytes, u64 lines);
  TextInput input(u64 first_line = 0) const;

 private:
  char* data_ = nullptr;
  u64 cap_ = 0, size_ = 0, lines_ = 0;
  bool pinned_ = false;
};

class CpuWordCount {
 public:
  explicit CpuWordCount(const JobConfig& cfg);
  WordCountResult run(const TextInput& in);
  std::vector<PackedKey> run_map_stage(const TextInput& in, WordCountResult* stats);
  WordCountResult run_reduce_stage(const PackedKey* keys, u64 n);

 private:
  JobConfig cfg_;
};

// Tokenize one line with the reference rules (delimiters, emit cap, truncation).  Used by
// the CPU engine and the tests; returns the number of tokens dropped by the emit cap.
int tokenize_line(const char* line, u64 len, const JobConfig& cfg, std::vector<PackedKey>* out,
                  u64* truncated);

// Sorted unique keys + counts -> entries with val = exclusive prefix of counts.
void entries_from_sorted_tokens(const PackedKey* sorted, u64 n, std::vector<WordCountEntry>* out);

// Device self-test of the string library: one GPU thread per
// string runs d_strlen / d_strcmp (with the next string) / d_strcpy_bounded / d_strtok_r /
// d_itoa; the rows come back for comparison with the host build.
constexpr int kStringTestMax = 128;
struct StringTestOut {
  int len, cmp_next, copy_len, ntok;
  int tok_off[8];
  char copy[30];
  char itoa_buf[34];
};
std::vector<StringTestOut> run_string_selftest(const std::vector<std::string>& strings,
                                               const std::vector<int>& ints,
                                               const std::string& delims, int device = 0);

}  // namespace locust
