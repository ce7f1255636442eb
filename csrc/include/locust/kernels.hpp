// Host-side launchers for the HIP/CDNA4 kernels.  Every launcher only enqueues work on
// the given stream (no allocation, no synchronisation), so whole pipelines can be
// captured into a hipGraph.  Element counts that are produced on the device (token
// count, unique count) are passed as device pointers and kernels early-exit past them;
// host-side `cap` arguments only bound the grid.
#pragma once

#include <hip/hip_runtime.h>

#include "locust/common.hpp"
#include "locust/config.hpp"
#include "locust/dstring.hpp"
#include "locust/kv.hpp"

namespace locust {

// Packed keys, structure-of-arrays: w[j][i] is word j of key i.
struct KeysSoA {
  u64* w[kKeyWords];
};
struct ConstKeysSoA {
  const u64* w[kKeyWords];
  ConstKeysSoA() = default;
  ConstKeysSoA(const KeysSoA& k) {  // NOLINT: implicit by design
    for (int j = 0; j < kKeyWords; ++j) w[j] = k.w[j];
  }
};

// Device-side counters written by the pipeline stages.
struct MapCounters {
  u32 num_records;      // records to sort: emitted tokens (kv_num_map) or received records
  u32 num_unique;       // kv_num_reduce
  u32 overflow_lines;   // lines that had more than emits_per_line tokens (WARN lines)
  u32 truncated;        // tokens longer than max_key_len (truncated)
  u32 num_newlines;     // line index size
  u32 max_key_len;      // longest token seen (before truncation)
  u64 total_count;      // sum of record counts (== num_records when every count is 1)
};

// Look-back scratch: a zeroed region of 64-bit status words plus a tile counter.
struct LookbackScratch {
  u64* status;
  u32* tile_counter;
};

// ---------------- map.hip ----------------
constexpr int kMapBlock = 256;
constexpr int kMapSegSteps = 16;                              // 64-B steps per wave
constexpr int kMapTileBytes = (kMapBlock / 64) * kMapSegSteps * 64;  // 4 KiB per workgroup
constexpr int kLineIdxBlock = 256;
constexpr int kLineIdxItems = 16;                             // bytes per thread
constexpr int kLineIdxTile = kLineIdxBlock * kLineIdxItems;

// Newline positions (stable order) -> nl_pos[0..num_newlines).  `text` has `bytes` bytes.
void launch_line_index(const char* text, u64 bytes, u64* nl_pos, MapCounters* ctr,
                       LookbackScratch lb, hipStream_t s);

// Reference-layout map: one thread per line runs device strtok_r in place over `text`
// (which must have a writable NUL byte at text[bytes]) and writes up to E tokens into
// slots [line*E + k]; line_counts[line] = number of emitted tokens.
void launch_map_compat(char* text, u64 bytes, const u64* nl_pos, u32 num_lines,
                       const char* d_delims, int emits_per_line, int max_key_len,
                       KeysSoA slots, u32* line_counts, MapCounters* ctr, hipStream_t s);

// Stable compaction of the fixed slots into a dense key array (Process step 1).
void launch_compact_slots(const u32* line_counts, u32 num_lines, int emits_per_line,
                          ConstKeysSoA slots, KeysSoA out, MapCounters* ctr,
                          LookbackScratch lb, hipStream_t s);

// Byte-parallel tokenizer: tokens compacted in text order straight into `out`.
void launch_map_fast(const char* text, u64 bytes, const DelimMask& dm, int emits_per_line,
                     int max_key_len, KeysSoA out, u64 out_cap, MapCounters* ctr,
                     LookbackScratch lb, hipStream_t s);

// ---------------- radix_sort.hip ----------------
constexpr int kSortBlock = 256;
constexpr int kSortItems = 16;
constexpr int kSortTile = kSortBlock * kSortItems;  // 4096 keys per tile
constexpr int kNumPositions = kKeyBytes;            // one 8-bit digit per key byte

struct SortPassInfo {
  u32 active;      // digit position not constant -> needs a pass
  u32 src;         // 0 = (keys_a, vals_a), 1 = (keys_b, vals_b)
};
struct SortPlan {
  u32 n;
  u32 word_active[kKeyWords];  // any live pass in this word
  u32 word_src[kKeyWords];     // buffer holding the permutation when the word starts
  u32 final_src;               // buffer holding the final permutation (vals)
  u32 num_active;
  u32 pad[2];
  SortPassInfo pass[kNumPositions];           // indexed by key byte position
  u32 digit_offset[kNumPositions][256];       // exclusive scan of the digit histogram
};

struct RadixWorkspace {
  u32* hist;           // [kNumPositions][256], zeroed per sort
  SortPlan* plan;      // device plan
  u64* keys[2];        // ping-pong key words
  u32* vals[2];        // ping-pong permutation
  u32* status;         // per-pass look-back status [tiles][256]: [31:30] flag, [29:0] count
  u32* tile_counters;  // [kNumPositions]
  u64 cap;             // max keys
};

u64 radix_status_words(u64 cap);  // u32 status words needed for one pass

// Phase 1: zero scratch, digit histograms for all 32 byte positions, plan on device.
void radix_sort_prepare(ConstKeysSoA keys, const u32* d_n, RadixWorkspace& ws, hipStream_t s);
// Phase 2: run the passes.  When `host_plan` is non-null (a copy of the device plan read
// back by the caller), only live passes are launched with exactly-sized grids; otherwise
// every pass is launched and inactive ones early-exit on the device plan (graph mode).
void radix_sort_run(ConstKeysSoA keys, const u32* d_n, RadixWorkspace& ws,
                    const SortPlan* host_plan, hipStream_t s);
// After radix_sort_run: gathers keys (and optional u64 counts) into sorted order; the final permutation is
// ws.vals[plan.final_src] (resolved on the device).
void launch_gather_sorted(ConstKeysSoA keys, const RadixWorkspace& ws, KeysSoA sorted,
                          u32* perm_out, const u64* counts_in, u64* counts_out, u64 cap,
                          hipStream_t s);

// ---------------- reduce.hip ----------------
constexpr int kReduceBlock = 256;
constexpr int kReduceItems = 8;
constexpr int kReduceTile = kReduceBlock * kReduceItems;

// Exclusive scan of u64 record counts in sorted order (weighted reduce: combined or
// shuffled records carry counts > 1).  Writes ctr->total_count.
void launch_scan_counts(const u64* counts, u64 cap, u64* prefix, MapCounters* ctr,
                        LookbackScratch lb, hipStream_t s);

// Reduce steps 1+2: segment-head marking (key[i] != key[i-1]) fused with the stable
// compaction of heads.  head_val[j] = start of run j in token units: i itself when
// `prefix` is null (every count 1: the reference's kernFindUniqBool value), else prefix[i].
// Writes ctr->num_unique (and ctr->total_count when prefix is null).
void launch_mark_compact_heads(ConstKeysSoA sorted, const u64* prefix, u64 cap, ReducePath path,
                               KeysSoA head_keys, u64* head_val, MapCounters* ctr,
                               LookbackScratch lb, hipStream_t s);
// Reduce step 3 (kernGetCount): count[j] = val[j+1] - val[j]; last = total - val[last].
void launch_adjacent_diff(const u64* head_val, u64 cap, ReducePath path, u64* head_count,
                          const MapCounters* ctr, hipStream_t s);
// val[j] += *offset (global start index of this rank's key range).
void launch_add_offset(u64* head_val, u64 cap, const u64* d_offset, const MapCounters* ctr,
                       hipStream_t s);

// Output records for the host: {packed key, val, count}.
struct OutRecord {
  u64 w[kKeyWords];
  u64 val;
  u64 count;
};
static_assert(sizeof(OutRecord) == 48, "OutRecord 48 B");
void launch_pack_output(ConstKeysSoA head_keys, const u64* head_val, const u64* head_count,
                        u64 cap, const MapCounters* ctr, OutRecord* out, hipStream_t s);

// ---------------- shuffle.hip ----------------
// SoA keys (+ counts, null = 1) -> AoS KeyCount records (the all-to-all payload).
void launch_pack_records(ConstKeysSoA keys, const u64* counts, const u32* d_n, u64 cap,
                         KeyCount* out, hipStream_t s);
// AoS KeyCount -> SoA keys + counts; sets ctr->num_records = n (host-known).
void launch_unpack_records(const KeyCount* in, u64 n, KeysSoA keys, u64* counts, hipStream_t s);
// S evenly spaced keys of a sorted array of *d_n keys: sample[k] = keys[floor((k+0.5)*n/S)].
void launch_sample_keys(ConstKeysSoA sorted, const u32* d_n, u32 num_samples, PackedKey* out,
                        hipStream_t s);
// offsets[p] = lower_bound(sorted, splitter[p-1]) for p in 1..P-1, offsets[0] = 0,
// offsets[P] = n.
void launch_bucket_offsets(ConstKeysSoA sorted, const u32* d_n, const PackedKey* splitters,
                           u32 num_buckets, u64* offsets, hipStream_t s);

}  // namespace locust
