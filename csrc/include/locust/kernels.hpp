// Host-side launchers for the HIP/CDNA4 kernels.  Every launcher only enqueues work on
// the given stream (no allocation, no synchronisation), so whole pipelines can be
// captured into a hipGraph.  Element counts that are produced on the device (token
// count, unique count) are passed as device pointers and kernels early-exit past them;
// host-side `cap` arguments only bound the grid.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>

#include "locust/common.hpp"
#include "locust/config.hpp"
#include "locust/dstring.hpp"
#include "locust/engine.hpp"
#include "locust/exch.hpp"
#include "locust/kv.hpp"
#include "locust/partmap.hpp"
#include "locust/slot.hpp"

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
struct alignas(8) MapCounters {
  u32 num_records;      // records to sort: emitted tokens (kv_num_map) or received records
  // tokens a combining map emitted (num_records counts its records); shares one 64-bit
  // word with num_records, so a combining tile updates both with a single atomic
  u32 map_tokens;
  u32 num_unique;       // kv_num_reduce
  u32 overflow_lines;   // lines that had more than emits_per_line tokens (WARN lines)
  u32 truncated;        // tokens longer than max_key_len (truncated)
  u32 num_newlines;     // line index size
  u32 max_key_len;      // longest token seen (before truncation)
  u64 total_count;      // sum of record counts (== num_records when every count is 1)
  u32 flags;            // kCtr* status bits
  u32 pad;
};
static_assert(offsetof(MapCounters, map_tokens) == 4, "num_records + map_tokens: one u64");
constexpr u32 kCtrDictOverflow = 1u;  // dictionary table full: rerun on the radix path
constexpr u32 kCtrSortOverflow = 2u;  // a psort partition held more than kPsortMax tokens
constexpr u32 kCtrNotEmitted = 0x80000000u;  // rank_emit skipped (too many distinct keys)

// Look-back scratch: a zeroed region of 64-bit status words plus a tile counter.
struct LookbackScratch {
  u64* status;
  u32* tile_counter;
};

// ---------------- map.hip ----------------
constexpr int kMapBlock = 256;
// Tile bytes = 4 waves x steps x 64 B.  Small inputs: 1 KiB tiles (run as 16 waves x one
// 64-B step, launch_map_fast: more workgroups in flight; 768-B tiles measured neutral,
// profiles/r6/map/tile768_ab.txt), large inputs 16 steps (4 KiB tiles: fewer overlaps).
constexpr int kMapSegStepsSmall = 4;
constexpr int kMapSegStepsLarge = 16;
constexpr int kMapTileBytesMin = (kMapBlock / 64) * kMapSegStepsSmall * 64;
constexpr u64 kMapLargeInput = 8ull << 20;  // switch to large tiles above 8 MiB
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

// ---------------- partition map: see locust/partmap.hpp ----------------
struct PartMap {                 // device view of a PartMapTables image
  const u64* lo = nullptr;       // [kDictParts + 1] range starts; null: first key byte
};
__device__ __forceinline__ u32 part_of(const PartMap& pm, u64 w0) {
  return pm.lo ? part_of_w0(pm.lo, w0) : (u32)(w0 >> 56);
}

// Byte-parallel tokenizer: tokens compacted in text order straight into `out`.
// trace (diagnostics, optional): per tile < 4096, s_memrealtime stamps at trace[t*8+0..5].
// part_off (optional): the tokens of each tile (map_tile_bytes(bytes): 1 KiB below
// kMapLargeInput, else 4 KiB) are written grouped by PartMap partition and
// part_off[t * kPartTable + p] is the absolute index of tile t's first partition-p token
// ([.. + kPartTable - 1] = the tile's end), so a partition's tokens are found without
// scanning every token's tag.
// counts (optional, 4 KiB tiles with part_off): per-tile combining -- in every tile, the
// first one-word key (<= 7 bytes) of each partition and all its repeats become ONE record
// at the head of the partition's run, with counts[i] = its multiplicity (1 for the other
// records); num_records then counts records, not tokens.  Zipfian text loses most of its
// hot-key volume before it is ever written.
constexpr int kPartTable = 257;
constexpr int kMapTileBytesLarge = (kMapBlock / 64) * kMapSegStepsLarge * 64;
inline u64 map_tile_bytes(u64 bytes) {
  return bytes < kMapLargeInput ? (u64)kMapTileBytesMin : (u64)kMapTileBytesLarge;
}
// part_occ (optional, small 1 KiB tiles with part_off): per tile, kPartOccWords words of a
// 256-bit mask of its non-empty partitions (OrderedExtra::part_occ).
constexpr int kPartOccWords = kDictParts / 32;
void launch_map_fast(const char* text, u64 bytes, const DelimMask& dm, int emits_per_line,
                     int max_key_len, KeysSoA out, u8* parts, u64 out_cap, MapCounters* ctr,
                     LookbackScratch lb, hipStream_t s, u64* trace = nullptr,
                     u32* part_off = nullptr, PartMap pm = PartMap{}, bool large_tiles = false,
                     u64* counts = nullptr, u32* part_occ = nullptr, u32* plan_flag = nullptr);

// ---------------- radix_sort.hip ----------------
constexpr int kSortBlock = 256;
constexpr int kSortItems = 16;
constexpr int kSortTile = kSortBlock * kSortItems;  // 4096 keys per tile
constexpr int kNumPositions = kKeyBytes;            // one 8-bit digit per key byte

constexpr int kSmallSortMax = 8192;                  // single-workgroup LDS sort up to here
constexpr u64 kUnknownCount = ~0ull;                 // "n only known on the device"

struct SortPassInfo {
  u32 active;      // digit position not constant -> needs a pass
  u32 src;         // reserved
};
struct SortPlan {
  u32 n;
  u32 pad[3];
  SortPassInfo pass[kNumPositions];           // indexed by key byte position
  u32 digit_offset[kNumPositions][256];       // exclusive scan of the digit histogram
};

struct RadixWorkspace {
  u32* hist_part;      // [radix_hist_blocks(cap)][kNumPositions * 256] partial histograms
  SortPlan* plan;      // device plan
  u64* keys[2];        // ping-pong key words
  u32* vals[2];        // ping-pong permutation
  u32* tile_counters;  // [kNumPositions], followed immediately by `status`
  u32* status;         // per-pass look-back status [tiles][256]: [31:30] flag, [29:0] count
  u64 cap;             // max keys
};

u64 radix_status_words(u64 cap);  // u32 status words needed for one pass
u32 radix_hist_blocks(u64 cap);   // histogram blocks (partials) for `cap` keys
u64 radix_zero_bytes(u64 cap);    // bytes of tile_counters + status zeroed per sort

// Sorts the *d_n packed keys (SoA) into `sorted` (+ optional counts permuted alongside,
// + optional permutation).  host_n: the count if the host knows it (then n <= 8192 runs
// the single-workgroup LDS sort, larger n reads the plan back and launches only live
// passes with exact grids), or kUnknownCount (graph mode: every kernel is launched and
// the ones not needed early-exit on the device-side count / plan).
// skip_upto: in graph mode, every kernel also exits when *d_n <= skip_upto (another sort
// handles that range; 0 = none).
void radix_sort(ConstKeysSoA keys, const u32* d_n, u64 host_n, RadixWorkspace& ws,
                const u64* counts_in, KeysSoA sorted, u64* counts_out, u32* perm_out,
                SortPlan* h_plan, hipStream_t s, u32 skip_upto = 0);

// ---------------- psort.hip ----------------
// Partitioned LDS radix sort of the tokens of a small-input fast map (part_off = its
// per-tile partition table over `ntiles` tiles, launch_map_fast): workgroup p sorts the
// tokens of PartMap partition p in LDS and writes them at their global sorted position.
// The map's counters must still be in `ctr` (num_records); a partition with more than
// kPsortMax tokens sets kCtrSortOverflow (then `sorted` is incomplete).  part_w
// (optional, host-mapped): per-partition work (tokens + kPartDistinctWeight x distinct
// first words), for the partition map's retuning.
constexpr int kPsortMax = 5120;
// trace (diagnostics, optional): per partition p, stamps at trace[p*16 + k] (see psort.hip).
void launch_psort(ConstKeysSoA tokens, const u32* part_off, u32 ntiles, u64 cap, KeysSoA sorted,
                  MapCounters* ctr, u32* part_w, hipStream_t s, u64* trace = nullptr);

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

// Output records for the host: {packed key, count}, 40 B (KeyCount's layout).  The
// reference's val (start of the key's run in the sorted token order) is the exclusive
// prefix of the counts and is rebuilt on the host (EntryVals, engine.hpp) instead of
// crossing PCIe with every record (round 2 wrote 48-B {key, val, count} records).
struct OutRecord {
  u64 w[kKeyWords];
  u64 count;
};
static_assert(sizeof(OutRecord) == 40, "OutRecord 40 B");
constexpr u32 kOutWords = sizeof(OutRecord) / 8;  // 5 u64 words per record
// Unweighted reduce steps 1-3 + output records in one kernel (LDS-staged tiles): `out`
// (room for out_cap records; host-mapped allowed) receives {key, count} in key order,
// ctr->num_unique / total_count are set and ctr_out (optional, host-mapped) gets a
// snapshot.  `lb` needs div_up(cap, kReduceTile) + 1 zeroed status words and a zeroed
// tile counter.
void launch_reduce_fused(ConstKeysSoA sorted, u64 cap, MapCounters* ctr, OutRecord* out,
                         u64 out_cap, MapCounters* ctr_out, LookbackScratch lb, hipStream_t s);
// Process + Reduce of the reference algorithm in ONE kernel (psort.hip): the partitioned
// LDS sort above, then inside each partition's workgroup the head mark (key[i] !=
// key[i-1]; runs never cross partitions, which are key ranges), counts as distances to the
// next head, the record index from a look-back over the
// partitions' head counts -- and the records straight into `out` (host-mapped allowed).
// The sorted token array is never written.  Self-cleaning like the ordered dictionary
// kernel: `status` (kDictParts look-back words) and `done_counter` must be zero before and
// are left zero; the last workgroup to finish re-zeroes the map's look-back words
// (map_lb, map_words) and counters, writes the ctr_out snapshot and, if given, publishes
// host_done_value to host_done (the lean job's completion word).  A partition past
// kPsortMax tokens sets kCtrSortOverflow: no records, nothing re-zeroed, the host redoes
// the pass with the device-wide sort.
struct PsortReduceArgs {
  OutRecord* out = nullptr;
  u64 out_cap = 0;
  MapCounters* ctr_out = nullptr;
  u64* status = nullptr;
  u32* done_counter = nullptr;
  LookbackScratch map_lb{};
  u32 map_words = 0;
  u32* host_done = nullptr;
  u32 host_done_value = 0;
};
void launch_psort_reduce(ConstKeysSoA tokens, const u32* part_off, u32 ntiles, u64 cap,
                         MapCounters* ctr, u32* part_w, const PsortReduceArgs& ra, hipStream_t s,
                         u64* trace = nullptr);
// ctr_out (optional, host-mapped): a snapshot of the final counters.
void launch_pack_output(ConstKeysSoA head_keys, const u64* head_val, const u64* head_count,
                        u64 cap, const MapCounters* ctr, OutRecord* out, hipStream_t s,
                        MapCounters* ctr_out = nullptr);

// ---------------- dict.hip ----------------
constexpr int kRankSortMax = 32768;  // all-pairs rank sort up to here, radix above

struct DictSlot {  // one hash-table slot (40 B): key words 1..3 stored XOR a magic value
  u64 w[kKeyWords];
  u32 id;          // dense id + 1 (0 = not yet published)
  u32 pad;
};
struct DictWorkspace {
  DictSlot* table;  // power-of-two slots, zeroed per run
  u32 mask;         // slots - 1 (this run)
  KeysSoA ukeys;    // dense distinct keys (ids from ctr->num_unique)
  u64* ucount;      // per-id occurrence counts, zeroed per run
  u64* uval;        // per-id weighted rank (= output val), zeroed per run
  u32 ucap;         // capacity of ukeys/ucount/uval: a key that would get id >= ucap sets
                    // kCtrDictOverflow (num_unique may then exceed ucap; consumers clamp)
  u32* urank;       // per-id rank (rank sort output), zeroed per run
};
// Partitioned build (small inputs): every token carries its partition (parts[i], the first
// byte of its key, written by the map kernel or by unpack_records); workgroup p aggregates
// partition p in LDS and appends its distinct keys to ukeys/ucount (and zeroes uval/urank).
// No table and no reset needed.  parts must be readable up to align_up(n, 16).
constexpr u64 kPartBuildMaxTokens = 1ull << 18;  // beyond: the HBM-table insert scales better
void launch_dict_part_build(ConstKeysSoA tokens, const u64* counts, const u8* parts,
                            const u32* d_n, u64 cap, const DictWorkspace& dw, MapCounters* ctr,
                            hipStream_t s);
// Ordered build (partitions = PartMap ranges, default the first key byte): aggregation,
// per-partition LDS sort,
// look-back offsets and the final (key, count) records in ONE kernel.  `out` needs
// room for every distinct key; `lb` needs kDictParts + 1 zeroed status words and a zeroed
// tile counter.  Sets ctr->num_unique / total_count (and ctr_out, if given, like the
// emit kernels); a partition past kPartSlots distinct keys sets kCtrDictOverflow.
// `trace` (diagnostics, optional): per partition p, s_memtime stamps at trace[p*16 + k]:
// 0 start, 1 built, 2 published, 8 histogram, 7 bucketed, 9 ranked, 3 sorted, 4 prefix
// known, 5 written; the key count at [p*16+6].
// Optional extra outputs of the ordered build (the distributed map): the sorted distinct
// keys as KeyCount records and/or SoA keys + counts, and the gather slot's header (`tmpl`
// completed on the device by the last partition).  `out` may then be null.
struct OrderedExtra {
  KeyCount* recs = nullptr;
  KeysSoA sorted{};
  u64* counts = nullptr;
  SlotHeader* hdr = nullptr;
  SlotHeader tmpl{};
  // Self-cleaning job: unless a partition overflowed, the last workgroup to finish
  // re-zeroes the accumulated counters of `ctr` (num_unique / total_count keep this run's
  // values), this kernel's look-back scratch and the map's (`map_lb`, map_words status
  // words), so the next job needs no memset in front.
  bool self_clean = false;
  LookbackScratch map_lb{};
  u32 map_words = 0;
  u32* done_counter = nullptr;  // zeroed counter of finished workgroups (self_clean)
  // With self_clean (optional, host-mapped): the last workgroup publishes host_done_value
  // here once every workgroup's writes are visible system-wide -- the lean job's completion
  // word without a kernel of its own behind this one.
  u32* host_done = nullptr;
  u32 host_done_value = 0;
  // Tokens from the small-input fast map with its per-tile partition table (launch_map_fast
  // part_off): partitions read their token ranges from it instead of scanning the tags.
  const u32* part_off = nullptr;
  u32 part_tiles = 0;
  // With part_off and part_occ (the map's per-tile occupancy masks): plan the workgroups
  // inside the job from THIS job's map statistics.  Every workgroup ORs the occupancy
  // masks (which partitions are non-empty: exact), estimates the partitions' token counts
  // from the same evenly spaced rows of the per-tile table, deals the kDictParts
  // workgroups out over the non-empty partitions in proportion to them, and a partition
  // with K > 1 workgroups is cut into K key ranges at quantiles of a sample of its own
  // tokens (every sibling draws the same sample): virtual partitions in key order, one
  // look-back over all of them.  A first-letter partition map on English text leaves ~200
  // of 256 workgroups idle and puts 's'/'t' on the critical path without it.  (Inputs of
  // at most kPartBlock tiles; larger ones keep one workgroup per partition.)
  const u32* part_occ = nullptr;
  // With part_occ (optional, zeroed device word): the map sets it when a tile holds
  // kPlanTrigger tokens of one partition; the ordered kernel plans only then (otherwise
  // one workgroup per map partition, without the plan's loads), and the self-clean
  // re-zeroes it.  Null: plan every pass.
  u32* plan_flag = nullptr;
  u32 split_min = 0;            // planned workgroups: tokens per extra sibling (0: default)
  // The partition map the tokens' partitions were computed with (default: first byte).
  PartMap pm{};
  // Optional (host-mapped): part_w[p] = partition p's work (tokens + kPartDistinctWeight x
  // distinct keys), written every run; the host retunes `pm` when it is unbalanced.
  u32* part_w = nullptr;
  // Records `out` holds: a job with more distinct keys writes none (the host sees
  // num_unique > out_cap and takes another path).
  u64 out_cap = ~0ull;
  // Compact host output (kv.hpp compact records) instead of the 40-B
  // records at `out`: virtual partition v writes its entries, in key order, from word
  // 5 * (entries before v) of `cout` -- where its 40-B records would have started, so the
  // look-back is unchanged and the capacity is out_cap records' worth of words -- and
  // ctab[v] = entries | words << 16 | first entry << 32 (host-mapped, every v of the launch;
  // ~0: not written).
  u64* cout = nullptr;
  u64* ctab = nullptr;
};
void launch_dict_ordered(ConstKeysSoA tokens, const u64* counts, const u8* parts,
                         const u32* d_n, u64 cap, MapCounters* ctr, OutRecord* out,
                         MapCounters* ctr_out, LookbackScratch lb, hipStream_t s,
                         u64* trace = nullptr, const OrderedExtra& ex = OrderedExtra{});
// Writes `value` to the host-mapped `word` once everything earlier on `s` has completed
// (signal.hip; the lean job path polls it instead of synchronising the stream).
void launch_signal_host(u32* word, u32 value, hipStream_t s);
// bytes (a multiple of 16, 16-B aligned) from device memory into a host-mapped buffer
// through its device pointer, by a kernel (signal.hip)
void launch_copy_to_mapped(void* dst_mapped_dev, const void* src, u64 bytes, hipStream_t s);

// Large ordered build (passes past kPartBuildMaxTokens whose map wrote a partition table,
// dict.hip): launch_dict_partials splits tiles [tile_begin, tile_end) into `nslices`
// slices; workgroup (p, k) aggregates partition p's records of slice k and writes the
// distinct keys + counts to partial slot p * nslots + slot_base + k (`partials`:
// kDictParts * nslots * kPartSlotsHost records, `partial_n`: one length per slot, all ones
// if its table overflowed).  Upload pieces each get their own slot, filled right after the
// piece's map (the aggregation overlaps the remaining H2D).  launch_dict_ordered_partials
// merges each partition's nslots slots and finishes like launch_dict_ordered (overflow:
// kCtrDictOverflow).
constexpr int kOrdWorkers = 4;         // slices of a one-launch large pass
constexpr int kMaxPartialSlots = 32;   // slots per partition (pieces of a piecewise pass)
constexpr int kPartSlotsHost = 2048;  // distinct keys per LDS table (dict.hip kPartSlots)
// trace (diagnostics, optional): kDictParts * kOrdWorkers * 8 stamps (see dict.hip).
// counts: per-record multiplicities of a combining map (null: every record is 1).
void launch_dict_partials(ConstKeysSoA tokens, const u64* counts, const u32* part_off,
                          u32 tile_begin, u32 tile_end, u32 nslices, u32 slot_base, u32 nslots,
                          u64 cap, KeyCount* partials, u32* partial_n, hipStream_t s,
                          u64* trace = nullptr);
void launch_dict_ordered_partials(const KeyCount* partials, const u32* partial_n, u32 nslots,
                                  MapCounters* ctr, OutRecord* out, MapCounters* ctr_out,
                                  LookbackScratch lb, hipStream_t s, u64* trace = nullptr,
                                  const OrderedExtra& ex = OrderedExtra{});
// Same, over runs of KeyCount records each sorted by key (the gather strategy's per-rank
// combined outputs); duplicates across runs are summed.  Run 0 is `own`, runs 1.. lie
// back to back in `recv`; `meta` (device) = [nruns <= 64, len_0, len_1, ...].
constexpr int kMaxMergeRunsHost = kMaxSlotRanks;
void launch_dict_merge_runs(const KeyCount* own, const KeyCount* recv, const u32* meta,
                            MapCounters* ctr, OutRecord* out, MapCounters* ctr_out,
                            LookbackScratch lb, hipStream_t s, PartMap pm = PartMap{});
// ---------------- partplan.hip ----------------
// A partition map cut at equal weights of a sample's distinct keys (first words
// ukeys_w0[0 .. min(*d_u, ucap)), in any order, with their sample counts; a key seen once
// weighs more: it stands for the rare keys not sampled yet): writes out->lo (device).
void launch_part_plan(const u64* ukeys_w0, const u64* ucount, const u32* d_u, u32 ucap,
                      PartMapTables* out, hipStream_t s);
// ---------------- merge.hip ----------------
// Merge of sorted runs (same run layout and meta as launch_dict_merge_runs) by lock-step
// binary search + one look-back scan: `merged` (room for every record, bounded by `cap`)
// is scratch; out / ctr / ctr_out as for launch_dict_ordered.  `lb` needs
// merge_scratch_words(cap) status words and a tile counter; the merge resets them itself
// (no memset needed).  Requires fewer than 2^22 records and a total count below 2^40
// (checked by the caller).
u64 merge_scratch_words(u64 cap);
void launch_merge_sorted_runs(const KeyCount* own, const KeyCount* recv, const u32* meta,
                              u64 cap, KeyCount* merged, MapCounters* ctr, OutRecord* out,
                              MapCounters* ctr_out, LookbackScratch lb, hipStream_t s);
// Same over the all-gathered slots: `nslots` slots of kSlotHeaderRecords + slot_records
// records each, run q = slot q's records, its length min(header.n, slot_records) (0 when
// the header's status is not kSlotOk).  `merged` needs nslots * slot_records records.
// hdr_out (optional, host-mapped): every slot's header, copied by the merge.
void launch_merge_slots(const KeyCount* slots, u32 nslots, u32 slot_records, KeyCount* merged,
                        MapCounters* ctr, OutRecord* out, MapCounters* ctr_out,
                        LookbackScratch lb, SlotHeader* hdr_out, hipStream_t s);
constexpr u64 kMergeMaxRecords = (1ull << 22) - 1;
constexpr u64 kMergeMaxCount = (1ull << 40) - 1;

// Hash every token (with its count; null = 1) into the table; distinct keys land in
// ukeys[0 .. ctr->num_unique) with summed counts in ucount.
void launch_dict_insert(ConstKeysSoA tokens, const u64* counts, const u32* d_n, u64 cap,
                        const DictWorkspace& dw, MapCounters* ctr, hipStream_t s);
// rank[i] = number of keys smaller than key i (distinct keys; rank zeroed by the caller);
// with counts/val also val[i] = total count of the smaller keys (zeroed by the caller).
// Early-exits (device-side) when *d_u > kRankSortMax.
void launch_rank_sort(ConstKeysSoA keys, const u64* counts, const u32* d_u, u64 cap, u32* rank,
                      u64* val, hipStream_t s);
// out[rank[i]] = {key i, count i} (val feeds total_count only); optional host-mapped
// counter snapshot.
void launch_rank_emit(ConstKeysSoA keys, const u64* counts, const u32* rank, const u64* val,
                      u64 cap, const MapCounters* ctr, OutRecord* out, MapCounters* ctr_out,
                      hipStream_t s);
void launch_rank_scatter(ConstKeysSoA keys, const u64* counts, const u32* rank, const u32* d_u,
                         u64 cap, KeysSoA sorted, u64* sorted_counts, hipStream_t s);
// Scan of the sorted counts (-> ctr->total_count) and the OutRecords.
void launch_scan_pack(ConstKeysSoA sorted, const u64* counts, u64 cap, MapCounters* ctr,
                      OutRecord* out, LookbackScratch lb, hipStream_t s,
                      MapCounters* ctr_out = nullptr, u32 emit_limit = 0xFFFFFFFFu);

// ---------------- shuffle.hip ----------------
// SoA keys (+ counts, null = 1) -> AoS KeyCount records (the all-to-all payload).
void launch_pack_records(ConstKeysSoA keys, const u64* counts, const u32* d_n, u64 cap,
                         KeyCount* out, hipStream_t s);

// AoS KeyCount -> SoA keys + counts (+ parts, optional: partition tag per record for the
// partitioned dictionary builds).
void launch_unpack_records(const KeyCount* in, u64 n, KeysSoA keys, u64* counts, u8* parts,
                           hipStream_t s, PartMap pm = PartMap{});
// S evenly spaced keys of a sorted array of *d_n keys: sample[k] = keys[floor((k+0.5)*n/S)].
void launch_sample_keys(ConstKeysSoA sorted, const u32* d_n, u32 num_samples, PackedKey* out,
                        hipStream_t s);
// This rank's ExchMsg1 from the device counters (asynchronous-map exchange, exchange.hip):
// tmpl's status (host-side failure) or kExchMapRedo on a partition overflow; n_local,
// tokens (map_tokens of a combining map, else num_records) and the map statistics.  With
// num_samples, the same launch writes the samples of `sorted` (as launch_sample_keys) as
// PackedKeys right behind the header.
void launch_exch_header(const MapCounters* ctr, const ExchMsg1& tmpl, bool combined,
                        ExchMsg1* out, hipStream_t s, ConstKeysSoA sorted = ConstKeysSoA{},
                        const u32* d_n = nullptr, u32 num_samples = 0);
// offsets[p] = lower_bound(sorted, splitter[p-1]) for p in 1..P-1, offsets[0] = 0,
// offsets[P] = n.
void launch_bucket_offsets(ConstKeysSoA sorted, const u32* d_n, const PackedKey* splitters,
                           u32 num_buckets, u64* offsets, hipStream_t s);

// ---------------- exchange.hip (device-resident shuffle, locust/exch.hpp) ----------------
// Merge of nslots all-to-all slots (as launch_merge_slots) writing at most out_limit
// output records (counters still count all of them).
// The shuffle tail in two launches around the C3 all-gather:
// launch_merge_rank_slots merges the received slots into `merged` and sums the distinct
// keys / tokens / compact words into `acc`, kMergeAccSpread (firsts, tokens, words) u64
// triples (zeroed beforehand:
// launch_exch_report sums and re-zeroes them); launch_merge_emit_compact then writes this
// rank's range as compact
// records (kv.hpp) straight into the shared host output -- region `region` (or the root's,
// root_msg), word kOutWords x (region x region_records + the lower ranks' records) of
// `dst` -- and stamps `seq` when the whole range is out (locust/shm.hpp).  Nothing is
// written when a report flags a problem.  `lb`: merge_scratch_words status words + a tile
// counter, reset by launch_merge_rank_slots (a second emit of the same merge needs them
// zeroed again).
constexpr int kMergeAccSpread = 64;
void launch_merge_rank_slots(const KeyCount* slots, u32 nslots, u32 slot_records,
                             KeyCount* merged, u64* acc, LookbackScratch lb, hipStream_t s);
void launch_merge_emit_compact(const KeyCount* slots, u32 nslots, u32 slot_records,
                               const KeyCount* merged, const ExchMsg3* msg3_all,
                               const ExchMsg1* root_msg, u64 region, u32 regions,
                               u64 region_records, u32 P, u32 me, u32 gather_records, u64* dst,
                               u64* stamps, u64 seq, u32* done, LookbackScratch lb,
                               hipStream_t s);
void launch_exch_plan(const char* msg1_all, u32 P, u32 S, ConstKeysSoA keys, const u32* d_n,
                      u32 slot_records, ExchCtl* ctl, hipStream_t s,
                      u64* trace = nullptr);
void launch_exch_pack(const KeyCount* recs, const u32* d_n, u64 cap, const ExchCtl* ctl, u32 P,
                      u32 slot_records, char* send, hipStream_t s);
// (acc: launch_merge_rank_slots' accumulators, summed and re-zeroed here)
void launch_exch_report(const char* recv, u32 P, u32 slot_records, const ExchCtl* ctl,
                        u64* acc, u32 gather_records, ExchMsg3* msg3, hipStream_t s);
// ---- device self-test of the string library (tests only; StringTestOut in engine.hpp) ----
void launch_string_selftest(const char* blob, const u32* off, u32 n, const char* delims,
                            const int* ints, StringTestOut* out, hipStream_t s);

// ---------------- code-object warm-up ----------------
// The runtime loads a file's code object at the first launch of one of its kernels (lazy
// loading); a one-shot job would pay that inside its first kernels.  warm_kernel_modules()
// loads every kernel file of this library up front (engine construction) -- and only them:
// HIP_ENABLE_DEFERRED_LOADING=0 would also load the RCCL library's device code (a
// 573 MB fat binary), +1.3 GB of host memory and ~150 ms per process.
void warm_module_dict();
void warm_module_exchange();
void warm_module_map();
void warm_module_merge();
void warm_module_partplan();
void warm_module_psort();
void warm_module_radix_sort();
void warm_module_reduce();
void warm_module_shuffle();
void warm_module_signal();
void warm_module_tokenize();
inline void warm_kernel_modules() {
  warm_module_dict();
  warm_module_exchange();
  warm_module_map();
  warm_module_merge();
  warm_module_partplan();
  warm_module_psort();
  warm_module_radix_sort();
  warm_module_reduce();
  warm_module_shuffle();
  warm_module_signal();
  warm_module_tokenize();
}

}  // namespace locust
