// Runtime job configuration.
//
// The reference fixes everything at compile time (/root/reference/MapReduce/src/
// main.cu:18-37: MAX_LINES_FILE_READ=5800, EMITS_PER_LINE=20, GPU_IMPLEMENTATION,
// SHARE_MEMORY, GRID_SIZE=128, BLOCK_SIZE=256).  Here every switch is a runtime field of
// JobConfig (CLI flags and LOCUST_* env vars map onto it) and there is no
// line cap: buffers are sized from the input.
#pragma once

#include <string>

#include "locust/common.hpp"
#include "locust/dstring.hpp"

namespace locust {

enum class Backend { kGpu, kCpu };

// Reduce-stage boundary/adjacent-difference kernels: LDS-staged tiles (the reference's
// SHARE_MEMORY=1 column of README.md:84-88) or plain global loads (SHARE_MEMORY=0).
enum class ReducePath { kLds, kGlobal };

// Map kernel: kCompat = one thread per line running device strtok_r into fixed
// [line*E + k] slots (reference layout, main.cu:136-159) followed by a scan-based
// compaction; kFast = wave-cooperative byte-parallel tokenizer that emits compacted
// tokens in one pass (decoupled look-back).
enum class MapPath { kCompat, kFast };

// Process-stage key sort: kRadix = LSD radix sort of packed keys (8-bit digits, constant
// digit positions skipped); kDict = dictionary sort: hash the keys into a GPU table,
// rank only the distinct keys (all-pairs weighted rank, or radix past 32K distinct); the
// output (val = start of the key's run in the sorted token order) follows from the ranks.
enum class SortPath { kRadix, kDict };

struct JobConfig {
  Backend backend = Backend::kGpu;
  int device = 0;
  int emits_per_line = 20;                   // EMITS_PER_LINE (main.cu:19)
  int max_key_len = kMaxKeyLen;              // longer tokens are truncated and counted
  std::string delimiters = kDefaultDelims;   // main.cu:138
  bool ref_compat = false;                   // reproduce B1: whole-file load drops last line
  ReducePath reduce_path = ReducePath::kLds;
  MapPath map_path = MapPath::kFast;
  SortPath sort_path = SortPath::kDict;
  bool combine = false;                      // map-side combine (distributed shuffle)
  bool check = false;                        // LOCUST_CHECK invariants after each stage
  bool sync_plan = true;                     // read the sort plan back: launch only live passes
  // > 0: a device pass holds at most this many text bytes; larger inputs stream through
  // in line-aligned chunks (dictionary path).  0: one pass holds the whole input.
  u64 chunk_bytes = 0;
  // Streamed files: bytes per piece of the pinned read ring (0: 16 MiB).  Ranks of one
  // process each keep a ring, so `MapReduce <file> --gpus N` shrinks it with N.
  u64 ring_piece_bytes = 0;
  // Map input read straight from pinned host memory instead of an H2D copy: -1 auto
  // (inputs <= kZeroCopyMaxBytes), 0 never, 1 always (fast map path only).
  int zero_copy_text = -1;
  // Replay the dictionary job as one captured hipGraph (one launch instead of ~6 launches
  // and 6 event records): -1 auto (dictionary path, fast map), 0 off, 1 on.  Per-stage
  // times are then not split (StageTimes.gpu_ms has the whole device time).
  int graph = -1;
  // Also take host timers where the reference put them (main.cu:405-468, BASELINE.md "How
  // the reference measured these"): Map = kernel launch only, Process = until the sort is
  // done (includes the map kernel), Reduce = until the last reduce kernel is LAUNCHED.
  // Adds host synchronisations, so it is a separate measurement mode.
  bool ref_timers = false;
  // Engines sharing one GPU's HBM (ranks of one process on one device): each plans its
  // device pass against free memory / hbm_share (plan_device_pass, engine.hpp).
  int hbm_share = 1;
  // An engine that only merges (key, count) records -- stage 2's device merge: no text is
  // ever uploaded, so construction skips the text buffer, the spare output buffers and the
  // piecewise upload's copy queues (two hardware queues and their warm-up copies: 50 ms of
  // a reducer's ~90 ms setup, measured).
  bool records_only = false;
};
constexpr u64 kZeroCopyMaxBytes = 1ull << 20;

// Fills the fields that have LOCUST_* environment overrides (LOCUST_CHECK=1,
// LOCUST_REDUCE_PATH=lds|global, LOCUST_MAP_PATH=compat|fast, LOCUST_SORT=radix|dict).
void apply_env_overrides(JobConfig& cfg);

const char* to_string(ReducePath p);
const char* to_string(MapPath p);
const char* to_string(SortPath p);

}  // namespace locust
