// Stage-split execution: the reduce side of the reference's two-stage protocol
// (/root/reference/MapReduce/src/main.cu:421-446, README.md:24-29).
//
// The reference's stage 2 reads one "/tmp/out.txt" of per-token "key \t1" lines and counts
// runs by position without sorting (B7).  Here stage 1 spills its combined, sorted
// (key, count) output with a sparse index (io.hpp SpillIndex), and stage 2 treats every
// spill as a sorted run: it reads its key range of each spill (an index seek), merges the
// runs summing counts -- on the device (launch_merge_sorted_runs, rounds of <= 64 runs,
// key-range splits past the kernel's record limit) or on the host -- and never expands a
// count into tokens.  Spills without an index, or unsorted ones (a reference-format file
// written elsewhere), are read whole and sorted/combined first.
//
// Key-range reducers (the GIF's design, README.md:29): with R reducers, reducer r keeps the
// keys in [splitter[r-1], splitter[r]), the splitters cut the index samples of all spills at
// equal record weight (every reducer computes the same ones), and its global val base is
// the count of every smaller key -- from the index's count_before plus the records between
// the sample and its range start.  Concatenating reducers 0..R-1 gives the single-stage
// output byte for byte, val included.
#pragma once

#include <memory>
#include <string>
#include <vector>

#include "locust/engine.hpp"
#include "locust/io.hpp"

namespace locust {

// Sorts by key and sums the counts of equal keys (keys strictly increase afterwards).
void sort_combine(std::vector<KeyCount>* recs);
// Sums adjacent equal keys of a sorted vector.
void combine_adjacent(std::vector<KeyCount>* recs);
// k-way merge of sorted runs with distinct keys each; equal keys across runs are summed.
std::vector<WordCountEntry> merge_runs_host(const std::vector<std::vector<KeyCount>>& runs);
// The same on the device (GpuWordCount::merge_runs): rounds of <= 64 runs, split by key
// range past the merge kernel's record limit.  `cfg` picks the device; *setup_ms gets the
// engine construction time (the rest is the merge).
std::vector<WordCountEntry> merge_runs_device(const JobConfig& cfg,
                                              const std::vector<std::vector<KeyCount>>& runs,
                                              double* setup_ms = nullptr);
// An index for a spill held in memory (sorted, distinct records; samples every stride-th).
SpillIndex index_records(const std::vector<KeyCount>& recs);
// reducers - 1 splitter keys cutting the samples of all indexes at equal record weight
// (independent of the order of `idx`).
std::vector<PackedKey> plan_reducer_splitters(const std::vector<SpillIndex>& idx, int reducers);

// ---- stage 1 ----
// The part of the input a map stage reads: a line window (the reference's per-node line
// ranges, main.cu:369-374) or a byte window whose ends move to line starts (byte_window),
// which a launcher gets from the file size alone -- no newline scan of the prefix.
struct MapWindow {
  i64 line_start = -1, line_end = -1;  // line_start < 0: no line window
  bool by_bytes = false;
  u64 byte_begin = 0, byte_end = ~0ull;
};
struct MapStageResult {
  WordCountResult result;  // counts and stage times (entries released after the spill)
  u64 lines = 0, input_bytes = 0;
  u64 byte_begin = 0, byte_end = 0;  // the bytes of the file mapped
  u64 spill_records = 0;
  bool streamed = false;   // the window streamed through the engine (larger than a pass)
  double job_ms = 0, spill_write_ms = 0;
  // job_ms = window_ms (finding the window's bytes) + setup_ms (engine construction) +
  // run_ms (read / stream + map + combine) + the records' copy out of the engine
  double window_ms = 0, setup_ms = 0, run_ms = 0;
  SpillIndex index;
  GpuWordCount::Stats engine;  // the GPU engine's HBM plan (device bytes, free HBM, chunks)
  // the GPU engine itself, alive until the last copy of the result goes (a one-shot CLI
  // leaks it into its _exit instead of tearing it down)
  std::shared_ptr<void> engine_keep;
};
// Stage 1 over a window of `file` (none: the whole file): the job's combined output -- one
// (key, count) record per distinct key, key order -- spilled to `spill` in `fmt`, with its
// index at spill_index_path(spill).  GPU: the window's bytes (find_line_window or
// byte_window) are read into the engine's pinned buffer, or streamed past one device pass
// (chunk_bytes, default 256 MiB), with hipEvent stage times.  cfg.ref_compat: the
// reference's spill instead -- one record per token, sorted -- from the reference's loader
// (the CPU build ignores the window and drops the last line, B1); not with a byte window.
MapStageResult map_stage(const JobConfig& cfg, const std::string& file, const MapWindow& win,
                         const std::string& spill, SpillFormat fmt);
inline MapStageResult map_stage(const JobConfig& cfg, const std::string& file, i64 line_start,
                                i64 line_end, const std::string& spill, SpillFormat fmt) {
  MapWindow w;
  w.line_start = line_start;
  w.line_end = line_end;
  return map_stage(cfg, file, w, spill, fmt);
}

struct ReduceStageStats {
  u64 input_files = 0, indexed_files = 0, loaded_files = 0;
  u64 records_read = 0;  // spill records read (below the range and inside it)
  u64 run_records = 0;   // records merged
  double read_ms = 0, setup_ms = 0, merge_ms = 0;  // merge_ms excludes setup_ms
  std::vector<PackedKey> splitters;
};
// Stage 2 of reducer `reducer` of `reducers` over the spills `files`: the merged entries
// of its key range, val_base = the token count of all smaller keys.  The GPU backend
// merges on the device, the CPU backend on the host.
WordCountResult reduce_spills(const JobConfig& cfg, const std::vector<std::string>& files,
                              int reducer, int reducers, ReduceStageStats* stats = nullptr);

}  // namespace locust
