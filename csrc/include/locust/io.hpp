// Host I/O: input loader with line windows, intermediate spill files, output printer.
//
// Reference (/root/reference/MapReduce/src/main.cu:40-134):
//   loadFile             getline loop into a fixed 5,800-slot stack array; whole-file mode
//                        drops the last line (B1); window [line_start, line_end).
//   writeKeyIntValues    "%s \t%d\n" per non-empty record -> /tmp/out.txt
//   loadIntermediateFile split at the first TAB (key keeps the trailing space, B8)
//   printKeyIntValues    "print key: %s \t val: %d \t count: %d\n"
#pragma once

#include <cstdio>
#include <string>
#include <vector>

#include "locust/engine.hpp"

namespace locust {

struct LoadedText {
  std::vector<char> storage;  // the selected lines, '\n'-separated
  TextInput input;            // points into storage
  u64 file_lines = 0;         // lines in the whole file
  bool window = false;        // a [line_start, line_end) window was requested
};

// line_start < 0 selects the whole file.  With ref_compat the reference's line-count
// quirks are reproduced (B1: the whole-file load and a window running past EOF lose the
// last line).  A window is read block by block up to its last line and keeps only its own
// bytes (file_lines then counts the lines scanned); the whole file is read with parallel
// preads straight into the result.
LoadedText load_lines(const std::string& path, i64 line_start, i64 line_end, bool ref_compat);
// Bytes of a file (throws if it cannot be opened).
u64 file_size(const std::string& path);
// The whole file into dst (room for cap bytes) by parallel preads; returns its size and
// sets *lines (a final line without '\n' counts).  dst may be pinned memory.
u64 read_file_into(const std::string& path, char* dst, u64 cap, u64* lines, u32 threads = 0);
// Per-rank input shards of a file: P byte ranges cut at line starts,
// found by reading small windows around the P-1 cut points only.  A line never spans two
// ranges; a range may be empty (more ranks than lines).
struct FileRange {
  u64 offset = 0, bytes = 0;
};
std::vector<FileRange> file_shards(const std::string& path, int parts);
// [off, off + n) of a file into dst by parallel preads; sets *lines like read_file_into.
u64 read_file_range_into(const std::string& path, char* dst, u64 off, u64 n, u64* lines,
                         u32 threads = 0);
LoadedText text_from_buffer(const char* data, u64 bytes, i64 line_start, i64 line_end,
                            bool ref_compat);
u64 count_lines(const char* data, u64 bytes);
// The '\n' bytes of [data, data + bytes): 32 bytes per compare with AVX2 when the CPU has it
// (16 with SSE2), counts summed in byte lanes -- the streamed reads count every piece's
// newlines, and std::count's scalar loop ran at ~1 GB/s per thread (tools/read_probe.cpp).
u64 count_newlines(const char* data, u64 bytes);
// The byte range [begin, end) of the line window [line_start, line_end) of a file (the
// reference's per-node line ranges, main.cu:369-374) and its line count, found by a parallel
// newline scan in bounded memory (never the whole file in memory).  line_end < 0: to the
// end of the file.  The scan starts from a per-file sparse line index (the newline count
// at every 8 MiB block start, cached under the file's identity like the partition map:
// line_index_cache_path), so only the first window that passes a block pays for it.
struct LineWindow {
  u64 begin = 0, end = 0;  // bytes
  u64 lines = 0;           // lines in [begin, end) (a final line without '\n' counts)
};
LineWindow find_line_window(const std::string& path, i64 line_start, i64 line_end,
                            u32 threads = 0);
// The sparse line index's cache file ("" when disabled: LOCUST_LINE_CACHE=0, or no cache
// directory / no such file).  Same directory rules as partmap_cache_path.
std::string line_index_cache_path(const std::string& input);
// The first line start at or after byte `off`: off when off == 0 or byte off-1 is '\n',
// else just after the next '\n' (the file size when there is none).
u64 line_start_at(const std::string& path, u64 off);
// A byte window [begin, end) of a file moved to line starts (line_start_at of both ends),
// exactly as file_shards cuts: windows [a0, a1), [a1, a2), ... of any offsets hold every
// line once.  Only the bytes from each end to its next newline are read; lines = 0 (the
// reader of the range counts them).
LineWindow byte_window(const std::string& path, u64 begin, u64 end);

// ---- spill files (map-output checkpoint) ----
enum class SpillFormat { kText, kBinary, kKiv };
// Text: the reference's "%s \t%d\n" (one line per record).  Binary: 32-byte header
// ("LCSTSPL1", version, key words, record count) then 40-B KeyCount records.  Kiv: the
// reference's own 40-B record, KeyIntValuePair (/root/reference/MapReduce/src/
// KeyValue.h:13-18: char key[30], int value @32, int count @36), after a 32-byte header
// ("LCSTKIV1", version, record size 40, record count); a spill stores value = the
// record's count and count = 0, as the reference's map emits (key, 1, 0).
//
// Stage 1 writes its COMBINED map output: one record per distinct key with its count, in
// key order (the reference writes one "key \t1" line per token, main.cu:421-433; --ref-compat
// keeps that).  Next to every spill it writes a sparse index, <spill>.idx: every stride-th
// record's key, record number, byte offset and the token count of the records before it.
// A reducer seeks with it to its key range and knows the count of every smaller key (its
// global val base) without reading them; the samples also give the reducers' splitters.
struct SpillSample {
  PackedKey key;
  u64 record = 0, offset = 0, count_before = 0;
};
struct SpillIndex {
  bool sorted = false;     // keys never decrease
  bool distinct = false;   // and never repeat
  u64 records = 0, total_count = 0;
  u64 spill_bytes = 0;     // size of the spill it describes (a stale index is ignored)
  u64 stride = 1;
  std::vector<SpillSample> samples;  // samples[0] is record 0
};
// Writes the spill; with idx, also fills it (the caller writes it with write_spill_index).
void write_spill(const std::string& path, const std::vector<KeyCount>& recs, SpillFormat fmt,
                 SpillIndex* idx = nullptr);
std::string spill_index_path(const std::string& spill);
void write_spill_index(const std::string& path, const SpillIndex& idx);
// False when absent, unreadable or not matching the spill's current size.
bool read_spill_index(const std::string& spill, SpillIndex* idx);
// Reads any of the three (detected by magic).  Text keys lose the writer's trailing space.
std::vector<KeyCount> read_spill(const std::string& path);
// Sequential reader of any spill format from a record's byte offset (an index sample's).
class SpillReader {
 public:
  explicit SpillReader(const std::string& path);
  ~SpillReader();
  SpillReader(const SpillReader&) = delete;
  SpillReader& operator=(const SpillReader&) = delete;
  SpillFormat format() const { return fmt_; }
  u64 first_record_offset() const { return first_; }
  u64 bytes() const { return size_; }
  void seek(u64 offset);
  // The next record and its byte offset; false at the end.
  bool next(KeyCount* rec, u64* offset = nullptr);

 private:
  bool fill();
  std::string path_;
  std::FILE* f_ = nullptr;
  SpillFormat fmt_ = SpillFormat::kText;
  u64 size_ = 0, first_ = 0, pos_ = 0;  // pos_: file offset of buf_[at_]
  std::vector<char> buf_;
  size_t at_ = 0, len_ = 0;
};
// Final (key, val, count) results as KeyIntValuePair records (value = val), the reference's
// reduce output array (main.cu:470-473); the same header.  Values past INT_MAX and keys
// past 29 bytes are refused.
void write_kiv_results(const std::string& path, const WordCountResult& r);
// KeyIntValuePair records of a kiv file: (key, value, count).
struct KivRecord {
  PackedKey key;
  i64 value, count;
};
std::vector<KivRecord> read_kiv(const std::string& path);
std::vector<KeyCount> tokens_to_records(const std::vector<PackedKey>& toks);
std::vector<KeyCount> entries_to_records(const EntryList& e);

// Records in packed-key order (== the reference's unsigned byte order, KeyValue.h:23-28).
inline bool record_less(const KeyCount& a, const KeyCount& b) { return key_compare(a.w, b.w) < 0; }

// ---- per-file partition-map cache (the one-shot CLI) ----
// A process of `./MapReduce <file>` runs one job, on the data-independent starting map;
// the map tuned from its output (a load-balancing hint, kDictParts + 1 words) is kept in
// a small cache keyed by the input file's identity (real path, size, mtime, inode) and the
// job's tokenizer settings, so the next run on the same file starts tuned -- the role
// MIOpen's performance database plays for its kernels.  A stale or damaged entry can only
// cost speed: any ascending map gives the same results.  Directory: LOCUST_CACHE_DIR, else
// $XDG_CACHE_HOME/locust, else ~/.cache/locust; LOCUST_PART_CACHE=0 disables it ("").
std::string partmap_cache_path(const std::string& input, const JobConfig& cfg);
bool load_partmap_cache(const std::string& path, std::vector<u64>* lo);
void save_partmap_cache(const std::string& path, const std::vector<u64>& lo);  // best effort

// ---- output ----
// GPU build format (main.cu:132): "print key: %s \t val: %d \t count: %d\n".
void format_gpu_output(const WordCountResult& r, std::string* out);
// CPU build format (main.cu:286): "print key: %s \t value: %s\n" with value = count.
void format_cpu_output(const WordCountResult& r, std::string* out);
void write_all(std::FILE* f, const std::string& s);

std::string key_to_string(const PackedKey& k);

}  // namespace locust
