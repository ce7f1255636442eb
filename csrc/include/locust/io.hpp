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

// ---- spill files (map-output checkpoint) ----
enum class SpillFormat { kText, kBinary, kKiv };
// Text: the reference's "%s \t%d\n" (one line per record).  Binary: 32-byte header
// ("LCSTSPL1", version, key words, record count) then 40-B KeyCount records.  Kiv: the
// reference's own 40-B record, KeyIntValuePair (/root/reference/MapReduce/src/
// KeyValue.h:13-18: char key[30], int value @32, int count @36), after a 32-byte header
// ("LCSTKIV1", version, record size 40, record count); a spill stores value = the
// record's count and count = 0, as the reference's map emits (key, 1, 0).
void write_spill(const std::string& path, const std::vector<KeyCount>& recs, SpillFormat fmt);
// Reads any of the three (detected by magic).  Text keys lose the writer's trailing space.
std::vector<KeyCount> read_spill(const std::string& path);
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
std::vector<PackedKey> records_to_tokens(const std::vector<KeyCount>& recs);

// ---- output ----
// GPU build format (main.cu:132): "print key: %s \t val: %d \t count: %d\n".
void format_gpu_output(const WordCountResult& r, std::string* out);
// CPU build format (main.cu:286): "print key: %s \t value: %s\n" with value = count.
void format_cpu_output(const WordCountResult& r, std::string* out);
void write_all(std::FILE* f, const std::string& s);

std::string key_to_string(const PackedKey& k);

}  // namespace locust
