// Synthetic text generator for the large WordCount configurations (SURVEY.md §2.1 C35,
// §5.7; BASELINE.json configs "1M-line synthetic text" and "10 GB synthetic text").
//
// The reference only ships hamlet.txt (4,463 lines).  The generated text has Hamlet's
// shape: lines of 0..99 characters, a Zipfian vocabulary (a few words carry most of the
// tokens, as "the" is 3% of Hamlet), English-like word lengths, some capitalised words
// (distinct keys, the reference does not fold case), punctuation from the reference's
// delimiter set and a few characters outside it ('!', '?') that stay inside tokens.
//
// Generation is deterministic in (seed, block of 1,024 lines): the same spec gives the
// same bytes for any thread count, and a rank can generate just its own shard.
#pragma once

#include <string>
#include <vector>

#include "locust/common.hpp"

namespace locust {

struct GenSpec {
  u64 lines = 0;          // target line count (used when > 0)
  u64 bytes = 0;          // else: target size; the text is cut at the last full line
  u64 seed = 1;
  u32 vocab = 50000;      // distinct base words (capitalisation adds variants)
  double zipf_s = 1.0;    // word frequency ~ 1 / rank^s
  u32 max_line_chars = 99;  // the reference's value[100] line width (KeyValue.h:9)
  u32 threads = 0;        // 0: hardware concurrency
  u64 first_block = 0;    // generate blocks [first_block, ...): a shard of a larger text
};

constexpr u64 kGenBlockLines = 1024;

// Appends the generated text to `out`; returns the number of lines.
u64 gen_text(const GenSpec& spec, std::string* out);
// Into a caller buffer of `cap` bytes (e.g. pinned host memory).  Stops at the spec's
// target or at the last full line that fits.  Returns bytes written; *lines gets the count.
u64 gen_text_into(const GenSpec& spec, char* buf, u64 cap, u64* lines);

// The base vocabulary (rank order) -- exposed for tests.
std::vector<std::string> gen_vocabulary(u32 vocab, u64 seed);

}  // namespace locust
