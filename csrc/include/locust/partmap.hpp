// Host side of the partition map (PartMap, kernels.hpp): the order-preserving assignment
// of key ranges to the ordered dictionary kernel's kDictParts workgroups (and to the
// partitioned radix sort's).
//
// The reference has no counterpart -- its Process stage is one comparison sort over every
// record (/root/reference/MapReduce/src/main.cu:414-415).  Here each workgroup owns one key
// range; with ranges = first letters (the default) the 's'/'c'/'t' workgroups of English
// text carry 10-15 % of the tokens each and form the critical path while most others idle,
// and a large vocabulary puts thousands of distinct keys into one letter -- more than a
// workgroup's LDS table holds.  part_map_from_entries cuts the key space at the first key
// WORD (an 8-byte prefix) wherever the work or the distinct keys of a range reach their
// share: only keys sharing all of their first 8 bytes always stay together.
#pragma once

#include <cstddef>
#include <vector>

#include "locust/common.hpp"

namespace locust {

struct WordCountEntry;
class EntryList;

constexpr int kDictParts = 256;
constexpr u32 kPartDistinctWeight = 3;  // work of one distinct key, in tokens

// Device image of a partition map (one H2D copy): partition p holds the keys whose first
// word w0 satisfies lo[p] <= w0 < lo[p + 1]; lo[0] = 0, ascending (equal neighbours = an
// empty partition), lo[kDictParts] = ~0 (unused by the lookup).
struct PartMapTables {
  u64 lo[kDictParts + 1];
};

// Partition of a first key word: the largest p with lo[p] <= w0 (8-step binary search over
// lo[1..255]; monotone in w0, so partitions concatenate in key order).
LOCUST_HD inline u32 part_of_w0(const u64* lo, u64 w0) {
  u32 p = 0;
  for (u32 step = kDictParts / 2; step; step >>= 1)
    if (lo[p + step] <= w0) p += step;
  return p;
}

// The starting map (no key seen yet): letters split on their second byte, digits and
// UTF-8 lead bytes one partition each (partmap.cpp).
void part_map_default(PartMapTables* t);
// partition = first key byte (the round-2 default; A/B and tests)
void part_map_default_first_byte(PartMapTables* t);

// Balanced map from a job's sorted (key, count) output: greedy key ranges of ~total/256
// work (count + kPartDistinctWeight per distinct key, the ordered kernel's part_w measure)
// and at most `max_distinct` distinct keys each, cut only between different first words.
// Returns the largest partition's predicted work (0 for no entries: default map).
u64 part_map_from_entries(const EntryList& e, PartMapTables* t, u32 max_distinct = 1024);
// The same in two steps: the output's first-word groups (one pass; the retune worker makes
// them first and then lets go of the job's output buffer), and the map from them.
struct PartGroup {  // the distinct keys sharing one first word
  u64 w0, work;
  u32 distinct;
};
void part_map_groups(const EntryList& e, std::vector<PartGroup>* g);
u64 part_map_from_groups(const std::vector<PartGroup>& g, PartMapTables* t,
                         u32 max_distinct = 1024);

inline u32 part_map_lookup(const PartMapTables& t, u64 w0) { return part_of_w0(t.lo, w0); }

}  // namespace locust
