// Host side of the partition map (PartMap, kernels.hpp): the order-preserving assignment
// of 2-byte key prefixes to the ordered dictionary kernel's kDictParts workgroups.
//
// The reference has no counterpart -- its Process stage is one comparison sort over every
// record (/root/reference/MapReduce/src/main.cu:414-415).  Here the Process+Reduce kernel
// gives each workgroup one key range; with ranges = first letters (the default) the
// 's'/'c'/'t' workgroups of English text carry 10-15 % of the tokens each and form the
// critical path while most others idle.  part_map_build splits hot letters by their second
// byte and merges rare ones so every workgroup gets ~1/256 of the work.
#pragma once

#include <cstddef>

#include "locust/common.hpp"

namespace locust {

struct WordCountEntry;

// The ordered dictionary build gives each of its kDictParts workgroups one PARTITION of
// the key space: a contiguous range of 2-byte key prefixes, so concatenating the
// partitions in order is the global key order.  partition(c, d) = base[c] +
// #{ thresholds t of row c : t != 0 && t <= d }, at most kPartMaxThr thresholds per first
// byte c, so the lookup is 2.3 KB of table that the map kernel stages in LDS.  lo[p] =
// first 2-byte prefix of partition p (lo[kDictParts] = 65536), for the in-partition sort.
constexpr int kDictParts = 256;
constexpr int kPartMaxThr = 8;
constexpr u32 kPartDistinctWeight = 3;  // work of one distinct key, in tokens
LOCUST_HD inline u32 part_of_prefix(u32 c, u32 d, u32 base, u64 thr) {
  u32 n = 0;
  for (int i = 0; i < kPartMaxThr; ++i) {  // constant trip count: unrolled at -O3
    const u32 t = (u32)(thr >> (8 * i)) & 0xffu;
    n += (t != 0u && t <= d) ? 1u : 0u;
  }
  return base + n;
}

// Device image of a partition map (one H2D copy): base[256], thr[256], lo[257].
struct PartMapTables {
  u64 thr[256];
  u32 lo[kDictParts + 1];
  u8 base[256];
};

// partition = first key byte (what the ordered kernel did before balancing)
void part_map_default(PartMapTables* t);

// Balanced map from per-2-byte-prefix work (`weight`, 65,536 entries) and distinct-key
// counts (`distinct`): greedy ranges of ~total/256 work, at most kPartMaxThr splits per
// first byte, at most `max_distinct` distinct keys per partition where splitting allows.
// Returns the largest partition's predicted work.
u64 part_map_build(const u64* weight, const u32* distinct, PartMapTables* t,
                   u32 max_distinct = 1024);

// The same from a job's sorted (key, count) output: work = count + kPartDistinctWeight per
// distinct key (the ordered kernel's part_w measure).
u64 part_map_from_entries(const WordCountEntry* e, size_t n, PartMapTables* t);

// Partition of a 2-byte prefix under `t` (host mirror of the device lookup).
inline u32 part_map_lookup(const PartMapTables& t, u32 prefix) {
  return part_of_prefix(prefix >> 8, prefix & 0xffu, t.base[prefix >> 8], t.thr[prefix >> 8]);
}

}  // namespace locust
