// Partition-map construction (see locust/partmap.hpp).
#include "locust/partmap.hpp"

#include <algorithm>
#include <cstring>
#include <vector>

#include "locust/engine.hpp"

namespace locust {

void part_map_default(PartMapTables* t) {
  std::memset(t, 0, sizeof(*t));
  for (u32 c = 0; c < 256; ++c) t->base[c] = (u8)c;
  for (u32 p = 0; p <= (u32)kDictParts; ++p) t->lo[p] = p << 8;
}

namespace {

// One greedy pass with target work `target` per partition; returns the number of
// partitions and the largest partition's work.
// Mid-row splits the greedy would make in row c with `target`, starting from the work
// (acc, accd) carried into the row.
u32 row_splits(const u64* weight, const u32* distinct, u32 c, u64 target, u32 max_distinct,
               u64 acc, u64 accd) {
  u32 n = 0;
  for (u32 d = 0; d < 256; ++d) {
    const u32 b = (c << 8) | d;
    if (acc > 0 && (acc + weight[b] > target || accd + distinct[b] > max_distinct)) {
      if (d != 0) ++n;
      acc = accd = 0;
    }
    acc += weight[b];
    accd += distinct[b];
  }
  return n;
}

u32 assign(const u64* weight, const u32* distinct, u64 target, u32 max_distinct,
           PartMapTables* t, u64* max_work) {
  u32 pid = 0;
  u64 acc = 0, accd = 0, worst = 0;
  for (u32 c = 0; c < 256; ++c) {
    u32 nthr = 0;
    u64 thr = 0;
    // A row that wants more than kPartMaxThr splits (a hot first letter: 's', 't') gets a
    // coarser target of its own, so its splits spread over the whole row instead of the
    // thresholds running out half way and the row's tail landing in one partition.
    u64 rt = target;
    while (row_splits(weight, distinct, c, rt, max_distinct, acc, accd) > (u32)kPartMaxThr)
      rt += rt / 16 + 1;
    for (u32 d = 0; d < 256; ++d) {
      const u32 b = (c << 8) | d;
      const u64 w = weight[b];
      const u64 dd = distinct[b];
      if (acc > 0 && (acc + w > rt || accd + dd > max_distinct)) {
        // start a new partition at b: free at a row start, one threshold mid-row
        if (d == 0 || nthr < (u32)kPartMaxThr) {
          worst = std::max(worst, acc);
          ++pid;
          acc = accd = 0;
          if (d != 0) thr |= (u64)d << (8 * nthr++);
        }
      }
      if (d == 0) t->base[c] = (u8)std::min<u32>(pid, 255);
      acc += w;
      accd += dd;
    }
    t->thr[c] = thr;
  }
  worst = std::max(worst, acc);
  *max_work = worst;
  return pid + 1;
}

}  // namespace

u64 part_map_build(const u64* weight, const u32* distinct, PartMapTables* t, u32 max_distinct) {
  u64 total = 0;
  for (u32 b = 0; b < 65536; ++b) total += weight[b];
  part_map_default(t);
  if (!total) return 0;
  u64 target = std::max<u64>(1, (total + kDictParts - 1) / kDictParts);
  u64 worst = 0;
  for (int tries = 0; tries < 200; ++tries) {
    PartMapTables cand;
    std::memset(&cand, 0, sizeof(cand));
    const u32 parts = assign(weight, distinct, target, max_distinct, &cand, &worst);
    if (parts <= (u32)kDictParts) {
      // lo[p]: first prefix of partition p (empty trailing partitions start at 65536)
      for (u32 p = 0; p <= (u32)kDictParts; ++p) cand.lo[p] = 65536;
      for (u32 b = 65536; b-- > 0;) cand.lo[part_map_lookup(cand, b)] = b;
      for (u32 p = (u32)kDictParts; p-- > 0;)
        if (cand.lo[p] > cand.lo[p + 1]) cand.lo[p] = cand.lo[p + 1];
      cand.lo[0] = 0;
      *t = cand;
      return worst;
    }
    target += target / 16 + 1;  // too many partitions: coarser ranges
  }
  return 0;  // unreachable in practice: the default map stays
}

u64 part_map_from_entries(const WordCountEntry* e, size_t n, PartMapTables* t) {
  std::vector<u64> w(65536, 0);
  std::vector<u32> d(65536, 0);
  for (size_t i = 0; i < n; ++i) {
    const u32 b = (u32)(e[i].key.w[0] >> 48);
    w[b] += e[i].count + kPartDistinctWeight;
    d[b] += 1;
  }
  return part_map_build(w.data(), d.data(), t);
}

}  // namespace locust
