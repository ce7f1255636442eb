// Partition-map construction (see locust/partmap.hpp).
#include "locust/partmap.hpp"

#include <algorithm>
#include <vector>

#include "locust/engine.hpp"

namespace locust {

void part_map_default(PartMapTables* t) {
  for (u32 p = 0; p < (u32)kDictParts; ++p) t->lo[p] = (u64)p << 56;
  t->lo[kDictParts] = ~0ull;
}

namespace {

struct Group {  // the distinct keys sharing one first word
  u64 w0, work;
  u32 distinct;
};

// One greedy sweep with target work `target`; fills lo[] when the ranges fit into
// kDictParts partitions and returns their count (else kDictParts + 1).
u32 assign(const std::vector<Group>& g, u64 target, u32 max_distinct, PartMapTables* t,
           u64* worst) {
  u32 p = 0;
  u64 acc = 0, accd = 0, w = 0;
  t->lo[0] = 0;
  for (const Group& x : g) {
    if (acc > 0 && (acc + x.work > target || accd + x.distinct > max_distinct)) {
      w = std::max(w, acc);
      if (++p >= (u32)kDictParts) return kDictParts + 1;
      t->lo[p] = x.w0;
      acc = accd = 0;
    }
    acc += x.work;
    accd += x.distinct;
  }
  w = std::max(w, acc);
  for (u32 q = p + 1; q <= (u32)kDictParts; ++q) t->lo[q] = ~0ull;  // empty tail
  *worst = w;
  return p + 1;
}

}  // namespace

u64 part_map_from_entries(const WordCountEntry* e, size_t n, PartMapTables* t,
                          u32 max_distinct) {
  part_map_default(t);
  std::vector<Group> g;
  u64 total = 0;
  for (size_t i = 0; i < n; ++i) {
    const u64 w0 = e[i].key.w[0];
    const u64 work = e[i].count + kPartDistinctWeight;
    if (g.empty() || g.back().w0 != w0) g.push_back({w0, 0, 0});
    g.back().work += work;
    g.back().distinct += 1;
    total += work;
  }
  if (!total) return 0;
  u64 target = std::max<u64>(1, (total + kDictParts - 1) / kDictParts);
  for (int tries = 0; tries < 400; ++tries) {
    PartMapTables cand;
    u64 worst = 0;
    if (assign(g, target, max_distinct, &cand, &worst) <= (u32)kDictParts) {
      *t = cand;
      return worst;
    }
    target += target / 16 + 1;  // too many ranges: coarser
    if (tries > 100) max_distinct += max_distinct / 8 + 1;
  }
  return 0;  // unreachable in practice: the default map stays
}

}  // namespace locust
