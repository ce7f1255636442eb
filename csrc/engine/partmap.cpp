// Partition-map construction (see locust/partmap.hpp).
#include "locust/partmap.hpp"

#include <algorithm>
#include <cstdlib>
#include <vector>

#include "locust/engine.hpp"

namespace locust {

void part_map_default_first_byte(PartMapTables* t) {
  for (u32 p = 0; p < (u32)kDictParts; ++p) t->lo[p] = (u64)p << 56;
  t->lo[kDictParts] = ~0ull;
}

// The map a job starts from before anything is known about its keys (a fresh engine's
// first job -- every `./MapReduce <file>` -- and LOCUST_PART_TUNE=0).  Words start with a
// letter far more often than with any other byte, so the letters get several partitions
// each, cut on the second byte: lowercase four ([.., 'g'), ['g', 'n'), ['n', 't'),
// ['t', ..)), uppercase three (ALL-CAPS words / [a-m] / [n-z] second letters); digits and
// every UTF-8 lead byte (0xC2-0xF4) one each; the remaining byte ranges one each.  248
// partitions (asserted below); the rest stay empty.  A first-byte map left ~50 of the 256
// partitions occupied on English text, so the ordered kernel split the hot letters across
// sibling workgroups that each scan the whole letter's tokens (whole Hamlet: ordered
// kernel 28.1 vs 22.1 us with a tuned map, profiles/r3_s4/).  Data-independent: no input
// is sampled.  Round 5 added third-byte cuts fitted to Hamlet ('th', 'co' words); on 7
// held-out texts they were 0.998-1.040x the plain letters map and helped only the fixture
// (profiles/r6/partmap/heldout.md), so round 6 removed them.  The letters map beat the
// first-byte map on 7 of the 8 texts there (LOCUST_PART_DEFAULT=byte keeps that A/B).
void part_map_default(PartMapTables* t) {
  if (const char* e = std::getenv("LOCUST_PART_DEFAULT"); e && e[0] == 'b')  // A/B: "byte"
    return part_map_default_first_byte(t);
  std::vector<u64> lo;
  auto cut = [&](u32 b0, u32 b1) { lo.push_back(((u64)b0 << 56) | ((u64)b1 << 48)); };
  cut(0x00, 0);    // controls, space, punctuation before the digits
  for (u32 d = '0'; d <= '9'; ++d) cut(d, 0);
  cut(0x3A, 0);    // :;<=>?@
  for (u32 c = 'A'; c <= 'Z'; ++c) {
    cut(c, 0);
    cut(c, 'a');
    cut(c, 'n');
  }
  cut(0x5B, 0);    // [\]^_`
  for (u32 c = 'a'; c <= 'z'; ++c) {
    cut(c, 0);
    cut(c, 'g');
    cut(c, 'n');
    cut(c, 't');
  }
  cut(0x7B, 0);    // {|}~ DEL, UTF-8 continuation bytes, C0/C1
  for (u32 b = 0xC2; b <= 0xF4; ++b) cut(b, 0);
  cut(0xF5, 0);    // bytes no UTF-8 text starts with
  LOCUST_CHECK_ARG(lo.size() == 248u && lo.size() <= (size_t)kDictParts,
                   "default partition map: unexpected partition count");
  for (u32 p = 0; p < (u32)kDictParts; ++p) t->lo[p] = p < lo.size() ? lo[p] : ~0ull;
  t->lo[kDictParts] = ~0ull;
}

namespace {

using Group = PartGroup;

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

void part_map_groups(const EntryList& entries, std::vector<PartGroup>* out) {
  std::vector<Group>& g = *out;
  g.clear();
  for (const WordCountEntry e : entries) {  // compact lists decode on the fly
    const u64 w0 = e.key.w[0];
    const u64 work = e.count + kPartDistinctWeight;
    if (g.empty() || g.back().w0 != w0) g.push_back({w0, 0, 0});
    g.back().work += work;
    g.back().distinct += 1;
  }
}

u64 part_map_from_entries(const EntryList& entries, PartMapTables* t, u32 max_distinct) {
  std::vector<Group> g;
  part_map_groups(entries, &g);
  return part_map_from_groups(g, t, max_distinct);
}

u64 part_map_from_groups(const std::vector<PartGroup>& g, PartMapTables* t, u32 max_distinct) {
  part_map_default(t);
  u64 total = 0;
  for (const Group& x : g) total += x.work;
  if (!total) return 0;
  // The smallest work target whose greedy sweep fits kDictParts ranges: the range count
  // only falls as the target grows, so a binary search finds it in ~log2(total) sweeps
  // (a linear 1/16 step search took up to 400: 1.6 ms of host time for Hamlet's output).
  // If even target = total does not fit, the distinct-key cap is what binds: raise it.
  PartMapTables cand;
  u64 worst = 0;
  for (int widen = 0; widen < 64; ++widen) {
    if (assign(g, total, max_distinct, &cand, &worst) <= (u32)kDictParts) break;
    max_distinct += max_distinct / 8 + 1;
  }
  u64 lo = std::max<u64>(1, (total + kDictParts - 1) / kDictParts), hi = total;
  while (lo < hi) {  // invariant: hi fits
    const u64 mid = lo + (hi - lo) / 2;
    if (assign(g, mid, max_distinct, &cand, &worst) <= (u32)kDictParts)
      hi = mid;
    else
      lo = mid + 1;
  }
  if (assign(g, hi, max_distinct, &cand, &worst) > (u32)kDictParts) return 0;  // default map stays
  *t = cand;
  return worst;
}

}  // namespace locust
