// Gather-strategy slot header (host and device code; no HIP dependency).
#pragma once

#include "locust/common.hpp"
#include "locust/kv.hpp"

namespace locust {

// Header of one rank's slot in the gather strategy's single all-gather (80 B: the two
// KeyCount records in front of the slot's records).  Written on the device at the end of
// the map, so the exchange needs no host round trip first.
struct SlotHeader {
  i32 status;         // kSlotOk; kSlotFailed (host-side failure); kSlotRedo: this job
                      // takes the standard path (LDS overflow redo, unmergeable records)
  u32 record_flags;   // ShardEngine::kRecords* of the records that follow
  u64 n;              // records of this rank (the slot holds min(n, slot_records))
  u64 lines, tokens, overflow_lines, truncated, max_key_len;
  u64 slot_cap;       // largest slot this rank can send (ShardEngine::slot_capacity())
  u64 pad[2];
};
static_assert(sizeof(SlotHeader) == 2 * sizeof(KeyCount), "SlotHeader is two records");
constexpr u32 kSlotHeaderRecords = 2;
constexpr i32 kSlotOk = 0, kSlotFailed = 1, kSlotRedo = 2;
// Smallest slot (records) of the one-all-gather gather strategy: the first job's slot
// size before any rank's record count is known; later jobs size slots from the previous
// job's largest rank.
constexpr u32 kSlotRecordsMin = 2048;
// Most ranks the one-all-gather gather strategy merges (the merge kernels' run table).
constexpr int kMaxSlotRanks = 64;

}  // namespace locust
