// Device-resident shuffle ("exchange") of the distributed job: message layouts shared by
// the host driver (dist.cpp) and the kernels (exchange.hip).  No HIP dependency.
//
// The reference has no shuffle at all (/tmp/out.txt with the network hop
// missing; the GIF's letter-range reducers are design only).  Round 1 built the
// sample-sort all-to-all with every control step staged through host memory -- five host
// round trips per job.  The exchange runs the same algorithm with every decision on the
// device:
//
//   H2D      this rank's ExchMsg1 (status, record count, map statistics, the root's output
//            region) + S samples (or both built on the device behind an asynchronous map)
//   C1       ncclAllGather of the messages
//   plan     one workgroup: weighted-quantile splitters from all ranks' samples (every
//            rank computes the same), 64-ary searches of them in the local sorted records
//   pack     records -> P slots (SlotHeader + the bucket) at a fixed pitch
//   C2       the slots to their ranks (every xGMI link busy at once)
//   merge    the P received sorted runs -> this rank's key range (merge.hip)
//   report   ExchMsg3 (overflow flags, range size, token total, largest bucket)
//   C3       ncclAllGather of the reports: every rank sees every flag and total
//   emit     this rank's range -> the shared host output (locust/shm.hpp) at its global
//            offset (val is rebuilt on the host from the counts); a completion stamp.  Every
//            rank drains its own range over its own PCIe link: no gather to the root.
//
// Two schedules:
//   one sync   C2 is ncclAllToAll of fixed-size slots sized by an earlier job (largest
//              bucket / range + 1/8).  A job whose data outgrows them is flagged in the
//              reports, which every rank holds, and every rank redoes the exchange sized.
//   two syncs  (the first job, or an outgrown one) C1 -> plan -> C1b: ncclAllGather of
//              every rank's bucket offsets (ExchCtl) -> host sync: every rank holds the
//              exact P x P count matrix -> C2 is grouped ncclSend/ncclRecv with exact
//              per-peer sizes -> merge -> report -> C3 -> emit -> host sync.
#pragma once

#include "locust/common.hpp"
#include "locust/kv.hpp"

namespace locust {

struct ExchMsg1 {       // 64 B, followed by S PackedKey samples
  i32 status;           // 0 = ok
  u32 record_flags;     // ShardEngine::kRecords* of this rank's records
  u64 n_local;          // sorted distinct records of this rank
  u64 lines, tokens, overflow_lines, truncated, max_key_len;
  u64 out_region;       // the root's: shared output region of this job (kExchNoRegion)
};
// The root holds no free output region (live results hold them all): grow, then emit.
constexpr u64 kExchNoRegion = ~0ull;
static_assert(sizeof(ExchMsg1) == 64, "ExchMsg1 64 B");

constexpr u32 kExchSendOverflow = 1;   // a bucket of this rank exceeded the slot
constexpr u32 kExchRecvTruncated = 2;  // a received slot was truncated or failed
constexpr u32 kExchAbort = 4;          // a rank's ExchMsg1 reported a failure
constexpr u32 kExchTooManySamples = 8; // the device planner cannot take this many samples
// ExchMsg1::status of a rank whose asynchronous map must be redone (an LDS partition of the
// ordered build overflowed): every rank sees it and the job continues on the standard path
constexpr i32 kExchMapRedo = 3;

struct ExchMsg3 {       // 64 B
  i32 status;           // 0 = ok
  u32 flags;            // kExch*
  u64 max_bucket;       // largest bucket this rank had to send
  u64 n_out;            // distinct keys of this rank's key range
  u64 total;            // token total of this rank's key range
  u64 out_words;        // 8-B words of its compact result records (the host output it writes)
  u64 pad[3];
};
static_assert(sizeof(ExchMsg3) == 64, "ExchMsg3 64 B");

constexpr u32 kExchGatherOverflow = 16; // this rank's range exceeded its range buffer

constexpr u32 kExchMaxPlanSamples = 1024;  // P x S the one-workgroup planner sorts in LDS
constexpr u32 kExchSamples = 64;           // samples per rank
constexpr u32 kExchMaxRanks = 64;

// Device scratch of one exchange, written by the plan kernel, read by pack and report.
struct ExchCtl {
  u64 off[kExchMaxRanks + 1];  // bucket offsets in this rank's sorted records
  u64 max_bucket;
  u32 flags;                   // kExchSendOverflow | kExchAbort | kExchTooManySamples
  u32 pad;
};

LOCUST_HD inline u64 exch_msg1_bytes(u32 samples) { return sizeof(ExchMsg1) + (u64)samples * sizeof(PackedKey); }
// All-to-all slot: a SlotHeader (two KeyCount records) + slot_records KeyCount records.
LOCUST_HD inline u64 exch_slot_bytes(u32 slot_records) { return (u64)(2 + slot_records) * sizeof(KeyCount); }
// Range buffer: gather_records (key, count) 40-B records (the size is in ExchMsg3).
// Next job's slot size for a largest observed bucket / range of `used` records.
inline u32 exch_grow(u64 used) {
  const u64 want = used + used / 8 + 64;
  return (u32)((want + 63) & ~63ull);
}

}  // namespace locust
