// Single-pass decoupled look-back (chained scan) for CDNA4.
//
// Replaces the reference's thrust::partition calls (/root/reference/MapReduce/src/
// main.cu:411,447,462) with a one-kernel scan: each workgroup takes a tile id from an
// atomic counter (so every tile it waits on has already started: no dispatch-order
// assumption), publishes its aggregate, and wave 0 looks back 64 predecessors at a time.
//
// Status words are 64-bit self-describing granules: [63:62] flag, [61:0] value, written
// with ONE relaxed agent-scope atomic store and read with relaxed agent-scope atomic loads
// (MI355X per-XCD L2s are not coherent with each other; agent-scope atomics are).
// Flag 0 = not yet published, 1 = tile aggregate only, 2 = inclusive prefix.
#pragma once

#include "locust/device/wave.hpp"

namespace locust {
namespace dev {

constexpr uint64_t kLbFlagShift = 62;
constexpr uint64_t kLbAgg = 1ull << kLbFlagShift;
constexpr uint64_t kLbInc = 2ull << kLbFlagShift;
constexpr uint64_t kLbValMask = (1ull << kLbFlagShift) - 1;

// Dynamic tile id in launch order.  `slot` is an LDS word.  All threads call it.
__device__ __forceinline__ uint32_t acquire_tile(uint32_t* counter, uint32_t* slot) {
  if (threadIdx.x == 0) *slot = atomicAdd(counter, 1u);
  __syncthreads();
  uint32_t t = *slot;
  __syncthreads();
  return t;
}

// Wave-parallel look-back.  Must be called by all 64 lanes of ONE wave.  Publishes the
// tile's aggregate, accumulates the exclusive prefix from predecessors, then publishes the
// inclusive prefix.  Returns the exclusive prefix in every lane of the calling wave.
__device__ __forceinline__ uint64_t wave_lookback(uint64_t* status, uint32_t tile,
                                                  uint64_t aggregate) {
  const int lane = lane_id();
  if (tile == 0) {
    if (lane == 0) st_agent(&status[0], kLbInc | aggregate);
    return 0;
  }
  if (lane == 0) st_agent(&status[tile], kLbAgg | aggregate);
  uint64_t excl = 0;
  int64_t base = (int64_t)tile - 1;
  for (;;) {
    const int64_t idx = base - lane;
    uint64_t s = (idx >= 0) ? ld_agent(&status[idx]) : kLbInc;
    const uint32_t flag = (uint32_t)(s >> kLbFlagShift);
    const uint64_t inc_mask = ballot(flag == 2);
    const uint64_t inv_mask = ballot(flag == 0);
    const int first_inc = inc_mask ? (__ffsll((unsigned long long)inc_mask) - 1) : 64;
    const uint64_t upto = first_inc >= 63 ? ~0ull : ((2ull << first_inc) - 1);
    if (inv_mask & upto) {
      __builtin_amdgcn_s_sleep(1);
      continue;  // a predecessor in the window has not published yet: re-read
    }
    uint64_t v = (lane <= first_inc) ? (s & kLbValMask) : 0;
    excl += wave_reduce_sum(v);
    if (first_inc < 64) break;
    base -= 64;
  }
  if (lane == 0) st_agent(&status[tile], kLbInc | (excl + aggregate));
  return excl;
}

// Split look-back: publish the tile's aggregate now (one lane), do independent work, and
// resolve the prefix later with wave_lookback_resolve -- successors can already sum this
// tile's aggregate while it works, so the wait overlaps that work.
__device__ __forceinline__ void publish_aggregate(uint64_t* status, uint32_t tile,
                                                  uint64_t aggregate) {
  st_agent(&status[tile], (tile == 0 ? kLbInc : kLbAgg) | aggregate);
}

// Second half of a split look-back (all 64 lanes of ONE wave): accumulates the exclusive
// prefix from predecessors and publishes the inclusive prefix.
__device__ __forceinline__ uint64_t wave_lookback_resolve(uint64_t* status, uint32_t tile,
                                                          uint64_t aggregate) {
  const int lane = lane_id();
  if (tile == 0) return 0;
  uint64_t excl = 0;
  int64_t base = (int64_t)tile - 1;
  for (;;) {
    const int64_t idx = base - lane;
    uint64_t s = (idx >= 0) ? ld_agent(&status[idx]) : kLbInc;
    const uint32_t flag = (uint32_t)(s >> kLbFlagShift);
    const uint64_t inc_mask = ballot(flag == 2);
    const uint64_t inv_mask = ballot(flag == 0);
    const int first_inc = inc_mask ? (__ffsll((unsigned long long)inc_mask) - 1) : 64;
    const uint64_t upto = first_inc >= 63 ? ~0ull : ((2ull << first_inc) - 1);
    if (inv_mask & upto) {
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    uint64_t v = (lane <= first_inc) ? (s & kLbValMask) : 0;
    excl += wave_reduce_sum(v);
    if (first_inc < 64) break;
    base -= 64;
  }
  if (lane == 0) st_agent(&status[tile], kLbInc | (excl + aggregate));
  return excl;
}

// Workgroup-level helper: all threads call; wave 0 performs the look-back and the
// exclusive tile prefix is broadcast through `slot` (an LDS u64).
__device__ __forceinline__ uint64_t block_lookback(uint64_t* status, uint32_t tile,
                                                   uint64_t aggregate, uint64_t* slot) {
  if (wave_id() == 0) {
    uint64_t e = wave_lookback(status, tile, aggregate);
    if (lane_id() == 0) *slot = e;
  }
  __syncthreads();
  uint64_t e = *slot;
  __syncthreads();
  return e;
}

}  // namespace dev
}  // namespace locust
