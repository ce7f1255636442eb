// One workgroup's LSD radix sort in LDS: the stable counting pass shared by the
// single-workgroup sort (radix_sort.hip, n <= kSmallSortMax) and the partitioned sort
// (psort.hip, one key range per workgroup).
//
// Items are local indices 0..n); the caller keeps the current key word of every item in
// `word` (indexed by item) and a permutation in `perm[cur]`.  One pass on an 8-bit digit
// moves the permutation into `perm[cur ^ 1]`, stable:
//   A. each wave owns a contiguous chunk of permutation positions and ranks its items
//      among equal digits with 8 ballots per 64 items (wave64 match-any), keeping the
//      wave's per-digit totals in `cnt[wave][digit]` (one writer per digit per round:
//      plain LDS stores, no atomics);
//   B. thread d < 256 turns the 16 wave totals of digit d into exclusive wave offsets
//      (`wex`), zeroes `cnt` for the next pass, and a DPP wave scan over the 256 digit
//      totals gives each digit's start (plus the totals of the scan waves below);
//   C. every item is scattered to start + wave offset + rank.
// Three barriers per pass.  Counts are u16: a wave's chunk holds at most kMaxN / waves
// items (<= 65,535).
#pragma once

#include "locust/device/wave.hpp"

namespace locust {
namespace dev {

template <int kBlock, int kMaxN, typename Perm>
struct LdsRadix {
  static constexpr int kWaves = kBlock / 64;
  static constexpr int kRounds = kMaxN / kBlock;  // items per lane, at most
  static_assert(kMaxN % kBlock == 0, "kMaxN must be a multiple of the block");
  static_assert(kBlock >= 256, "one thread per digit in phase B");

  const uint64_t* word;     // [kMaxN] current key word per item
  Perm (*perm)[kMaxN];      // [2][kMaxN] ping-pong permutation of item ids
  uint16_t (*cnt)[256];     // [kWaves][256] per-wave digit totals (zero between passes)
  uint16_t (*wex)[256];     // [kWaves][256] exclusive wave offsets of the current pass
  uint32_t* start;          // [256] digit starts, scan-wave local
  uint32_t* wsum;           // [4] digit-scan wave totals

  // Zero `cnt` once before the first pass (the passes keep it zeroed); caller syncs.
  __device__ void init() const {
    for (int i = threadIdx.x; i < kWaves * 256; i += kBlock) (&cnt[0][0])[i] = 0;
  }

  // One stable pass on digit (word >> shift) & 0xff over items at perm[cur][0..n).  Ends
  // with a barrier: perm[cur ^ 1] holds the result.
  __device__ void pass(uint32_t n, uint32_t shift, int cur) const { pass(word, n, shift, cur); }
  // The same with the key words in `w` (e.g. one LDS array per key word).
  __device__ void pass(const uint64_t* w_arr, uint32_t n, uint32_t shift, int cur) const {
    const int lane = lane_id(), w = wave_id(), t = threadIdx.x;
    const uint32_t chunk = ((((n + kWaves - 1) / kWaves) + 63) / 64) * 64;
    const uint32_t c0 = (uint32_t)w * chunk;
    uint32_t idx[kRounds], dig[kRounds], rank[kRounds];
#pragma unroll
    for (int r = 0; r < kRounds; ++r) {
      const uint32_t p = c0 + (uint32_t)r * 64 + lane;
      const bool valid = (uint32_t)r * 64 < chunk && p < n;
      idx[r] = valid ? (uint32_t)perm[cur][p] : 0u;
      dig[r] = valid ? (uint32_t)(w_arr[idx[r]] >> shift) & 0xffu : 256u;
    }
    // ---- A: wave-local stable ranks ----
#pragma unroll
    for (int r = 0; r < kRounds; ++r) {
      const bool valid = dig[r] < 256u;
      const uint32_t d = dig[r] & 0xffu;
      uint64_t m = ballot(valid);
      if (!m) continue;  // wave-uniform
#pragma unroll
      for (int bb = 0; bb < 8; ++bb) {
        const bool bit = (d >> bb) & 1u;
        const uint64_t x = ballot(bit);
        m &= bit ? x : ~x;
      }
      uint32_t prev = 0;
      if (valid) prev = cnt[w][d];
      __builtin_amdgcn_wave_barrier();
      const uint32_t below = lanes_below(m);
      if (valid && below == 0) cnt[w][d] = (uint16_t)(prev + (uint32_t)__popcll(m));
      __builtin_amdgcn_wave_barrier();
      rank[r] = prev + below;
    }
    __syncthreads();
    // ---- B: offsets across waves, then across digits ----
    if (t < 256) {
      uint32_t run = 0;
#pragma unroll
      for (int ww = 0; ww < kWaves; ++ww) {
        const uint32_t c = cnt[ww][t];
        wex[ww][t] = (uint16_t)run;
        cnt[ww][t] = 0;
        run += c;
      }
      const uint32_t inc = wave_inclusive_scan(run);
      if (lane == 63) wsum[w] = inc;
      start[t] = inc - run;
    }
    __syncthreads();
    // ---- C: stable scatter ----
    const uint32_t s0 = wsum[0], s1 = wsum[1], s2 = wsum[2];
#pragma unroll
    for (int r = 0; r < kRounds; ++r) {
      if (dig[r] < 256u) {
        const uint32_t d = dig[r];
        const uint32_t q = d >> 6;
        const uint32_t add = (q > 0 ? s0 : 0u) + (q > 1 ? s1 : 0u) + (q > 2 ? s2 : 0u);
        perm[cur ^ 1][start[d] + add + wex[w][d] + rank[r]] = (Perm)idx[r];
      }
    }
    __syncthreads();
  }
};

}  // namespace dev
}  // namespace locust
