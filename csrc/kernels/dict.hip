// Dictionary sort path (Process/Reduce stages, default): the reference's
// "stream compaction + key sort" and "boundary mark + adjacent difference" computed on the
// distinct keys only.
//
// The reference sorts every emitted token (/root/reference/MapReduce/src/main.cu:414) and
// then recovers per-key runs by boundary marking (main.cu:161-238).  The output it prints
// is a function of the distinct keys and their multiplicities only: val = the start of a
// key's run in the sorted token array = the exclusive prefix sum of the counts of all
// smaller keys (rebuilt on the host, engine.hpp EntryVals); count = the run length.  So:
//
//   dict_insert   two-level hash aggregation.  A workgroup takes 1,024 consecutive tokens
//                 and combines duplicates in an LDS hash table (LDS atomics); only the
//                 chunk's distinct keys go to the HBM table: CAS on the first key word,
//                 the other words are self-validating atomic stores (no fences or flags),
//                 the claimer draws a dense id and writes the key to the dense unique
//                 array, and each distinct key adds its chunk count with one atomic.  Hot
//                 keys ("the" is 3% of Hamlet) cost one HBM atomic per chunk, not per token.
//   rank_sort     U distinct keys (U <= kRankSortMax): rank = number of smaller keys,
//                 counted by a persistent grid over (256-key x 1024-key) tile pairs with
//                 the j-tile in LDS (broadcast 16-byte reads) -- all-pairs work, but spread
//                 over every CU in one launch instead of ~14 dependent radix passes.
//                 Larger U goes to the LSD radix sort (radix_sort.hip).
//   rank_scatter  sorted[rank[i]] = key[i], counts alongside.
//   scan_pack     exclusive scan of the counts with decoupled look-back -> the token
//                 total, and the final 40-B (key, count) records for the D2H.
#include <algorithm>
#include <type_traits>

#include "locust/device/hash.hpp"
#include "locust/device/lds_radix.hpp"
#include "locust/device/lookback.hpp"
#include "locust/device/wave.hpp"
#include "locust/hip_check.hpp"
#include "locust/kernels.hpp"
#include "map_tile.hpp"

namespace locust {
namespace {

using dev::ballot;
using dev::lane_id;
using dev::wave_id;

// Words 1..3 are stored XOR kWordMagic: a packed key word can never equal kWordMagic
// (bytes 00 00 FF FF 00 00 FF FF: a NUL followed by non-NUL bytes), so a stored 0 means
// "not written yet" and a zero-initialised table needs no sentinel fill.
constexpr u64 kWordMagic = 0x0000FFFF0000FFFFull;
constexpr u32 kIdFull = 0xFFFFFFFFu;  // slot id of a key that did not fit the dense arrays

using dev::key_hash;
using dev::key_part;

__device__ __forceinline__ u64 cas_agent(u64* p, u64 expected, u64 desired) {
  __hip_atomic_compare_exchange_strong(p, &expected, desired, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
  return expected;  // the value found
}

// Global (HBM) table insert of one distinct key with its count.  Returns false when the
// table is full.
__device__ bool global_insert(const DictWorkspace& dw, const u64* k, u64 count,
                              MapCounters* ctr, u64 h) {
  u32 slot = (u32)h & dw.mask;
  for (u32 probes = 0; probes <= dw.mask;) {
    DictSlot* sl = dw.table + slot;
    u64 w0 = dev::ld_agent(&sl->w[0]);
    if (w0 == 0) {
      w0 = cas_agent(&sl->w[0], 0, k[0]);
      if (w0 == 0) {  // claimed: dense id, dense key, then publish the other words
        // One id-counter atomic per wave: the claiming lanes of this step share it.
        const u64 claim = ballot(true);
        const int leader = __ffsll((unsigned long long)claim) - 1;
        u32 base = 0;
        if (lane_id() == leader) base = atomicAdd(&ctr->num_unique, (u32)__popcll(claim));
        const u32 id = (u32)__shfl((int)base, leader, 64) + dev::lanes_below(claim);
        const bool fits = id < dw.ucap;
        if (fits) {
#pragma unroll
          for (int j = 0; j < kKeyWords; ++j) dw.ukeys.w[j][id] = k[j];
          // ucount is zero-initialised and only ever updated by device-scope atomics (a
          // plain store could sit dirty in this XCD's L2 and later overwrite other adds)
          atomicAdd(reinterpret_cast<unsigned long long*>(&dw.ucount[id]), (unsigned long long)count);
        }
#pragma unroll
        for (int j = 1; j < kKeyWords; ++j) dev::st_agent(&sl->w[j], k[j] ^ kWordMagic);
        // a key past the dense capacity is still published (as kIdFull), so later
        // inserters of it stop probing instead of waiting for an id that never comes
        dev::st_agent(&sl->id, fits ? id + 1 : kIdFull);
        return fits;
      }
    }
    if (w0 == k[0]) {
      const u32 sid = dev::ld_agent(&sl->id);
      const u64 x1 = dev::ld_agent(&sl->w[1]);
      const u64 x2 = dev::ld_agent(&sl->w[2]);
      const u64 x3 = dev::ld_agent(&sl->w[3]);
      if (sid == 0 || x1 == 0 || x2 == 0 || x3 == 0) continue;  // claimer still writing
      if ((x1 ^ kWordMagic) == k[1] && (x2 ^ kWordMagic) == k[2] && (x3 ^ kWordMagic) == k[3]) {
        if (sid == kIdFull) return false;
        atomicAdd(reinterpret_cast<unsigned long long*>(&dw.ucount[sid - 1]),
                  (unsigned long long)count);
        return true;
      }
    }
    slot = (slot + 1) & dw.mask;  // linear probing
    ++probes;
  }
  return false;
}

// Persistent LDS cache of a workgroup: 1,024 slots (40 KB).  A workgroup streams its
// tokens 256 at a time (one per thread) through the cache; a key found in (or claimed
// in) the first kLdsProbes slots of its probe sequence is counted in LDS, any other key
// goes straight to the HBM table.  Frequent keys get cached by the first chunks and stay
// cached for the whole stream, so a Zipfian input costs ~one HBM atomic per frequent key
// per workgroup.  The cache is flushed to the HBM table at the end.
constexpr int kInsBlock = 256;
constexpr int kLdsSlots = 1024;
constexpr int kLdsProbes = 8;

struct LdsSlot {
  u64 w[kKeyWords];  // w[0] raw (0 = empty), w[1..3] XOR kWordMagic (0 = not written)
  u64 count;
};

__device__ __forceinline__ bool lds_insert(LdsSlot* tab, const u64* k, u64 c, u64 h) {
  u32 slot = (u32)(h >> 40) & (kLdsSlots - 1);
  for (int probe = 0; probe < kLdsProbes;) {
    LdsSlot& sl = tab[slot];
    u64 w0 = sl.w[0];
    if (w0 == 0) {
      w0 = atomicCAS(reinterpret_cast<unsigned long long*>(&sl.w[0]), 0ull, (unsigned long long)k[0]);
      if (w0 == 0) {
#pragma unroll
        for (int j = 1; j < kKeyWords; ++j) sl.w[j] = k[j] ^ kWordMagic;
        atomicAdd(reinterpret_cast<unsigned long long*>(&sl.count), (unsigned long long)c);
        return true;
      }
    }
    if (w0 == k[0]) {
      const u64 x1 = __hip_atomic_load(&sl.w[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      const u64 x2 = __hip_atomic_load(&sl.w[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      const u64 x3 = __hip_atomic_load(&sl.w[3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      if (x1 == 0 || x2 == 0 || x3 == 0) continue;  // claimer (another wave) still writing
      if ((x1 ^ kWordMagic) == k[1] && (x2 ^ kWordMagic) == k[2] && (x3 ^ kWordMagic) == k[3]) {
        atomicAdd(reinterpret_cast<unsigned long long*>(&sl.count), (unsigned long long)c);
        return true;
      }
    }
    slot = (slot + 1) & (kLdsSlots - 1);
    ++probe;
  }
  return false;
}

__global__ __launch_bounds__(kInsBlock) void dict_insert_kernel(ConstKeysSoA tokens,
                                                                const u64* __restrict__ counts,
                                                                const u32* __restrict__ d_n,
                                                                DictWorkspace dw,
                                                                MapCounters* __restrict__ ctr,
                                                                u32 n_cap) {
  __shared__ LdsSlot s_tab[kLdsSlots];
  for (int i = threadIdx.x; i < kLdsSlots; i += kInsBlock) {
#pragma unroll
    for (int j = 0; j < kKeyWords; ++j) s_tab[i].w[j] = 0;
    s_tab[i].count = 0;
  }
  __syncthreads();
  const u32 n = min(*d_n, n_cap);  // the producer never writes past its capacity
  bool overflow = false;
  for (u32 i = blockIdx.x * kInsBlock + threadIdx.x; i < n; i += gridDim.x * kInsBlock) {
    u64 k[kKeyWords];
#pragma unroll
    for (int j = 0; j < kKeyWords; ++j) k[j] = tokens.w[j][i];
    const u64 c = counts ? counts[i] : 1ull;
    if (k[0] == 0 || c == 0) continue;
    const u64 h = key_hash(k);
    if (!lds_insert(s_tab, k, c, h)) overflow |= !global_insert(dw, k, c, ctr, h);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kLdsSlots; i += kInsBlock) {
    const LdsSlot& sl = s_tab[i];
    if (sl.w[0] == 0) continue;
    const u64 kk[kKeyWords] = {sl.w[0], sl.w[1] ^ kWordMagic, sl.w[2] ^ kWordMagic,
                               sl.w[3] ^ kWordMagic};
    overflow |= !global_insert(dw, kk, sl.count, ctr, key_hash(kk));
  }
  if (overflow) atomicOr(&ctr->flags, kCtrDictOverflow);
}

// ---------------------------------------------------------------------------------
// Partitioned build (small inputs): the map kernel tags every token with its hash
// partition (top hash byte).  Workgroup p owns partition p: it streams the partition
// bytes (16 per load), inserts ITS tokens into a private 2,048-slot LDS table, then writes
// the partition's distinct keys densely at an offset drawn with one atomic.  Every key is
// aggregated by exactly one workgroup, so there is no HBM table, no table reset, no
// global atomics per token, and the counts are written with plain stores.
// ---------------------------------------------------------------------------------
// Gather one packed key.  Keys are NUL-padded big-endian words, so a word whose last byte
// is 0 ends the key and the remaining words are 0: most English words fit in the first
// word, and the other three gathers are skipped.
__device__ __forceinline__ void load_key(ConstKeysSoA t, u32 i, u64* k) {
  k[0] = t.w[0][i];
  k[1] = k[2] = k[3] = 0;
  if (k[0] & 0xffull) {
    k[1] = t.w[1][i];
    if (k[1] & 0xffull) {
      k[2] = t.w[2][i];
      if (k[2] & 0xffull) k[3] = t.w[3][i];
    }
  }
}

constexpr int kPartBlock = 1024;       // 16 waves: latency hiding for the gathers
constexpr int kPartSlots = 2048;       // 80 KB of LDS
static_assert(kPartSlots == kPartSlotsHost, "partial slot size");
constexpr int kPartWindow = kPartBlock * 16;  // partition bytes scanned per round
constexpr u32 kOrdTagWindow = kPartBlock * 32;  // ordered build: tags scanned per round
constexpr int kPartPerThread = kPartSlots / kPartBlock;
// The ordered kernel's tile-source partitions clear only the first kSmallTable slots of
// their table; one of more than kSmallTableTokens tokens (so possibly more distinct keys
// than 3/4 of that) clears the rest before its first insert (grow_table).
constexpr u32 kSmallTable = 512;
constexpr u32 kSmallTableTokens = kSmallTable * 3 / 4;

// A key not placed within kPartProbes slots reports the table full (the caller falls back):
// probing a nearly full table to the end made an overflowing pass quadratic.  (512: a
// planned range holds up to ~1,500 of the 2,048 slots; linear probing at 75 % load runs
// clusters past 128.)
constexpr int kPartProbes = 512;
// occ (optional, LDS, zeroed with the table): the table's claimed slots.  With it a key
// probes past kPartProbes -- up to the whole table -- while the table is below 31/32 full,
// so a planned range that lands at ~95 % load (in-job plans of large passes: measured up to
// 1,936 of 2,048 on synth1m) still fits instead of sending the whole pass to the fallback;
// a table at 31/32 stops at kPartProbes as before (no quadratic overflowing pass).
constexpr u32 kPartOccFull = kPartSlots - kPartSlots / 32;
// mask (optional): a table of mask + 1 <= kPartSlots slots (a power of two; the ordered
// kernel's small partitions clear and use only the first kSmallTable slots).
__device__ __forceinline__ bool part_lds_insert(LdsSlot* tab, const u64* k, u64 c, u64 h,
                                                u32* occ = nullptr, u32 mask = kPartSlots - 1) {
  u32 slot = (u32)(h >> 8) & mask;
  const int limit = occ ? kPartSlots : (int)min((u32)kPartProbes, mask + 1);
  for (int probe = 0; probe < limit;) {
    if (occ && probe >= kPartProbes && (probe & 63) == 0 &&
        __hip_atomic_load(occ, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= kPartOccFull)
      return false;
    LdsSlot& sl = tab[slot];
    u64 w0 = sl.w[0];
    if (w0 == 0) {
      w0 = atomicCAS(reinterpret_cast<unsigned long long*>(&sl.w[0]), 0ull, (unsigned long long)k[0]);
      if (w0 == 0) {
#pragma unroll
        for (int j = 1; j < kKeyWords; ++j)
          __hip_atomic_store(&sl.w[j], k[j] ^ kWordMagic, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        atomicAdd(reinterpret_cast<unsigned long long*>(&sl.count), (unsigned long long)c);
        if (occ) atomicAdd(occ, 1u);
        return true;
      }
    }
    if (w0 == k[0]) {
      const u64 x1 = __hip_atomic_load(&sl.w[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      const u64 x2 = __hip_atomic_load(&sl.w[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      const u64 x3 = __hip_atomic_load(&sl.w[3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      if (x1 == 0 || x2 == 0 || x3 == 0) continue;  // claimer (another wave) still writing
      if ((x1 ^ kWordMagic) == k[1] && (x2 ^ kWordMagic) == k[2] && (x3 ^ kWordMagic) == k[3]) {
        atomicAdd(reinterpret_cast<unsigned long long*>(&sl.count), (unsigned long long)c);
        return true;
      }
    }
    slot = (slot + 1) & mask;
    ++probe;
  }
  return false;
}

// Gathers and inserts the tokens s_list[0 .. lim): every thread issues the first-word
// loads of up to kGatherBatch tokens before it inserts any, so a partition of up to
// kGatherBatch x 1,024 tokens pays ONE global-load latency instead of one per 1,024-token
// round (the tokens were written by the map on other XCDs: these are L2 misses).  Longer
// keys' further words are rare (English words fit in 8 bytes) and gathered after.
constexpr int kGatherBatch = 4;
// Inserts one batch of gathered tokens: k[r][0] (and k[r][1] if eager_w1) and c[r] are
// loaded for list entry idx[r].  [rlo, rhi) (rlast: no upper bound): only keys whose first
// word lies in the range are inserted (a virtual partition's share of its map partition;
// the default takes all); the further words of those are gathered here.
template <int kB>
__device__ __forceinline__ bool insert_gathered(ConstKeysSoA tokens, const u32* idx,
                                                u64 (*k)[kKeyWords], u64* c, LdsSlot* s_tab,
                                                u64 rlo, u64 rhi, bool rlast, bool eager_w1,
                                                bool weighted, u32 mask = kPartSlots - 1) {
  bool full = false;
#pragma unroll
  for (int r = 0; r < kB; ++r)  // outside the range: neither gathered nor inserted
    if (k[r][0] < rlo || (!rlast && k[r][0] >= rhi)) k[r][0] = 0;
#pragma unroll
  for (int r = 0; r < kB; ++r) {
    if (!(k[r][0] & 0xffull))
      k[r][1] = 0;
    else if (!eager_w1)
      k[r][1] = tokens.w[1][idx[r]];
  }
#pragma unroll
  for (int r = 0; r < kB; ++r)
    if (k[r][1] & 0xffull) {
      k[r][2] = tokens.w[2][idx[r]];
      if (k[r][2] & 0xffull) k[r][3] = tokens.w[3][idx[r]];
    }
#pragma unroll
  for (int r = 0; r < kB; ++r) {
    bool live = k[r][0] != 0 && c[r] != 0;
    // Hot keys: the lanes holding the same key as the wave's first live lane are combined
    // into one insert by that lane (Zipfian text: a hot partition's waves are mostly one
    // or two keys, and 64 LDS atomics on one slot serialise).
    const u64 lm = dev::ballot(live);
    if (lm) {
      const int L = __ffsll((unsigned long long)lm) - 1;
      bool same = live;
#pragma unroll
      for (int j = 0; j < kKeyWords; ++j) {
        const u32 lo = (u32)__builtin_amdgcn_readlane((int)(u32)k[r][j], L);
        const u32 hi = (u32)__builtin_amdgcn_readlane((int)(u32)(k[r][j] >> 32), L);
        same &= k[r][j] == (((u64)hi << 32) | lo);
      }
      const u64 sm = dev::ballot(same);
      if (__popcll(sm) > 1) {
        const u64 tot = weighted ? dev::wave_reduce_sum(same ? c[r] : 0ull) : (u64)__popcll(sm);
        if (dev::lane_id() == L) c[r] = tot;
        else if (same) live = false;
      }
    }
    if (live) full |= !part_lds_insert(s_tab, k[r], c[r], key_hash(k[r]), nullptr, mask);
  }
  return full;
}

template <int kGatherBatch = kGatherBatch>
// eager_w1: load key word 1 of every token together with word 0 (one round trip for
// the keys of 8-15 bytes, whose word 1 was a second, dependent load); word 1 of a
// shorter key is not written by the map, so it is masked, never used.
__device__ __forceinline__ bool gather_insert(ConstKeysSoA tokens, const u64* counts,
                                              const u32* s_list, u32 lim, u32 n_cap,
                                              LdsSlot* s_tab, u64 rlo = 0, u64 rhi = ~0ull,
                                              bool rlast = true, bool eager_w1 = false,
                                              u32 mask = kPartSlots - 1) {
  bool full = false;
  for (u32 e0 = 0; e0 < lim; e0 += kGatherBatch * kPartBlock) {
    u32 idx[kGatherBatch];
    u64 k[kGatherBatch][kKeyWords];
    u64 c[kGatherBatch];
#pragma unroll
    for (int r = 0; r < kGatherBatch; ++r) {
      const u32 e = e0 + (u32)r * kPartBlock + threadIdx.x;
      idx[r] = e < lim ? s_list[e] : 0xFFFFFFFFu;
    }
#pragma unroll
    for (int r = 0; r < kGatherBatch; ++r) {
      const bool ok = idx[r] < n_cap;
      k[r][0] = ok ? tokens.w[0][idx[r]] : 0;
      k[r][1] = ok && eager_w1 ? tokens.w[1][idx[r]] : 0;
      c[r] = ok ? (counts ? counts[idx[r]] : 1ull) : 0;
      k[r][2] = k[r][3] = 0;
    }
    full |= insert_gathered<kGatherBatch>(tokens, idx, k, c, s_tab, rlo, rhi, rlast, eager_w1,
                                          counts != nullptr, mask);
  }
  return full;
}

// Ascending sort of one u64 per lane across the wave (bitonic network over the 64 lanes).
__device__ __forceinline__ u64 wave_sort_u64(u64 x) {
  const u32 lane = (u32)dev::lane_id();
#pragma unroll
  for (u32 k = 2; k <= 64; k <<= 1)
#pragma unroll
    for (u32 j = k >> 1; j; j >>= 1) {
      const u64 o = __shfl_xor((unsigned long long)x, (int)j, 64);
      const bool keep_min = ((lane & j) == 0) == ((lane & k) == 0);
      x = keep_min ? (o < x ? o : x) : (o > x ? o : x);
    }
  return x;
}

__device__ __forceinline__ u64 readlane_u64(u64 x, u32 lane) {
  const u32 lo = (u32)__builtin_amdgcn_readlane((int)(u32)x, (int)lane);
  const u32 hi = (u32)__builtin_amdgcn_readlane((int)(u32)(x >> 32), (int)lane);
  return ((u64)hi << 32) | lo;
}

// Per round: every thread loads 16 partition bytes (the next round's load is issued before
// this round's inserts), appends the indices of its partition's tokens to an LDS list,
// then the whole workgroup gathers those tokens' keys (independent loads across threads)
// and inserts them.
__global__ __launch_bounds__(kPartBlock) void dict_part_build_kernel(
    ConstKeysSoA tokens, const u64* __restrict__ counts, const u8* __restrict__ parts,
    const u32* __restrict__ d_n, u32 n_cap, DictWorkspace dw, MapCounters* __restrict__ ctr) {
  __shared__ LdsSlot s_tab[kPartSlots];
  __shared__ u32 s_list[kPartWindow];  // worst case: every byte of a round matches
  __shared__ u32 s_count;
  __shared__ u32 s_scan[kPartBlock / 64 + 1];
  __shared__ u32 s_base;
  for (int i = threadIdx.x; i < kPartSlots; i += kPartBlock) {
#pragma unroll
    for (int j = 0; j < kKeyWords; ++j) s_tab[i].w[j] = 0;
    s_tab[i].count = 0;
  }
  if (threadIdx.x == 0) s_count = 0;
  __syncthreads();
  const u32 p = blockIdx.x;
  const u32 n = min(*d_n, n_cap);
  bool full = false;
  u32 pos = threadIdx.x * 16u;
  uint4 v = pos < n ? *reinterpret_cast<const uint4*>(parts + pos) : uint4{0, 0, 0, 0};
  for (u32 round = 0; round < n; round += kPartWindow, pos += kPartWindow) {
    // match mask of this thread's 16 bytes
    u32 mask = 0;
    const u32 wv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int b = 0; b < 4; ++b)
        if (((wv[q] >> (8 * b)) & 0xffu) == p && pos + (u32)(q * 4 + b) < n) mask |= 1u << (q * 4 + b);
    const u32 next = pos + kPartWindow;
    if (next < n) v = *reinterpret_cast<const uint4*>(parts + next);  // prefetch next round
    if (mask) {
      u32 at = atomicAdd(&s_count, (u32)__popc(mask));
      while (mask) {
        const int b = __ffs(mask) - 1;
        mask &= mask - 1;
        s_list[at++] = pos + (u32)b;
      }
    }
    __syncthreads();
    const u32 cnt = s_count;
    for (u32 e = threadIdx.x; e < cnt; e += kPartBlock) {
      const u32 i = s_list[e];
      u64 k[kKeyWords];
      load_key(tokens, i, k);
      const u64 c = counts ? counts[i] : 1ull;
      if (k[0] == 0 || c == 0) continue;
      full |= !part_lds_insert(s_tab, k, c, key_hash(k));
    }
    __syncthreads();
    if (threadIdx.x == 0) s_count = 0;
    __syncthreads();
  }
  // dense output: thread t owns slots [t * 2, t * 2 + 2)
  u32 mine = 0;
#pragma unroll
  for (int r = 0; r < kPartPerThread; ++r) mine += s_tab[threadIdx.x * kPartPerThread + r].w[0] != 0;
  u32 total = 0;
  const u32 excl = dev::block_exclusive_scan<u32, kPartBlock>(mine, s_scan, &total);
  if (threadIdx.x == 0) s_base = total ? atomicAdd(&ctr->num_unique, total) : 0u;
  __syncthreads();
  u32 id = s_base + excl;
#pragma unroll
  for (int r = 0; r < kPartPerThread; ++r) {
    const LdsSlot& sl = s_tab[threadIdx.x * kPartPerThread + r];
    if (sl.w[0] == 0) continue;
    if (id < dw.ucap) {
      dw.ukeys.w[0][id] = sl.w[0];
#pragma unroll
      for (int j = 1; j < kKeyWords; ++j) dw.ukeys.w[j][id] = sl.w[j] ^ kWordMagic;
      dw.ucount[id] = sl.count;
      dw.uval[id] = 0;  // the rank sort accumulates into these
      dw.urank[id] = 0;
    } else {
      full = true;
    }
    ++id;
  }
  if (full) atomicOr(&ctr->flags, kCtrDictOverflow);
}

// ---------------------------------------------------------------------------------
// Ordered build: Process AND Reduce in one kernel (small inputs).
//
// The partition of a token is its key's FIRST BYTE, so partitions are ordered: every key
// of partition p sorts before every key of partition p+1.  Workgroup p (taken in launch
// order from a ticket counter) aggregates its partition in LDS as above, compacts the
// distinct keys, publishes (distinct keys, tokens) through a decoupled look-back, and --
// while its predecessors resolve -- bitonic-sorts its keys in LDS.  Its output slice then
// starts at the exclusive prefix of distinct keys, and each key's val (start of its run in
// the sorted token order) is the prefix of tokens plus the scan of counts inside the
// partition.  The records go straight to the output (host-mapped: zero-copy).  No rank
// sort over all keys (U^2), no separate emit, one launch after the map.
//
// A partition with more than kPartSlots distinct keys (or any table overflow) marks the
// run kCtrDictOverflow; the host then reruns the Process stage on the HBM-table path.
// ---------------------------------------------------------------------------------
constexpr u64 kOrdM = (1ull << 20) - 1;        // look-back value: [m:20][ovf:9][tokens:33]
constexpr u32 kSplitMinTokens = 128;           // planned workgroups: tokens per extra sibling
constexpr u32 kPlanRows = 16;                  // table rows the plan estimates tokens from
constexpr u32 kSmallRank = 256;                // partitions up to here: all-pairs ranks
constexpr int kOrdOvfShift = 20;
constexpr int kOrdTokShift = 29;

__device__ __forceinline__ bool ord_greater(u64 aw0, u32 as, u64 bw0, u32 bs, const LdsSlot* tab) {
  if (aw0 != bw0) return aw0 > bw0;
  if (as == 0xFFFFFFFFu || bs == 0xFFFFFFFFu) return as == 0xFFFFFFFFu && bs != 0xFFFFFFFFu;
#pragma unroll
  for (int j = 1; j < kKeyWords; ++j) {
    const u64 x = tab[as].w[j] ^ kWordMagic, y = tab[bs].w[j] ^ kWordMagic;
    if (x != y) return x > y;
  }
  return false;
}

// Inserts partition p's records of tiles t, t + kPartBlock, ... (< t_end) into the LDS
// table: every thread walks its own tiles' runs straight from the per-tile table (no LDS
// list, no barrier between finding the runs and loading the keys), kPartialBatch key
// gathers in flight, the next tile's run prefetched.  (a, len) is this thread's first run,
// loaded by the caller before its table clear.  combine: lanes holding the wave's first
// live key fold into one insert (hot keys).  Returns true if the table overflowed.
constexpr int kPartialBatch = 8;
__device__ __forceinline__ bool walk_runs_insert(ConstKeysSoA tokens, const u64* counts,
                                                 const u32* part_off, u32 p, u32 t, u32 t_end,
                                                 u32 a, u32 len, u32 n_cap, LdsSlot* s_tab,
                                                 bool combine, u32* ntok_out,
                                                 u32* s_full = nullptr, u32* s_occ = nullptr) {
  bool full = false;
  u32 ntok = 0;
  // s_full (LDS, zeroed by the caller before its barrier): set by the first failed insert
  // of any wave; every wave stops at its next batch.  The slot's records are discarded once
  // the table overflowed, so the rest of the walk is wasted work -- with a cold partition map
  // (first key byte) a hot partition's remaining ~10^5 tokens each probed kPartProbes full
  // slots: 3-8 ms per partials launch instead of ~25-55 us.
  // The loop trip counts are per lane; the wave keeps going while any lane has work.
  while (dev::ballot(t < t_end)) {
    if (s_full && __builtin_amdgcn_readfirstlane(
                      (int)__hip_atomic_load(s_full, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)))
      break;
    u32 na = 0, nlen = 0;  // the next tile's run, prefetched
    const u32 tn = t + kPartBlock;
    if (tn < t_end) {
      na = part_off[(u64)tn * kPartTable + p];
      nlen = part_off[(u64)tn * kPartTable + p + 1] - na;
    }
    for (u32 j0 = 0; dev::ballot(j0 < len); j0 += kPartialBatch) {
      if (s_full && __builtin_amdgcn_readfirstlane(
                        (int)__hip_atomic_load(s_full, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)))
        break;
      u64 kk[kPartialBatch][kKeyWords];
      u64 cc[kPartialBatch];
#pragma unroll
      for (int r = 0; r < kPartialBatch; ++r) {
        const u32 idx = a + j0 + (u32)r;
        const bool ok = j0 + (u32)r < len && idx < n_cap;
        kk[r][0] = ok ? tokens.w[0][idx] : 0;
        cc[r] = ok && counts ? counts[idx] : 1ull;
        kk[r][1] = kk[r][2] = kk[r][3] = 0;
      }
#pragma unroll
      for (int r = 0; r < kPartialBatch; ++r) {
        const u32 idx = a + j0 + (u32)r;
        if (kk[r][0] & 0xffull) {
          kk[r][1] = tokens.w[1][idx];
          if (kk[r][1] & 0xffull) {
            kk[r][2] = tokens.w[2][idx];
            if (kk[r][2] & 0xffull) kk[r][3] = tokens.w[3][idx];
          }
        }
      }
#pragma unroll
      for (int r = 0; r < kPartialBatch; ++r) {
        bool live = kk[r][0] != 0 && cc[r] != 0;
        u64 c = cc[r];
        const u64 lm = dev::ballot(live);
        if (lm && combine) {
          const int L = __ffsll((unsigned long long)lm) - 1;
          bool same = live;
#pragma unroll
          for (int j = 0; j < kKeyWords; ++j) {
            const u32 lo = (u32)__builtin_amdgcn_readlane((int)(u32)kk[r][j], L);
            const u32 hi = (u32)__builtin_amdgcn_readlane((int)(u32)(kk[r][j] >> 32), L);
            same &= kk[r][j] == (((u64)hi << 32) | lo);
          }
          const u64 sm = dev::ballot(same);
          if (__popcll(sm) > 1) {
            const u64 tot = counts ? dev::wave_reduce_sum(same ? c : 0ull) : (u64)__popcll(sm);
            if (dev::lane_id() == L) c = tot;
            else if (same) live = false;
          }
        }
        if (live && !part_lds_insert(s_tab, kk[r], c, key_hash(kk[r]), s_occ)) {
          full = true;
          if (s_full) __hip_atomic_store(s_full, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      }
    }
    ntok += len;
    t = tn;
    a = na;
    len = nlen;
  }
  if (ntok_out) *ntok_out = ntok;
  return full;
}

// Token source of the ordered kernel: the map output (or unpacked records), found by
// scanning the one-byte partition tags of every token.
struct TagSource {
  ConstKeysSoA tokens;
  const u64* counts;
  const u8* parts;
  const u32* d_n;
  u32 n_cap;
  // Inserts partition p's tokens into `s_tab`; `s_list` / `s_count` are LDS scratch.
  // Returns true if the table overflowed.
  struct Pre {};
  __device__ Pre prefetch(u32) const { return {}; }
  __device__ bool build(u32 p, Pre, LdsSlot* s_tab, u32* s_list, u32& s_count, u64*) const {
    // Rounds of kOrdTagWindow tags (32 per thread, two 16-B loads, the next round's
    // prefetched): whole Hamlet (32,940 tokens) is one round + a short tail instead of
    // three.  A round appends at most kPartWindow matches to the list; a partition with
    // more in one window (over half of all tokens) reports an overflow, and the host
    // redoes the Process stage on the HBM-table path.
    const u32 n = min(*d_n, n_cap);
    bool full = false;
    u32 pos = threadIdx.x * 32u;
    uint4 v0 = pos < n ? *reinterpret_cast<const uint4*>(parts + pos) : uint4{0, 0, 0, 0};
    uint4 v1 = pos + 16 < n ? *reinterpret_cast<const uint4*>(parts + pos + 16) : uint4{0, 0, 0, 0};
    for (u32 round = 0; round < n; round += kOrdTagWindow, pos += kOrdTagWindow) {
      u32 mask = 0;
      const u32 wv[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
      for (int q = 0; q < 8; ++q)
#pragma unroll
        for (int b = 0; b < 4; ++b)
          if (((wv[q] >> (8 * b)) & 0xffu) == p && pos + (u32)(q * 4 + b) < n) mask |= 1u << (q * 4 + b);
      const u32 next = pos + kOrdTagWindow;
      if (next < n) v0 = *reinterpret_cast<const uint4*>(parts + next);
      if (next + 16 < n) v1 = *reinterpret_cast<const uint4*>(parts + next + 16);
      {
        // one LDS atomic per wave: the wave's matches are appended as one run
        const u32 nm = (u32)__popc(mask);
        const u32 incl = dev::wave_inclusive_scan(nm);
        u32 wbase = 0;
        if (dev::lane_id() == 63 && incl) wbase = atomicAdd(&s_count, incl);
        wbase = (u32)__shfl((int)wbase, 63, 64);
        u32 at = wbase + incl - nm;
        while (mask) {
          const int b = __ffs(mask) - 1;
          mask &= mask - 1;
          if (at < (u32)kPartWindow) s_list[at] = pos + (u32)b;
          ++at;
        }
      }
      __syncthreads();
      const u32 cnt = s_count;
      full |= cnt > (u32)kPartWindow;
      full |= gather_insert(tokens, counts, s_list, min(cnt, (u32)kPartWindow), n, s_tab);
      __syncthreads();
      if (threadIdx.x == 0) s_count = 0;
      __syncthreads();
    }
    return full;
  }
};

// Token source of the ordered kernel after the small-input fast map: the map grouped each
// 1 KiB tile's tokens by partition and recorded where every partition's run starts
// (launch_map_fast part_off), so workgroup p reads two words per tile instead of
// scanning the partition tags of every token.
struct TileSource {
  ConstKeysSoA tokens;
  const u32* part_off;
  u32 ntiles;
  u32 n_cap;  // token capacity: indices past it were never written
  // This thread's first run (tile threadIdx.x), loaded before the kernel clears its table
  // so that the load overlaps the clear and its barrier.
  struct Pre {
    u32 a, b;
  };
  __device__ Pre prefetch(u32 p) const {
    const u32 t = threadIdx.x;
    if (t >= ntiles) return {0, 0};
    return {part_off[(u64)t * kPartTable + p], part_off[(u64)t * kPartTable + p + 1]};
  }
  // stamp (diagnostics, optional): [12] list built, [13] gathered + inserted.  (Walking
  // each thread's own tile runs instead, as the partials kernel does, measured slower
  // here: 21 vs 13.5 us span -- a small pass has ~180 tiles, so most lanes idle while the
  // hot tiles' lanes insert serially; the list spreads the tokens over all 1,024.)
  // The table mask for a partition of ntok tokens (uniform), growing a small table (the
  // caller's barrier follows before any insert); thread 0 records it in *s_tmask.
  __device__ static u32 grow_table(u32 ntok, u32 mask, LdsSlot* s_tab, u32* s_tmask) {
    if (mask == (u32)kPartSlots - 1 || ntok <= kSmallTableTokens) return mask;
    for (u32 i = mask + 1 + threadIdx.x; i < (u32)kPartSlots; i += kPartBlock) {
#pragma unroll
      for (int j = 0; j < kKeyWords; ++j) s_tab[i].w[j] = 0;
      s_tab[i].count = 0;
    }
    if (threadIdx.x == 0) *s_tmask = kPartSlots - 1;
    return kPartSlots - 1;
  }
  // mask: the cleared table's (kPartSlots - 1, or kSmallTable - 1 for tile sources)
  __device__ bool build(u32 p, Pre pre, LdsSlot* s_tab, u32* s_list, u32& s_count,
                        u64* stamp, u32 mask = kPartSlots - 1, u32* s_tmask = nullptr) const {
    bool full = false;
    for (u32 t0 = 0; t0 < ntiles; t0 += kPartBlock) {
      const u32 t = t0 + threadIdx.x;
      u32 a = 0, len = 0;
      if (t0 == 0) {
        a = pre.a;
        len = pre.b - pre.a;
      } else if (t < ntiles) {
        a = part_off[(u64)t * kPartTable + p];
        len = part_off[(u64)t * kPartTable + p + 1] - a;
      }
      {
        // one LDS atomic per wave: the wave's runs are appended back to back
        const u32 incl = dev::wave_inclusive_scan(len);
        u32 wbase = 0;
        if (dev::lane_id() == 63 && incl) wbase = atomicAdd(&s_count, incl);
        wbase = (u32)__shfl((int)wbase, 63, 64);
        u32 at = wbase + incl - len;
        for (u32 j = 0; j < len; ++j, ++at)
          if (at < (u32)kPartWindow) s_list[at] = a + j;
      }
      __syncthreads();
      if (stamp && threadIdx.x == 0) stamp[12] = __builtin_amdgcn_s_memtime();
      const u32 cnt = s_count;
      full |= cnt > (u32)kPartWindow;  // the host redoes the Process stage on the HBM table
      if (t0 == 0 && mask != (u32)kPartSlots - 1) {  // uniform: a small table, grown if needed
        const u32 m2 = grow_table(ntiles > (u32)kPartBlock ? ~0u : cnt, mask, s_tab, s_tmask);
        if (m2 != mask) __syncthreads();
        mask = m2;
      }
      full |= gather_insert(tokens, nullptr, s_list, min(cnt, (u32)kPartWindow), n_cap, s_tab, 0,
                            ~0ull, true, true, mask);
      if (stamp && threadIdx.x == 0) stamp[13] = __builtin_amdgcn_s_memtime();
      __syncthreads();
      if (threadIdx.x == 0) s_count = 0;
      __syncthreads();
    }
    return full;
  }
  // Virtual partition j of K over map partition p: the key range between the j-th and
  // (j+1)-th K-quantile of a sample of the partition's tokens.  The list of the
  // partition's tokens is built in tile order at positions from a block scan of the runs
  // (not the atomic order of the plain build), so all K siblings draw the same sample, sort
  // it the same way and agree on every cut: each key lands in exactly one sibling, which
  // then inserts only its own range.  `pre`: this thread's run (tile threadIdx.x; the plan
  // admits at most kPartBlock tiles).
  // A partition of at most kGatherBatch x 1,024 tokens: the tokens' first two words are
  // loaded once, the samples taken from those registers and sorted by every wave in
  // registers -- one global round trip per sibling, no LDS rank pass; larger ones sample
  // the list first, then gather (the cuts are the same: same sample positions).
  static constexpr u32 kSplitSamples = 64;
  __device__ bool build_split(u32 p, Pre pre, u32 j, u32 K, LdsSlot* s_tab, u32* s_list,
                              u32* s_scan, u64* stamp, u32 mask = kPartSlots - 1,
                              u32* s_tmask = nullptr) const {
    u64* s_samp = reinterpret_cast<u64*>(s_list + kPartWindow - 256);  // [64]
    u64* s_sort = reinterpret_cast<u64*>(s_list + kPartWindow - 128);  // [64]
    const u32 a = pre.a, len = threadIdx.x < ntiles ? pre.b - pre.a : 0u;
    u32 n = 0;
    const u32 at = dev::block_exclusive_scan<u32, kPartBlock>(len, s_scan, &n);
    const u32 lim = min(n, (u32)kPartWindow - 256);  // the sample area sits at the list's end
    mask = grow_table(n, mask, s_tab, s_tmask);  // (the barrier after the fill covers it)
    if (stamp && threadIdx.x == 0) stamp[28] = __builtin_amdgcn_s_memtime();
    for (u32 k = 0; k < len && at + k < lim; ++k) s_list[at + k] = a + k;
    __syncthreads();
    if (stamp && threadIdx.x == 0) stamp[26] = __builtin_amdgcn_s_memtime();
    const u32 S = lim < kSplitSamples ? lim : kSplitSamples;
    const bool last = j + 1 >= K;
    // a list cut short by the sample area is an overflow: the host redoes the pass
    bool full = n > lim;
    if (lim <= (u32)(kGatherBatch * kPartBlock)) {
      u32 idx[kGatherBatch];
      u64 k[kGatherBatch][kKeyWords];
      u64 c[kGatherBatch];
#pragma unroll
      for (int r = 0; r < kGatherBatch; ++r) {
        const u32 e = (u32)r * kPartBlock + threadIdx.x;
        idx[r] = e < lim ? s_list[e] : 0xFFFFFFFFu;
      }
#pragma unroll
      for (int r = 0; r < kGatherBatch; ++r) {
        const bool ok = idx[r] < n_cap;
        k[r][0] = ok ? tokens.w[0][idx[r]] : 0;
        k[r][1] = ok ? tokens.w[1][idx[r]] : 0;
        c[r] = ok ? 1ull : 0ull;
        k[r][2] = k[r][3] = 0;
      }
      // list position e is sample s when s = ceil(e S / lim) lands on it (S <= lim: the
      // positions floor(s lim / S) are distinct)
#pragma unroll
      for (int r = 0; r < kGatherBatch; ++r) {
        const u32 e = (u32)r * kPartBlock + threadIdx.x;
        if (e < lim) {
          const u32 sidx = (u32)(((u64)e * S + lim - 1) / lim);
          if (sidx < S && (u32)((u64)sidx * lim / S) == e) s_samp[sidx] = idx[r] < n_cap ? k[r][0] : 0ull;
        }
      }
      if (stamp && threadIdx.x == 0) stamp[27] = __builtin_amdgcn_s_memtime();  // its loads are in
      __syncthreads();
      const u32 lane = (u32)dev::lane_id();
      const u64 srt = wave_sort_u64(lane < S ? s_samp[lane] : ~0ull);  // the S samples first
      const u64 lo = j == 0 || !S ? 0ull : readlane_u64(srt, (u32)((u64)j * S / K));
      const u64 hi = last || !S ? ~0ull : readlane_u64(srt, (u32)((u64)(j + 1) * S / K));
      if (stamp && threadIdx.x == 0) stamp[12] = __builtin_amdgcn_s_memtime();
      if (!(lo == hi && !last))
        full |= insert_gathered<kGatherBatch>(tokens, idx, k, c, s_tab, lo, hi, last, true, false,
                                              mask);
      if (stamp && threadIdx.x == 0) stamp[13] = __builtin_amdgcn_s_memtime();
      __syncthreads();  // the list area is reused after the build
      return full;
    }
    if (threadIdx.x < S) {
      const u32 idx = s_list[(u32)((u64)threadIdx.x * lim / S)];
      s_samp[threadIdx.x] = idx < n_cap ? tokens.w[0][idx] : 0ull;
    }
    __syncthreads();
    if (threadIdx.x < S) {  // rank = sorted position (ties by sample index)
      const u64 w = s_samp[threadIdx.x];
      u32 r = 0;
      for (u32 k = 0; k < S; ++k) {
        const u64 o = s_samp[k];
        r += (o < w || (o == w && k < threadIdx.x)) ? 1u : 0u;
      }
      s_sort[r] = w;
    }
    __syncthreads();
    const u64 lo = j == 0 || !S ? 0ull : s_sort[(u64)j * S / K];
    const u64 hi = last || !S ? ~0ull : s_sort[(u64)(j + 1) * S / K];
    if (stamp && threadIdx.x == 0) stamp[12] = __builtin_amdgcn_s_memtime();
    if (!(lo == hi && !last))  // else an empty range (a hot first word took it)
      full |= gather_insert(tokens, nullptr, s_list, lim, n_cap, s_tab, lo, hi, last, true, mask);
    if (stamp && threadIdx.x == 0) stamp[13] = __builtin_amdgcn_s_memtime();
    __syncthreads();  // the list area is reused after the build
    return full;
  }
};

// Token source of the gather-strategy merge: runs of KeyCount records, each sorted by
// key (the ranks' combined outputs).  Run 0 is `own`; runs 1.. lie back to back in `recv`.
// The run count and lengths are read from device memory (`meta` = [nruns, len0, len1,
// ...]), so a captured graph stays valid when they change.  A workgroup binary-searches
// its partition's range in every run and reads only those records (contiguous, no tag
// scan, no unpack).
constexpr int kMaxMergeRuns = 64;
struct RunsSource {
  const KeyCount* own;
  const KeyCount* recv;
  const u32* meta;
  PartMap pm;
  __device__ u32 part(u64 w0) const { return part_of(pm, w0); }
  struct Pre {};
  __device__ Pre prefetch(u32) const { return {}; }
  __device__ bool build(u32 p, Pre, LdsSlot* s_tab, u32* s_list, u32& s_count, u64*) const {
    // s_list: [lo, hi) per run | exclusive prefix of the partition's records | run offsets
    u32* s_lo = s_list;
    u32* s_pre = s_list + 2 * kMaxMergeRuns;
    u32* s_off = s_pre + kMaxMergeRuns + 1;
    const u32 nruns = min(meta[0], (u32)kMaxMergeRuns);
    if (threadIdx.x == 0) {
      u32 acc = 0;
      for (u32 q = 1; q < nruns; ++q) {
        s_off[q] = acc;
        acc += meta[1 + q];
      }
    }
    __syncthreads();
    if (threadIdx.x < nruns) {
      const u32 q = threadIdx.x;
      const KeyCount* r = q == 0 ? own : recv + s_off[q];
      const u32 n = meta[1 + q];
      u32 a = 0, b = n;  // first record with first byte >= p
      while (a < b) {
        const u32 mid = (a + b) >> 1;
        if (part(r[mid].w[0]) < p) a = mid + 1; else b = mid;
      }
      u32 c = a, d = n;  // first record with first byte > p
      while (c < d) {
        const u32 mid = (c + d) >> 1;
        if (part(r[mid].w[0]) <= p) c = mid + 1; else d = mid;
      }
      s_lo[2 * q] = a;
      s_lo[2 * q + 1] = c;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      u32 acc = 0;
      for (u32 q = 0; q < nruns; ++q) {
        s_pre[q] = acc;
        acc += s_lo[2 * q + 1] - s_lo[2 * q];
      }
      s_pre[nruns] = acc;
    }
    __syncthreads();
    const u32 total = s_pre[nruns];
    bool full = false;
    for (u32 e = threadIdx.x; e < total; e += kPartBlock) {
      u32 q = 0;
      while (q + 1 < nruns && s_pre[q + 1] <= e) ++q;
      const KeyCount* r = q == 0 ? own : recv + s_off[q];
      const KeyCount& rec = r[s_lo[2 * q] + (e - s_pre[q])];
      const u64 k[kKeyWords] = {rec.w[0], rec.w[1], rec.w[2], rec.w[3]};
      if (k[0] == 0 || rec.count == 0) continue;
      full |= !part_lds_insert(s_tab, k, rec.count, key_hash(k));
    }
    __syncthreads();
    return full;
  }
};

// ---------------------------------------------------------------------------------
// Large ordered build (passes past kPartBuildMaxTokens, fast map with a partition table):
// the single-kernel build would give one workgroup a hot partition's hundreds of
// thousands of tokens, so the aggregation is split in two launches.
//  dict_partials_kernel: workgroup (p, k) aggregates partition p's tokens in the k-th of
//    `nslices` slices of a tile range in an LDS table and writes the distinct keys with their
//    counts to its partial slot (KeyCount records, kPartSlots per slot) -- no global
//    atomics, no HBM hash table, hot keys combined per wave before the LDS insert.
//  dict_ordered_kernel<PartialsSource>: workgroup p merges its `nslots` partials in LDS
//    and runs the ordered kernel's sort, look-back and record output.
// ---------------------------------------------------------------------------------
constexpr u32 kPartialFull = 0xFFFFFFFFu;  // partial_n of a slot whose table overflowed

// Every thread walks the partition's runs of its own tiles (walk_runs_insert; no LDS list:
// the table is the workgroup's only LDS, so two workgroups share a CU).
__global__ __launch_bounds__(kPartBlock) void dict_partials_kernel(
    ConstKeysSoA tokens, const u64* __restrict__ counts, const u32* __restrict__ part_off,
    u32 tile_begin, u32 tile_end, u32 nslices, u32 slot_base, u32 nslots, u32 n_cap,
    KeyCount* __restrict__ partials, u32* __restrict__ partial_n,
    u64* __restrict__ trace) {
  // worker k of partition p: the workers of one partition are kDictParts apart in
  // dispatch order, so a hot partition's slices land on different CUs and XCDs
  const u32 p = blockIdx.x % kDictParts, k = blockIdx.x / kDictParts;
  const u64 slot = (u64)p * nslots + slot_base + k;
  // trace (diagnostics, LOCUST_ORD_TRACE): per slot, at trace[slot*8 + i] (100 MHz device
  // clock): 0 entry, 1 table cleared, 2 inserts done, 3 exit; 4 tokens, 5 distinct
  if (trace && threadIdx.x == 0) trace[slot * 8] = __builtin_amdgcn_s_memrealtime();
  __shared__ LdsSlot s_tab[kPartSlots];
  __shared__ u32 s_scan[kPartBlock / 64 + 1];
  __shared__ u32 s_tok;
  __shared__ u32 s_full;  // the table overflowed: every wave stops walking
  __shared__ u32 s_occ;   // claimed table slots (part_lds_insert)
  if (threadIdx.x == 0) {
    s_tok = 0;
    s_full = 0;
    s_occ = 0;
  }
  const u32 ntiles = tile_end - tile_begin;
  const u32 t0 = tile_begin + (u32)((u64)ntiles * k / nslices);
  const u32 t1 = tile_begin + (u32)((u64)ntiles * (k + 1) / nslices);
  // this thread's first run, loaded before the table clear (overlaps it)
  u32 a = 0, len = 0;
  u32 t = t0 + threadIdx.x;
  if (t < t1) {
    a = part_off[(u64)t * kPartTable + p];
    len = part_off[(u64)t * kPartTable + p + 1] - a;
  }
  for (int i = threadIdx.x; i < kPartSlots; i += kPartBlock) {
#pragma unroll
    for (int j = 0; j < kKeyWords; ++j) s_tab[i].w[j] = 0;
    s_tab[i].count = 0;
  }
  __syncthreads();
  if (trace && threadIdx.x == 0) trace[slot * 8 + 1] = __builtin_amdgcn_s_memrealtime();
  u32 ntok = 0;
  const bool full = walk_runs_insert(tokens, counts, part_off, p, t, t1, a, len, n_cap, s_tab,
                                     true, &ntok, &s_full, &s_occ);
  if (trace) atomicAdd(&s_tok, ntok);
  __syncthreads();  // every wave's inserts are in the table before it is read
  if (trace && threadIdx.x == 0) {
    trace[slot * 8 + 2] = __builtin_amdgcn_s_memrealtime();
    trace[slot * 8 + 4] = s_tok;
  }
  // dense records: thread t owns slots [t * kPartPerThread, (t + 1) * kPartPerThread)
  u32 mine = 0;
#pragma unroll
  for (int r = 0; r < kPartPerThread; ++r) mine += s_tab[threadIdx.x * kPartPerThread + r].w[0] != 0;
  u32 total = 0;
  const u32 excl = dev::block_exclusive_scan<u32, kPartBlock>(mine, s_scan, &total);
  const int any_full = __syncthreads_or(full ? 1 : 0);
  if (threadIdx.x == 0) partial_n[slot] = any_full ? kPartialFull : total;
  if (trace && threadIdx.x == 0) {
    trace[slot * 8 + 5] = total;
    trace[slot * 8 + 3] = __builtin_amdgcn_s_memrealtime();  // before the writes
  }
  if (any_full) return;
  KeyCount* out = partials + slot * kPartSlots;
  u32 id = excl;
#pragma unroll
  for (int r = 0; r < kPartPerThread; ++r) {
    const LdsSlot& sl = s_tab[threadIdx.x * kPartPerThread + r];
    if (sl.w[0] == 0) continue;
    KeyCount kc;
    kc.w[0] = sl.w[0];
#pragma unroll
    for (int j = 1; j < kKeyWords; ++j) kc.w[j] = sl.w[j] ^ kWordMagic;
    kc.count = sl.count;
    out[id++] = kc;
  }
}

// Token source of the ordered kernel after dict_partials_kernel: partition p's `nslots`
// partial slots, each a dense run of distinct keys with counts.
struct PartialsSource {
  const KeyCount* partials;
  const u32* partial_n;
  u32 nslots;  // slots per partition (<= kMaxPartialSlots)
  struct Pre {};
  __device__ Pre prefetch(u32) const { return {}; }
  __device__ bool build(u32 p, Pre, LdsSlot* s_tab, u32* s_list, u32& s_count, u64*) const {
    // s_list: [0, nslots] exclusive prefix of the slots' lengths (full: overflow)
    if (dev::wave_id() == 0) {
      const u32 q = (u32)dev::lane_id();
      const u32 nq = q < nslots ? partial_n[(u64)p * nslots + q] : 0u;
      const bool bad = q < nslots && nq == kPartialFull;
      const u32 v = bad ? 0u : nq;
      const u32 inc = dev::wave_inclusive_scan(v);
      if (q <= nslots) s_list[q] = inc - v;
      if (q == 0) s_count = dev::ballot(bad) ? 1u : 0u;
    }
    u32* occ = s_list + 128;  // claimed table slots (s_list[0 .. nslots] is the prefix)
    if (threadIdx.x == 0) *occ = 0;
    __syncthreads();
    const u32 total = s_list[nslots];
    bool full = s_count != 0;
    if (!full) {
      for (u32 e = threadIdx.x; e < total; e += kPartBlock) {
        u32 q = 0;  // the slot holding record e: binary search of the prefix
#pragma unroll
        for (u32 step = 32; step; step >>= 1)
          if (q + step < nslots && s_list[q + step] <= e) q += step;
        const KeyCount& rec = partials[((u64)p * nslots + q) * kPartSlots + (e - s_list[q])];
        const u64 kk[kKeyWords] = {rec.w[0], rec.w[1], rec.w[2], rec.w[3]};
        if (kk[0] == 0 || rec.count == 0) continue;
        full |= !part_lds_insert(s_tab, kk, rec.count, key_hash(kk), occ);
      }
    }
    __syncthreads();
    if (threadIdx.x == 0) s_count = 0;  // the ordered kernel reuses it
    __syncthreads();
    return full;
  }
};

// The compact records (kv.hpp) of m sorted entries into dst, consecutive lanes on
// consecutive words (whole lines of the host-mapped output).  word(i, j): word j of sorted
// entry i, j < kKeyWords a key word, j == kKeyWords its count.  Scratch (LDS): s_coff
// [m] u32, s_own [5 m] u16, s_scan >= kPartBlock / 64 u32.  Returns the words (uniform).
template <class Word>
__device__ u32 write_compact_records(u64* __restrict__ dst, u32 m, Word word, u32* s_coff,
                                     u16* s_own, u32* s_scan) {
  constexpr u32 kPer = kPartSlots / kPartBlock;  // entries per thread
  u32 nw[kPer], tot = 0;
#pragma unroll
  for (u32 r = 0; r < kPer; ++r) {
    const u32 i = threadIdx.x * kPer + r;
    nw[r] = 0;
    if (i < m) {
      const u64 kw[kKeyWords] = {word(i, 0), word(i, 1), word(i, 2), word(i, 3)};
      nw[r] = compact_words(kw, word(i, kKeyWords));
      tot += nw[r];
    }
  }
  u32 total = 0;
  u32 at = dev::block_exclusive_scan<u32, kPartBlock>(tot, s_scan, &total);
#pragma unroll
  for (u32 r = 0; r < kPer; ++r) {
    const u32 i = threadIdx.x * kPer + r;
    if (i < m) {
      s_coff[i] = at;
      for (u32 k = 0; k < nw[r]; ++k) s_own[at + k] = (u16)i;
      at += nw[r];
    }
  }
  __syncthreads();
  for (u32 q = threadIdx.x; q < total; q += kPartBlock) {
    const u32 i = s_own[q];
    const u32 k = q - s_coff[i];
    const u64 kw[kKeyWords] = {word(i, 0), word(i, 1), word(i, 2), word(i, 3)};
    u64 o[kCompactMaxWords];
    (void)compact_record(kw, word(i, kKeyWords), o);
    // selects, not an indexed register array (that would go through scratch)
    dst[q] = k == 0 ? o[0] : k == 1 ? o[1] : k == 2 ? o[2] : k == 3 ? o[3] : o[4];
  }
  return total;
}

// The ordered kernel's workgroup (dict_ordered_kernel).  guess: the partition whose runs
// are worth prefetching while the ticket atomic is in flight (the block index; ~0u: none).
template <class Src>
__device__ __forceinline__ void ordered_partition(
    Src src, MapCounters* __restrict__ ctr,
    OutRecord* __restrict__ out, MapCounters* __restrict__ ctr_out, u64* __restrict__ status,
    u32* __restrict__ tile_ctr, u64* __restrict__ trace, const OrderedExtra& ex, u32 guess_p) {
#define ORD_STAMP(k_)                                                          \
  if (trace && threadIdx.x == 0) trace[(u64)v * 32 + (k_)] = __builtin_amdgcn_s_memtime()
  __shared__ LdsSlot s_tab[kPartSlots];
  __shared__ __attribute__((aligned(16))) u32 s_list[kPartWindow];  // later: sort arrays
  __shared__ u32 s_count;
  __shared__ u64 s_scan[kPartBlock / 64 + 1];
  __shared__ u32 s_tile;
  __shared__ u64 s_prefix;
  __shared__ u32 s_cm, s_cfull;  // compaction: distinct keys, overflow flag
  __shared__ u64 s_ctok;         // compaction: tokens
  __shared__ u64 s_wand[kKeyWords], s_wor[kKeyWords];  // large partitions: AND / OR per key
                                                        // word (its varying bytes)
  __shared__ u32 s_rstart[256], s_rwsum[4];  // large partitions: LdsRadix digit starts
  // partition = ticket, not blockIdx: a workgroup then only ever waits in the look-back
  // on workgroups that are already running.  With blockIdx, kernels of several processes
  // sharing the GPU (the TCP / loopback rehearsals) could fill the CUs with spinning
  // workgroups whose predecessors were never dispatched: measured as multi-second stalls
  // and a hang with four ranks on one GPU.
  // 100 MHz, device-wide
  const u64 rt_entry = trace ? __builtin_amdgcn_s_memrealtime() : 0;
  // v: this workgroup's virtual partition = its ticket (the look-back order); p: the map
  // partition whose tokens it reads; (vj, vk): its share of p (see OrderedExtra::part_occ).
  // Without a plan, v == p and vk == 1.
  constexpr bool kTiles = std::is_same<Src, TileSource>::value;
  bool vplan = false;
  if constexpr (kTiles) vplan = ex.part_occ != nullptr && src.ntiles > 0 && src.ntiles <= kPartBlock;
  __shared__ u32 s_vpre[kDictParts + 1];
  __shared__ u32 s_vred[8];
  __shared__ u32 s_occ[kPartOccWords];
  u32 tp = 0, occw = 0;  // (plan) loaded before the ticket: one round trip for all
  // the plan's loads: partition thread q its estimated tokens, the others the occupancy
  auto plan_loads = [&]() {
    if constexpr (kTiles) {
      const u32 nt = src.ntiles;
      if (threadIdx.x < kDictParts) {
        // this partition's tokens, estimated from kPlanRows evenly spaced table rows
        const u32 q = threadIdx.x;
        u32 sum = 0;
#pragma unroll
        for (u32 r = 0; r < kPlanRows; ++r) {
          const u32 t = (u32)((u64)r * nt / kPlanRows);
          sum += src.part_off[(u64)t * kPartTable + q + 1] - src.part_off[(u64)t * kPartTable + q];
        }
        tp = (u32)((u64)sum * nt / kPlanRows);
      } else {
        // occupancy: thread (word w, tile slice) ORs its tiles' word w -- every load issued
        // before the first is used (one round trip, not one per tile: nt <= kPartBlock)
        const u32 i = threadIdx.x - kDictParts, w = i % kPartOccWords;
        constexpr u32 kStride = (kPartBlock - kDictParts) / kPartOccWords;
        constexpr u32 kLoads = (kPartBlock + kStride - 1) / kStride;
        u32 o[kLoads];
#pragma unroll
        for (u32 k = 0; k < kLoads; ++k) {
          const u32 t = i / kPartOccWords + k * kStride;
          o[k] = t < nt ? ex.part_occ[(u64)t * kPartOccWords + w] : 0u;
        }
#pragma unroll
        for (u32 k = 0; k < kLoads; ++k) occw |= o[k];
      }
    }
  };
  // plan_flag: plan only if the map saw a crowded partition -- the flag's load rides with
  // the ticket and the guessed prefetch; the plan's own loads wait for it
  const bool triggered = vplan && ex.plan_flag != nullptr;
  u32 flag = 0;
  if (triggered) flag = __hip_atomic_load(ex.plan_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (vplan && !triggered) plan_loads();
  // Tickets almost always come out in dispatch order: prefetch the run table for
  // p = blockIdx.x while the ticket atomic is in flight, reload only on a mismatch.  (With
  // a plan too: a plan that splits nothing keeps v = p, and the guess holds.)
  const bool guessing = guess_p != ~0u;
  const typename Src::Pre guess = guessing ? src.prefetch(guess_p) : typename Src::Pre{};
  // The ticket atomic is issued first and the table cleared while it and the plan's loads
  // are in flight (the clear needs neither).  The table's slots in use: all, or (tile
  // sources) the first kSmallTable until a build finds more tokens (grow_table).
  __shared__ u32 s_tmask;
  u32 ticket = 0;
  if (threadIdx.x == 0) ticket = atomicAdd(tile_ctr, 1u);  // its value is waited for below
  const u32 tmask0 = kTiles ? kSmallTable - 1 : (u32)kPartSlots - 1;
  for (int i = threadIdx.x; i <= (int)tmask0; i += kPartBlock) {
#pragma unroll
    for (int j = 0; j < kKeyWords; ++j) s_tab[i].w[j] = 0;
    s_tab[i].count = 0;
  }
  if (threadIdx.x == 0) {
    s_count = 0;
    s_cm = 0;
    s_ctok = 0;
    s_cfull = 0;
    s_tmask = tmask0;
    s_tile = ticket;
  }
  if (triggered) {  // uniform: every thread read the same word
    vplan = flag != 0;
    if (vplan) plan_loads();
  }
  u32 v, p, vj = 0, vk = 1;
  bool identity = !vplan;  // v = p: one workgroup per map partition
  if (!vplan) {
    __syncthreads();  // s_tile (and the cleared table)
    v = p = s_tile;
  } else {
    if (threadIdx.x < kPartOccWords) s_occ[threadIdx.x] = 0;
    __syncthreads();
    if (threadIdx.x >= kDictParts && occw) atomicOr(&s_occ[(threadIdx.x - kDictParts) % kPartOccWords], occw);
    __syncthreads();
    const bool occupied = threadIdx.x < kDictParts && ((s_occ[threadIdx.x >> 5] >> (threadIdx.x & 31)) & 1u);
    if (threadIdx.x < kDictParts) {  // non-empty partitions E (exact), estimated tokens T
      if (!occupied) tp = 0;
      const u64 nz = dev::ballot(occupied);
      const u32 tsum = dev::wave_reduce_sum(tp);
      if (dev::lane_id() == 0) {
        s_vred[dev::wave_id()] = (u32)__popcll(nz);
        s_vred[4 + dev::wave_id()] = tsum;
      }
    }
    __syncthreads();
    v = s_tile;
    const u32 E = s_vred[0] + s_vred[1] + s_vred[2] + s_vred[3];
    const u32 T = s_vred[4] + s_vred[5] + s_vred[6] + s_vred[7];
    // workgroups of partition q: one if it has tokens, plus its token share of the idle
    // ones (at least kSplitMinTokens tokens per extra one); the sum is at most kDictParts
    u32 K = 0;
    if (occupied) {
      const u32 extra = T ? (u32)((u64)tp * (u32)(kDictParts - E) / T) : 0u;
      K = 1u + min(extra, tp / (ex.split_min ? ex.split_min : kSplitMinTokens));
    }
    u32 kinc = 0;
    if (threadIdx.x < kDictParts) {
      kinc = dev::wave_inclusive_scan(K);
      if (dev::lane_id() == 63) s_vred[dev::wave_id()] = kinc;
    }
    __syncthreads();
    if (threadIdx.x < kDictParts) {
      u32 off = 0;
      for (int i = 0; i < dev::wave_id(); ++i) off += s_vred[i];
      s_vpre[threadIdx.x] = off + kinc - K;
      if (threadIdx.x == kDictParts - 1) s_vpre[kDictParts] = off + kinc;
    }
    __syncthreads();
    const u32 V = s_vpre[kDictParts];
    // nothing split (V == E): one workgroup per map partition, v = p, as without a plan --
    // the run table prefetched for the guessed partition is then usually the right one
    identity = V == E;
    // the map partition holding v: the last q with s_vpre[q] <= v (s_vpre[256] = V > v)
    p = 0;
    vk = 0;  // v >= V: an idle workgroup -- an empty virtual partition in the chain
    if (identity) {
      p = v;
      vk = 1;
    } else if (v < V) {
#pragma unroll
      for (u32 step = kDictParts / 2; step; step >>= 1)
        if (s_vpre[p + step] <= v) p += step;
      vj = v - s_vpre[p];
      vk = s_vpre[p + 1] - s_vpre[p];
    }
  }
  ORD_STAMP(0);
  if (trace && threadIdx.x == 0) {
    trace[(u64)v * 32 + 10] = rt_entry;
    trace[(u64)v * 32 + 20] = 0;
    trace[(u64)v * 32 + 16] = 0;
    trace[(u64)v * 32 + 17] = ~0ull;
    trace[(u64)v * 32 + 18] = 0;
    trace[(u64)v * 32 + 19] = 0;
    trace[(u64)v * 32 + 26] = 0;
    trace[(u64)v * 32 + 27] = 0;
    trace[(u64)v * 32 + 28] = 0;
  }
  const typename Src::Pre first = identity && guessing && p == guess_p ? guess
                                  : vk ? src.prefetch(p) : typename Src::Pre{};
  __syncthreads();
  ORD_STAMP(14);  // table cleared
  bool full = false;
  if constexpr (kTiles) {
    if (vk > 1)
      full = src.build_split(p, first, vj, vk, s_tab, s_list, reinterpret_cast<u32*>(s_scan),
                             trace ? trace + (u64)v * 32 : nullptr, tmask0, &s_tmask);
    else if (vk == 1)
      full = src.build(p, first, s_tab, s_list, s_count, trace ? trace + (u64)v * 32 : nullptr,
                       tmask0, &s_tmask);
  } else {
    full = src.build(p, first, s_tab, s_list, s_count, trace ? trace + (u64)v * 32 : nullptr);
  }
  ORD_STAMP(1);
  // ---- compact: dense (w0, slot) arrays in the list area ----
  u64* s_w0 = reinterpret_cast<u64*>(s_list);            // [kPartSlots]
  u32* s_slot = s_list + 2 * kPartSlots;                 // [kPartSlots]
  const u32 nslots = s_tmask + 1;  // (the build's barriers publish a grown table's mask)
  u32 mine = 0;
  u64 wsum = 0;
#pragma unroll
  for (int r = 0; r < kPartPerThread; ++r) {
    const u32 slot = threadIdx.x * kPartPerThread + r;
    const LdsSlot& sl = s_tab[slot < nslots ? slot : 0];
    if (slot < nslots && sl.w[0]) {
      ++mine;
      wsum += sl.count;
    }
  }
  // Positions in the compacted arrays: any order will do (they are sorted next), so a wave
  // takes its slice with ONE LDS atomic and its lanes' offsets come from two ballots --
  // no block scan, one barrier.  Token sums and the overflow flag ride along.
  u32* s_rk = s_list + 3 * kPartSlots + 2 * kSmallRank;         // [kSmallRank] ranks
  u32* s_rkw = s_rk + kSmallRank;  // [kSmallRank] compact word offsets (weighted ranks)
  u64* s_out = reinterpret_cast<u64*>(s_rk + 2 * kSmallRank);    // [5 x kSmallRank] records
  u64* s_k123 = s_out + 6 * kSmallRank;                          // [3 x kSmallRank] words 1-3
  u32* s_cw = reinterpret_cast<u32*>(s_k123 + 3 * kSmallRank);   // [kSmallRank] compact words
  // this thread's live slots from position d on: (w0, slot) and, for the small path, the
  // key's other words and compact size
  auto write_compacted = [&](u32 d) {
#pragma unroll
    for (int r = 0; r < kPartPerThread; ++r) {
      const u32 slot = threadIdx.x * kPartPerThread + r;
      if (slot < nslots && s_tab[slot].w[0]) {
        s_w0[d] = s_tab[slot].w[0];
        s_slot[d] = slot;
        if (d < kSmallRank) {
          u64 kw[kKeyWords];
          kw[0] = s_tab[slot].w[0];
#pragma unroll
          for (int j = 1; j < kKeyWords; ++j) {
            kw[j] = s_tab[slot].w[j] ^ kWordMagic;
            s_k123[3 * d + j - 1] = kw[j];
          }
          s_cw[d] = compact_words(kw, s_tab[slot].count);
        }
        ++d;
      }
    }
    if (threadIdx.x < kSmallRank) {
      s_rk[threadIdx.x] = 0;
      s_rkw[threadIdx.x] = 0;
    }
  };
  u32 cpos = 0;
  {
    const u64 b0 = dev::ballot(mine >= 1), b1 = dev::ballot(mine >= 2);
    const u64 wfull = dev::ballot(full);
    const u64 wtok_incl = dev::wave_inclusive_scan(wsum);
    u32 wbase = 0;
    if (dev::lane_id() == 63) {
      wbase = atomicAdd(&s_cm, (u32)(__popcll(b0) + __popcll(b1)));
      atomicAdd(reinterpret_cast<unsigned long long*>(&s_ctok), (unsigned long long)wtok_incl);
      if (wfull) s_cfull = 1u;
    }
    wbase = (u32)__builtin_amdgcn_readlane((int)wbase, 63);
    cpos = wbase + dev::lanes_below(b0) + dev::lanes_below(b1);
  }
  __syncthreads();  // the sums are complete
  const u32 m = s_cm;
  const int any_full = s_cfull != 0u;
  const u64 tok = s_ctok;
  // Small partitions (the common case once the partition map is balanced) skip the
  // bucket sort: ranks come from one all-pairs pass (see below).
  const bool small = !any_full && m <= kSmallRank;
  // ---- publish (distinct keys, tokens, overflow) now; the look-back resolves after the
  // sort, which does not need the prefix -- so waiting for predecessors overlaps it ----
  const u64 agg = (u64)m | ((u64)(any_full ? 1 : 0) << kOrdOvfShift) | (tok << kOrdTokShift);
  if (threadIdx.x == 0) dev::publish_aggregate(status, v, agg);
  ORD_STAMP(2);
  // the compacted arrays after the publish: successors stop waiting sooner
  write_compacted(cpos);
  __syncthreads();
  u64 pre = 0;
  u32 cwords = ~0u;  // compact words written (ex.cout), ~0u: none
  if (small) {
    // ---- small partition: all-pairs ranks: rank_i = #{j : key_j < key_i}, the sorted
    // position in one pass, no bucket sort.  Wave 0 resolves the look-back meanwhile. ----
    if (dev::wave_id() == 0) {
      // Look-back in ONE round trip: wave 0 reads every predecessor's status word at once
      // (4 per lane, p < 256) instead of walking back 64 words per dependent round trip
      // (~1-2 us each across XCDs).  prefix = the highest inclusive value found + the
      // aggregates above it.  Predecessors hold lower tickets, so they are running and
      // publish soon; a lane spins until its word is published.
      const u32 lane = (u32)dev::lane_id();
      u64 st[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const u32 q = lane + 64u * k;
        st[k] = q < v ? dev::ld_agent(&status[q]) : dev::kLbAgg;  // beyond v: aggregate 0
      }
      // unpublished words are re-read together, every round (one round trip per round, not
      // one per group of 64 in turn)
      auto pending = [&]() {
        bool any = false;
#pragma unroll
        for (int k = 0; k < 4; ++k) any |= lane + 64u * k < v && (st[k] >> dev::kLbFlagShift) == 0;
        return any;
      };
      while (dev::ballot(pending())) {
        __builtin_amdgcn_s_sleep(1);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const u32 q = lane + 64u * k;
          if (q < v && (st[k] >> dev::kLbFlagShift) == 0) st[k] = dev::ld_agent(&status[q]);
        }
      }
      int hi_inc = -1;  // highest predecessor with an inclusive value
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const u64 b = dev::ballot((st[k] >> dev::kLbFlagShift) == 2);
        if (b) hi_inc = 64 * k + 63 - __clzll((long long)b);
      }
      u64 pv = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int q = (int)lane + 64 * k;
        if (q >= hi_inc && q < (int)v) pv += st[k] & dev::kLbValMask;
      }
      pv = dev::wave_inclusive_scan(pv);
      if (lane == 63) s_prefix = pv;
      if (trace && lane == 0) trace[(u64)v * 32 + 15] = __builtin_amdgcn_s_memtime();  // resolved
    } else if (m > 1) {
      if (trace && dev::lane_id() == 0)  // the first ranking wave's start
        atomicMin(reinterpret_cast<unsigned long long*>(&trace[(u64)v * 32 + 17]),
                  (unsigned long long)__builtin_amdgcn_s_memtime());
      // Waves 1..15 split the work as (key group of 64, candidate slice): lane i of its
      // group compares its full key with every candidate of the slice -- the candidates'
      // words are LDS broadcasts, four in flight -- and the partial rank goes to LDS with
      // one atomic.  Full-key compares: no tie pass.
      const u32 G = (m + 63) / 64;                 // key groups (m <= kSmallRank = 256)
      const u32 S = (u32)(kPartBlock / 64 - 1) / G;  // candidate slices per group (>= 3)
      const u32 wv = (u32)dev::wave_id() - 1u, g = wv % G, sl = wv / G;
      if (sl < S) {
        const u32 i = g * 64 + (u32)dev::lane_id();
        const bool own = i < m;
        u64 k0 = 0, k1 = 0, k2 = 0, k3 = 0;
        if (own) {
          k0 = s_w0[i];
          k1 = s_k123[3 * i];
          k2 = s_k123[3 * i + 1];
          k3 = s_k123[3 * i + 2];
        }
        const u32 j0 = sl * m / S, j1 = (sl + 1) * m / S;
        u32 cnt = 0;
        u32 wcnt = 0;  // compact words of the smaller keys: this key's compact offset
        // first words only (12 of the 36 LDS bytes per candidate): the further words are
        // read for a candidate whose first word equals this key's -- rare (keys of 8+
        // bytes sharing their first 8), and a divergent branch
        for (u32 j = j0; j < j1; j += 4) {
          u64 c0[4];
          u32 cw[4];
#pragma unroll
          for (u32 q = 0; q < 4; ++q) {
            const u32 jj = j + q < j1 ? j + q : j0;
            c0[q] = s_w0[jj];
            cw[q] = s_cw[jj];
          }
#pragma unroll
          for (u32 q = 0; q < 4; ++q) {
            const u32 jj = j + q;
            bool lt = jj < j1 && c0[q] < k0;
            if (jj < j1 && c0[q] == k0 && jj != i) {
              const u64 c1 = s_k123[3 * jj], c2 = s_k123[3 * jj + 1], c3 = s_k123[3 * jj + 2];
              lt = c1 < k1 || (c1 == k1 && (c2 < k2 || (c2 == k2 && c3 < k3)));
            }
            cnt += lt ? 1u : 0u;
            wcnt += lt ? cw[q] : 0u;
          }
        }
        // one lane per wave: 64 lanes' same-address atomics serialise and inflated the
        // traced ranking / look-back phases by ~10 us
        if (trace && dev::lane_id() == 0)
          atomicMax(reinterpret_cast<unsigned long long*>(&trace[(u64)v * 32 + 18]),
                    (unsigned long long)__builtin_amdgcn_s_memtime());
        if (own && cnt) {
          atomicAdd(&s_rk[i], cnt);
          atomicAdd(&s_rkw[i], wcnt);
        }
      }
      if (trace && dev::lane_id() == 0)  // the slowest ranking wave's end
        atomicMax(reinterpret_cast<unsigned long long*>(&trace[(u64)v * 32 + 16]),
                  (unsigned long long)__builtin_amdgcn_s_memtime());
    }
    __syncthreads();
    pre = s_prefix;
    if (threadIdx.x == 0 && v != 0)  // inclusive value for later walkers
      dev::st_agent(&status[v], dev::kLbInc | (pre + agg));
    ORD_STAMP(3);
    ORD_STAMP(4);
    // stage the 40-B records (= KeyCount) in sorted order -- or, for the host output, the
    // compact records at their weighted ranks -- then write them with consecutive lanes on
    // consecutive words (full lines: matters most for the host-mapped output)
    const bool cstage = ex.cout && !ex.recs && !ex.sorted.w[0];
    __shared__ u32 s_cwords;
    for (u32 i = threadIdx.x; i < m; i += kPartBlock) {
      const LdsSlot& sl = s_tab[s_slot[i]];
      const u64 w1 = sl.w[1] ^ kWordMagic, w2 = sl.w[2] ^ kWordMagic, w3 = sl.w[3] ^ kWordMagic;
      if (cstage) {
        const u64 kw[kKeyWords] = {sl.w[0], w1, w2, w3};
        u64 rec[kCompactMaxWords];
        const u32 nwd = compact_record(kw, sl.count, rec);
        u64* o = s_out + s_rkw[i];
#pragma unroll
        for (u32 q = 0; q < (u32)kCompactMaxWords; ++q)
          if (q < nwd) o[q] = rec[q];
        if (s_rk[i] == m - 1) s_cwords = s_rkw[i] + nwd;  // the last key's end
      } else {
        u64* o = s_out + kOutWords * s_rk[i];
        o[0] = sl.w[0];
        o[1] = w1;
        o[2] = w2;
        o[3] = w3;
        o[4] = sl.count;
      }
    }
    __syncthreads();
    const u64 base_m = pre & kOrdM;
    if (((pre >> kOrdOvfShift) & 511u) == 0) {  // uniform per workgroup
      if (cstage) {  // the staged compact records, at the word their 40-B ones would start
        const u32 cw = m ? s_cwords : 0u;
        if (base_m + m <= ex.out_cap) {
          u64* dst = ex.cout + kOutWords * base_m;
          for (u32 q = threadIdx.x; q < cw; q += kPartBlock) dst[q] = s_out[q];
          cwords = cw;
        }
      } else if (out && base_m + m <= ex.out_cap) {  // 8 B per lane, consecutive lanes
        u64* dst = reinterpret_cast<u64*>(out + base_m);
        for (u32 q = threadIdx.x; q < kOutWords * m; q += kPartBlock) dst[q] = s_out[q];
      }
      if (ex.recs) {  // the same words as a KeyCount slice
        u64* dst = reinterpret_cast<u64*>(ex.recs + base_m);
        for (u32 q = threadIdx.x; q < kOutWords * m; q += kPartBlock) dst[q] = s_out[q];
      }
      if (ex.sorted.w[0]) {
        for (u32 i = threadIdx.x; i < m; i += kPartBlock) {
#pragma unroll
          for (int j = 0; j < kKeyWords; ++j) ex.sorted.w[j][base_m + i] = s_out[kOutWords * i + j];
          if (ex.counts) ex.counts[base_m + i] = s_out[kOutWords * i + 4];
        }
      }
    }
  } else {
  // ---- sort the partition's distinct keys ----
  __syncthreads();  // the build's table, (w0, slot) lists and token window are complete
  if (!any_full && m > 1 && m <= (u32)kPartBlock) {
    // Bitonic network over the next power of two N >= m, one key per thread, (w0, slot) in
    // registers; padding sorts last (w0 = ~0: no key is all 0xFF bytes).  Strides below
    // 64 exchange through cross-lane shuffles, the 10 longer ones (N = 1024) through
    // double-buffered LDS with one barrier each.  Keys tied on their first word compare
    // their other words in the table (ord_greater).  The LSD radix below took ~61K cycles
    // for a 1,022-key partition of synth1m (10-14 byte passes, 3-4 barriers each): the
    // ordered kernel's records could not start their PCIe drain before that.
    const u32 N = m <= 64u ? 64u : 1u << (32 - __clz((int)(m - 1)));
    u64* s_bw = reinterpret_cast<u64*>(s_list + 3 * kPartSlots);  // [2][kPartBlock]
    u32* s_bs = s_list + 7 * kPartSlots;                           // [2][kPartBlock]
    const u32 t = threadIdx.x;
    u64 w = ~0ull;
    u32 sl = 0xFFFFFFFFu;
    if (t < m) {
      w = s_w0[t];
      sl = s_slot[t];
    }
    int buf = 0;
    for (u32 k = 2; k <= N; k <<= 1) {
      for (u32 jj = k >> 1; jj > 0; jj >>= 1) {
        u64 pw;
        u32 ps;
        if (jj >= 64u) {  // partner in another wave (uniform branch)
          if (t < N) {
            s_bw[buf * kPartBlock + t] = w;
            s_bs[buf * kPartBlock + t] = sl;
          }
          __syncthreads();
          pw = t < N ? s_bw[buf * kPartBlock + (t ^ jj)] : ~0ull;
          ps = t < N ? s_bs[buf * kPartBlock + (t ^ jj)] : 0xFFFFFFFFu;
          buf ^= 1;
        } else {
          pw = (u64)__shfl_xor((long long)w, (int)jj, 64);
          ps = (u32)__shfl_xor((int)sl, (int)jj, 64);
        }
        if (t < N) {
          const bool up = (t & k) == 0, lower = (t & jj) == 0;
          const bool less = ord_greater(pw, ps, w, sl, s_tab);  // mine < partner
          if ((lower == up) ? !less : less) {
            w = pw;
            sl = ps;
          }
        }
      }
    }
    __syncthreads();  // every thread has its first (w0, slot) loaded
    if (t < m) {
      s_w0[t] = w;
      s_slot[t] = sl;
    }
  } else if (!any_full && m > 1) {
    // LSD radix sort of the partition's distinct keys in LDS over the bytes that vary
    // (dev::LdsRadix, as the partitioned token sort): word 3 down to word 0, low byte to
    // high, stable.  A bucket + all-pairs ranking degenerated on skewed key sets
    // -- most keys in one bucket, long keys tied on their first word: up to 295K cycles
    // for one 1,003-key partition of the synthetic text (git history keeps that path).
    using Radix = dev::LdsRadix<kPartBlock, kPartSlots, u16>;
    u64* s_word = reinterpret_cast<u64*>(s_list + 3 * kPartSlots);          // [kPartSlots]
    auto s_perm = reinterpret_cast<u16 (*)[kPartSlots]>(s_list + 5 * kPartSlots);  // [2][..]
    auto s_rcnt = reinterpret_cast<u16 (*)[256]>(s_list + 6 * kPartSlots);   // [16][256]
    auto s_rwex = reinterpret_cast<u16 (*)[256]>(s_list + 7 * kPartSlots);   // [16][256]
    const Radix R{s_word, s_perm, s_rcnt, s_rwex, s_rstart, s_rwsum};
    R.init();
    for (u32 i = threadIdx.x; i < m; i += kPartBlock) s_perm[0][i] = (u16)i;
    if (threadIdx.x < (u32)kKeyWords) {
      s_wand[threadIdx.x] = ~0ull;
      s_wor[threadIdx.x] = 0;
    }
    int cur = 0;
    for (int j = kKeyWords - 1; j >= 0; --j) {
      __syncthreads();  // the previous word's passes are done with s_word
      u64 a_ = ~0ull, o_ = 0;
      for (u32 i = threadIdx.x; i < m; i += kPartBlock) {
        const u64 w = j == 0 ? s_w0[i] : s_tab[s_slot[i]].w[j] ^ kWordMagic;
        s_word[i] = w;
        a_ &= w;
        o_ |= w;
      }
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) {
        a_ &= __shfl_xor(a_, off, 64);
        o_ |= __shfl_xor(o_, off, 64);
      }
      if (dev::lane_id() == 0) {
        atomicAnd(reinterpret_cast<unsigned long long*>(&s_wand[j]), (unsigned long long)a_);
        atomicOr(reinterpret_cast<unsigned long long*>(&s_wor[j]), (unsigned long long)o_);
      }
      __syncthreads();
      const u64 diff = s_wand[j] ^ s_wor[j];  // bits that differ between keys
      for (u32 b = 0; b < 8; ++b)
        if ((diff >> (8 * b)) & 0xffull) {
          R.pass(s_word, m, 8 * b, cur);
          cur ^= 1;
        }
    }
    // sorted position d holds item s_perm[cur][d]: permute (w0, slot) through registers
    constexpr u32 kPer2 = kPartSlots / kPartBlock;
    u64 pw[kPer2];
    u32 ps[kPer2];
#pragma unroll
    for (u32 r = 0; r < kPer2; ++r) {
      const u32 d = threadIdx.x + r * kPartBlock;
      if (d < m) {
        const u32 it = s_perm[cur][d];
        pw[r] = s_w0[it];
        ps[r] = s_slot[it];
      }
    }
    __syncthreads();
#pragma unroll
    for (u32 r = 0; r < kPer2; ++r) {
      const u32 d = threadIdx.x + r * kPartBlock;
      if (d < m) {
        s_w0[d] = pw[r];
        s_slot[d] = ps[r];
      }
    }
  }
  __syncthreads();
  ORD_STAMP(3);
  if (dev::wave_id() == 0) {
    const u64 e = dev::wave_lookback_resolve(status, v, agg);
    if (dev::lane_id() == 0) s_prefix = e;
  }
  __syncthreads();
  pre = s_prefix;
  ORD_STAMP(4);
  const u64 base_m = pre & kOrdM;
  const u32 ovf_before = (u32)((pre >> kOrdOvfShift) & 511u);
  // ---- write the records ----
  if (!any_full && ovf_before == 0) {  // uniform per workgroup
    // every output is written with consecutive lanes on consecutive words: full-line
    // writes, which matters most for the host-mapped output (each partial line would be
    // its own PCIe write).  The 40-B records and the KeyCount slice are the same words.
    auto word = [&](u32 q) {
      const u32 i = q / kOutWords, wd = q - kOutWords * i;
      const LdsSlot& sl = s_tab[s_slot[i]];
      return wd == 0 ? sl.w[0] : wd < (u32)kKeyWords ? sl.w[wd] ^ kWordMagic : sl.count;
    };
    if (ex.cout && base_m + m <= ex.out_cap) {
      // scratch past the sorted (w0, slot) arrays: s_list[24 KB, 52 KB)
      u32* s_coff = s_list + 3 * kPartSlots;
      u16* s_own = reinterpret_cast<u16*>(s_coff + kPartSlots);
      cwords = write_compact_records(
          ex.cout + kOutWords * base_m, m,
          [&](u32 i, u32 j) {
            const LdsSlot& sl = s_tab[s_slot[i]];
            return j == 0 ? sl.w[0] : j < (u32)kKeyWords ? sl.w[j] ^ kWordMagic : sl.count;
          },
          s_coff, s_own, reinterpret_cast<u32*>(s_scan));
    } else if (out && base_m + m <= ex.out_cap) {
      u64* dst = reinterpret_cast<u64*>(out + base_m);
      for (u32 q = threadIdx.x; q < kOutWords * m; q += kPartBlock) dst[q] = word(q);
    }
    if (ex.recs) {
      u64* dst = reinterpret_cast<u64*>(ex.recs + base_m);
      for (u32 q = threadIdx.x; q < kOutWords * m; q += kPartBlock) dst[q] = word(q);
    }
    if (ex.sorted.w[0]) {
      for (u32 i = threadIdx.x; i < m; i += kPartBlock) {
        const LdsSlot& sl = s_tab[s_slot[i]];
        ex.sorted.w[0][base_m + i] = sl.w[0];
#pragma unroll
        for (int j = 1; j < kKeyWords; ++j) ex.sorted.w[j][base_m + i] = sl.w[j] ^ kWordMagic;
        if (ex.counts) ex.counts[base_m + i] = sl.count;
      }
    }
  }
  }  // bucket-sorted (large) partition
  const u64 base_m = pre & kOrdM;
  const u64 base_tok = pre >> kOrdTokShift;
  const u32 ovf_before = (u32)((pre >> kOrdOvfShift) & 511u);
  ORD_STAMP(5);
  if (ex.ctab && threadIdx.x == 0)
    ex.ctab[v] = cwords == ~0u ? ~0ull : (u64)m | ((u64)cwords << 16) | (base_m << 32);
  static_assert((u64)kPartSlots * kCompactMaxWords < (1u << 16), "ctab: entries / words fields");
  if (trace && threadIdx.x == 0) trace[(u64)v * 32 + 6] = m;
  if (trace && threadIdx.x == 0) trace[(u64)v * 32 + 11] = __builtin_amdgcn_s_memrealtime();
  if (ex.part_w && threadIdx.x == 0 && vj == 0 && vk > 0) {  // partition work, for the retuning
    // (a partition split over vk workgroups: its first one's share, times vk)
    const u64 w = (tok + (u64)kPartDistinctWeight * m) * (vplan ? vk : 1u);
    ex.part_w[p] = (u32)(w < 0xffffffffull ? w : 0xffffffffull);
  }
  // ---- the run's counters: the last partition's look-back prefix ----
  auto publish_totals = [&](u32 u, u64 total, u64 ovf_total) {
    ctr->num_unique = u;
    ctr->total_count = total;
    if (ovf_total) ctr->flags |= kCtrDictOverflow;
    if (ctr_out) {
      ctr_out->num_records = ctr->num_records;
      ctr_out->map_tokens = ctr->map_tokens;
      ctr_out->num_unique = u;
      ctr_out->overflow_lines = ctr->overflow_lines;
      ctr_out->truncated = ctr->truncated;
      ctr_out->num_newlines = ctr->num_newlines;
      ctr_out->max_key_len = ctr->max_key_len;
      ctr_out->total_count = total;
      ctr_out->flags = ctr->flags | (ovf_total ? kCtrDictOverflow : 0u);
    }
    if (ex.hdr) {  // the gather slot's header: this rank's records are complete
      // field by field from the template: a whole-struct copy went through private memory
      // (64 B of scratch per lane for every ordered kernel, and its setup at each launch)
      SlotHeader* hd = ex.hdr;
      hd->status = ovf_total ? kSlotRedo : ex.tmpl.status;
      hd->record_flags = ex.tmpl.record_flags;
      hd->n = u;
      hd->lines = ex.tmpl.lines;
      hd->tokens = ctr->num_records;
      hd->overflow_lines = ctr->overflow_lines;
      hd->truncated = ctr->truncated;
      hd->max_key_len = ctr->max_key_len;
      hd->slot_cap = ex.tmpl.slot_cap;
      hd->pad[0] = ex.tmpl.pad[0];
      hd->pad[1] = ex.tmpl.pad[1];
    }
  };
  const u64 ovf_total = ovf_before + (any_full ? 1u : 0u);  // uniform per workgroup
  if (v == kDictParts - 1 && threadIdx.x == 0)
    publish_totals((u32)(base_m + m), base_tok + tok, ovf_total);
  if (ex.self_clean) {
    // Self-cleaning job: the LAST workgroup to finish (not partition 255 -- a partition
    // resolves its prefix from its predecessors' aggregates, so later ones may finish
    // first while earlier ones still read look-back words) re-zeroes the counters and
    // every look-back word, unless a partition overflowed (the host then redoes the
    // Process stage from these counters and resets everything itself).
    __syncthreads();
    if (threadIdx.x == 0) {
      // release this workgroup's counter / status writes (and, when the host is told of the
      // end, its host-mapped records: system scope); release only -- the last workgroup
      // acquires (an acq_rel fence here also invalidated this XCD's caches, every time)
      if (ex.host_done)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      else
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      s_count = atomicAdd(ex.done_counter, 1u) == (u32)kDictParts - 1 ? 1u : 0u;
      if (trace) trace[(u64)v * 32 + 25] = __builtin_amdgcn_s_memrealtime();
    }
    __syncthreads();
    if (s_count) {
      // Tell the host first: every workgroup's records, counters and headers are out --
      // each one, this one included, released them at system scope (L2 written back, the
      // writes waited for) before counting itself done, and this one saw all 256 counts.
      // So the store is relaxed: a release here wrote the L2 back again and waited for the
      // acquire's load below, two more memory round trips before the host could see it.
      // The re-zeroing below touches device scratch only, which the next job's kernels --
      // behind this one on the stream -- see complete; the host's turnaround overlaps it.
      if (ex.host_done && threadIdx.x == 0)
        __hip_atomic_store(ex.host_done, ex.host_done_value, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
      // acquire every other workgroup's (acquire only: this one released its own already)
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      const u32 flags = __hip_atomic_load(&ctr->flags, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (!(flags & kCtrDictOverflow)) {
        for (u32 i = threadIdx.x; i < ex.map_words; i += kPartBlock) ex.map_lb.status[i] = 0;
        for (u32 i = threadIdx.x; i <= (u32)kDictParts; i += kPartBlock) status[i] = 0;
        if (threadIdx.x == 0) {
          // the accumulated counters; num_unique / total_count are assignments the next
          // run overwrites, and stay readable for what follows this kernel
          ctr->num_records = 0;
          ctr->overflow_lines = 0;
          ctr->truncated = 0;
          ctr->num_newlines = 0;
          ctr->max_key_len = 0;
          ctr->flags = 0;
          *tile_ctr = 0;
          *ex.map_lb.tile_counter = 0;
          *ex.done_counter = 0;
          if (ex.plan_flag) *ex.plan_flag = 0;
        }
      }
      __syncthreads();
      if (trace && threadIdx.x == 0) trace[(u64)v * 32 + 24] = __builtin_amdgcn_s_memrealtime();
    }
  }
}
#undef ORD_STAMP

template <class Src>
__global__ __launch_bounds__(kPartBlock) void dict_ordered_kernel(
    Src src, MapCounters* __restrict__ ctr,
    OutRecord* __restrict__ out, MapCounters* __restrict__ ctr_out, u64* __restrict__ status,
    u32* __restrict__ tile_ctr, u64* __restrict__ trace, OrderedExtra ex) {
  ordered_partition(src, ctr, out, ctr_out, status, tile_ctr, trace, ex, blockIdx.x);
}

// rank[i] += #{ j in tile : key[j] < key[i] }, persistent over (i-tile, j-tile) pairs.
constexpr int kRankI = 256;
constexpr int kRankJ = 256;

__device__ __forceinline__ bool key_lt(const u64* a, const u64* b) {
#pragma unroll
  for (int j = 0; j < kKeyWords; ++j)
    if (a[j] != b[j]) return a[j] < b[j];
  return false;
}

// With `counts`, val[i] also accumulates the total count of the smaller keys: the
// "weighted rank" IS the reference's val (start of the key's run in the sorted token
// array), so no scan over the sorted counts is needed afterwards.
template <bool kWeighted>
__global__ __launch_bounds__(kRankI) void rank_sort_kernel(ConstKeysSoA keys,
                                                           const u64* __restrict__ counts,
                                                           const u32* __restrict__ d_u,
                                                           u32* __restrict__ rank,
                                                           u64* __restrict__ val,
                                                           u32 ucap) {
  __shared__ __attribute__((aligned(16))) u64 s_w0[kRankJ];
  __shared__ __attribute__((aligned(16))) u64 s_cnt[kRankJ];
  __shared__ u64 s_rest[kRankJ][kKeyWords - 1];
  const u32 u = min(*d_u, ucap);  // > ucap only after a dictionary overflow (result unused)
  if (u > (u32)kRankSortMax) return;  // radix path handles it
  const u32 ti = (u32)div_up(u, kRankI), tj = (u32)div_up(u, kRankJ);
  for (u32 pair = blockIdx.x; pair < ti * tj; pair += gridDim.x) {
    const u32 bi = pair % ti, bj = pair / ti;
    const u32 j0 = bj * kRankJ;
    const u32 jn = min((u32)kRankJ, u - j0);
    __syncthreads();  // previous pair's readers are done with the tile
    {
      constexpr int kTrips = kRankJ / kRankI;
      u64 v[kTrips][kKeyWords], cv[kTrips];  // issue every load before any LDS store
#pragma unroll
      for (int r = 0; r < kTrips; ++r) {
        const u32 t = threadIdx.x + r * kRankI;
#pragma unroll
        for (int q = 0; q < kKeyWords; ++q) v[r][q] = t < jn ? keys.w[q][j0 + t] : 0;
        cv[r] = (kWeighted && t < jn) ? counts[j0 + t] : 0;
      }
#pragma unroll
      for (int r = 0; r < kTrips; ++r) {
        const u32 t = threadIdx.x + r * kRankI;
        // padding keys are all-ones: never smaller than a real key
        s_w0[t] = t < jn ? v[r][0] : ~0ull;
        s_cnt[t] = cv[r];
#pragma unroll
        for (int q = 1; q < kKeyWords; ++q) s_rest[t][q - 1] = v[r][q];
      }
    }
    __syncthreads();
    const u32 i = bi * kRankI + threadIdx.x;
    if (i >= u) continue;
    u64 me[kKeyWords];
#pragma unroll
    for (int q = 0; q < kKeyWords; ++q) me[q] = keys.w[q][i];
    u32 cnt = 0, eq = 0;
    u64 acc = 0;
    // 16-byte broadcast reads, 4 keys per step, independent accumulations
    for (u32 t = 0; t < (u32)kRankJ; t += 4) {
      const uint4 a = *reinterpret_cast<const uint4*>(&s_w0[t]);
      const uint4 b = *reinterpret_cast<const uint4*>(&s_w0[t + 2]);
      uint4 ca{0, 0, 0, 0}, cb{0, 0, 0, 0};
      if (kWeighted) {
        ca = *reinterpret_cast<const uint4*>(&s_cnt[t]);
        cb = *reinterpret_cast<const uint4*>(&s_cnt[t + 2]);
      }
      const u64 o[4] = {((u64)a.y << 32) | a.x, ((u64)a.w << 32) | a.z,
                        ((u64)b.y << 32) | b.x, ((u64)b.w << 32) | b.z};
      const u64 oc[4] = {((u64)ca.y << 32) | ca.x, ((u64)ca.w << 32) | ca.z,
                         ((u64)cb.y << 32) | cb.x, ((u64)cb.w << 32) | cb.z};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const bool lt = o[q] < me[0];
        cnt += lt;
        if (kWeighted) acc += lt ? oc[q] : 0;
        eq += o[q] == me[0];
      }
    }
    // the key itself is in exactly one j-tile; any other first-word tie needs the rest
    const bool self_here = i >= j0 && i < j0 + jn;
    if (eq > (self_here ? 1u : 0u)) {
      for (u32 t = 0; t < jn; ++t) {
        if (s_w0[t] != me[0] || j0 + t == i) continue;
        u64 other[kKeyWords] = {s_w0[t], s_rest[t][0], s_rest[t][1], s_rest[t][2]};
        if (key_lt(other, me)) {
          ++cnt;
          if (kWeighted) acc += s_cnt[t];
        }
      }
    }
    if (cnt) {
      atomicAdd(&rank[i], cnt);
      if (kWeighted) atomicAdd(reinterpret_cast<unsigned long long*>(&val[i]), (unsigned long long)acc);
    }
  }
}

// Output records straight from the weighted ranks: out[rank[i]] = {key i, count i}.
// `out` may be host-mapped pinned memory (zero-copy: the records travel over PCIe as the
// kernel writes them, and the host needs no D2H copy).  `ctr_out` (optional, host-mapped)
// receives the final counters.
__global__ __launch_bounds__(256) void rank_emit_kernel(ConstKeysSoA keys,
                                                        const u64* __restrict__ counts,
                                                        const u32* __restrict__ rank,
                                                        const u64* __restrict__ val,
                                                        const MapCounters* __restrict__ ctr,
                                                        OutRecord* __restrict__ out,
                                                        MapCounters* __restrict__ ctr_out,
                                                        u32 ucap) {
  const u32 u = min(ctr->num_unique, ucap);
  if (blockIdx.x == 0 && threadIdx.x == 0 && ctr_out) {
    // field by field: total_count belongs to the thread that emits rank u-1
    ctr_out->num_records = ctr->num_records;
    ctr_out->map_tokens = ctr->map_tokens;
    ctr_out->num_unique = u;
    ctr_out->overflow_lines = ctr->overflow_lines;
    ctr_out->truncated = ctr->truncated;
    ctr_out->num_newlines = ctr->num_newlines;
    ctr_out->max_key_len = ctr->max_key_len;
    ctr_out->flags = ctr->flags | (u > (u32)kRankSortMax ? kCtrNotEmitted : 0u);
    if (u == 0) ctr_out->total_count = 0;
  }
  if (u > (u32)kRankSortMax) return;
  for (u32 i = blockIdx.x * 256 + threadIdx.x; i < u; i += gridDim.x * 256) {
    const u32 r = rank[i];
    OutRecord rec;
#pragma unroll
    for (int q = 0; q < kKeyWords; ++q) rec.w[q] = keys.w[q][i];
    rec.count = counts[i];
    out[r] = rec;
    if (r == u - 1 && ctr_out) ctr_out->total_count = val[i] + rec.count;
  }
}

__global__ __launch_bounds__(256) void rank_scatter_kernel(ConstKeysSoA keys,
                                                           const u64* __restrict__ counts,
                                                           const u32* __restrict__ rank,
                                                           const u32* __restrict__ d_u,
                                                           KeysSoA sorted,
                                                           u64* __restrict__ sorted_counts,
                                                           u32 ucap) {
  const u32 u = min(*d_u, ucap);
  if (u > (u32)kRankSortMax) return;
  for (u32 i = blockIdx.x * 256 + threadIdx.x; i < u; i += gridDim.x * 256) {
    const u32 r = rank[i];
#pragma unroll
    for (int q = 0; q < kKeyWords; ++q) sorted.w[q][r] = keys.w[q][i];
    sorted_counts[r] = counts[i];
  }
}

// Exclusive scan of the sorted counts (look-back) fused with the output records.
constexpr int kPackItems = 8;
constexpr int kPackTile = 256 * kPackItems;
__global__ __launch_bounds__(256) void scan_pack_kernel(ConstKeysSoA sorted,
                                                        const u64* __restrict__ counts,
                                                        MapCounters* __restrict__ ctr,
                                                        OutRecord* __restrict__ out,
                                                        u64* __restrict__ status,
                                                        u32* __restrict__ tile_ctr,
                                                        MapCounters* __restrict__ ctr_out,
                                                        u32 emit_limit) {
  __shared__ u64 s_scan[256 / 64 + 1];
  __shared__ u32 s_tile;
  __shared__ u64 s_prefix;
  const u32 u = ctr->num_unique;
  if (blockIdx.x == 0 && threadIdx.x == 0 && ctr_out) {
    // field by field: total_count belongs to the last tile
    ctr_out->num_records = ctr->num_records;
    ctr_out->map_tokens = ctr->map_tokens;
    ctr_out->num_unique = u;
    ctr_out->overflow_lines = ctr->overflow_lines;
    ctr_out->truncated = ctr->truncated;
    ctr_out->num_newlines = ctr->num_newlines;
    ctr_out->max_key_len = ctr->max_key_len;
    ctr_out->flags = ctr->flags | (u > emit_limit ? kCtrNotEmitted : 0u);
    if (u == 0) ctr_out->total_count = 0;
  }
  if (u > emit_limit) return;  // the producer (rank scatter) did not run: radix fallback
  const u32 num_tiles = (u32)div_up(u, kPackTile);
  const u32 tile = dev::acquire_tile(tile_ctr, &s_tile);
  if (tile >= num_tiles) return;
  const u32 first = tile * kPackTile + threadIdx.x * kPackItems;
  u64 c[kPackItems];
  u64 sum = 0;
#pragma unroll
  for (int t = 0; t < kPackItems; ++t) {
    c[t] = first + t < u ? counts[first + t] : 0;
    sum += c[t];
  }
  u64 total;
  const u64 excl = dev::block_exclusive_scan<u64, 256>(sum, s_scan, &total);
  (void)excl;
  const u64 base = dev::block_lookback(status, tile, total, &s_prefix);
#pragma unroll
  for (int t = 0; t < kPackItems; ++t) {
    const u32 i = first + t;
    if (i < u) {
      OutRecord r;
#pragma unroll
      for (int q = 0; q < kKeyWords; ++q) r.w[q] = sorted.w[q][i];
      r.count = c[t];
      out[i] = r;
    }
  }
  if (tile == num_tiles - 1 && threadIdx.x == 0) {
    ctr->total_count = base + total;
    if (ctr_out) ctr_out->total_count = base + total;
  }
}

u32 grid_for(u64 n, u32 block, u32 max_blocks = 2048) {
  u64 b = div_up(n ? n : 1, block);
  return (u32)(b > max_blocks ? max_blocks : b);
}

}  // namespace

void launch_dict_insert(ConstKeysSoA tokens, const u64* counts, const u32* d_n, u64 cap,
                        const DictWorkspace& dw, MapCounters* ctr, hipStream_t s) {
  dict_insert_kernel<<<dim3(grid_for(cap, kInsBlock, 1024)), dim3(kInsBlock), 0, s>>>(
      tokens, counts, d_n, dw, ctr, (u32)std::min<u64>(cap, 0xFFFFFFFFu));
  LOCUST_HIP_LAUNCH_CHECK();
}

void launch_dict_part_build(ConstKeysSoA tokens, const u64* counts, const u8* parts,
                            const u32* d_n, u64 cap, const DictWorkspace& dw, MapCounters* ctr,
                            hipStream_t s) {
  dict_part_build_kernel<<<dim3(kDictParts), dim3(kPartBlock), 0, s>>>(
      tokens, counts, parts, d_n, (u32)std::min<u64>(cap, 0xFFFFFFFFu), dw, ctr);
  LOCUST_HIP_LAUNCH_CHECK();
}

void launch_dict_ordered(ConstKeysSoA tokens, const u64* counts, const u8* parts,
                         const u32* d_n, u64 cap, MapCounters* ctr, OutRecord* out,
                         MapCounters* ctr_out, LookbackScratch lb, hipStream_t s, u64* trace,
                         const OrderedExtra& ex) {
  if (ex.part_off && !counts) {
    const TileSource src{tokens, ex.part_off, ex.part_tiles, (u32)std::min<u64>(cap, 0xFFFFFFFFu)};
    dict_ordered_kernel<TileSource><<<dim3(kDictParts), dim3(kPartBlock), 0, s>>>(
        src, ctr, out, ctr_out, lb.status, lb.tile_counter, trace, ex);
  } else {
    const TagSource src{tokens, counts, parts, d_n, (u32)std::min<u64>(cap, 0xFFFFFFFFu)};
    dict_ordered_kernel<TagSource><<<dim3(kDictParts), dim3(kPartBlock), 0, s>>>(
        src, ctr, out, ctr_out, lb.status, lb.tile_counter, trace, ex);
  }
  LOCUST_HIP_LAUNCH_CHECK();
}

void launch_dict_partials(ConstKeysSoA tokens, const u64* counts, const u32* part_off,
                          u32 tile_begin, u32 tile_end, u32 nslices, u32 slot_base, u32 nslots,
                          u64 cap, KeyCount* partials, u32* partial_n, hipStream_t s,
                          u64* trace) {
  LOCUST_CHECK_ARG(nslices >= 1 && slot_base + nslices <= nslots &&
                       nslots <= (u32)kMaxPartialSlots && tile_begin <= tile_end,
                   "partials: bad slot layout");
  dict_partials_kernel<<<dim3(kDictParts * nslices), dim3(kPartBlock), 0, s>>>(
      tokens, counts, part_off, tile_begin, tile_end, nslices, slot_base, nslots, (u32)std::min<u64>(cap, 0xFFFFFFFFu), partials, partial_n, trace);
  LOCUST_HIP_LAUNCH_CHECK();
}

void launch_dict_ordered_partials(const KeyCount* partials, const u32* partial_n, u32 nslots,
                                  MapCounters* ctr, OutRecord* out, MapCounters* ctr_out,
                                  LookbackScratch lb, hipStream_t s, u64* trace,
                                  const OrderedExtra& ex) {
  LOCUST_CHECK_ARG(nslots >= 1 && nslots <= (u32)kMaxPartialSlots, "partials: bad slot count");
  const PartialsSource src{partials, partial_n, nslots};
  dict_ordered_kernel<PartialsSource><<<dim3(kDictParts), dim3(kPartBlock), 0, s>>>(
      src, ctr, out, ctr_out, lb.status, lb.tile_counter, trace, ex);
  LOCUST_HIP_LAUNCH_CHECK();
}

void launch_dict_merge_runs(const KeyCount* own, const KeyCount* recv, const u32* meta,
                            MapCounters* ctr, OutRecord* out, MapCounters* ctr_out,
                            LookbackScratch lb, hipStream_t s, PartMap pm) {
  const RunsSource src{own, recv, meta, pm};
  OrderedExtra ex;
  ex.pm = pm;
  dict_ordered_kernel<RunsSource><<<dim3(kDictParts), dim3(kPartBlock), 0, s>>>(
      src, ctr, out, ctr_out, lb.status, lb.tile_counter, nullptr, ex);
  LOCUST_HIP_LAUNCH_CHECK();
}

void launch_rank_sort(ConstKeysSoA keys, const u64* counts, const u32* d_u, u64 cap, u32* rank,
                      u64* val, hipStream_t s) {
  // persistent grid: enough blocks to cover every CU a few times for the largest U
  const u64 umax = cap < (u64)kRankSortMax ? cap : (u64)kRankSortMax;
  const u64 pairs = div_up(umax, kRankI) * div_up(umax, kRankJ);
  const u32 grid = (u32)(pairs < 2048 ? (pairs ? pairs : 1) : 2048);
  const u32 ucap = (u32)std::min<u64>(cap, 0xFFFFFFFFu);
  if (val && counts)
    rank_sort_kernel<true><<<dim3(grid), dim3(kRankI), 0, s>>>(keys, counts, d_u, rank, val, ucap);
  else
    rank_sort_kernel<false><<<dim3(grid), dim3(kRankI), 0, s>>>(keys, nullptr, d_u, rank, nullptr,
                                                               ucap);
  LOCUST_HIP_LAUNCH_CHECK();
}

void launch_rank_emit(ConstKeysSoA keys, const u64* counts, const u32* rank, const u64* val,
                      u64 cap, const MapCounters* ctr, OutRecord* out, MapCounters* ctr_out,
                      hipStream_t s) {
  rank_emit_kernel<<<dim3(grid_for(cap, 256)), dim3(256), 0, s>>>(
      keys, counts, rank, val, ctr, out, ctr_out, (u32)std::min<u64>(cap, 0xFFFFFFFFu));
  LOCUST_HIP_LAUNCH_CHECK();
}

void launch_rank_scatter(ConstKeysSoA keys, const u64* counts, const u32* rank, const u32* d_u,
                         u64 cap, KeysSoA sorted, u64* sorted_counts, hipStream_t s) {
  rank_scatter_kernel<<<dim3(grid_for(cap, 256)), dim3(256), 0, s>>>(
      keys, counts, rank, d_u, sorted, sorted_counts, (u32)std::min<u64>(cap, 0xFFFFFFFFu));
  LOCUST_HIP_LAUNCH_CHECK();
}

void launch_scan_pack(ConstKeysSoA sorted, const u64* counts, u64 cap, MapCounters* ctr,
                      OutRecord* out, LookbackScratch lb, hipStream_t s, MapCounters* ctr_out,
                      u32 emit_limit) {
  const u32 tiles = (u32)div_up(cap ? cap : 1, kPackTile);
  scan_pack_kernel<<<dim3(tiles), dim3(256), 0, s>>>(sorted, counts, ctr, out, lb.status,
                                                     lb.tile_counter, ctr_out, emit_limit);
  LOCUST_HIP_LAUNCH_CHECK();
}

// Loads this file's code object (one module per file) now rather than at its first launch.
void warm_module_dict() {
  hipFuncAttributes a;
  (void)hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&dict_insert_kernel));
}

}  // namespace locust
