// Dictionary sort path (Process/Reduce stages, default): the reference's
// "stream compaction + key sort" and "boundary mark + adjacent difference" computed on the
// distinct keys only.
//
// The reference sorts every emitted token (/root/reference/MapReduce/src/main.cu:414) and
// then recovers per-key runs by boundary marking (main.cu:161-238).  The output it prints
// is a function of the distinct keys and their multiplicities only: val = the start of a
// key's run in the sorted token array = the exclusive prefix sum of the counts of all
// smaller keys; count = the run length.  So:
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
//   scan_pack     exclusive scan of the counts with decoupled look-back -> val, and the
//                 final (key, val, count) records for the D2H.
#include "locust/device/lookback.hpp"
#include "locust/device/wave.hpp"
#include "locust/hip_check.hpp"
#include "locust/kernels.hpp"

namespace locust {
namespace {

using dev::ballot;
using dev::lane_id;
using dev::wave_id;

// Words 1..3 are stored XOR kWordMagic: a packed key word can never equal kWordMagic
// (bytes 00 00 FF FF 00 00 FF FF: a NUL followed by non-NUL bytes), so a stored 0 means
// "not written yet" and a zero-initialised table needs no sentinel fill.
constexpr u64 kWordMagic = 0x0000FFFF0000FFFFull;

__device__ __forceinline__ u64 mix64(u64 x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}

__device__ __forceinline__ u64 key_hash(const u64* k) {
  return mix64(k[0] ^ mix64(k[1] ^ (k[2] * 0x9e3779b97f4a7c15ull) ^ (k[3] << 1)));
}

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
        const u32 id = atomicAdd(&ctr->num_unique, 1u);
#pragma unroll
        for (int j = 0; j < kKeyWords; ++j) dw.ukeys.w[j][id] = k[j];
        // ucount is zero-initialised and only ever updated by device-scope atomics (a
        // plain store could sit dirty in this XCD's L2 and later overwrite other adds)
        atomicAdd(reinterpret_cast<unsigned long long*>(&dw.ucount[id]), (unsigned long long)count);
#pragma unroll
        for (int j = 1; j < kKeyWords; ++j) dev::st_agent(&sl->w[j], k[j] ^ kWordMagic);
        dev::st_agent(&sl->id, id + 1);
        return true;
      }
    }
    if (w0 == k[0]) {
      const u32 sid = dev::ld_agent(&sl->id);
      const u64 x1 = dev::ld_agent(&sl->w[1]);
      const u64 x2 = dev::ld_agent(&sl->w[2]);
      const u64 x3 = dev::ld_agent(&sl->w[3]);
      if (sid == 0 || x1 == 0 || x2 == 0 || x3 == 0) continue;  // claimer still writing
      if ((x1 ^ kWordMagic) == k[1] && (x2 ^ kWordMagic) == k[2] && (x3 ^ kWordMagic) == k[3]) {
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

// LDS pre-aggregation table: 2,048 slots for a chunk of 1,024 tokens (load <= 0.5).
constexpr int kInsBlock = 256;
constexpr int kInsPerThread = 4;
constexpr int kInsChunk = kInsBlock * kInsPerThread;
constexpr int kLdsSlots = 2048;

struct LdsSlot {
  u64 w[kKeyWords];  // w[0] raw (0 = empty), w[1..3] XOR kWordMagic (0 = not written)
  u64 count;
};

__global__ __launch_bounds__(kInsBlock) void dict_insert_kernel(ConstKeysSoA tokens,
                                                                const u64* __restrict__ counts,
                                                                const u32* __restrict__ d_n,
                                                                DictWorkspace dw,
                                                                MapCounters* __restrict__ ctr) {
  __shared__ LdsSlot s_tab[kLdsSlots];
  const u32 n = *d_n;
  for (u32 c0 = blockIdx.x * kInsChunk; c0 < n; c0 += gridDim.x * kInsChunk) {
    for (int i = threadIdx.x; i < kLdsSlots; i += kInsBlock) {
#pragma unroll
      for (int j = 0; j < kKeyWords; ++j) s_tab[i].w[j] = 0;
      s_tab[i].count = 0;
    }
    // all loads of the chunk first (one latency), then the LDS inserts
    u64 k[kInsPerThread][kKeyWords];
    u64 c[kInsPerThread];
#pragma unroll
    for (int t = 0; t < kInsPerThread; ++t) {
      const u32 i = c0 + t * kInsBlock + threadIdx.x;
      const bool ok = i < n;
#pragma unroll
      for (int j = 0; j < kKeyWords; ++j) k[t][j] = ok ? tokens.w[j][i] : 0;
      c[t] = ok ? (counts ? counts[i] : 1ull) : 0;
    }
    __syncthreads();
#pragma unroll
    for (int t = 0; t < kInsPerThread; ++t) {
      if (!c[t] || k[t][0] == 0) continue;
      u32 slot = (u32)key_hash(k[t]) & (kLdsSlots - 1);
      for (;;) {
        LdsSlot& sl = s_tab[slot];
        u64 w0 = sl.w[0];
        if (w0 == 0) {
          w0 = atomicCAS(reinterpret_cast<unsigned long long*>(&sl.w[0]), 0ull,
                         (unsigned long long)k[t][0]);
          if (w0 == 0) {
#pragma unroll
            for (int j = 1; j < kKeyWords; ++j) sl.w[j] = k[t][j] ^ kWordMagic;
            atomicAdd(reinterpret_cast<unsigned long long*>(&sl.count), (unsigned long long)c[t]);
            break;
          }
        }
        if (w0 == k[t][0]) {
          const u64 x1 = __hip_atomic_load(&sl.w[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          const u64 x2 = __hip_atomic_load(&sl.w[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          const u64 x3 = __hip_atomic_load(&sl.w[3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          if (x1 == 0 || x2 == 0 || x3 == 0) continue;  // claimer still writing
          if ((x1 ^ kWordMagic) == k[t][1] && (x2 ^ kWordMagic) == k[t][2] &&
              (x3 ^ kWordMagic) == k[t][3]) {
            atomicAdd(reinterpret_cast<unsigned long long*>(&sl.count), (unsigned long long)c[t]);
            break;
          }
        }
        slot = (slot + 1) & (kLdsSlots - 1);
      }
    }
    __syncthreads();
    // flush the chunk's distinct keys to the HBM table
    for (int i = threadIdx.x; i < kLdsSlots; i += kInsBlock) {
      const LdsSlot& sl = s_tab[i];
      if (sl.w[0] == 0) continue;
      const u64 kk[kKeyWords] = {sl.w[0], sl.w[1] ^ kWordMagic, sl.w[2] ^ kWordMagic,
                                 sl.w[3] ^ kWordMagic};
      if (!global_insert(dw, kk, sl.count, ctr, key_hash(kk))) atomicOr(&ctr->flags, kCtrDictOverflow);
    }
    __syncthreads();
  }
}

// rank[i] += #{ j in tile : key[j] < key[i] }, persistent over (i-tile, j-tile) pairs.
constexpr int kRankI = 256;
constexpr int kRankJ = 1024;

__device__ __forceinline__ bool key_lt(const u64* a, const u64* b) {
#pragma unroll
  for (int j = 0; j < kKeyWords; ++j)
    if (a[j] != b[j]) return a[j] < b[j];
  return false;
}

__global__ __launch_bounds__(kRankI) void rank_sort_kernel(ConstKeysSoA keys,
                                                           const u32* __restrict__ d_u,
                                                           u32* __restrict__ rank) {
  __shared__ __attribute__((aligned(16))) u64 s_w0[kRankJ];
  __shared__ u64 s_rest[kRankJ][kKeyWords - 1];
  const u32 u = *d_u;
  if (u > (u32)kRankSortMax) return;  // radix path handles it
  const u32 ti = (u32)div_up(u, kRankI), tj = (u32)div_up(u, kRankJ);
  for (u32 pair = blockIdx.x; pair < ti * tj; pair += gridDim.x) {
    const u32 bi = pair % ti, bj = pair / ti;
    const u32 j0 = bj * kRankJ;
    const u32 jn = min((u32)kRankJ, u - j0);
    __syncthreads();  // previous pair's readers are done with the tile
    {
      constexpr int kTrips = kRankJ / kRankI;
      u64 v[kTrips][kKeyWords];  // issue every load before any LDS store
#pragma unroll
      for (int r = 0; r < kTrips; ++r) {
        const u32 t = threadIdx.x + r * kRankI;
#pragma unroll
        for (int q = 0; q < kKeyWords; ++q) v[r][q] = t < jn ? keys.w[q][j0 + t] : 0;
      }
#pragma unroll
      for (int r = 0; r < kTrips; ++r) {
        const u32 t = threadIdx.x + r * kRankI;
        // padding keys are all-ones: never smaller than a real key
        s_w0[t] = t < jn ? v[r][0] : ~0ull;
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
    // 16-byte broadcast reads, 8 keys per step, independent accumulations
    for (u32 t = 0; t < (u32)kRankJ; t += 8) {
      const uint4 a = *reinterpret_cast<const uint4*>(&s_w0[t]);
      const uint4 b = *reinterpret_cast<const uint4*>(&s_w0[t + 2]);
      const uint4 c = *reinterpret_cast<const uint4*>(&s_w0[t + 4]);
      const uint4 d = *reinterpret_cast<const uint4*>(&s_w0[t + 6]);
      const u64 o[8] = {((u64)a.y << 32) | a.x, ((u64)a.w << 32) | a.z,
                        ((u64)b.y << 32) | b.x, ((u64)b.w << 32) | b.z,
                        ((u64)c.y << 32) | c.x, ((u64)c.w << 32) | c.z,
                        ((u64)d.y << 32) | d.x, ((u64)d.w << 32) | d.z};
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        cnt += o[q] < me[0];
        eq += o[q] == me[0];
      }
    }
    // the key itself is in exactly one j-tile; any other first-word tie needs the rest
    const bool self_here = i >= j0 && i < j0 + jn;
    if (eq > (self_here ? 1u : 0u)) {
      for (u32 t = 0; t < jn; ++t) {
        if (s_w0[t] != me[0] || j0 + t == i) continue;
        u64 other[kKeyWords] = {s_w0[t], s_rest[t][0], s_rest[t][1], s_rest[t][2]};
        cnt += key_lt(other, me);
      }
    }
    if (cnt) atomicAdd(&rank[i], cnt);
  }
}

__global__ __launch_bounds__(256) void rank_scatter_kernel(ConstKeysSoA keys,
                                                           const u64* __restrict__ counts,
                                                           const u32* __restrict__ rank,
                                                           const u32* __restrict__ d_u,
                                                           KeysSoA sorted,
                                                           u64* __restrict__ sorted_counts) {
  const u32 u = *d_u;
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
                                                        u32* __restrict__ tile_ctr) {
  __shared__ u64 s_scan[256 / 64 + 1];
  __shared__ u32 s_tile;
  __shared__ u64 s_prefix;
  const u32 u = ctr->num_unique;
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
  const u64 base = dev::block_lookback(status, tile, total, &s_prefix);
  u64 run = base + excl;
#pragma unroll
  for (int t = 0; t < kPackItems; ++t) {
    const u32 i = first + t;
    if (i < u) {
      OutRecord r;
#pragma unroll
      for (int q = 0; q < kKeyWords; ++q) r.w[q] = sorted.w[q][i];
      r.val = run;
      r.count = c[t];
      out[i] = r;
    }
    run += c[t];
  }
  if (tile == num_tiles - 1 && threadIdx.x == 0) ctr->total_count = base + total;
}

u32 grid_for(u64 n, u32 block, u32 max_blocks = 2048) {
  u64 b = div_up(n ? n : 1, block);
  return (u32)(b > max_blocks ? max_blocks : b);
}

}  // namespace

void launch_dict_insert(ConstKeysSoA tokens, const u64* counts, const u32* d_n, u64 cap,
                        const DictWorkspace& dw, MapCounters* ctr, hipStream_t s) {
  dict_insert_kernel<<<dim3(grid_for(cap, kInsChunk, 4096)), dim3(kInsBlock), 0, s>>>(
      tokens, counts, d_n, dw, ctr);
  LOCUST_HIP_LAUNCH_CHECK();
}

void launch_rank_sort(ConstKeysSoA keys, const u32* d_u, u64 cap, u32* rank, hipStream_t s) {
  // persistent grid: enough blocks to cover every CU a few times for the largest U
  const u64 umax = cap < (u64)kRankSortMax ? cap : (u64)kRankSortMax;
  const u64 pairs = div_up(umax, kRankI) * div_up(umax, kRankJ);
  const u32 grid = (u32)(pairs < 2048 ? (pairs ? pairs : 1) : 2048);
  rank_sort_kernel<<<dim3(grid), dim3(kRankI), 0, s>>>(keys, d_u, rank);
  LOCUST_HIP_LAUNCH_CHECK();
}

void launch_rank_scatter(ConstKeysSoA keys, const u64* counts, const u32* rank, const u32* d_u,
                         u64 cap, KeysSoA sorted, u64* sorted_counts, hipStream_t s) {
  rank_scatter_kernel<<<dim3(grid_for(cap, 256)), dim3(256), 0, s>>>(keys, counts, rank, d_u,
                                                                    sorted, sorted_counts);
  LOCUST_HIP_LAUNCH_CHECK();
}

void launch_scan_pack(ConstKeysSoA sorted, const u64* counts, u64 cap, MapCounters* ctr,
                      OutRecord* out, LookbackScratch lb, hipStream_t s) {
  const u32 tiles = (u32)div_up(cap ? cap : 1, kPackTile);
  scan_pack_kernel<<<dim3(tiles), dim3(256), 0, s>>>(sorted, counts, ctr, out, lb.status,
                                                     lb.tile_counter);
  LOCUST_HIP_LAUNCH_CHECK();
}

}  // namespace locust
