// Reduce stage kernels (/root/reference/MapReduce/src/
// main.cu:161-238, 453-465).
//
// Reference reduce = kernFindUniqBool (mark each sorted KV whose key differs from its left
// neighbour, writing (key, start index)) -> thrust::partition (compact the heads) ->
// kernGetCount (count = next head's start - this head's start; last uses the total).
// Here steps 1+2 are one kernel (mark + block scan + look-back + stable scatter), step 3
// is the adjacent-difference kernel.  Both exist in an LDS-staged variant (a tile plus a
// one-element halo staged in LDS, no barrier after an early return: reference bug B9) and
// a global-load variant, mirroring the reference's SHARE_MEMORY switch.  Grids cover the
// whole input (reference bug B3: fixed 32,768-thread grid).
//
// Generalisation used by the combiner and the multi-GPU shuffle: records may carry counts.
// Then the "index" of a record is the exclusive prefix sum of counts (scan kernel below),
// and the same head-mark + adjacent-difference computes per-key totals and start indices
// in token units -- with unit counts the prefix IS the index and nothing changes.
#include "locust/device/lookback.hpp"
#include "locust/device/wave.hpp"
#include "locust/hip_check.hpp"
#include "locust/kernels.hpp"

namespace locust {
namespace {

using dev::lane_id;
using dev::wave_id;

__device__ __forceinline__ bool keys_differ(ConstKeysSoA k, u32 a, u32 b) {
  bool diff = false;
#pragma unroll
  for (int j = 0; j < kKeyWords; ++j) diff |= k.w[j][a] != k.w[j][b];
  return diff;
}

// ---- exclusive scan of u64 counts ----
constexpr int kScanItems = 8;
constexpr int kScanTile = kReduceBlock * kScanItems;
__global__ __launch_bounds__(kReduceBlock) void scan_counts_kernel(
    const u64* __restrict__ counts, u64* __restrict__ prefix, MapCounters* __restrict__ ctr,
    u64* __restrict__ status, u32* __restrict__ tile_ctr) {
  __shared__ u64 s_scan[kReduceBlock / 64 + 1];
  __shared__ u32 s_tile;
  __shared__ u64 s_prefix;
  const u32 n = ctr->num_records;
  const u32 num_tiles = (u32)div_up(n, kScanTile);
  const u32 tile = dev::acquire_tile(tile_ctr, &s_tile);
  if (tile >= num_tiles) return;
  const u32 first = tile * kScanTile + threadIdx.x * kScanItems;
  u64 v[kScanItems];
  u64 sum = 0;
#pragma unroll
  for (int t = 0; t < kScanItems; ++t) {
    v[t] = (first + t < n) ? counts[first + t] : 0;
    sum += v[t];
  }
  u64 total;
  const u64 excl = dev::block_exclusive_scan<u64, kReduceBlock>(sum, s_scan, &total);
  const u64 base = dev::block_lookback(status, tile, total, &s_prefix);
  u64 run = base + excl;
#pragma unroll
  for (int t = 0; t < kScanItems; ++t) {
    if (first + t < n) prefix[first + t] = run;
    run += v[t];
  }
  if (tile == num_tiles - 1 && threadIdx.x == 0) ctr->total_count = base + total;
}

template <bool kLds>
__global__ __launch_bounds__(kReduceBlock) void mark_compact_heads_kernel(
    ConstKeysSoA sorted, const u64* __restrict__ prefix, KeysSoA head_keys,
    u64* __restrict__ head_val, MapCounters* __restrict__ ctr, u64* __restrict__ status,
    u32* __restrict__ tile_ctr) {
  // LDS image: word j of tile item t at s_keys[j][t + 1]; slot 0 is the left halo.
  __shared__ u64 s_keys[kLds ? kKeyWords : 1][kLds ? kReduceTile + 1 : 1];
  __shared__ u32 s_scan[kReduceBlock / 64 + 1];
  __shared__ u32 s_tile;
  __shared__ u64 s_prefix;
  const u32 n = ctr->num_records;
  const u32 num_tiles = (u32)div_up(n, kReduceTile);
  const u32 tile = dev::acquire_tile(tile_ctr, &s_tile);
  if (tile >= num_tiles) return;
  const u32 base = tile * kReduceTile;
  const u32 first = base + threadIdx.x * kReduceItems;  // blocked: items [first, first+8)
  u32 flags = 0;
  if constexpr (kLds) {
    // Coalesced striped load into LDS, then blocked reads.  All of a thread's global loads
    // are issued before any LDS store (a rolled loop would pay one load latency per trip).
    constexpr int kTrips = (kReduceTile + 1 + kReduceBlock - 1) / kReduceBlock;
    u64 v[kTrips][kKeyWords];
#pragma unroll
    for (int r = 0; r < kTrips; ++r) {
      const int i = threadIdx.x + r * kReduceBlock;
      const i64 g = (i64)base + i - 1;
      const bool ok = i < kReduceTile + 1 && g >= 0 && g < (i64)n;
#pragma unroll
      for (int j = 0; j < kKeyWords; ++j) v[r][j] = ok ? sorted.w[j][g] : ~0ull;
    }
#pragma unroll
    for (int r = 0; r < kTrips; ++r) {
      const int i = threadIdx.x + r * kReduceBlock;
      if (i < kReduceTile + 1) {
#pragma unroll
        for (int j = 0; j < kKeyWords; ++j) s_keys[j][i] = v[r][j];
      }
    }
    __syncthreads();
#pragma unroll
    for (int t = 0; t < kReduceItems; ++t) {
      const u32 i = first + t;
      if (i >= n) break;
      const u32 li = threadIdx.x * kReduceItems + t + 1;
      bool head = (i == 0);
      if (!head) {
#pragma unroll
        for (int j = 0; j < kKeyWords; ++j) head |= s_keys[j][li] != s_keys[j][li - 1];
      }
      if (head) flags |= 1u << t;
    }
  } else {
#pragma unroll
    for (int t = 0; t < kReduceItems; ++t) {
      const u32 i = first + t;
      if (i >= n) break;
      if (i == 0 || keys_differ(sorted, i, i - 1)) flags |= 1u << t;
    }
  }
  u32 total;
  const u32 excl =
      dev::block_exclusive_scan<u32, kReduceBlock>((u32)__popc(flags), s_scan, &total);
  const u64 pfx = dev::block_lookback(status, tile, total, &s_prefix);
  u64 out = pfx + excl;
  while (flags) {
    const int t = __ffs(flags) - 1;
    flags &= flags - 1;
    const u32 i = first + t;
#pragma unroll
    for (int j = 0; j < kKeyWords; ++j) head_keys.w[j][out] = sorted.w[j][i];
    head_val[out] = prefix ? prefix[i] : (u64)i;
    ++out;
  }
  if (tile == num_tiles - 1 && threadIdx.x == 0) {
    ctr->num_unique = (u32)(pfx + total);
    if (!prefix) ctr->total_count = n;
  }
}

// ---- fused LDS reduce: steps 1-3 and the output records in one kernel ----
// The tile (plus a one-key halo on each side) is staged in LDS as for the LDS head mark;
// heads are marked and compacted (block scan + look-back for the global head index); each
// head's count is the distance to the next head -- inside the tile from the LDS list of
// head positions, for the tile's last head by looking past the tile end (the halo key,
// then 64 keys per step by one wave for a run that continues: rare); and the records go
// straight to `out` (host-mapped: zero-copy) as consecutive 8-B words.  Replaces the
// separate mark/compact, adjacent-difference and pack launches -- and their two extra
// round trips through memory -- for unweighted reduces.
__global__ __launch_bounds__(kReduceBlock) void reduce_fused_kernel(
    ConstKeysSoA sorted, MapCounters* __restrict__ ctr, OutRecord* __restrict__ out,
    MapCounters* __restrict__ ctr_out, u64* __restrict__ status, u32* __restrict__ tile_ctr,
    u32 out_cap) {
  __shared__ u64 s_keys[kKeyWords][kReduceTile + 2];  // [0] left halo, [kReduceTile+1] right
  __shared__ u16 s_hpos[kReduceTile + 1];             // local positions of the tile's heads
  __shared__ u32 s_scan[kReduceBlock / 64 + 1];
  __shared__ u32 s_tile;
  __shared__ u64 s_prefix;
  __shared__ u32 s_end;  // end of the tile's last run (absolute)
  const u32 n = ctr->num_records;
  const u32 num_tiles = (u32)div_up(n, kReduceTile);
  if (n == 0) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      ctr->num_unique = 0;
      ctr->total_count = 0;
      if (ctr_out) *ctr_out = *ctr;
    }
    return;
  }
  // Tickets almost always come out in dispatch order: the keys of tile blockIdx.x are
  // loaded while the ticket atomic is in flight, and reloaded only on a mismatch.
  constexpr int kTrips = (kReduceTile + 2 + kReduceBlock - 1) / kReduceBlock;
  u64 v[kTrips][kKeyWords];
  auto load_tile = [&](u32 tl) {
#pragma unroll
    for (int r = 0; r < kTrips; ++r) {
      const int i = threadIdx.x + r * kReduceBlock;
      const i64 g = (i64)tl * kReduceTile + i - 1;
      const bool ok = i < kReduceTile + 2 && g >= 0 && g < (i64)n;
#pragma unroll
      for (int j = 0; j < kKeyWords; ++j) v[r][j] = ok ? sorted.w[j][g] : ~0ull;
    }
  };
  if (blockIdx.x < num_tiles) load_tile(blockIdx.x);
  const u32 tile = dev::acquire_tile(tile_ctr, &s_tile);
  if (tile >= num_tiles) return;
  if (tile != blockIdx.x) load_tile(tile);
  const u32 base = tile * kReduceTile;
  const u32 tn = min((u32)kReduceTile, n - base);  // items in this tile
  {
#pragma unroll
    for (int r = 0; r < kTrips; ++r) {
      const int i = threadIdx.x + r * kReduceBlock;
      if (i < kReduceTile + 2) {
#pragma unroll
        for (int j = 0; j < kKeyWords; ++j) s_keys[j][i] = v[r][j];
      }
    }
  }
  __syncthreads();
  u32 flags = 0;
  const u32 first = threadIdx.x * kReduceItems;  // local, blocked
#pragma unroll
  for (int t = 0; t < kReduceItems; ++t) {
    const u32 li = first + t;
    if (li >= tn) break;
    bool head = base + li == 0;
    if (!head) {
#pragma unroll
      for (int j = 0; j < kKeyWords; ++j) head |= s_keys[j][li + 1] != s_keys[j][li];
    }
    if (head) flags |= 1u << t;
  }
  u32 total;
  const u32 excl =
      dev::block_exclusive_scan<u32, kReduceBlock>((u32)__popc(flags), s_scan, &total);
  {
    u32 at = excl, f = flags;
    while (f) {
      const int t = __ffs(f) - 1;
      f &= f - 1;
      s_hpos[at++] = (u16)(first + t);
    }
  }
  if (threadIdx.x == 0) s_end = base + tn;
  __syncthreads();
  // End of the last head's run: the tile end unless the key continues past it.
  if (total && base + tn < n && dev::wave_id() == 0) {
    const u32 lh = s_hpos[total - 1];
    bool same = true;
#pragma unroll
    for (int j = 0; j < kKeyWords; ++j) same &= s_keys[j][tn + 1] == s_keys[j][lh + 1];
    if (same) {  // wave-uniform: the run continues into the next tile
      u32 pos = base + tn;
      for (;;) {
        const u32 g = pos + (u32)dev::lane_id();
        bool diff = g >= n;
        if (!diff) {
#pragma unroll
          for (int j = 0; j < kKeyWords; ++j) diff |= sorted.w[j][g] != s_keys[j][lh + 1];
        }
        const u64 b = dev::ballot(diff);
        if (b) {
          pos += (u32)(__ffsll((unsigned long long)b) - 1);
          break;
        }
        pos += 64;
      }
      if (dev::lane_id() == 0) s_end = min(pos, n);
    }
  }
  const u64 pfx = dev::block_lookback(status, tile, total, &s_prefix);  // syncs
  if (total) {
    u64* o = reinterpret_cast<u64*>(out + pfx);
    const u32 lim = pfx >= out_cap ? 0u : (u32)min<u64>(total, (u64)out_cap - pfx);
    for (u32 q = threadIdx.x; q < kOutWords * lim; q += kReduceBlock) {  // {key, count}
      const u32 h = q / kOutWords, f = q - kOutWords * h;
      const u32 li = s_hpos[h];
      u64 v;
      if (f < (u32)kKeyWords) {
        v = s_keys[f][li + 1];
      } else {
        const u32 end = h + 1 < total ? base + s_hpos[h + 1] : s_end;
        v = (u64)end - (base + li);
      }
      o[q] = v;
    }
  }
  if (tile == num_tiles - 1 && threadIdx.x == 0) {
    ctr->num_unique = (u32)(pfx + total);
    ctr->total_count = n;
    if (ctr_out) {
      MapCounters c = *ctr;
      c.num_unique = (u32)(pfx + total);
      c.total_count = n;
      *ctr_out = c;
    }
  }
}

template <bool kLds>
__global__ __launch_bounds__(kReduceBlock) void adjacent_diff_kernel(
    const u64* __restrict__ head_val, u64* __restrict__ head_count,
    const MapCounters* __restrict__ ctr) {
  __shared__ u64 s_val[kLds ? kReduceBlock + 1 : 1];
  const u32 u = ctr->num_unique;
  const u64 end = ctr->total_count;
  for (u32 base = blockIdx.x * kReduceBlock; base < u; base += gridDim.x * kReduceBlock) {
    const u32 j = base + threadIdx.x;
    if constexpr (kLds) {
      s_val[threadIdx.x] = j < u ? head_val[j] : end;
      if (threadIdx.x == 0) {
        const u32 r = base + kReduceBlock;
        s_val[kReduceBlock] = r < u ? head_val[r] : end;
      }
      __syncthreads();
      if (j < u) head_count[j] = s_val[threadIdx.x + 1] - s_val[threadIdx.x];
      __syncthreads();
    } else {
      if (j < u) head_count[j] = (j + 1 < u ? head_val[j + 1] : end) - head_val[j];
    }
  }
}

__global__ __launch_bounds__(256) void add_offset_kernel(u64* __restrict__ head_val,
                                                         const u64* __restrict__ d_offset,
                                                         const MapCounters* __restrict__ ctr) {
  const u32 u = ctr->num_unique;
  const u64 off = *d_offset;
  for (u32 j = blockIdx.x * 256 + threadIdx.x; j < u; j += gridDim.x * 256) head_val[j] += off;
}

// Output records, written as consecutive 8-B words by consecutive lanes (word q = record
// q / 5, field q % 5: key words, count; the heads' vals only served the adjacent
// difference): full cache lines, which matters when `out` is host-mapped memory
// (zero-copy results: every partial line would be its own PCIe write).  `ctr_out`
// (optional, host-mapped) receives the final counters; the host waits for the kernel.
__global__ __launch_bounds__(256) void pack_output_kernel(ConstKeysSoA head_keys,
                                                          const u64* __restrict__ head_val,
                                                          const u64* __restrict__ head_count,
                                                          const MapCounters* __restrict__ ctr,
                                                          OutRecord* __restrict__ out,
                                                          MapCounters* __restrict__ ctr_out) {
  const u32 u = ctr->num_unique;
  if (ctr_out && blockIdx.x == 0 && threadIdx.x == 0) *ctr_out = *ctr;
  u64* o = reinterpret_cast<u64*>(out);
  const u64 words = (u64)kOutWords * u;
  for (u64 q = blockIdx.x * 256ull + threadIdx.x; q < words; q += gridDim.x * 256ull) {
    const u32 j = (u32)(q / kOutWords), f = (u32)(q - (u64)kOutWords * j);
    o[q] = f < (u32)kKeyWords ? head_keys.w[f][j] : head_count[j];
  }
}

u32 grid_for(u64 n, u32 block, u32 max_blocks = 2048) {
  u64 b = div_up(n ? n : 1, block);
  return (u32)(b > max_blocks ? max_blocks : b);
}

}  // namespace

void launch_scan_counts(const u64* counts, u64 cap, u64* prefix, MapCounters* ctr,
                        LookbackScratch lb, hipStream_t s) {
  const u32 tiles = (u32)div_up(cap ? cap : 1, kScanTile);
  scan_counts_kernel<<<dim3(tiles), dim3(kReduceBlock), 0, s>>>(counts, prefix, ctr, lb.status,
                                                                 lb.tile_counter);
  LOCUST_HIP_LAUNCH_CHECK();
}

void launch_mark_compact_heads(ConstKeysSoA sorted, const u64* prefix, u64 cap, ReducePath path,
                               KeysSoA head_keys, u64* head_val, MapCounters* ctr,
                               LookbackScratch lb, hipStream_t s) {
  const u32 tiles = (u32)div_up(cap ? cap : 1, kReduceTile);
  if (path == ReducePath::kLds)
    mark_compact_heads_kernel<true><<<dim3(tiles), dim3(kReduceBlock), 0, s>>>(
        sorted, prefix, head_keys, head_val, ctr, lb.status, lb.tile_counter);
  else
    mark_compact_heads_kernel<false><<<dim3(tiles), dim3(kReduceBlock), 0, s>>>(
        sorted, prefix, head_keys, head_val, ctr, lb.status, lb.tile_counter);
  LOCUST_HIP_LAUNCH_CHECK();
}

void launch_reduce_fused(ConstKeysSoA sorted, u64 cap, MapCounters* ctr, OutRecord* out,
                         u64 out_cap, MapCounters* ctr_out, LookbackScratch lb, hipStream_t s) {
  const u32 tiles = (u32)div_up(cap ? cap : 1, kReduceTile);
  reduce_fused_kernel<<<dim3(tiles), dim3(kReduceBlock), 0, s>>>(
      sorted, ctr, out, ctr_out, lb.status, lb.tile_counter,
      (u32)(out_cap < 0xffffffffull ? out_cap : 0xffffffffull));
  LOCUST_HIP_LAUNCH_CHECK();
}

void launch_adjacent_diff(const u64* head_val, u64 cap, ReducePath path, u64* head_count,
                          const MapCounters* ctr, hipStream_t s) {
  const u32 grid = grid_for(cap, kReduceBlock);
  if (path == ReducePath::kLds)
    adjacent_diff_kernel<true><<<dim3(grid), dim3(kReduceBlock), 0, s>>>(head_val, head_count, ctr);
  else
    adjacent_diff_kernel<false><<<dim3(grid), dim3(kReduceBlock), 0, s>>>(head_val, head_count, ctr);
  LOCUST_HIP_LAUNCH_CHECK();
}

void launch_add_offset(u64* head_val, u64 cap, const u64* d_offset, const MapCounters* ctr,
                       hipStream_t s) {
  add_offset_kernel<<<dim3(grid_for(cap, 256)), dim3(256), 0, s>>>(head_val, d_offset, ctr);
  LOCUST_HIP_LAUNCH_CHECK();
}

void launch_pack_output(ConstKeysSoA head_keys, const u64* head_val, const u64* head_count,
                        u64 cap, const MapCounters* ctr, OutRecord* out, hipStream_t s,
                        MapCounters* ctr_out) {
  pack_output_kernel<<<dim3(grid_for(6 * cap, 256)), dim3(256), 0, s>>>(
      head_keys, head_val, head_count, ctr, out, ctr_out);
  LOCUST_HIP_LAUNCH_CHECK();
}

// Loads this file's code object (one module per file) now rather than at its first launch.
void warm_module_reduce() {
  hipFuncAttributes a;
  (void)hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&scan_counts_kernel));
}

}  // namespace locust
