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

__global__ __launch_bounds__(256) void pack_output_kernel(ConstKeysSoA head_keys,
                                                          const u64* __restrict__ head_val,
                                                          const u64* __restrict__ head_count,
                                                          const MapCounters* __restrict__ ctr,
                                                          OutRecord* __restrict__ out) {
  const u32 u = ctr->num_unique;
  for (u32 j = blockIdx.x * 256 + threadIdx.x; j < u; j += gridDim.x * 256) {
    OutRecord r;
#pragma unroll
    for (int w = 0; w < kKeyWords; ++w) r.w[w] = head_keys.w[w][j];
    r.val = head_val[j];
    r.count = head_count[j];
    out[j] = r;
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
                        u64 cap, const MapCounters* ctr, OutRecord* out, hipStream_t s) {
  pack_output_kernel<<<dim3(grid_for(cap, 256)), dim3(256), 0, s>>>(head_keys, head_val,
                                                                   head_count, ctr, out);
  LOCUST_HIP_LAUNCH_CHECK();
}

}  // namespace locust
