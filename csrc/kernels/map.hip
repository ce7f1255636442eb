// Map stage kernels: line index, reference-layout strtok_r map, slot compaction, and the
// byte-parallel wave64 tokenizer.
//
// Reference behaviour being reproduced (/root/reference/
// MapReduce/src/main.cu:136-159, 411): tokens are split on " ,.-;:'()\"\t", runs of
// delimiters are skipped, at most EMITS_PER_LINE (20) tokens are emitted per line, each
// token is emitted with value 1.  The reference launches a fixed <<<128,256>>> grid with
// no grid-stride loop; every kernel here covers its whole input.
#include "locust/device/lookback.hpp"
#include "locust/device/wave.hpp"
#include "locust/dstring.hpp"
#include "locust/hip_check.hpp"
#include "locust/kernels.hpp"

namespace locust {
namespace {

using dev::ballot;
using dev::lane_id;
using dev::lanes_below;
using dev::wave_id;

// ---------------------------------------------------------------------------------
// Line index: positions of '\n', stable, one pass with decoupled look-back.
// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(kLineIdxBlock) void line_index_kernel(
    const char* __restrict__ text, u64 bytes, u64* __restrict__ nl_pos,
    MapCounters* __restrict__ ctr, u64* __restrict__ status, u32* __restrict__ tile_ctr) {
  __shared__ u32 s_tile;
  __shared__ u64 s_prefix;
  __shared__ u32 s_scan[kLineIdxBlock / 64 + 1];
  const u64 num_tiles = div_up(bytes, (u64)kLineIdxTile);
  const u32 tile = dev::acquire_tile(tile_ctr, &s_tile);
  if (tile >= num_tiles) return;
  // Each thread owns kLineIdxItems consecutive bytes, loaded as one 16-B vector.
  const u64 base = (u64)tile * kLineIdxTile + (u64)threadIdx.x * kLineIdxItems;
  u32 nl_mask = 0;
  if (base + kLineIdxItems <= bytes) {
    const uint4 v = *reinterpret_cast<const uint4*>(text + base);
    const u32 words[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 16; ++k)
      if (((words[k >> 2] >> (8 * (k & 3))) & 0xffu) == '\n') nl_mask |= 1u << k;
  } else {
    for (int k = 0; k < kLineIdxItems; ++k)
      if (base + k < bytes && text[base + k] == '\n') nl_mask |= 1u << k;
  }
  u32 cnt = __popc(nl_mask);
  u32 total;
  u32 excl = dev::block_exclusive_scan<u32, kLineIdxBlock>(cnt, s_scan, &total);
  u64 prefix = dev::block_lookback(status, tile, total, &s_prefix);
  u64 out = prefix + excl;
  while (nl_mask) {
    int k = __ffs(nl_mask) - 1;
    nl_mask &= nl_mask - 1;
    nl_pos[out++] = base + k;
  }
  if (tile == num_tiles - 1 && threadIdx.x == 0) ctr->num_newlines = (u32)(prefix + total);
}

// ---------------------------------------------------------------------------------
// Reference-layout map (C19/C20): thread per line, device strtok_r, fixed slots.
// ---------------------------------------------------------------------------------
__device__ __forceinline__ void store_key(KeysSoA out, u64 idx, const u64* w) {
#pragma unroll
  for (int j = 0; j < kKeyWords; ++j) out.w[j][idx] = w[j];
}

__global__ __launch_bounds__(256) void map_compat_kernel(
    char* __restrict__ text, u64 bytes, const u64* __restrict__ nl_pos, u32 num_lines,
    const char* __restrict__ delims, int E, int max_key, KeysSoA slots,
    u32* __restrict__ line_counts, MapCounters* __restrict__ ctr) {
  for (u32 i = blockIdx.x * blockDim.x + threadIdx.x; i < num_lines;
       i += gridDim.x * blockDim.x) {
    const u64 start = i == 0 ? 0 : nl_pos[i - 1] + 1;
    const u64 end = (i < ctr->num_newlines) ? nl_pos[i] : bytes;
    text[end] = 0;  // the line's '\n' (or the pad byte) becomes its terminator
    char* save = nullptr;
    char* tok = d_strtok_r(text + start, delims, &save);
    int count = 0;
    u32 trunc = 0;
    while (tok != nullptr) {
      if (count >= E) {  // "WARN: Exceeded emit limit" (main.cu:141-143)
        atomicAdd(&ctr->overflow_lines, 1u);
        break;
      }
      int len = d_strlen(tok);
      u64 w[kKeyWords];
      if (len > max_key) ++trunc;
      pack_key(tok, len > max_key ? max_key : len, w);
      store_key(slots, (u64)i * E + count, w);
      atomicMax(&ctr->max_key_len, (u32)len);
      ++count;
      tok = d_strtok_r(nullptr, delims, &save);
    }
    line_counts[i] = (u32)count;
    if (trunc) atomicAdd(&ctr->truncated, trunc);
  }
}

// Stable compaction of fixed slots: scan of per-line counts with look-back, each thread
// copies its line's tokens (replaces thrust::partition over 116,000 slots, main.cu:411).
constexpr int kCompactBlock = 256;
__global__ __launch_bounds__(kCompactBlock) void compact_slots_kernel(
    const u32* __restrict__ line_counts, u32 num_lines, int E, ConstKeysSoA slots,
    KeysSoA out, MapCounters* __restrict__ ctr, u64* __restrict__ status,
    u32* __restrict__ tile_ctr) {
  __shared__ u32 s_tile;
  __shared__ u64 s_prefix;
  __shared__ u32 s_scan[kCompactBlock / 64 + 1];
  const u32 num_tiles = (u32)div_up(num_lines, kCompactBlock);
  const u32 tile = dev::acquire_tile(tile_ctr, &s_tile);
  if (tile >= num_tiles) return;
  const u32 line = tile * kCompactBlock + threadIdx.x;
  const u32 c = line < num_lines ? line_counts[line] : 0;
  u32 total;
  u32 excl = dev::block_exclusive_scan<u32, kCompactBlock>(c, s_scan, &total);
  u64 prefix = dev::block_lookback(status, tile, total, &s_prefix);
  const u64 dst = prefix + excl;
  for (u32 k = 0; k < c; ++k) {
    const u64 src = (u64)line * E + k;
#pragma unroll
    for (int j = 0; j < kKeyWords; ++j) out.w[j][dst + k] = slots.w[j][src];
  }
  if (tile == num_tiles - 1 && threadIdx.x == 0) ctr->num_records = (u32)(prefix + total);
}

}  // namespace

void launch_line_index(const char* text, u64 bytes, u64* nl_pos, MapCounters* ctr,
                       LookbackScratch lb, hipStream_t s) {
  if (bytes == 0) return;
  const u64 tiles = div_up(bytes, (u64)kLineIdxTile);
  line_index_kernel<<<dim3((u32)tiles), dim3(kLineIdxBlock), 0, s>>>(text, bytes, nl_pos, ctr,
                                                                     lb.status, lb.tile_counter);
  LOCUST_HIP_LAUNCH_CHECK();
}

void launch_map_compat(char* text, u64 bytes, const u64* nl_pos, u32 num_lines,
                       const char* d_delims, int emits_per_line, int max_key_len,
                       KeysSoA slots, u32* line_counts, MapCounters* ctr, hipStream_t s) {
  if (num_lines == 0) return;
  const u32 blocks = (u32)div_up(num_lines, 256);
  map_compat_kernel<<<dim3(blocks), dim3(256), 0, s>>>(text, bytes, nl_pos, num_lines, d_delims,
                                                        emits_per_line, max_key_len, slots,
                                                        line_counts, ctr);
  LOCUST_HIP_LAUNCH_CHECK();
}

void launch_compact_slots(const u32* line_counts, u32 num_lines, int emits_per_line,
                          ConstKeysSoA slots, KeysSoA out, MapCounters* ctr,
                          LookbackScratch lb, hipStream_t s) {
  if (num_lines == 0) return;
  const u32 tiles = (u32)div_up(num_lines, kCompactBlock);
  compact_slots_kernel<<<dim3(tiles), dim3(kCompactBlock), 0, s>>>(
      line_counts, num_lines, emits_per_line, slots, out, ctr, lb.status, lb.tile_counter);
  LOCUST_HIP_LAUNCH_CHECK();
}

// Loads this file's code object (one module per file) now rather than at its first launch.
void warm_module_map() {
  hipFuncAttributes a;
  (void)hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&line_index_kernel));
}

}  // namespace locust
