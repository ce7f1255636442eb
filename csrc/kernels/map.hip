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

// ---------------------------------------------------------------------------------
// Byte-parallel tokenizer.  One wave owns a 1 KiB segment (16 steps x 64 bytes, one
// byte per lane per step).  Token starts come from a 64-bit ballot of "not delimiter and
// previous byte is a delimiter"; the per-line ordinal needed for the 20-emit cap is the
// popcount of starts since the last newline, carried across steps.  The ordinal carried
// INTO a segment comes from a backward scan to the previous newline (stopped once it
// exceeds the cap).  Emit counts are scanned across waves and tiles (look-back), then
// each emitting lane packs its token straight into the dense output.
// ---------------------------------------------------------------------------------
struct DelimLds {
  u32 bits[8];  // 256-bit delimiter set incl. '\n' and NUL
};

__device__ __forceinline__ bool lds_is_delim(const DelimLds& d, u32 c) {
  return (d.bits[c >> 5] >> (c & 31)) & 1u;
}

__device__ __forceinline__ u32 load_byte(const char* text, u64 bytes, i64 pos) {
  // Bytes outside [0, bytes) behave like a newline (line boundary).
  return (pos >= 0 && (u64)pos < bytes) ? (u32)(unsigned char)text[pos] : (u32)'\n';
}

// Token starts since the last '\n' strictly before `pos`, saturated at cap+1.
__device__ u32 backward_line_ordinal(const char* text, u64 bytes, i64 pos, const DelimLds& d,
                                     u32 cap) {
  const int lane = lane_id();
  u32 count = 0;
  i64 hi = pos;  // scan [lo, hi)
  while (hi > 0) {
    const i64 lo = hi - 64;
    const i64 p = lo + lane;
    const u32 c = load_byte(text, bytes, p);   // p < 0 reads as '\n'
    const u32 cprev = load_byte(text, bytes, p - 1);
    const bool is_d = lds_is_delim(d, c);
    const bool start = !is_d && lds_is_delim(d, cprev);
    const u64 nl = ballot(c == '\n');
    u64 st = ballot(start);
    if (nl) {
      const int last_nl = 63 - __clzll((long long)nl);
      st &= (last_nl >= 63) ? 0ull : (~0ull << (last_nl + 1));
      count += __popcll(st);
      break;
    }
    count += __popcll(st);
    if (count > cap) break;
    hi = lo;
  }
  return count > cap + 1 ? cap + 1 : count;
}

__global__ __launch_bounds__(kMapBlock) void map_fast_kernel(
    const char* __restrict__ text, u64 bytes, DelimMask dm, int E, int max_key, KeysSoA out,
    u64 out_cap, MapCounters* __restrict__ ctr, u64* __restrict__ status,
    u32* __restrict__ tile_ctr) {
  __shared__ DelimLds s_delim;
  __shared__ u32 s_tile;
  __shared__ u64 s_prefix;
  __shared__ u32 s_wave_cnt[kMapBlock / 64];
  const int lane = lane_id(), w = wave_id();
  if (threadIdx.x < 8) {
    const u32 i = threadIdx.x;
    u32 b = (u32)(dm.m[i >> 1] >> (32 * (i & 1)));
    if (i == 0) b |= 1u;             // NUL
    if (i == 0) b |= 1u << '\n';     // newline
    s_delim.bits[i] = b;
  }
  const u64 num_tiles = div_up(bytes, (u64)kMapTileBytes);
  const u32 tile = dev::acquire_tile(tile_ctr, &s_tile);  // contains __syncthreads
  if (tile >= num_tiles) return;
  const DelimLds d = s_delim;
  const i64 seg = (i64)tile * kMapTileBytes + (i64)w * (kMapSegSteps * 64);

  // ---- phase 1: token starts, in-line ordinals, emit masks ----
  u32 line_ord = backward_line_ordinal(text, bytes, seg, d, (u32)E);
  bool prev_delim = lds_is_delim(d, load_byte(text, bytes, seg - 1));
  u64 emit_mask[kMapSegSteps];
  u32 emitted = 0, overflow = 0;
#pragma unroll
  for (int s = 0; s < kMapSegSteps; ++s) {
    const i64 p = seg + s * 64 + lane;
    const u32 c = ((u64)p < bytes) ? (u32)(unsigned char)text[p] : (u32)'\n';
    const bool is_d = lds_is_delim(d, c);
    bool pd = __shfl_up((int)is_d, 1, 64);
    if (lane == 0) pd = prev_delim;
    prev_delim = __shfl((int)is_d, 63, 64);
    const bool start = !is_d && pd && ((u64)p < bytes);
    const u64 st = ballot(start);
    const u64 nl = ballot(c == '\n' && (u64)p < bytes);
    // ordinal of this lane's token within its line
    const u64 below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    const u64 nl_below = nl & below;
    u32 ord;
    if (nl_below) {
      const int q = 63 - __clzll((long long)nl_below);
      ord = __popcll(st & below & (~0ull << (q + 1)));
    } else {
      ord = line_ord + __popcll(st & below);
    }
    const bool emit = start && ord < (u32)E;
    overflow += __popcll(ballot(start && ord == (u32)E));
    emit_mask[s] = ballot(emit);
    emitted += __popcll(emit_mask[s]);
    if (nl) {
      const int q = 63 - __clzll((long long)nl);
      line_ord = (q >= 63) ? 0 : __popcll(st & (~0ull << (q + 1)));
    } else {
      line_ord += __popcll(st);
    }
    if (line_ord > (u32)E + 1) line_ord = (u32)E + 1;
  }

  // ---- phase 2: wave counts -> tile prefix (look-back) ----
  if (lane == 0) s_wave_cnt[w] = emitted;
  __syncthreads();
  u32 wave_excl = 0, tile_total = 0;
#pragma unroll
  for (int i = 0; i < kMapBlock / 64; ++i) {
    const u32 v = s_wave_cnt[i];
    if (i < w) wave_excl += v;
    tile_total += v;
  }
  const u64 prefix = dev::block_lookback(status, tile, tile_total, &s_prefix);
  if (lane == 0 && overflow) atomicAdd(&ctr->overflow_lines, overflow);

  // ---- phase 3: pack and write emitted tokens ----
  u64 dst = prefix + wave_excl;
  u32 trunc = 0, maxlen = 0;
#pragma unroll
  for (int s = 0; s < kMapSegSteps; ++s) {
    const u64 m = emit_mask[s];
    if (m & (1ull << lane)) {
      const u64 idx = dst + lanes_below(m);
      const u64 p = (u64)(seg + s * 64 + lane);
      u64 kw[kKeyWords] = {0, 0, 0, 0};
      int len = 0;
      for (;;) {
        const u64 q = p + len;
        if (q >= bytes) break;
        const u32 c = (u32)(unsigned char)text[q];
        if (lds_is_delim(d, c)) break;
        if (len < max_key) kw[len >> 3] |= (u64)c << (56 - 8 * (len & 7));
        ++len;
      }
      if (len > max_key) ++trunc;
      maxlen = len > (int)maxlen ? (u32)len : maxlen;
      if (idx < out_cap) {
#pragma unroll
        for (int j = 0; j < kKeyWords; ++j) out.w[j][idx] = kw[j];
      }
    }
    dst += __popcll(m);
  }
  trunc = dev::wave_reduce_sum(trunc);
  maxlen = dev::wave_reduce_max(maxlen);
  if (lane == 0) {
    if (trunc) atomicAdd(&ctr->truncated, trunc);
    atomicMax(&ctr->max_key_len, maxlen);
  }
  if (tile == num_tiles - 1 && threadIdx.x == 0) ctr->num_records = (u32)(prefix + tile_total);
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

void launch_map_fast(const char* text, u64 bytes, const DelimMask& dm, int emits_per_line,
                     int max_key_len, KeysSoA out, u64 out_cap, MapCounters* ctr,
                     LookbackScratch lb, hipStream_t s) {
  if (bytes == 0) return;
  const u64 tiles = div_up(bytes, (u64)kMapTileBytes);
  map_fast_kernel<<<dim3((u32)tiles), dim3(kMapBlock), 0, s>>>(
      text, bytes, dm, emits_per_line, max_key_len, out, out_cap, ctr, lb.status,
      lb.tile_counter);
  LOCUST_HIP_LAUNCH_CHECK();
}

}  // namespace locust
