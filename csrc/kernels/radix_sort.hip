// LSD radix sort of packed string keys (Process stage).
//
// The reference sorts 40-B KeyIntValuePair structs with thrust::sort and a byte-loop
// comparator (/root/reference/MapReduce/src/main.cu:414-415, KeyValue.h:20-33): a
// comparison merge sort that re-reads up to 30 key bytes per compare.  Here keys are
// packed big-endian into 4 x u64 words (locust/kv.hpp) and sorted least-significant word
// first; within a word, 8-bit digits least-significant first.  Digit positions whose
// byte is the same in every key (e.g. every byte past the longest word: Hamlet needs 14
// of 32 passes) are skipped.  Two regimes:
//
//  * n <= kSmallSortMax (8192): ONE 1024-thread workgroup sorts entirely in LDS -- the
//    current key word and both permutation buffers live in LDS, constant positions come
//    from a block-wide AND/OR reduction, and the final gather of keys/counts is fused.
//    One launch instead of ~20 (the regime of the README's 700/4,500-line configs).
//  * larger n: one histogram kernel counts all 32 digit positions (per-block partial
//    histograms, no global atomics), a 32-block plan kernel scans them, and each live
//    pass is ONE onesweep-style kernel: a 4096-key tile per 256-thread workgroup, wave64
//    match-any ranking through 8 ballots, per-digit decoupled look-back across tiles
//    (8 predecessors per load batch), stable scatter.  Only (u64 key word, u32 index)
//    pairs move per pass; the next word is gathered once through the permutation.
#include <algorithm>

#include "locust/device/lds_radix.hpp"
#include "locust/device/lookback.hpp"
#include "locust/device/wave.hpp"
#include "locust/hip_check.hpp"
#include "locust/kernels.hpp"

namespace locust {
namespace {

using dev::ballot;
using dev::lane_id;
using dev::lanes_below;
using dev::wave_id;

constexpr u32 kRxFlagAgg = 1u << 30;
constexpr u32 kRxFlagInc = 2u << 30;
constexpr u32 kRxValMask = (1u << 30) - 1;

LOCUST_HD inline u32 pos_shift(int pos) { return 56u - 8u * (u32)(pos & 7); }

// Ping-pong parity of the pass schedule, from the 32-bit mask of live digit positions
// (bit p = position p).  Passes of word w run bytes 7..0 and alternate buffers starting
// at buffer 0 (the word's prepare kernel writes it); buffer 2 = identity permutation.
LOCUST_HD inline u32 word_bits(u32 act, int w) { return (act >> (8 * w)) & 0xffu; }
LOCUST_HD inline u32 popc32(u32 x) {
  u32 c = 0;
  for (; x; x &= x - 1) ++c;
  return c;
}
LOCUST_HD inline u32 pass_src(u32 act, int pos) {
  const int w = pos / 8, b = pos % 8;
  return popc32(word_bits(act, w) >> (b + 1)) & 1u;  // live passes of this word before it
}
LOCUST_HD inline u32 word_src(u32 act, int w) {  // buffer holding the permutation at word start
  for (int v = w + 1; v < kKeyWords; ++v)
    if (word_bits(act, v))  // the nearest higher live word ran last: ended in popc & 1
      return popc32(word_bits(act, v)) & 1u;
  return 2u;
}
LOCUST_HD inline u32 final_src(u32 act) {
  for (int v = 0; v < kKeyWords; ++v)
    if (word_bits(act, v)) return popc32(word_bits(act, v)) & 1u;
  return 2u;
}

// Live-position mask read by one wave: lanes 0..31 load a flag each, one ballot.
__device__ __forceinline__ u32 live_mask(const SortPlan* plan) {
  const int lane = lane_id();
  const bool a = lane < kNumPositions && plan->pass[lane].active;
  return (u32)ballot(a);
}

// ---------------------------------------------------------------------------------
// Small-n path: whole sort in one workgroup.
// ---------------------------------------------------------------------------------
constexpr int kSmallBlock = 1024;
constexpr int kSmallWaves = kSmallBlock / 64;
using SmallRadix = dev::LdsRadix<kSmallBlock, kSmallSortMax, u16>;

__global__ __launch_bounds__(kSmallBlock) void radix_small_kernel(
    ConstKeysSoA keys, const u32* __restrict__ d_n, const u64* __restrict__ counts_in,
    KeysSoA sorted, u64* __restrict__ counts_out, u32* __restrict__ perm_out,
    SortPlan* __restrict__ plan) {
  __shared__ u64 s_word[kSmallSortMax];
  __shared__ u16 s_perm[2][kSmallSortMax];
  __shared__ u16 s_cnt[kSmallWaves][256];
  __shared__ u16 s_wex[kSmallWaves][256];
  __shared__ u32 s_start[256];
  __shared__ u64 s_and[kSmallWaves][kKeyWords], s_or[kSmallWaves][kKeyWords];
  __shared__ u32 s_wsum[4];
  const u32 n = *d_n;
  if (threadIdx.x == 0 && plan) plan->n = n;
  if (n > (u32)kSmallSortMax) return;  // the multi-tile path handles it
  const int lane = lane_id(), w = wave_id(), t = threadIdx.x;
  const SmallRadix rx{s_word, s_perm, s_cnt, s_wex, s_start, s_wsum};
  rx.init();

  // ---- constant digit positions: AND/OR of every key word ----
  u64 a[kKeyWords], o[kKeyWords];
#pragma unroll
  for (int j = 0; j < kKeyWords; ++j) {
    a[j] = ~0ull;
    o[j] = 0;
  }
  for (u32 i = t; i < n; i += kSmallBlock) {
#pragma unroll
    for (int j = 0; j < kKeyWords; ++j) {
      const u64 x = keys.w[j][i];
      a[j] &= x;
      o[j] |= x;
    }
  }
#pragma unroll
  for (int j = 0; j < kKeyWords; ++j) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      a[j] &= __shfl_xor(a[j], off, 64);
      o[j] |= __shfl_xor(o[j], off, 64);
    }
    if (lane == 0) {
      s_and[w][j] = a[j];
      s_or[w][j] = o[j];
    }
  }
  for (u32 i = t; i < n; i += kSmallBlock) s_perm[0][i] = (u16)i;
  __syncthreads();
  u64 diff[kKeyWords];
#pragma unroll
  for (int j = 0; j < kKeyWords; ++j) {
    u64 aa = ~0ull, oo = 0;
    for (int ww = 0; ww < kSmallWaves; ++ww) {
      aa &= s_and[ww][j];
      oo |= s_or[ww][j];
    }
    diff[j] = aa ^ oo;  // bits that differ between keys
  }

  int cur = 0;
  for (int wd = kKeyWords - 1; wd >= 0; --wd) {
    if (!diff[wd]) continue;
    for (u32 i = t; i < n; i += kSmallBlock) s_word[i] = keys.w[wd][i];
    __syncthreads();
    for (int b = 7; b >= 0; --b) {
      const u32 shift = 56u - 8u * (u32)b;
      if (!((diff[wd] >> shift) & 0xffull)) continue;  // constant position
      rx.pass(n, shift, cur);
      cur ^= 1;
    }
  }
  __syncthreads();
  // ---- fused gather: sorted keys (+ counts) and the permutation ----
  for (u32 i = t; i < n; i += kSmallBlock) {
    const u32 p = s_perm[cur][i];
#pragma unroll
    for (int j = 0; j < kKeyWords; ++j) sorted.w[j][i] = keys.w[j][p];
    if (counts_out) counts_out[i] = counts_in[p];
    if (perm_out) perm_out[i] = p;
  }
}

// ---------------------------------------------------------------------------------
// Large-n path.
// ---------------------------------------------------------------------------------
constexpr int kHistBlock = 256;

// Per-block partial histograms of all 32 digit positions, written with plain coalesced
// stores (no global atomics: a per-bin atomic flush from every block serialises on the
// hot bins).
__global__ __launch_bounds__(kHistBlock) void radix_hist_kernel(ConstKeysSoA keys,
                                                                const u32* __restrict__ d_n,
                                                                u32* __restrict__ part,
                                                                u32 skip_le) {
  __shared__ u32 s_hist[kNumPositions * 256];
  __shared__ u32 s_zero[kKeyWords];
  for (int i = threadIdx.x; i < kNumPositions * 256; i += kHistBlock) s_hist[i] = 0;
  if (threadIdx.x < kKeyWords) s_zero[threadIdx.x] = 0;
  __syncthreads();
  const u32 n = *d_n;
  if (n > skip_le) {
    for (u32 i = blockIdx.x * kHistBlock + threadIdx.x; i < n; i += gridDim.x * kHistBlock) {
      u64 x[kKeyWords];
#pragma unroll
      for (int w = 0; w < kKeyWords; ++w) x[w] = keys.w[w][i];
#pragma unroll
      for (int w = 0; w < kKeyWords; ++w) {
        const u64 zmask = ballot(x[w] == 0);
        if (x[w] == 0) {
          if (lanes_below(zmask) == 0) atomicAdd(&s_zero[w], (u32)__popcll(zmask));
          continue;
        }
#pragma unroll
        for (int b = 0; b < 8; ++b)
          atomicAdd(&s_hist[(8 * w + b) * 256 + ((x[w] >> (56 - 8 * b)) & 0xff)], 1u);
      }
    }
  }
  __syncthreads();
  u32* out = part + (u64)blockIdx.x * (kNumPositions * 256);
  for (int i = threadIdx.x; i < kNumPositions * 256; i += kHistBlock) {
    u32 c = s_hist[i];
    if ((i & 255) == 0) c += s_zero[(i / 256) / 8];
    out[i] = c;
  }
}

// One block per digit position: sum the partials, scan 256 bins, decide liveness.
__global__ __launch_bounds__(256) void radix_plan_kernel(const u32* __restrict__ part, u32 blocks,
                                                         const u32* __restrict__ d_n,
                                                         SortPlan* __restrict__ plan, u32 skip_le) {
  __shared__ u32 s_scan[256 / 64 + 1];
  const u32 n = *d_n;
  const int pos = blockIdx.x;
  if (pos == 0 && threadIdx.x == 0) plan->n = n;
  if (n <= skip_le) return;
  u32 c = 0;
  for (u32 b = 0; b < blocks; ++b) c += part[(u64)b * (kNumPositions * 256) + pos * 256 + threadIdx.x];
  u32 total;
  const u32 excl = dev::block_exclusive_scan<u32, 256>(c, s_scan, &total);
  plan->digit_offset[pos][threadIdx.x] = excl;
  const int one_bin = __syncthreads_or(c == n);
  if (threadIdx.x == 0) {
    plan->pass[pos].active = (n > 1 && !one_bin) ? 1u : 0u;
    plan->pass[pos].src = 0;
  }
}

// ---- per word: gather this word through the current permutation ----
__global__ __launch_bounds__(256) void radix_prepare_word_kernel(
    const u64* __restrict__ word, const SortPlan* __restrict__ plan, int w, u64* __restrict__ keys0,
    u32* __restrict__ vals0, const u32* __restrict__ vals1, u32 skip_le) {
  const u32 n = plan->n;
  if (n <= skip_le) return;
  const u32 act = live_mask(plan);
  if (!word_bits(act, w)) return;
  const u32 src = word_src(act, w);
  for (u32 i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const u32 perm = src == 2 ? i : (src == 0 ? vals0[i] : vals1[i]);
    keys0[i] = word[perm];
    vals0[i] = perm;
  }
}

// ---- one stable counting pass over an 8-bit digit ----
__global__ __launch_bounds__(kSortBlock) void radix_pass_kernel(
    const SortPlan* __restrict__ plan, int pos, u64* __restrict__ keys0, u32* __restrict__ vals0,
    u64* __restrict__ keys1, u32* __restrict__ vals1, u32* __restrict__ status,
    u32* __restrict__ tile_counter, u32 skip_le) {
  __shared__ u32 s_hist[kSortBlock / 64][256];
  __shared__ u32 s_base[256];
  __shared__ u32 s_tile;
  const u32 n = plan->n;
  const u32 act = live_mask(plan);
  if (n <= skip_le || !((act >> pos) & 1u)) return;
  const u32 num_tiles = (u32)div_up(n, kSortTile);
  for (int i = threadIdx.x; i < (kSortBlock / 64) * 256; i += kSortBlock) (&s_hist[0][0])[i] = 0;
  const u32 doff = plan->digit_offset[pos][threadIdx.x];  // prefetched off the critical path
  const u32 tile = dev::acquire_tile(tile_counter, &s_tile);
  if (tile >= num_tiles) return;
  const u32 src = pass_src(act, pos);
  const u64* kin = src ? keys1 : keys0;
  const u32* vin = src ? vals1 : vals0;
  u64* kout = src ? keys0 : keys1;
  u32* vout = src ? vals0 : vals1;
  const u32 shift = pos_shift(pos);
  const int lane = lane_id(), w = wave_id();
  const u32 base = tile * kSortTile + (u32)w * (kSortItems * 64);

  u64 k[kSortItems];
  u32 v[kSortItems];
  u32 rank[kSortItems];
#pragma unroll
  for (int j = 0; j < kSortItems; ++j) {
    const u32 idx = base + j * 64 + lane;
    const bool valid = idx < n;
    k[j] = valid ? kin[idx] : 0;
    v[j] = valid ? vin[idx] : 0;
  }
  // Wave-local stable ranking: round j precedes round j+1, lanes in order.
#pragma unroll
  for (int j = 0; j < kSortItems; ++j) {
    const u32 idx = base + j * 64 + lane;
    const bool valid = idx < n;
    const u32 d = (u32)(k[j] >> shift) & 0xffu;
    u64 m = ballot(valid);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const bool bit = (d >> b) & 1u;
      const u64 bb = ballot(bit);
      m &= bit ? bb : ~bb;
    }
    u32 prev = 0;
    if (valid) prev = s_hist[w][d];
    __builtin_amdgcn_wave_barrier();
    const u32 below = lanes_below(m);
    if (valid && below == 0) s_hist[w][d] = prev + (u32)__popcll(m);
    __builtin_amdgcn_wave_barrier();
    rank[j] = prev + below;
  }
  __syncthreads();
  // Per digit (thread = digit): wave-exclusive offsets, tile total, look-back.
  {
    const u32 d = threadIdx.x;
    u32 run = 0;
#pragma unroll
    for (int ww = 0; ww < kSortBlock / 64; ++ww) {
      const u32 c = s_hist[ww][d];
      s_hist[ww][d] = run;
      run += c;
    }
    u32* st = status + (u64)tile * 256 + d;
    u32 excl = 0;
    if (tile == 0) {
      dev::st_agent(st, kRxFlagInc | run);
    } else {
      dev::st_agent(st, kRxFlagAgg | run);
      // Batched look-back: 8 predecessors' words are loaded at once, so a chain of
      // aggregates costs one load latency per 8 tiles instead of one per tile.
      constexpr int kBatch = 8;
      i64 tt = (i64)tile - 1;
      for (;;) {
        u32 s[kBatch];
#pragma unroll
        for (int q = 0; q < kBatch; ++q)
          s[q] = (tt - q >= 0) ? dev::ld_agent(status + (u64)(tt - q) * 256 + d) : kRxFlagInc;
        int q = 0;
        bool done = false;
        for (; q < kBatch; ++q) {
          const u32 flag = s[q] >> 30;
          if (flag == 0) break;
          excl += s[q] & kRxValMask;
          if (flag == 2) {
            done = true;
            break;
          }
        }
        if (done) break;
        tt -= q;
        if (q < kBatch) __builtin_amdgcn_s_sleep(1);  // an unpublished predecessor: re-poll
      }
      dev::st_agent(st, kRxFlagInc | (excl + run));
    }
    s_base[d] = doff + excl;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kSortItems; ++j) {
    const u32 idx = base + j * 64 + lane;
    if (idx < n) {
      const u32 d = (u32)(k[j] >> shift) & 0xffu;
      const u32 dst = s_base[d] + s_hist[w][d] + rank[j];
      kout[dst] = k[j];
      vout[dst] = v[j];
    }
  }
}

__global__ __launch_bounds__(256) void gather_sorted_kernel(
    ConstKeysSoA keys, const SortPlan* __restrict__ plan, const u32* __restrict__ vals0,
    const u32* __restrict__ vals1, KeysSoA sorted, u32* __restrict__ perm_out,
    const u64* __restrict__ counts_in, u64* __restrict__ counts_out, u32 skip_le) {
  const u32 n = plan->n;
  if (n <= skip_le) return;  // the small kernel (or another sort) handled it
  const u32 src = final_src(live_mask(plan));
  for (u32 i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const u32 p = src == 2 ? i : (src == 0 ? vals0[i] : vals1[i]);
#pragma unroll
    for (int j = 0; j < kKeyWords; ++j) sorted.w[j][i] = keys.w[j][p];
    if (perm_out) perm_out[i] = p;
    if (counts_out) counts_out[i] = counts_in[p];
  }
}

u32 grid_for(u64 n, u32 block, u32 max_blocks = 2048) {
  u64 b = div_up(n ? n : 1, block);
  return (u32)(b > max_blocks ? max_blocks : b);
}

}  // namespace

u64 radix_status_words(u64 cap) { return div_up(cap ? cap : 1, kSortTile) * 256; }
u32 radix_hist_blocks(u64 cap) { return grid_for(cap, kHistBlock * 16, 512); }

u64 radix_zero_bytes(u64 cap) {
  return (u64)kNumPositions * 4 + (u64)kNumPositions * radix_status_words(cap) * 4;
}

void radix_sort(ConstKeysSoA keys, const u32* d_n, u64 host_n, RadixWorkspace& ws,
                const u64* counts_in, KeysSoA sorted, u64* counts_out, u32* perm_out,
                SortPlan* h_plan, hipStream_t s, u32 skip_upto) {
  const bool known = host_n != kUnknownCount;
  const u32 skip_le = known ? (u32)kSmallSortMax : std::max<u32>((u32)kSmallSortMax, skip_upto);
  if ((!known && skip_upto < (u32)kSmallSortMax) || (known && host_n <= (u64)kSmallSortMax)) {
    radix_small_kernel<<<dim3(1), dim3(kSmallBlock), 0, s>>>(keys, d_n, counts_in, sorted,
                                                              counts_out, perm_out, ws.plan);
    LOCUST_HIP_LAUNCH_CHECK();
    if (known) return;
  }
  const u64 cap = known ? host_n : ws.cap;
  LOCUST_CHECK_ARG(cap <= ws.cap, "radix sort: n exceeds workspace capacity");
  // tile counters and the status region of every pass are one contiguous block
  LOCUST_HIP_CHECK(hipMemsetAsync(ws.tile_counters, 0,
                                  (u64)kNumPositions * 4 +
                                      (u64)kNumPositions * radix_status_words(ws.cap) * 4,
                                  s));
  const u32 hb = radix_hist_blocks(cap);
  radix_hist_kernel<<<dim3(hb), dim3(kHistBlock), 0, s>>>(keys, d_n, ws.hist_part, skip_le);
  LOCUST_HIP_LAUNCH_CHECK();
  radix_plan_kernel<<<dim3(kNumPositions), dim3(256), 0, s>>>(ws.hist_part, hb, d_n, ws.plan,
                                                              skip_le);
  LOCUST_HIP_LAUNCH_CHECK();
  const SortPlan* hp = nullptr;
  u32 act = 0;
  if (known && h_plan) {
    LOCUST_HIP_CHECK(hipMemcpyAsync(h_plan, ws.plan, offsetof(SortPlan, digit_offset),
                                    hipMemcpyDeviceToHost, s));
    LOCUST_HIP_CHECK(hipStreamSynchronize(s));
    hp = h_plan;
    for (int p = 0; p < kNumPositions; ++p) act |= (hp->pass[p].active ? 1u : 0u) << p;
  }
  const u64 status_stride = radix_status_words(ws.cap);
  for (int w = kKeyWords - 1; w >= 0; --w) {
    if (hp && !word_bits(act, w)) continue;
    radix_prepare_word_kernel<<<dim3(grid_for(cap, 256)), dim3(256), 0, s>>>(
        keys.w[w], ws.plan, w, ws.keys[0], ws.vals[0], ws.vals[1], skip_le);
    LOCUST_HIP_LAUNCH_CHECK();
    for (int b = 7; b >= 0; --b) {
      const int pos = 8 * w + b;
      if (hp && !hp->pass[pos].active) continue;
      const u32 tiles = (u32)div_up(cap ? cap : 1, kSortTile);
      radix_pass_kernel<<<dim3(tiles), dim3(kSortBlock), 0, s>>>(
          ws.plan, pos, ws.keys[0], ws.vals[0], ws.keys[1], ws.vals[1],
          ws.status + (u64)pos * status_stride, ws.tile_counters + pos, skip_le);
      LOCUST_HIP_LAUNCH_CHECK();
    }
  }
  gather_sorted_kernel<<<dim3(grid_for(cap, 256)), dim3(256), 0, s>>>(
      keys, ws.plan, ws.vals[0], ws.vals[1], sorted, perm_out, counts_in, counts_out, skip_le);
  LOCUST_HIP_LAUNCH_CHECK();
}

// Loads this file's code object (one module per file) now rather than at its first launch.
void warm_module_radix_sort() {
  hipFuncAttributes a;
  (void)hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&radix_small_kernel));
}

}  // namespace locust
