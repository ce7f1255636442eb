// LSD radix sort of packed string keys (Process stage).
//
// The reference sorts 40-B KeyIntValuePair structs with thrust::sort and a byte-loop
// comparator (/root/reference/MapReduce/src/main.cu:414-415, KeyValue.h:20-33): a
// comparison merge sort that re-reads up to 30 key bytes per compare.  Here keys are
// packed big-endian into 4 x u64 words (locust/kv.hpp) and sorted least-significant word
// first; within a word, 8-bit digits least-significant first.  One histogram kernel
// counts all 32 digit positions at once; a plan kernel marks positions whose digits are
// all equal (e.g. every byte past the longest word: Hamlet needs 14 of 32 passes) so
// they are skipped.  Each live pass is ONE kernel: a 4096-key tile per 256-thread
// workgroup, wave64 match-any ranking through 8 ballots, per-digit decoupled look-back
// across tiles, stable scatter.  Only (u64 key word, u32 index) pairs move per pass; the
// next word is gathered once through the permutation.
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

__device__ __forceinline__ u32 pos_shift(int pos) { return 56u - 8u * (u32)(pos & 7); }

// ---- histogram of every digit position ----
constexpr int kHistBlock = 256;
__global__ __launch_bounds__(kHistBlock) void radix_hist_kernel(ConstKeysSoA keys,
                                                                const u32* __restrict__ d_n,
                                                                int max_pos,
                                                                u32* __restrict__ hist) {
  __shared__ u32 s_hist[kNumPositions * 256];
  __shared__ u32 s_zero[kKeyWords];
  for (int i = threadIdx.x; i < kNumPositions * 256; i += kHistBlock) s_hist[i] = 0;
  if (threadIdx.x < kKeyWords) s_zero[threadIdx.x] = 0;
  __syncthreads();
  const u32 n = *d_n;
  const int max_word = (max_pos + 7) / 8;
  for (u32 i = blockIdx.x * kHistBlock + threadIdx.x; i < n; i += gridDim.x * kHistBlock) {
    for (int w = 0; w < max_word; ++w) {
      const u64 x = keys.w[w][i];
      const u64 zmask = ballot(x == 0);
      if (x == 0) {
        if (lanes_below(zmask) == 0) atomicAdd(&s_zero[w], (u32)__popcll(zmask));
        continue;
      }
#pragma unroll
      for (int b = 0; b < 8; ++b) {
        const int pos = 8 * w + b;
        if (pos < max_pos) atomicAdd(&s_hist[pos * 256 + ((x >> (56 - 8 * b)) & 0xff)], 1u);
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kNumPositions * 256; i += kHistBlock) {
    u32 c = s_hist[i];
    const int pos = i / 256;
    if ((i & 255) == 0 && pos < 8 * max_word) c += s_zero[pos / 8];
    if (c) atomicAdd(&hist[i], c);
  }
}

// ---- plan: live positions, digit offsets, ping-pong parity ----
__global__ __launch_bounds__(256) void radix_plan_kernel(const u32* __restrict__ hist,
                                                         const u32* __restrict__ d_n,
                                                         int max_pos, SortPlan* __restrict__ plan) {
  __shared__ u32 s_scan[256 / 64 + 1];
  __shared__ u32 s_active[kNumPositions];
  const u32 n = *d_n;
  for (int pos = 0; pos < kNumPositions; ++pos) {
    const u32 c = (pos < max_pos) ? hist[pos * 256 + threadIdx.x] : 0;
    u32 total;
    const u32 excl = dev::block_exclusive_scan<u32, 256>(c, s_scan, &total);
    plan->digit_offset[pos][threadIdx.x] = excl;
    const int all_one_bin = __syncthreads_or(c == n);
    if (threadIdx.x == 0) s_active[pos] = (pos < max_pos && n > 1 && !all_one_bin) ? 1u : 0u;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    plan->n = n;
    u32 cur = 2;  // 2 = identity permutation, 0/1 = vals[0]/vals[1]
    u32 num_active = 0;
    for (int w = kKeyWords - 1; w >= 0; --w) {
      u32 any = 0;
      for (int b = 0; b < 8; ++b) any |= s_active[8 * w + b];
      plan->word_active[w] = any;
      plan->word_src[w] = cur;
      for (int b = 0; b < 8; ++b) {
        plan->pass[8 * w + b].active = s_active[8 * w + b];
        plan->pass[8 * w + b].src = 0;
      }
      if (!any) continue;
      u32 par = 0;  // the word's prepare writes buffer 0
      for (int b = 7; b >= 0; --b) {
        const int pos = 8 * w + b;
        if (!s_active[pos]) continue;
        plan->pass[pos].src = par;
        par ^= 1u;
        ++num_active;
      }
      cur = par;
    }
    plan->final_src = cur;
    plan->num_active = num_active;
  }
}

// ---- per word: gather this word through the current permutation ----
__global__ __launch_bounds__(256) void radix_prepare_word_kernel(
    const u64* __restrict__ word, const SortPlan* __restrict__ plan, int w, u64* __restrict__ keys0,
    u32* __restrict__ vals0, const u32* __restrict__ vals1) {
  if (!plan->word_active[w]) return;
  const u32 n = plan->n;
  const u32 src = plan->word_src[w];
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
    u32* __restrict__ tile_counter) {
  __shared__ u32 s_hist[kSortBlock / 64][256];
  __shared__ u32 s_base[256];
  __shared__ u32 s_tile;
  if (!plan->pass[pos].active) return;
  const u32 n = plan->n;
  const u32 num_tiles = (u32)div_up(n, kSortTile);
  for (int i = threadIdx.x; i < (kSortBlock / 64) * 256; i += kSortBlock) (&s_hist[0][0])[i] = 0;
  const u32 tile = dev::acquire_tile(tile_counter, &s_tile);
  if (tile >= num_tiles) return;
  const u32 src = plan->pass[pos].src;
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
      u32 t = tile - 1;
      for (;;) {
        const u32 s = dev::ld_agent(status + (u64)t * 256 + d);
        const u32 flag = s >> 30;
        if (flag == 0) {
          __builtin_amdgcn_s_sleep(1);
          continue;
        }
        excl += s & kRxValMask;
        if (flag == 2) break;
        --t;
      }
      dev::st_agent(st, kRxFlagInc | (excl + run));
    }
    s_base[d] = plan->digit_offset[pos][d] + excl;
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
    const u64* __restrict__ counts_in, u64* __restrict__ counts_out) {
  const u32 n = plan->n;
  const u32 src = plan->final_src;
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

void radix_sort_prepare(ConstKeysSoA keys, const u32* d_n, RadixWorkspace& ws, hipStream_t s) {
  // hist, tile counters and the status region of every pass are one contiguous block.
  const u64 zero_bytes = (u64)kNumPositions * 256 * 4 + (u64)kNumPositions * 4 +
                         (u64)kNumPositions * radix_status_words(ws.cap) * 4;
  LOCUST_HIP_CHECK(hipMemsetAsync(ws.hist, 0, zero_bytes, s));
  const int max_pos = kNumPositions;
  radix_hist_kernel<<<dim3(grid_for(ws.cap, kHistBlock, 1024)), dim3(kHistBlock), 0, s>>>(
      keys, d_n, max_pos, ws.hist);
  LOCUST_HIP_LAUNCH_CHECK();
  radix_plan_kernel<<<dim3(1), dim3(256), 0, s>>>(ws.hist, d_n, max_pos, ws.plan);
  LOCUST_HIP_LAUNCH_CHECK();
}

void radix_sort_run(ConstKeysSoA keys, const u32* d_n, RadixWorkspace& ws,
                    const SortPlan* host_plan, hipStream_t s) {
  (void)d_n;
  const u64 n = host_plan ? host_plan->n : ws.cap;
  const u64 status_stride = radix_status_words(ws.cap);
  for (int w = kKeyWords - 1; w >= 0; --w) {
    if (host_plan && !host_plan->word_active[w]) continue;
    radix_prepare_word_kernel<<<dim3(grid_for(n, 256)), dim3(256), 0, s>>>(
        keys.w[w], ws.plan, w, ws.keys[0], ws.vals[0], ws.vals[1]);
    LOCUST_HIP_LAUNCH_CHECK();
    for (int b = 7; b >= 0; --b) {
      const int pos = 8 * w + b;
      if (host_plan && !host_plan->pass[pos].active) continue;
      const u32 tiles = (u32)div_up(n ? n : 1, kSortTile);
      radix_pass_kernel<<<dim3(tiles), dim3(kSortBlock), 0, s>>>(
          ws.plan, pos, ws.keys[0], ws.vals[0], ws.keys[1], ws.vals[1],
          ws.status + (u64)pos * status_stride, ws.tile_counters + pos);
      LOCUST_HIP_LAUNCH_CHECK();
    }
  }
}

void launch_gather_sorted(ConstKeysSoA keys, const RadixWorkspace& ws, KeysSoA sorted,
                          u32* perm_out, const u64* counts_in, u64* counts_out, u64 cap,
                          hipStream_t s) {
  gather_sorted_kernel<<<dim3(grid_for(cap, 256)), dim3(256), 0, s>>>(
      keys, ws.plan, ws.vals[0], ws.vals[1], sorted, perm_out, counts_in, counts_out);
  LOCUST_HIP_LAUNCH_CHECK();
}

}  // namespace locust
