// Partitioned LDS radix sort: the Process stage of the reference algorithm (sort every
// emitted token) for passes whose map wrote a per-tile partition table.
//
// Reference: thrust::sort of 40-B KeyIntValuePair structs with a byte-loop comparator
// (/root/reference/MapReduce/src/main.cu:414-415, KeyValue.h:20-33).  The device-wide LSD
// sort (radix_sort.hip) needs one dependent kernel per live byte position -- 14 on whole
// Hamlet, each only 8 tiles wide at 33K tokens, ~9 us apiece.  This kernel uses what the
// small-input fast map already knows instead: it grouped every 1 KiB tile's tokens by
// PartMap partition (order-preserving 2-byte-prefix ranges, locust/partmap.hpp) and
// recorded where each partition's run starts (launch_map_fast part_off).  So the sort
// splits into 256 independent key ranges, and workgroup p (one per partition):
//   1. collects partition p's token indices from the table (two words per tile) and its
//      output offset, sum over tiles of part_off[t][p] - part_off[t][0] (the tokens of
//      lower partitions in tile t): no look-back, no workgroup waits on another;
//   2. gathers its keys' first two words into LDS (once: every pass and the output read
//      them there) and finds the byte positions that vary inside the partition (AND/OR
//      reduction: the shared prefix and the NUL padding drop out);
//   3. LSD-sorts the partition in LDS, one stable 8-bit counting pass per live position
//      (dev::LdsRadix: wave64 match-any ranks, u16 local indices, 3 barriers a pass);
//   4. writes its slice of the globally sorted token array.
// One launch, no host synchronisation, graph-capturable.  A partition with more than
// kPsortMax tokens sets kCtrSortOverflow and the host sorts the pass with radix_sort.
#include <cstdlib>

#include "locust/device/lds_radix.hpp"
#include "locust/device/lookback.hpp"
#include "locust/device/wave.hpp"
#include "locust/hip_check.hpp"
#include "locust/kernels.hpp"

namespace locust {
namespace {

using dev::lane_id;
using dev::wave_id;

constexpr int kPsBlock = 512;  // 8 waves: 256 VGPRs a lane (1,024 threads spilled the pass state)
constexpr int kPsWaves = kPsBlock / 64;
constexpr int kPsRounds = kPsortMax / kPsBlock;  // keys held per thread
using PsRadix = dev::LdsRadix<kPsBlock, kPsortMax, u16>;

// The end of every fused workgroup: its look-back (unless done already), the run's
// counters from the last partition, and the completion count -- the last workgroup to
// finish writes the counter snapshot, re-zeroes the scratch (unless a partition
// overflowed) and tells the host.
__device__ __forceinline__ void reduce_tail(u32 p, u32 U, u64 pfx, MapCounters* ctr,
                                            const PsortReduceArgs& ra, u64& s_prefix,
                                            u32& s_last, bool looked_back = false) {
  if (!looked_back) pfx = dev::block_lookback(ra.status, p, U, &s_prefix);
  if (p == (u32)kDictParts - 1 && threadIdx.x == 0) {
    ctr->num_unique = (u32)(pfx + U);
    ctr->total_count = ctr->num_records;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    // this workgroup's records (host-mapped) and counter writes; release only (the last
    // workgroup acquires)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    s_last = atomicAdd(ra.done_counter, 1u) == (u32)kDictParts - 1 ? 1u : 0u;
  }
  __syncthreads();
  if (!s_last) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // every other workgroup's (acquire only)
  const u32 flags = __hip_atomic_load(&ctr->flags, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (threadIdx.x == 0 && ra.ctr_out) {
    MapCounters c = *ctr;
    *ra.ctr_out = c;
  }
  // the host first (records, counters out), then the device scratch re-zeroing, which the
  // next job's kernels behind this one on the stream see complete (as dict.hip)
  if (ra.host_done && threadIdx.x == 0)  // a system-scope release store
    __hip_atomic_store(ra.host_done, ra.host_done_value, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  __syncthreads();
  if (!(flags & kCtrSortOverflow)) {
    for (u32 i = threadIdx.x; i < ra.map_words; i += kPsBlock) ra.map_lb.status[i] = 0;
    for (u32 i = threadIdx.x; i < (u32)kDictParts; i += kPsBlock) ra.status[i] = 0;
    if (threadIdx.x == 0) {
      // the accumulated counters; num_unique / total_count are this run's assignments
      ctr->num_records = 0;
      ctr->overflow_lines = 0;
      ctr->truncated = 0;
      ctr->num_newlines = 0;
      ctr->max_key_len = 0;
      ctr->flags = 0;
      *ra.map_lb.tile_counter = 0;
      *ra.done_counter = 0;
    }
  }
}

// kReduce: the fused Process + Reduce (launch_psort_reduce) -- step 4 marks heads and
// writes the output records instead of the sorted slice, and every workgroup (empty and
// overflowing partitions included) takes part in the look-back and the completion count.
template <bool kReduce>
__global__ __launch_bounds__(kPsBlock) void psort_kernel(ConstKeysSoA tokens,
                                                         const u32* __restrict__ part_off,
                                                         u32 ntiles, u32 n_cap, KeysSoA sorted,
                                                         MapCounters* __restrict__ ctr,
                                                         u32* __restrict__ part_w,
                                                         u64* __restrict__ trace,
                                                         PsortReduceArgs ra) {
  // trace (diagnostics, LOCUST_ORD_TRACE): per partition, s_memtime at [p*16 + k]: 0 start,
  // 1 list built, 2 keys loaded, 3 sorted, 4 written; [5] tokens, [6] passes; [10]/[11]
  // entry/exit on the 100 MHz device-wide clock
#define PS_STAMP(k_) \
  if (trace && threadIdx.x == 0) trace[(u64)blockIdx.x * 16 + (k_)] = __builtin_amdgcn_s_memtime()
  if (trace && threadIdx.x == 0) {
    for (int k = 1; k < 16; ++k) trace[(u64)blockIdx.x * 16 + k] = 0;
    trace[(u64)blockIdx.x * 16 + 10] = __builtin_amdgcn_s_memrealtime();
  }
  PS_STAMP(0);
  __shared__ u32 s_list[kPsortMax];   // global token index of local item i
  __shared__ u64 s_w0[kPsortMax];     // key words 0 and 1 of local item i (LDS-resident:
  __shared__ u64 s_w1[kPsortMax];     // gathered once, read by every pass and the output)
  __shared__ u16 s_perm[2][kPsortMax];
  __shared__ u16 s_cnt[kPsWaves][256];
  __shared__ u16 s_wex[kPsWaves][256];
  __shared__ u32 s_start[256];
  __shared__ u32 s_wsum[4];
  __shared__ u64 s_and[kPsWaves][kKeyWords], s_or[kPsWaves][kKeyWords];
  __shared__ u32 s_count, s_below, s_heads;
  __shared__ u16 s_hpos[kReduce ? kPsortMax + 1 : 1];  // local positions of the heads
  __shared__ u32 s_scan[kPsWaves + 1];
  __shared__ u64 s_prefix;
  __shared__ u32 s_last;
  const u32 p = blockIdx.x;
  const int lane = lane_id(), w = wave_id(), t = (int)threadIdx.x;
  const PsRadix rx{s_w0, s_perm, s_cnt, s_wex, s_start, s_wsum};
  rx.init();
  if (t == 0) {
    s_count = 0;
    s_below = 0;
    s_heads = 0;
  }
  __syncthreads();

  // ---- 1. this partition's tokens and its output offset; the first kEarly keys of each
  // tile's run are loaded right behind the table row (their round trip overlaps the scan
  // and the append), the rest -- flagged kLate in s_list -- in step 2 ----
  constexpr u32 kEarly = 4;
  constexpr u32 kLate = 0x80000000u;
  u32 below = 0;
  for (u32 t0 = 0; t0 < ntiles; t0 += kPsBlock) {
    const u32 tile = t0 + (u32)t;
    u32 a = 0, len = 0;
    if (tile < ntiles) {
      const u32* row = part_off + (u64)tile * kPartTable;
      const u32 z = row[0];
      a = row[p];
      len = row[p + 1] - a;
      below += a - z;
    }
    u64 e0[kEarly], e1[kEarly];
#pragma unroll
    for (u32 j = 0; j < kEarly; ++j) {
      const bool ok = j < len && a + j < n_cap;
      e0[j] = ok ? tokens.w[0][a + j] : 0;
      e1[j] = ok ? tokens.w[1][a + j] : 0;
    }
    // one LDS atomic per wave: the wave's runs are appended back to back (any order will
    // do -- equal keys are indistinguishable in the output)
    const u32 incl = dev::wave_inclusive_scan(len);
    u32 wbase = 0;
    if (lane == 63 && incl) wbase = atomicAdd(&s_count, incl);
    wbase = (u32)__builtin_amdgcn_readlane((int)wbase, 63);
    u32 at = wbase + incl - len;
#pragma unroll
    for (u32 j = 0; j < kEarly; ++j)
      if (j < len && at + j < (u32)kPsortMax) {
        s_list[at + j] = a + j;
        s_w0[at + j] = e0[j];
        s_w1[at + j] = e1[j];
      }
    for (u32 j = kEarly; j < len; ++j)
      if (at + j < (u32)kPsortMax) s_list[at + j] = (a + j) | kLate;
  }
  below = dev::wave_reduce_sum(below);
  if (lane == 0 && below) atomicAdd(&s_below, below);
  __syncthreads();
  const u32 m = s_count, base = s_below;
  PS_STAMP(1);
  if (trace && t == 0) trace[(u64)p * 16 + 5] = m;
  if (m > (u32)kPsortMax) {  // uniform: the host sorts this pass with radix_sort
    if (t == 0) atomicOr(&ctr->flags, kCtrSortOverflow);
    if constexpr (kReduce) {
      reduce_tail(p, 0, 0, ctr, ra, s_prefix, s_last);
      return;
    }
    return;
  }
  if (m == 0) {
    if (part_w && t == 0) part_w[p] = 0;
    if constexpr (kReduce) reduce_tail(p, 0, 0, ctr, ra, s_prefix, s_last);
    return;
  }

  // ---- 2. keys: words 0-1 into LDS (all first-word loads in flight at once, second words
  // only for keys that run past 8 bytes); AND/OR over the partition: which byte positions
  // vary (words 2-3 only for keys past 16 bytes, re-gathered if a pass needs them) ----
  u64 a[kKeyWords], o[kKeyWords];
#pragma unroll
  for (int j = 0; j < kKeyWords; ++j) {
    a[j] = ~0ull;
    o[j] = 0;
  }
  {
    u32 gi[kPsRounds];
    bool late[kPsRounds];
    u64 x0[kPsRounds], x1[kPsRounds];
#pragma unroll
    for (int r = 0; r < kPsRounds; ++r) {
      const u32 i = (u32)t + (u32)r * kPsBlock;
      const u32 v = i < m ? s_list[i] : 0xFFFFFFFFu;
      late[r] = i < m && (v & kLate);
      gi[r] = i < m ? (v & ~kLate) : 0xFFFFFFFFu;
      if (late[r]) s_list[i] = gi[r];  // plain indices from here on
    }
    // words 0 and 1: loaded in step 1 (in LDS), or now for the runs' later keys, all in
    // one round trip (word 1 is read even for short keys, where it is 0: a second
    // dependent round of gathers costs more than the extra bytes)
#pragma unroll
    for (int r = 0; r < kPsRounds; ++r) {
      const u32 i = (u32)t + (u32)r * kPsBlock;
      const bool ok = gi[r] < n_cap;
      x0[r] = !ok ? 0 : late[r] ? tokens.w[0][gi[r]] : s_w0[i];
      x1[r] = !ok ? 0 : late[r] ? tokens.w[1][gi[r]] : s_w1[i];
    }
#pragma unroll
    for (int r = 0; r < kPsRounds; ++r) {
      if (gi[r] >= n_cap) continue;
      const u32 i = (u32)t + (u32)r * kPsBlock;
      s_w0[i] = x0[r];
      s_w1[i] = x1[r];
      u64 x2 = 0, x3 = 0;
      if (x1[r] & 0xffull) {
        x2 = tokens.w[2][gi[r]];
        if (x2 & 0xffull) x3 = tokens.w[3][gi[r]];
      }
      a[0] &= x0[r];
      o[0] |= x0[r];
      a[1] &= x1[r];
      o[1] |= x1[r];
      a[2] &= x2;
      o[2] |= x2;
      a[3] &= x3;
      o[3] |= x3;
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
  for (u32 i = (u32)t; i < m; i += kPsBlock) s_perm[0][i] = (u16)i;
  __syncthreads();
  u64 diff[kKeyWords];
  bool long_keys = false;  // some key of the partition runs past 16 bytes
#pragma unroll
  for (int j = 0; j < kKeyWords; ++j) {
    u64 aa = ~0ull, oo = 0;
#pragma unroll
    for (int ww = 0; ww < kPsWaves; ++ww) {
      aa &= s_and[ww][j];
      oo |= s_or[ww][j];
    }
    diff[j] = aa ^ oo;
    if (j >= 2) long_keys |= oo != 0;
  }

  PS_STAMP(2);
  int cur = 0;
  bool any_diff = false;
#pragma unroll
  for (int j = 0; j < kKeyWords; ++j) any_diff |= diff[j] != 0;
  // ---- 3a. small partitions of short keys: one all-pairs ranking pass.  A partition of
  // the tuned map holds a few hundred tokens whose keys still differ in 6-10 byte positions
  // (words of one initial letter): as many LSD passes, each with three barriers and a
  // 256-bin scan whatever m is (~3 us apiece; 9 passes put p=255 at 29K ticks on whole
  // Hamlet).  Ranking every key against the partition's (LDS broadcast reads, no
  // barriers) costs m compares a thread: ~1K cycles at m = 512. ----
  // live byte positions = LSD passes; measured on whole Hamlet: ~3,000 ticks a pass vs
  // ~135 ticks a key for the ranking -- rank only where that is cheaper
  u32 lsd_passes = 0;
#pragma unroll
  for (int j = 0; j < kKeyWords; ++j)
#pragma unroll
    for (int b = 0; b < 8; ++b) lsd_passes += ((diff[j] >> (8 * b)) & 0xffull) ? 1u : 0u;
  if (any_diff && !long_keys && m <= 2u * kPsBlock && m < 22u * lsd_passes) {
    // eight independent compares per step: the broadcast LDS reads of a step are all in
    // flight together (one at a time, each compare waited out the LDS latency)
    constexpr u32 kU = 8;
    const u32 m8 = m & ~(kU - 1);
    for (u32 i = (u32)t; i < m; i += kPsBlock) {
      const u64 a0 = s_w0[i], a1 = s_w1[i];
      u32 r[kU] = {};
      for (u32 j = 0; j < m8; j += kU) {
        u64 b0[kU], b1[kU];
#pragma unroll
        for (u32 u = 0; u < kU; ++u) {
          b0[u] = s_w0[j + u];
          b1[u] = s_w1[j + u];
        }
        // bitwise, not short-circuit: no branches (and no exec-mask juggling) in the loop
#pragma unroll
        for (u32 u = 0; u < kU; ++u)
          r[u] += (u32)((b0[u] < a0) |
                        ((b0[u] == a0) & ((b1[u] < a1) | ((b1[u] == a1) & (j + u < i)))));
      }
      u32 rank = 0;
#pragma unroll
      for (u32 u = 0; u < kU; ++u) rank += r[u];
      for (u32 j = m8; j < m; ++j) {
        const u64 b0 = s_w0[j], b1 = s_w1[j];
        rank += (u32)((b0 < a0) | ((b0 == a0) & ((b1 < a1) | ((b1 == a1) & (j < i)))));
      }
      s_perm[0][rank] = (u16)i;
    }
    __syncthreads();
    any_diff = false;  // sorted
  }
  // ---- 3. LSD passes over the live byte positions, least significant first ----
  for (int wd = kKeyWords - 1; any_diff && wd >= 0; --wd) {
    if (!diff[wd]) continue;
    const u64* warr = wd == 0 ? s_w0 : s_w1;
    if (wd >= 2) {
      // rare (keys past 16 bytes): word wd into the word-1 array for its passes, word 1
      // itself restored afterwards
      for (u32 i = (u32)t; i < m; i += kPsBlock) {
        const u32 g = s_list[i];
        u64 x = (g < n_cap && (s_w1[i] & 0xffull)) ? tokens.w[2][g] : 0;
        if (wd == 3) x = (x & 0xffull) ? tokens.w[3][g] : 0;
        s_w1[i] = x;
      }
      __syncthreads();
    }
    for (int b = 7; b >= 0; --b) {
      const u32 shift = 56u - 8u * (u32)b;
      if (!((diff[wd] >> shift) & 0xffull)) continue;
      rx.pass(warr, m, shift, cur);
      cur ^= 1;
    }
    if (wd >= 2) {
      for (u32 i = (u32)t; i < m; i += kPsBlock) {
        const u32 g = s_list[i];
        s_w1[i] = (g < n_cap && (s_w0[i] & 0xffull)) ? tokens.w[1][g] : 0;
      }
      __syncthreads();
    }
  }

  PS_STAMP(3);
  if (trace && t == 0) {
    u32 np = 0;
    for (int j = 0; j < kKeyWords; ++j)
      for (int b = 0; b < 8; ++b) np += ((diff[j] >> (8 * b)) & 0xffull) ? 1u : 0u;
    trace[(u64)p * 16 + 6] = np;
  }
  if constexpr (kReduce) {
    // ---- 4'. heads in sorted order (block scans over rounds of kPsBlock items), their
    // positions in LDS, the record prefix from the look-back, then the records ----
    auto word23 = [&](u32 li, int j) -> u64 {  // words 2-3 of a long key, from the tokens
      if (!long_keys || !(s_w1[li] & 0xffull)) return 0;
      const u32 g = s_list[li];
      const u64 x2 = tokens.w[2][g];
      return j == 2 ? x2 : (x2 & 0xffull) ? tokens.w[3][g] : 0;
    };
    u32 running = 0, firsts = 0;
    for (u32 r0 = 0; r0 < m; r0 += kPsBlock) {
      const u32 i = r0 + (u32)t;
      bool head = false;
      if (i < m) {
        const u32 li = s_perm[cur][i];
        head = i == 0;
        if (!head) {
          const u32 lp = s_perm[cur][i - 1];
          firsts += s_w0[li] != s_w0[lp] ? 1u : 0u;
          head = s_w0[li] != s_w0[lp] || s_w1[li] != s_w1[lp] ||
                 word23(li, 2) != word23(lp, 2) || word23(li, 3) != word23(lp, 3);
        } else {
          firsts += 1;
        }
      }
      u32 tot;
      const u32 ex = dev::block_exclusive_scan<u32, kPsBlock>(head ? 1u : 0u, s_scan, &tot);
      if (head) s_hpos[running + ex] = (u16)i;
      running += tot;
    }
    const u32 U = running;
    if (part_w) {
      firsts = dev::wave_reduce_sum(firsts);
      if (lane == 0 && firsts) atomicAdd(&s_heads, firsts);
    }
    PS_STAMP(4);
    const u64 pfx = dev::block_lookback(ra.status, p, U, &s_prefix);  // syncs (s_hpos too)
    u64* o = reinterpret_cast<u64*>(ra.out + pfx);
    const u32 lim = pfx >= ra.out_cap ? 0u : (u32)min<u64>(U, ra.out_cap - pfx);
    for (u32 q = (u32)t; q < kOutWords * lim; q += kPsBlock) {  // 40-B {key, count}
      const u32 h = q / kOutWords, f = q - kOutWords * h;
      const u32 i = s_hpos[h];
      const u32 li = s_perm[cur][i];
      u64 v;
      if (f == 0) v = s_w0[li];
      else if (f == 1) v = s_w1[li];
      else if (f < 4) v = word23(li, (int)f);
      else v = (u64)((h + 1 < U ? s_hpos[h + 1] : m) - i);
      o[q] = v;
    }
    if (trace && t == 0) trace[(u64)p * 16 + 11] = __builtin_amdgcn_s_memrealtime();
    if (part_w && t == 0) {
      const u64 wk = (u64)m + (u64)kPartDistinctWeight * s_heads;
      part_w[p] = (u32)(wk < 0xffffffffull ? wk : 0xffffffffull);
    }
    reduce_tail(p, U, pfx, ctr, ra, s_prefix, s_last, /*looked_back=*/true);
    return;
  }
  // ---- 4. the partition's slice of the sorted token array, from LDS (words 2-3 gathered
  // only when the partition has keys past 16 bytes); distinct first words counted on the
  // way for the partition map's retuning ----
  u32 heads = 0;
  for (u32 i = (u32)t; i < m; i += kPsBlock) {
    const u32 li = s_perm[cur][i];
    const u64 out = (u64)base + i;
    const u64 k0 = s_w0[li], k1 = s_w1[li];
    if (out < n_cap) {
      u64 k2 = 0, k3 = 0;
      if (long_keys && (k1 & 0xffull)) {
        const u32 g = s_list[li];
        k2 = tokens.w[2][g];
        if (k2 & 0xffull) k3 = tokens.w[3][g];
      }
      sorted.w[0][out] = k0;
      sorted.w[1][out] = k1;
      sorted.w[2][out] = k2;
      sorted.w[3][out] = k3;
    }
    heads += (i == 0 || k0 != s_w0[s_perm[cur][i - 1]]) ? 1u : 0u;
  }
  PS_STAMP(4);
  if (trace && t == 0) trace[(u64)p * 16 + 11] = __builtin_amdgcn_s_memrealtime();
  if (part_w) {
    heads = dev::wave_reduce_sum(heads);
    if (lane == 0 && heads) atomicAdd(&s_heads, heads);
    __syncthreads();
    if (t == 0) {
      const u64 wk = (u64)m + (u64)kPartDistinctWeight * s_heads;
      part_w[p] = (u32)(wk < 0xffffffffull ? wk : 0xffffffffull);
    }
  }
}
#undef PS_STAMP

}  // namespace

void launch_psort(ConstKeysSoA tokens, const u32* part_off, u32 ntiles, u64 cap, KeysSoA sorted,
                  MapCounters* ctr, u32* part_w, hipStream_t s, u64* trace) {
  LOCUST_CHECK_ARG(cap < (1ull << 32), "psort: capacity beyond 32-bit token indices");
  PsortReduceArgs ra;
  psort_kernel<false><<<dim3(kDictParts), dim3(kPsBlock), 0, s>>>(
      tokens, part_off, ntiles, (u32)cap, sorted, ctr, part_w, trace, ra);
  LOCUST_HIP_LAUNCH_CHECK();
}

void launch_psort_reduce(ConstKeysSoA tokens, const u32* part_off, u32 ntiles, u64 cap,
                         MapCounters* ctr, u32* part_w, const PsortReduceArgs& ra, hipStream_t s,
                         u64* trace) {
  LOCUST_CHECK_ARG(cap < (1ull << 32), "psort: capacity beyond 32-bit token indices");
  LOCUST_CHECK_ARG(ra.out && ra.status && ra.done_counter, "psort_reduce: missing buffers");
  psort_kernel<true><<<dim3(kDictParts), dim3(kPsBlock), 0, s>>>(
      tokens, part_off, ntiles, (u32)cap, KeysSoA{}, ctr, part_w, trace, ra);
  LOCUST_HIP_LAUNCH_CHECK();
}

// Loads this file's code object (one module per file) now rather than at its first launch.
void warm_module_psort() {
  hipFuncAttributes a;
  (void)hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&psort_kernel<true>));
}

}  // namespace locust
