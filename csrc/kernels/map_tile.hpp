// The fast map's tile (Map stage): the body of map_fast_kernel (tokenize.hip).  See
// tokenize.hip for the algorithm.
#pragma once

#include "locust/device/hash.hpp"
#include "locust/device/lookback.hpp"
#include "locust/device/wave.hpp"
#include "locust/kernels.hpp"

namespace locust {
namespace maptile {


using dev::ballot;
using dev::lane_id;
using dev::lanes_below;
using dev::wave_id;

// Left context staged before the tile for the backward line-ordinal scans: 128 bytes, so
// the first wave of a tile finds the previous '\n' in LDS for any line up to 128 bytes
// (Hamlet's longest is 75).  With 64 a wave whose segment starts more than 64 bytes into
// a line read the text before the window byte by byte over PCIe (zero-copy input): a
// dependent host round trip in the middle of the map (tile timeline: masks up to 2.6 us).
constexpr int kPre = 128;
constexpr int kPost = 64;  // right overhang staged after the tile (>= 40 for packing)

// Delimiter set incl. '\n' and NUL (a NUL also kills the rest of its line, see
// backward_line_ordinal), held in scalar registers.
// (Passed by reference to the kernel's own argument: a by-value copy inside a device
// function became a private array that the backend promoted to LDS -- 32 B x 1,024 threads
// of it, and every membership test a dynamically indexed LDS read: the map kernel took
// 20 us instead of 13.)
struct Delims {
  u64 m0, m1, m2, m3;
  __device__ __forceinline__ bool has(u32 c) const {
    const u64 m = (c & 128u) ? ((c & 64u) ? m3 : m2) : ((c & 64u) ? m1 : m0);
    return (m >> (c & 63u)) & 1ull;
  }
};

__device__ __forceinline__ u32 global_byte(const char* text, u64 bytes, i64 pos) {
  // Bytes outside [0, bytes) behave like a newline (a line boundary).
  return (pos >= 0 && (u64)pos < bytes) ? (u32)(unsigned char)text[pos] : (u32)'\n';
}

template <int kStaged>
struct TileText {
  const unsigned char* lds;  // staged bytes [lo, lo + kStaged)
  i64 lo;
  const char* text;
  u64 bytes;
  __device__ __forceinline__ u32 at(i64 pos) const {
    const i64 r = pos - lo;
    if (r >= 0 && r < kStaged) return lds[r];
    return global_byte(text, bytes, pos);
  }
};

// Token starts since the last '\n' strictly before `pos`, saturated at cap + 1, and whether
// the line is already dead at `pos`: the reference tokenizes a NUL-terminated copy of the
// line (my_strcpy, /root/reference/MapReduce/src/main.cu:55-59), so bytes after an embedded
// NUL up to the next '\n' are invisible.  The scan stops at the line's '\n', at a NUL (the
// rest of the line is dead), or once the count saturates: a saturated ordinal already
// suppresses every later emit (and the overflow count) of the line, exactly as dead bytes
// would, so a NUL further back need not be found.
template <typename TT>
__device__ __forceinline__ u32 backward_line_ordinal(const TT& tt, i64 pos, const Delims& d, u32 cap,
                                     bool* dead) {
  const int lane = lane_id();
  u32 count = 0;
  *dead = false;
  i64 hi = pos;  // scan [hi - 64, hi)
  while (hi > 0) {
    const i64 p = hi - 64 + lane;
    const u32 c = tt.at(p);  // p < 0 reads as '\n'
    const u32 cprev = tt.at(p - 1);
    const bool start = !d.has(c) && d.has(cprev);
    const u64 nl = ballot(c == '\n');
    const u64 nul = ballot(c == 0u);
    u64 st = ballot(start);
    if (nl) {
      const int last_nl = 63 - __clzll((long long)nl);
      const u64 after = (last_nl >= 63) ? 0ull : (~0ull << (last_nl + 1));
      if (nul & after) {
        *dead = true;
        break;
      }
      count += __popcll(st & after);
      break;
    }
    if (nul) {
      *dead = true;
      break;
    }
    count += __popcll(st);
    if (count > cap) break;
    hi -= 64;
  }
  return count > cap + 1 ? cap + 1 : count;
}

// Length of the token starting at this lane's byte: bit 0 of dmask >> lane is the token's
// first (non-delimiter) byte; the next step's mask covers a token crossing the step.
__device__ __forceinline__ u32 token_length(u64 dmask, u64 dmask_next, int lane) {
  const u64 rest = dmask >> lane;
  if (rest) return (u32)__ffsll((unsigned long long)rest) - 1;
  return (u32)(64 - lane) + (dmask_next ? (u32)__ffsll((unsigned long long)dmask_next) - 1 : 64u);
}

// Big-endian packed key of the `keep` bytes at LDS offset o: five aligned u64 LDS words,
// funnel-shifted, masked and byte-swapped.
__device__ __forceinline__ void pack_token(const unsigned char* s_text, int o, u32 keep,
                                           u64* kw) {
  const int base = o & ~7;
  const u32 sh = (u32)(o & 7) * 8u;
  u64 q[5];
#pragma unroll
  for (int k = 0; k < 5; ++k) q[k] = *reinterpret_cast<const u64*>(s_text + base + 8 * k);
#pragma unroll
  for (int j = 0; j < kKeyWords; ++j) {
    u64 raw = sh ? ((q[j] >> sh) | (q[j + 1] << (64u - sh))) : q[j];
    const int rem = (int)keep - 8 * j;
    if (rem <= 0) raw = 0;
    else if (rem < 8) raw &= (1ull << (8 * rem)) - 1ull;
    kw[j] = __builtin_bswap64(raw);
  }
}

// Tokens of one partition in one 1 KiB tile from which the map asks the ordered kernel to
// plan (split) the pass: whole Hamlet peaks at 27 under the starting map (most tiles below
// 16), a pass whose keys crowd one partition puts ~150 there.
constexpr u32 kPlanTrigger = 48;

// Tile of block b of a G-block launch with consecutive tiles on one XCD: the blocks of a
// launch go to the XCDs round-robin (b = 8 k + x runs on XCD x), so XCD x takes the x-th
// eighth of the tiles in order.  A bijection on [0, G).  Neighbouring tiles then read their
// overlapping context and adjacent lines of the zero-copy text through one XCD: the fast
// map's staging of a Hamlet-sized input 7.9 -> 6.35 us (tools/micro/stage_read.hip).
__device__ __forceinline__ u32 xcd_tile(u32 b, u32 G) {
  constexpr u32 kXcds = 8;
  const u32 q = G / kXcds, r = G % kXcds, x = b % kXcds, k = b / kXcds;
  return x * q + (x < r ? x : r) + k;
}

// The partition map's range starts in LDS, skewed: entry i at i + (i >> 5).  A binary
// search's lanes read entries 2^k apart -- without the skew every such entry of a level
// sits on the same ds_read_b64 bank ((a/4) mod 64: entries 32 apart share one), up to
// 4-way conflicts per level (0.18 of the map's LDS cycles); with it the
// entries of any level fall on distinct banks.
constexpr int kPloSkewed = kDictParts + 1 + ((kDictParts + 1) >> 5) + 1;
__device__ __forceinline__ int plo_at(int i) { return i + (i >> 5); }
__device__ __forceinline__ u32 part_of_w0_skewed(const u64* s_plo, u64 w0) {
  u32 p = 0;
#pragma unroll
  for (u32 step = kDictParts / 2; step; step >>= 1)
    if (s_plo[plo_at((int)(p + step))] <= w0) p += step;
  return p;
}

// The tile's LDS, declared __shared__ by the calling kernel and passed in: LDS variables
// declared inside a device function are lowered to module scope, where every kernel of the
// file that reaches any instantiation pays for all of them (map_fast_kernel<1, 1024> grew
// from 4.4 to 37 KB of LDS that way).
template <int kSteps, int kBlock>
struct MapTileLds {
  static constexpr int kSeg = kSteps * 64;
  static constexpr int kTile = (kBlock / 64) * kSeg;
  static constexpr int kStaged = kPre + kTile + kPost;
  static constexpr bool kCombineTile = kSteps > 1;
  static constexpr int kListPerWave = kSteps > 1 ? kSeg / 2 : 1;
  __attribute__((aligned(16))) unsigned char text[kStaged];
  u64 prefix;
  u32 wave_cnt[kBlock / 64];
  // partition grouping (with part_off): per-partition counts, then offsets
  u32 pcnt[kPartTable];
  // per-tile combining (large grouped tiles with `counts`): the first short key (<= 7 bytes,
  // one word) of each partition claims a slot; its repeats in the tile become one record
  u64 hot[kCombineTile ? kDictParts : 1];
  u32 hotc[kCombineTile ? kDictParts : 1];
  // the partition map's range starts (PartMap), staged once per tile (skewed: plo_at), 2 KB,
  // searched per token
  u64 plo[kPloSkewed];
  // grouped large tiles: each wave's token starts (LDS offset | length << 16), at most one
  // per two bytes of its segment
  u32 list[(kBlock / 64) * kListPerWave];
};

// One map tile (the body of map_fast_kernel): kBlock threads, tile index `tile` (the
// XCD-ordered block index of map_fast_kernel).
template <int kSteps, int kBlock>
__device__ __forceinline__ void map_tile(
    MapTileLds<kSteps, kBlock>& lds, const u32 tile, const char* __restrict__ text, u64 bytes,
    const Delims& d, int E, int max_key, KeysSoA out, u8* __restrict__ parts, u64 out_cap,
    MapCounters* __restrict__ ctr, u64* __restrict__ trace, u32* __restrict__ part_off, PartMap pm,
    u64* __restrict__ counts, u32* __restrict__ part_occ, u32* __restrict__ plan_flag = nullptr) {
  // trace (diagnostics, LOCUST_MAP_TRACE): per tile, s_memrealtime (100 MHz, device-wide)
  // at entry, tile acquired, text staged, masks done, prefix known, keys written.
  const u64 t_entry = trace ? __builtin_amdgcn_s_memrealtime() : 0;
#define MAP_STAMP(k_)                                                           \
  if (trace && threadIdx.x == 0 && tile < 4096) trace[(u64)tile * 8 + (k_)] = __builtin_amdgcn_s_memrealtime()
  using L = MapTileLds<kSteps, kBlock>;
  constexpr int kSeg = L::kSeg;
  constexpr int kTile = L::kTile;
  constexpr int kStaged = L::kStaged;
  constexpr bool kCombineTile = L::kCombineTile;
  constexpr int kListPerWave = L::kListPerWave;
  constexpr int kListRounds = kListPerWave / 64 > 0 ? kListPerWave / 64 : 1;
  unsigned char* s_text = lds.text;
  u64& s_prefix = lds.prefix;
  u32* s_wave_cnt = lds.wave_cnt;
  u32* s_pcnt = lds.pcnt;
  u64* s_hot = lds.hot;
  u32* s_hotc = lds.hotc;
  u64* s_plo = lds.plo;
  u32* s_list = lds.list;
  const bool combine = kCombineTile && part_off && counts;
  const int lane = lane_id(), w = wave_id();
  const u64 num_tiles = div_up(bytes, (u64)kTile);
  // Tokens are emitted in no particular order across tiles (every consumer sorts or
  // hashes them), so a tile needs no ticket order and no look-back.
  if (tile >= num_tiles) return;
  if (trace && threadIdx.x == 0 && tile < 4096) trace[(u64)tile * 8] = t_entry;
  MAP_STAMP(1);
  if (part_off)
    for (int i = threadIdx.x; i < kPartTable; i += kBlock) s_pcnt[i] = 0;  // before a barrier
  if (combine)
    for (int i = threadIdx.x; i < kDictParts; i += kBlock) {
      s_hot[i] = 0;
      s_hotc[i] = 0;
    }

  if (pm.lo)  // visible after the staging barrier below
    for (int i = threadIdx.x; i <= kDictParts; i += kBlock) s_plo[plo_at(i)] = pm.lo[i];
  // Partition of a packed key: binary search of its first word (default: first byte).
  auto part_of = [&](u64 w0) -> u32 {
    return pm.lo ? part_of_w0_skewed(s_plo, w0) : (u32)(w0 >> 56);
  };

  // ---- stage the tile (+ context) into LDS with 16-B loads ----
  const i64 tile_base = (i64)tile * kTile;
  const i64 lo = tile_base - kPre;
  // Every text buffer carries >= 16 readable bytes past its end (the engine's padding), so
  // a chunk that starts inside the text is one 16-B load; its bytes past the end read as
  // '\n' like global_byte's.  Only chunks wholly outside the text are synthesised.
  for (int c = threadIdx.x; c < kStaged / 16; c += kBlock) {
    const i64 g = lo + (i64)c * 16;
    if (g >= 0 && (u64)g < bytes) {
      uint4 v = *reinterpret_cast<const uint4*>(text + g);
      *reinterpret_cast<uint4*>(s_text + c * 16) = v;
      if ((u64)(g + 16) > bytes)
        for (int k = (int)(bytes - (u64)g); k < 16; ++k) s_text[c * 16 + k] = (unsigned char)'\n';
    } else {
      const uint32_t nl4 = 0x0a0a0a0au;
      *reinterpret_cast<uint4*>(s_text + c * 16) = uint4{nl4, nl4, nl4, nl4};
    }
  }
  __syncthreads();
  MAP_STAMP(2);
  const TileText<kStaged> tt{s_text, lo, text, bytes};
  const i64 seg = tile_base + (i64)w * kSeg;
  const int seg_lds = kPre + w * kSeg;

  // ---- phase 1: delimiter masks, token starts, in-line ordinals, emit masks ----
  bool line_dead;  // an embedded NUL earlier in the current line (see backward scan)
  u32 line_ord = backward_line_ordinal(tt, seg, d, (u32)E, &line_dead);
  bool prev_delim = d.has(s_text[seg_lds - 1]);
  u64 emit_mask[kSteps];
  u64 dmask[kSteps + 1];
  u32 emitted = 0, overflow = 0;
  const u64 below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
#pragma unroll
  for (int s = 0; s < kSteps; ++s) {
    const i64 p = seg + s * 64 + lane;
    const bool in = (u64)p < bytes;
    const u32 c = s_text[seg_lds + s * 64 + lane];
    const bool is_d = d.has(c);
    dmask[s] = ballot(is_d);
    const bool pd = lane == 0 ? prev_delim : ((dmask[s] >> (lane - 1)) & 1ull);
    prev_delim = (dmask[s] >> 63) & 1ull;
    const u64 nl = ballot(in && c == '\n');
    const u64 nul = ballot(in && c == 0u);
    const u64 nl_below = nl & below;
    // Dead byte: a NUL after the line's last '\n' below this lane (or carried in).
    bool dead = line_dead && !nl_below;
    if (const u64 nul_below = nul & below) {
      dead = dead || !nl_below || (63 - __clzll((long long)nul_below)) >
                                      (63 - __clzll((long long)nl_below));
    }
    const bool start = in && !is_d && pd && !dead;
    const u64 st = ballot(start);
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
      line_dead = (q >= 63) ? false : ((nul >> (q + 1)) != 0ull);
    } else {
      line_ord += __popcll(st);
      line_dead = line_dead || nul != 0ull;
    }
    if (line_ord > (u32)E + 1) line_ord = (u32)E + 1;
  }
  dmask[kSteps] = ballot(d.has(s_text[seg_lds + kSteps * 64 + lane]));  // lookahead

  // ---- small grouped tiles (kSteps == 1, part_off): the token's partition and its rank
  // in the tile's partition run are drawn before the first barrier, and the tile's slice
  // of the token array is reserved while wave 0 scans the partition counts -- the global
  // atomic's round trip overlaps the scan, and the tile takes two barriers, not four ----
  if constexpr (kSteps == 1) {
    if (part_off) {
      MAP_STAMP(6);  // (wave 0's) masks
      const u64 m = emit_mask[0];
      const bool em = (m >> lane) & 1ull;
      u64 kw[kKeyWords] = {0, 0, 0, 0};
      u32 part = 0, loc = 0, len = 0;
      if (em) {
        len = token_length(dmask[0], dmask[1], lane);
        pack_token(s_text, seg_lds + lane, len < (u32)max_key ? len : (u32)max_key, kw);
        part = part_of(kw[0]);
        loc = atomicAdd(&s_pcnt[part], 1u);
      }
      if (lane == 0) s_wave_cnt[w] = emitted;
      MAP_STAMP(7);  // (wave 0's) keys packed and ranked
      __syncthreads();  // wave counts and partition counts complete
      MAP_STAMP(3);
      if (lane == 0 && overflow) atomicAdd(&ctr->overflow_lines, overflow);
      if (threadIdx.x < 64) {
        u32 tile_total = 0;
#pragma unroll
        for (int i = 0; i < kBlock / 64; ++i) tile_total += s_wave_cnt[i];
        // issued now, its value needed only after the scan below
        u64 slice = 0;
        if (threadIdx.x == 0 && tile_total) slice = atomicAdd(&ctr->num_records, tile_total);
        // exclusive scan of the 256 partition counts by one wave
        const u32 l = threadIdx.x;
        const u32 h0 = s_pcnt[4 * l], h1 = s_pcnt[4 * l + 1], h2 = s_pcnt[4 * l + 2],
                  h3 = s_pcnt[4 * l + 3];
        // a partition crowding this tile (kPlanTrigger tokens of ~180): the ordered kernel
        // plans this pass (OrderedExtra::plan_flag); one atomic per such tile
        if (plan_flag && dev::ballot(h0 >= kPlanTrigger || h1 >= kPlanTrigger ||
                                     h2 >= kPlanTrigger || h3 >= kPlanTrigger) &&
            l == 0)
          atomicOr(plan_flag, 1u);
        if (part_occ) {  // the tile's 256-bit partition occupancy: 8 words, lane 8w writes w
          u32 occ = ((h0 ? 1u : 0u) | (h1 ? 2u : 0u) | (h2 ? 4u : 0u) | (h3 ? 8u : 0u)) << (4 * (l & 7));
          occ |= (u32)__shfl_xor((int)occ, 1, 64);
          occ |= (u32)__shfl_xor((int)occ, 2, 64);
          occ |= (u32)__shfl_xor((int)occ, 4, 64);
          if ((l & 7) == 0) part_occ[(u64)tile * kPartOccWords + (l >> 3)] = occ;
        }
        const u32 sum4 = h0 + h1 + h2 + h3;
        const u32 inc = dev::wave_inclusive_scan(sum4);
        const u32 ex = inc - sum4;
        s_pcnt[4 * l] = ex;
        s_pcnt[4 * l + 1] = ex + h0;
        s_pcnt[4 * l + 2] = ex + h0 + h1;
        s_pcnt[4 * l + 3] = ex + h0 + h1 + h2;
        if (l == 63) s_pcnt[kDictParts] = inc;
        if (threadIdx.x == 0) s_prefix = slice;
      }
      __syncthreads();
      const u64 prefix = s_prefix;
      MAP_STAMP(4);
      for (int i = threadIdx.x; i < kPartTable; i += kBlock)
        part_off[(u64)tile * kPartTable + i] = (u32)(prefix + s_pcnt[i]);
      u32 trunc = 0, maxlen = 0;
      if (em) {
        const u64 idx = prefix + s_pcnt[part] + loc;
        if (len > (u32)max_key) trunc = 1;
        maxlen = len;
        if (idx < out_cap) {
#pragma unroll
          for (int j = 0; j < kKeyWords; ++j) out.w[j][idx] = kw[j];
          if (parts) parts[idx] = (u8)part;
        }
      }
      trunc = dev::wave_reduce_sum(trunc);
      maxlen = dev::wave_reduce_max(maxlen);
      if (lane == 0 && trunc) atomicAdd(&ctr->truncated, trunc);
      if (lane == 0 && maxlen > (u32)max_key) atomicMax(&ctr->max_key_len, maxlen);
      MAP_STAMP(5);
      return;
    }
  }

  // ---- phase 2: wave counts -> tile prefix (look-back) ----
  if (lane == 0) s_wave_cnt[w] = emitted;
  __syncthreads();
  MAP_STAMP(3);
  u32 wave_excl = 0, tile_total = 0;
#pragma unroll
  for (int i = 0; i < kBlock / 64; ++i) {
    const u32 v = s_wave_cnt[i];
    if (i < w) wave_excl += v;
    tile_total += v;
  }
  // this tile's slice of the token array: one atomic per tile (a combining tile reserves
  // its records once it has counted them)
  if (threadIdx.x == 0 && !combine) s_prefix = tile_total ? atomicAdd(&ctr->num_records, tile_total) : 0;
  __syncthreads();
  const u64 prefix = s_prefix;
  MAP_STAMP(4);
  if (lane == 0 && overflow) atomicAdd(&ctr->overflow_lines, overflow);

  if constexpr (kSteps > 1) {
    if (part_off) {
      // ---- phase 3 (grouped, large tiles): a lane owns a byte, so only the ~1 in 7 lanes
      // at a token start would work per step.  Each wave first compacts its segment's
      // token starts into an LDS list (offset + length); two dense sweeps over the list
      // then draw the partition ranks (first sweep) and write the keys once the tile's
      // partition offsets are known (second sweep, keys repacked from LDS) ----
      constexpr u32 kCombined = 0xFFFFu;  // folded into its partition's hot record
      u32* my_list = s_list + w * kListPerWave;
      u32 n_w = 0;
#pragma unroll
      for (int s = 0; s < kSteps; ++s) {
        const u64 m = emit_mask[s];
        if ((m >> lane) & 1ull) {
          const u32 len = token_length(dmask[s], dmask[s + 1], lane);
          my_list[n_w + lanes_below(m)] =
              (u32)(seg_lds + s * 64 + lane) | ((len < 255u ? len : 255u) << 16);
        }
        n_w += __popcll(m);
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      u32 info[kListRounds];  // partition << 16 | rank in the partition (kCombined: folded)
#pragma unroll
      for (int r = 0; r < kListRounds; ++r) {
        info[r] = 0;
        const u32 i = (u32)r * 64 + lane;
        if ((u32)r * 64 >= n_w) break;  // wave-uniform
        if (i < n_w) {
          const u32 e = my_list[i];
          const u32 len = e >> 16;
          u64 kw[kKeyWords];
          pack_token(s_text, (int)(e & 0xffffu), len < (u32)max_key ? len : (u32)max_key, kw);
          const u32 part = part_of(kw[0]);
          bool folded = false;
          if (combine && (kw[0] & 0xffull) == 0) {  // a one-word key
            const u64 old = atomicCAS(reinterpret_cast<unsigned long long*>(&s_hot[part]), 0ull,
                                      (unsigned long long)kw[0]);
            if (old == 0 || old == kw[0]) {
              atomicAdd(&s_hotc[part], 1u);
              folded = true;
            }
          }
          info[r] = (part << 16) | (folded ? kCombined : atomicAdd(&s_pcnt[part], 1u));
        }
      }
      __syncthreads();
      if (combine) {  // a partition with a hot record: it leads the partition's run
        for (int i = threadIdx.x; i < kDictParts; i += kBlock) s_pcnt[i] += s_hotc[i] ? 1u : 0u;
        __syncthreads();
      }
      if (threadIdx.x < 64) {  // exclusive scan of the 256 partition counts by one wave
        const u32 l = threadIdx.x;
        const u32 h0 = s_pcnt[4 * l], h1 = s_pcnt[4 * l + 1], h2 = s_pcnt[4 * l + 2],
                  h3 = s_pcnt[4 * l + 3];
        const u32 sum4 = h0 + h1 + h2 + h3;
        const u32 inc = dev::wave_inclusive_scan(sum4);
        const u32 ex = inc - sum4;
        s_pcnt[4 * l] = ex;
        s_pcnt[4 * l + 1] = ex + h0;
        s_pcnt[4 * l + 2] = ex + h0 + h1;
        s_pcnt[4 * l + 3] = ex + h0 + h1 + h2;
        if (l == 63) {
          s_pcnt[kDictParts] = inc;
          // a combining tile reserves its records (hot records + the rest) only now, and
          // counts its tokens in the same atomic: (map_tokens : num_records) is one u64
          // (same-address atomics serialise at the memory side -- one per tile, not two)
          if (combine) {
            const u64 add = ((u64)tile_total << 32) | inc;
            s_prefix = add ? (u32)atomicAdd(reinterpret_cast<unsigned long long*>(&ctr->num_records),
                                            (unsigned long long)add)
                           : 0u;
          }
        }
      }
      __syncthreads();
      MAP_STAMP(6);
      const u64 gprefix = combine ? s_prefix : prefix;
      for (int i = threadIdx.x; i < kPartTable; i += kBlock)
        part_off[(u64)tile * kPartTable + i] = (u32)(gprefix + s_pcnt[i]);
      if (combine) {  // the hot records
        for (int i = threadIdx.x; i < kDictParts; i += kBlock) {
          const u32 c = s_hotc[i];
          const u64 idx = gprefix + s_pcnt[i];
          if (c && idx < out_cap) {
            out.w[0][idx] = s_hot[i];
#pragma unroll
            for (int j = 1; j < kKeyWords; ++j) out.w[j][idx] = 0;
            counts[idx] = c;
            if (parts) parts[idx] = (u8)i;
          }
        }
      }
      u32 trunc = 0, maxlen = 0;
#pragma unroll
      for (int r = 0; r < kListRounds; ++r) {
        const u32 i = (u32)r * 64 + lane;
        if ((u32)r * 64 >= n_w) break;  // wave-uniform
        if (i < n_w) {
          const u32 e = my_list[i];
          const u32 len = e >> 16;
          if (len > (u32)max_key) ++trunc;
          maxlen = len > maxlen ? len : maxlen;
          const u32 rank = info[r] & 0xffffu;
          if (rank == kCombined) continue;
          const u32 part = info[r] >> 16;
          u64 kw[kKeyWords];
          pack_token(s_text, (int)(e & 0xffffu), len < (u32)max_key ? len : (u32)max_key, kw);
          const u64 idx = gprefix + s_pcnt[part] + (combine && s_hotc[part] ? 1u : 0u) + rank;
          if (idx < out_cap) {
#pragma unroll
            for (int j = 0; j < kKeyWords; ++j) out.w[j][idx] = kw[j];
            if (parts) parts[idx] = (u8)part;
            if (combine) counts[idx] = 1;
          }
        }
      }
      trunc = dev::wave_reduce_sum(trunc);
      maxlen = dev::wave_reduce_max(maxlen);
      if (lane == 0 && trunc) atomicAdd(&ctr->truncated, trunc);
      if (lane == 0 && maxlen > (u32)max_key) atomicMax(&ctr->max_key_len, maxlen);
      MAP_STAMP(5);
      return;
    }
  }
  // ---- phase 3: length from masks, pack from LDS words, write ----
  u64 dst = prefix + wave_excl;
  u32 trunc = 0, maxlen = 0;
#pragma unroll
  for (int s = 0; s < kSteps; ++s) {
    const u64 m = emit_mask[s];
    if (m & (1ull << lane)) {
      const u64 idx = dst + lanes_below(m);
      const u32 len = token_length(dmask[s], dmask[s + 1], lane);
      if (len > (u32)max_key) ++trunc;
      maxlen = len > maxlen ? len : maxlen;
      u64 kw[kKeyWords];
      pack_token(s_text, seg_lds + s * 64 + lane, len < (u32)max_key ? len : (u32)max_key, kw);
      if (idx < out_cap) {
#pragma unroll
        for (int j = 0; j < kKeyWords; ++j) out.w[j][idx] = kw[j];
        // partition tag for the dictionary's partitioned builds (order-preserving, so
        // per-partition sorts concatenate into the global order)
        if (parts) parts[idx] = (u8)part_of(kw[0]);
      }
    }
    dst += __popcll(m);
  }
  // Rare events only: one atomic per wave that actually truncated a token.  (A per-wave
  // atomicMax on one shared word serialises the waves at the memory side, so the longest
  // token is only recorded when it exceeded the key width.)
  trunc = dev::wave_reduce_sum(trunc);
  maxlen = dev::wave_reduce_max(maxlen);
  if (lane == 0 && trunc) atomicAdd(&ctr->truncated, trunc);
  if (lane == 0 && maxlen > (u32)max_key) atomicMax(&ctr->max_key_len, maxlen);
  MAP_STAMP(5);
#undef MAP_STAMP
}


}  // namespace maptile
}  // namespace locust
