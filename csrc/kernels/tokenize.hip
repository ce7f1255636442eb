// Byte-parallel wave64 tokenizer (Map stage, fast path).
//
// Semantics are those of the reference map() (/root/reference/MapReduce/src/main.cu:136-153:
// strtok_r over " ,.-;:'()\"\t", at most EMITS_PER_LINE tokens per line, value 1), but the
// work is spread over bytes instead of lines:
//
//  * A workgroup owns a tile of wave segments (STEPS x 64 bytes each): 16 waves x one step
//    (1 KiB) for inputs below kMapLargeInput, 4 waves x 16 steps (4 KiB) above.  The tile
//    plus 128 bytes of left context (kPre) and 64 bytes of right overhang (kPost) is staged
//    into LDS with 16-byte vector loads, so every later byte access is an LDS read.
//  * Each step, every lane looks at one byte.  The delimiter set lives in four u64 kernel
//    arguments (SGPRs), so the membership test is a few VALU ops.  Ballots give the step's
//    delimiter mask; token start = not-delimiter && previous byte is a delimiter.  The
//    per-line ordinal (for the 20-emit cap) is the popcount of starts since the last
//    '\n', carried across steps; the ordinal carried INTO a segment comes from a backward
//    scan to the previous newline, stopped once it exceeds the cap.
//  * Emit counts are summed across the tile's waves; one atomic per tile reserves the tile's
//    slice of the token array (tokens are not kept in text order across tiles: every
//    consumer hashes or sorts them, so no ticket and no look-back chain is needed -- the
//    tiles all start at once and the zero-copy text reads overlap), then each emitting
//    lane finds its token's length from the delimiter
//    masks (count-trailing-zeros, no per-byte loop), reads 40 bytes of LDS as five
//    aligned u64 words, funnel-shifts, masks and byte-swaps them into the big-endian
//    packed key, and writes it straight into the dense SoA output.  The map output is
//    born compacted, so the reference's 116,000-slot thrust::partition (main.cu:411) has
//    nothing left to do.  With a partition map (part_off) the tile writes its tokens
//    grouped by partition and records where each partition's run starts (map_tile.hpp),
//    which is how the ordered kernel finds a partition's tokens.
#include <cstdlib>

#include "locust/hip_check.hpp"
#include "locust/kernels.hpp"
#include "map_tile.hpp"

namespace locust {
namespace {

using namespace maptile;

template <int kSteps, int kBlock>
__global__ __launch_bounds__(kBlock) void map_fast_kernel(
    const char* __restrict__ text, u64 bytes, Delims d, int E, int max_key, KeysSoA out,
    u8* __restrict__ parts, u64 out_cap, MapCounters* __restrict__ ctr, u64* __restrict__ trace,
    u32* __restrict__ part_off, PartMap pm, u64* __restrict__ counts, u32* __restrict__ part_occ,
    u32* __restrict__ plan_flag) {
  __shared__ MapTileLds<kSteps, kBlock> lds;
  // consecutive tiles per XCD: neighbouring tiles share L2 lines of the text and tables
  const u32 tile = xcd_tile(blockIdx.x, gridDim.x);
  map_tile<kSteps, kBlock>(lds, tile, text, bytes, d, E, max_key, out, parts, out_cap, ctr,
                           trace, part_off, pm, counts, part_occ, plan_flag);
}

}  // namespace

void launch_map_fast(const char* text, u64 bytes, const DelimMask& dm, int emits_per_line,
                     int max_key_len, KeysSoA out, u8* parts, u64 out_cap, MapCounters* ctr,
                     LookbackScratch lb, hipStream_t s, u64* trace, u32* part_off,
                     PartMap pm, bool large_tiles, u64* counts, u32* part_occ,
                     u32* plan_flag) {
  if (bytes == 0) return;
  const Delims d{dm.m[0] | 1ull | (1ull << '\n'), dm.m[1], dm.m[2], dm.m[3]};
  if (bytes < kMapLargeInput && !large_tiles) {
    // Small inputs: 1 KiB tiles as 16 waves x ONE 64-byte step -- the same text per
    // workgroup (and the same PCIe reads), the least serial work per wave.  Measured A/B
    // in one process against 4 waves x 4 steps, 8 x 2 and 8 x 1 (profiles/r1_s2/
    // map_shape_ab.txt): 1-3 % faster whole jobs.
    const u64 tiles = div_up(bytes, (u64)kMapTileBytesMin);
    constexpr int kBlock = kMapTileBytesMin;  // one byte per lane: 16 waves of 64 lanes
    map_fast_kernel<1, kBlock><<<dim3((u32)tiles), dim3(kBlock), 0, s>>>(
        text, bytes, d, emits_per_line, max_key_len, out, parts, out_cap, ctr, trace, part_off, pm,
        nullptr, part_off ? part_occ : nullptr, part_off && part_occ ? plan_flag : nullptr);
  } else {
    constexpr int kTile = (kMapBlock / 64) * kMapSegStepsLarge * 64;
    const u64 tiles = div_up(bytes, (u64)kTile);
    map_fast_kernel<kMapSegStepsLarge, kMapBlock><<<dim3((u32)tiles), dim3(kMapBlock), 0, s>>>(
        text, bytes, d, emits_per_line, max_key_len, out, parts, out_cap, ctr, trace, part_off, pm,
        part_off ? counts : nullptr, nullptr, nullptr);
  }
  LOCUST_HIP_LAUNCH_CHECK();
}

// Loads this file's code object (one module per file) now rather than at its first launch.
void warm_module_tokenize() {
  hipFuncAttributes a;
  (void)hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&map_fast_kernel<1, 1024>));
}

}  // namespace locust
