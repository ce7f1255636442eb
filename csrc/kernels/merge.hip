// Root merge of the gather strategy: P sorted runs of combined (key, count) records -> the
// globally sorted (key, val, count) output, in two short kernels.
//
// The reference has no merge at all: its reducer expects one pre-sorted /tmp/out.txt
// (main.cu:437-465, bug B7), and the cross-node transfer that would feed it is missing
// (README.md:24).  Here every rank's combined output arrives sorted, so the root does not
// rebuild a dictionary over them; it merges:
//
//   merge_rank   one thread per record: lock-step binary searches in every other run give
//                the record's position in the stable (key, run) merge order, whether a
//                lower run already holds the key (then this copy is a duplicate), and --
//                for the first copy -- the key's total count over all runs.  Records are
//                scattered to their merged slots (duplicates with count 0).
//   merge_emit   decoupled look-back scan over the merged slots of (#first copies, count
//                sum): the first copies are compacted into the output with val = the
//                exclusive prefix of the counts (the reference's val: start index of the
//                key's run in the globally sorted token array, main.cu:161-208).
//
// Runs are at most 64 (one per rank), the lock-step search keeps up to 8 runs' probes in
// flight per thread, and the output goes straight into host-mapped memory.
#include "locust/device/lookback.hpp"
#include "locust/hip_check.hpp"
#include "locust/kernels.hpp"

namespace locust {
namespace {

constexpr int kMergeBlock = 256;
constexpr int kMergeLanes = 8;                        // runs searched in lock step
constexpr int kEmitItems = 4;                          // merged slots per thread
constexpr int kEmitTile = kMergeBlock * kEmitItems;    // 1,024 slots: 48 KB of LDS staging
constexpr int kEmitCountBits = 40;                     // look-back value: [firsts:22][counts:40]
constexpr u64 kEmitCountMask = (1ull << kEmitCountBits) - 1;

// -1 / 0 / +1: order of record key `a` against key `k` (unsigned words, big-endian bytes).
__device__ __forceinline__ int cmp_key(const KeyCount* a, const u64* k) {
  const u64 a0 = a->w[0];
  if (a0 != k[0]) return a0 < k[0] ? -1 : 1;
#pragma unroll
  for (int j = 1; j < kKeyWords; ++j) {
    const u64 aj = a->w[j];
    if (aj != k[j]) return aj < k[j] ? -1 : 1;
  }
  return 0;
}

// Where the runs are: packed (run 0 = `own`, runs 1.. back to back in `recv`, lengths in
// `meta` = [nruns, len0, len1, ...]) or all-gathered slots (fixed stride, a SlotHeader in
// front of each slot's records).  Read from device memory at run time, so a captured graph
// stays valid when the lengths change.
struct RunsView {
  const KeyCount* own;
  const KeyCount* recv;
  const u32* meta;
  const KeyCount* slots;  // non-null: slot layout
  u32 nslots, slot_records;
};

struct RunTable {
  u32 nruns;
  u32 off[kMaxMergeRunsHost + 1];  // start of run q in the concatenated index space
  const KeyCount* base[kMaxMergeRunsHost];
};

__device__ __forceinline__ void load_runs(const RunsView& v, RunTable& t) {
  if (threadIdx.x == 0) {
    u32 acc = 0;
    if (v.slots) {
      const u32 nr = min(v.nslots, (u32)kMaxMergeRunsHost);
      const u64 stride = (u64)kSlotHeaderRecords + v.slot_records;
      for (u32 q = 0; q < nr; ++q) {
        const KeyCount* slot = v.slots + q * stride;
        const SlotHeader* h = reinterpret_cast<const SlotHeader*>(slot);
        const u32 len = h->status == kSlotOk ? (u32)min(h->n, (u64)v.slot_records) : 0u;
        t.off[q] = acc;
        t.base[q] = slot + kSlotHeaderRecords;
        acc += len;
      }
      t.off[nr] = acc;
      t.nruns = nr;
    } else {
      const u32 nr = min(v.meta[0], (u32)kMaxMergeRunsHost);
      for (u32 q = 0; q < nr; ++q) {
        t.off[q] = acc;
        t.base[q] = q == 0 ? v.own : v.recv + (acc - v.meta[1]);  // runs 1.. back to back
        acc += v.meta[1 + q];
      }
      t.off[nr] = acc;
      t.nruns = nr;
    }
  }
  __syncthreads();
}

__global__ __launch_bounds__(kMergeBlock) void merge_rank_kernel(
    RunsView view, KeyCount* __restrict__ merged, LookbackScratch lb, u32 emit_tiles,
    SlotHeader* __restrict__ hdr_out) {
  __shared__ RunTable t;
  if (blockIdx.x == 0) {
    // merge_emit's look-back scratch, reset here (stream order) instead of by a memset
    for (u32 i = threadIdx.x; i < emit_tiles; i += kMergeBlock) lb.status[i] = 0;
    if (threadIdx.x == 0) *lb.tile_counter = 0;
    // the slot headers for the host (the root needs no separate copy)
    if (hdr_out && view.slots) {
      const u64 stride = (u64)kSlotHeaderRecords + view.slot_records;
      for (u32 q = threadIdx.x; q < view.nslots; q += kMergeBlock)
        hdr_out[q] = *reinterpret_cast<const SlotHeader*>(view.slots + q * stride);
    }
  }
  load_runs(view, t);
  const u32 nruns = t.nruns;
  const u32 total = t.off[nruns];
  for (u32 g = blockIdx.x * kMergeBlock + threadIdx.x; g < total; g += gridDim.x * kMergeBlock) {
    u32 q = 0;
    while (q + 1 < nruns && t.off[q + 1] <= g) ++q;
    const u32 i = g - t.off[q];
    const KeyCount rec = t.base[q][i];
    const u64 k[kKeyWords] = {rec.w[0], rec.w[1], rec.w[2], rec.w[3]};
    u64 pos = i;
    u64 count = rec.count;
    bool first = true;
    for (u32 r0 = 0; r0 < nruns; r0 += kMergeLanes) {
      const KeyCount* base[kMergeLanes];
      u32 lo[kMergeLanes], len[kMergeLanes];
      bool eq[kMergeLanes];
#pragma unroll
      for (int l = 0; l < kMergeLanes; ++l) {
        const u32 r = r0 + l;
        const bool live = r < nruns && r != q;
        base[l] = live ? t.base[r] : nullptr;
        lo[l] = 0;
        len[l] = live ? t.off[r + 1] - t.off[r] : 0;
        eq[l] = false;
      }
      // lower_bound in every live run, one probe per run per step (independent loads)
      for (;;) {
        bool any = false;
#pragma unroll
        for (int l = 0; l < kMergeLanes; ++l) {
          if (len[l]) {
            any = true;
            const u32 half = len[l] >> 1;
            const int c = cmp_key(base[l] + lo[l] + half, k);
            if (c < 0) {
              lo[l] += half + 1;
              len[l] -= half + 1;
            } else {
              eq[l] |= c == 0;  // keys are distinct within a run: lower_bound lands here
              len[l] = half;
            }
          }
        }
        if (!any) break;
      }
#pragma unroll
      for (int l = 0; l < kMergeLanes; ++l) {
        const u32 r = r0 + l;
        if (r >= nruns || r == q) continue;
        if (r < q) {
          pos += lo[l] + (eq[l] ? 1 : 0);  // equal keys of lower runs come first
          first &= !eq[l];
        } else {
          pos += lo[l];
          if (eq[l]) count += base[l][lo[l]].count;
        }
      }
    }
    KeyCount out;
#pragma unroll
    for (int j = 0; j < kKeyWords; ++j) out.w[j] = k[j];
    out.count = first ? count : 0;  // later copies of a key carry nothing
    merged[pos] = out;
  }
}

__global__ __launch_bounds__(kMergeBlock) void merge_emit_kernel(
    const KeyCount* __restrict__ merged, RunsView view, MapCounters* __restrict__ ctr,
    OutRecord* __restrict__ out, MapCounters* __restrict__ ctr_out, u64* __restrict__ status,
    u32* __restrict__ tile_ctr) {
  __shared__ u64 s_scan[kMergeBlock / 64 + 1];
  __shared__ u32 s_tile;
  __shared__ u64 s_prefix;
  __shared__ RunTable t;
  // the tile's output records, staged so that the (host-mapped) writes are full lines
  __shared__ __attribute__((aligned(16))) u64 s_out[kEmitTile * 6];
  const u32 tile = dev::acquire_tile(tile_ctr, &s_tile);
  load_runs(view, t);
  const u32 total = t.off[t.nruns];
  const u32 ntiles = total ? (u32)div_up(total, (u64)kEmitTile) : 1u;
  if (tile >= ntiles) return;  // uniform per workgroup; nobody waits on these tiles
  const u32 i0 = tile * kEmitTile + threadIdx.x * kEmitItems;
  KeyCount v[kEmitItems];
  u64 agg = 0;
#pragma unroll
  for (int e = 0; e < kEmitItems; ++e) {
    const u32 i = i0 + e;
    if (i < total) {
      v[e] = merged[i];
    } else {
      v[e].count = 0;
    }
    if (v[e].count) agg += (1ull << kEmitCountBits) + v[e].count;
  }
  u64 tile_sum = 0;
  const u64 excl = dev::block_exclusive_scan<u64, kMergeBlock>(agg, s_scan, &tile_sum);
  const u64 before = dev::block_lookback(status, tile, tile_sum, &s_prefix);
  u32 li = (u32)(excl >> kEmitCountBits);  // index inside the tile's output slice
  u64 val = (before + excl) & kEmitCountMask;
#pragma unroll
  for (int e = 0; e < kEmitItems; ++e) {
    if (!v[e].count) continue;
    u64* o = s_out + 6 * li;
#pragma unroll
    for (int j = 0; j < kKeyWords; ++j) o[j] = v[e].w[j];
    o[4] = val;
    o[5] = v[e].count;
    ++li;
    val += v[e].count;
  }
  __syncthreads();
  const u32 m = (u32)(tile_sum >> kEmitCountBits);
  const u64 base = before >> kEmitCountBits;
  // consecutive lanes, consecutive 16-B chunks of out[base .. base + m)
  const uint4* src = reinterpret_cast<const uint4*>(s_out);
  uint4* dst = reinterpret_cast<uint4*>(out + base);
  for (u32 q = threadIdx.x; q < 3 * m; q += kMergeBlock) dst[q] = src[q];
  if (tile == ntiles - 1 && threadIdx.x == 0) {
    const u64 all = before + tile_sum;
    const u32 u = (u32)(all >> kEmitCountBits);
    const u64 tok = all & kEmitCountMask;
    ctr->num_records = total;
    ctr->num_unique = u;
    ctr->total_count = tok;
    if (ctr_out) {
      MapCounters c{};
      c.num_records = total;
      c.num_unique = u;
      c.total_count = tok;
      *ctr_out = c;
    }
  }
}

void launch_merge_view(const RunsView& v, u64 cap, KeyCount* merged, MapCounters* ctr,
                       OutRecord* out, MapCounters* ctr_out, LookbackScratch lb,
                       SlotHeader* hdr_out, hipStream_t s) {
  const u64 c = cap ? cap : 1;
  const u32 rank_grid = (u32)std::min<u64>(div_up(c, kMergeBlock), 4096);
  const u32 emit_grid = (u32)div_up(c, (u64)kEmitTile);
  merge_rank_kernel<<<dim3(rank_grid), dim3(kMergeBlock), 0, s>>>(v, merged, lb, emit_grid,
                                                                  hdr_out);
  LOCUST_HIP_LAUNCH_CHECK();
  merge_emit_kernel<<<dim3(emit_grid), dim3(kMergeBlock), 0, s>>>(merged, v, ctr, out, ctr_out,
                                                                  lb.status, lb.tile_counter);
  LOCUST_HIP_LAUNCH_CHECK();
}

}  // namespace

u64 merge_scratch_words(u64 cap) { return div_up(cap ? cap : 1, (u64)kEmitTile); }

void launch_merge_sorted_runs(const KeyCount* own, const KeyCount* recv, const u32* meta,
                              u64 cap, KeyCount* merged, MapCounters* ctr, OutRecord* out,
                              MapCounters* ctr_out, LookbackScratch lb, hipStream_t s) {
  launch_merge_view(RunsView{own, recv, meta, nullptr, 0, 0}, cap, merged, ctr, out, ctr_out, lb,
                    nullptr, s);
}

void launch_merge_slots(const KeyCount* slots, u32 nslots, u32 slot_records, KeyCount* merged,
                        MapCounters* ctr, OutRecord* out, MapCounters* ctr_out,
                        LookbackScratch lb, SlotHeader* hdr_out, hipStream_t s) {
  launch_merge_view(RunsView{nullptr, nullptr, nullptr, slots, nslots, slot_records},
                    (u64)nslots * slot_records, merged, ctr, out, ctr_out, lb, hdr_out, s);
}

}  // namespace locust
