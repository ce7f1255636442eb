// Root merge of the gather strategy: P sorted runs of combined (key, count) records -> the
// globally sorted (key, count) output, in two short kernels.
//
// The reference has no merge at all: its reducer expects one pre-sorted /tmp/out.txt
// (main.cu:437-465, bug B7), and the cross-node transfer that would feed it is missing
// (README.md:24).  Here every rank's combined output arrives sorted, so the root does not
// rebuild a dictionary over them; it merges:
//
//   merge_rank   eight threads per record, one per other run: a galloping search in that
//                run gives the record's position in the stable (key, run) merge order, whether
//                a lower run already holds the key (then this copy is a duplicate), and --
//                for the first copy -- the key's total count over all runs; the group sums
//                its parts by shuffles.  Records are scattered to their merged slots
//                (duplicates with count 0).
//   merge_emit   decoupled look-back scan over the merged slots of (#first copies, count
//                sum): the first copies are compacted into the output (the reference's
//                val, the exclusive prefix of the counts -- start index of the key's run
//                in the globally sorted token array, main.cu:161-208 -- is rebuilt on the
//                host) and the token total comes from the scan.
//
// Runs are at most 64 (one per rank); the output goes straight into host-mapped memory.
// The search is latency bound (one dependent load per step): a thread per record searching
// all runs in turn took 41-49 us at 8 runs of ~1.5-5.6 K records, a thread per (record,
// run) 8-12 us -- eight times the waves to overlap the probe chains -- and galloping from
// the record's scaled position 9 us (profiles/r1_s4).
#include "locust/device/lookback.hpp"
#include "locust/hip_check.hpp"
#include "locust/kernels.hpp"

namespace locust {
namespace {

constexpr int kMergeBlock = 256;
constexpr int kMergeSub = 8;                          // threads per record (runs in flight)
constexpr int kEmitItems = 4;                          // merged slots per thread
constexpr int kEmitTile = kMergeBlock * kEmitItems;    // 1,024 slots: 48 KB of LDS staging
constexpr int kEmitCountBits = 40;                     // look-back value: [firsts:22][counts:40]
constexpr u64 kEmitCountMask = (1ull << kEmitCountBits) - 1;

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

// Wave 0 builds the run table: lane q reads run q's length (all loads in flight at once --
// a one-thread loop would pay a memory round trip per run) and a wave scan gives offsets.
__device__ __forceinline__ void load_runs(const RunsView& v, RunTable& t) {
  static_assert(kMaxMergeRunsHost <= 64, "one lane per run");
  if (threadIdx.x < 64) {
    const u32 q = threadIdx.x;
    u32 nr, len = 0;
    const KeyCount* base = nullptr;
    if (v.slots) {
      nr = min(v.nslots, (u32)kMaxMergeRunsHost);
      const u64 stride = (u64)kSlotHeaderRecords + v.slot_records;
      if (q < nr) {
        const KeyCount* slot = v.slots + q * stride;
        const SlotHeader* h = reinterpret_cast<const SlotHeader*>(slot);
        const u32 status = h->status;
        const u64 n = h->n;
        len = status == kSlotOk ? (u32)min(n, (u64)v.slot_records) : 0u;
        base = slot + kSlotHeaderRecords;
      }
    } else {
      nr = min(v.meta[0], (u32)kMaxMergeRunsHost);
      if (q < nr) len = v.meta[1 + q];
    }
    const u32 incl = dev::wave_inclusive_scan(len);
    const u32 excl = incl - len;
    if (!v.slots && q < nr) base = q == 0 ? v.own : v.recv + (excl - v.meta[1]);  // back to back
    if (q < nr) {
      t.off[q] = excl;
      t.base[q] = base;
    }
    if (q + 1 == max(nr, 1u)) {
      t.off[nr] = nr ? incl : 0u;
      t.nruns = nr;
    }
  }
  __syncthreads();
}

// Lower bound of key k in one sorted run in global memory (rlen >= 1), on the first key word
// (one load per step), then the landing record loaded whole; keys sharing their first word
// with k but smaller walk on (rare).  Returns the position; *eq / *cnt: whether the record
// there equals k, and its count.
//
// The search gallops from `hint` (the record's relative position in its own run, scaled
// to this run): runs of similar key distributions -- every rank's combined output of the
// same kind of text -- put the answer within a few records of it, found in 2-4 dependent
// loads instead of log2(rlen) ~ 13; far off, the doubling steps cost at most about twice
// a plain binary search.
__device__ __forceinline__ u32 run_lower_bound(const KeyCount* __restrict__ run, u32 rlen,
                                               u32 hint, const u64* k, bool* eq, u64* cnt) {
  // bracket the first position whose word >= k[0] in [lo, lo + len] by doubling steps
  u32 lo, len;
  if (run[hint].w[0] < k[0]) {  // answer > hint
    u32 step = 1;
    lo = hint + 1;
    while (lo + step - 1 < rlen && run[lo + step - 1].w[0] < k[0]) {
      lo += step;
      step <<= 1;
    }
    len = min(lo + step - 1, rlen) - lo;
  } else {  // answer <= hint
    u32 hi = hint, step = 1;
    while (hi >= step && run[hi - step].w[0] >= k[0]) {
      hi -= step;
      step <<= 1;
    }
    lo = hi >= step ? hi - step + 1 : 0;
    len = hi - lo;
  }
  while (len) {
    const u32 half = len >> 1;
    const bool lt = run[lo + half].w[0] < k[0];
    lo = lt ? lo + half + 1 : lo;
    len = lt ? len - half - 1 : half;
  }
  *eq = false;
  *cnt = 0;
  for (; lo < rlen; ++lo) {
    const KeyCount c = run[lo];
    if (c.w[0] != k[0]) break;
    const int cmp = c.w[1] != k[1] ? (c.w[1] < k[1] ? -1 : 1)
                  : c.w[2] != k[2] ? (c.w[2] < k[2] ? -1 : 1)
                  : c.w[3] != k[3] ? (c.w[3] < k[3] ? -1 : 1) : 0;
    if (cmp >= 0) {
      *eq = cmp == 0;
      *cnt = c.count;
      break;
    }
  }
  return lo;
}

// kMergeSub threads per record, one per run of a group of kMergeSub runs: 8x the waves of a
// thread-per-record search, so the dependent probe chains of many records overlap.
// acc (optional, zeroed): the merge's distinct keys, token total and compact-record words
// -- the shuffle tail reports them before anything is emitted -- as kMergeAccSpread
// (firsts, tokens, words) triples: block b adds its sums to triple b % kMergeAccSpread (one same-address atomic per block
// serialised ~25K wave atomics at the memory side: 0.4 ms per job at synth1m scale).
__global__ __launch_bounds__(kMergeBlock) void merge_rank_kernel(
    RunsView view, KeyCount* __restrict__ merged, LookbackScratch lb, u32 emit_tiles,
    SlotHeader* __restrict__ hdr_out, u64* __restrict__ acc) {
  __shared__ u64 s_acc[3 * (kMergeBlock / 64)];
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
  const u64 work = (u64)t.off[nruns] * kMergeSub;
  const u32 sub = threadIdx.x % kMergeSub;
  u32 my_firsts = 0;  // (acc) first copies this thread emitted, their counts and the
  u64 my_tokens = 0;  // words of their compact records (what the emit writes to the host)
  u64 my_words = 0;
  // whole groups of kMergeSub lanes enter or leave the loop together (shuffles below)
  for (u64 gt = (u64)blockIdx.x * kMergeBlock + threadIdx.x; gt < work;
       gt += (u64)gridDim.x * kMergeBlock) {
    const u32 g = (u32)(gt / kMergeSub);
    u32 q = 0;
    while (q + 1 < nruns && t.off[q + 1] <= g) ++q;
    const u32 i = g - t.off[q];
    const KeyCount rec = t.base[q][i];  // the same address for the whole group
    const u64 k[kKeyWords] = {rec.w[0], rec.w[1], rec.w[2], rec.w[3]};
    u32 before = 0;   // records of other runs ordered before this one
    u32 dup = 0;      // a lower run holds the key: this copy is not the first
    u64 others = 0;   // counts of the key in higher runs
    for (u32 r = sub; r < nruns; r += kMergeSub) {
      const u32 rlen = t.off[r + 1] - t.off[r];
      if (r == q || !rlen) continue;
      bool eq;
      u64 cnt;
      const u32 own = t.off[q + 1] - t.off[q];
      const u32 hint = (u32)min((u64)i * rlen / own, (u64)rlen - 1);
      const u32 lo = run_lower_bound(t.base[r], rlen, hint, k, &eq, &cnt);
      if (r < q) {
        before += lo + (eq ? 1 : 0);  // equal keys of lower runs come first
        dup |= eq ? 1u : 0u;
      } else {
        before += lo;
        others += eq ? cnt : 0;
      }
    }
#pragma unroll
    for (int m = 1; m < kMergeSub; m <<= 1) {
      before += __shfl_xor(before, m, kMergeSub);
      dup |= __shfl_xor(dup, m, kMergeSub);
      others += __shfl_xor(others, m, kMergeSub);
    }
    if (sub == 0) {
      KeyCount out;
#pragma unroll
      for (int j = 0; j < kKeyWords; ++j) out.w[j] = k[j];
      out.count = dup ? 0 : rec.count + others;  // later copies of a key carry nothing
      merged[(u64)i + before] = out;
      my_firsts += dup ? 0u : 1u;
      my_tokens += out.count;
      my_words += dup ? 0u : compact_words(out.w, out.count);
    }
  }
  if (acc) {  // uniform: every thread of the block gets here
    const u64 f = dev::wave_reduce_sum((u64)my_firsts);
    const u64 tk = dev::wave_reduce_sum(my_tokens);
    const u64 wd = dev::wave_reduce_sum(my_words);
    if (dev::lane_id() == 0) {
      s_acc[3 * dev::wave_id()] = f;
      s_acc[3 * dev::wave_id() + 1] = tk;
      s_acc[3 * dev::wave_id() + 2] = wd;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      u64 bf = 0, bt = 0, bw = 0;
#pragma unroll
      for (int w = 0; w < kMergeBlock / 64; ++w) {
        bf += s_acc[3 * w];
        bt += s_acc[3 * w + 1];
        bw += s_acc[3 * w + 2];
      }
      if (bf) {
        u64* a = acc + 3 * (blockIdx.x % kMergeAccSpread);
        atomicAdd(reinterpret_cast<unsigned long long*>(a), (unsigned long long)bf);
        atomicAdd(reinterpret_cast<unsigned long long*>(a + 1), (unsigned long long)bt);
        atomicAdd(reinterpret_cast<unsigned long long*>(a + 2), (unsigned long long)bw);
      }
    }
  }
}

// The shuffle tail's emit: this rank's merged key range straight from
// the merge slots into the shared host output as compact records (kv.hpp), at word
// kOutWords x (the region's first record + the lower ranks' records) -- rank p's segment
// starts where its 40-B records would have, so the root needs only the all-gathered
// counts.  Per tile: the first copies' sizes, a block scan and a look-back over the words
// give each record's offset; the tile is staged in LDS and written with consecutive lanes
// on consecutive words.  Every workgroup fences at system scope and counts itself done;
// the last stores `seq` into this rank's stamp (locust/shm.hpp).
__global__ __launch_bounds__(kMergeBlock) void merge_emit_compact_kernel(
    const KeyCount* __restrict__ merged, RunsView view, const ExchMsg3* __restrict__ msg3_all,
    const ExchMsg1* __restrict__ root_msg, u64 region, u32 regions, u64 region_records, u32 P,
    u32 me, u32 gather_records, u64* __restrict__ dst, u64* __restrict__ stamps, u64 seq,
    u32* __restrict__ done, u64* __restrict__ status, u32* __restrict__ tile_ctr) {
  __shared__ u64 s_scan[kMergeBlock / 64 + 1];
  __shared__ u32 s_tile, s_bad;
  __shared__ u64 s_prefix, s_base;
  __shared__ RunTable t;
  __shared__ __attribute__((aligned(16))) u64 s_out[kEmitTile * kOutWords];
  if (threadIdx.x == 0) {
    // the region: the host's, or the one the root announced in its all-gathered header
    if (root_msg) region = root_msg->out_region;
    u64 r = 0;
    u32 bad = 0;
    for (u32 q = 0; q < P && q < kExchMaxRanks; ++q) {
      const ExchMsg3 m = msg3_all[q];
      bad |= (u32)m.status | m.flags;
      if (q < me) r += m.n_out <= gather_records ? m.n_out : gather_records;
    }
    const u64 n = msg3_all[me].n_out;
    // a failed or overflowing job, no free region (the host grows the output and emits
    // again) or a range past its region: write nothing, stamp nothing
    s_bad = bad | (n > gather_records || region >= regions || r + n > region_records ? 1u : 0u);
    s_base = (u64)kOutWords * (region * region_records + r);
  }
  __syncthreads();
  if (s_bad) return;  // uniform over the grid: the host sees the reports
  const u32 tile = dev::acquire_tile(tile_ctr, &s_tile);
  load_runs(view, t);
  const u32 total = t.off[t.nruns];
  const u32 ntiles = total ? (u32)div_up(total, (u64)kEmitTile) : 1u;
  if (tile < ntiles) {  // uniform per workgroup; nobody waits on tiles past the end
    const u32 i0 = tile * kEmitTile + threadIdx.x * kEmitItems;
    KeyCount v[kEmitItems];
    u32 nw[kEmitItems];
    u64 words = 0;
#pragma unroll
    for (int e = 0; e < kEmitItems; ++e) {
      const u32 i = i0 + e;
      v[e].count = 0;
      if (i < total) v[e] = merged[i];
      nw[e] = v[e].count ? compact_words(v[e].w, v[e].count) : 0u;
      words += nw[e];
    }
    u64 tile_words = 0;
    u64 at = dev::block_exclusive_scan<u64, kMergeBlock>(words, s_scan, &tile_words);
    const u64 before = dev::block_lookback(status, tile, tile_words, &s_prefix);
#pragma unroll
    for (int e = 0; e < kEmitItems; ++e) {
      if (!v[e].count) continue;
      u64* o = s_out + at;
      u64 rec[kCompactMaxWords];
      (void)compact_record(v[e].w, v[e].count, rec);
#pragma unroll
      for (u32 j = 0; j < (u32)kCompactMaxWords; ++j)  // static indices: registers, no scratch
        if (j < nw[e]) o[j] = rec[j];
      at += nw[e];
    }
    __syncthreads();
    u64* out = dst + s_base + before;
    for (u32 q = threadIdx.x; q < (u32)tile_words; q += kMergeBlock) out[q] = s_out[q];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    // this workgroup's records (host memory): one system-scope release, not an acq_rel
    // fence in every thread
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    const u32 prev = atomicAdd(done, 1u);
    if (prev == gridDim.x - 1) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // every workgroup's records
      *done = 0u;  // the next job's launch is stream-ordered behind this one
      __hip_atomic_store(stamps + me, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

__global__ __launch_bounds__(kMergeBlock) void merge_emit_kernel(
    const KeyCount* __restrict__ merged, RunsView view, MapCounters* __restrict__ ctr,
    OutRecord* __restrict__ out, MapCounters* __restrict__ ctr_out, u64* __restrict__ status,
    u32* __restrict__ tile_ctr, u64 out_limit) {
  __shared__ u64 s_scan[kMergeBlock / 64 + 1];
  __shared__ u32 s_tile;
  __shared__ u64 s_prefix;
  __shared__ RunTable t;
  // the tile's output records, staged so that the (host-mapped) writes are full lines
  __shared__ __attribute__((aligned(16))) u64 s_out[kEmitTile * kOutWords];
  // a ticket, not blockIdx: a tile only waits on tiles already running (see
  // dict_ordered_kernel: kernels of processes sharing a GPU could otherwise deadlock)
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
#pragma unroll
  for (int e = 0; e < kEmitItems; ++e) {
    if (!v[e].count) continue;
    u64* o = s_out + kOutWords * li;
#pragma unroll
    for (int j = 0; j < kKeyWords; ++j) o[j] = v[e].w[j];
    o[4] = v[e].count;
    ++li;
  }
  __syncthreads();
  const u32 m = (u32)(tile_sum >> kEmitCountBits);
  const u64 base = before >> kEmitCountBits;
  // consecutive lanes, consecutive 8-B words of out[base .. base + m), at most
  // out_limit records in all (the exchange's fixed gather slot: the count still says how
  // many there were, and the report flags the overflow)
  const u32 mw = base >= out_limit ? 0u : (u32)min((u64)m, out_limit - base);
  u64* dst = reinterpret_cast<u64*>(out + base);
  for (u32 q = threadIdx.x; q < kOutWords * mw; q += kMergeBlock) dst[q] = s_out[q];
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
                       SlotHeader* hdr_out, hipStream_t s, u64 out_limit = ~0ull) {
  const u64 c = cap ? cap : 1;
  const u32 rank_grid = (u32)std::min<u64>(div_up(c * kMergeSub, kMergeBlock), 8192);
  const u32 emit_grid = (u32)div_up(c, (u64)kEmitTile);
  merge_rank_kernel<<<dim3(rank_grid), dim3(kMergeBlock), 0, s>>>(v, merged, lb, emit_grid,
                                                                  hdr_out, nullptr);
  LOCUST_HIP_LAUNCH_CHECK();
  merge_emit_kernel<<<dim3(emit_grid), dim3(kMergeBlock), 0, s>>>(merged, v, ctr, out, ctr_out,
                                                                  lb.status, lb.tile_counter,
                                                                  out_limit);
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

void launch_merge_rank_slots(const KeyCount* slots, u32 nslots, u32 slot_records,
                             KeyCount* merged, u64* acc, LookbackScratch lb, hipStream_t s) {
  const RunsView v{nullptr, nullptr, nullptr, slots, nslots, slot_records};
  const u64 c = std::max<u64>((u64)nslots * slot_records, 1);
  const u32 rank_grid = (u32)std::min<u64>(div_up(c * kMergeSub, kMergeBlock), 8192);
  merge_rank_kernel<<<dim3(rank_grid), dim3(kMergeBlock), 0, s>>>(
      v, merged, lb, (u32)div_up(c, (u64)kEmitTile), nullptr, acc);
  LOCUST_HIP_LAUNCH_CHECK();
}

void launch_merge_emit_compact(const KeyCount* slots, u32 nslots, u32 slot_records,
                               const KeyCount* merged, const ExchMsg3* msg3_all,
                               const ExchMsg1* root_msg, u64 region, u32 regions,
                               u64 region_records, u32 P, u32 me, u32 gather_records, u64* dst,
                               u64* stamps, u64 seq, u32* done, LookbackScratch lb,
                               hipStream_t s) {
  const RunsView v{nullptr, nullptr, nullptr, slots, nslots, slot_records};
  const u64 c = std::max<u64>((u64)nslots * slot_records, 1);
  // tiles past this rank's merged slots exit at once (their count still completes the grid)
  const u32 grid = (u32)div_up(c, (u64)kEmitTile);
  merge_emit_compact_kernel<<<dim3(grid), dim3(kMergeBlock), 0, s>>>(
      merged, v, msg3_all, root_msg, region, regions, region_records, P, me, gather_records, dst,
      stamps, seq, done, lb.status, lb.tile_counter);
  LOCUST_HIP_LAUNCH_CHECK();
}

// Loads this file's code object (one module per file) now rather than at its first launch.
void warm_module_merge() {
  hipFuncAttributes a;
  (void)hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&merge_rank_kernel));
}

}  // namespace locust
