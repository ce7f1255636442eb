// Kernels of the device-resident shuffle (locust/exch.hpp): plan (splitters + bucket
// offsets), pack (records -> fixed-pitch all-to-all slots), report (this rank's ExchMsg3)
// and emit (this rank's range -> the shared host output at its global offset, global val).
// The merge of the received slots is merge.hip's.  Every decision the round-1 driver made
// on the host between collectives (dist.cpp: choose_splitters, bucket_offsets, the count
// and total all-gathers) is taken here on the device, so the whole exchange is enqueued
// behind the map with no host round trip.
#include <algorithm>
#include <cstdlib>

#include "locust/device/wave.hpp"
#include "locust/exch.hpp"
#include "locust/hip_check.hpp"
#include "locust/kernels.hpp"

namespace locust {
namespace {

constexpr int kPlanBlock = 1024;

__device__ __forceinline__ bool key4_less(const u64* a, const u64* b) {
#pragma unroll
  for (int j = 0; j < kKeyWords; ++j)
    if (a[j] != b[j]) return a[j] < b[j];
  return false;
}

// ONE workgroup.  (1) every rank's status; (2) the P x S samples sorted in LDS by
// all-pairs ranks (stable); (3) weighted quantiles -> P-1 splitters: splitter p is the
// first sample (sorted) whose inclusive weight exceeds total * p / P, each sample of rank r
// weighing n_local(r) -- every rank computes the same from the same all-gathered bytes;
// (4) one wave per splitter: lower bound in this rank's sorted keys by a 64-ary search
// (64 probes per dependent load round instead of one), (5) bucket counts and flags.
__global__ __launch_bounds__(kPlanBlock) void exch_plan_kernel(
    const char* __restrict__ msg1_all, u32 P, u32 S, ConstKeysSoA keys,
    const u32* __restrict__ d_n, u32 slot_records, ExchCtl* __restrict__ ctl,
    u64* __restrict__ trace) {
  // trace (diagnostics, LOCUST_EXCH_TRACE): device clock at entry and after each phase
#define PLAN_STAMP(k_) \
  if (trace && threadIdx.x == 0) trace[k_] = __builtin_amdgcn_s_memrealtime()
  PLAN_STAMP(0);
  if (trace && threadIdx.x == 0) trace[7] = __builtin_amdgcn_s_memtime();  // shader clock
  __shared__ u64 s_k[kExchMaxPlanSamples][kKeyWords];
  __shared__ u64 s_w[kExchMaxPlanSamples];
  __shared__ u32 s_at[kExchMaxPlanSamples];  // sorted position -> sample
  __shared__ u32 s_unsorted;
  __shared__ u64 s_incl[kExchMaxPlanSamples];
  __shared__ u64 s_split[kExchMaxRanks][kKeyWords];
  __shared__ u64 s_off[kExchMaxRanks + 1];
  __shared__ u64 s_scan[kPlanBlock / 64 + 1];
  __shared__ u32 s_flags;
  __shared__ u64 s_maxb;
  const u32 t = threadIdx.x;
  const u64 mb = exch_msg1_bytes(S);
  const u32 NS = P * S;
  if (t == 0) {
    s_flags = (NS > kExchMaxPlanSamples || P > kExchMaxRanks) ? kExchTooManySamples : 0u;
    s_maxb = 0;
  }
  __syncthreads();
  if (t < P) {
    const ExchMsg1* h = reinterpret_cast<const ExchMsg1*>(msg1_all + (u64)t * mb);
    if (h->status) atomicOr(&s_flags, kExchAbort);
  }
  const bool fits = NS <= kExchMaxPlanSamples && P <= kExchMaxRanks;
  PLAN_STAMP(1);
  if (fits) {
    for (u32 i = t; i < NS; i += kPlanBlock) {
      const u32 r = i / S, q = i - r * S;
      const char* base = msg1_all + (u64)r * mb;
      const PackedKey* sp = reinterpret_cast<const PackedKey*>(base + sizeof(ExchMsg1));
#pragma unroll
      for (int j = 0; j < kKeyWords; ++j) s_k[i][j] = sp[q].w[j];
      s_w[i] = reinterpret_cast<const ExchMsg1*>(base)->n_local;
    }
  }
  __syncthreads();
  PLAN_STAMP(2);
  // Stable ranks (order: key, then rank, then index).  Every rank's samples arrive sorted
  // (picked at increasing positions of its sorted keys), so a sample's rank is its index in
  // its own list plus, per other list, a binary search: an upper bound in the lists before
  // its own, a lower bound in those after.  An all-pairs walk (one thread per sample over
  // all NS candidates) took 26 us at NS = 64 -- every step a dependent LDS load with a
  // divergent tie branch.  A list that is not sorted falls back to that walk.
  if (t == 0) s_unsorted = 0;
  __syncthreads();
  if (fits)
    for (u32 i = t; i < NS; i += kPlanBlock)
      if (i % S && key4_less(s_k[i], s_k[i - 1])) s_unsorted = 1;
  __syncthreads();
  if (fits && !s_unsorted) {
    for (u32 i = t; i < NS; i += kPlanBlock) {
      const u32 r = i / S;
      u64 ki[kKeyWords];
#pragma unroll
      for (int w = 0; w < kKeyWords; ++w) ki[w] = s_k[i][w];
      u32 rank = i - r * S;
      for (u32 rr = 0; rr < P; ++rr) {
        if (rr == r) continue;
        const u32 base = rr * S;
        u32 lo = 0, hi = S;
        while (lo < hi) {
          const u32 mid = (lo + hi) >> 1;
          const bool before = rr < r ? !key4_less(ki, s_k[base + mid])   // <= ki
                                     : key4_less(s_k[base + mid], ki);   // <  ki
          if (before) lo = mid + 1; else hi = mid;
        }
        rank += lo;
      }
      s_at[rank] = i;
    }
  } else if (fits) {
    for (u32 i = t; i < NS; i += kPlanBlock) {
      u32 rank = 0;
      for (u32 j = 0; j < NS; ++j) {
        const bool lt = key4_less(s_k[j], s_k[i]);
        rank += (lt || (j < i && !key4_less(s_k[i], s_k[j]))) ? 1u : 0u;
      }
      s_at[rank] = i;
    }
  }
  __syncthreads();
  PLAN_STAMP(3);
  // inclusive weight prefix in sorted order (NS <= kPlanBlock: one sample per thread)
  const u64 w = (fits && t < NS) ? s_w[s_at[t]] : 0ull;
  u64 total = 0;
  const u64 excl = dev::block_exclusive_scan<u64, kPlanBlock>(w, s_scan, &total);
  if (fits && t < NS) s_incl[t] = excl + w;
  __syncthreads();
  if (t >= 1 && t < P) {
    // splitter t-1: first sorted sample with inclusive weight > total * t / P
    const u64 target = fits ? total * t / P : 0;
    u32 lo = 0, hi = fits ? NS : 0;
    while (lo < hi) {
      const u32 mid = (lo + hi) >> 1;
      if (s_incl[mid] > target) hi = mid; else lo = mid + 1;
    }
#pragma unroll
    for (int j = 0; j < kKeyWords; ++j) s_split[t - 1][j] = lo < NS && fits ? s_k[s_at[lo]][j] : ~0ull;
  }
  __syncthreads();
  PLAN_STAMP(4);
  // bucket offsets: wave v searches splitters v, v + 16, ...
  const u32 n = *d_n;
  const int lane = dev::lane_id(), wv = dev::wave_id();
  for (u32 p = (u32)wv; p + 1 < P; p += kPlanBlock / 64) {
    u64 s[kKeyWords];
#pragma unroll
    for (int j = 0; j < kKeyWords; ++j) s[j] = s_split[p][j];
    u32 lo = 0, hi = n;  // the answer (first key >= s, or n) lies in [lo, hi]
    while (lo < hi) {
      const u32 step = (hi - lo + 63) / 64;
      const u32 pos = lo + (u32)lane * step;
      bool lt = false;
      if (pos < hi) {
        u64 k[kKeyWords];
#pragma unroll
        for (int j = 0; j < kKeyWords; ++j) k[j] = keys.w[j][pos];
        lt = key4_less(k, s);
      }
      const u64 b = dev::ballot(lt);
      const u32 cnt = (u32)__popcll(b);  // probes below s: a prefix of the lanes
      if (cnt == 0) {
        hi = lo;
      } else {
        const u32 last = lo + (cnt - 1) * step;  // key[last] < s
        const u32 nxt = lo + cnt * step;         // first probe >= s (if inside)
        lo = last + 1;
        if (nxt < hi) hi = nxt;
      }
    }
    if (lane == 0) s_off[p + 1] = lo;
  }
  if (t == 0) {
    s_off[0] = 0;
    s_off[P < kExchMaxRanks ? P : kExchMaxRanks] = n;
  }
  __syncthreads();
  if (t < P && P <= kExchMaxRanks) {
    const u64 c = s_off[t + 1] - s_off[t];
    atomicMax(reinterpret_cast<unsigned long long*>(&s_maxb), (unsigned long long)c);
    if (c > slot_records) atomicOr(&s_flags, kExchSendOverflow);
  }
  __syncthreads();
  PLAN_STAMP(5);
  for (u32 i = t; i <= P && i <= kExchMaxRanks; i += kPlanBlock) ctl->off[i] = s_off[i];
  if (t == 0) {
    ctl->flags = s_flags;
    ctl->max_bucket = s_maxb;
  }
  PLAN_STAMP(6);
  if (trace && threadIdx.x == 0) trace[8] = __builtin_amdgcn_s_memtime();
#undef PLAN_STAMP
}

// Records -> the P all-to-all slots: record i of bucket d goes to slot d position
// i - off[d] (buckets are contiguous in the sorted records); block 0 writes the headers.
__global__ __launch_bounds__(256) void exch_pack_kernel(const KeyCount* __restrict__ recs,
                                                        const u32* __restrict__ d_n,
                                                        const ExchCtl* __restrict__ ctl, u32 P,
                                                        u32 slot_records, char* __restrict__ send) {
  __shared__ u64 s_off[kExchMaxRanks + 1];
  for (u32 i = threadIdx.x; i <= P; i += 256) s_off[i] = ctl->off[i];
  const u32 flags = ctl->flags;
  __syncthreads();
  const u64 sb = exch_slot_bytes(slot_records);
  if (blockIdx.x == 0 && threadIdx.x < P) {
    const u32 d = threadIdx.x;
    const u64 c = s_off[d + 1] - s_off[d];
    SlotHeader h{};
    h.status = (flags & (kExchAbort | kExchTooManySamples)) ? kSlotFailed
               : c > slot_records                           ? kSlotRedo
                                                            : kSlotOk;
    h.record_flags = 3u;  // sorted, distinct (ShardEngine::kRecordsSorted | kRecordsDistinct)
    h.n = c;
    h.slot_cap = slot_records;
    *reinterpret_cast<SlotHeader*>(send + (u64)d * sb) = h;
  }
  if (flags & (kExchAbort | kExchTooManySamples)) return;
  const u32 n = *d_n;
  for (u32 i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    u32 lo = 0, hi = P;  // last d with off[d] <= i
    while (hi - lo > 1) {
      const u32 mid = (lo + hi) >> 1;
      if (s_off[mid] <= i) lo = mid; else hi = mid;
    }
    const u64 j = i - s_off[lo];
    if (j < slot_records) {
      KeyCount* dst = reinterpret_cast<KeyCount*>(send + (u64)lo * sb) + kSlotHeaderRecords;
      dst[j] = recs[i];
    }
  }
}

// This rank's report: flags (own plan + any truncated / failed incoming slot + a range
// larger than the gather slot), largest bucket, range size and token total.
__global__ __launch_bounds__(64) void exch_report_kernel(const char* __restrict__ recv, u32 P,
                                                         u32 slot_records,
                                                         const ExchCtl* __restrict__ ctl,
                                                         u64* __restrict__ acc,
                                                         u32 gather_records,
                                                         ExchMsg3* __restrict__ msg3) {
  static_assert(kMergeAccSpread == 64, "one accumulator triple per lane");
  const u64 sb = exch_slot_bytes(slot_records);
  bool bad = false;
  for (u32 q = threadIdx.x; q < P; q += 64) {
    const SlotHeader* h = reinterpret_cast<const SlotHeader*>(recv + (u64)q * sb);
    bad |= h->status != kSlotOk || h->n > slot_records;
  }
  const u64 any = dev::ballot(bad);
  // the merge's range: its (firsts, tokens, words) triples, then zeroed for the next job
  const u64 n_range = dev::wave_reduce_sum(acc[3 * threadIdx.x]);
  const u64 tok_range = dev::wave_reduce_sum(acc[3 * threadIdx.x + 1]);
  const u64 words_range = dev::wave_reduce_sum(acc[3 * threadIdx.x + 2]);
  acc[3 * threadIdx.x] = 0;
  acc[3 * threadIdx.x + 1] = 0;
  acc[3 * threadIdx.x + 2] = 0;
  if (threadIdx.x == 0) {
    ExchMsg3 m{};
    const u32 cf = ctl->flags;
    const u64 n_out = (cf & (kExchAbort | kExchTooManySamples)) ? 0 : n_range;
    m.status = 0;
    m.flags = cf | (any ? kExchRecvTruncated : 0u) | (n_out > gather_records ? kExchGatherOverflow : 0u);
    m.max_bucket = ctl->max_bucket;
    m.n_out = n_out;
    m.total = (cf & (kExchAbort | kExchTooManySamples)) ? 0 : tok_range;
    m.out_words = (cf & (kExchAbort | kExchTooManySamples)) ? 0 : words_range;
    *msg3 = m;
  }
}

// The header, and (S > 0) the S samples behind it in the same launch: one dependent
// launch less between the ordered kernel and the all-gather (each is ~4.7 us on the
// exchange's critical path, profiles/r4/kexch_v2.summary.txt).
__global__ void exch_header_kernel(const MapCounters* __restrict__ ctr, ExchMsg1 h,
                                   u32 combined, ExchMsg1* __restrict__ out, ConstKeysSoA sorted,
                                   const u32* __restrict__ d_n, u32 S) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    if (!h.status && (ctr->flags & kCtrDictOverflow)) h.status = kExchMapRedo;
    h.n_local = h.status ? 0 : ctr->num_unique;
    h.tokens = combined ? ctr->map_tokens : ctr->num_records;
    h.overflow_lines = ctr->overflow_lines;
    h.truncated = ctr->truncated;
    h.max_key_len = ctr->max_key_len;
    *out = h;
  }
  if (!S) return;
  // sample[k] = keys[floor((k + 0.5) n / S)], "+inf" for an empty shard (launch_sample_keys)
  PackedKey* smp = reinterpret_cast<PackedKey*>(out + 1);
  const u32 n = *d_n;
  for (u32 k = blockIdx.x * blockDim.x + threadIdx.x; k < S; k += gridDim.x * blockDim.x) {
    PackedKey q;
    const u64 i = n ? ((2ull * k + 1) * n) / (2ull * S) : 0;
#pragma unroll
    for (int w = 0; w < kKeyWords; ++w) q.w[w] = n ? sorted.w[w][i] : ~0ull;
    smp[k] = q;
  }
}

}  // namespace

void launch_exch_header(const MapCounters* ctr, const ExchMsg1& tmpl, bool combined,
                        ExchMsg1* out, hipStream_t s, ConstKeysSoA sorted, const u32* d_n,
                        u32 num_samples) {
  LOCUST_CHECK_ARG(!num_samples || d_n, "exchange header: samples need the key count");
  exch_header_kernel<<<dim3(std::max<u32>(1u, (num_samples + 63) / 64)), dim3(64), 0, s>>>(
      ctr, tmpl, combined ? 1u : 0u, out, sorted, d_n, num_samples);
  LOCUST_HIP_LAUNCH_CHECK();
}

void launch_exch_plan(const char* msg1_all, u32 P, u32 S, ConstKeysSoA keys, const u32* d_n,
                      u32 slot_records, ExchCtl* ctl, hipStream_t s, u64* trace) {
  exch_plan_kernel<<<dim3(1), dim3(kPlanBlock), 0, s>>>(msg1_all, P, S, keys, d_n, slot_records,
                                                         ctl, trace);
  LOCUST_HIP_LAUNCH_CHECK();
}

void launch_exch_pack(const KeyCount* recs, const u32* d_n, u64 cap, const ExchCtl* ctl, u32 P,
                      u32 slot_records, char* send, hipStream_t s) {
  const u64 blocks = std::min<u64>(std::max<u64>(div_up(cap ? cap : 1, 256), 1), 4096);
  exch_pack_kernel<<<dim3((u32)blocks), dim3(256), 0, s>>>(recs, d_n, ctl, P, slot_records, send);
  LOCUST_HIP_LAUNCH_CHECK();
}

void launch_exch_report(const char* recv, u32 P, u32 slot_records, const ExchCtl* ctl,
                        u64* acc, u32 gather_records, ExchMsg3* msg3, hipStream_t s) {
  exch_report_kernel<<<dim3(1), dim3(64), 0, s>>>(recv, P, slot_records, ctl, acc,
                                                   gather_records, msg3);
  LOCUST_HIP_LAUNCH_CHECK();
}

// Loads this file's code object (one module per file) now rather than at its first launch.
void warm_module_exchange() {
  hipFuncAttributes a;
  (void)hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&exch_header_kernel));
}

}  // namespace locust
