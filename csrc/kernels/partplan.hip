// In-job partition map of a large single pass (the two-kernel ordered build, dict.hip):
// the map's key ranges chosen from THIS job's text instead of the previous job's output.
//
// The reference has no counterpart (one comparison sort over every record,
// /root/reference/MapReduce/src/main.cu:414-415).  Here each of the kDictParts workgroups
// of the partials and ordered kernels owns one key range, and a range's distinct keys
// must fit one workgroup's 2,048-slot LDS table.  A first-byte map puts ~17K distinct keys
// into one letter of a 200K-word vocabulary; the engine then falls back to an HBM table
// (a 10x slower job).  So before the first upload piece is mapped, the engine maps a
// line-aligned prefix of it (<= 1 MiB) into scratch, deduplicates its keys in an HBM
// hash table (dict_insert_kernel) and this kernel cuts the key space at equal weights of
// those distinct keys: every range gets ~1/256 of the estimated vocabulary of the whole
// pass, the measure that bounds the LDS tables.  Hot words stay cheap anyway: the
// combining map folds their repeats per tile.
#include "locust/device/wave.hpp"
#include "locust/hip_check.hpp"
#include "locust/kernels.hpp"

namespace locust {
namespace {

constexpr int kPlanBlock = 1024;
// Sizing, from an offline replay of the plan on the generator's 1M-line text (fullest range
// of the whole pass, in distinct keys; the mean is 792): 2,048 samples of a 512 KiB prefix
// 3,100 (sampling noise, ~8 samples per range); 8,192 1,800; 8,192 of a 1 MiB prefix,
// singletons weighted 9x, 1,768 -- the setting here; 16,384 of 1.5 MiB 1,477, but the
// larger sample and sort cost ~0.4 ms of compute in front of the first piece's map.
constexpr u32 kPlanSamples = 8192;
constexpr u32 kPlanPer = kPlanSamples / kPlanBlock;
// A key the prefix saw once (a hapax) stands for the rare keys of the whole pass the prefix
// has not seen yet (Good-Turing): it weighs kSingletonWeight, a repeated key 1.
constexpr u32 kSingletonWeight = 9;

// One workgroup: kPlanSamples of the U distinct keys (dense, in hash-arrival order -- no
// key order) with their weights, bitonic-sorted in LDS by first word (72 KB); range q
// starts at the sample holding the q/256 quantile of the weights.
__global__ __launch_bounds__(kPlanBlock) void part_plan_kernel(const u64* __restrict__ w0,
                                                               const u64* __restrict__ count,
                                                               const u32* __restrict__ d_u,
                                                               u32 ucap,
                                                               PartMapTables* __restrict__ out) {
  __shared__ u64 s_k[kPlanSamples];
  __shared__ u8 s_w[kPlanSamples];
  __shared__ u32 s_scan[kPlanBlock / 64 + 1];
  const u32 U = min(*d_u, ucap);
  const u32 S = U < kPlanSamples ? U : kPlanSamples;
#pragma unroll
  for (u32 r = 0; r < kPlanPer; ++r) {
    const u32 i = threadIdx.x + r * kPlanBlock;
    u64 k = ~0ull;  // padding sorts last, weight 0
    u8 w = 0;
    if (i < S) {
      const u64 idx = (u64)i * U / S;
      k = w0[idx];
      w = count[idx] == 1 ? (u8)kSingletonWeight : (u8)1;
    }
    s_k[i] = k;
    s_w[i] = w;
  }
  __syncthreads();
  for (u32 k = 2; k <= kPlanSamples; k <<= 1) {
    for (u32 j = k >> 1; j > 0; j >>= 1) {
      // kPlanSamples / 2 compare-exchange pairs per stage, kPlanPer / 2 per thread: pair
      // c = (i with bit j clear) -- no idle half of the threads
#pragma unroll
      for (u32 r = 0; r < kPlanPer / 2; ++r) {
        const u32 c = threadIdx.x + r * kPlanBlock;
        const u32 i = ((c & ~(j - 1)) << 1) | (c & (j - 1)), l = i | j;
        const u64 a = s_k[i], b = s_k[l];
        if ((a > b) == ((i & k) == 0)) {
          s_k[i] = b;
          s_k[l] = a;
          const u8 t = s_w[i];
          s_w[i] = s_w[l];
          s_w[l] = t;
        }
      }
      __syncthreads();
    }
  }
  // weight prefix of this thread's kPlanPer consecutive samples
  u32 mine = 0;
#pragma unroll
  for (u32 r = 0; r < kPlanPer; ++r) mine += s_w[threadIdx.x * kPlanPer + r];
  u32 W = 0;
  u32 pre = dev::block_exclusive_scan<u32, kPlanBlock>(mine, s_scan, &W);
  if (threadIdx.x == 0) {
    out->lo[0] = 0;
    out->lo[kDictParts] = ~0ull;
  }
  if (W == 0) {  // nothing sampled: the default (first byte)
    for (u32 q = 1 + threadIdx.x; q < (u32)kDictParts; q += kPlanBlock) out->lo[q] = (u64)q << 56;
    return;
  }
  // sample e covers weight [pre_e, pre_e + w_e): it starts every range q whose quantile
  // q * W / 256 falls in it -- each q in 1..255 exactly once
#pragma unroll
  for (u32 r = 0; r < kPlanPer; ++r) {
    const u32 e = threadIdx.x * kPlanPer + r, w = s_w[e];
    const u32 qa = (u32)((u64)pre * kDictParts / W), qb = (u32)((u64)(pre + w) * kDictParts / W);
    for (u32 q = qa + 1; q <= qb; ++q)
      if (q < (u32)kDictParts) out->lo[q] = s_k[e];
    pre += w;
  }
}

}  // namespace

void launch_part_plan(const u64* ukeys_w0, const u64* ucount, const u32* d_u, u32 ucap,
                      PartMapTables* out, hipStream_t s) {
  part_plan_kernel<<<dim3(1), dim3(kPlanBlock), 0, s>>>(ukeys_w0, ucount, d_u, ucap, out);
  LOCUST_HIP_LAUNCH_CHECK();
}

// Loads this file's code object (one module per file) now rather than at its first launch.
void warm_module_partplan() {
  hipFuncAttributes a;
  (void)hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&part_plan_kernel));
}

}  // namespace locust
