// Shuffle kernels for the multi-GPU WordCount.
//
// The reference has no data plane: mappers write /tmp/out.txt and the transfer to
// reducers is missing (main.cu:428-441, README.md:24).  Its design (img/MapReduce.gif)
// routes keys to reducers by first letter.  Here each GPU range-partitions its locally
// sorted records by sample-sort splitters (so every bucket is a contiguous slice and rank
// order == key order), packs them as 40-B KeyCount records and exchanges them with one
// RCCL all-to-all-v over xGMI.
#include "locust/device/hash.hpp"
#include "locust/hip_check.hpp"
#include "locust/kernels.hpp"

namespace locust {
namespace {

u32 grid_for(u64 n, u32 block, u32 max_blocks = 2048) {
  u64 b = div_up(n ? n : 1, block);
  return (u32)(b > max_blocks ? max_blocks : b);
}

__global__ __launch_bounds__(256) void pack_records_kernel(ConstKeysSoA keys,
                                                           const u64* __restrict__ counts,
                                                           const u32* __restrict__ d_n,
                                                           KeyCount* __restrict__ out) {
  const u32 n = *d_n;
  for (u32 i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    KeyCount r;
#pragma unroll
    for (int w = 0; w < kKeyWords; ++w) r.w[w] = keys.w[w][i];
    r.count = counts ? counts[i] : 1;
    out[i] = r;
  }
}

__global__ __launch_bounds__(256) void unpack_records_kernel(const KeyCount* __restrict__ in,
                                                             u64 n, KeysSoA keys,
                                                             u64* __restrict__ counts,
                                                             u8* __restrict__ parts, PartMap pm) {
  for (u64 i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
    const KeyCount r = in[i];
#pragma unroll
    for (int w = 0; w < kKeyWords; ++w) keys.w[w][i] = r.w[w];
    counts[i] = r.count;
    if (parts) parts[i] = (u8)part_of(pm, r.w[0]);  // see PartMap / launch_dict_ordered
  }
}

// Sorted output records (from the ordered dictionary kernel) -> SoA sorted keys + counts
// (for sampling and the splitter search) and the 40-B shuffle records.
__global__ void sample_keys_kernel(ConstKeysSoA sorted, const u32* __restrict__ d_n, u32 s,
                                   PackedKey* __restrict__ out) {
  const u32 n = *d_n;
  for (u32 k = blockIdx.x * blockDim.x + threadIdx.x; k < s; k += gridDim.x * blockDim.x) {
    PackedKey p;
    if (n == 0) {
      for (int w = 0; w < kKeyWords; ++w) p.w[w] = ~0ull;  // "+inf": sorts after every key
    } else {
      const u64 i = ((2ull * k + 1) * n) / (2ull * s);
      for (int w = 0; w < kKeyWords; ++w) p.w[w] = sorted.w[w][i];
    }
    out[k] = p;
  }
}

__device__ __forceinline__ bool less_than(ConstKeysSoA a, u64 i, const PackedKey& b) {
#pragma unroll
  for (int w = 0; w < kKeyWords; ++w) {
    const u64 x = a.w[w][i];
    if (x != b.w[w]) return x < b.w[w];
  }
  return false;
}

__global__ void bucket_offsets_kernel(ConstKeysSoA sorted, const u32* __restrict__ d_n,
                                      const PackedKey* __restrict__ splitters, u32 num_buckets,
                                      u64* __restrict__ offsets) {
  const u32 n = *d_n;
  const u32 p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p > num_buckets) return;
  if (p == 0) {
    offsets[0] = 0;
    return;
  }
  if (p == num_buckets) {
    offsets[p] = n;
    return;
  }
  const PackedKey sp = splitters[p - 1];
  u64 lo = 0, hi = n;  // first index with key >= splitter
  while (lo < hi) {
    const u64 mid = (lo + hi) >> 1;
    if (less_than(sorted, mid, sp))
      lo = mid + 1;
    else
      hi = mid;
  }
  offsets[p] = lo;
}

}  // namespace

void launch_pack_records(ConstKeysSoA keys, const u64* counts, const u32* d_n, u64 cap,
                         KeyCount* out, hipStream_t s) {
  pack_records_kernel<<<dim3(grid_for(cap, 256)), dim3(256), 0, s>>>(keys, counts, d_n, out);
  LOCUST_HIP_LAUNCH_CHECK();
}

void launch_unpack_records(const KeyCount* in, u64 n, KeysSoA keys, u64* counts, u8* parts,
                           hipStream_t s, PartMap pm) {
  if (!n) return;
  unpack_records_kernel<<<dim3(grid_for(n, 256)), dim3(256), 0, s>>>(in, n, keys, counts, parts,
                                                                     pm);
  LOCUST_HIP_LAUNCH_CHECK();
}

void launch_sample_keys(ConstKeysSoA sorted, const u32* d_n, u32 num_samples, PackedKey* out,
                        hipStream_t s) {
  if (!num_samples) return;
  sample_keys_kernel<<<dim3(grid_for(num_samples, 64)), dim3(64), 0, s>>>(sorted, d_n,
                                                                          num_samples, out);
  LOCUST_HIP_LAUNCH_CHECK();
}

void launch_bucket_offsets(ConstKeysSoA sorted, const u32* d_n, const PackedKey* splitters,
                           u32 num_buckets, u64* offsets, hipStream_t s) {
  bucket_offsets_kernel<<<dim3(grid_for(num_buckets + 1, 64)), dim3(64), 0, s>>>(
      sorted, d_n, splitters, num_buckets, offsets);
  LOCUST_HIP_LAUNCH_CHECK();
}

// Loads this file's code object (one module per file) now rather than at its first launch.
void warm_module_shuffle() {
  hipFuncAttributes a;
  (void)hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&pack_records_kernel));
}

}  // namespace locust
