// Wave64 / workgroup primitives for CDNA4 (gfx950).
//
// A CDNA wavefront is 64 lanes: ballots are 64-bit, lane ranks come from v_mbcnt, and a
// 256-thread workgroup is 4 waves.  Everything here is written for that shape directly
// (no warp-size abstraction).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace locust {
namespace dev {

constexpr int kWave = 64;

__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & 63); }
__device__ __forceinline__ int wave_id() { return (int)(threadIdx.x >> 6); }

// Number of set bits of `mask` in lanes strictly below this lane (v_mbcnt_lo/hi).
__device__ __forceinline__ uint32_t lanes_below(uint64_t mask) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                   __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }

// Inclusive prefix sum across the 64 lanes of a wave.
template <typename T>
__device__ __forceinline__ T wave_inclusive_scan(T v) {
  const int lane = lane_id();
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    T n = __shfl_up(v, off, 64);
    if (lane >= off) v += n;
  }
  return v;
}

template <typename T>
__device__ __forceinline__ T wave_reduce_sum(T v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

template <typename T>
__device__ __forceinline__ T wave_reduce_max(T v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    T o = __shfl_xor(v, off, 64);
    v = o > v ? o : v;
  }
  return v;
}

// Workgroup-wide exclusive scan of one value per thread.  `smem` needs
// (blockDim.x/64 + 1) slots.  Returns the exclusive prefix; *total receives the sum.
template <typename T, int kBlock>
__device__ __forceinline__ T block_exclusive_scan(T v, T* smem, T* total) {
  constexpr int kWaves = kBlock / 64;
  const int lane = lane_id(), w = wave_id();
  T inc = wave_inclusive_scan(v);
  if (lane == 63) smem[w] = inc;
  __syncthreads();
  if (threadIdx.x == 0) {
    T run = 0;
#pragma unroll
    for (int i = 0; i < kWaves; ++i) {
      T t = smem[i];
      smem[i] = run;
      run += t;
    }
    smem[kWaves] = run;
  }
  __syncthreads();
  T res = smem[w] + inc - v;
  *total = smem[kWaves];
  __syncthreads();  // smem reusable by the caller after return
  return res;
}

// ---- agent-scope (device-wide, cross-XCD) atomics used by look-back protocols ----
// Status words are single self-describing granules (flag bits + value), written by one
// atomic store and read by atomic loads, so no separate fence is needed
// (cdna_hip_programming.md §6 Guideline 16, recipe R2).
__device__ __forceinline__ uint64_t ld_agent(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld_agent(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace dev
}  // namespace locust
