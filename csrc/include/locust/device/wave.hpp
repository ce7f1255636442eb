// Wave64 / workgroup primitives for CDNA4 (gfx950).
//
// A CDNA wavefront is 64 lanes: ballots are 64-bit, lane ranks come from v_mbcnt, and a
// 256-thread workgroup is 4 waves.  Everything here is written for that shape directly
// (no warp-size abstraction).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

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

// DPP lane moves (GFX9 / CDNA: row_shr within 16-lane rows, row_bcast across rows): a
// register-to-register move in the VALU, a few cycles -- unlike __shfl_* (ds_bpermute, an
// LDS round trip).  Lanes without a source keep `old` (0 here).
template <int kCtrl, int kRowMask>
__device__ __forceinline__ uint32_t dpp_mov(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kCtrl, kRowMask, 0xf, false);
}
template <int kCtrl, int kRowMask>
__device__ __forceinline__ uint64_t dpp_mov(uint64_t v) {
  const uint32_t lo = dpp_mov<kCtrl, kRowMask>((uint32_t)v);
  const uint32_t hi = dpp_mov<kCtrl, kRowMask>((uint32_t)(v >> 32));
  return ((uint64_t)hi << 32) | lo;
}

// Inclusive prefix sum across the 64 lanes of a wave: Hillis-Steele inside each 16-lane
// row by row_shr 1/2/4/8, then row 15's total broadcast into rows 1 and 3 and row 31's
// into rows 2 and 3 (the classic GFX9 DPP scan; 6 moves + 6 adds, no LDS traffic).
template <typename T>
__device__ __forceinline__ T wave_inclusive_scan(T v) {
  static_assert(sizeof(T) == 4 || sizeof(T) == 8, "32- or 64-bit scan");
  using U = typename std::conditional<sizeof(T) == 4, uint32_t, uint64_t>::type;
  U x = (U)v;
  x += dpp_mov<0x111, 0xf>(x);  // row_shr:1
  x += dpp_mov<0x112, 0xf>(x);  // row_shr:2
  x += dpp_mov<0x114, 0xf>(x);  // row_shr:4
  x += dpp_mov<0x118, 0xf>(x);  // row_shr:8
  x += dpp_mov<0x142, 0xa>(x);  // row_bcast:15 -> rows 1, 3
  x += dpp_mov<0x143, 0xc>(x);  // row_bcast:31 -> rows 2, 3
  return (T)x;
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
// One barrier: every wave publishes its total, then each thread adds up the totals of
// the waves below it (kWaves broadcast LDS reads) instead of one thread scanning them
// serially between two barriers.
template <typename T, int kBlock>
__device__ __forceinline__ T block_exclusive_scan(T v, T* smem, T* total) {
  constexpr int kWaves = kBlock / 64;
  const int lane = lane_id(), w = wave_id();
  T inc = wave_inclusive_scan(v);
  if (lane == 63) smem[w] = inc;
  __syncthreads();
  T below = 0, all = 0;
#pragma unroll
  for (int i = 0; i < kWaves; ++i) {
    const T t = smem[i];
    below += i < w ? t : T(0);
    all += t;
  }
  *total = all;
  __syncthreads();  // smem reusable by the caller after return
  return below + inc - v;
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
