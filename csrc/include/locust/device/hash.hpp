// Key hashing shared by the map kernel (which tags every token with its hash partition)
// and the dictionary kernels.
#pragma once

#include <hip/hip_runtime.h>

#include "locust/common.hpp"

namespace locust {
namespace dev {

__device__ __forceinline__ u64 mix64(u64 x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}

__device__ __forceinline__ u64 key_hash(const u64* k) {
  return mix64(k[0] ^ mix64(k[1] ^ (k[2] * 0x9e3779b97f4a7c15ull) ^ (k[3] << 1)));
}

// Hash partition of a key (256 partitions): the top byte of its hash.
__device__ __forceinline__ u32 key_part(u64 h) { return (u32)(h >> 56); }

}  // namespace dev
}  // namespace locust
