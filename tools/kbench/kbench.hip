// Kernel micro-benchmarks (diagnostics): times individual launchers with hipEvents.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>
#include "locust/hip_check.hpp"
#include "locust/kernels.hpp"

using namespace locust;

__global__ void empty_kernel() {}

__global__ void clock_kernel(unsigned long long* out, int iters) {
  // measures the shader clock: s_memtime ticks vs wall (s_memrealtime 100 MHz)
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  float x = threadIdx.x;
  for (int i = 0; i < iters; ++i) x = x * 1.000001f + 0.5f;
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0 && blockIdx.x == 0) { out[0] = t1 - t0; out[1] = r1 - r0; out[2] = (unsigned long long)x; }
}

template <typename F>
float time_it(hipStream_t s, int reps, F f) {
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  for (int i = 0; i < 3; ++i) f();
  hipEventRecord(a, s);
  for (int i = 0; i < reps; ++i) f();
  hipEventRecord(b, s);
  hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  return ms * 1000.f / reps;  // us
}

int main(int argc, char** argv) {
  const u32 U = argc > 1 ? atoi(argv[1]) : 5608;
  hipStream_t s; LOCUST_HIP_CHECK(hipStreamCreate(&s));
  std::mt19937_64 rng(1);
  std::vector<u64> h(U * 4);
  for (u32 i = 0; i < U; ++i) { h[i] = rng() | 1ull << 62; h[U + i] = rng() >> 8; h[2*U+i] = 0; h[3*U+i] = 0; }
  u64* d; LOCUST_HIP_CHECK(hipMalloc(&d, h.size() * 8));
  LOCUST_HIP_CHECK(hipMemcpy(d, h.data(), h.size() * 8, hipMemcpyHostToDevice));
  u32* du; LOCUST_HIP_CHECK(hipMalloc(&du, 4)); LOCUST_HIP_CHECK(hipMemcpy(du, &U, 4, hipMemcpyHostToDevice));
  u32* rank; LOCUST_HIP_CHECK(hipMalloc(&rank, U * 4));
  KeysSoA k{{d, d + U, d + 2 * U, d + 3 * U}};
  unsigned long long* clk; hipMalloc(&clk, 24);
  printf("empty kernel: %.2f us\n", time_it(s, 200, [&] { empty_kernel<<<1, 64, 0, s>>>(); }));
  printf("empty kernel 2048 blocks: %.2f us\n", time_it(s, 200, [&] { empty_kernel<<<2048, 256, 0, s>>>(); }));
  printf("memset 4 B: %.2f us\n", time_it(s, 200, [&] { hipMemsetAsync(rank, 0, 4, s); }));
  printf("memset %u B: %.2f us\n", U * 4, time_it(s, 200, [&] { hipMemsetAsync(rank, 0, U * 4, s); }));
  clock_kernel<<<1, 64, 0, s>>>(clk, 1 << 20);
  unsigned long long hc[3]; hipMemcpy(hc, clk, 24, hipMemcpyDeviceToHost);
  printf("clock: %llu shader ticks / %llu ref ticks (100MHz) -> %.0f MHz\n", hc[0], hc[1], hc[1] ? hc[0] * 100.0 / hc[1] : 0);
  for (u64 cap : {(u64)U, (u64)89260}) {
    printf("rank_sort U=%u cap=%llu: %.2f us\n", U, (unsigned long long)cap, time_it(s, 50, [&] {
      hipMemsetAsync(rank, 0, U * 4, s);
      launch_rank_sort(k, du, cap, rank, s);
    }));
  }
  return 0;
}
