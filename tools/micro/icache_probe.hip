// Does instruction fetch cost the headline's kernels time?  dict_ordered_kernel<TileSource>
// is 57.7 KB of code and map_fast_kernel<1, 1024> 8.8 KB; a job runs both, once each.  This
// times, inside the kernel (s_memrealtime, 100 MHz), the same 2,048 dependent VALU adds laid
// out three ways: straight-line (8 KB of code), as a 64-add loop body (256 B), and
// straight-line right after an "evictor" kernel of 56 KB of other code -- and the
// straight-line kernel with 16 waves per workgroup (the map's shape), where the waves of a
// CU share the fetch.  Per launch: the median wave's duration and the launch's span (first
// wave start -> last wave end).  Straight ~= loop: fetch is hidden; straight-after-evictor >>
// straight: a job's kernels refetch each other's code every job.
// Build: make icache_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

using u64 = unsigned long long;

#define CHECK(x)                                                               \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
      return 1;                                                                \
    }                                                                          \
  } while (0)

template <int N>
__global__ void straight_kernel(u64* out, unsigned y) {
  const u64 t0 = __builtin_amdgcn_s_memrealtime();
  unsigned x = threadIdx.x;
  // one asm block (.rept): exactly N 4-byte VOP2 adds, no compiler unrolling or nops
  asm volatile(".rept %c2\n v_add_u32 %0, %0, %1\n .endr" : "+v"(x) : "v"(y), "i"(N));
  const u64 t1 = __builtin_amdgcn_s_memrealtime();
  const unsigned wave = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
  if (threadIdx.x % 64 == 0) {
    out[2 * wave] = t0;
    out[2 * wave + 1] = t1 + (x == 0xdeadbeefu);  // keeps x live
  }
}

__global__ void loop_kernel(u64* out, unsigned y, int rounds) {
  const u64 t0 = __builtin_amdgcn_s_memrealtime();
  unsigned x = threadIdx.x;
#pragma nounroll
  for (int r = 0; r < rounds; ++r) {
    asm volatile(".rept 64\n v_add_u32 %0, %0, %1\n .endr" : "+v"(x) : "v"(y));
  }
  const u64 t1 = __builtin_amdgcn_s_memrealtime();
  const unsigned wave = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
  if (threadIdx.x % 64 == 0) {
    out[2 * wave] = t0;
    out[2 * wave + 1] = t1 + (x == 0xdeadbeefu);
  }
}

constexpr int kAdds = 2048;     // 8 KB of v_add_u32
constexpr int kEvict = 14336;   // 56 KB

struct Stat {
  double wave_us, span_us;
};

static Stat stat_of(const std::vector<u64>& h, int waves) {
  std::vector<double> d(waves);
  u64 lo = ~0ull, hi = 0;
  for (int w = 0; w < waves; ++w) {
    d[w] = (double)(h[2 * w + 1] - h[2 * w]) / 100.0;  // 100 MHz ticks -> us
    lo = std::min(lo, h[2 * w]);
    hi = std::max(hi, h[2 * w + 1]);
  }
  std::sort(d.begin(), d.end());
  return {d[waves / 2], (double)(hi - lo) / 100.0};
}

int main() {
  CHECK(hipSetDevice(0));
  const int kMaxWaves = 256 * 16;
  u64* d_out = nullptr;
  u64* d_junk = nullptr;
  CHECK(hipMalloc(&d_out, sizeof(u64) * 2 * kMaxWaves));
  CHECK(hipMalloc(&d_junk, sizeof(u64) * 2 * kMaxWaves));
  hipStream_t s;
  CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  std::vector<u64> h(2 * kMaxWaves);
  const int kReps = 30;

  auto run = [&](const char* name, int blocks, int threads, bool evict, auto launch) -> int {
    const int waves = blocks * threads / 64;
    std::vector<double> wv, sp;
    for (int r = 0; r < kReps + 3; ++r) {
      if (evict) straight_kernel<kEvict><<<256, 64, 0, s>>>(d_junk, 3u);
      launch(blocks, threads);
      CHECK(hipGetLastError());
      CHECK(hipStreamSynchronize(s));
      if (r < 3) continue;  // first launches load the code object
      CHECK(hipMemcpy(h.data(), d_out, sizeof(u64) * 2 * waves, hipMemcpyDeviceToHost));
      const Stat st = stat_of(h, waves);
      wv.push_back(st.wave_us);
      sp.push_back(st.span_us);
    }
    std::sort(wv.begin(), wv.end());
    std::sort(sp.begin(), sp.end());
    std::printf("%-44s wave median %6.2f us (min %6.2f)  span median %6.2f us (min %6.2f)\n", name,
                wv[wv.size() / 2], wv[0], sp[sp.size() / 2], sp[0]);
    return 0;
  };
  auto straight = [&](int b, int t) { straight_kernel<kAdds><<<b, t, 0, s>>>(d_out, 3u); };
  auto looped = [&](int b, int t) { loop_kernel<<<b, t, 0, s>>>(d_out, 3u, kAdds / 64); };

  int rc = 0;
  rc |= run("straight 8 KB, 256 x 1 wave, back to back", 256, 64, false, straight);
  rc |= run("loop 256 B, 256 x 1 wave, back to back", 256, 64, false, looped);
  rc |= run("straight 8 KB, 256 x 1 wave, after evictor", 256, 64, true, straight);
  rc |= run("loop 256 B, 256 x 1 wave, after evictor", 256, 64, true, looped);
  rc |= run("straight 8 KB, 187 x 16 waves, back to back", 187, 1024, false, straight);
  rc |= run("loop 256 B, 187 x 16 waves, back to back", 187, 1024, false, looped);
  rc |= run("straight 8 KB, 187 x 16 waves, after evictor", 187, 1024, true, straight);
  CHECK(hipStreamDestroy(s));
  CHECK(hipFree(d_out));
  CHECK(hipFree(d_junk));
  return rc;
}
