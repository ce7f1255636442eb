// H2D copy rate into a freshly allocated device arena, allocated and freed in turn like
// consecutive engines of one process (tools/s10g_probe.py: every other engine's streamed
// 10 GB job ran its chunk copies at ~30 instead of ~57 GB/s).  Each cycle: hipMalloc an
// arena of ARENA GiB, copy TOTAL GiB of pinned host text into 256 MiB chunks at its
// start (alternating two chunk slots), report GB/s, hipFree.
//
// Usage: arena_cycle [cycles] [arena GiB] [total GiB] [keep: 0|1]
//   keep=1: the arena is cached and reused instead of freed (a caching allocator).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e = (x);                                                            \
    if (e != hipSuccess) {                                                         \
      std::printf("%s failed: %s\n", #x, hipGetErrorString(e));                    \
      std::exit(1);                                                                \
    }                                                                              \
  } while (0)

int main(int argc, char** argv) {
  const int cycles = argc > 1 ? std::atoi(argv[1]) : 4;
  const size_t arena = (size_t)((argc > 2 ? std::atof(argv[2]) : 2.0) * (1ull << 30));
  const size_t total = (size_t)((argc > 3 ? std::atof(argv[3]) : 4.0) * (1ull << 30));
  const bool keep = argc > 4 && std::atoi(argv[4]) != 0;
  const size_t chunk = 256ull << 20;
  char* h = nullptr;
  CK(hipHostMalloc(reinterpret_cast<void**>(&h), total, hipHostMallocDefault));
  std::memset(h, 'a', total);
  char* cached = nullptr;
  for (int c = 0; c < cycles; ++c) {
    char* d = cached;
    if (!d) CK(hipMalloc(reinterpret_cast<void**>(&d), arena));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventRecord(a, s));
    for (size_t off = 0, k = 0; off + chunk <= total; off += chunk, ++k)
      CK(hipMemcpyAsync(d + (k & 1) * chunk, h + off, chunk, hipMemcpyHostToDevice, s));
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    std::printf("cycle %d: arena %p  %.1f GB/s\n", c, (void*)d, (total / chunk * chunk) / (ms * 1e6));
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    CK(hipStreamDestroy(s));
    if (keep)
      cached = d;
    else
      CK(hipFree(d));
  }
  if (cached) CK(hipFree(cached));
  CK(hipHostFree(h));
  return 0;
}
