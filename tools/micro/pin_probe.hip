// What page-locking a streaming engine's 64 MiB read ring costs, by allocation method
// (stage 1 pays it once per process: ~10 ms of its ~60 ms fixed cost, ROUND6.md):
//   hipHostMalloc of 4 x 16 MiB (the engine's way), one 64 MiB hipHostMalloc,
//   malloc + hipHostRegister, mmap + MADV_HUGEPAGE + first touch + hipHostRegister,
// each followed by one 16 MiB H2D copy from it (the pages must be usable for DMA).
// Build: hipcc --offload-arch=gfx950 -O2 tools/micro/pin_probe.hip -o build/pin_probe
#include <hip/hip_runtime.h>
#include <sys/mman.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                          \
  do {                                                                 \
    hipError_t e_ = (x);                                               \
    if (e_ != hipSuccess) {                                            \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));     \
      std::exit(2);                                                    \
    }                                                                  \
  } while (0)

static double ms_since(std::chrono::steady_clock::time_point t) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

int main() {
  constexpr size_t kPiece = 16u << 20, kRing = 4 * kPiece;
  CK(hipSetDevice(0));
  CK(hipFree(nullptr));
  void* dev = nullptr;
  CK(hipMalloc(&dev, kPiece));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  auto copy_ms = [&](const void* src) {
    const auto t = std::chrono::steady_clock::now();
    CK(hipMemcpyAsync(dev, src, kPiece, hipMemcpyHostToDevice, s));
    CK(hipStreamSynchronize(s));
    return ms_since(t);
  };
  (void)copy_ms(std::calloc(1, kPiece));  // the copy path's own first use
  for (int rep = 0; rep < 3; ++rep) {
    {
      const auto t = std::chrono::steady_clock::now();
      void* p[4];
      for (auto& x : p) CK(hipHostMalloc(&x, kPiece, hipHostMallocDefault));
      const double a = ms_since(t);
      std::printf("hipHostMalloc 4 x 16 MiB:           %7.2f ms, copy %.3f ms\n", a, copy_ms(p[0]));
      for (auto& x : p) CK(hipHostFree(x));
    }
    {
      const auto t = std::chrono::steady_clock::now();
      void* p = nullptr;
      CK(hipHostMalloc(&p, kRing, hipHostMallocDefault));
      const double a = ms_since(t);
      std::printf("hipHostMalloc 64 MiB:               %7.2f ms, copy %.3f ms\n", a, copy_ms(p));
      CK(hipHostFree(p));
    }
    {
      const auto t = std::chrono::steady_clock::now();
      void* p = std::aligned_alloc(4096, kRing);
      std::memset(p, 0, kRing);
      const double touch = ms_since(t);
      CK(hipHostRegister(p, kRing, hipHostRegisterDefault));
      const double a = ms_since(t);
      std::printf("malloc + touch + hipHostRegister:   %7.2f ms (touch %.2f), copy %.3f ms\n", a,
                  touch, copy_ms(p));
      CK(hipHostUnregister(p));
      std::free(p);
    }
    {
      const auto t = std::chrono::steady_clock::now();
      void* p = mmap(nullptr, kRing, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
      if (p == MAP_FAILED) return 3;
      const int adv = madvise(p, kRing, MADV_HUGEPAGE);
      std::memset(p, 0, kRing);
      const double touch = ms_since(t);
      CK(hipHostRegister(p, kRing, hipHostRegisterDefault));
      const double a = ms_since(t);
      std::printf("mmap + THP(%s) + touch + register: %7.2f ms (touch %.2f), copy %.3f ms\n",
                  adv == 0 ? "ok" : "no", a, touch, copy_ms(p));
      CK(hipHostUnregister(p));
      munmap(p, kRing);
    }
  }
  std::printf("THP setting: ");
  std::fflush(stdout);
  if (FILE* f = std::fopen("/sys/kernel/mm/transparent_hugepage/enabled", "r")) {
    char buf[128] = {0};
    if (std::fgets(buf, sizeof(buf), f)) std::printf("%s", buf);
    std::fclose(f);
  }
  CK(hipStreamDestroy(s));
  CK(hipFree(dev));
  return 0;
}
