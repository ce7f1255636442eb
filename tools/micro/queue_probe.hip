// What a process's first kernel launch costs by the stream it uses (the engine's
// construction logs "stream 15-17 ms": a non-blocking stream's creation and first launch):
//   created   hipStreamCreateWithFlags(non-blocking), launch, synchronize
//   null      the legacy default stream, launch, synchronize
//   perthread hipStreamPerThread, launch, synchronize
// then a second stream created after the first (a second hardware queue).
// Usage: build/queue_probe MODE   (one fresh process per mode: tools/exit_probe.py style)
// Build: hipcc --offload-arch=gfx950 -O2 tools/micro/queue_probe.hip -o build/queue_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstring>

__global__ void tiny(int* p) {
  if (p && threadIdx.x == 0) p[0] += 1;
}

#define CK(x)                                                      \
  do {                                                             \
    hipError_t e_ = (x);                                           \
    if (e_ != hipSuccess) {                                        \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); \
      return 2;                                                    \
    }                                                              \
  } while (0)

using Clock = std::chrono::steady_clock;
static double ms(Clock::time_point a, Clock::time_point b) {
  return std::chrono::duration<double, std::milli>(b - a).count();
}

int main(int argc, char** argv) {
  const char* mode = argc > 1 ? argv[1] : "created";
  const auto t0 = Clock::now();
  CK(hipSetDevice(0));
  CK(hipFree(nullptr));
  int* d = nullptr;
  CK(hipMalloc(&d, 256));
  const auto t1 = Clock::now();
  hipStream_t s = nullptr;
  if (std::strcmp(mode, "created") == 0) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  if (std::strcmp(mode, "perthread") == 0) s = hipStreamPerThread;
  const auto t2 = Clock::now();
  tiny<<<1, 64, 0, s>>>(d);
  CK(hipGetLastError());
  const auto t3 = Clock::now();
  CK(hipStreamSynchronize(s));
  const auto t4 = Clock::now();
  tiny<<<1, 64, 0, s>>>(d);
  CK(hipStreamSynchronize(s));
  const auto t5 = Clock::now();
  hipStream_t s2;
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  tiny<<<1, 64, 0, s2>>>(d);
  CK(hipStreamSynchronize(s2));
  const auto t6 = Clock::now();
  std::printf("%-9s init+context %7.2f  create %6.2f  first launch %6.2f  first sync %6.2f  "
              "second launch+sync %6.3f  second stream create+launch+sync %6.2f ms\n",
              mode, ms(t0, t1), ms(t1, t2), ms(t2, t3), ms(t3, t4), ms(t4, t5), ms(t5, t6));
  return 0;
}
