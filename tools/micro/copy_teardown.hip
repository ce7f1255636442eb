// H2D copy rate from one large pinned host buffer before and after a teardown step of
// another user of the device: a stream destroyed, a fine-grained (mapped) pinned buffer
// freed, a device buffer freed, or all three.  tools/stream_probe.py showed a streamed
// 10 GB job falling from 57 to ~30 GB/s on the middle chunks after another engine was
// destroyed; this isolates which runtime call does it.
//
// Usage: copy_teardown <step: none|stream|mapped|devfree|all> [GB]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e = (x);                                                            \
    if (e != hipSuccess) {                                                         \
      std::printf("%s failed: %s\n", #x, hipGetErrorString(e));                    \
      std::exit(1);                                                                \
    }                                                                              \
  } while (0)

static void pass(const char* tag, char* h, char* d[2], size_t total, size_t chunk, hipStream_t s) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  std::vector<float> ms;
  for (size_t off = 0, k = 0; off + chunk <= total; off += chunk, ++k) {
    CK(hipEventRecord(a, s));
    CK(hipMemcpyAsync(d[k & 1], h + off, chunk, hipMemcpyHostToDevice, s));
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float t = 0;
    CK(hipEventElapsedTime(&t, a, b));
    ms.push_back(t);
  }
  double sum = 0;
  std::printf("%-8s GB/s per chunk:", tag);
  for (float t : ms) {
    std::printf(" %.0f", chunk / (t * 1e6));
    sum += t;
  }
  std::printf("  | total %.1f GB/s\n", ms.size() * chunk / (sum * 1e6));
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
}

int main(int argc, char** argv) {
  const char* step = argc > 1 ? argv[1] : "all";
  const size_t total = (size_t)((argc > 2 ? std::atof(argv[2]) : 8.0) * (1ull << 30));
  const size_t chunk = 256ull << 20;
  char* h = nullptr;
  CK(hipHostMalloc(reinterpret_cast<void**>(&h), total, hipHostMallocDefault));
  std::memset(h, 'a', total);
  char* d[2];
  CK(hipMalloc(reinterpret_cast<void**>(&d[0]), chunk));
  CK(hipMalloc(reinterpret_cast<void**>(&d[1]), chunk));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  pass("before", h, d, total, chunk, s);
  pass("again", h, d, total, chunk, s);
  const bool all = !std::strcmp(step, "all");
  if (all || !std::strcmp(step, "stream")) {
    hipStream_t t;
    CK(hipStreamCreateWithFlags(&t, hipStreamNonBlocking));
    CK(hipMemcpyAsync(d[0], h, 4 << 20, hipMemcpyHostToDevice, t));
    CK(hipStreamSynchronize(t));
    CK(hipStreamDestroy(t));
  }
  if (all || !std::strcmp(step, "mapped")) {
    void* m = nullptr;
    CK(hipHostMalloc(&m, 12 << 20, hipHostMallocMapped | hipHostMallocCoherent));
    CK(hipHostFree(m));
  }
  if (all || !std::strcmp(step, "devfree")) {
    void* x = nullptr;
    CK(hipMalloc(&x, 1ull << 30));
    CK(hipMemset(x, 0, 1ull << 30));
    CK(hipDeviceSynchronize());
    CK(hipFree(x));
  }
  pass(step, h, d, total, chunk, s);
  pass("again", h, d, total, chunk, s);
  return 0;
}
