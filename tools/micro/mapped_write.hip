// Kernel writes into host-mapped (fine-grained) memory vs a D2H DMA of the same bytes:
// 9.5 MiB (the synth1m output), 16 B per lane, consecutive lanes on consecutive chunks.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e = (x);                                                            \
    if (e != hipSuccess) {                                                         \
      std::printf("%s failed: %s\n", #x, hipGetErrorString(e));                    \
      return 1;                                                                    \
    }                                                                              \
  } while (0)

using v2u64 = unsigned long long __attribute__((ext_vector_type(2)));

__global__ void write_kernel(v2u64* __restrict__ dst, unsigned long long n) {
  for (unsigned long long i = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x; i < n;
       i += (unsigned long long)gridDim.x * blockDim.x)
    dst[i] = v2u64{i, i ^ 0x5555ull};
}

int main() {
  const unsigned long long bytes = 9728ull << 10, n = bytes / 16;
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  v2u64 *h = nullptr, *d = nullptr, *dev = nullptr;
  CK(hipHostMalloc(&h, bytes, hipHostMallocMapped | hipHostMallocCoherent));
  CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&d), h, 0));
  CK(hipMalloc(&dev, bytes));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int grid : {256, 1024, 4096}) {
    for (int it = 0; it < 3; ++it) write_kernel<<<grid, 1024, 0, s>>>(d, n);
    CK(hipEventRecord(a, s));
    for (int it = 0; it < 10; ++it) write_kernel<<<grid, 1024, 0, s>>>(d, n);
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    std::printf("kernel -> mapped host, grid %4d: %.1f us  %.1f GB/s\n", grid, ms * 100.f,
                bytes / (ms / 10 * 1e-3) / 1e9);
  }
  write_kernel<<<1024, 1024, 0, s>>>(dev, n);
  for (int it = 0; it < 3; ++it) CK(hipMemcpyAsync(h, dev, bytes, hipMemcpyDeviceToHost, s));
  CK(hipEventRecord(a, s));
  for (int it = 0; it < 10; ++it) CK(hipMemcpyAsync(h, dev, bytes, hipMemcpyDeviceToHost, s));
  CK(hipEventRecord(b, s));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  std::printf("DMA device -> host:           %.1f us  %.1f GB/s\n", ms * 100.f,
              bytes / (ms / 10 * 1e-3) / 1e9);
  return 0;
}
