// The fast map's staging pattern on a Hamlet-sized input (188 KiB): one workgroup of 1,024
// threads per 1 KiB tile reads its tile plus 128 B before and 64 B after (16-B loads) from
// pinned host memory into LDS.  Varies the host allocation (default / coherent /
// non-coherent) and the tile order (block index, or consecutive tiles on one XCD so the
// neighbours' overlapping context could hit that XCD's L2).  Kernel time per launch from
// hipEvents over many launches.
//   hipcc --offload-arch=gfx950 -O2 tools/micro/stage_read.hip -o build/stage_read
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>

#define CK(x)                                                          \
  do {                                                                 \
    hipError_t e = (x);                                                \
    if (e != hipSuccess) {                                             \
      std::printf("%s failed: %s\n", #x, hipGetErrorString(e));        \
      return 1;                                                        \
    }                                                                  \
  } while (0)

constexpr int kTile = 1024, kPre = 128, kPost = 64, kStaged = kPre + kTile + kPost;

template <bool kXcd>
__global__ __launch_bounds__(1024) void stage_kernel(const char* __restrict__ text,
                                                     unsigned long long bytes,
                                                     unsigned* __restrict__ sink) {
  __shared__ __attribute__((aligned(16))) unsigned char s[kStaged];
  const unsigned G = gridDim.x, b = blockIdx.x;
  unsigned tile = b;
  if (kXcd) {  // consecutive tiles on one XCD (blocks b = 8k + x run on XCD x)
    const unsigned q = G / 8, r = G % 8, x = b % 8, k = b / 8;
    tile = x * q + (x < r ? x : r) + k;
  }
  const long long lo = (long long)tile * kTile - kPre;
  for (int c = threadIdx.x; c < kStaged / 16; c += blockDim.x) {
    const long long g = lo + (long long)c * 16;
    uint4 v = {0, 0, 0, 0};
    if (g >= 0 && (unsigned long long)g < bytes) v = *reinterpret_cast<const uint4*>(text + g);
    *reinterpret_cast<uint4*>(s + c * 16) = v;
  }
  __syncthreads();
  unsigned acc = 0;
  for (int i = threadIdx.x; i < kStaged; i += blockDim.x) acc += s[i];
  if (acc == 0xFFFFFFFFu) sink[b] = acc;
}

int main() {
  const unsigned long long bytes = 188 * 1024ull;
  const unsigned G = (unsigned)((bytes + kTile - 1) / kTile);
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  unsigned* sink;
  CK(hipMalloc(&sink, 4096 * 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const struct {
    const char* name;
    unsigned flags;
  } kinds[] = {{"default", hipHostMallocDefault},
               {"coherent", hipHostMallocMapped | hipHostMallocCoherent},
               {"noncoherent", hipHostMallocMapped | hipHostMallocNonCoherent}};
  for (const auto& k : kinds) {
    char* h = nullptr;
    CK(hipHostMalloc(&h, bytes + 256, k.flags));
    std::memset(h, 'a', bytes + 256);
    char* d = nullptr;
    CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&d), h, 0));
    for (int xcd = 0; xcd < 2; ++xcd) {
      const int N = 2000;
      for (int i = 0; i < 100; ++i) {
        if (xcd) stage_kernel<true><<<G, 1024, 0, st>>>(d, bytes, sink);
        else stage_kernel<false><<<G, 1024, 0, st>>>(d, bytes, sink);
      }
      CK(hipStreamSynchronize(st));
      float best = 1e30f, sum = 0;
      for (int rep = 0; rep < 5; ++rep) {
        CK(hipEventRecord(e0, st));
        for (int i = 0; i < N / 5; ++i) {
          if (xcd) stage_kernel<true><<<G, 1024, 0, st>>>(d, bytes, sink);
          else stage_kernel<false><<<G, 1024, 0, st>>>(d, bytes, sink);
        }
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const float us = ms * 1e3f / (N / 5);
        best = us < best ? us : best;
        sum += us;
      }
      std::printf("%-12s %-10s %7.2f us/launch (best of 5: %.2f)\n", k.name,
                  xcd ? "xcd-order" : "block", sum / 5, best);
    }
    CK(hipHostFree(h));
  }
  return 0;
}
