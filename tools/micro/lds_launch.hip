// Fixed cost of a launch as a function of the workgroup's static LDS, its size and the
// grid -- the ordered kernel (256 x 1024 threads, ~147 KB LDS) spends ~10 us of its ~22 us
// outside its workgroups' own span (LOCUST_ORD_TRACE).  Also: the cost of a system-scope
// release per workgroup after it wrote 4 KiB (the ordered kernel's self-clean handshake).
// Kernel durations: run under `rocprofv3 --kernel-trace --stats`; the host loop prints the
// event-timed mean per launch too.
//   hipcc --offload-arch=gfx950 -O2 tools/micro/lds_launch.hip -o build/lds_launch
#include <hip/hip_runtime.h>

#include <cstdio>

#define CK(x)                                                          \
  do {                                                                 \
    hipError_t e = (x);                                                \
    if (e != hipSuccess) {                                             \
      std::printf("%s failed: %s\n", #x, hipGetErrorString(e));        \
      return 1;                                                        \
    }                                                                  \
  } while (0)

template <int kLds, int kBlock>
__global__ __launch_bounds__(kBlock) void k_lds(unsigned* out) {
  __shared__ unsigned s[kLds / 4 > 0 ? kLds / 4 : 1];
  s[threadIdx.x % (kLds / 4 > 0 ? kLds / 4 : 1)] = threadIdx.x;
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = s[(blockIdx.x * 7) % (kLds / 4 > 0 ? kLds / 4 : 1)];
}

// every workgroup writes 4 KiB, then (kFence) a system- or agent-scope release + a counter
template <int kFence, int kBlock>
__global__ __launch_bounds__(kBlock) void k_fence(unsigned* out, unsigned* ctr) {
  for (int i = threadIdx.x; i < 1024; i += kBlock) out[(size_t)blockIdx.x * 1024 + i] = i ^ blockIdx.x;
  __syncthreads();
  if (threadIdx.x == 0) {
    if (kFence == 2) __threadfence_system();
    if (kFence == 1) __threadfence();
    if (kFence == 0) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    atomicAdd(ctr, 1u);
  }
}

template <class F>
static float time_launches(hipStream_t s, F f, int n) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int i = 0; i < 20; ++i) f();
  (void)hipEventRecord(a, s);
  for (int i = 0; i < n; ++i) f();
  (void)hipEventRecord(b, s);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms * 1000.f / n;
}

int main() {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  unsigned *out, *ctr;
  CK(hipMalloc(&out, 512 * 4096 * 4));
  CK(hipMalloc(&ctr, 64));
  const int N = 400;
#define RUN(LDS, BLK, GRID)                                                                      \
  std::printf("lds %6d B  block %4d  grid %4d: %7.2f us/launch\n", LDS, BLK, GRID,              \
              time_launches(s, [&] { k_lds<LDS, BLK><<<GRID, BLK, 0, s>>>(out); }, N));
  RUN(0, 256, 256)
  RUN(0, 1024, 256)
  RUN(16384, 1024, 256)
  RUN(65536, 1024, 256)
  RUN(98304, 1024, 256)
  RUN(147456, 1024, 256)
  RUN(147456, 256, 256)
  RUN(147456, 1024, 512)
  RUN(0, 1024, 512)
#undef RUN
#define RUNF(F, BLK, GRID)                                                                       \
  std::printf("fence %d  block %4d  grid %4d: %7.2f us/launch\n", F, BLK, GRID,                 \
              time_launches(s, [&] { k_fence<F, BLK><<<GRID, BLK, 0, s>>>(out, ctr); }, N));
  RUNF(0, 1024, 256)
  RUNF(1, 1024, 256)
  RUNF(2, 1024, 256)
#undef RUNF
  CK(hipStreamSynchronize(s));
  return 0;
}
