// Launch + completion latency floor on this box: empty-kernel launch/sync, 2-kernel graph
// replay/sync, and graph replay with the host polling a mapped completion word.
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdio>

#define CK(x)                                                          \
  do {                                                                 \
    hipError_t e = (x);                                                \
    if (e != hipSuccess) {                                             \
      std::printf("%s failed: %s\n", #x, hipGetErrorString(e));        \
      return 1;                                                        \
    }                                                                  \
  } while (0)

__global__ void k_empty(int* p) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && p) p[1] = 0;
}
__global__ void k_flag(volatile unsigned* flag, unsigned v) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    __threadfence_system();
    *flag = v;
  }
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

int main() {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  int* d;
  CK(hipMalloc(&d, 64));
  unsigned* hflag;
  CK(hipHostMalloc(&hflag, 64, hipHostMallocMapped | hipHostMallocCoherent));
  unsigned* dflag;
  CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&dflag), hflag, 0));
  const int N = 2000;
  // (a) one kernel + hipStreamSynchronize
  for (int i = 0; i < 100; ++i) k_empty<<<1, 64, 0, s>>>(d);
  CK(hipStreamSynchronize(s));
  double t0 = now_us();
  for (int i = 0; i < N; ++i) {
    k_empty<<<1, 64, 0, s>>>(d);
    CK(hipStreamSynchronize(s));
  }
  std::printf("kernel+sync          %.2f us/iter\n", (now_us() - t0) / N);
  // (b) graph of two kernels (256 blocks each) + sync
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed));
  k_empty<<<256, 256, 0, s>>>(d);
  k_empty<<<256, 1024, 0, s>>>(d);
  k_flag<<<1, 64, 0, s>>>(dflag, 0);
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  for (int i = 0; i < 100; ++i) CK(hipGraphLaunch(ge, s));
  CK(hipStreamSynchronize(s));
  t0 = now_us();
  for (int i = 0; i < N; ++i) {
    CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
  }
  std::printf("graph(3)+sync        %.2f us/iter\n", (now_us() - t0) / N);
  // (c) the same kernels launched directly + sync
  t0 = now_us();
  for (int i = 0; i < N; ++i) {
    k_empty<<<256, 256, 0, s>>>(d);
    k_empty<<<256, 1024, 0, s>>>(d);
    k_flag<<<1, 64, 0, s>>>(dflag, 0);
    CK(hipStreamSynchronize(s));
  }
  std::printf("3 launches+sync      %.2f us/iter\n", (now_us() - t0) / N);
  // (d) direct launches, host polls the mapped flag, then a cheap query
  t0 = now_us();
  for (int i = 1; i <= N; ++i) {
    k_empty<<<256, 256, 0, s>>>(d);
    k_empty<<<256, 1024, 0, s>>>(d);
    k_flag<<<1, 64, 0, s>>>(dflag, (unsigned)i);
    while (reinterpret_cast<volatile unsigned*>(hflag)[0] != (unsigned)i) {
    }
  }
  CK(hipStreamSynchronize(s));
  std::printf("3 launches+poll flag %.2f us/iter\n", (now_us() - t0) / N);
  // (e) event record + hipEventSynchronize
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  t0 = now_us();
  for (int i = 0; i < N; ++i) {
    k_empty<<<256, 256, 0, s>>>(d);
    k_empty<<<256, 1024, 0, s>>>(d);
    CK(hipEventRecord(ev, s));
    CK(hipEventSynchronize(ev));
  }
  std::printf("2 launches+event sync %.2f us/iter\n", (now_us() - t0) / N);
  return 0;
}
