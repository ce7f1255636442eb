// Where a one-shot GPU process's exit time goes (tools/exit_probe.py
// drives it).  Each mode does one more level of GPU start-up, prints CLOCK_MONOTONIC right
// before _exit(0), and the parent times from that stamp to the reap:
//   none     no HIP call at all (the loader and libamdhip64's static init only)
//   count    hipGetDeviceCount (the runtime's device discovery)
//   context  + hipSetDevice + hipFree(nullptr) (the device's context)
//   stream   + one non-blocking stream, one kernel launch, hipStreamSynchronize
//   memory   + 1 GiB hipMalloc, 64 MiB hipHostMalloc
//   streams2 stream + a second stream with a launch (a second hardware queue)
// Build: hipcc --offload-arch=gfx950 -O2 tools/exit_probe.hip -o build/exit_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <ctime>
#include <unistd.h>

__global__ void probe_kernel(int* p) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && p) p[0] = 1;
}

static unsigned long long mono_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (unsigned long long)ts.tv_sec * 1000000000ull + (unsigned long long)ts.tv_nsec;
}

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));         \
      return 2;                                                            \
    }                                                                      \
  } while (0)

int main(int argc, char** argv) {
  const char* mode = argc > 1 ? argv[1] : "none";
  const unsigned long long t_main = mono_ns();
  const bool count = std::strcmp(mode, "none") != 0;
  const bool context = count && std::strcmp(mode, "count") != 0;
  const bool stream = context && std::strcmp(mode, "context") != 0;
  const bool memory = std::strcmp(mode, "memory") == 0;
  const bool streams2 = std::strcmp(mode, "streams2") == 0;
  if (count) {
    int n = 0;
    CK(hipGetDeviceCount(&n));
    if (n < 1) return 3;
  }
  if (context) {
    CK(hipSetDevice(0));
    CK(hipFree(nullptr));
  }
  int* d = nullptr;
  if (stream) {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CK(hipMalloc(&d, 4096));
    probe_kernel<<<1, 64, 0, s>>>(d);
    CK(hipGetLastError());
    CK(hipStreamSynchronize(s));
    if (streams2) {
      hipStream_t s2;
      CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
      probe_kernel<<<1, 64, 0, s2>>>(d);
      CK(hipGetLastError());
      CK(hipStreamSynchronize(s2));
    }
  }
  if (memory) {
    void* big = nullptr;
    void* pinned = nullptr;
    CK(hipMalloc(&big, 1ull << 30));
    CK(hipMemset(big, 0, 1ull << 30));
    CK(hipHostMalloc(&pinned, 64ull << 20, hipHostMallocDefault));
    std::memset(pinned, 0, 64ull << 20);
    CK(hipDeviceSynchronize());
  }
  const unsigned long long t_exit = mono_ns();
  std::printf("%llu %llu\n", t_main, t_exit);
  std::fflush(stdout);
  _exit(0);
}
