// Host RSS of the HIP runtime's own first-use steps (what a one-shot CLI job pays before
// its engine allocates anything).  Build: hipcc --offload-arch=gfx950 -O2 tools/rss_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <atomic>
#include <vector>
#include <cstdlib>
#include <thread>
#include <cstring>

// "RssAnon/RssFile/RssShmem" of /proc/self/status, kB.
static void rss(char* out, size_t n) {
  std::FILE* f = std::fopen("/proc/self/status", "r");
  unsigned long long a = 0, fi = 0, sh = 0, v = 0;
  char line[256];
  while (f && std::fgets(line, sizeof(line), f)) {
    if (std::sscanf(line, "RssAnon: %llu", &v) == 1) a = v;
    if (std::sscanf(line, "RssFile: %llu", &v) == 1) fi = v;
    if (std::sscanf(line, "RssShmem: %llu", &v) == 1) sh = v;
  }
  if (f) std::fclose(f);
  std::snprintf(out, n, "rss %7llu kB (anon %7llu file %7llu shmem %7llu)", a + fi + sh, a, fi, sh);
}

__global__ void touch(int* p) { p[threadIdx.x] = threadIdx.x; }

// The mappings holding >= 8 MiB of resident memory (/proc/self/smaps): where the runtime's
// first-use RSS lives (address range, name, Rss, Anonymous).
static void big_mappings(const char* when) {
  std::FILE* f = std::fopen("/proc/self/smaps", "r");
  if (!f) return;
  char line[512], head[512] = {0};
  unsigned long long rss = 0, anon = 0, v = 0;
  auto flush = [&] {
    if (head[0] && rss >= 8192) std::printf("  [%s] %8llu kB rss %8llu kB anon  %s", when, rss, anon, head);
  };
  while (std::fgets(line, sizeof(line), f)) {
    if (std::sscanf(line, "Rss: %llu", &v) == 1) { rss = v; continue; }
    if (std::sscanf(line, "Anonymous: %llu", &v) == 1) { anon = v; continue; }
    // a mapping header: "start-end perms offset dev inode [name]"
    unsigned long long a0, a1;
    if (std::sscanf(line, "%llx-%llx", &a0, &a1) == 2 && std::strchr(line, ' ') &&
        line[std::strcspn(line, " ") - 1] != ':') {
      flush();
      std::snprintf(head, sizeof(head), "%s", line);
      rss = anon = 0;
    }
  }
  flush();
  std::fclose(f);
}

#define STEP(what, call)                                                         \
  do {                                                                           \
    hipError_t e_ = (call);                                                      \
    char b_[160];                                                                \
    rss(b_, sizeof(b_));                                                         \
    std::printf("%-30s %s %s\n", what, e_ == hipSuccess ? "ok " : "ERR", b_);     \
  } while (0)

int main() {
  char b0[160];
  rss(b0, sizeof(b0));
  std::printf("%-30s     %s\n", "start", b0);
  STEP("hipInit", hipInit(0));
  int n = 0;
  STEP("hipGetDeviceCount", hipGetDeviceCount(&n));
  STEP("hipSetDevice", hipSetDevice(0));
  STEP("hipFree(0)", hipFree(nullptr));
  hipStream_t s;
  STEP("hipStreamCreate", hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  big_mappings("stream");
  int* d = nullptr;
  STEP("hipMalloc 1 GiB", hipMalloc(&d, 1ull << 30));
  touch<<<1, 64, 0, s>>>(d);
  STEP("first kernel", hipStreamSynchronize(s));
  void* h = nullptr;
  STEP("hipHostMalloc 64 MiB", hipHostMalloc(&h, 64ull << 20, hipHostMallocDefault));
  void* m = nullptr;
  STEP("hipHostMalloc mapped 16 MiB", hipHostMalloc(&m, 16ull << 20, hipHostMallocMapped));
  STEP("hipMemcpyAsync H2D 64 MiB", hipMemcpyAsync(d, h, 64ull << 20, hipMemcpyHostToDevice, s));
  STEP("sync", hipStreamSynchronize(s));
  big_mappings("copy");
  hipStream_t s2[4];
  for (int k = 0; k < 4; ++k) STEP("another stream", hipStreamCreateWithFlags(&s2[k], hipStreamNonBlocking));
  // streams beyond the hardware queues: what their first kernel, first H2D copy and
  // first D2H copy cost (a multi-rank run's engines each bring 2-3 streams)
  hipStream_t s3[12];
  for (int k = 0; k < 12; ++k) {
    STEP("stream", hipStreamCreateWithFlags(&s3[k], hipStreamNonBlocking));
    touch<<<1, 64, 0, s3[k]>>>(d);
    STEP("  its first kernel", hipStreamSynchronize(s3[k]));
    STEP("  its first H2D 4 MiB", hipMemcpyAsync(d, h, 4ull << 20, hipMemcpyHostToDevice, s3[k]));
    STEP("  sync", hipStreamSynchronize(s3[k]));
    STEP("  its first D2H 4 MiB", hipMemcpyAsync(h, d, 4ull << 20, hipMemcpyDeviceToHost, s3[k]));
    STEP("  sync", hipStreamSynchronize(s3[k]));
  }
  // large device arenas (a 256 MiB-chunk engine reserves ~34 GB), device-to-device
  // copies, memsets, events and a registered host range
  void* big[3] = {};
  for (int k = 0; k < 3; ++k) STEP("hipMalloc 32 GiB", hipMalloc(&big[k], 32ull << 30));
  STEP("D2D 64 MiB", hipMemcpyAsync(big[0], big[1], 64ull << 20, hipMemcpyDeviceToDevice, s));
  STEP("  sync", hipStreamSynchronize(s));
  STEP("memset 64 MiB", hipMemsetAsync(big[2], 0, 64ull << 20, s));
  STEP("  sync", hipStreamSynchronize(s));
  hipEvent_t evs[64];
  for (int k = 0; k < 64; ++k) (void)hipEventCreateWithFlags(&evs[k], hipEventDisableTiming);
  STEP("64 events", hipSuccess);
  void* reg = std::malloc(64ull << 20);
  std::memset(reg, 1, 64ull << 20);
  STEP("malloc+touch 64 MiB", hipSuccess);
  STEP("hipHostRegister it", hipHostRegister(reg, 64ull << 20, hipHostRegisterMapped));
  for (int k = 0; k < 3; ++k) STEP("hipFree 32 GiB", hipFree(big[k]));
  // a thread of its own (the multi-rank CLI's ranks are threads)
  for (int t = 0; t < 4; ++t) {
    std::thread th([&] {
      (void)hipSetDevice(0);
      hipStream_t ts;
      STEP("thread: stream", hipStreamCreateWithFlags(&ts, hipStreamNonBlocking));
      touch<<<1, 64, 0, ts>>>(d);
      STEP("thread:  first kernel", hipStreamSynchronize(ts));
      STEP("thread:  first H2D 4 MiB", hipMemcpyAsync(d, h, 4ull << 20, hipMemcpyHostToDevice, ts));
      STEP("thread:  sync", hipStreamSynchronize(ts));
    });
    th.join();
  }
  // eight threads copying at the same time, each on a stream of its own (the multi-rank
  // CLI's ranks stream their shards concurrently)
  {
    std::vector<std::thread> ths;
    std::atomic<int> ready{0};
    void* dd = nullptr;
    (void)hipMalloc(&dd, 8ull * (64ull << 20));
    for (int t = 0; t < 8; ++t)
      ths.emplace_back([&, t] {
        (void)hipSetDevice(0);
        hipStream_t ts;
        (void)hipStreamCreateWithFlags(&ts, hipStreamNonBlocking);
        void* hh = nullptr;
        (void)hipHostMalloc(&hh, 64ull << 20, hipHostMallocDefault);
        ready.fetch_add(1);
        while (ready.load() < 8) {
        }
        for (int k = 0; k < 16; ++k)
          (void)hipMemcpyAsync(static_cast<char*>(dd) + (size_t)t * (64ull << 20), hh, 64ull << 20,
                               hipMemcpyHostToDevice, ts);
        (void)hipStreamSynchronize(ts);
      });
    for (auto& th : ths) th.join();
    STEP("8 threads x concurrent H2D", hipSuccess);
  }
  // eight threads launching kernels at the same time, each on a stream of its own, with
  // an event per launch the host waits on (the rank threads' map loops do both)
  {
    std::vector<std::thread> ths;
    std::atomic<int> ready{0};
    for (int t = 0; t < 8; ++t)
      ths.emplace_back([&, t] {
        (void)hipSetDevice(0);
        hipStream_t ts;
        (void)hipStreamCreateWithFlags(&ts, hipStreamNonBlocking);
        hipEvent_t ev;
        (void)hipEventCreateWithFlags(&ev, hipEventDisableTiming);
        ready.fetch_add(1);
        while (ready.load() < 8) {
        }
        for (int k = 0; k < 2000; ++k) {
          touch<<<64, 256, 0, ts>>>(d + t);
          if (k % 16 == 0) {
            (void)hipEventRecord(ev, ts);
            (void)hipEventSynchronize(ev);
          }
        }
        (void)hipStreamSynchronize(ts);
      });
    for (auto& th : ths) th.join();
    STEP("8 threads x concurrent kernels", hipSuccess);
  }
  return 0;
}
