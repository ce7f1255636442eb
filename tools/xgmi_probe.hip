// Inter-GPU data-plane probe for the node `MapReduce --gpus N` runs on:
//   * every ordered device pair: can-access-peer, then a 256 MiB peer copy (hipMemcpyPeerAsync
//     after hipDeviceEnablePeerAccess) -- GB/s, or "staged" when the runtime has no direct path;
//   * one process, an RCCL clique over all visible GPUs (ncclCommInitAll, as the CLI's
//     `--comm rccl`): ncclAllToAll bus bandwidth from 1 MiB to 1 GiB per rank, and the
//     fixed-slot all-to-all of the shuffle at its synth1m size.
// On a one-GPU box the pair table is empty and the all-to-all is one rank's self copy (the
// code path still runs).  Build + run (one call):
//   hipcc --offload-arch=gfx950 -O2 tools/xgmi_probe.hip -lrccl -o build/xgmi_probe
//   ./build/xgmi_probe [max_mib]
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                   \
    }                                                                                 \
  } while (0)
#define NK(x)                                                                         \
  do {                                                                                \
    ncclResult_t r_ = (x);                                                            \
    if (r_ != ncclSuccess) {                                                          \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, ncclGetErrorString(r_)); \
      std::exit(1);                                                                   \
    }                                                                                 \
  } while (0)

int main(int argc, char** argv) {
  const size_t max_mib = argc > 1 ? (size_t)std::atoi(argv[1]) : 1024;
  int n = 0;
  CK(hipGetDeviceCount(&n));
  std::printf("visible GPUs: %d\n", n);
  // ---- peer copies ----
  const size_t pbytes = 256ull << 20;
  for (int a = 0; a < n; ++a)
    for (int b = 0; b < n; ++b) {
      if (a == b) continue;
      int can = 0;
      CK(hipDeviceCanAccessPeer(&can, a, b));
      void *src = nullptr, *dst = nullptr;
      CK(hipSetDevice(b));
      CK(hipMalloc(&dst, pbytes));
      CK(hipSetDevice(a));
      CK(hipMalloc(&src, pbytes));
      if (can) {
        const hipError_t e = hipDeviceEnablePeerAccess(b, 0);
        if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) CK(e);
        (void)hipGetLastError();
      }
      hipStream_t s;
      CK(hipStreamCreate(&s));
      hipEvent_t e0, e1;
      CK(hipEventCreate(&e0));
      CK(hipEventCreate(&e1));
      CK(hipMemcpyPeerAsync(dst, b, src, a, pbytes, s));  // warm
      CK(hipEventRecord(e0, s));
      for (int k = 0; k < 5; ++k) CK(hipMemcpyPeerAsync(dst, b, src, a, pbytes, s));
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      std::printf("peer copy GPU %d -> GPU %d: %s, %.1f GB/s\n", a, b,
                  can ? "direct" : "staged (no peer access)", 5.0 * pbytes / (ms * 1e-3) / 1e9);
      CK(hipStreamDestroy(s));
      CK(hipFree(src));
      CK(hipSetDevice(b));
      CK(hipFree(dst));
    }
  // ---- RCCL clique all-to-all ----
  std::vector<int> devs(n);
  for (int i = 0; i < n; ++i) devs[i] = i;
  std::vector<ncclComm_t> comms(n);
  NK(ncclCommInitAll(comms.data(), n, devs.data()));
  std::vector<hipStream_t> st(n);
  std::vector<char*> sb(n), rb(n);
  const size_t maxb = max_mib << 20;
  for (int i = 0; i < n; ++i) {
    CK(hipSetDevice(i));
    CK(hipStreamCreate(&st[i]));
    CK(hipMalloc(&sb[i], maxb));
    CK(hipMalloc(&rb[i], maxb));
  }
  auto run = [&](size_t per_rank, int iters) {
    const size_t chunk = per_rank / n;  // bytes to each peer
    NK(ncclGroupStart());
    for (int i = 0; i < n; ++i) NK(ncclAllToAll(sb[i], rb[i], chunk, ncclUint8, comms[i], st[i]));
    NK(ncclGroupEnd());
    for (int i = 0; i < n; ++i) {
      CK(hipSetDevice(i));
      CK(hipStreamSynchronize(st[i]));
    }
    hipEvent_t e0, e1;
    CK(hipSetDevice(0));
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, st[0]));
    for (int k = 0; k < iters; ++k) {
      NK(ncclGroupStart());
      for (int i = 0; i < n; ++i) NK(ncclAllToAll(sb[i], rb[i], chunk, ncclUint8, comms[i], st[i]));
      NK(ncclGroupEnd());
    }
    CK(hipSetDevice(0));
    CK(hipEventRecord(e1, st[0]));
    for (int i = 0; i < n; ++i) {
      CK(hipSetDevice(i));
      CK(hipStreamSynchronize(st[i]));
    }
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double t = ms * 1e-3 / iters;
    // bus bandwidth as nccl-tests defines it for all-to-all: bytes * (n - 1) / n per rank
    const double bus = n > 1 ? per_rank * (double)(n - 1) / n / t / 1e9 : per_rank / t / 1e9;
    std::printf("ncclAllToAll %d ranks, %8.2f MiB per rank: %8.3f ms, bus %.1f GB/s\n", n,
                per_rank / 1048576.0, t * 1e3, bus);
  };
  for (size_t mib = 1; mib <= max_mib; mib *= 4) run(mib << 20, mib >= 256 ? 5 : 20);
  // the shuffle's fixed-slot all-to-all at synth1m (~202K distinct keys x 40 B over the ranks)
  run(((size_t)202645 * 40 / n + 4095) / 4096 * 4096 * n, 50);
  for (int i = 0; i < n; ++i) NK(ncclCommDestroy(comms[i]));
  return 0;
}
