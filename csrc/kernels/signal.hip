// Job-completion word for the host (lean job path, pipeline.hpp run()): one lane publishes
// the job's sequence number into host-mapped memory after everything before it on the
// stream has completed.  The host polls that word instead of hipStreamSynchronize --
// measured on the box (tools/micro/launch_lat.hip): 3 launches + sync 16.7 us per
// iteration, the same + polling a mapped word 11.2 us, a 3-node graph replay + sync 20.1 us.
#include <algorithm>

#include "locust/hip_check.hpp"
#include "locust/kernels.hpp"

namespace locust {
namespace {

__global__ void signal_host_kernel(u32* __restrict__ word, u32 value) {
  if (threadIdx.x == 0)  // vector store with system-scope release ordering
    __hip_atomic_store(word, value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Device buffer -> host-mapped buffer (its device alias), 8 B per lane (40-B records:
// sizes are multiples of 8), consecutive lanes on consecutive words (whole lines),
// grid-stride.  The fallback paths' results reach the mapped output this way: a
// hipMemcpyAsync into the fine-grained host buffer measured 7.3 ms for 9.7 MB on a cold
// engine (host-staged), a kernel's posted writes run at the link rate like the ordered
// kernel's own record stores.
__global__ __launch_bounds__(256) void copy_to_mapped_kernel(u64* __restrict__ dst,
                                                             const u64* __restrict__ src, u64 n) {
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x)
    dst[i] = src[i];
}

}  // namespace

void launch_copy_to_mapped(void* dst_mapped_dev, const void* src, u64 bytes, hipStream_t s) {
  LOCUST_CHECK_ARG(bytes % 8 == 0 && reinterpret_cast<uintptr_t>(dst_mapped_dev) % 8 == 0 &&
                       reinterpret_cast<uintptr_t>(src) % 8 == 0,
                   "copy_to_mapped: 8-byte aligned buffers and sizes");
  const u64 n = bytes / 8;
  if (!n) return;
  const u64 blocks = std::min<u64>(div_up(n, 256), 2048);
  copy_to_mapped_kernel<<<dim3((u32)blocks), dim3(256), 0, s>>>(
      reinterpret_cast<u64*>(dst_mapped_dev), reinterpret_cast<const u64*>(src), n);
  LOCUST_HIP_LAUNCH_CHECK();
}

void launch_signal_host(u32* word, u32 value, hipStream_t s) {
  signal_host_kernel<<<dim3(1), dim3(64), 0, s>>>(word, value);
}

// Loads this file's code object (one module per file) now rather than at its first launch.
void warm_module_signal() {
  hipFuncAttributes a;
  (void)hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&signal_host_kernel));
}

}  // namespace locust
