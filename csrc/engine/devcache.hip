// Process-wide device block cache; see locust/devcache.hpp.
#include "locust/devcache.hpp"

#include <hip/hip_runtime.h>
#include <sys/mman.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <mutex>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "locust/common.hpp"
#include "locust/hip_check.hpp"

namespace locust {
namespace {

constexpr size_t kPage = 2ull << 20;

struct Block {
  int device;
  void* p;
  size_t bytes;
};

struct Cache {
  std::mutex mu;
  std::vector<Block> free;
  size_t held = 0;
  const bool on = [] {
    const char* e = std::getenv("LOCUST_DEV_CACHE");
    return !(e && e[0] == '0');
  }();
  // Bytes of idle blocks kept.  The cache is per process: with several rank processes on
  // one GPU (LOCAL_WORLD_SIZE ranks on fewer devices, the tcpdev rehearsals) one rank's
  // idle blocks could starve another's hipMalloc, so the default shares 64 GB between the
  // processes per device.  LOCUST_DEV_CACHE_GB overrides it for this process.
  const size_t cap = [] {
    if (const char* e = std::getenv("LOCUST_DEV_CACHE_GB")) {
      const double gb = std::atof(e);
      return (size_t)(gb > 0 ? gb * 1e9 : 0);
    }
    int per_dev = 1;
    if (const char* w = std::getenv("LOCAL_WORLD_SIZE")) {
      int ndev = 0;
      // device_count is safe before the runtime is initialised (no GPU context)
      if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) ndev = 1;
      per_dev = std::max(1, (std::atoi(w) + ndev - 1) / ndev);
    }
    return (size_t)(64e9 / per_dev);
  }();
};

Cache& cache() {
  static Cache* c = new Cache();  // never destroyed: blocks may be freed at exit
  return *c;
}

int current_device() {
  int d = 0;
  (void)hipGetDevice(&d);
  return d;
}

}  // namespace

void* dev_block_alloc(size_t bytes, size_t* got) {
  const size_t want = (bytes + kPage - 1) / kPage * kPage;
  const int dev = current_device();
  Cache& c = cache();
  if (c.on) {
    std::lock_guard<std::mutex> lk(c.mu);
    size_t best = c.free.size();
    for (size_t i = 0; i < c.free.size(); ++i) {
      const Block& b = c.free[i];
      if (b.device == dev && b.bytes >= want && b.bytes <= want + want / 4 &&
          (best == c.free.size() || b.bytes < c.free[best].bytes))
        best = i;
    }
    if (best < c.free.size()) {
      const Block b = c.free[best];
      c.free.erase(c.free.begin() + (long)best);
      c.held -= b.bytes;
      if (got) *got = b.bytes;
      LOCUST_LOG_DEBUG("device block %zu MB reused (device %d)", b.bytes >> 20, dev);
      return b.p;
    }
  }
  void* p = nullptr;
  hipError_t e = hipMalloc(&p, want);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    dev_block_trim();
    LOCUST_HIP_CHECK(hipMalloc(&p, want));
  }
  if (got) *got = want;
  return p;
}

void dev_block_free(void* p, size_t bytes) {
  if (!p) return;
  Cache& c = cache();
  // the block's own device (an engine may be destroyed on another thread or device than
  // the one that made it: clique ranks)
  int dev = current_device();
  hipPointerAttribute_t a{};
  if (hipPointerGetAttributes(&a, p) == hipSuccess)
    dev = a.device;
  else
    (void)hipGetLastError();
  if (c.on) {
    std::lock_guard<std::mutex> lk(c.mu);
    if (c.held + bytes <= c.cap) {
      c.free.push_back(Block{dev, p, bytes});
      c.held += bytes;
      return;
    }
  }
  const int cur = current_device();
  (void)hipSetDevice(dev);
  (void)hipFree(p);
  (void)hipSetDevice(cur);
}

void dev_block_trim() {
  Cache& c = cache();
  std::vector<Block> blocks;
  {
    std::lock_guard<std::mutex> lk(c.mu);
    blocks.swap(c.free);
    c.held = 0;
  }
  int cur = current_device();
  for (const Block& b : blocks) {
    (void)hipSetDevice(b.device);
    (void)hipFree(b.p);
  }
  (void)hipSetDevice(cur);
}

size_t dev_block_cached(size_t* bytes) {
  Cache& c = cache();
  std::lock_guard<std::mutex> lk(c.mu);
  if (bytes) *bytes = c.held;
  return c.free.size();
}

namespace {

// pinned_alloc's huge-page buffers: base -> mapped length (never destroyed: engines may be
// freed from static destructors or left to the process exit)
struct HugePinned {
  std::mutex mu;
  std::unordered_map<void*, size_t> len;
};
HugePinned& huge_pinned() {
  static HugePinned* h = new HugePinned;
  return *h;
}

constexpr size_t kHugePinMin = 4ull << 20;

void* huge_pinned_alloc(size_t bytes, unsigned flags) {
  static const bool on = [] {
    const char* e = std::getenv("LOCUST_HUGE_PIN");
    return !(e && e[0] == '0');
  }();
  if (!on) return nullptr;
  const size_t n = (bytes + kPage - 1) / kPage * kPage;
  void* m = ::mmap(nullptr, n, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  if (m == MAP_FAILED) return nullptr;
  (void)::madvise(m, n, MADV_HUGEPAGE);
  // a child process (subprocess spawns) must not share these pages copy-on-write: a write
  // by this process before the child's exec would move the page under the device mapping
  (void)::madvise(m, n, MADV_DONTFORK);
  std::memset(m, 0, n);  // first touch: the pages exist (huge where THP allows) on this node
  // registered memory is fine-grained (coherent) unless registered coarse-grained, so the
  // mapped + coherent result buffers the kernels write over PCIe may take this path too
  const unsigned rf = hipHostRegisterMapped | ((flags & hipHostMallocPortable) ? hipHostRegisterPortable : 0u);
  if (hipHostRegister(m, n, rf) != hipSuccess) {
    (void)hipGetLastError();
    ::munmap(m, n);
    return nullptr;
  }
  HugePinned& h = huge_pinned();
  std::lock_guard<std::mutex> lk(h.mu);
  h.len[m] = n;
  return m;
}

}  // namespace

void pinned_free(void* p) {
  if (!p) return;
  size_t n = 0;
  {
    HugePinned& h = huge_pinned();
    std::lock_guard<std::mutex> lk(h.mu);
    auto it = h.len.find(p);
    if (it != h.len.end()) {
      n = it->second;
      h.len.erase(it);
    }
  }
  if (n) {
    (void)hipHostUnregister(p);
    ::munmap(p, n);
  } else {
    (void)hipHostFree(p);
  }
}

void* pinned_alloc(size_t bytes, unsigned flags, const char* what) {
  static std::atomic<unsigned long long> total{0};
  constexpr unsigned kHugeFlags = hipHostMallocMapped | hipHostMallocCoherent | hipHostMallocPortable;
  // (small buffers too measured no different: the map's zero-copy staging of whole Hamlet
  // from 2 MiB pages, profiles/r6/map/huge_text_ab.txt)
  void* p = (flags & ~kHugeFlags) == 0 && bytes >= kHugePinMin ? huge_pinned_alloc(bytes, flags) : nullptr;
  if (!p) LOCUST_HIP_CHECK(hipHostMalloc(&p, bytes, flags));
  const unsigned long long t = total.fetch_add(bytes) + bytes;
  if (bytes >= (1u << 20))
    LOCUST_LOG_DEBUG("pinned %.1f MiB: %s (allocated so far %.1f MiB)", bytes / 1048576.0, what,
                     t / 1048576.0);
  return p;
}

}  // namespace locust
