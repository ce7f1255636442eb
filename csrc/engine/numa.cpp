// NUMA placement of the in-process clique's rank threads (the
// multi-process ranks are placed by locust_amd/parallel/numa.py before their first GPU
// call).  A rank thread pins itself to the CPUs of its GPU's NUMA node before it builds
// its engine, so the engine's pinned buffers -- the rank's copy of its shard among them --
// are first touched on that node and its H2D never crosses the socket link.
#include "locust/numa.hpp"

#include <pthread.h>
#include <sched.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstring>

#include <cstdio>
#include <fstream>
#include <sstream>

#include "locust/common.hpp"

namespace locust {

std::vector<int> parse_cpulist(const std::string& text) {
  std::vector<int> out;
  std::stringstream ss(text);
  std::string part;
  while (std::getline(ss, part, ',')) {
    size_t a = part.find_first_not_of(" \t\n"), b = part.find_last_not_of(" \t\n");
    if (a == std::string::npos) continue;
    part = part.substr(a, b - a + 1);
    const size_t dash = part.find('-');
    try {
      if (dash == std::string::npos) {
        out.push_back(std::stoi(part));
      } else {
        const int lo = std::stoi(part.substr(0, dash)), hi = std::stoi(part.substr(dash + 1));
        for (int c = lo; c <= hi; ++c) out.push_back(c);
      }
    } catch (const std::exception&) {
      return {};
    }
  }
  return out;
}

namespace {
std::string read_file(const std::string& path) {
  std::ifstream f(path);
  if (!f) return {};
  std::stringstream ss;
  ss << f.rdbuf();
  return ss.str();
}
}  // namespace

GpuPlacement placement_for_bdf(const std::string& bdf_in, const std::string& sys_root) {
  GpuPlacement p;
  std::string bdf = bdf_in;
  for (char& c : bdf) c = (char)std::tolower((unsigned char)c);
  p.bdf = bdf;
  const std::string node = read_file(sys_root + "/bus/pci/devices/" + bdf + "/numa_node");
  try {
    p.numa_node = node.empty() ? -1 : std::stoi(node);
  } catch (const std::exception&) {
    p.numa_node = -1;
  }
  if (p.numa_node >= 0)
    p.cpus = parse_cpulist(
        read_file(sys_root + "/devices/system/node/node" + std::to_string(p.numa_node) + "/cpulist"));
  return p;
}

bool bind_thread_to(const GpuPlacement& p) {
  if (p.cpus.empty()) return false;
  cpu_set_t allowed, set;
  CPU_ZERO(&allowed);
  CPU_ZERO(&set);
  if (sched_getaffinity(0, sizeof(allowed), &allowed) != 0) return false;
  int n = 0;
  for (int c : p.cpus)
    if (c >= 0 && c < CPU_SETSIZE && CPU_ISSET(c, &allowed)) {
      CPU_SET(c, &set);
      ++n;
    }
  if (!n) return false;
  return pthread_setaffinity_np(pthread_self(), sizeof(set), &set) == 0;
}

bool numa_enabled() {
  const char* e = std::getenv("LOCUST_NUMA");
  return !(e && e[0] == '0');
}

bool spans_numa_nodes(const std::vector<int>& rank_nodes) {
  int first = -1;
  for (int n : rank_nodes) {
    if (n < 0) continue;
    if (first < 0) first = n;
    else if (n != first) return true;
  }
  return false;
}

std::vector<NumaSlice> plan_rank_slices(u64 header_bytes, u64 region_bytes, u32 regions,
                                        const std::vector<int>& rank_nodes, u64 page) {
  std::vector<NumaSlice> out;
  const u64 P = rank_nodes.size();
  if (!P || !page) return out;
  auto add = [&](u64 lo, u64 hi, int node) {
    lo = align_up(lo, page);  // a page straddling two slices goes to the later one
    hi = align_up(hi, page);
    if (hi <= lo || node < 0) return;
    if (!out.empty() && out.back().node == node && out.back().offset + out.back().bytes == lo)
      out.back().bytes += hi - lo;
    else
      out.push_back({lo, hi - lo, node});
  };
  // the header page(s) and region boundaries stay whole pages: [0, header) -> rank 0
  add(0, header_bytes, rank_nodes[0]);
  for (u32 k = 0; k < regions; ++k) {
    const u64 base = header_bytes + (u64)k * region_bytes;
    for (u64 p = 0; p < P; ++p)
      add(base + region_bytes * p / P, base + region_bytes * (p + 1) / P, rank_nodes[p]);
  }
  return out;
}

namespace {
constexpr int kMpolPreferred = 1;  // <linux/mempolicy.h>; no libnuma in this image
constexpr int kMpolFNode = 1 << 0, kMpolFAddr = 1 << 1;
constexpr int kMaskWords = 16;     // nodes 0..1023
}  // namespace

int place_slices(void* base, const std::vector<NumaSlice>& plan) {
  int placed = 0;
  for (const NumaSlice& s : plan) {
    if (s.node < 0 || s.node >= 64 * kMaskWords || !s.bytes) continue;
    unsigned long mask[kMaskWords] = {0};
    mask[s.node / 64] = 1ul << (s.node % 64);
    // maxnode counts bits + 1 (the kernel drops the last one)
    const long r = ::syscall(SYS_mbind, static_cast<char*>(base) + s.offset, (unsigned long)s.bytes,
                             kMpolPreferred, mask, (unsigned long)(64 * kMaskWords + 1), 0u);
    if (r != 0) {
      LOCUST_LOG_WARN("mbind of %llu B at +%llu to NUMA node %d failed: %s",
                      (unsigned long long)s.bytes, (unsigned long long)s.offset, s.node,
                      std::strerror(errno));
      continue;
    }
    ++placed;
    LOCUST_LOG_INFO("shared output bytes [%llu, %llu) preferred on NUMA node %d",
                    (unsigned long long)s.offset, (unsigned long long)(s.offset + s.bytes), s.node);
  }
  return placed;
}

int page_node(const void* p) {
  int node = -1;
  const long r = ::syscall(SYS_get_mempolicy, &node, nullptr, 0ul, const_cast<void*>(p),
                           (unsigned long)(kMpolFNode | kMpolFAddr));
  return r == 0 ? node : -1;
}

}  // namespace locust
