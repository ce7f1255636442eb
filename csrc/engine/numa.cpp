// NUMA placement of the in-process clique's rank threads (the
// multi-process ranks are placed by locust_amd/parallel/numa.py before their first GPU
// call).  A rank thread pins itself to the CPUs of its GPU's NUMA node before it builds
// its engine, so the engine's pinned buffers -- the rank's copy of its shard among them --
// are first touched on that node and its H2D never crosses the socket link.
#include "locust/numa.hpp"

#include <pthread.h>
#include <sched.h>

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

}  // namespace locust
