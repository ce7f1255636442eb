// NUMA placement of GPU ranks (see csrc/engine/numa.cpp, locust_amd/parallel/numa.py).
#pragma once

#include <string>
#include <vector>

namespace locust {

struct GpuPlacement {
  std::string bdf;        // PCI address, lower case (domain:bus:dev.fn)
  int numa_node = -1;     // -1: unknown (no binding)
  std::vector<int> cpus;  // the node's CPUs
};

// "0-3,8,10-11" -> {0, 1, 2, 3, 8, 10, 11} (empty on a malformed list).
std::vector<int> parse_cpulist(const std::string& text);
// The NUMA node and CPUs of the GPU at PCI address `bdf`, from sysfs under `sys_root`.
GpuPlacement placement_for_bdf(const std::string& bdf, const std::string& sys_root = "/sys");
// Pins the calling thread to p.cpus (those of them it may use); false if nothing to do.
bool bind_thread_to(const GpuPlacement& p);
// LOCUST_NUMA=0 switches placement off.
bool numa_enabled();

}  // namespace locust
