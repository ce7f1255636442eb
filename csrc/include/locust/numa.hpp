// NUMA placement of GPU ranks (see csrc/engine/numa.cpp, locust_amd/parallel/numa.py).
#pragma once

#include <string>
#include <vector>

#include "locust/common.hpp"

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

// ---- page placement of the shared distributed output ----
// The output segment is [header | region 0 | region 1 | ...]; in every region rank p writes
// its key range, and the sample sort balances the ranges, so slice p of each region (its
// p-th 1/P, page aligned) is placed on rank p's node and the header (the stamps the root
// polls) on rank 0's.  Adjacent slices of one node merge; a rank of unknown node (-1)
// leaves its slice to the default policy.
struct NumaSlice {
  u64 offset = 0, bytes = 0;  // page-aligned byte range of the segment
  int node = -1;
};
std::vector<NumaSlice> plan_rank_slices(u64 header_bytes, u64 region_bytes, u32 regions,
                                        const std::vector<int>& rank_nodes, u64 page = 4096);
// true when the ranks span more than one known node (placement has something to do).
bool spans_numa_nodes(const std::vector<int>& rank_nodes);
// mbind(MPOL_PREFERRED) of each slice of the mapping at base, before its pages exist
// (shmem applies it as the object's shared policy: whichever rank populates a page puts it
// on the slice's node).  Returns the slices bound; failures are logged, not fatal.
int place_slices(void* base, const std::vector<NumaSlice>& plan);
// The node holding the page at p (touched), or -1 (get_mempolicy).
int page_node(const void* p);

}  // namespace locust
