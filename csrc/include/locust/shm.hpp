// Shared host output of a distributed job (no rank-0 output funnel).
//
// Every rank writes its final key range straight into ONE host buffer at its global
// offset, over its own PCIe link, and rank 0 reads the finished output from it.  The
// buffer is a POSIX shared-memory segment that every rank maps itself -- the same code for
// ranks that are processes (torchrun, one GPU each) and ranks that are threads (the CLI's
// RCCL clique, loopback rehearsals): each mapping is registered with the HIP runtime
// separately (hipHostRegister, shard_engine.hip), so a GPU writes it directly.
//
// Naming and lifetime: "/locust-<group>-<gen>", where <group> is the communicator's
// agreed group id (Communicator::group_id) and <gen> counts the segment's regrowths.  Every
// rank computes the same sizes from collective data, so every rank creates-or-opens the
// same names at the same point of the job sequence; the first one creates it.  Each rank
// unlinks the name after the job in which it mapped it (the mapping stays valid), so a
// finished or crashed job leaves nothing in /dev/shm once its first job has completed.
//
// Layout: a 4 KiB header (one u64 completion stamp per rank) followed by the records.
#pragma once

#include <string>
#include <vector>

#include "locust/numa.hpp"

#include "locust/common.hpp"

namespace locust {

constexpr u64 kShmHeaderBytes = 4096;
constexpr int kShmMaxRanks = 512;  // stamps in the header

class ShmSegment {
 public:
  ShmSegment() = default;
  ShmSegment(const ShmSegment&) = delete;
  ShmSegment& operator=(const ShmSegment&) = delete;
  ~ShmSegment() { close(); }

  // Create-or-open `name` with `bytes` (every opener passes the same size) and map it.
  // `plan` (optional): NUMA slices applied to the mapping before its pages are reserved
  // (locust/numa.hpp place_slices; every opener passes the same plan).
  void open(const std::string& name, u64 bytes, const std::vector<NumaSlice>* plan = nullptr);
  // Remove the name (mappings stay valid); idempotent, and a name another rank removed
  // first is not an error.
  void unlink();
  void close();

  char* data() const { return base_; }
  u64 bytes() const { return bytes_; }
  const std::string& name() const { return name_; }
  bool linked() const { return linked_; }

  // Completion stamps (header) and records (after it).
  u64* stamps() const { return reinterpret_cast<u64*>(base_); }
  char* records() const { return base_ + kShmHeaderBytes; }

 private:
  char* base_ = nullptr;
  u64 bytes_ = 0;
  std::string name_;
  bool linked_ = false;
};

std::string shm_segment_name(u64 group, u32 gen);
// The next generation number of the group's shared output on this rank.  Per (group,
// rank) and process-wide: the engines of one rank (a job may switch engines) draw from one
// counter, so a name is never created twice -- a slow rank's late unlink can then never
// remove a newer segment of the same name.  Every rank draws at the same points of the
// job sequence, so the numbers agree.
u32 next_segment_gen(u64 group, int rank);
// Segment size for `records` output records of `record_bytes` each (whole pages).
u64 shm_segment_bytes(u64 records, u64 record_bytes);
// A fresh 64-bit group token (pid, clocks, an address and the OS entropy pool mixed).
u64 new_group_token();

}  // namespace locust
