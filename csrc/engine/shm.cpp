// POSIX shared-memory segments of the distributed output (locust/shm.hpp).
#include "locust/shm.hpp"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <random>

namespace locust {

std::string shm_segment_name(u64 group, u32 gen) {
  char buf[64];
  std::snprintf(buf, sizeof(buf), "/locust-%016llx-%u", (unsigned long long)group, gen);
  return buf;
}

u32 next_segment_gen(u64 group, int rank) {
  static std::mutex mu;
  static std::map<std::pair<u64, int>, u32> gens;
  std::lock_guard<std::mutex> lk(mu);
  return ++gens[{group, rank}];
}

u64 shm_segment_bytes(u64 records, u64 record_bytes) {
  return align_up(kShmHeaderBytes + records * record_bytes, (u64)4096);
}

u64 new_group_token() {
  u64 x = (u64)::getpid() * 0x9E3779B97F4A7C15ull;
  x ^= (u64)std::chrono::steady_clock::now().time_since_epoch().count();
  x ^= (u64)std::chrono::system_clock::now().time_since_epoch().count() << 17;
  x ^= reinterpret_cast<u64>(&x);
  try {
    std::random_device rd;
    x ^= ((u64)rd() << 32) ^ (u64)rd();
  } catch (...) {
  }
  // splitmix finaliser: every bit of the inputs reaches every bit of the token
  x ^= x >> 30;
  x *= 0xBF58476D1CE4E5B9ull;
  x ^= x >> 27;
  x *= 0x94D049BB133111EBull;
  x ^= x >> 31;
  return x ? x : 1;
}

void ShmSegment::open(const std::string& name, u64 bytes, const std::vector<NumaSlice>* plan) {
  close();
  LOCUST_CHECK_ARG(bytes >= kShmHeaderBytes && bytes % 4096 == 0, "shm segment: bad size");
  const int fd = ::shm_open(name.c_str(), O_CREAT | O_RDWR, 0600);
  if (fd < 0)
    throw Error("shm_open " + name + " failed: " + std::strerror(errno));
  // every opener sets the same size: a no-op after the first
  struct stat st{};
  if (::fstat(fd, &st) != 0 || (u64)st.st_size != bytes) {
    if (::ftruncate(fd, (off_t)bytes) != 0) {
      const int e = errno;
      ::close(fd);
      throw Error("shm segment " + name + ": ftruncate to " + std::to_string(bytes) +
                  " B failed: " + std::strerror(e));
    }
  }
  void* p = ::mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  if (p == MAP_FAILED) {
    const int e = errno;
    ::close(fd);
    throw Error("shm segment " + name + ": mmap failed: " + std::strerror(e));
  }
  // NUMA slices first: shmem keeps them as the object's policy, so the reservation below
  // (whichever rank gets there first) already allocates each page on its slice's node
  if (plan && !plan->empty()) place_slices(p, *plan);
  // reserve the pages now: a full /dev/shm (a container's default is 64 MiB) is a clean
  // error here rather than a SIGBUS at the first write
  const int fe = ::posix_fallocate(fd, 0, (off_t)bytes);
  ::close(fd);
  if (fe != 0 && fe != EOPNOTSUPP && fe != EINVAL) {
    ::munmap(p, bytes);
    throw Error("shm segment " + name + ": cannot reserve " + std::to_string(bytes >> 20) +
                " MiB in /dev/shm: " + std::strerror(fe));
  }
  base_ = static_cast<char*>(p);
  bytes_ = bytes;
  name_ = name;
  linked_ = true;
}

void ShmSegment::unlink() {
  if (!linked_) return;
  (void)::shm_unlink(name_.c_str());  // ENOENT: another rank removed it first
  linked_ = false;
}

void ShmSegment::close() {
  if (base_) ::munmap(base_, bytes_);
  base_ = nullptr;
  bytes_ = 0;
  unlink();
  name_.clear();
}

}  // namespace locust
