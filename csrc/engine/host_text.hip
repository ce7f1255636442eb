// Pinned host text buffer (see HostText in locust/engine.hpp).
#include <cstdlib>

#include "locust/engine.hpp"
#include "locust/hip_check.hpp"

namespace locust {

HostText::HostText(u64 capacity) : cap_(capacity) {
  const u64 bytes = capacity + 64;  // room for the zero padding the upload appends
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) == hipSuccess && ndev > 0 &&
      hipHostMalloc(reinterpret_cast<void**>(&data_), bytes, hipHostMallocDefault) == hipSuccess) {
    pinned_ = true;
  } else {
    (void)hipGetLastError();
    data_ = static_cast<char*>(std::malloc(bytes));
    if (!data_) throw Error("HostText: cannot allocate " + std::to_string(bytes) + " bytes");
  }
}

HostText::~HostText() {
  if (!data_) return;
  if (pinned_)
    (void)hipHostFree(data_);
  else
    std::free(data_);
}

void HostText::set_size(u64 bytes, u64 lines) {
  LOCUST_CHECK_ARG(bytes <= cap_, "HostText: size exceeds capacity");
  size_ = bytes;
  lines_ = lines;
}

TextInput HostText::input(u64 first_line) const {
  TextInput in;
  in.data = data_;
  in.bytes = size_;
  in.num_lines = lines_;
  in.first_line = first_line;
  return in;
}

}  // namespace locust
