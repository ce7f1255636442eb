// roctx range helpers (see locust/trace.hpp).
#include "locust/trace.hpp"

#include <rocprofiler-sdk-roctx/roctx.h>

#include <cstdlib>
#include <cstring>

namespace locust {

bool roctx_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("LOCUST_ROCTX");
    return !(e && std::strcmp(e, "0") == 0);
  }();
  return on;
}

void roctx_push(const char* name) { roctxRangePushA(name); }
void roctx_pop() { roctxRangePop(); }

}  // namespace locust
