// HIP / RCCL error checking.  Included only by translation units that talk to the
// HIP runtime, so the CPU-only parts of the framework do not depend on it.
#pragma once

#include <hip/hip_runtime.h>

#include <string>

#include "locust/common.hpp"

#define LOCUST_HIP_CHECK(expr)                                                        \
  do {                                                                                \
    hipError_t _e = (expr);                                                           \
    if (_e != hipSuccess)                                                             \
      ::locust::throw_error(__FILE__, __LINE__,                                       \
                            std::string("HIP error ") + hipGetErrorName(_e) + ": " +  \
                                hipGetErrorString(_e) + " in `" #expr "`");           \
  } while (0)

// Checks for asynchronous launch errors right after a kernel launch.
#define LOCUST_HIP_LAUNCH_CHECK() LOCUST_HIP_CHECK(hipGetLastError())
