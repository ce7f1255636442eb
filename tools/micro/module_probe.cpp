// What loading each kernel file's code object costs in a fresh process (the engine's
// "modules" phase, 8 ms in total: warm_kernel_modules at construction).  Times every
// warm_module_X() in turn after the runtime and the device context are up.
// Build: make module_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

#include "locust/kernels.hpp"

int main() {
  if (hipSetDevice(0) != hipSuccess || hipFree(nullptr) != hipSuccess) return 2;
  struct Mod {
    const char* name;
    void (*fn)();
  } mods[] = {{"dict", locust::warm_module_dict},         {"exchange", locust::warm_module_exchange},
              {"map", locust::warm_module_map},           {"merge", locust::warm_module_merge},
              {"partplan", locust::warm_module_partplan}, {"psort", locust::warm_module_psort},
              {"radix_sort", locust::warm_module_radix_sort}, {"reduce", locust::warm_module_reduce},
              {"shuffle", locust::warm_module_shuffle},   {"signal", locust::warm_module_signal},
              {"tokenize", locust::warm_module_tokenize}};
  double total = 0;
  for (const Mod& m : mods) {
    const auto t0 = std::chrono::steady_clock::now();
    m.fn();
    const double ms =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    total += ms;
    std::printf("%-11s %6.2f ms\n", m.name, ms);
  }
  std::printf("%-11s %6.2f ms\n", "total", total);
  return 0;
}
