// Locust-MI355X: common error handling, logging and small utilities.
//
// The reference checks no CUDA/HIP return code anywhere (SURVEY.md §4, §5.3;
// /root/reference/MapReduce/src/main.cu:393-472).  Every HIP and RCCL call in this
// framework goes through LOCUST_HIP_CHECK / LOCUST_RCCL_CHECK, which throw a
// rank-tagged locust::Error instead of continuing on garbage.
#pragma once

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <string>

#ifndef LOCUST_HD
#if defined(__HIPCC__)
#define LOCUST_HD __host__ __device__
#else
#define LOCUST_HD
#endif
#endif

namespace locust {

using u8 = uint8_t;
using u16 = uint16_t;
using u32 = uint32_t;
using u64 = uint64_t;
using i64 = int64_t;
using i32 = int32_t;

class Error : public std::runtime_error {
 public:
  explicit Error(const std::string& what) : std::runtime_error(what) {}
};

// Rank tag used in error messages and logs; set by the distributed driver.
int& log_rank();

enum class LogLevel : int { kError = 0, kWarn = 1, kInfo = 2, kDebug = 3 };
LogLevel log_level();  // from LOCUST_LOG=error|warn|info|debug (default warn)
void log_msg(LogLevel lvl, const char* fmt, ...) __attribute__((format(printf, 2, 3)));

#define LOCUST_LOG_INFO(...) ::locust::log_msg(::locust::LogLevel::kInfo, __VA_ARGS__)
#define LOCUST_LOG_DEBUG(...) ::locust::log_msg(::locust::LogLevel::kDebug, __VA_ARGS__)
#define LOCUST_LOG_WARN(...) ::locust::log_msg(::locust::LogLevel::kWarn, __VA_ARGS__)

[[noreturn]] void throw_error(const char* file, int line, const std::string& msg);

#define LOCUST_CHECK_ARG(cond, msg)                                   \
  do {                                                                \
    if (!(cond)) ::locust::throw_error(__FILE__, __LINE__, (msg));    \
  } while (0)

LOCUST_HD inline u64 div_up(u64 a, u64 b) { return (a + b - 1) / b; }
LOCUST_HD inline u64 align_up(u64 a, u64 b) { return div_up(a, b) * b; }

// Fault injection: LOCUST_FAULT="<rank>:<stage>" makes the given rank
// throw at the start of <stage> (map|shuffle|reduce|gather) so tests can verify that a
// failing rank turns into a clean, agreed-upon job failure instead of a hang.
bool fault_injected(int rank, const char* stage);
// The distributed job stage this process last entered (a string literal), and how many it
// has entered: read by a watchdog thread (bench.py) while the job may be stuck in it.
void set_current_stage(const char* stage);
const char* current_stage();
u64 stages_entered();

// Monotonic host clock in nanoseconds.
u64 now_ns();
// now_ns() when this library's static initialisation ran (the process's start-up split:
// loader + the HIP runtime's static init before it, the rest of static init after).
u64 library_init_ns();
// Resident host memory of this process, kB: VmRSS (peak = false) or VmHWM (peak = true).
u64 process_rss_kb(bool peak = false);
// "rss N kB (anon A, file F, shmem S; peak P)" from /proc/self/status (debug logs)
std::string process_rss_breakdown();

}  // namespace locust
