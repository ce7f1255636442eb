// Shared host-side pieces: logging, errors, env config, tokenizer oracle, result checks.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <malloc.h>

#include <cstdio>
#include <cstdarg>
#include <cstring>
#include <string>
#include <thread>

#include "locust/config.hpp"
#include "locust/dstring.hpp"
#include "locust/engine.hpp"

namespace locust {

int& log_rank() {
  static thread_local int r = -1;
  return r;
}

LogLevel log_level() {
  static LogLevel lvl = [] {
    const char* e = std::getenv("LOCUST_LOG");
    if (!e) return LogLevel::kWarn;
    std::string s(e);
    if (s == "error") return LogLevel::kError;
    if (s == "info") return LogLevel::kInfo;
    if (s == "debug") return LogLevel::kDebug;
    return LogLevel::kWarn;
  }();
  return lvl;
}

void log_msg(LogLevel lvl, const char* fmt, ...) {
  if ((int)lvl > (int)log_level()) return;
  static const char* names[] = {"ERROR", "WARN", "INFO", "DEBUG"};
  char buf[2048];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  // stderr only: stdout stays byte-compatible with the reference.
  if (log_rank() >= 0)
    std::fprintf(stderr, "[locust %s r%d] %s\n", names[(int)lvl], log_rank(), buf);
  else
    std::fprintf(stderr, "[locust %s] %s\n", names[(int)lvl], buf);
}

void throw_error(const char* file, int line, const std::string& msg) {
  std::string where = std::string(file) + ":" + std::to_string(line);
  std::string rank = log_rank() >= 0 ? ("rank " + std::to_string(log_rank()) + ": ") : "";
  throw Error(rank + msg + " (" + where + ")");
}

namespace {
std::atomic<const char*> g_stage{"none"};
std::atomic<u64> g_stages{0};
}  // namespace
void set_current_stage(const char* stage) {
  g_stage.store(stage, std::memory_order_relaxed);
  g_stages.fetch_add(1, std::memory_order_relaxed);
}
const char* current_stage() { return g_stage.load(std::memory_order_relaxed); }
u64 stages_entered() { return g_stages.load(std::memory_order_relaxed); }

bool fault_injected(int rank, const char* stage) {
  const char* e = std::getenv("LOCUST_FAULT");
  if (!e || !*e) return false;
  std::string s(e);
  auto colon = s.find(':');
  if (colon == std::string::npos) return false;
  int r = std::atoi(s.substr(0, colon).c_str());
  if (r != rank) return false;
  const std::string what = s.substr(colon + 1);
  if (what == std::string("hang_") + stage) {
    // a rank that stops answering (the SCALE watchdog's test, tests/test_scale_ready.py):
    // it never returns, like a peer stuck in a collective
    std::fprintf(stderr, "locust: rank %d: injected hang (LOCUST_FAULT) in stage '%s'\n", rank,
                 stage);
    std::fflush(stderr);
    for (;;) std::this_thread::sleep_for(std::chrono::seconds(1));
  }
  return what == stage;
}

namespace {
const u64 g_library_init_ns = now_ns();
}  // namespace
u64 library_init_ns() { return g_library_init_ns; }

u64 now_ns() {
  return (u64)std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

u64 process_rss_kb(bool peak) {
  std::FILE* f = std::fopen("/proc/self/status", "r");
  if (!f) return 0;
  char line[256];
  unsigned long long kb = 0;
  const char* key = peak ? "VmHWM: %llu kB" : "VmRSS: %llu kB";
  while (std::fgets(line, sizeof(line), f))
    if (std::sscanf(line, key, &kb) == 1) break;
  std::fclose(f);
  return kb;
}

std::string process_rss_breakdown() {
  std::FILE* f = std::fopen("/proc/self/status", "r");
  if (!f) return "rss unknown";
  char line[256];
  unsigned long long rss = 0, hwm = 0, anon = 0, file = 0, shmem = 0, v = 0;
  while (std::fgets(line, sizeof(line), f)) {
    if (std::sscanf(line, "VmRSS: %llu kB", &v) == 1) rss = v;
    if (std::sscanf(line, "VmHWM: %llu kB", &v) == 1) hwm = v;
    if (std::sscanf(line, "RssAnon: %llu kB", &v) == 1) anon = v;
    if (std::sscanf(line, "RssFile: %llu kB", &v) == 1) file = v;
    if (std::sscanf(line, "RssShmem: %llu kB", &v) == 1) shmem = v;
  }
  std::fclose(f);
  // the heap's share of anon: bytes in use (arena + mmap'ed chunks) and the arenas' size
  const struct mallinfo2 mi = mallinfo2();
  char buf[256];
  std::snprintf(buf, sizeof(buf),
                "rss %llu kB (anon %llu, file %llu, shmem %llu; peak %llu; malloc in use %llu kB, "
                "arenas %llu kB, mmap'ed %llu kB)",
                rss, anon, file, shmem, hwm,
                (unsigned long long)((mi.uordblks + mi.hblkhd) >> 10),
                (unsigned long long)(mi.arena >> 10), (unsigned long long)(mi.hblkhd >> 10));
  return buf;
}

void apply_env_overrides(JobConfig& cfg) {
  if (const char* e = std::getenv("LOCUST_CHECK")) cfg.check = std::atoi(e) != 0;
  if (const char* e = std::getenv("LOCUST_REDUCE_PATH")) {
    std::string s(e);
    if (s == "lds") cfg.reduce_path = ReducePath::kLds;
    if (s == "global") cfg.reduce_path = ReducePath::kGlobal;
  }
  if (const char* e = std::getenv("LOCUST_MAP_PATH")) {
    std::string s(e);
    if (s == "compat") cfg.map_path = MapPath::kCompat;
    if (s == "fast") cfg.map_path = MapPath::kFast;
  }
  if (const char* e = std::getenv("LOCUST_SORT")) {
    std::string s(e);
    if (s == "radix") cfg.sort_path = SortPath::kRadix;
    if (s == "dict") cfg.sort_path = SortPath::kDict;
  }
  if (const char* e = std::getenv("LOCUST_CHUNK_MB")) cfg.chunk_bytes = (u64)std::atoll(e) << 20;
  if (const char* e = std::getenv("LOCUST_ZERO_COPY")) cfg.zero_copy_text = std::atoi(e);
  if (const char* e = std::getenv("LOCUST_GRAPH")) cfg.graph = std::atoi(e);
}

const char* to_string(ReducePath p) { return p == ReducePath::kLds ? "lds" : "global"; }
const char* to_string(MapPath p) { return p == MapPath::kCompat ? "compat" : "fast"; }
const char* to_string(SortPath p) { return p == SortPath::kRadix ? "radix" : "dict"; }

int tokenize_line(const char* line, u64 len, const JobConfig& cfg, std::vector<PackedKey>* out,
                  u64* truncated) {
  // The reference works on a NUL-terminated copy (main.cu:55-59); text after an embedded
  // NUL is invisible to strtok_r, exactly as here.
  std::string buf(line, len);
  char* save = nullptr;
  char* tok = d_strtok_r(&buf[0], cfg.delimiters.c_str(), &save);
  int count = 0;
  int dropped = 0;
  while (tok != nullptr) {
    if (count >= cfg.emits_per_line) {
      dropped = 1;
      break;
    }
    int n = d_strlen(tok);
    if (n > cfg.max_key_len) {
      if (truncated) ++*truncated;
      n = cfg.max_key_len;
    }
    PackedKey k;
    pack_key(tok, n, k.w);
    out->push_back(k);
    ++count;
    tok = d_strtok_r(nullptr, cfg.delimiters.c_str(), &save);
  }
  return dropped;
}

void entries_from_sorted_tokens(const PackedKey* sorted, u64 n, std::vector<WordCountEntry>* out) {
  out->clear();
  u64 i = 0;
  while (i < n) {
    u64 j = i + 1;
    while (j < n && key_compare(sorted[j].w, sorted[i].w) == 0) ++j;
    out->push_back(WordCountEntry{sorted[i], j - i});
    i = j;
  }
}

// LOCUST_CHECK invariants: keys strictly increasing, no empty runs,
// counts sum to the token count.  (Runs are contiguous by construction: val is the
// prefix of the counts, EntryVals.)
void validate_result(const WordCountResult& r) {
  u64 sum = 0, j = 0;
  PackedKey prev{};
  for (const WordCountEntry e : r.entries) {  // compact lists decode on the fly
    if (j && key_compare(prev.w, e.key.w) >= 0)
      throw Error("LOCUST_CHECK: output keys not strictly increasing at entry " +
                  std::to_string(j));
    if (e.count == 0) throw Error("LOCUST_CHECK: zero count at entry " + std::to_string(j));
    sum += e.count;
    prev = e.key;
    ++j;
  }
  if (j != r.entries.size()) throw Error("LOCUST_CHECK: entry count mismatch");
  if (sum != r.num_tokens)
    throw Error("LOCUST_CHECK: sum(count)=" + std::to_string(sum) +
                " != num_tokens=" + std::to_string(r.num_tokens));
  if (r.entries.size() != r.num_unique) throw Error("LOCUST_CHECK: num_unique mismatch");
}

}  // namespace locust
