// ./MapReduce -- command line driver (SURVEY.md §2.6 API surface; /root/reference/
// MapReduce/src/main.cu:358-532).
//
// Positional CLI of the reference, byte-compatible stdout:
//   MapReduce <file>                                   whole file, one process
//   MapReduce <file> <line_start> <line_end>           window [start, end)
//   MapReduce <file> <start> <end> <node_num> <stage>  stage 0 = all, 1 = map only
//                                                      (writes a spill), 2 = reduce only
// plus long flags (runtime switches replacing the reference's #defines):
//   --backend gpu|cpu  --reduce-path lds|global  --map-path compat|fast
//   --sort radix|dict  --gpus N  --comm auto|rccl|loopback  --strategy auto|gather|shuffle
//   --emits-per-line N  --max-key N  --ref-compat
//   --stage map|reduce  --spill-dir DIR  --spill-format text|binary|kiv  --inputs a,b,...
//   --export-kiv FILE (results as the reference's 40-B KeyIntValuePair records)
//   --warmup N  --iters N  --json FILE  --quiet  --check  --device N  --chunk-mb N
//   --ref-timers (stage times taken where the reference's host timers were)
// and a synthetic-text generator (BASELINE configs "1M lines" / "10 GB"):
//   MapReduce --gen FILE (--gen-lines N | --gen-bytes N) [--seed S] [--vocab V]
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "locust/dist.hpp"
#include "locust/engine.hpp"
#include "locust/gen.hpp"
#include "locust/io.hpp"
#include "locust/stage.hpp"

using namespace locust;

namespace {

unsigned long long peak_rss_kb();

// A one-shot GPU run ends with _exit once its output is flushed (the
// HIP runtime's teardown -- streams, pinned and device memory, code objects -- took most of
// the ~80 ms outside main()).  Off with LOCUST_FAST_EXIT=0, and under a profiler (rocprofv3
// preloads its tool library and flushes its traces at the runtime's exit).
bool fast_exit_ok() {
  if (const char* e = std::getenv("LOCUST_FAST_EXIT"))
    if (e[0] == '0') return false;
  if (const char* p = std::getenv("LD_PRELOAD"))
    if (std::strstr(p, "rocprof") || std::strstr(p, "roctracer")) return false;
  for (char** e = environ; e && *e; ++e)
    if (std::strncmp(*e, "ROCPROF", 7) == 0) return false;
  return true;
}
bool g_fast_exit = false;  // run() left its GPU state for the process exit to reclaim

struct CliArgs {
  std::string file;
  i64 line_start = -1, line_end = -1;
  int node = 0;
  int stage = 0;
  bool window = false;
  bool byte_range = false;  // --byte-range A:B (stage 1): a byte window instead of lines
  u64 byte_begin = 0, byte_end = ~0ull;
  JobConfig cfg;
  int gpus = 1;
  bool gpus_given = false;   // --gpus on the command line (even --gpus 1: RCCL rank)
  LocalComm comm = LocalComm::kAuto;
  DistStrategy strategy = DistStrategy::kAuto;  // --gpus N: after-map strategy (--strategy)
  std::string spill_dir = "/tmp";
  SpillFormat spill_fmt = SpillFormat::kText;
  std::vector<std::string> inputs;
  int reducer = 0, reducers = 1;  // --reducer r/R: key range r of R (stage 2)
  std::string result_file;        // --result-file: the result lines go there, not stdout
  int out_format = 0;             // --output-format: 0 by mode, 1 gpu (with val), 2 cpu
  int warmup = 0, iters = 1;
  std::string json;
  std::string export_kiv;  // final results as KeyIntValuePair records (--export-kiv FILE)
  bool quiet = false;
  std::string gen_out;  // generator mode
  GenSpec gen;
};

void usage() {
  std::printf("Missing or invalid arguments.\n");
  std::printf("mapreduce <filename> [line_start] [line_end] [node_num] [stage]\n");
}

void help() {
  std::printf(
      "usage: MapReduce <file> [line_start line_end [node_num stage]] [flags]\n"
      "       MapReduce --gen FILE (--gen-lines N | --gen-bytes N) [--seed S] [--vocab V]\n"
      "\n"
      "  stage 0: the whole job; 1: map only, writes the combined spill <spill-dir>/out.<node>.*\n"
      "  and its index; 2: reduce only, merges spills (--inputs a,b,... or out.<node>.*)\n"
      "\n"
      "  --backend gpu|cpu          --reduce-path lds|global   --map-path fast|compat\n"
      "  --sort dict|radix          --gpus N                   --comm auto|loopback|rccl\n"
      "  --strategy auto|gather|shuffle                        --device N\n"
      "  --emits-per-line N         --max-key N                --ref-compat\n"
      "  --stage map|reduce         --spill-dir DIR            --spill-format text|binary|kiv\n"
      "  --inputs a,b,...           --reducer r/R              --result-file FILE\n"
      "  --byte-range A:B           (stage 1: bytes [A, B) moved to line starts; B empty: EOF)\n"
      "  --output-format gpu|cpu    (result lines with val, or the CPU build's)\n"
      "  --export-kiv FILE          --json FILE|-              --quiet --check --combine\n"
      "  --warmup N --iters N       --chunk-mb N               --ref-timers\n"
      "  --help\n"
      "\n"
      "Environment: LOCUST_LOG=info|debug and the LOCUST_* switches in docs/ENVIRONMENT.md.\n");
}

std::vector<std::string> split(const std::string& s, char c) {
  std::vector<std::string> out;
  size_t p = 0;
  while (p <= s.size()) {
    size_t q = s.find(c, p);
    if (q == std::string::npos) q = s.size();
    if (q > p) out.push_back(s.substr(p, q - p));
    p = q + 1;
  }
  return out;
}

bool parse(int argc, char** argv, CliArgs* a) {
  std::vector<std::string> pos;
  apply_env_overrides(a->cfg);
  for (int i = 1; i < argc; ++i) {
    std::string s = argv[i];
    auto need = [&](const char* name) -> std::string {
      if (i + 1 >= argc) throw Error(std::string("missing value for ") + name);
      return argv[++i];
    };
    if (s == "--backend") {
      std::string v = need("--backend");
      a->cfg.backend = v == "cpu" ? Backend::kCpu : Backend::kGpu;
    } else if (s == "--reduce-path") {
      a->cfg.reduce_path = need("--reduce-path") == "global" ? ReducePath::kGlobal : ReducePath::kLds;
    } else if (s == "--map-path") {
      a->cfg.map_path = need("--map-path") == "compat" ? MapPath::kCompat : MapPath::kFast;
    } else if (s == "--sort") {
      a->cfg.sort_path = need("--sort") == "dict" ? SortPath::kDict : SortPath::kRadix;
    } else if (s == "--gpus") {
      a->gpus = std::atoi(need("--gpus").c_str());
      a->gpus_given = true;
    } else if (s == "--comm") {
      const std::string v = need("--comm");
      a->comm = v == "rccl" ? LocalComm::kRccl : v == "loopback" ? LocalComm::kLoopback
                                                               : LocalComm::kAuto;
    } else if (s == "--strategy") {
      const std::string v = need("--strategy");
      if (v != "auto" && v != "gather" && v != "shuffle") throw Error("--strategy auto|gather|shuffle");
      a->strategy = v == "gather" ? DistStrategy::kGather : v == "shuffle" ? DistStrategy::kShuffle
                                                                          : DistStrategy::kAuto;
    } else if (s == "--device") {
      a->cfg.device = std::atoi(need("--device").c_str());
    } else if (s == "--emits-per-line") {
      a->cfg.emits_per_line = std::atoi(need("--emits-per-line").c_str());
    } else if (s == "--max-key") {
      a->cfg.max_key_len = std::atoi(need("--max-key").c_str());
    } else if (s == "--ref-compat") {
      a->cfg.ref_compat = true;
    } else if (s == "--check") {
      a->cfg.check = true;
    } else if (s == "--combine") {
      a->cfg.combine = true;
    } else if (s == "--no-sync-plan") {
      a->cfg.sync_plan = false;
    } else if (s == "--stage") {
      std::string v = need("--stage");
      a->stage = v == "map" || v == "1" ? 1 : (v == "reduce" || v == "2" ? 2 : 0);
    } else if (s == "--spill-dir") {
      a->spill_dir = need("--spill-dir");
    } else if (s == "--spill-format") {
      const std::string v = need("--spill-format");
      a->spill_fmt = v == "binary" ? SpillFormat::kBinary : v == "kiv" ? SpillFormat::kKiv
                                                                     : SpillFormat::kText;
    } else if (s == "--export-kiv") {
      a->export_kiv = need("--export-kiv");
    } else if (s == "--inputs") {
      a->inputs = split(need("--inputs"), ',');
    } else if (s == "--reducer") {
      const std::string v = need("--reducer");
      const size_t sl = v.find('/');
      if (sl == std::string::npos) throw Error("--reducer r/R");
      a->reducer = std::atoi(v.substr(0, sl).c_str());
      a->reducers = std::atoi(v.substr(sl + 1).c_str());
      if (a->reducers < 1 || a->reducer < 0 || a->reducer >= a->reducers)
        throw Error("--reducer r/R needs 0 <= r < R");
    } else if (s == "--byte-range") {
      const std::string v = need("--byte-range");
      const size_t c = v.find(':');
      if (c == std::string::npos || c == 0) throw Error("--byte-range A:B");
      char* endp = nullptr;
      a->byte_begin = std::strtoull(v.c_str(), &endp, 10);
      if (endp != v.c_str() + c) throw Error("--byte-range A:B");
      if (c + 1 < v.size()) {
        a->byte_end = std::strtoull(v.c_str() + c + 1, &endp, 10);
        if (*endp) throw Error("--byte-range A:B");
      }
      if (a->byte_end < a->byte_begin) throw Error("--byte-range A:B needs A <= B");
      a->byte_range = true;
    } else if (s == "--result-file") {
      a->result_file = need("--result-file");
    } else if (s == "--output-format") {
      const std::string v = need("--output-format");
      if (v != "gpu" && v != "cpu") throw Error("--output-format gpu|cpu");
      a->out_format = v == "gpu" ? 1 : 2;
    } else if (s == "--warmup") {
      a->warmup = std::atoi(need("--warmup").c_str());
    } else if (s == "--iters") {
      a->iters = std::max(1, std::atoi(need("--iters").c_str()));
    } else if (s == "--json") {
      a->json = need("--json");
    } else if (s == "--quiet") {
      a->quiet = true;
    } else if (s == "--ref-timers") {
      a->cfg.ref_timers = true;
    } else if (s == "--chunk-mb") {
      a->cfg.chunk_bytes = (u64)std::atoll(need("--chunk-mb").c_str()) << 20;
    } else if (s == "--gen") {
      a->gen_out = need("--gen");
    } else if (s == "--gen-lines") {
      a->gen.lines = (u64)std::atoll(need("--gen-lines").c_str());
    } else if (s == "--gen-bytes") {
      a->gen.bytes = (u64)std::atoll(need("--gen-bytes").c_str());
    } else if (s == "--seed") {
      a->gen.seed = (u64)std::atoll(need("--seed").c_str());
    } else if (s == "--vocab") {
      a->gen.vocab = (u32)std::atoll(need("--vocab").c_str());
    } else if (s.size() > 2 && s[0] == '-' && s[1] == '-') {
      throw Error("unknown flag " + s);
    } else {
      pos.push_back(s);
    }
  }
  if (a->cfg.emits_per_line <= 0) throw Error("--emits-per-line must be > 0");
  if (a->cfg.max_key_len < 1 || a->cfg.max_key_len > kKeyBytes - 1)
    throw Error("--max-key must be in [1, " + std::to_string(kKeyBytes - 1) + "]");
  if (!a->gen_out.empty()) return true;
  if (pos.empty()) return false;
  a->file = pos[0];
  if (pos.size() > 1) {
    a->window = true;
    a->line_start = std::strtol(pos[1].c_str(), nullptr, 10);
    a->line_end = pos.size() > 2 ? std::strtol(pos[2].c_str(), nullptr, 10) : -1;
  }
  if (pos.size() > 3) {
    a->node = (int)std::strtol(pos[3].c_str(), nullptr, 10);
    if (pos.size() > 4) a->stage = (int)std::strtol(pos[4].c_str(), nullptr, 10);
  }
  if (a->byte_range) {
    if (a->stage != 1) throw Error("--byte-range is a stage-1 (map) flag");
    a->window = false;  // the byte window replaces the positional line window
  }
  return true;
}

const char* spill_ext(SpillFormat f) {
  return f == SpillFormat::kBinary ? ".kv" : f == SpillFormat::kKiv ? ".kiv" : ".txt";
}
std::string spill_path(const CliArgs& a, int node) {
  return a.spill_dir + "/out." + std::to_string(node) + spill_ext(a.spill_fmt);
}
// Stage 2 without --inputs: this node's spill in the --spill-format named, else whichever
// of out.N.txt / .kv / .kiv exists (read_spill tells the formats apart by content).
std::string find_spill(const CliArgs& a, int node) {
  const std::string want = spill_path(a, node);
  if (access(want.c_str(), R_OK) == 0) return want;
  for (SpillFormat f : {SpillFormat::kText, SpillFormat::kBinary, SpillFormat::kKiv}) {
    const std::string p = a.spill_dir + "/out." + std::to_string(node) + spill_ext(f);
    if (access(p.c_str(), R_OK) == 0) return p;
  }
  return want;  // (its open fails with the path in the message)
}

// --json: one record per run, in every mode: counts, honest and
// reference-semantics stage times, and for --gpus N every rank's stage times and the bytes
// each of its links carried.
struct JsonOut {
  std::string body;
  void kv(const char* k, const std::string& raw) {
    body += (body.empty() ? "{" : ", ");
    body += "\"" + std::string(k) + "\": " + raw;
  }
  void num(const char* k, double v) {
    char b[64];
    std::snprintf(b, sizeof(b), "%.6f", v);
    kv(k, b);
  }
  void u(const char* k, unsigned long long v) { kv(k, std::to_string(v)); }
  void str(const char* k, const std::string& v) {
    std::string e;
    for (char c : v) {
      if ((unsigned char)c < 0x20) {  // control bytes (a TAB delimiter) as \u00XX
        char u[8];
        std::snprintf(u, sizeof(u), "\\u%04x", (unsigned)(unsigned char)c);
        e += u;
        continue;
      }
      if (c == '"' || c == '\\') e.push_back('\\');
      e.push_back(c);
    }
    kv(k, "\"" + e + "\"");
  }
  std::string done() const { return body + "}"; }
};

std::string u64_list(const std::vector<u64>& v) {
  std::string s = "[";
  for (size_t i = 0; i < v.size(); ++i) s += (i ? ", " : "") + std::to_string(v[i]);
  return s + "]";
}

void emit_json(const CliArgs& a, const std::string& text) {
  if (a.json.empty()) return;
  std::FILE* f = a.json == "-" ? stderr : std::fopen(a.json.c_str(), "w");
  if (!f) throw Error("cannot write json: " + a.json);
  std::fprintf(f, "%s\n", text.c_str());
  if (f != stderr) std::fclose(f);
}

JsonOut json_head(const CliArgs& a, const char* mode) {
  JsonOut j;
  j.str("mode", mode);
  j.str("backend", a.cfg.backend == Backend::kCpu ? "cpu" : "gpu");
  j.kv("gpus", std::to_string(a.gpus));
  j.str("map_path", to_string(a.cfg.map_path));
  j.str("reduce_path", to_string(a.cfg.reduce_path));
  j.str("sort", to_string(a.cfg.sort_path));
  return j;
}

void json_counts(JsonOut& j, const WordCountResult& r) {
  j.u("lines", r.num_lines);
  j.u("tokens", r.num_tokens);
  j.u("unique", r.num_unique);
  j.u("overflow_lines", r.overflow_lines);
  j.u("truncated", r.truncated);
  j.u("max_key_len", r.max_key_len);
}

// Where a one-shot single-GPU run's time goes, main() to the JSON line (run_direct):
// runtime init (the first HIP call), engine construction (code objects, device arena,
// pinned buffers), the file read, the first job, later jobs and the formatted output.
// Process start to main() (loader, static init) is the caller's wall clock minus these.
struct Startup {
  u64 main = 0, init = 0, engine = 0, read = 0, first = 0, jobs = 0, out = 0;
};
Startup g_startup;
const char* g_part_map = nullptr;  // "cache" / "default": run_direct's starting map

// The GPU engine's HBM plan (plan_device_pass): its device memory, the GPU's free and
// total memory before it, and whether the input streams (chunk size, map window).
GpuWordCount::Stats g_engine_stats;
bool g_engine_stats_set = false;
void json_hbm(JsonOut& j, const GpuWordCount::Stats& s) {
  j.u("hbm_device_bytes", s.device_bytes);
  j.u("hbm_free_bytes", s.hbm_free);
  j.u("hbm_total_bytes", s.hbm_total);
  j.kv("device_streaming", s.streaming ? "true" : "false");
  j.u("device_chunk_bytes", s.chunk_bytes);
  j.u("device_map_window", s.map_window);
}

void write_json(const CliArgs& a, const WordCountResult& r, const std::vector<double>& walls) {
  if (a.json.empty()) return;
  std::vector<double> w = walls;
  std::sort(w.begin(), w.end());
  const double med = w.empty() ? 0 : w[w.size() / 2];
  JsonOut j = json_head(a, "full");
  json_counts(j, r);
  j.num("map_ms", r.times.map_ms);
  j.num("process_ms", r.times.process_ms);
  j.num("reduce_ms", r.times.reduce_ms);
  j.num("h2d_ms", r.times.h2d_ms);
  j.num("d2h_ms", r.times.d2h_ms);
  j.num("ref_map_ms", r.times.ref_map_ms);
  j.num("ref_process_ms", r.times.ref_process_ms);
  j.num("ref_reduce_ms", r.times.ref_reduce_ms);
  j.num("wall_ms_median", med);
  j.kv("iters", std::to_string(w.size()));
  j.u("chunks", r.chunks);
  if (g_part_map) j.str("part_map", g_part_map);  // the one-shot CLI's starting map
  if (g_engine_stats_set) json_hbm(j, g_engine_stats);
  // peak resident memory of this process image (VmHWM: unlike getrusage's ru_maxrss it is
  // not inherited through the fork + exec that started us)
  j.u("max_rss_kb", peak_rss_kb());
  if (g_startup.init) {
    const Startup& t = g_startup;
    const u64 end = now_ns();
    auto ms = [](u64 a0, u64 a1) { return a1 > a0 ? (a1 - a0) * 1e-6 : 0.0; };
    JsonOut st;
    st.num("runtime_init_ms", ms(t.main, t.init));
    st.num("engine_ms", ms(t.init, t.engine));
    st.num("read_ms", ms(t.engine, t.read));
    st.num("first_job_ms", ms(t.read, t.first));
    st.num("later_jobs_ms", ms(t.first, t.jobs));
    st.num("output_ms", ms(t.jobs, end));
    st.num("main_to_json_ms", ms(t.main, end));
    // before main(): the loader and the libraries' static initialisation, split at this
    // library's own (LOCUST_T0: the spawner's CLOCK_MONOTONIC ns, tools/cli_cold.py)
    st.num("library_to_main_ms", ms(library_init_ns(), t.main));
    if (const char* t0 = std::getenv("LOCUST_T0"))
      st.num("spawn_to_library_ms", ms((u64)std::strtoull(t0, nullptr, 10), library_init_ns()));
    j.kv("startup", st.done());
  }
  emit_json(a, j.done());
}

void write_json_dist(const CliArgs& a, const DistResult& root, const std::vector<DistResult>& ranks) {
  if (a.json.empty()) return;
  JsonOut j = json_head(a, "multi_gpu");
  json_counts(j, root.result);
  j.str("strategy", root.strategy == DistStrategy::kGather    ? "gather"
                    : root.strategy == DistStrategy::kLocal   ? "local"
                                                              : "shuffle");
  j.num("wall_ms", root.total_ms);
  j.str("comm", !ranks.empty() && ranks[0].rccl_clique ? "rccl" : "loopback");
  j.u("peak_rss_kb", peak_rss_kb());
  {  // page-locked host memory: every rank's engine, plus the shared output block once
    u64 pinned = ranks.empty() ? 0 : ranks[0].shared_pinned_bytes;
    for (const DistResult& d : ranks) pinned += d.pinned_bytes;
    j.u("pinned_bytes", pinned);
    u64 hbm = 0;
    for (const DistResult& d : ranks) hbm += d.hbm_device_bytes;
    j.u("hbm_device_bytes", hbm);  // every rank's engines (one GPU or several)
    if (!ranks.empty()) j.u("hbm_total_bytes", ranks[0].hbm_total_bytes);
    u64 used = 0;
    for (const DistResult& d : ranks) used = std::max(used, d.hbm_used_bytes);
    j.u("hbm_used_bytes_max", used);
  }
  std::string rk = "[";
  for (size_t r = 0; r < ranks.size(); ++r) {
    const DistResult& d = ranks[r];
    JsonOut x;
    x.kv("rank", std::to_string(r));
    x.num("map_ms", d.map_ms);
    x.num("shuffle_ms", d.shuffle_ms);
    x.num("reduce_ms", d.reduce_ms);
    x.num("gather_ms", d.gather_ms);
    x.num("total_ms", d.total_ms);
    x.u("local_records", d.local_records);
    x.u("range_tokens", d.range_tokens);
    x.u("range_unique", d.range_unique);
    x.u("sent_bytes", d.sent_bytes);
    x.u("recv_bytes", d.recv_bytes);
    x.kv("sent_to", u64_list(d.sent_to));
    x.kv("recv_from", u64_list(d.recv_from));
    x.u("output_bytes", d.output_bytes);
    x.kv("device_exchange", d.device_exchange ? "true" : "false");
    x.u("host_syncs", (u64)d.host_syncs);
    x.u("input_bytes", d.input_bytes);
    x.kv("input_streamed", d.input_streamed ? "true" : "false");
    x.kv("peer_p2p", std::to_string(d.peer_p2p));
    x.u("pinned_bytes", d.pinned_bytes);
    x.u("hbm_device_bytes", d.hbm_device_bytes);
    x.u("hbm_free_bytes", d.hbm_free_bytes);
    x.u("hbm_total_bytes", d.hbm_total_bytes);
    x.u("hbm_used_bytes", d.hbm_used_bytes);
    rk += (r ? ", " : "") + x.done();
  }
  j.kv("ranks", rk + "]");
  emit_json(a, j.done());
}

long long ns(double ms) { return (long long)(ms * 1e6 + 0.5); }

// Writes the synthetic text in 64 MiB pieces (bounded memory for 10 GB files).
int generate(const CliArgs& a) {
  std::FILE* f = std::fopen(a.gen_out.c_str(), "wb");
  if (!f) throw Error("cannot write " + a.gen_out);
  const u64 piece_lines = 1u << 20;  // whole 1,024-line blocks per piece
  u64 lines = 0, bytes = 0;
  std::string buf;
  for (u64 first = 0;; first += piece_lines / kGenBlockLines) {
    GenSpec g = a.gen;
    g.first_block = first;
    if (a.gen.lines) {
      if (lines >= a.gen.lines) break;
      g.lines = std::min<u64>(piece_lines, a.gen.lines - lines);
      g.bytes = 0;
    } else {
      if (bytes >= a.gen.bytes) break;
      g.lines = std::min<u64>(piece_lines, a.gen.bytes);  // cut below by bytes
    }
    buf.clear();
    u64 nl = gen_text(g, &buf);
    if (!a.gen.lines && bytes + buf.size() > a.gen.bytes) {
      const size_t cut = buf.rfind('\n', a.gen.bytes - bytes - 1);
      if (cut == std::string::npos || a.gen.bytes == bytes) break;
      buf.resize(cut + 1);
      nl = count_newlines(buf.data(), buf.size());
    }
    write_all(f, buf);
    lines += nl;
    bytes += buf.size();
    if (!a.gen.lines && nl < piece_lines) break;
  }
  std::fclose(f);
  std::printf("generated %llu lines, %llu bytes -> %s\n", (unsigned long long)lines,
              (unsigned long long)bytes, a.gen_out.c_str());
  return 0;
}

// The result lines: the GPU build's "print key: k \t val: v \t count: c" (main.cu:132) or
// the CPU build's "print key: k \t value: c" (main.cu:286).  By default the backend's own
// build -- except --gpus N, always the GPU build's (the multi-GPU mode; --backend cpu there
// only rehearses its ranks, docs/PARITY.md) -- and --output-format overrides.
void format_results(const CliArgs& a, bool cpu_default, const WordCountResult& r,
                    std::string* out) {
  if (a.quiet) return;
  const bool cpu = a.out_format ? a.out_format == 2 : cpu_default;
  (cpu ? format_cpu_output : format_gpu_output)(r, out);
}

// The result lines to stdout, or to --result-file (a range reducer on a worker daemon,
// whose reply carries only the tail of stdout).
void emit_results(const CliArgs& a, const std::string& out) {
  if (a.result_file.empty()) {
    std::fflush(stdout);
    write_all(stdout, out);
    return;
  }
  std::FILE* f = std::fopen(a.result_file.c_str(), "wb");
  if (!f) throw Error("cannot write " + a.result_file);
  write_all(f, out);
  if (std::fclose(f) != 0) throw Error("error closing " + a.result_file);
}

void print_gpu_result(const CliArgs& a, const WordCountResult& r, const std::vector<double>& walls) {
  const bool rt = a.cfg.ref_timers;
  std::printf("GPU mapping %lld nanoseconds \n", ns(rt ? r.times.ref_map_ms : r.times.map_ms));
  for (u64 k = 0; k < r.overflow_lines; ++k) std::printf("WARN: Exceeded emit limit\n");
  std::printf("GPU stream compaction and sorting %lld nanoseconds \n",
              ns(rt ? r.times.ref_process_ms : r.times.process_ms));
  std::printf("GPU reduce %lld nanoseconds \n", ns(rt ? r.times.ref_reduce_ms : r.times.reduce_ms));
  if (r.truncated)
    LOCUST_LOG_WARN("%llu tokens longer than %d chars were truncated",
                    (unsigned long long)r.truncated, a.cfg.max_key_len);
  std::string out;
  format_results(a, false, r, &out);
  emit_results(a, out);
  std::fflush(stdout);
  write_json(a, r, walls);
  if (!a.export_kiv.empty()) write_kiv_results(a.export_kiv, r);
  std::printf("\nDone\n");
}

// Peak resident host memory (kB, VmHWM of /proc/self/status).
unsigned long long peak_rss_kb() {
  std::FILE* f = std::fopen("/proc/self/status", "r");
  if (!f) return 0;
  char line[256];
  unsigned long long kb = 0;
  while (std::fgets(line, sizeof(line), f))
    if (std::sscanf(line, "VmHWM: %llu kB", &kb) == 1) break;
  std::fclose(f);
  return kb;
}

// Stream threshold: files past one device pass (--chunk-mb, default 256 MiB) stream.
constexpr u64 kDefaultStreamChunk = 256ull << 20;

// The RSS stamps of --json runs at LOCUST_LOG=info (reading /proc costs the one-shot CLI).
void log_rss(const char* when) {
  if ((int)log_level() >= (int)LogLevel::kInfo)
    LOCUST_LOG_INFO("%s: %s", when, process_rss_breakdown().c_str());
}

int run_direct(const CliArgs& a) {
  JobConfig cfg = a.cfg;
  const u64 size = file_size(a.file);
  const u64 chunk = cfg.chunk_bytes ? cfg.chunk_bytes : kDefaultStreamChunk;
  WordCountResult r;
  std::vector<double> walls;
  log_rss("before the engine");
  Startup& st = g_startup;
  (void)visible_device_count();  // the HIP runtime's own start-up, timed apart
  st.init = now_ns();
  // The engine outlives the output: its teardown (stream, pinned buffers) is not a job's
  std::unique_ptr<GpuWordCount> eng;
  // the partition map tuned by an earlier run on this file (io.hpp partition-map cache)
  const std::string pmc = partmap_cache_path(a.file, cfg);
  std::vector<u64> cached;
  auto start_map = [&]() {
    g_part_map = load_partmap_cache(pmc, &cached) && eng->set_partition_map(cached) ? "cache"
                                                                                    : "default";
  };
  if (size > chunk) {
    cfg.chunk_bytes = chunk;
    eng.reset(new GpuWordCount(cfg, size, size));
    g_engine_stats = eng->stats();
    g_engine_stats_set = true;
    start_map();
    st.engine = st.read = now_ns();  // the file is read by the job, piece by piece
    log_rss("with the streaming engine");
    for (int i = 0; i < a.warmup + a.iters; ++i) {
      auto src = open_file_source(a.file);
      r = eng->run_source(*src);
      if (i >= a.warmup) walls.push_back(r.times.wall_ms);
      if (i == 0) st.first = now_ns();
    }
  } else {
    eng.reset(new GpuWordCount(cfg, std::max<u64>(size, 1), std::max<u64>(size, 1)));
    g_engine_stats = eng->stats();
    g_engine_stats_set = true;
    start_map();
    st.engine = now_ns();
    TextInput in;
    in.data = eng->input_buffer();
    in.bytes = read_file_into(a.file, eng->input_buffer(), std::max<u64>(size, 1), &in.num_lines);
    in.first_line = 0;
    st.read = now_ns();
    std::vector<u64> stamps;  // per job: start, after run(), after the result is stored
    stamps.reserve(3 * (size_t)(a.warmup + a.iters));
    std::vector<StageTimes> jt;  // per job: its own host split (launch / wait / copy)
    jt.reserve((size_t)(a.warmup + a.iters));
    for (int i = 0; i < a.warmup + a.iters; ++i) {
      stamps.push_back(now_ns());
      if (i < a.warmup) {
        jt.push_back(eng->run(in).times);
        stamps.push_back(now_ns());
      } else {
        WordCountResult x = eng->run(in);
        stamps.push_back(now_ns());
        jt.push_back(x.times);
        r = std::move(x);
        walls.push_back(r.times.wall_ms);
      }
      stamps.push_back(now_ns());
      if (i == 0) st.first = stamps.back();
    }
    if ((int)log_level() >= (int)LogLevel::kDebug)
      for (size_t k = 0; k + 2 < stamps.size(); k += 3)
        LOCUST_LOG_DEBUG("job %zu: starts %+.3f ms, run() %.3f ms (launch %.3f, wait %.3f, copy "
                         "%.3f), result stored %.3f ms", k / 3, (stamps[k] - st.read) * 1e-6,
                         (stamps[k + 1] - stamps[k]) * 1e-6, jt[k / 3].host_launch_ms,
                         jt[k / 3].host_wait_ms, jt[k / 3].host_copy_ms,
                         (stamps[k + 2] - stamps[k + 1]) * 1e-6);
    r.num_lines = in.num_lines;
  }
  st.jobs = now_ns();
  log_rss("after the job");
  std::printf("Length: %i\n", (int)r.num_lines);
  print_gpu_result(a, r, walls);
  log_rss("after the output");
  // keep this run's tuned map for the next run on the file (after the output: not a job's)
  const u64 t_down = now_ns();
  std::vector<u64> lo;
  if (!pmc.empty() && eng->partition_map(&lo) && lo != cached) save_partmap_cache(pmc, lo);
  if (fast_exit_ok()) {
    // the process ends right after this (main: _exit): the driver reclaims the engine's
    // queues and memory with the process -- no per-buffer teardown
    (void)eng.release();
    g_fast_exit = true;
    return 0;
  }
  eng.reset();
  LOCUST_LOG_DEBUG("engine teardown %.3f ms", (now_ns() - t_down) * 1e-6);
  return 0;
}

// ---------------- stage 1: map only -> spill (main.cu:421-433) ----------------
// The combined map output -- one (key, count) record per distinct key, in key order -- and
// its index.  A GPU line window is found by a newline scan and read straight from the file
// into the engine's pinned buffer; past one device pass (--chunk-mb, 256 MiB) it streams
// through a streaming engine, so host memory stays bounded for any window size.
// --ref-compat keeps the reference's spill: one "key \t1" record per token, sorted.
int run_map_stage(const CliArgs& a) {
  const bool cpu = a.cfg.backend == Backend::kCpu;
  const char* dev = cpu ? "CPU" : "GPU";
  const std::string path = spill_path(a, a.node);
  // the HIP runtime's own start-up (once per process, ~0.1-0.2 s), timed apart from the
  // job like run_direct's: job_ms is this window's work, comparable across processes
  const u64 t_init = now_ns();
  if (!cpu) (void)visible_device_count();
  const double runtime_init_ms = (now_ns() - t_init) * 1e-6;
  MapWindow win;
  if (a.byte_range) {
    win.by_bytes = true;
    win.byte_begin = a.byte_begin;
    win.byte_end = a.byte_end;
  } else if (a.window) {
    win.line_start = a.line_start;
    win.line_end = a.line_end;
  }
  MapStageResult m = map_stage(a.cfg, a.file, win, path, a.spill_fmt);
  if (m.engine_keep && fast_exit_ok()) {  // main _exits after the output: no teardown
    new std::shared_ptr<void>(std::move(m.engine_keep));  // never destroyed
    g_fast_exit = true;
  }
  const WordCountResult& r = m.result;
  if (!cpu) std::printf("Length: %i\n", (int)m.lines);
  for (u64 k = 0; k < r.overflow_lines; ++k) std::printf("WARN: Exceeded emit limit\n");
  // event-timed on the GPU: H2D + map, then compaction/combine + sort
  std::printf("%s mapping %lld nanoseconds \n", dev, ns(r.times.h2d_ms + r.times.map_ms));
  std::printf("%s stream compaction and sorting %lld nanoseconds \n", dev,
              ns(r.times.process_ms + r.times.reduce_ms));
  if (!a.json.empty()) {
    JsonOut j = json_head(a, "map_stage");
    json_counts(j, r);
    j.u("spill_records", m.spill_records);
    j.u("spill_bytes", m.index.spill_bytes);
    j.str("spill", path);
    j.str("input", a.file);
    j.kv("line_start", std::to_string(a.window ? a.line_start : 0));
    j.kv("line_end", std::to_string(a.window ? a.line_end : -1));
    if (a.byte_range) {  // the range asked for, and the bytes it moved to
      j.u("byte_range_begin", a.byte_begin);
      j.kv("byte_range_end", a.byte_end == ~0ull ? "-1" : std::to_string(a.byte_end));
    }
    j.u("byte_begin", m.byte_begin);
    j.u("byte_end", m.byte_end);
    {  // the input's identity and the tokenizer settings (a resume checks both)
      struct stat st {};
      if (::stat(a.file.c_str(), &st) == 0) {
        j.u("input_size", (unsigned long long)st.st_size);
        j.u("input_mtime_ns", (unsigned long long)st.st_mtim.tv_sec * 1000000000ull +
                                  (unsigned long long)st.st_mtim.tv_nsec);
        j.u("input_inode", (unsigned long long)st.st_ino);
      }
      j.kv("emits_per_line", std::to_string(a.cfg.emits_per_line));
      j.kv("max_key", std::to_string(a.cfg.max_key_len));
      j.str("delimiters", a.cfg.delimiters);
    }
    j.kv("combined", a.cfg.ref_compat ? "false" : "true");
    j.kv("streamed", m.streamed ? "true" : "false");
    j.u("input_bytes", m.input_bytes);
    j.num("map_ms", r.times.h2d_ms + r.times.map_ms);
    j.num("process_ms", r.times.process_ms + r.times.reduce_ms);
    j.num("job_ms", m.job_ms);
    j.num("runtime_init_ms", runtime_init_ms);
    j.num("window_ms", m.window_ms);
    j.num("setup_ms", m.setup_ms);
    j.num("run_ms", m.run_ms);
    j.num("spill_write_ms", m.spill_write_ms);
    if (!cpu && !a.cfg.ref_compat) json_hbm(j, m.engine);
    j.u("peak_rss_kb", peak_rss_kb());
    emit_json(a, j.done());
  }
  std::printf("MODE_MULTI: Finished map\n");
  return 0;
}

// ---------------- stage 2: reduce only (main.cu:437-486) ----------------
// Every spill is a sorted run (the reference's reducer needed one pre-sorted file, B7):
// this reducer's key range of each is read (an index seek) and merged, counts summed --
// never expanded into tokens.  --reducer r/R: key range r of R, with its global val base.
int run_reduce_stage(const CliArgs& a) {
  const bool cpu = a.cfg.backend == Backend::kCpu;
  std::vector<std::string> files = a.inputs;
  if (files.empty()) files.push_back(find_spill(a, a.node));
  const u64 t_init = now_ns();  // the HIP runtime's start-up, apart from setup_ms
  if (!cpu) (void)visible_device_count();
  const double runtime_init_ms = (now_ns() - t_init) * 1e-6;
  ReduceStageStats st;
  WordCountResult r = reduce_spills(a.cfg, files, a.reducer, a.reducers, &st);
  std::printf("%s reduce %lld nanoseconds \n", cpu ? "CPU" : "GPU", ns(st.merge_ms));
  std::string out;
  format_results(a, cpu, r, &out);
  emit_results(a, out);
  if (!a.json.empty()) {
    JsonOut j = json_head(a, "reduce_stage");
    json_counts(j, r);
    j.u("input_files", st.input_files);
    j.u("indexed_files", st.indexed_files);
    j.u("records_read", st.records_read);
    j.u("input_records", st.run_records);
    j.kv("reducer", std::to_string(a.reducer));
    j.kv("reducers", std::to_string(a.reducers));
    j.u("val_base", r.val_base);
    j.num("read_ms", st.read_ms);
    j.num("runtime_init_ms", runtime_init_ms);
    j.num("setup_ms", st.setup_ms);
    j.num("merge_ms", st.merge_ms);
    j.num("wall_ms", r.times.wall_ms);
    j.u("peak_rss_kb", peak_rss_kb());
    emit_json(a, j.done());
  }
  if (!a.export_kiv.empty()) write_kiv_results(a.export_kiv, r);
  std::printf("\nDone\n");
  return 0;
}

int run(const CliArgs& a) {
  if (!a.gen_out.empty()) return generate(a);
  const bool cpu = a.cfg.backend == Backend::kCpu;
  const char* dev = cpu ? "CPU" : "GPU";
  if (a.window)
    std::printf("Using custom start and end locations: (%i, %i)\n", (int)a.line_start,
                (int)a.line_end);

  if (a.stage == 2) return run_reduce_stage(a);
  if (a.stage == 1) return run_map_stage(a);

  // CPU build ignores the line window (its loadFile takes none, main.cu:242) -- only
  // reproduced under --ref-compat.
  const bool use_window = a.window && !(cpu && a.cfg.ref_compat);
  // A whole file on one GPU (the fast dictionary path): no loader copy at all -- the file
  // is read by parallel preads straight into the engine's pinned input buffer, or, past
  // one device pass, streamed through two pinned chunks (host memory stays bounded).
  const bool direct = !cpu && !use_window && a.stage == 0 && !a.gpus_given && a.gpus <= 1 &&
                      !a.cfg.ref_compat && a.cfg.map_path == MapPath::kFast &&
                      a.cfg.sort_path == SortPath::kDict;
  if (direct) return run_direct(a);
  // ---------------- multi-GPU in one process (one thread per rank) ----------------------
  // An explicit --gpus N (N >= 1) runs N ranks.  --comm auto: an ncclCommInitAll clique
  // over xGMI when N > 1 and every rank has a GPU of its own, loopback ranks otherwise
  // (one rank, or N ranks rehearsed on fewer GPUs); --comm rccl / loopback force either.
  // A whole file is never loaded: every rank reads only its own line-aligned byte range
  // (run_single_process_file); a line window is loaded first, then sharded.
  const bool multi = (a.gpus > 1 || (a.gpus_given && !cpu)) && a.stage == 0;
  // (the compat map sizes its slots per line: its ranks get the loaded text, whose line
  // count is exact, not a file range sized by bytes)
  const bool file_ranks = multi && !use_window && !a.cfg.ref_compat &&
                          a.cfg.map_path != MapPath::kCompat;
  LoadedText text;
  if (!file_ranks) {
    text = load_lines(a.file, use_window ? a.line_start : -1, use_window ? a.line_end : -1,
                      a.cfg.ref_compat);
    if (!cpu) std::printf("Length: %i\n", (int)text.input.num_lines);
  }
  if (multi) {
    DistConfig dc;
    dc.job = a.cfg;
    // ranks always combine map-side (the output is the same; the device exchange and the
    // gather slots move one record per distinct key instead of one per token)
    dc.job.combine = true;
    dc.world = std::max(1, a.gpus);
    dc.strategy = a.strategy;
    std::vector<DistResult> ranks;
    DistResult dr = file_ranks ? run_single_process_file(dc, a.file, a.comm, &ranks)
                               : run_single_process_multi_gpu(dc, text.input, a.comm, &ranks);
    // the communicator the ranks actually used (a failed clique falls back to loopback)
    LOCUST_LOG_INFO("%d ranks in one process over %s", dc.world,
                    !ranks.empty() && ranks[0].rccl_clique ? "an RCCL clique" : "loopback");
    log_rss("after the job");
    if (file_ranks && !cpu) std::printf("Length: %i\n", (int)dr.result.num_lines);
    std::printf("%s mapping %lld nanoseconds \n", dev, ns(dr.map_ms));
    std::printf("%s stream compaction and sorting %lld nanoseconds \n", dev, ns(dr.shuffle_ms));
    std::printf("%s reduce %lld nanoseconds \n", dev, ns(dr.reduce_ms));
    std::string out;
    format_results(a, false, dr.result, &out);
    emit_results(a, out);
    write_json_dist(a, dr, ranks);
    std::printf("\nDone\n");
    return 0;
  }

  // ---------------- stage 0: full pipeline ----------------
  WordCountResult r;
  std::vector<double> walls;
  if (cpu) {
    CpuWordCount eng(a.cfg);
    for (int i = 0; i < a.warmup; ++i) eng.run(text.input);
    for (int i = 0; i < a.iters; ++i) {
      r = eng.run(text.input);
      walls.push_back(r.times.wall_ms);
    }
    std::printf("CPU mapping %lld nanoseconds \n", ns(r.times.map_ms));
    std::printf("CPU sorting %lld nanoseconds \n", ns(r.times.process_ms));
    std::printf("CPU reducing %lld nanoseconds \n", ns(r.times.reduce_ms));
  } else {
    GpuWordCount eng(a.cfg, text.input.bytes, text.input.num_lines);
    for (int i = 0; i < a.warmup; ++i) eng.run(text.input);
    for (int i = 0; i < a.iters; ++i) {
      r = eng.run(text.input);
      walls.push_back(r.times.wall_ms);
    }
    print_gpu_result(a, r, walls);
    return 0;
  }
  if (r.truncated)
    LOCUST_LOG_WARN("%llu tokens longer than %d chars were truncated",
                    (unsigned long long)r.truncated, a.cfg.max_key_len);
  std::string out;
  format_results(a, cpu, r, &out);
  emit_results(a, out);
  write_json(a, r, walls);
  if (!a.export_kiv.empty()) write_kiv_results(a.export_kiv, r);
  std::printf("\nDone\n");
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  // before any thread or RCCL use (see locust_amd/__init__.py); a user's setting wins
  g_startup.main = now_ns();
  setenv("NCCL_GRAPH_REGISTER", "0", 0);
  for (int i = 1; i < argc; ++i)
    if (std::strcmp(argv[i], "--help") == 0 || std::strcmp(argv[i], "-h") == 0) {
      help();
      return 0;
    }
  std::printf("Running\n");
  CliArgs a;
  try {
    if (!parse(argc, argv, &a)) {
      usage();
      return -1;
    }
    const int rc = run(a);
    if (rc == 0 && (g_fast_exit || (a.cfg.backend == Backend::kGpu && fast_exit_ok()))) {
      std::fflush(nullptr);
      _exit(0);  // skip the HIP runtime's teardown (fast_exit_ok)
    }
    return rc;
  } catch (const std::exception& e) {
    std::fflush(stdout);
    std::fprintf(stderr, "MapReduce: error: %s\n", e.what());
    return 2;
  }
}
