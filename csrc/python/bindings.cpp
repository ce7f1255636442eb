// Python bindings (pybind11) for the native engine: `locust_amd._locust`.
//
// The hot path stays in C++/HIP; Python only moves the input bytes in and formatted
// results out.  The GPU engine is created lazily, so importing the module never touches
// the HIP runtime (the driver's CPU-only build check imports it on a machine without GPU).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>
#include <string>
#include <tuple>

#include "locust/devcache.hpp"
#include "locust/dist.hpp"
#include "locust/dstring.hpp"
#include "locust/engine.hpp"
#include "locust/gen.hpp"
#include "locust/io.hpp"
#include "locust/stage.hpp"
#include "locust/numa.hpp"
#include "locust/partmap.hpp"
#include "locust/shm.hpp"

namespace py = pybind11;
using namespace locust;

namespace {

struct PyResult {
  WordCountResult r;
  py::list entries() const {
    py::list out;
    EntryVals vals(r);
    for (const auto& e : r.entries)
      out.append(py::make_tuple(py::bytes(key_to_string(e.key)), vals.next(e), e.count));
    return out;
  }
  py::dict times() const {
    py::dict d;
    d["h2d_ms"] = r.times.h2d_ms;
    d["map_ms"] = r.times.map_ms;
    d["process_ms"] = r.times.process_ms;
    d["reduce_ms"] = r.times.reduce_ms;
    d["d2h_ms"] = r.times.d2h_ms;
    d["wall_ms"] = r.times.wall_ms;
    d["gpu_ms"] = r.times.gpu_ms;
    d["host_launch_ms"] = r.times.host_launch_ms;
    d["host_wait_ms"] = r.times.host_wait_ms;
    d["host_copy_ms"] = r.times.host_copy_ms;
    d["ref_map_ms"] = r.times.ref_map_ms;
    d["ref_process_ms"] = r.times.ref_process_ms;
    d["ref_reduce_ms"] = r.times.ref_reduce_ms;
    d["graph"] = r.times.graph;
    d["lean"] = r.times.lean;
    return d;
  }
  py::bytes format(bool cpu_format) const {
    std::string s;
    (cpu_format ? format_cpu_output : format_gpu_output)(r, &s);
    return py::bytes(s);
  }
};

TextInput as_input(const std::string& text, u64 first_line = 0) {
  TextInput in;
  in.data = text.data();
  in.bytes = text.size();
  in.num_lines = count_lines(text.data(), text.size());
  in.first_line = first_line;
  return in;
}

PackedKey to_key(const std::string& s) {
  PackedKey k;
  pack_key(s.data(), (int)std::min<size_t>(s.size(), kKeyBytes), k.w);
  return k;
}

class PyGpuEngine {
 public:
  py::dict stats() const {
    const GpuWordCount::Stats st = eng_.stats();
    py::dict d;
    d["retunes"] = st.retunes;
    d["fallbacks"] = st.fallbacks;
    d["planned_passes"] = st.planned_passes;
    d["devplan_failed"] = st.devplan_failed;
    d["device_bytes"] = st.device_bytes;
    d["hbm_free"] = st.hbm_free;
    d["hbm_total"] = st.hbm_total;
    d["streaming"] = st.streaming;
    d["chunk_bytes"] = st.chunk_bytes;
    d["map_window"] = st.map_window;
    return d;
  }
  PyGpuEngine(const JobConfig& cfg, u64 max_bytes, u64 max_lines)
      : eng_(cfg, max_bytes, max_lines), max_bytes_(max_bytes) {}
  GpuWordCount& engine() { return eng_; }
  PyResult run(const std::string& text) {
    py::gil_scoped_release nogil;
    return PyResult{eng_.run(as_input(text))};
  }
  std::vector<py::bytes> map_stage(const std::string& text) {
    std::vector<PackedKey> toks;
    {
      py::gil_scoped_release nogil;
      toks = eng_.run_map_stage(as_input(text), nullptr);
    }
    std::vector<py::bytes> out;
    for (const auto& k : toks) out.emplace_back(key_to_string(k));
    return out;
  }
  PyResult reduce_stage(const std::vector<std::string>& keys) {
    std::vector<PackedKey> toks;
    for (const auto& s : keys) toks.push_back(to_key(s));
    py::gil_scoped_release nogil;
    return PyResult{eng_.run_reduce_stage(toks.data(), toks.size())};
  }
  py::tuple sort_keys(const std::vector<std::string>& keys) {
    std::vector<PackedKey> toks;
    for (const auto& s : keys) toks.push_back(to_key(s));
    std::vector<PackedKey> sorted;
    std::vector<u32> perm;
    {
      py::gil_scoped_release nogil;
      perm = eng_.sort_keys(toks.data(), toks.size(), &sorted);
    }
    std::vector<py::bytes> out;
    for (const auto& k : sorted) out.emplace_back(key_to_string(k));
    return py::make_tuple(out, perm);
  }
  std::vector<py::bytes> compact_slots(const std::vector<u32>& line_counts,
                                       const std::vector<std::string>& slot_keys) {
    std::vector<PackedKey> slots;
    for (const auto& s : slot_keys) slots.push_back(to_key(s));
    LOCUST_CHECK_ARG(slots.size() == line_counts.size() * (u64)eng_.config().emits_per_line,
                     "need num_lines * emits_per_line slot keys");
    std::vector<PackedKey> dense;
    {
      py::gil_scoped_release nogil;
      dense = eng_.compact_slots(line_counts.data(), (u32)line_counts.size(), slots.data());
    }
    std::vector<py::bytes> out;
    for (const auto& k : dense) out.emplace_back(key_to_string(k));
    return out;
  }
  PyResult reduce_sorted(const std::vector<std::string>& keys) {
    std::vector<PackedKey> toks;
    for (const auto& s : keys) toks.push_back(to_key(s));
    py::gil_scoped_release nogil;
    return PyResult{eng_.reduce_sorted(toks.data(), toks.size())};
  }
  // runs: lists of (key bytes, count), each sorted with distinct keys.
  PyResult merge_runs(const std::vector<std::vector<std::pair<std::string, u64>>>& runs) {
    std::vector<std::vector<KeyCount>> rr(runs.size());
    for (size_t q = 0; q < runs.size(); ++q)
      for (const auto& kc : runs[q]) {
        KeyCount rec;
        const PackedKey k = to_key(kc.first);
        for (int w = 0; w < kKeyWords; ++w) rec.w[w] = k.w[w];
        rec.count = kc.second;
        rr[q].push_back(rec);
      }
    py::gil_scoped_release nogil;
    return PyResult{eng_.merge_runs(rr)};
  }
  u64 capacity() const { return eng_.token_capacity(); }
  // Stage the text in the engine's pinned buffer once; run_loaded() then skips the copy.
  void load(const std::string& text) {
    loaded_in_ = as_input(text);
    if (text.size() <= eng_.text_capacity()) {
      std::memcpy(eng_.input_buffer(), text.data(), text.size());
      loaded_ = eng_.input_buffer();
    } else {
      // larger than one device pass: keep it pinned, the engine streams it in chunks
      big_ = std::make_unique<HostText>(text.size());
      std::memcpy(big_->data(), text.data(), text.size());
      big_->set_size(text.size(), loaded_in_.num_lines);
      loaded_ = big_->data();
    }
    loaded_in_.data = loaded_;
  }
  PyResult run_loaded() {
    LOCUST_CHECK_ARG(loaded_ != nullptr, "call load() first");
    py::gil_scoped_release nogil;
    return PyResult{eng_.run(loaded_in_)};
  }
  // Text in pinned host memory, any size (larger than the capacity: streamed in chunks).
  PyResult run_text(const HostText& t) {
    py::gil_scoped_release nogil;
    return PyResult{eng_.run(t.input())};
  }
  // A file streamed through a streaming engine (the CLI's run_direct past one pass).
  PyResult run_file(const std::string& path) {
    py::gil_scoped_release nogil;
    auto src = open_file_source(path);
    return PyResult{eng_.run_source(*src)};
  }

 private:
  GpuWordCount eng_;
  u64 max_bytes_;
  std::unique_ptr<HostText> big_;
  char* loaded_ = nullptr;
  TextInput loaded_in_;
};

py::list strtok_r_tokens(const std::string& line, const std::string& delims) {
  std::string buf = line;
  py::list out;
  char* save = nullptr;
  for (char* t = d_strtok_r(&buf[0], delims.c_str(), &save); t;
       t = d_strtok_r(nullptr, delims.c_str(), &save))
    out.append(py::bytes(t));
  return out;
}

LocalComm local_comm(const std::string& c) {
  if (c == "auto") return LocalComm::kAuto;
  if (c == "loopback") return LocalComm::kLoopback;
  if (c == "rccl") return LocalComm::kRccl;
  throw Error("comm must be auto, loopback or rccl, not " + c);
}

PyResult run_multi(const std::string& text, const DistConfig& cfg, const std::string& comm) {
  TextInput in = as_input(text);
  const LocalComm lc = local_comm(comm);
  py::gil_scoped_release nogil;
  DistResult d = run_single_process_multi_gpu(cfg, in, lc);
  return PyResult{d.result};
}

py::dict dist_to_dict(const DistResult& d);

py::list run_multi_schedule(const std::string& text, const std::vector<DistConfig>& schedule,
                            const std::string& comm) {
  TextInput in = as_input(text);
  const LocalComm lc = local_comm(comm);
  std::vector<DistResult> rs;
  {
    py::gil_scoped_release nogil;
    rs = run_single_process_schedule(schedule, in, lc);
  }
  py::list out;
  for (const auto& d : rs) out.append(py::make_tuple(PyResult{d.result}, dist_to_dict(d)));
  return out;
}

py::dict dist_to_dict(const DistResult& d) {
  py::dict x;
  x["map_ms"] = d.map_ms;
  x["shuffle_ms"] = d.shuffle_ms;
  x["device_exchange"] = d.device_exchange;
  x["host_syncs"] = d.host_syncs;
  x["output_bytes"] = d.output_bytes;
  x["reduce_ms"] = d.reduce_ms;
  x["gather_ms"] = d.gather_ms;
  x["total_ms"] = d.total_ms;
  x["local_records"] = d.local_records;
  x["sent_bytes"] = d.sent_bytes;
  x["recv_bytes"] = d.recv_bytes;
  x["range_tokens"] = d.range_tokens;
  x["range_unique"] = d.range_unique;
  x["strategy"] = d.strategy == DistStrategy::kGather  ? "gather"
                  : d.strategy == DistStrategy::kLocal ? "local"
                                                       : "shuffle";
  x["input_bytes"] = d.input_bytes;
  x["input_streamed"] = d.input_streamed;
  x["peer_p2p"] = d.peer_p2p;
  x["rccl_clique"] = d.rccl_clique;
  x["pinned_bytes"] = d.pinned_bytes;
  x["shared_pinned_bytes"] = d.shared_pinned_bytes;
  x["hbm_device_bytes"] = d.hbm_device_bytes;
  x["hbm_free_bytes"] = d.hbm_free_bytes;
  x["hbm_total_bytes"] = d.hbm_total_bytes;
  x["hbm_used_bytes"] = d.hbm_used_bytes;
  x["sent_to"] = d.sent_to;
  x["recv_from"] = d.recv_from;
  return x;
}

// A file's multi-rank job in this process: every rank reads only its own byte range.
py::tuple run_multi_file(const std::string& path, const DistConfig& cfg, const std::string& comm) {
  const LocalComm lc = local_comm(comm);
  std::vector<DistResult> ranks;
  DistResult d;
  {
    py::gil_scoped_release nogil;
    d = run_single_process_file(cfg, path, lc, &ranks);
  }
  py::list infos;
  for (const auto& x : ranks) infos.append(dist_to_dict(x));
  return py::make_tuple(PyResult{d.result}, infos);
}

// A rank of a multi-process job: its communicator and engine live across runs.
class PyDistRank {
 public:
  PyDistRank(const DistConfig& cfg, int rank, const std::string& comm, const std::string& host,
             int port, u64 max_bytes, u64 max_lines, double timeout_s, int listen_fd)
      : cfg_(cfg), max_bytes_(max_bytes) {
    py::gil_scoped_release nogil;
    if (comm == "tcp") {
      comm_ = make_tcp_comm(rank, cfg.world, host, port, timeout_s, listen_fd);
    } else if (comm == "tcpdev") {
      comm_ = make_staged_device_comm(make_tcp_comm(rank, cfg.world, host, port, timeout_s, listen_fd));
    } else if (comm == "rccl") {
      comm_ = make_rccl_comm(rank, cfg.world, cfg.job.device, host, port, timeout_s, listen_fd);
    } else {
      throw Error("unknown communicator " + comm);
    }
    engines_.push_back(make_engine(max_bytes, max_lines));
    eng_ = engines_[0].get();
  }
  // Another engine on the same communicator (a second input shape, e.g. the synthetic
  // strong-scaling config next to the Hamlet headline); returns its index for use_engine.
  // Every rank must add and select engines in the same order.
  int add_engine(u64 max_bytes, u64 max_lines) {
    py::gil_scoped_release nogil;
    engines_.push_back(make_engine(max_bytes, max_lines));
    return (int)engines_.size() - 1;
  }
  void use_engine(int i) {
    LOCUST_CHECK_ARG(i >= 0 && (size_t)i < engines_.size(), "no such engine");
    eng_ = engines_[(size_t)i].get();
    engine_caps_idx_ = i;
    loaded_ = false;  // load() the new engine's shard
  }
  py::tuple run(const std::string& shard_text_bytes, u64 first_line) {
    TextInput in = as_input(shard_text_bytes, first_line);
    DistResult d;
    {
      py::gil_scoped_release nogil;
      d = run_distributed(cfg_, *comm_, *eng_, in);
    }
    return py::make_tuple(PyResult{d.result}, dist_to_dict(d));
  }
  // Keep the shard resident (in the engine's pinned buffer when it has one) so repeated
  // runs skip the Python->native copy, like GpuEngine.load().
  void load(const std::string& shard_text_bytes, u64 first_line) {
    loaded_in_ = as_input(shard_text_bytes, first_line);
    char* pinned = eng_->input_buffer();
    if (pinned) {
      LOCUST_CHECK_ARG(shard_text_bytes.size() <= caps_[(size_t)engine_caps_idx_],
                       "shard exceeds engine capacity");
      if (shard_text_bytes.size() <= cfg_.job.chunk_bytes || !cfg_.job.chunk_bytes) {
        std::memcpy(pinned, shard_text_bytes.data(), shard_text_bytes.size());
        loaded_in_.data = pinned;
      } else {
        big_ = std::make_unique<HostText>(shard_text_bytes.size());
        std::memcpy(big_->data(), shard_text_bytes.data(), shard_text_bytes.size());
        loaded_in_.data = big_->data();
      }
    } else {
      loaded_text_ = shard_text_bytes;
      loaded_in_.data = loaded_text_.data();
    }
    loaded_ = true;
  }
  // A HostText shard (pinned; may exceed the engine capacity: streamed).  The caller
  // keeps it alive (the binding ties its lifetime to this rank).
  void load_text(const HostText& t, u64 first_line) {
    loaded_in_ = t.input(first_line);
    loaded_ = true;
  }
  py::tuple run_loaded() {
    LOCUST_CHECK_ARG(loaded_, "call load() first");
    DistResult d;
    {
      py::gil_scoped_release nogil;
      d = run_distributed(cfg_, *comm_, *eng_, loaded_in_);
    }
    return py::make_tuple(PyResult{d.result}, dist_to_dict(d));
  }
  void barrier() {
    py::gil_scoped_release nogil;
    comm_->barrier();
  }
  // Max over ranks of a double (timing aggregation for the benchmark).
  double allreduce_max(double v) {
    std::vector<double> all((size_t)comm_->size());
    {
      py::gil_scoped_release nogil;
      comm_->allgather_host(&v, all.data(), sizeof(double));
    }
    double m = v;
    for (double x : all) m = std::max(m, x);
    return m;
  }
  // Every rank's bytes (any length) on every rank: lengths first, then padded payloads.
  py::list allgather_bytes(const std::string& mine) {
    const u64 P = (u64)comm_->size();
    std::vector<u64> lens(P);
    std::vector<char> all;
    u64 mx = 0;
    {
      py::gil_scoped_release nogil;
      const u64 n = mine.size();
      comm_->allgather_host(&n, lens.data(), sizeof(u64));
      for (u64 l : lens) mx = std::max(mx, l);
      std::string pad = mine;
      pad.resize(std::max<u64>(mx, 1));
      all.resize(std::max<u64>(mx, 1) * P);
      comm_->allgather_host(pad.data(), all.data(), std::max<u64>(mx, 1));
    }
    py::list out;
    for (u64 r = 0; r < P; ++r)
      out.append(py::bytes(all.data() + r * std::max<u64>(mx, 1), lens[r]));
    return out;
  }
  int rank() const { return comm_->rank(); }
  int size() const { return comm_->size(); }
  int comm_count() const { return comm_->comm_count(); }
  std::string comm_name() const { return comm_->name(); }
  void set_strategy(DistStrategy s) { cfg_.strategy = s; }

 private:
  std::unique_ptr<ShardEngine> make_engine(u64 max_bytes, u64 max_lines) {
    caps_.push_back(max_bytes);
    return cfg_.job.backend == Backend::kGpu ? make_gpu_shard_engine(cfg_.job, max_bytes, max_lines)
                                             : make_cpu_shard_engine(cfg_.job);
  }
  DistConfig cfg_;
  u64 max_bytes_;
  std::unique_ptr<Communicator> comm_;
  std::vector<std::unique_ptr<ShardEngine>> engines_;
  std::vector<u64> caps_;
  int engine_caps_idx_ = 0;
  ShardEngine* eng_ = nullptr;
  bool loaded_ = false;
  std::unique_ptr<HostText> big_;
  std::string loaded_text_;
  TextInput loaded_in_;
};

}  // namespace

PYBIND11_MODULE(_locust, m) {
  m.doc() = "Locust-MI355X native engine (HIP/CDNA4 kernels, RCCL shuffle)";

  py::enum_<Backend>(m, "Backend").value("gpu", Backend::kGpu).value("cpu", Backend::kCpu);
  py::enum_<ReducePath>(m, "ReducePath")
      .value("lds", ReducePath::kLds)
      .value("global_", ReducePath::kGlobal);
  py::enum_<MapPath>(m, "MapPath").value("compat", MapPath::kCompat).value("fast", MapPath::kFast);
  py::enum_<SortPath>(m, "SortPath").value("radix", SortPath::kRadix).value("dict", SortPath::kDict);

  py::class_<JobConfig>(m, "JobConfig")
      .def(py::init<>())
      .def_readwrite("backend", &JobConfig::backend)
      .def_readwrite("device", &JobConfig::device)
      .def_readwrite("emits_per_line", &JobConfig::emits_per_line)
      .def_readwrite("max_key_len", &JobConfig::max_key_len)
      .def_readwrite("delimiters", &JobConfig::delimiters)
      .def_readwrite("ref_compat", &JobConfig::ref_compat)
      .def_readwrite("reduce_path", &JobConfig::reduce_path)
      .def_readwrite("map_path", &JobConfig::map_path)
      .def_readwrite("sort_path", &JobConfig::sort_path)
      .def_readwrite("combine", &JobConfig::combine)
      .def_readwrite("check", &JobConfig::check)
      .def_readwrite("sync_plan", &JobConfig::sync_plan)
      .def_readwrite("chunk_bytes", &JobConfig::chunk_bytes)
      .def_readwrite("zero_copy_text", &JobConfig::zero_copy_text)
      .def_readwrite("graph", &JobConfig::graph)
      .def_readwrite("ref_timers", &JobConfig::ref_timers)
      .def_readwrite("hbm_share", &JobConfig::hbm_share);
  m.def("plan_device_pass", [](const JobConfig& cfg, u64 max_bytes, u64 max_lines, u64 cap_records,
                               u64 free_bytes) {
    const DevicePassPlan p = plan_device_pass(cfg, max_bytes, max_lines, cap_records, free_bytes);
    py::dict d;
    d["streaming"] = p.streaming;
    d["chunk_bytes"] = p.chunk_bytes;
    d["pass_bytes"] = p.pass_bytes;
    d["map_window"] = p.map_window;
    d["cap_lines"] = p.cap_lines;
    d["cap"] = p.cap;
    d["ucap"] = p.ucap;
    d["rcap"] = p.rcap;
    d["device_bytes"] = p.device_bytes;
    d["budget_bytes"] = p.budget_bytes;
    d["why"] = p.why;
    return d;
  }, py::arg("cfg"), py::arg("max_bytes"), py::arg("max_lines"), py::arg("cap_records") = 0,
        py::arg("free_bytes") = 0,
        "The HBM plan of an engine's device pass (no GPU needed): sizes and device bytes.");

  py::enum_<DistStrategy>(m, "DistStrategy")
      .value("auto", DistStrategy::kAuto)
      .value("shuffle", DistStrategy::kShuffle)
      .value("gather", DistStrategy::kGather)
      .value("local", DistStrategy::kLocal);
  py::class_<DistConfig>(m, "DistConfig")
      .def(py::init<>())
      .def_readwrite("job", &DistConfig::job)
      .def_readwrite("world", &DistConfig::world)
      .def_readwrite("samples_per_rank", &DistConfig::samples_per_rank)
      .def_readwrite("gather", &DistConfig::gather)
      .def_readwrite("strategy", &DistConfig::strategy)
      .def_readwrite("gather_max_records", &DistConfig::gather_max_records);

  py::class_<PyResult>(m, "Result")
      .def("entries", &PyResult::entries)
      .def("times", &PyResult::times)
      .def("format", &PyResult::format, py::arg("cpu_format") = false)
      .def("write_kiv", [](const PyResult& p, const std::string& path) { write_kiv_results(path, p.r); },
           py::arg("path"), "The results as the reference's 40-B KeyIntValuePair records.")
      .def_property_readonly("num_lines", [](const PyResult& p) { return p.r.num_lines; })
      .def_property_readonly("num_tokens", [](const PyResult& p) { return p.r.num_tokens; })
      .def_property_readonly("num_unique", [](const PyResult& p) { return p.r.num_unique; })
      .def_property_readonly("overflow_lines", [](const PyResult& p) { return p.r.overflow_lines; })
      .def_property_readonly("truncated", [](const PyResult& p) { return p.r.truncated; })
      .def_property_readonly("max_key_len", [](const PyResult& p) { return p.r.max_key_len; })
      .def_property_readonly("compact", [](const PyResult& p) { return p.r.entries.compact(); },
                             "entries are the device's compact records (kv.hpp)")
      .def_property_readonly("wire_bytes", [](const PyResult& p) { return p.r.entries.wire_bytes(); },
                             "bytes the device wrote for the entries (compact or 40-B records)")
      .def_static("from_compact", [](const std::vector<u64>& words,
                                     const std::vector<std::pair<u64, u64>>& segs, u64 val_base) {
        // host-side decoder test: segments (word offset, entries) over a word buffer
        auto buf = std::make_shared<std::vector<u64>>(words);
        std::vector<EntrySegment> sv;
        u64 n = 0;
        for (const auto& sg : segs) {
          LOCUST_CHECK_ARG(sg.first <= buf->size(), "segment beyond the words");
          sv.push_back({buf->data() + sg.first, sg.second});
          n += sg.second;
        }
        PyResult p;
        p.r.entries.adopt_compact(buf, std::move(sv), n);
        p.r.val_base = val_base;
        p.r.num_unique = n;
        return p;
      }, py::arg("words"), py::arg("segments"), py::arg("val_base") = 0);

  py::class_<PyGpuEngine>(m, "GpuEngine")
      .def(py::init<const JobConfig&, u64, u64>(), py::arg("cfg"), py::arg("max_bytes"),
           py::arg("max_lines"))
      .def("run", &PyGpuEngine::run)
      .def("load", &PyGpuEngine::load)
      .def("run_loaded", &PyGpuEngine::run_loaded)
      .def("stats", &PyGpuEngine::stats)
      .def("partition_map", [](PyGpuEngine& e) {
        std::vector<u64> lo;
        const bool tuned = e.engine().partition_map(&lo);
        return py::make_tuple(tuned, lo);
      }, "(tuned, the kDictParts + 1 range starts) after any background retune")
      .def("set_partition_map", [](PyGpuEngine& e, const std::vector<u64>& lo) {
        return e.engine().set_partition_map(lo);
      }, py::arg("lo"))
      .def("run_text", &PyGpuEngine::run_text, py::arg("text"))
      .def("run_file", &PyGpuEngine::run_file, py::arg("path"),
           "Stream a file through this (streaming) engine, piece by piece.")
      .def("map_stage", &PyGpuEngine::map_stage)
      .def("reduce_stage", &PyGpuEngine::reduce_stage)
      .def("sort_keys", &PyGpuEngine::sort_keys)
      .def("compact_slots", &PyGpuEngine::compact_slots)
      .def("reduce_sorted", &PyGpuEngine::reduce_sorted)
      .def("merge_runs", &PyGpuEngine::merge_runs)
      .def_property_readonly("capacity", &PyGpuEngine::capacity);

  m.def("cpu_run", [](const JobConfig& cfg, const std::string& text) {
    CpuWordCount eng(cfg);
    return PyResult{eng.run(as_input(text))};
  });
  m.def("cpu_map_stage", [](const JobConfig& cfg, const std::string& text) {
    CpuWordCount eng(cfg);
    std::vector<py::bytes> out;
    for (const auto& k : eng.run_map_stage(as_input(text), nullptr)) out.emplace_back(key_to_string(k));
    return out;
  });
  m.def("run_multi_schedule", &run_multi_schedule, py::arg("text"), py::arg("schedule"),
        py::arg("comm") = "auto",
        "Several jobs back to back on the same in-process ranks; [(Result, info)] of rank 0.");
  m.def("run_multi", &run_multi, py::arg("text"), py::arg("cfg"), py::arg("comm") = "auto",
        "Multi-rank WordCount in this process (one thread per rank): an RCCL clique "
        "(ncclCommInitAll) when every rank has a GPU of its own, else loopback.");
  m.def("run_multi_file", &run_multi_file, py::arg("path"), py::arg("cfg"),
        py::arg("comm") = "auto",
        "Multi-rank WordCount of a file in this process: rank r reads only its own "
        "line-aligned byte range (pinned one-pass read, or streamed past one pass); "
        "returns (rank 0's result, per-rank info dicts).");
  m.def("file_shards", [](const std::string& path, int parts) {
    py::list out;
    for (const auto& r : file_shards(path, parts)) out.append(py::make_tuple(r.offset, r.bytes));
    return out;
  }, py::arg("path"), py::arg("parts"), "Line-aligned byte ranges (offset, bytes) of a file.");
  m.def("peer_access", &enable_peer_access, py::arg("devices"),
        "Enable peer access between every pair of the devices; returns the n x n matrix "
        "(row-major) of direct-access flags.");
  m.def("peer_access_row", &peer_access_row, py::arg("device"),
        "hipDeviceCanAccessPeer(device, d) for every visible device d.");
  m.def("device_count", &visible_device_count,
        "Visible GPUs (initialises the HIP runtime in this process).");
  m.def("local_comm_for", [](const DistConfig& cfg, const std::string& comm) {
    return resolve_local_comm(cfg, local_comm(comm)) == LocalComm::kRccl ? "rccl" : "loopback";
  }, py::arg("cfg"), py::arg("comm") = "auto");

  m.def(
      "gen_text",
      [](u64 lines, u64 bytes, u64 seed, u32 vocab, double zipf_s, u64 first_block, u32 threads) {
        GenSpec g;
        g.lines = lines;
        g.bytes = bytes;
        g.seed = seed;
        g.vocab = vocab;
        g.zipf_s = zipf_s;
        g.first_block = first_block;
        g.threads = threads;
        std::string out;
        {
          py::gil_scoped_release nogil;
          gen_text(g, &out);
        }
        return py::bytes(out);
      },
      py::arg("lines") = 0, py::arg("bytes") = 0, py::arg("seed") = 1, py::arg("vocab") = 50000,
      py::arg("zipf_s") = 1.0, py::arg("first_block") = 0, py::arg("threads") = 0,
      "Synthetic Hamlet-shaped text (deterministic in seed and 1,024-line block).");
  m.def("gen_vocabulary", [](u32 vocab, u64 seed) {
    std::vector<py::bytes> out;
    for (const auto& w : gen_vocabulary(vocab, seed)) out.emplace_back(w);
    return out;
  }, py::arg("vocab"), py::arg("seed") = 1);

  py::class_<HostText>(m, "HostText",
                       "Input text in pinned host memory (DMA without staging; any size).")
      .def(py::init<u64>(), py::arg("capacity"))
      .def_static(
          "from_bytes",
          [](const std::string& b) {
            auto t = std::make_unique<HostText>(b.size());
            std::memcpy(t->data(), b.data(), b.size());
            t->set_size(b.size(), count_lines(b.data(), b.size()));
            return t;
          },
          py::arg("data"))
      .def_static(
          "generate",
          [](u64 lines, u64 bytes, u64 seed, u32 vocab, double zipf_s, u64 first_block,
             u32 threads, u64 capacity) {
            GenSpec g;
            g.lines = lines;
            g.bytes = bytes;
            g.seed = seed;
            g.vocab = vocab;
            g.zipf_s = zipf_s;
            g.first_block = first_block;
            g.threads = threads;
            // lines mode: ~44 B per line on average, 100 B at most
            const u64 cap = capacity ? capacity : (bytes ? bytes : lines * 100 + 64);
            auto t = std::make_unique<HostText>(cap);
            u64 nl = 0, n = 0;
            {
              py::gil_scoped_release nogil;
              n = gen_text_into(g, t->data(), cap, &nl);
            }
            t->set_size(n, nl);
            return t;
          },
          py::arg("lines") = 0, py::arg("bytes") = 0, py::arg("seed") = 1,
          py::arg("vocab") = 50000, py::arg("zipf_s") = 1.0, py::arg("first_block") = 0,
          py::arg("threads") = 0, py::arg("capacity") = 0)
      .def_property_readonly("size", &HostText::size)
      .def_property_readonly("lines", &HostText::lines)
      .def_property_readonly("pinned", &HostText::pinned)
      .def("to_bytes", [](const HostText& t) { return py::bytes(t.data(), t.size()); });

  m.def(
      "device_string_selftest",
      [](const std::vector<std::string>& strings, const std::vector<int>& ints,
         const std::string& delims) {
        std::vector<StringTestOut> rows;
        {
          py::gil_scoped_release nogil;
          rows = run_string_selftest(strings, ints, delims);
        }
        py::list out;
        for (const auto& o : rows) {
          py::list offs;
          for (int k = 0; k < std::min(o.ntok, 8); ++k) offs.append(o.tok_off[k]);
          out.append(py::make_tuple(o.len, o.cmp_next, o.copy_len, py::bytes(o.copy), o.ntok,
                                    offs, std::string(o.itoa_buf)));
        }
        return out;
      },
      py::arg("strings"), py::arg("ints"), py::arg("delims"),
      "Run strlen/strcmp/strcpy_bounded/strtok_r/itoa on the GPU (one thread per string).");

  py::class_<PyDistRank>(m, "DistRank")
      .def(py::init<const DistConfig&, int, const std::string&, const std::string&, int, u64, u64,
                    double, int>(),
           py::arg("cfg"), py::arg("rank"), py::arg("comm"), py::arg("host"), py::arg("port"),
           py::arg("max_bytes"), py::arg("max_lines"), py::arg("timeout_s") = 300.0,
           py::arg("listen_fd") = -1)
      .def("add_engine", &PyDistRank::add_engine, py::arg("max_bytes"), py::arg("max_lines"))
      .def("use_engine", &PyDistRank::use_engine)
      .def_property_readonly("comm_count", &PyDistRank::comm_count)
      .def_property_readonly("comm_name", &PyDistRank::comm_name)
      .def("run", &PyDistRank::run, py::arg("shard"), py::arg("first_line") = 0)
      .def("load", &PyDistRank::load, py::arg("shard"), py::arg("first_line") = 0)
      .def("run_loaded", &PyDistRank::run_loaded)
      .def("load_text", &PyDistRank::load_text, py::arg("text"), py::arg("first_line") = 0,
           py::keep_alive<1, 2>())
      .def("set_strategy", &PyDistRank::set_strategy)
      .def("barrier", &PyDistRank::barrier)
      .def("allreduce_max", &PyDistRank::allreduce_max)
      .def("allgather_bytes", &PyDistRank::allgather_bytes)
      .def_property_readonly("rank", &PyDistRank::rank)
      .def_property_readonly("size", &PyDistRank::size);

  m.def("load_lines",
        [](const std::string& path, i64 start, i64 end, bool ref_compat) {
          LoadedText t = load_lines(path, start, end, ref_compat);
          return py::make_tuple(py::bytes(t.storage.data(), t.storage.size()), t.input.num_lines,
                                t.input.first_line, t.file_lines);
        },
        py::arg("path"), py::arg("line_start") = -1, py::arg("line_end") = -1,
        py::arg("ref_compat") = false);
  m.def("gpu_placement", [](const std::string& bdf, const std::string& sys_root) {
    const GpuPlacement pl = placement_for_bdf(bdf, sys_root);
    return py::make_tuple(pl.bdf, pl.numa_node, pl.cpus);
  }, py::arg("bdf"), py::arg("sys_root") = "/sys");
  m.def("parse_cpulist", &parse_cpulist);
  m.def("plan_rank_slices", [](u64 header, u64 region, u32 regions, const std::vector<int>& nodes,
                               u64 page) {
    py::list out;
    for (const auto& s : plan_rank_slices(header, region, regions, nodes, page))
      out.append(py::make_tuple(s.offset, s.bytes, s.node));
    return out;
  }, py::arg("header"), py::arg("region"), py::arg("regions"), py::arg("nodes"),
        py::arg("page") = 4096, "NUMA slices (offset, bytes, node) of a shared output segment");
  m.def("spans_numa_nodes", &spans_numa_nodes);
  // A shm segment placed by `plan` ([(offset, bytes, node)]): returns the node of each
  // page's first byte after the segment was reserved and touched (-1: unknown).
  m.def("shm_placement_probe", [](u64 bytes, const std::vector<std::tuple<u64, u64, int>>& plan) {
    std::vector<NumaSlice> pl;
    for (const auto& t : plan) pl.push_back({std::get<0>(t), std::get<1>(t), std::get<2>(t)});
    ShmSegment seg;
    seg.open(shm_segment_name(new_group_token(), 1), align_up(bytes, 4096), &pl);
    std::vector<int> nodes;
    for (u64 o = 0; o < seg.bytes(); o += 4096) {
      seg.data()[o] = 1;
      nodes.push_back(page_node(seg.data() + o));
    }
    seg.close();
    return nodes;
  }, py::arg("bytes"), py::arg("plan"));
  // the shared output segment (locust/shm.hpp), for host-side tests
  py::class_<ShmSegment>(m, "ShmSegment")
      .def(py::init([](const std::string& name, u64 bytes) {
             auto s = std::make_unique<ShmSegment>();
             s->open(name, bytes);
             return s;
           }),
           py::arg("name"), py::arg("bytes"))
      .def_property_readonly("bytes", &ShmSegment::bytes)
      .def_property_readonly("name", &ShmSegment::name)
      .def_property_readonly("linked", &ShmSegment::linked)
      .def("write", [](ShmSegment& s, u64 off, const std::string& b) {
        LOCUST_CHECK_ARG(off + b.size() <= s.bytes(), "write past the segment");
        std::memcpy(s.data() + off, b.data(), b.size());
      })
      .def("read", [](ShmSegment& s, u64 off, u64 n) {
        LOCUST_CHECK_ARG(off + n <= s.bytes(), "read past the segment");
        return py::bytes(s.data() + off, n);
      })
      .def("unlink", &ShmSegment::unlink)
      .def("close", &ShmSegment::close);
  m.def("dev_cache_stats", [] {  // the process-wide device block cache (devcache.hpp)
    size_t bytes = 0;
    const size_t n = dev_block_cached(&bytes);
    py::dict d;
    d["blocks"] = n;
    d["bytes"] = bytes;
    return d;
  });
  m.def("dev_cache_trim", &dev_block_trim);
  m.def("shm_segment_name", &shm_segment_name);
  m.def("shm_segment_bytes", &shm_segment_bytes);
  m.def("next_segment_gen", &next_segment_gen);
  m.def("new_group_token", &new_group_token);
  m.def("file_source_chunks",  // the streamed file source's chunks (tests)
        [](const std::string& path, u64 cap, u32 threads) {
          auto src = open_file_source(path, threads);
          std::vector<char> buf(cap);
          py::list parts;
          for (u64 n; (n = src->next(buf.data(), cap)) != 0;) parts.append(py::bytes(buf.data(), n));
          return py::make_tuple(parts, src->lines());
        },
        py::arg("path"), py::arg("cap"), py::arg("threads") = 2);
  m.def("text_window",  // the in-memory window (the loader's reference semantics)
        [](const std::string& text, i64 start, i64 end, bool ref_compat) {
          LoadedText t = text_from_buffer(text.data(), text.size(), start, end, ref_compat);
          return py::make_tuple(py::bytes(t.storage.data(), t.storage.size()), t.input.num_lines,
                                t.input.first_line, t.file_lines);
        },
        py::arg("text"), py::arg("line_start") = -1, py::arg("line_end") = -1,
        py::arg("ref_compat") = false);
  m.def("shard_bounds", [](const std::string& text, int parts) {
    TextInput in = as_input(text);
    py::list out;
    for (const auto& s : shard_text(in, parts))
      out.append(py::make_tuple((u64)(s.data - in.data), s.bytes, s.num_lines, s.first_line));
    return out;
  });
  m.def("strtok_r_tokens", &strtok_r_tokens, py::arg("line"), py::arg("delims") = std::string(kDefaultDelims));
  m.def("itoa", [](int n, int base) {
    char buf[40];
    return std::string(d_itoa(n, buf, base));
  });
  m.def("strcmp", [](const std::string& a, const std::string& b) { return d_strcmp(a.c_str(), b.c_str()); });
  m.def("part_map_build", [](const std::vector<std::pair<std::string, u64>>& keys, u32 max_distinct) {
    // Balanced partition map (locust/partmap.hpp) for sorted (key, count) pairs: the
    // tables plus the predicted largest partition work.
    std::vector<WordCountEntry> e(keys.size());
    for (size_t i = 0; i < keys.size(); ++i) {
      e[i].key = to_key(keys[i].first);
      e[i].count = keys[i].second;
    }
    PartMapTables t;
    const u64 pred = part_map_from_entries(EntryList(std::vector<WordCountEntry>(e)), &t, max_distinct);
    py::dict d;
    d["lo"] = std::vector<u64>(t.lo, t.lo + kDictParts + 1);
    d["predicted_max"] = pred;
    std::vector<u32> part(e.size());  // partition of every input key
    for (size_t i = 0; i < e.size(); ++i) part[i] = part_map_lookup(t, e[i].key.w[0]);
    d["part"] = part;
    return d;
  }, py::arg("keys"), py::arg("max_distinct") = 1024);
  m.def("part_of_key", [](const std::vector<u64>& lo, const std::string& key) {
    LOCUST_CHECK_ARG(lo.size() == (size_t)kDictParts + 1, "lo needs kDictParts + 1 entries");
    return part_of_w0(lo.data(), to_key(key).w[0]);
  });
  m.def("pack_key", [](const std::string& s) {
    PackedKey k = to_key(s);
    return std::vector<u64>(k.w, k.w + kKeyWords);
  });
  m.def("write_spill",
        [](const std::string& path, const std::vector<std::pair<std::string, u64>>& recs,
           const std::string& fmt) {
          std::vector<KeyCount> v;
          for (const auto& r : recs) {
            KeyCount kc{};
            PackedKey k = to_key(r.first);
            for (int w = 0; w < kKeyWords; ++w) kc.w[w] = k.w[w];
            kc.count = r.second;
            v.push_back(kc);
          }
          write_spill(path, v, fmt == "binary" ? SpillFormat::kBinary
                               : fmt == "kiv"  ? SpillFormat::kKiv
                                               : SpillFormat::kText);
        }, py::arg("path"), py::arg("recs"), py::arg("fmt") = "text");
  m.def("read_kiv", [](const std::string& path) {
    py::list out;
    for (const auto& r : read_kiv(path))
      out.append(py::make_tuple(py::bytes(key_to_string(r.key)), r.value, r.count));
    return out;
  }, py::arg("path"), "KeyIntValuePair records of a kiv file: (key, value, count).");
  m.def("read_spill", [](const std::string& path) {
    py::list out;
    for (const auto& r : read_spill(path)) {
      PackedKey k;
      for (int w = 0; w < kKeyWords; ++w) k.w[w] = r.w[w];
      out.append(py::make_tuple(py::bytes(key_to_string(k)), r.count));
    }
    return out;
  });
  m.def("find_line_window", [](const std::string& path, i64 s, i64 e) {
    py::gil_scoped_release nogil;
    const LineWindow w = find_line_window(path, s, e);
    return std::make_tuple(w.begin, w.end, w.lines);
  }, py::arg("path"), py::arg("line_start"), py::arg("line_end"),
        "(begin, end, lines) of the line window [line_start, line_end) of a file");
  m.def("byte_window", [](const std::string& path, u64 a, u64 b) {
    py::gil_scoped_release nogil;
    const LineWindow w = byte_window(path, a, b);
    return std::make_tuple(w.begin, w.end, w.lines);
  }, py::arg("path"), py::arg("begin"), py::arg("end"),
        "(begin, end, 0): bytes [begin, end) of a file moved to line starts");
  m.def("line_start_at", &line_start_at, py::arg("path"), py::arg("offset"));
  m.def("count_newlines", [](py::bytes b) {
    const std::string_view v = b;
    return count_newlines(v.data(), v.size());
  });
  m.def("count_lines", [](py::bytes b) {
    const std::string_view v = b;
    return count_lines(v.data(), v.size());
  });
  m.def("line_index_cache_path", &line_index_cache_path, py::arg("path"));
  m.def("native_stage", [] { return py::make_tuple(std::string(current_stage()), stages_entered()); },
        "(the distributed stage this process last entered, stages entered so far)");
  m.def("spill_index", [](const std::string& spill) -> py::object {
    SpillIndex x;
    if (!read_spill_index(spill, &x)) return py::none();
    py::dict d;
    d["sorted"] = x.sorted;
    d["distinct"] = x.distinct;
    d["records"] = x.records;
    d["total_count"] = x.total_count;
    d["spill_bytes"] = x.spill_bytes;
    d["stride"] = x.stride;
    py::list smp;
    for (const SpillSample& v : x.samples)
      smp.append(py::make_tuple(py::bytes(key_to_string(v.key)), v.record, v.offset, v.count_before));
    d["samples"] = smp;
    return d;
  }, py::arg("spill"), "The spill's sparse index (<spill>.idx), or None.");
  m.def("reducer_splitters", [](const std::vector<std::string>& spills, int reducers) {
    std::vector<SpillIndex> idx(spills.size());
    for (size_t k = 0; k < spills.size(); ++k) {
      if (!read_spill_index(spills[k], &idx[k])) {
        std::vector<KeyCount> v = read_spill(spills[k]);
        sort_combine(&v);
        idx[k] = index_records(v);
      }
    }
    py::list out;
    for (const PackedKey& k : plan_reducer_splitters(idx, reducers)) out.append(py::bytes(key_to_string(k)));
    return out;
  }, py::arg("spills"), py::arg("reducers"));
  m.def("reduce_spills", [](const JobConfig& cfg, const std::vector<std::string>& files, int reducer,
                           int reducers) {
    ReduceStageStats st;
    WordCountResult r;
    {
      py::gil_scoped_release nogil;
      r = reduce_spills(cfg, files, reducer, reducers, &st);
    }
    py::dict d;
    d["input_files"] = st.input_files;
    d["indexed_files"] = st.indexed_files;
    d["loaded_files"] = st.loaded_files;
    d["records_read"] = st.records_read;
    d["run_records"] = st.run_records;
    d["read_ms"] = st.read_ms;
    d["setup_ms"] = st.setup_ms;
    d["merge_ms"] = st.merge_ms;
    return py::make_tuple(PyResult{std::move(r)}, d);
  }, py::arg("cfg"), py::arg("files"), py::arg("reducer") = 0, py::arg("reducers") = 1,
        "Stage 2 over spill files: (result, stats); key range `reducer` of `reducers`.");
  m.def("map_stage", [](const JobConfig& cfg, const std::string& file, i64 s, i64 e,
                        const std::string& spill, const std::string& fmt) {
    MapStageResult r;
    {
      py::gil_scoped_release nogil;
      r = map_stage(cfg, file, s, e, spill,
                    fmt == "binary" ? SpillFormat::kBinary : fmt == "kiv" ? SpillFormat::kKiv
                                                                         : SpillFormat::kText);
    }
    py::dict d;
    d["lines"] = r.lines;
    d["tokens"] = r.result.num_tokens;
    d["unique"] = r.result.num_unique;
    d["spill_records"] = r.spill_records;
    d["spill_bytes"] = r.index.spill_bytes;
    d["input_bytes"] = r.input_bytes;
    d["streamed"] = r.streamed;
    d["map_ms"] = r.result.times.h2d_ms + r.result.times.map_ms;
    d["process_ms"] = r.result.times.process_ms + r.result.times.reduce_ms;
    d["job_ms"] = r.job_ms;
    return d;
  }, py::arg("cfg"), py::arg("file"), py::arg("line_start"), py::arg("line_end"),
        py::arg("spill"), py::arg("fmt") = "binary",
        "Stage 1 over a line window: the combined, indexed spill (see locust/stage.hpp).");
  m.def("partmap_cache_path", &partmap_cache_path, py::arg("input"), py::arg("cfg"));
  m.def("load_partmap_cache", [](const std::string& path) -> py::object {
    std::vector<u64> lo;
    if (!load_partmap_cache(path, &lo)) return py::none();
    return py::cast(lo);
  }, py::arg("path"));
  m.def("save_partmap_cache", &save_partmap_cache, py::arg("path"), py::arg("lo"));
  py::register_exception<Error>(m, "LocustError");
}
