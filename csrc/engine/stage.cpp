// Reduce side of the stage split (see locust/stage.hpp).
#include "locust/stage.hpp"

#include <algorithm>
#include <exception>
#include <queue>
#include <thread>

namespace locust {

void combine_adjacent(std::vector<KeyCount>* recs) {
  std::vector<KeyCount>& v = *recs;
  size_t o = 0;
  for (size_t i = 0; i < v.size(); ++i) {
    if (o && key_compare(v[o - 1].w, v[i].w) == 0)
      v[o - 1].count += v[i].count;
    else
      v[o++] = v[i];
  }
  v.resize(o);
}

void sort_combine(std::vector<KeyCount>* recs) {
  std::sort(recs->begin(), recs->end(), record_less);
  combine_adjacent(recs);
}

std::vector<WordCountEntry> merge_runs_host(const std::vector<std::vector<KeyCount>>& runs) {
  struct Head {
    const KeyCount* p;
    const KeyCount* end;
  };
  auto later = [](const Head& a, const Head& b) { return key_compare(a.p->w, b.p->w) > 0; };
  std::priority_queue<Head, std::vector<Head>, decltype(later)> q(later);
  size_t total = 0;
  for (const auto& r : runs) {
    total += r.size();
    if (!r.empty()) q.push({r.data(), r.data() + r.size()});
  }
  std::vector<WordCountEntry> out;
  out.reserve(total);
  while (!q.empty()) {
    Head h = q.top();
    q.pop();
    if (!out.empty() && key_compare(out.back().key.w, h.p->w) == 0) {
      out.back().count += h.p->count;
    } else {
      WordCountEntry e;
      for (int w = 0; w < kKeyWords; ++w) e.key.w[w] = h.p->w[w];
      e.count = h.p->count;
      out.push_back(e);
    }
    if (++h.p != h.end) q.push(h);
  }
  return out;
}

SpillIndex index_records(const std::vector<KeyCount>& recs) {
  SpillIndex idx;
  idx.sorted = idx.distinct = true;
  idx.records = recs.size();
  idx.stride = std::max<u64>(16, div_up(recs.size(), 256));
  u64 cum = 0;
  for (u64 i = 0; i < recs.size(); ++i) {
    if (i % idx.stride == 0) {
      SpillSample s;
      for (int w = 0; w < kKeyWords; ++w) s.key.w[w] = recs[i].w[w];
      s.record = i;
      s.offset = i;  // in-memory: the record number
      s.count_before = cum;
      idx.samples.push_back(s);
    }
    cum += recs[i].count;
  }
  idx.total_count = cum;
  return idx;
}

std::vector<PackedKey> plan_reducer_splitters(const std::vector<SpillIndex>& idx, int reducers) {
  LOCUST_CHECK_ARG(reducers >= 1, "reducers must be >= 1");
  struct W {
    PackedKey key;
    u64 weight;
  };
  std::vector<W> all;
  u64 total = 0;
  for (const SpillIndex& x : idx)
    for (size_t j = 0; j < x.samples.size(); ++j) {
      const u64 next = j + 1 < x.samples.size() ? x.samples[j + 1].record : x.records;
      const u64 wgt = next > x.samples[j].record ? next - x.samples[j].record : 1;
      all.push_back({x.samples[j].key, wgt});
      total += wgt;
    }
  std::sort(all.begin(), all.end(),
            [](const W& a, const W& b) { return key_compare(a.key.w, b.key.w) < 0; });
  // Splitter i is the first sample key at which the weight of the samples BEFORE it
  // reaches i/R of the total: equal keys are one unit, so the cut does not depend on the
  // order of the indexes.  An empty or tiny input repeats its last key (empty ranges).
  std::vector<PackedKey> spl;
  u64 before = 0;
  size_t j = 0;
  for (int i = 1; i < reducers; ++i) {
    // before < total * i / R, exactly (the launcher's Python planner mirrors this)
    const unsigned __int128 target = (unsigned __int128)total * (unsigned)i;
    while (j < all.size() && (unsigned __int128)before * (unsigned)reducers < target) {
      const size_t k0 = j;
      while (j < all.size() && key_compare(all[j].key.w, all[k0].key.w) == 0) before += all[j++].weight;
    }
    PackedKey k{};
    if (j < all.size()) {
      k = all[j].key;
    } else {
      for (int w = 0; w < kKeyWords; ++w) k.w[w] = ~0ull;  // beyond every key
    }
    spl.push_back(k);
  }
  return spl;
}

MapStageResult map_stage(const JobConfig& cfg_in, const std::string& file, const MapWindow& win,
                         const std::string& spill, SpillFormat fmt) {
  constexpr u64 kDefaultStreamChunk = 256ull << 20;
  const bool cpu = cfg_in.backend == Backend::kCpu;
  const bool lwin = !win.by_bytes && win.line_start >= 0;
  LOCUST_CHECK_ARG(!(win.by_bytes && cfg_in.ref_compat),
                   "a byte window is not a reference-compatible stage 1 (use a line window)");
  MapStageResult out;
  WordCountResult& r = out.result;
  std::vector<KeyCount> recs;
  const u64 t0 = now_ns();
  LineWindow w;
  if (win.by_bytes) {
    w = byte_window(file, win.byte_begin, win.byte_end);
  } else if (lwin && !cfg_in.ref_compat) {
    w = find_line_window(file, win.line_start, win.line_end);
  } else {
    w.end = file_size(file);
  }
  out.byte_begin = w.begin;
  out.byte_end = w.end;
  out.input_bytes = w.end - w.begin;
  const u64 tw = now_ns();
  out.window_ms = (tw - t0) * 1e-6;
  u64 ts = tw, tr = tw;
  if (cpu || cfg_in.ref_compat) {
    LoadedText text;
    if (!cfg_in.ref_compat) {  // the window's bytes (a line or byte window, or the file)
      std::vector<char> buf(out.input_bytes);
      read_file_range_into(file, buf.data(), w.begin, out.input_bytes, nullptr);
      text = text_from_buffer(buf.data(), buf.size(), -1, -1, false);
    } else {
      const bool use_window = lwin && !(cpu && cfg_in.ref_compat);
      text = load_lines(file, use_window ? win.line_start : -1, use_window ? win.line_end : -1,
                        cfg_in.ref_compat);
      out.input_bytes = text.input.bytes;
    }
    out.lines = text.input.num_lines;
    ts = now_ns();
    if (cfg_in.ref_compat) {
      std::vector<PackedKey> toks;
      if (cpu) {
        toks = CpuWordCount(cfg_in).run_map_stage(text.input, &r);
      } else {
        GpuWordCount eng(cfg_in, std::max<u64>(out.input_bytes, 1), std::max<u64>(out.lines, 1));
        toks = eng.run_map_stage(text.input, &r);
      }
      r.num_tokens = toks.size();
      recs = tokens_to_records(toks);
    } else {
      r = CpuWordCount(cfg_in).run(text.input);
      recs = entries_to_records(r.entries);
    }
    tr = now_ns();
  } else {
    JobConfig cfg = cfg_in;
    cfg.graph = 0;  // stage events: the map and sort times
    const u64 chunk = cfg.chunk_bytes ? cfg.chunk_bytes : kDefaultStreamChunk;
    // the engine outlives the job in out.engine_keep: its teardown (~25 ms of pinned and
    // device frees for a streaming engine) is the caller's, and a one-shot CLI skips it
    if (out.input_bytes > chunk) {
      cfg.chunk_bytes = chunk;
      auto eng = std::make_shared<GpuWordCount>(cfg, out.input_bytes, out.input_bytes);
      ts = now_ns();
      auto src = open_file_range_source(file, w.begin, w.end);
      r = eng->run_source(*src);
      tr = now_ns();
      out.engine = eng->stats();
      out.lines = src->lines();
      out.streamed = true;
      out.engine_keep = eng;
    } else {
      auto eng = std::make_shared<GpuWordCount>(cfg, std::max<u64>(out.input_bytes, 1),
                                                std::max<u64>(out.input_bytes, 1));
      ts = now_ns();
      TextInput in;
      in.data = eng->input_buffer();
      in.bytes = read_file_range_into(file, eng->input_buffer(), w.begin, out.input_bytes, &out.lines);
      in.num_lines = out.lines;
      r = eng->run(in);
      tr = now_ns();
      out.engine = eng->stats();
      out.engine_keep = eng;
    }
    recs = entries_to_records(r.entries);
    if (lwin) out.lines = w.lines;
  }
  r.entries = EntryList{};
  r.num_lines = out.lines;
  const u64 t1 = now_ns();
  out.setup_ms = (ts - tw) * 1e-6;
  out.run_ms = (tr - ts) * 1e-6;
  write_spill(spill, recs, fmt, &out.index);
  write_spill_index(spill_index_path(spill), out.index);
  out.spill_records = recs.size();
  out.job_ms = (t1 - t0) * 1e-6;
  out.spill_write_ms = (now_ns() - t1) * 1e-6;
  return out;
}

namespace {

// [lo, hi) membership; a null bound is open.
bool below(const u64* k, const PackedKey* lo) { return lo && key_compare(k, lo->w) < 0; }
bool at_or_above(const u64* k, const PackedKey* hi) { return hi && key_compare(k, hi->w) >= 0; }

}  // namespace

WordCountResult reduce_spills(const JobConfig& cfg, const std::vector<std::string>& files,
                              int reducer, int reducers, ReduceStageStats* stats) {
  LOCUST_CHECK_ARG(reducers >= 1 && reducer >= 0 && reducer < reducers,
                   "--reducer r/R needs 0 <= r < R");
  LOCUST_CHECK_ARG(!files.empty(), "no spill files to reduce");
  ReduceStageStats st;
  st.input_files = files.size();
  const u64 t0 = now_ns();
  const size_t nf = files.size();
  std::vector<SpillIndex> idx(nf);
  std::vector<char> indexed(nf, 0);
  std::vector<std::vector<KeyCount>> loaded(nf);
  // Up to 8 threads over the spills, in both passes below: the files are independent.
  auto for_each_spill = [nf](const auto& fn) {
    const size_t nt = std::min<size_t>(nf, 8);
    std::vector<std::exception_ptr> err(nt);
    auto worker = [&](size_t t) {
      try {
        for (size_t k = t; k < nf; k += nt) fn(k);
      } catch (...) {
        err[t] = std::current_exception();
      }
    };
    std::vector<std::thread> th;
    for (size_t t = 1; t < nt; ++t) th.emplace_back(worker, t);
    worker(0);
    for (auto& x : th) x.join();
    for (auto& e : err)
      if (e) std::rethrow_exception(e);
  };
  std::vector<u64> nread(nf, 0);
  for_each_spill([&](size_t k) {
    if (read_spill_index(files[k], &idx[k]) && idx[k].sorted) {
      indexed[k] = 1;
      return;
    }
    // no (current) index: the whole spill, sorted and combined here (a reference-format
    // file: one "key \t1" line per token, sorted by one mapper only -- B7)
    loaded[k] = read_spill(files[k]);
    nread[k] = loaded[k].size();
    bool sorted = true;
    for (size_t i = 1; i < loaded[k].size() && sorted; ++i)
      sorted = key_compare(loaded[k][i - 1].w, loaded[k][i].w) <= 0;
    if (sorted)
      combine_adjacent(&loaded[k]);
    else
      sort_combine(&loaded[k]);
    idx[k] = index_records(loaded[k]);
  });
  for (size_t k = 0; k < nf; ++k) {
    st.indexed_files += indexed[k] ? 1 : 0;
    st.loaded_files += indexed[k] ? 0 : 1;
    st.records_read += nread[k];
  }
  if (reducers > 1) st.splitters = plan_reducer_splitters(idx, reducers);
  const PackedKey* lo = reducer > 0 ? &st.splitters[(size_t)reducer - 1] : nullptr;
  const PackedKey* hi = reducer < reducers - 1 ? &st.splitters[(size_t)reducer] : nullptr;

  // Each spill's part of the range (index seek, then the records up to the range's end).
  struct Part {
    std::vector<KeyCount> run;
    u64 base = 0, read = 0;
  };
  std::vector<Part> parts(nf);
  auto extract = [&](size_t k) {
    Part& pt = parts[k];
    std::vector<KeyCount>& run = pt.run;
    if (!indexed[k]) {
      for (const KeyCount& r : loaded[k]) {
        if (below(r.w, lo))
          pt.base += r.count;
        else if (at_or_above(r.w, hi))
          break;
        else
          run.push_back(r);
      }
      std::vector<KeyCount>().swap(loaded[k]);
      return;
    }
    const SpillIndex& x = idx[k];
    if (x.samples.empty()) return;
    // start at the last sample below the range (its count_before is exact)
    size_t j = 0;
    if (lo) {
      const auto it = std::lower_bound(
          x.samples.begin(), x.samples.end(), *lo,
          [](const SpillSample& s, const PackedKey& key) { return key_compare(s.key.w, key.w) < 0; });
      j = it == x.samples.begin() ? 0 : (size_t)(it - x.samples.begin()) - 1;
    }
    SpillReader rd(files[k]);
    rd.seek(x.samples[j].offset);
    u64 base = x.samples[j].count_before;
    KeyCount r;
    while (rd.next(&r)) {
      ++pt.read;
      if (below(r.w, lo)) {
        base += r.count;
        continue;
      }
      if (at_or_above(r.w, hi)) break;
      if (!run.empty() && key_compare(run.back().w, r.w) == 0)
        run.back().count += r.count;  // a sorted but not combined spill
      else
        run.push_back(r);
    }
    pt.base = base;
  };
  for_each_spill(extract);
  u64 val_base = 0;
  std::vector<std::vector<KeyCount>> runs;
  runs.reserve(nf);
  for (Part& pt : parts) {
    val_base += pt.base;
    st.records_read += pt.read;
    st.run_records += pt.run.size();
    if (!pt.run.empty()) runs.push_back(std::move(pt.run));
  }
  const u64 t1 = now_ns();
  WordCountResult res;
  std::vector<WordCountEntry> merged = cfg.backend == Backend::kCpu
                                           ? merge_runs_host(runs)
                                           : merge_runs_device(cfg, runs, &st.setup_ms);
  const u64 t2 = now_ns();
  res.val_base = val_base;
  res.num_unique = merged.size();
  for (const WordCountEntry& e : merged) res.num_tokens += e.count;
  for (const WordCountEntry& e : merged)
    res.max_key_len = std::max<u64>(res.max_key_len, key_bytes_used(e.key.w));
  res.entries = std::move(merged);
  st.read_ms = (t1 - t0) * 1e-6;
  st.merge_ms = (t2 - t1) * 1e-6 - st.setup_ms;
  res.times.reduce_ms = st.merge_ms;
  res.times.wall_ms = (t2 - t0) * 1e-6;
  if (stats) *stats = std::move(st);
  return res;
}

}  // namespace locust
