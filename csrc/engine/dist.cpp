// Distributed WordCount driver (backend-agnostic: any Communicator x any ShardEngine).
// See locust/dist.hpp for the stage list and SURVEY.md §2.4/§5.8 for the design.
#include "locust/dist.hpp"

#include <algorithm>
#include <cstring>
#include <exception>
#include <functional>

namespace locust {

std::vector<TextInput> shard_text(const TextInput& in, int parts) {
  LOCUST_CHECK_ARG(parts >= 1, "parts must be >= 1");
  std::vector<TextInput> out;
  u64 begin = 0;
  u64 line = in.first_line;
  for (int p = 0; p < parts; ++p) {
    u64 end = p == parts - 1 ? in.bytes : std::max(begin, (in.bytes * (u64)(p + 1)) / (u64)parts);
    if (end < in.bytes && end > 0) {
      // move to the start of the next line: the byte after the next '\n' at/after end-1
      const char* nl = static_cast<const char*>(
          memchr(in.data + end - 1, '\n', (size_t)(in.bytes - (end - 1))));
      end = nl ? (u64)(nl - in.data) + 1 : in.bytes;
    }
    if (end < begin) end = begin;
    TextInput s;
    s.data = in.data + begin;
    s.bytes = end - begin;
    // lines in this shard: newlines + a final partial line
    u64 nls = 0;
    for (const char* q = s.data; (q = static_cast<const char*>(memchr(q, '\n', (size_t)(s.data + s.bytes - q)))) != nullptr; ++q)
      ++nls;
    s.num_lines = nls + ((s.bytes && s.data[s.bytes - 1] != '\n') ? 1 : 0);
    s.first_line = line;
    line += s.num_lines;
    out.push_back(s);
    begin = end;
  }
  return out;
}

namespace {

struct MapStatsWire {
  u64 lines, tokens, overflow, truncated, max_key_len, local_records;
};

// Weighted quantile splitters from every rank's evenly spaced samples.
std::vector<PackedKey> choose_splitters(const std::vector<PackedKey>& samples, u32 s,
                                        const std::vector<u64>& counts, int parts) {
  struct W {
    PackedKey k;
    double w;
  };
  std::vector<W> all;
  double total = 0;
  for (size_t r = 0; r < counts.size(); ++r) {
    if (!counts[r]) continue;
    const double w = (double)counts[r] / (double)s;
    for (u32 i = 0; i < s; ++i) all.push_back({samples[r * s + i], w});
    total += (double)counts[r];
  }
  std::sort(all.begin(), all.end(), [](const W& a, const W& b) { return key_less(a.k, b.k); });
  std::vector<PackedKey> sp;
  double run = 0;
  size_t i = 0;
  for (int p = 1; p < parts; ++p) {
    const double target = total * p / parts;
    while (i < all.size() && run + all[i].w <= target) run += all[i++].w;
    PackedKey k;
    if (i < all.size()) {
      k = all[i].k;
    } else {
      for (int w = 0; w < kKeyWords; ++w) k.w[w] = ~0ull;
    }
    sp.push_back(k);
  }
  return sp;
}

}  // namespace

DistResult run_distributed(const DistConfig& cfg, Communicator& comm, ShardEngine& eng,
                           const TextInput& shard) {
  const int P = comm.size();
  const int me = comm.rank();
  log_rank() = me;
  DistResult res;
  std::string local_msg;
  auto run_local = [&](const char* stage, const std::function<void()>& fn) {
    int err = 0;
    if (fault_injected(me, stage)) {
      err = 1;
      local_msg = "injected fault (LOCUST_FAULT)";
    } else {
      try {
        fn();
      } catch (const std::exception& e) {
        err = 1;
        local_msg = e.what();
      }
    }
    const int bad = comm.agree(err);
    if (bad >= 0)
      throw Error(std::string("distributed job failed in stage '") + stage + "' on rank " +
                  std::to_string(bad) + (bad == me ? ": " + local_msg : ""));
  };

  const u64 t0 = now_ns();
  // ---------------- map ----------------
  u64 n_local = 0;
  run_local("map", [&] { n_local = eng.map_local(shard, cfg.job.combine); });
  res.local_records = n_local;
  const u64 t1 = now_ns();

  // ---------------- shuffle ----------------
  const u32 S = std::max<u32>(cfg.samples_per_rank, 1);
  std::vector<PackedKey> mine_samples;
  run_local("shuffle", [&] { mine_samples = eng.sample(S); });
  std::vector<PackedKey> samples((size_t)P * S);
  std::vector<u64> counts((size_t)P);
  comm.allgather_host(mine_samples.data(), samples.data(), (u64)S * sizeof(PackedKey));
  comm.allgather_host(&n_local, counts.data(), sizeof(u64));
  const std::vector<PackedKey> splitters = choose_splitters(samples, S, counts, P);
  std::vector<u64> offs;
  run_local("partition", [&] { offs = eng.bucket_offsets(splitters); });
  std::vector<u64> send_cnt((size_t)P), matrix((size_t)P * P);
  for (int p = 0; p < P; ++p) send_cnt[(size_t)p] = offs[(size_t)p + 1] - offs[(size_t)p];
  comm.allgather_host(send_cnt.data(), matrix.data(), (u64)P * sizeof(u64));
  std::vector<u64> sb((size_t)P), so((size_t)P), rb((size_t)P), ro((size_t)P);
  u64 n_recv = 0;
  for (int p = 0; p < P; ++p) {
    sb[(size_t)p] = send_cnt[(size_t)p] * sizeof(KeyCount);
    so[(size_t)p] = offs[(size_t)p] * sizeof(KeyCount);
    const u64 r = matrix[(size_t)p * P + me];
    rb[(size_t)p] = r * sizeof(KeyCount);
    ro[(size_t)p] = n_recv * sizeof(KeyCount);
    n_recv += r;
  }
  void* recv = nullptr;
  run_local("alloc", [&] { recv = eng.recv_records(n_recv); });
  comm.alltoallv(eng.send_records(), sb.data(), so.data(), recv, rb.data(), ro.data(), eng.stream());
  for (int p = 0; p < P; ++p) {
    if (p != me) {
      res.sent_bytes += sb[(size_t)p];
      res.recv_bytes += rb[(size_t)p];
    }
  }
  const u64 t2 = now_ns();

  // ---------------- reduce ----------------
  u64 total = 0, uniq = 0;
  run_local("reduce", [&] { eng.reduce_received(n_recv, &total, &uniq); });
  std::vector<u64> totals((size_t)P);
  comm.allgather_host(&total, totals.data(), sizeof(u64));
  u64 offset = 0;
  for (int p = 0; p < me; ++p) offset += totals[(size_t)p];
  std::vector<WordCountEntry> entries;
  run_local("finalize", [&] { eng.finalize(offset, &entries); });
  res.range_tokens = total;
  res.range_unique = uniq;
  const u64 t3 = now_ns();

  // ---------------- gather + stats ----------------
  WordCountResult local_stats;
  eng.map_stats(&local_stats);
  MapStatsWire mw{shard.num_lines, local_stats.num_tokens, local_stats.overflow_lines,
                  local_stats.truncated, local_stats.max_key_len, n_local};
  std::vector<MapStatsWire> all_stats((size_t)P);
  comm.allgather_host(&mw, all_stats.data(), sizeof(MapStatsWire));
  WordCountResult& r = res.result;
  for (const auto& s : all_stats) {
    r.num_lines += s.lines;
    r.num_tokens += s.tokens;
    r.overflow_lines += s.overflow;
    r.truncated += s.truncated;
    r.max_key_len = std::max(r.max_key_len, s.max_key_len);
  }
  if (cfg.gather) {
    std::vector<char> buf;
    comm.gatherv_host(entries.data(), entries.size() * sizeof(WordCountEntry), &buf, nullptr, 0);
    if (me == 0) {
      r.entries.resize(buf.size() / sizeof(WordCountEntry));
      if (!buf.empty()) std::memcpy(r.entries.data(), buf.data(), buf.size());
    }
  } else {
    r.entries = std::move(entries);
  }
  r.num_unique = me == 0 && cfg.gather ? r.entries.size() : uniq;
  const u64 t4 = now_ns();
  res.map_ms = (t1 - t0) * 1e-6;
  res.shuffle_ms = (t2 - t1) * 1e-6;
  res.reduce_ms = (t3 - t2) * 1e-6;
  res.gather_ms = (t4 - t3) * 1e-6;
  res.total_ms = (t4 - t0) * 1e-6;
  r.times.map_ms = res.map_ms;
  r.times.process_ms = res.shuffle_ms;
  r.times.reduce_ms = res.reduce_ms;
  r.times.wall_ms = res.total_ms;
  return res;
}

}  // namespace locust
