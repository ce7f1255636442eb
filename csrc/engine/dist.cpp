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

// Control-plane messages: every allgather carries the status word of the stage before it,
// so failure agreement costs no extra collective.  Three allgathers per job.
struct alignas(8) Msg1 {  // after map + sampling
  i32 status;
  u32 pad;
  u64 n_local;
};
struct alignas(8) Msg3 {  // after the reduce of the received key range
  i32 status;
  u32 pad;
  u64 total, uniq, lines, tokens, overflow, truncated, max_key_len;
};

DistResult run_distributed(const DistConfig& cfg, Communicator& comm, ShardEngine& eng,
                           const TextInput& shard) {
  const int P = comm.size();
  const int me = comm.rank();
  log_rank() = me;
  DistResult res;
  std::string local_msg;
  // Runs a local step, returning its status (0 ok) instead of throwing.
  auto local = [&](const char* stage, const std::function<void()>& fn) -> i32 {
    if (fault_injected(me, stage)) {
      local_msg = std::string("injected fault (LOCUST_FAULT) in stage '") + stage + "'";
      return 1;
    }
    try {
      fn();
    } catch (const std::exception& e) {
      local_msg = std::string("stage '") + stage + "': " + e.what();
      return 1;
    }
    return 0;
  };
  auto check = [&](const char* stage, const i32* statuses, u64 stride_bytes) {
    for (int r = 0; r < P; ++r) {
      const i32 st = *reinterpret_cast<const i32*>(reinterpret_cast<const char*>(statuses) +
                                                   (u64)r * stride_bytes);
      if (st)
        throw Error(std::string("distributed job failed in stage '") + stage + "' on rank " +
                    std::to_string(r) + (r == me ? ": " + local_msg : ""));
    }
  };

  const u64 t0 = now_ns();
  const u32 S = std::max<u32>(cfg.samples_per_rank, 1);
  // ---------------- map + sample, one allgather ----------------
  u64 n_local = 0;
  std::vector<PackedKey> mine_samples;
  const i32 st1 = local("map", [&] {
    n_local = eng.map_local(shard, cfg.job.combine);
    mine_samples = eng.sample(S);
  });
  if (mine_samples.size() != S) mine_samples.assign(S, PackedKey{{~0ull, ~0ull, ~0ull, ~0ull}});
  res.local_records = n_local;
  const u64 t1 = now_ns();
  const u64 m1 = sizeof(Msg1) + (u64)S * sizeof(PackedKey);
  std::vector<char> out1(m1), all1(m1 * (u64)P);
  {
    Msg1 h{st1, 0, n_local};
    std::memcpy(out1.data(), &h, sizeof(h));
    std::memcpy(out1.data() + sizeof(h), mine_samples.data(), (u64)S * sizeof(PackedKey));
  }
  comm.allgather_host(out1.data(), all1.data(), m1);
  check("map", reinterpret_cast<const i32*>(all1.data()), m1);
  std::vector<PackedKey> samples((size_t)P * S);
  std::vector<u64> counts((size_t)P);
  for (int r = 0; r < P; ++r) {
    const char* base = all1.data() + (u64)r * m1;
    Msg1 h;
    std::memcpy(&h, base, sizeof(h));
    counts[(size_t)r] = h.n_local;
    std::memcpy(&samples[(size_t)r * S], base + sizeof(h), (u64)S * sizeof(PackedKey));
  }
  const std::vector<PackedKey> splitters = choose_splitters(samples, S, counts, P);

  // ---------------- partition: one allgather of {status, send counts} ----------------
  std::vector<u64> offs;
  const i32 st2 = local("partition", [&] { offs = eng.bucket_offsets(splitters); });
  if (offs.size() != (size_t)P + 1) offs.assign((size_t)P + 1, 0);
  std::vector<u64> msg2((size_t)P + 1), matrix(((size_t)P + 1) * P);
  msg2[0] = (u64)(u32)st2;
  for (int p = 0; p < P; ++p) msg2[(size_t)p + 1] = offs[(size_t)p + 1] - offs[(size_t)p];
  comm.allgather_host(msg2.data(), matrix.data(), ((u64)P + 1) * sizeof(u64));
  check("partition", reinterpret_cast<const i32*>(matrix.data()), ((u64)P + 1) * sizeof(u64));
  std::vector<u64> sb((size_t)P), so((size_t)P), rb((size_t)P), ro((size_t)P);
  u64 n_recv = 0;
  for (int p = 0; p < P; ++p) {
    sb[(size_t)p] = msg2[(size_t)p + 1] * sizeof(KeyCount);
    so[(size_t)p] = offs[(size_t)p] * sizeof(KeyCount);
    const u64 r = matrix[(size_t)p * (P + 1) + 1 + me];
    rb[(size_t)p] = r * sizeof(KeyCount);
    ro[(size_t)p] = n_recv * sizeof(KeyCount);
    n_recv += r;
  }

  // ---------------- shuffle ----------------
  // The receive buffer is sized locally; an allocation failure surfaces in the reduce
  // status below (the all-to-all itself must be entered by every rank).
  void* recv = nullptr;
  i32 st3 = local("shuffle", [&] { recv = eng.recv_records(n_recv); });
  if (st3) n_recv = 0;  // still participate with empty receives
  if (eng.device_buffers() && !comm.device_buffers()) {
    // Device engine over a host-only communicator (TCP): stage through host memory.  This
    // is how several GPU ranks can share one device in tests (RCCL refuses that).
    std::vector<KeyCount> hs(n_local), hr(std::max<u64>(n_recv, 1));
    copy_device(hs.data(), eng.send_records(), n_local * sizeof(KeyCount), /*to_host=*/true,
                eng.stream());
    comm.alltoallv(hs.data(), sb.data(), so.data(), hr.data(), rb.data(), ro.data(), nullptr);
    if (!st3) copy_device(recv, hr.data(), n_recv * sizeof(KeyCount), /*to_host=*/false, eng.stream());
  } else {
    comm.alltoallv(eng.send_records(), sb.data(), so.data(), recv, rb.data(), ro.data(),
                   eng.stream());
  }
  for (int p = 0; p < P; ++p) {
    if (p != me) {
      res.sent_bytes += sb[(size_t)p];
      res.recv_bytes += rb[(size_t)p];
    }
  }
  const u64 t2 = now_ns();

  // ---------------- reduce, one allgather of {status, totals, map stats} ----------------
  u64 total = 0, uniq = 0;
  if (!st3) st3 = local("reduce", [&] { eng.reduce_received(n_recv, &total, &uniq); });
  WordCountResult local_stats;
  eng.map_stats(&local_stats);
  Msg3 m3{st3, 0, total, uniq, shard.num_lines, local_stats.num_tokens, local_stats.overflow_lines,
          local_stats.truncated, local_stats.max_key_len};
  std::vector<Msg3> all3((size_t)P);
  comm.allgather_host(&m3, all3.data(), sizeof(Msg3));
  check("reduce", &all3[0].status, sizeof(Msg3));
  u64 offset = 0;
  for (int p = 0; p < me; ++p) offset += all3[(size_t)p].total;
  std::vector<WordCountEntry> entries;
  eng.finalize(offset, &entries);
  res.range_tokens = total;
  res.range_unique = uniq;
  const u64 t3 = now_ns();

  // ---------------- gather ----------------
  WordCountResult& r = res.result;
  for (const auto& s : all3) {
    r.num_lines += s.lines;
    r.num_tokens += s.tokens;
    r.overflow_lines += s.overflow;
    r.truncated += s.truncated;
    r.max_key_len = std::max(r.max_key_len, s.max_key_len);
  }
  if (cfg.gather) {
    std::vector<u64> sizes((size_t)P);
    u64 all_uniq = 0;
    for (int p = 0; p < P; ++p) {
      sizes[(size_t)p] = all3[(size_t)p].uniq * sizeof(WordCountEntry);
      all_uniq += all3[(size_t)p].uniq;
    }
    if (me == 0) r.entries.resize(all_uniq);
    comm.gatherv_known(entries.data(), entries.size() * sizeof(WordCountEntry), sizes.data(),
                       me == 0 ? static_cast<void*>(r.entries.data()) : nullptr, 0);
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
