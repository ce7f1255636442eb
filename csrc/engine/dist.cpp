// Distributed WordCount driver (backend-agnostic: any Communicator x any ShardEngine).
// See locust/dist.hpp for the stage list and SURVEY.md §2.4/§5.8 for the design.
#include "locust/dist.hpp"
#include "locust/numa.hpp"
#include "locust/trace.hpp"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <chrono>
#include <functional>
#include <thread>

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

// The gather-slot job as ONE graph with the RCCL all-gather captured inside it: measured
// at one rank (79 vs 88 us per job).  A captured collective has never run with real peers
// (no multi-GPU box in development), so with several ranks the default is the separate
// launches (map graph, the collective on the stream, merge graph) -- the conventional RCCL
// use.  LOCUST_SLOT_GRAPH=1 captures at any world size, =0 never.
bool slot_graph_enabled(int world) {
  const char* v = std::getenv("LOCUST_SLOT_GRAPH");
  if (v && v[0] == '0') return false;
  if (v && v[0] == '1') return true;
  return world == 1;
}

// LOCUST_EXCHANGE=0 keeps every shuffle job on the host-staged path.
bool exch_enabled() {
  const char* v = std::getenv("LOCUST_EXCHANGE");
  return !(v && v[0] == '0');
}

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
// so failure agreement costs no extra collective.  Msg1 also carries the map statistics,
// so the gather strategy needs no further control traffic.
struct alignas(8) Msg1 {  // after map + sampling
  i32 status;
  u32 record_flags;  // ShardEngine::record_flags() of the sender
  u64 n_local, lines, tokens, overflow, truncated, max_key_len;
};
struct alignas(8) Msg3 {  // after the reduce of the received key range (shuffle strategy)
  i32 status;
  u32 pad;
  u64 total, uniq;
};

// LOCUST_EXCH_ASYNC=0: the device exchange waits for a synchronised map (two host syncs).
static bool exch_async_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("LOCUST_EXCH_ASYNC");
    return !e || e[0] != '0';
  }();
  return on;
}

// LOCUST_DIST_LOCAL=0: one-rank kAuto jobs run the exchange with themselves too.
static bool dist_local_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("LOCUST_DIST_LOCAL");
    return !e || e[0] != '0';
  }();
  return on;
}

namespace {
DistResult run_distributed_job(const DistConfig& cfg, Communicator& comm, ShardEngine& eng,
                               const TextInput& shard);
}  // namespace

DistResult run_distributed(const DistConfig& cfg, Communicator& comm, ShardEngine& eng,
                           const TextInput& shard) {
  DistResult res = run_distributed_job(cfg, comm, eng, shard);
  res.hbm_device_bytes = eng.device_bytes();  // the HBM plan's outcome, per rank
  res.hbm_free_bytes = eng.hbm_free();
  res.hbm_total_bytes = eng.hbm_total();
  res.hbm_used_bytes = eng.hbm_used_now();
  return res;
}

namespace {
DistResult run_distributed_job(const DistConfig& cfg, Communicator& comm, ShardEngine& eng,
                               const TextInput& shard) {
  const int P = comm.size();
  const int me = comm.rank();
  log_rank() = me;
  DistResult res;
  res.sent_to.assign((size_t)P, 0);
  res.recv_from.assign((size_t)P, 0);
  std::string local_msg;
  // Runs a local step, returning its status (0 ok) instead of throwing.
  auto local = [&](const char* stage, const std::function<void()>& fn) -> i32 {
    set_current_stage(stage);
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
  // Data-plane exchange through the engine's buffers; a device engine over a host-only
  // communicator (TCP) stages through host memory -- that is how several GPU ranks can
  // share one device in tests (RCCL refuses that).
  auto exchange = [&](u64 n_send, const u64* sb, const u64* so, void* recv, u64 n_recv,
                      const u64* rb, const u64* ro, bool recv_ok) {
    if (eng.device_buffers() && !comm.device_buffers()) {
      std::vector<KeyCount> hs(std::max<u64>(n_send, 1)), hr(std::max<u64>(n_recv, 1));
      copy_device(hs.data(), eng.send_records(), n_send * sizeof(KeyCount), /*to_host=*/true,
                  eng.stream());
      comm.alltoallv(hs.data(), sb, so, hr.data(), rb, ro, nullptr);
      if (recv_ok && n_recv)
        copy_device(recv, hr.data(), n_recv * sizeof(KeyCount), /*to_host=*/false, eng.stream());
    } else {
      comm.alltoallv(eng.send_records(), sb, so, recv, rb, ro, eng.stream());
    }
    for (int p = 0; p < P; ++p) {
      if (p != me) {
        res.sent_bytes += sb[p];
        res.recv_bytes += rb[p];
        res.sent_to[(size_t)p] += sb[p];
        res.recv_from[(size_t)p] += rb[p];
      }
    }
  };

  const u64 t0 = now_ns();
  const u32 S = std::max<u32>(cfg.samples_per_rank, 1);
  // ---------------- map + sample, one allgather ----------------
  u64 n_local = 0;
  std::vector<PackedKey> mine_samples;
  WordCountResult local_stats;
  // The strategy is only known after the first allgather; the engine prepares for the
  // predicted one (kAuto: whatever the previous job took) and patches up a mispredict.
  const DistStrategy plan = !cfg.gather ? DistStrategy::kShuffle
                            : cfg.strategy == DistStrategy::kAuto ? eng.last_strategy
                                                                  : cfg.strategy;
  TraceRange tr_job("locust:dist_job");
  WordCountResult& r = res.result;

  // ---------------- one rank: no exchange (kLocal) ----------------
  LOCUST_CHECK_ARG(cfg.strategy != DistStrategy::kLocal || P == 1,
                   "strategy 'local' is the one-rank job; use auto, gather or shuffle");
  if (P == 1 && (cfg.strategy == DistStrategy::kAuto || cfg.strategy == DistStrategy::kLocal) &&
      (dist_local_enabled() || cfg.strategy == DistStrategy::kLocal)) {
    bool whole = false;
    if (local("map", [&] { whole = eng.run_whole(shard, &r); }))
      throw Error(std::string("distributed job failed on rank 0: ") + local_msg);
    if (whole) {
      res.strategy = DistStrategy::kLocal;
      res.local_records = r.num_unique;
      res.range_tokens = r.num_tokens;
      res.range_unique = r.num_unique;
      res.total_ms = res.map_ms = (now_ns() - t0) * 1e-6;
      return res;
    }
  }

  // ---------------- gather strategy in ONE all-gather (predicted gather) ----------------
  // map (+ slot header on the device) -> all-gather of fixed-size slots -> root merge, all
  // enqueued on the engine's stream behind each other: one host synchronisation per job.
  // Every rank sees every header, so the decisions below (failure, fallback, next slot
  // size) are identical everywhere without another collective.
  bool mapped = false;
  i32 st_slot = 0;
  const bool slot_path = plan == DistStrategy::kGather && cfg.gather && cfg.job.combine &&
                         cfg.strategy != DistStrategy::kShuffle && P <= kMaxSlotRanks &&
                         comm.device_buffers() && eng.device_buffers();
  if (slot_path) {
    TraceRange tr("locust:slot_gather");
    const u32 slot_recs = eng.slot_records ? eng.slot_records : kSlotRecordsMin;
    const u64 slot_bytes = ((u64)kSlotHeaderRecords + slot_recs) * sizeof(KeyCount);
    // One graph for the whole job when the collective can be captured (RCCL); every rank
    // enters the all-gather exactly once either way.
    bool fused = false;
    if (comm.graph_capturable() && slot_graph_enabled(P)) {
      // `entered`: the all-gather was issued directly (uncaptured run) -- this rank is in
      // the collective sequence whatever happens next.  A capture only records it; a
      // refused capture runs the same work uncaptured, so a call made while capturing
      // does not count.
      bool entered = false;
      st_slot = local("map", [&] {
        fused = eng.enqueue_slot_job(shard, slot_recs, (u32)P, me == 0,
                                     [&](const void* send, void* recv, u64 bytes,
                                         bool capturing) {
                                       comm.allgather_device(send, recv, bytes, eng.stream());
                                       if (!capturing) entered = true;
                                     });
        if (fault_injected(me, "slot_after_allgather") && entered)
          throw Error("injected fault (LOCUST_FAULT) after the slot all-gather");
      });
      if (st_slot && entered) {
        // Failed after entering the collective (e.g. the root merge's launch): peers are
        // not waiting for a second all-gather, so drain the stream and fail this rank
        // only -- never enter the step-by-step sequence's all-gather as well.
        try {
          comm.sync_stream(eng.stream());
        } catch (const std::exception&) {
        }
        throw Error(std::string("distributed job failed in stage 'map' on rank ") +
                    std::to_string(me) + ": " + local_msg);
      }
      // a failure before the collective: fall through to the step-by-step sequence
    }
    if (!fused) {
      void* send = nullptr;
      if (!st_slot) st_slot = local("map", [&] { send = eng.enqueue_map_slot(shard, slot_recs); });
      if (st_slot) send = eng.write_slot_failure();  // the all-gather must still be entered
      void* recv = eng.slot_buffer((u32)P, slot_recs);
      comm.allgather_device(send, recv, slot_bytes, eng.stream());
      if (me == 0) eng.enqueue_merge_slots((u32)P, slot_recs);
      eng.enqueue_slot_headers((u32)P, slot_recs);
    }
    comm.sync_stream(eng.stream());
    const SlotHeader* hd = eng.slot_headers();
    for (int p = 0; p < P; ++p)
      if (hd[p].status == kSlotFailed)
        throw Error(std::string("distributed job failed in stage 'map' on rank ") +
                    std::to_string(p) + (p == me ? ": " + local_msg : ""));
    u64 sum = 0, max_n = 0, min_cap = ~0ull;
    bool fallback = false;
    for (int p = 0; p < P; ++p) {
      sum += hd[p].n;
      max_n = std::max(max_n, hd[p].n);
      min_cap = std::min(min_cap, hd[p].slot_cap);
      fallback |= hd[p].status != kSlotOk || hd[p].n > slot_recs;
    }
    // next job's slot: the largest rank's records + 1/16, within every rank's send buffer
    // (every rank receives P slots: padding costs P x as much as it saves in refits; at
    // whole Hamlet 6,144 records instead of 6,656 -- 8 % less all-gather traffic)
    const u64 want = align_up(max_n + max_n / 16 + 1, 256);
    eng.slot_records = (u32)std::max<u64>(kSlotRecordsMin, std::min<u64>(want, min_cap));
    fallback |= cfg.strategy == DistStrategy::kAuto && sum > cfg.gather_max_records;
    st_slot = local("map", [&] {
      n_local = eng.complete_map_slot(shard);
      eng.map_stats(&local_stats);
    });
    if (!fallback) {
      if (st_slot)
        throw Error(std::string("distributed job failed in stage 'map' on rank ") +
                    std::to_string(me) + ": " + local_msg);
      for (int p = 0; p < P; ++p) {
        r.num_lines += hd[p].lines;
        r.num_tokens += hd[p].tokens;
        r.overflow_lines += hd[p].overflow_lines;
        r.truncated += hd[p].truncated;
        r.max_key_len = std::max<u64>(r.max_key_len, hd[p].max_key_len);
      }
      res.strategy = DistStrategy::kGather;
      eng.last_strategy = DistStrategy::kGather;
      res.local_records = n_local;
      res.host_syncs = 1;  // the slot job's one synchronisation
      const u64 t1 = now_ns();
      if (me == 0) {
        u64 total = 0, uniq = 0;
        if (local("reduce", [&] { eng.finish_merge_slots(&total, &uniq); }))
          throw Error(std::string("distributed job failed on rank 0: ") + local_msg);
        eng.finalize(&r.entries);
        res.range_tokens = total;
        res.range_unique = uniq;
      }
      // the slot all-gather: every peer receives this rank's slot, and this rank every
      // peer's (the root included: it merges them)
      res.sent_bytes = slot_bytes * (u64)(P - 1);
      res.recv_bytes = slot_bytes * (u64)(P - 1);
      for (int p = 0; p < P; ++p)
        if (p != me) res.sent_to[(size_t)p] = res.recv_from[(size_t)p] = slot_bytes;
      r.num_unique = r.entries.size();
      const u64 t2 = now_ns();
      res.map_ms = (t1 - t0) * 1e-6;  // map + all-gather + merge, one synchronisation
      res.reduce_ms = (t2 - t1) * 1e-6;
      res.total_ms = (t2 - t0) * 1e-6;
      r.times.map_ms = res.map_ms;
      r.times.reduce_ms = res.reduce_ms;
      r.times.wall_ms = res.total_ms;
      return res;
    }
    // A rank needs a local redo, a slot overflowed or the records are too many for the
    // root: every rank continues on the standard path with its map already done.
    mapped = true;
  }

  // ---------------- shuffle on the device (locust/exch.hpp) ----------------
  // Every control step of the sample sort -- splitters, bucket offsets, overflow and
  // failure agreement, global val offsets -- runs in kernels between stream-ordered
  // collectives, and every rank writes its key range straight into the shared host output
  // (locust/shm.hpp).  With slot sizes agreed by an earlier job: ONE host sync (with an
  // asynchronous map even the map is not synchronised).  Otherwise (the first job, a job
  // whose data outgrew the slots, a gather job that fell back): TWO -- the all-gathered
  // plans give every rank the exact count matrix, then an all-to-all-v of exact sizes.
  // The host-staged sequence further down is only the path of host-only communicators
  // and CPU engines.
  eng.exch_group = comm.group_id();
  eng.exch_rank = me;
  eng.exch_in_process = comm.in_process();
  i32 st1 = mapped ? st_slot : 0;
  u64 t1 = 0;
  const bool dev_exch = exch_enabled() && cfg.gather && cfg.job.combine && comm.device_buffers() &&
                        eng.device_buffers() && eng.exch_group != 0 && S == kExchSamples &&
                        (u32)P <= kExchMaxRanks && (u32)P * S <= kExchMaxPlanSamples;
  if (dev_exch && eng.exch_numa_nodes.size() != (size_t)P) {
    // once per engine, before its first shared output exists: every rank's GPU node
    const int mine = numa_enabled() ? eng.numa_node() : -1;
    std::vector<int> nodes((size_t)P, -1);
    comm.allgather_host(&mine, nodes.data(), sizeof(int));
    eng.exch_numa_nodes = nodes;
  }
  if (dev_exch) {
    TraceRange tr("locust:device_exchange");
    bool one_sync = !mapped && eng.exch_slot_records && eng.exch_gather_records &&
                    (cfg.strategy == DistStrategy::kShuffle ||
                     (cfg.strategy == DistStrategy::kAuto && eng.exch_last_sum > cfg.gather_max_records));
    bool to_root = false;  // the sized exchange as the gather strategy
    bool async_ok = !mapped && exch_async_enabled() && eng.exch_map_async_ok(shard);
    bool map_done = mapped;
    int syncs = 0;
    ShardEngine::ExchCollectives coll;
    coll.allgather = [&](const void* snd, void* rcv, u64 b) {
      comm.allgather_device(snd, rcv, b, eng.stream());
    };
    coll.alltoall = [&](const void* snd, void* rcv, u64 b) {
      comm.alltoall_device(snd, rcv, b, eng.stream());
    };
    coll.alltoallv = [&](const void* snd, const u64* sb, const u64* so, void* rcv, const u64* rb,
                         const u64* ro) {
      comm.alltoallv_device(snd, sb, so, rcv, rb, ro, eng.stream());
    };
    // A failure after this rank entered the collectives: peers cannot be kept in step from
    // here; fail this rank (theirs time out or abort in their waits).
    auto enqueue = [&](const char* stage, const std::function<void()>& fn) {
      if (local(stage, fn)) {
        try {
          comm.sync_stream(eng.stream());
        } catch (const std::exception&) {
        }
        throw Error(std::string("distributed job failed in stage '") + stage + "' on rank " +
                    std::to_string(me) + ": " + local_msg);
      }
    };
    auto sync = [&] {
      comm.sync_stream(eng.stream());
      ++syncs;
    };
    auto header_failures = [&](const ExchMsg1* H) {
      bool redo = false;  // an asynchronous map overflowed a partition somewhere
      for (int p = 0; p < P; ++p) redo |= H[p].status == kExchMapRedo;
      for (int p = 0; p < P && !redo; ++p)
        if (H[p].status)
          throw Error(std::string("distributed job failed in stage '") +
                      (H[p].status == 2 ? "exchange" : "map") + "' on rank " +
                      std::to_string(p) + (p == me ? ": " + local_msg : ""));
      return redo;
    };
    for (;;) {
      const bool exch_async = async_ok && !map_done;
      if (exch_async) {
        st1 = local("map", [&] {
          TraceRange trm("locust:map_async");
          eng.exch_map_enqueue(shard, (u32)P, S);
        });
        mine_samples.assign(S, PackedKey{{~0ull, ~0ull, ~0ull, ~0ull}});  // (written on the device)
      } else if (!map_done) {
        st1 = local("map", [&] {
          TraceRange trm("locust:map");
          n_local = eng.map_local(shard, cfg.job.combine, DistStrategy::kShuffle);
          mine_samples = eng.sample(S);
          eng.map_stats(&local_stats);
        });
        map_done = true;
      } else if (!st1) {
        // mapped already (a gather job that fell back, or a one-sync exchange that was
        // outgrown): the records are sorted for the shuffle, the samples drawn now
        st1 = local("map", [&] { mine_samples = eng.sample(S); });
      }
      if (mine_samples.size() != S) mine_samples.assign(S, PackedKey{{~0ull, ~0ull, ~0ull, ~0ull}});
      if (!t1) t1 = now_ns();
      ExchMsg1 h{};
      h.status = st1;
      h.record_flags = eng.record_flags();
      h.n_local = st1 ? 0 : n_local;
      h.lines = shard.lines();  // a streamed source is drained by the map's enqueue
      h.tokens = local_stats.num_tokens;
      h.overflow_lines = local_stats.overflow_lines;
      h.truncated = local_stats.truncated;
      h.max_key_len = local_stats.max_key_len;
      if (!st1 && fault_injected(me, "exchange")) {
        h.status = 2;  // 1: the map failed, 2: the exchange
        local_msg = "injected fault (LOCUST_FAULT) in stage 'exchange'";
      }
      // test hook: this rank's asynchronous map "overflowed" (every rank redoes the job)
      if (exch_async && !st1 && fault_injected(me, "exch_map_redo")) h.status = kExchMapRedo;
      const TextInput* map_shard = exch_async ? &shard : nullptr;
      if (one_sync) {
        enqueue("shuffle", [&] { eng.enqueue_exchange(h, mine_samples, (u32)P, me, coll, map_shard); });
      } else {
        enqueue("shuffle", [&] {
          eng.enqueue_exchange_plan(h, mine_samples, (u32)P, me, coll, map_shard);
        });
      }
      sync();
      if (header_failures(eng.exch_headers())) {
        LOCUST_LOG_INFO("asynchronous map overflowed a partition: map again, exchange again");
        async_ok = false;
        map_done = false;
        continue;
      }
      if (exch_async) {
        if (local("map", [&] {
              n_local = eng.exch_map_complete(shard);
              eng.map_stats(&local_stats);
            }))
          throw Error(std::string("distributed job failed in stage 'map' on rank ") +
                      std::to_string(me) + ": " + local_msg);
        map_done = true;
      }
      if (!one_sync) {
        // every rank holds every plan: the exact count matrix sizes the all-to-all-v.  Few
        // records in all (auto) or the gather strategy: all of them to the root instead.
        u64 sum = 0;
        for (int p = 0; p < P; ++p) sum += eng.exch_plans()[p].off[P];
        to_root = cfg.strategy == DistStrategy::kGather ||
                  (cfg.strategy == DistStrategy::kAuto && sum <= cfg.gather_max_records);
        enqueue("shuffle", [&] { eng.enqueue_exchange_sized((u32)P, me, coll, to_root); });
        sync();
      }
      const ExchMsg1* H = eng.exch_headers();
      const ExchMsg3* R = eng.exch_reports();
      u32 flags = 0;
      u64 maxb = 0, maxo = 0;
      for (int p = 0; p < P; ++p) {
        if (R[p].status)
          throw Error("distributed job failed in stage 'shuffle' on rank " + std::to_string(p));
        flags |= R[p].flags;
        maxb = std::max<u64>(maxb, R[p].max_bucket);
        maxo = std::max<u64>(maxo, R[p].n_out);
      }
      eng.exch_last_sum = 0;
      for (int p = 0; p < P; ++p) eng.exch_last_sum += H[p].n_local;
      if (flags & kExchTooManySamples) throw Error("device exchange: too many samples for the planner");
      // next job's slot sizes: identical on every rank (computed from all-gathered reports;
      // a gather-shaped job says nothing about the shuffle's buckets)
      const bool first_sizing = eng.exch_slot_records == 0;
      if (!to_root && (!one_sync || (flags & (kExchSendOverflow | kExchRecvTruncated))))
        eng.exch_slot_records = std::max(eng.exch_slot_records, exch_grow(maxb));
      if (!to_root && (!one_sync || (flags & kExchGatherOverflow)))
        eng.exch_gather_records = std::max(eng.exch_gather_records, exch_grow(maxo));
      {
        // test hook: LOCUST_EXCH_SLOT=<records> caps the first slot size, so the next job
        // outgrows it and exercises the agreed fallback + regrowth
        const char* v = std::getenv("LOCUST_EXCH_SLOT");
        if (v && first_sizing && !to_root)
          eng.exch_slot_records = std::min<u32>(eng.exch_slot_records, (u32)std::max(1, std::atoi(v)));
      }
      if (flags && !one_sync)
        throw Error("device exchange: the sized exchange reported overflow flags " +
                    std::to_string(flags));
      if (flags) {
        // outgrown slots: every rank saw the same reports -- the sized exchange, this job
        LOCUST_LOG_INFO("device exchange slots outgrown (flags %u): sized exchange this job", flags);
        one_sync = false;
        continue;
      }
      if (H[0].out_region == kExchNoRegion && one_sync) {
        // the root's results hold every output region: grow the output, write again.
        // LOCUST_FAULT=<rank>:slow_regrow delays one rank here (test hook for the race below).
        if (fault_injected(me, "slow_regrow"))
          std::this_thread::sleep_for(std::chrono::milliseconds(300));
        enqueue("reduce", [&] { eng.enqueue_exchange_emit((u32)P, me); });
        // No collective follows the new generation's shm_open(O_CREAT) in this branch: a fast
        // rank could otherwise finish and unlink the name (exch_job_done) before a slow one
        // opens it, which would then create a separate empty segment.  Every rank has mapped
        // the new generation once this host barrier returns.
        comm.barrier();
        sync();
      }
      if ((int)log_level() >= (int)LogLevel::kDebug)
        for (int p = 0; p < P; ++p)
          LOCUST_LOG_DEBUG("exchange header %d: n_local %llu tokens %llu lines %llu", p,
                           (unsigned long long)H[p].n_local, (unsigned long long)H[p].tokens,
                           (unsigned long long)H[p].lines);
      for (int p = 0; p < P; ++p) {
        r.num_lines += H[p].lines;
        r.num_tokens += H[p].tokens;
        r.overflow_lines += H[p].overflow_lines;
        r.truncated += H[p].truncated;
        r.max_key_len = std::max<u64>(r.max_key_len, H[p].max_key_len);
      }
      res.local_records = n_local;
      if (one_sync) {
        const u64 sb = exch_slot_bytes(eng.exch_slot_records);
        for (int p = 0; p < P; ++p)
          if (p != me) res.sent_to[(size_t)p] = res.recv_from[(size_t)p] = sb;
      } else {
        const ExchCtl* pl = eng.exch_plans();
        for (int p = 0; p < P; ++p)
          if (p != me) {
            res.sent_to[(size_t)p] = exch_slot_bytes((u32)(pl[me].off[p + 1] - pl[me].off[p]));
            res.recv_from[(size_t)p] = exch_slot_bytes((u32)(pl[p].off[me + 1] - pl[p].off[me]));
          }
      }
      for (int p = 0; p < P; ++p) {
        res.sent_bytes += res.sent_to[(size_t)p];
        res.recv_bytes += res.recv_from[(size_t)p];
      }
      res.output_bytes = R[me].out_words * 8;  // compact records the emit wrote
      res.range_tokens = R[me].total;
      res.range_unique = R[me].n_out;
      res.strategy = to_root ? DistStrategy::kGather : DistStrategy::kShuffle;
      res.device_exchange = true;
      res.host_syncs = syncs;
      // auto: a job small enough for the gather strategy predicts it for the next one
      eng.last_strategy = cfg.strategy == DistStrategy::kAuto &&
                                  eng.exch_last_sum <= cfg.gather_max_records
                              ? DistStrategy::kGather
                              : DistStrategy::kShuffle;
      const u64 t2 = now_ns();
      if (me == 0) {
        u64 total = 0, uniq = 0;
        if (local("reduce", [&] { eng.exch_finish_root((u32)P, &total, &uniq); }))
          throw Error(std::string("distributed job failed on rank 0: ") + local_msg);
        eng.finalize(&r.entries);
      }
      eng.exch_job_done();
      r.num_unique = me == 0 ? r.entries.size() : R[me].n_out;
      const u64 t3 = now_ns();
      res.map_ms = (t1 - t0) * 1e-6;
      LOCUST_LOG_DEBUG("map done: %s", process_rss_breakdown().c_str());
      res.shuffle_ms = (t2 - t1) * 1e-6;  // the whole device exchange
      res.reduce_ms = (t3 - t2) * 1e-6;
      res.total_ms = (t3 - t0) * 1e-6;
      r.times.map_ms = res.map_ms;
      r.times.process_ms = res.shuffle_ms;
      r.times.reduce_ms = res.reduce_ms;
      r.times.wall_ms = res.total_ms;
      return res;
    }
  }
  // ---------------- host-staged shuffle (host-only communicators, CPU engines) ----------------
  if (!mapped) {
    st1 = local("map", [&] {
      TraceRange trm("locust:map");
      n_local = eng.map_local(shard, cfg.job.combine, plan);
      if (plan != DistStrategy::kGather) mine_samples = eng.sample(S);
      eng.map_stats(&local_stats);
    });
  }
  if (mine_samples.size() != S) mine_samples.assign(S, PackedKey{{~0ull, ~0ull, ~0ull, ~0ull}});
  res.local_records = n_local;
  t1 = now_ns();
  const u64 m1 = sizeof(Msg1) + (u64)S * sizeof(PackedKey);
  std::vector<char> out1(m1), all1(m1 * (u64)P);
  {
    Msg1 h{st1, eng.record_flags(), n_local, shard.lines(), local_stats.num_tokens, local_stats.overflow_lines,
           local_stats.truncated, local_stats.max_key_len};
    std::memcpy(out1.data(), &h, sizeof(h));
    std::memcpy(out1.data() + sizeof(h), mine_samples.data(), (u64)S * sizeof(PackedKey));
  }
  {
    TraceRange tr("locust:allgather_counts_samples");
    comm.allgather_host(out1.data(), all1.data(), m1);
  }
  check("map", reinterpret_cast<const i32*>(all1.data()), m1);
  std::vector<PackedKey> samples((size_t)P * S);
  std::vector<u64> counts((size_t)P);
  u64 sum_records = 0;
  u32 run_flags = ~0u;
  for (int p = 0; p < P; ++p) {
    const char* base = all1.data() + (u64)p * m1;
    Msg1 h;
    std::memcpy(&h, base, sizeof(h));
    counts[(size_t)p] = h.n_local;
    run_flags &= h.record_flags;
    sum_records += h.n_local;
    std::memcpy(&samples[(size_t)p * S], base + sizeof(h), (u64)S * sizeof(PackedKey));
    r.num_lines += h.lines;
    r.num_tokens += h.tokens;
    r.overflow_lines += h.overflow;
    r.truncated += h.truncated;
    r.max_key_len = std::max(r.max_key_len, h.max_key_len);
  }
  eng.exch_last_sum = sum_records;
  const bool use_gather =
      cfg.gather && (cfg.strategy == DistStrategy::kGather ||
                     (cfg.strategy == DistStrategy::kAuto && sum_records <= cfg.gather_max_records));
  res.strategy = use_gather ? DistStrategy::kGather : DistStrategy::kShuffle;
  eng.last_strategy = res.strategy;
  std::vector<u64> sb((size_t)P, 0), so((size_t)P, 0), rb((size_t)P, 0), ro((size_t)P, 0);

  if (use_gather) {
    // ---------------- gather-to-root: one grouped send/recv ----------------
    const u64 rec = sizeof(KeyCount);
    sb[0] = n_local * rec;
    void* recv = nullptr;
    i32 st = 0;
    if (me == 0) {
      // The root's own records stay put (reduce_gathered merges them in place); the
      // others land back to back at the start of the receive buffer.
      sb[0] = 0;
      u64 off = 0;
      for (int p = 1; p < P; ++p) {
        rb[(size_t)p] = counts[(size_t)p] * rec;
        ro[(size_t)p] = off;
        off += rb[(size_t)p];
      }
      st = local("shuffle", [&] { recv = eng.recv_records(sum_records); });
    }
    {
      TraceRange tr("locust:gather_to_root");
      exchange(n_local, sb.data(), so.data(), recv, me == 0 ? sum_records : 0, rb.data(),
               ro.data(), st == 0);
    }
    const u64 t2 = now_ns();
    if (me == 0) {
      // The root merges: a failure here is the job's failure (only the root holds output).
      u64 total = 0, uniq = 0;
      if (!st)
        st = local("reduce", [&] {
          const std::vector<u64> runs(counts.begin() + 1, counts.end());
          eng.reduce_gathered(runs, r.num_tokens, run_flags, &total, &uniq);
        });
      if (st)
        throw Error(std::string("distributed job failed on rank 0: ") + local_msg);
      eng.finalize(&r.entries);
      res.range_tokens = total;
      res.range_unique = uniq;
    }
    r.num_unique = r.entries.size();
    const u64 t3 = now_ns();
    res.map_ms = (t1 - t0) * 1e-6;
    LOCUST_LOG_DEBUG("map done: %s", process_rss_breakdown().c_str());
    res.shuffle_ms = (t2 - t1) * 1e-6;
    res.reduce_ms = (t3 - t2) * 1e-6;
    res.gather_ms = 0;
    res.total_ms = (t3 - t0) * 1e-6;
    r.times.map_ms = res.map_ms;
    r.times.process_ms = res.shuffle_ms;
    r.times.reduce_ms = res.reduce_ms;
    r.times.wall_ms = res.total_ms;
    return res;
  }

  if (plan == DistStrategy::kGather) {
    // Mispredicted: the map prepared for the gather (no samples).  Sort locally and run
    // the sampling round now.
    std::vector<char> out2(sizeof(i32) + (u64)S * sizeof(PackedKey)), all2(out2.size() * (u64)P);
    const i32 st = local("map", [&] { mine_samples = eng.sample(S); });
    if (mine_samples.size() != S) mine_samples.assign(S, PackedKey{{~0ull, ~0ull, ~0ull, ~0ull}});
    std::memcpy(out2.data(), &st, sizeof(i32));
    std::memcpy(out2.data() + sizeof(i32), mine_samples.data(), (u64)S * sizeof(PackedKey));
    comm.allgather_host(out2.data(), all2.data(), out2.size());
    check("map", reinterpret_cast<const i32*>(all2.data()), out2.size());
    for (int p = 0; p < P; ++p)
      std::memcpy(&samples[(size_t)p * S], all2.data() + (u64)p * out2.size() + sizeof(i32),
                  (u64)S * sizeof(PackedKey));
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
  u64 n_recv = 0;
  for (int p = 0; p < P; ++p) {
    sb[(size_t)p] = msg2[(size_t)p + 1] * sizeof(KeyCount);
    so[(size_t)p] = offs[(size_t)p] * sizeof(KeyCount);
    const u64 c = matrix[(size_t)p * (P + 1) + 1 + me];
    rb[(size_t)p] = c * sizeof(KeyCount);
    ro[(size_t)p] = n_recv * sizeof(KeyCount);
    n_recv += c;
  }

  // ---------------- shuffle ----------------
  // The receive buffer is sized locally; an allocation failure surfaces in the reduce
  // status below (the all-to-all itself must be entered by every rank).
  void* recv = nullptr;
  i32 st3 = local("shuffle", [&] { recv = eng.recv_records(n_recv); });
  {
    TraceRange tr("locust:alltoallv_shuffle");
    exchange(n_local, sb.data(), so.data(), recv, n_recv, rb.data(), ro.data(), st3 == 0);
  }
  const u64 t2 = now_ns();

  // ---------------- reduce, one allgather of {status, totals} ----------------
  u64 total = 0, uniq = 0;
  if (!st3)
    st3 = local("reduce", [&] {
      std::vector<u64> runs((size_t)P);
      for (int p = 0; p < P; ++p) runs[(size_t)p] = rb[(size_t)p] / sizeof(KeyCount);
      eng.reduce_received_runs(runs, r.num_tokens, run_flags, &total, &uniq);
    });
  Msg3 m3{st3, 0, total, uniq};
  std::vector<Msg3> all3((size_t)P);
  comm.allgather_host(&m3, all3.data(), sizeof(Msg3));
  check("reduce", &all3[0].status, sizeof(Msg3));
  {
    // sizes for the device exchange of the next shuffle job (every rank holds the whole
    // count matrix and every range size, so all compute the same)
    const bool first_sizing = eng.exch_slot_records == 0;
    u64 maxb = 0, maxo = 0;
    for (int p = 0; p < P; ++p) {
      maxo = std::max<u64>(maxo, all3[(size_t)p].uniq);
      for (int q = 0; q < P; ++q) maxb = std::max<u64>(maxb, matrix[(size_t)p * (P + 1) + 1 + q]);
    }
    eng.exch_slot_records = std::max(eng.exch_slot_records, exch_grow(maxb));
    eng.exch_gather_records = std::max(eng.exch_gather_records, exch_grow(maxo));
    // test hook: LOCUST_EXCH_SLOT=<records> caps the first slot size, so the next job
    // outgrows it and exercises the agreed fallback + regrowth
    const char* v = std::getenv("LOCUST_EXCH_SLOT");
    if (v && first_sizing)
      eng.exch_slot_records = std::min<u32>(eng.exch_slot_records, (u32)std::max(1, std::atoi(v)));
  }
  u64 offset = 0;
  for (int p = 0; p < me; ++p) offset += all3[(size_t)p].total;
  EntryList entries;
  eng.finalize(&entries);
  res.range_tokens = total;
  res.range_unique = uniq;
  const u64 t3 = now_ns();

  // ---------------- gather ----------------
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
    for (int p = 1; p < P; ++p) {  // the ranges' trip to rank 0
      if (me == 0) res.recv_from[(size_t)p] += sizes[(size_t)p];
      if (me == p) res.sent_to[0] += sizes[(size_t)p];
    }
  } else {
    r.entries = std::move(entries);
    r.val_base = offset;  // this rank's range starts after the lower ranks' tokens
  }
  r.num_unique = me == 0 && cfg.gather ? r.entries.size() : uniq;
  const u64 t4 = now_ns();
  res.map_ms = (t1 - t0) * 1e-6;
  LOCUST_LOG_DEBUG("map done: %s", process_rss_breakdown().c_str());
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
}  // namespace

}  // namespace locust
