// CPU reference pipeline: the golden oracle and the `--backend cpu` path.
//
// Semantics of the reference CPU build (/root/reference/MapReduce/src/
// main.cu:242-355, 489-527): strtok_r map with the 20-emit cap, std::sort, linear-scan
// reduce.  Unlike the reference it does not allocate a heap object per emitted token
// (main.cu:304) or sort 116,000 mostly-NULL pointers (main.cu:498); tokens are packed
// keys in one vector.
#include <algorithm>
#include <cstring>

#include "locust/engine.hpp"

namespace locust {

void validate_result(const WordCountResult& r);

CpuWordCount::CpuWordCount(const JobConfig& cfg) : cfg_(cfg) {}

namespace {

void map_lines(const TextInput& in, const JobConfig& cfg, std::vector<PackedKey>* toks,
               WordCountResult* r) {
  const char* p = in.data;
  const char* end = in.data + in.bytes;
  while (p < end) {
    const char* nl = static_cast<const char*>(memchr(p, '\n', (size_t)(end - p)));
    const char* le = nl ? nl : end;
    r->overflow_lines += (u64)tokenize_line(p, (u64)(le - p), cfg, toks, &r->truncated);
    p = nl ? nl + 1 : end;
  }
}

void reduce_sorted(const std::vector<PackedKey>& toks, WordCountResult* r) {
  std::vector<WordCountEntry> e;
  entries_from_sorted_tokens(toks.data(), toks.size(), &e);
  r->entries = std::move(e);
  r->num_unique = r->entries.size();
}

u64 max_len(const std::vector<PackedKey>& toks) {
  u64 m = 0;
  char buf[kKeyBytes + 1];
  for (const auto& k : toks) m = std::max<u64>(m, (u64)unpack_key(k.w, buf));
  return m;
}

}  // namespace

WordCountResult CpuWordCount::run(const TextInput& in) {
  WordCountResult r;
  r.num_lines = in.num_lines;
  std::vector<PackedKey> toks;
  const u64 t0 = now_ns();
  map_lines(in, cfg_, &toks, &r);
  const u64 t1 = now_ns();
  std::sort(toks.begin(), toks.end(), key_less);
  const u64 t2 = now_ns();
  r.num_tokens = toks.size();
  reduce_sorted(toks, &r);
  const u64 t3 = now_ns();
  r.max_key_len = max_len(toks);
  r.times.map_ms = (t1 - t0) * 1e-6;
  r.times.process_ms = (t2 - t1) * 1e-6;
  r.times.reduce_ms = (t3 - t2) * 1e-6;
  r.times.wall_ms = (t3 - t0) * 1e-6;
  if (cfg_.check) validate_result(r);
  return r;
}

std::vector<PackedKey> CpuWordCount::run_map_stage(const TextInput& in, WordCountResult* stats) {
  WordCountResult r;
  r.num_lines = in.num_lines;
  std::vector<PackedKey> toks;
  map_lines(in, cfg_, &toks, &r);
  std::sort(toks.begin(), toks.end(), key_less);
  r.num_tokens = toks.size();
  r.max_key_len = max_len(toks);
  if (stats) *stats = r;
  return toks;
}

WordCountResult CpuWordCount::run_reduce_stage(const PackedKey* keys, u64 n) {
  WordCountResult r;
  std::vector<PackedKey> toks(keys, keys + n);
  const u64 t1 = now_ns();
  std::sort(toks.begin(), toks.end(), key_less);
  const u64 t2 = now_ns();
  r.num_tokens = n;
  reduce_sorted(toks, &r);
  const u64 t3 = now_ns();
  r.max_key_len = max_len(toks);
  r.times.process_ms = (t2 - t1) * 1e-6;
  r.times.reduce_ms = (t3 - t2) * 1e-6;
  r.times.wall_ms = (t3 - t1) * 1e-6;
  if (cfg_.check) validate_result(r);
  return r;
}

}  // namespace locust

// =====================================================================================
// CPU shard engine: the distributed driver's per-rank engine on host memory.  Used for
// multi-process CPU tests (TCP communicator) and as the oracle of the GPU shuffle.
// =====================================================================================
#include "locust/dist.hpp"

namespace locust {
namespace {

class CpuShardEngine final : public ShardEngine {
 public:
  explicit CpuShardEngine(const JobConfig& cfg) : cfg_(cfg) {}
  bool device_buffers() const override { return false; }
  void* stream() override { return nullptr; }

  u64 map_local(const TextInput& shard, bool combine, DistStrategy) override {
    LOCUST_CHECK_ARG(!shard.source, "the CPU engine maps in-memory shards only");
    CpuWordCount eng(cfg_);
    stats_ = WordCountResult();
    std::vector<PackedKey> toks = eng.run_map_stage(shard, &stats_);
    local_.clear();
    if (combine) {
      std::vector<WordCountEntry> e;
      entries_from_sorted_tokens(toks.data(), toks.size(), &e);
      for (const auto& x : e) {
        KeyCount r;
        for (int w = 0; w < kKeyWords; ++w) r.w[w] = x.key.w[w];
        r.count = x.count;
        local_.push_back(r);
      }
    } else {
      for (const auto& k : toks) {
        KeyCount r;
        for (int w = 0; w < kKeyWords; ++w) r.w[w] = k.w[w];
        r.count = 1;
        local_.push_back(r);
      }
    }
    return local_.size();
  }

  std::vector<PackedKey> sample(u32 s) override {
    std::vector<PackedKey> out(s);
    const u64 n = local_.size();
    for (u32 k = 0; k < s; ++k) {
      if (!n) {
        for (int w = 0; w < kKeyWords; ++w) out[k].w[w] = ~0ull;
      } else {
        const u64 i = ((2ull * k + 1) * n) / (2ull * s);
        for (int w = 0; w < kKeyWords; ++w) out[k].w[w] = local_[i].w[w];
      }
    }
    return out;
  }

  std::vector<u64> bucket_offsets(const std::vector<PackedKey>& sp) override {
    std::vector<u64> off(sp.size() + 2);
    off[0] = 0;
    for (size_t p = 0; p < sp.size(); ++p) {
      auto it = std::lower_bound(local_.begin(), local_.end(), sp[p],
                                 [](const KeyCount& a, const PackedKey& b) {
                                   return key_compare(a.w, b.w) < 0;
                                 });
      off[p + 1] = (u64)(it - local_.begin());
    }
    off[sp.size() + 1] = local_.size();
    return off;
  }

  const void* send_records() override { return local_.data(); }
  void* recv_records(u64 n) override {
    recv_.resize(std::max<u64>(n, 1));
    return recv_.data();
  }

  void reduce_received(u64 n, u64* total_count, u64* num_unique) override {
    std::vector<KeyCount> recs(recv_.begin(), recv_.begin() + (long)n);
    std::stable_sort(recs.begin(), recs.end(), [](const KeyCount& a, const KeyCount& b) {
      return key_compare(a.w, b.w) < 0;
    });
    out_.clear();
    u64 pos = 0;
    for (size_t i = 0; i < recs.size();) {
      size_t j = i;
      u64 c = 0;
      while (j < recs.size() && key_compare(recs[j].w, recs[i].w) == 0) c += recs[j++].count;
      WordCountEntry e;
      for (int w = 0; w < kKeyWords; ++w) e.key.w[w] = recs[i].w[w];
      e.count = c;
      out_.push_back(e);
      pos += c;
      i = j;
    }
    *total_count = pos;
    *num_unique = out_.size();
  }

  void reduce_gathered(const std::vector<u64>& run_lens, u64 /*total_tokens*/, u32 /*run_flags*/,
                       u64* total_count, u64* num_unique) override {
    u64 n_other = 0;
    for (u64 l : run_lens) n_other += l;
    recv_.resize(std::max<u64>(n_other + local_.size(), 1));
    std::copy(local_.begin(), local_.end(), recv_.begin() + (long)n_other);
    reduce_received(n_other + local_.size(), total_count, num_unique);
  }

  void finalize(EntryList* out) override { out->assign(out_.data(), out_.data() + out_.size()); }

  void map_stats(WordCountResult* r) override { *r = stats_; }

 private:
  JobConfig cfg_;
  std::vector<KeyCount> local_, recv_;
  std::vector<WordCountEntry> out_;
  WordCountResult stats_;
};

}  // namespace

std::unique_ptr<ShardEngine> make_cpu_shard_engine(const JobConfig& cfg) {
  return std::unique_ptr<ShardEngine>(new CpuShardEngine(cfg));
}

}  // namespace locust
