#include "locust/io.hpp"
#include "locust/partmap.hpp"

#include <fcntl.h>
#include <immintrin.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

namespace locust {

u64 TextInput::lines() const { return source ? source->lines() : num_lines; }

u64 EntryList::wire_bytes() const {
  if (!compact_) return (u64)size() * sizeof(WordCountEntry);
  u64 words = 0;
  for (const EntrySegment& s : segs_) {
    const u64* p = s.words;
    for (u64 i = 0; i < s.n; ++i) p += compact_record_words(p[0]);
    words += (u64)(p - s.words);
  }
  return words * 8;
}

namespace {

// Byte-lane counters: each of 255 rounds adds at most 1 per lane, then one SAD folds them.
__attribute__((target("avx2"))) u64 count_newlines_avx2(const char* p, u64 n) {
  const __m256i nl = _mm256_set1_epi8('\n');
  const __m256i zero = _mm256_setzero_si256();
  u64 total = 0, i = 0;
  while (n - i >= 128) {
    const u64 rounds = std::min<u64>((n - i) / 128, 255);
    __m256i a0 = zero, a1 = zero, a2 = zero, a3 = zero;
    for (u64 r = 0; r < rounds; ++r, i += 128) {
      const __m256i* q = reinterpret_cast<const __m256i*>(p + i);
      a0 = _mm256_sub_epi8(a0, _mm256_cmpeq_epi8(_mm256_loadu_si256(q + 0), nl));
      a1 = _mm256_sub_epi8(a1, _mm256_cmpeq_epi8(_mm256_loadu_si256(q + 1), nl));
      a2 = _mm256_sub_epi8(a2, _mm256_cmpeq_epi8(_mm256_loadu_si256(q + 2), nl));
      a3 = _mm256_sub_epi8(a3, _mm256_cmpeq_epi8(_mm256_loadu_si256(q + 3), nl));
    }
    const __m256i s = _mm256_add_epi64(
        _mm256_add_epi64(_mm256_sad_epu8(a0, zero), _mm256_sad_epu8(a1, zero)),
        _mm256_add_epi64(_mm256_sad_epu8(a2, zero), _mm256_sad_epu8(a3, zero)));
    total += (u64)_mm256_extract_epi64(s, 0) + (u64)_mm256_extract_epi64(s, 1) +
             (u64)_mm256_extract_epi64(s, 2) + (u64)_mm256_extract_epi64(s, 3);
  }
  for (; i < n; ++i) total += p[i] == '\n';
  return total;
}

u64 count_newlines_sse2(const char* p, u64 n) {
  const __m128i nl = _mm_set1_epi8('\n');
  const __m128i zero = _mm_setzero_si128();
  u64 total = 0, i = 0;
  while (n - i >= 64) {
    const u64 rounds = std::min<u64>((n - i) / 64, 255);
    __m128i a0 = zero, a1 = zero, a2 = zero, a3 = zero;
    for (u64 r = 0; r < rounds; ++r, i += 64) {
      const __m128i* q = reinterpret_cast<const __m128i*>(p + i);
      a0 = _mm_sub_epi8(a0, _mm_cmpeq_epi8(_mm_loadu_si128(q + 0), nl));
      a1 = _mm_sub_epi8(a1, _mm_cmpeq_epi8(_mm_loadu_si128(q + 1), nl));
      a2 = _mm_sub_epi8(a2, _mm_cmpeq_epi8(_mm_loadu_si128(q + 2), nl));
      a3 = _mm_sub_epi8(a3, _mm_cmpeq_epi8(_mm_loadu_si128(q + 3), nl));
    }
    const __m128i s = _mm_add_epi64(_mm_add_epi64(_mm_sad_epu8(a0, zero), _mm_sad_epu8(a1, zero)),
                                    _mm_add_epi64(_mm_sad_epu8(a2, zero), _mm_sad_epu8(a3, zero)));
    total += (u64)_mm_cvtsi128_si64(s) + (u64)_mm_cvtsi128_si64(_mm_unpackhi_epi64(s, s));
  }
  for (; i < n; ++i) total += p[i] == '\n';
  return total;
}

}  // namespace

u64 count_newlines(const char* data, u64 bytes) {
  static const bool avx2 = __builtin_cpu_supports("avx2");
  return avx2 ? count_newlines_avx2(data, bytes) : count_newlines_sse2(data, bytes);
}

u64 count_lines(const char* data, u64 bytes) {
  // every '\n' ends a line, and a last line without one counts too
  return count_newlines(data, bytes) + (bytes && data[bytes - 1] != '\n' ? 1 : 0);
}

LoadedText text_from_buffer(const char* data, u64 bytes, i64 line_start, i64 line_end,
                            bool ref_compat) {
  LoadedText lt;
  lt.window = line_start >= 0;
  // Byte offset of every line start (one pass, memchr speed).
  std::vector<u64> starts;
  {
    const char* p = data;
    const char* end = data + bytes;
    while (p < end) {
      starts.push_back((u64)(p - data));
      const char* nl = static_cast<const char*>(memchr(p, '\n', (size_t)(end - p)));
      p = nl ? nl + 1 : end;
    }
  }
  const u64 total = starts.size();
  lt.file_lines = total;
  u64 first = 0, last = total;  // [first, last)
  if (line_start >= 0) {
    first = std::min<u64>((u64)line_start, total);
    last = line_end < 0 ? total : std::min<u64>(std::max<i64>(line_end, line_start), total);
    // Reference quirk (main.cu:62-63): a window that reaches EOF reports
    // line_num - line_start lines, i.e. loses the last line.
    if (ref_compat && line_end >= 0 && (u64)line_end >= total && last > first) --last;
  } else if (ref_compat && total > 0) {
    last = total - 1;  // B1: whole-file mode drops the last line
  }
  const u64 b0 = first < total ? starts[first] : bytes;
  const u64 b1 = last < total ? starts[last] : bytes;
  lt.storage.assign(data + b0, data + b1);
  lt.storage.reserve(lt.storage.size() + 64);
  lt.input.data = lt.storage.data();
  lt.input.bytes = lt.storage.size();
  lt.input.num_lines = last > first ? last - first : 0;
  lt.input.first_line = first;
  return lt;
}

namespace {

u32 io_threads(u32 threads, u64 bytes) {
  if (threads) return threads;
  const u32 hw = std::max(1u, std::thread::hardware_concurrency());
  // one thread per 8 MiB, at most 8 (the GPU box's CPU share is 16)
  return (u32)std::max<u64>(1, std::min<u64>({(u64)std::min(hw, 8u), bytes >> 23}));
}

struct Fd {
  int fd = -1;
  explicit Fd(const std::string& path) : fd(::open(path.c_str(), O_RDONLY | O_CLOEXEC)) {
    if (fd < 0) throw Error("cannot open input file: " + path + ": " + std::strerror(errno));
  }
  ~Fd() {
    if (fd >= 0) ::close(fd);
  }
  u64 size() const {
    struct stat st;
    if (fstat(fd, &st) != 0) throw Error("cannot stat input file");
    return (u64)st.st_size;
  }
};

// One slice [a, b) of a read into dst: preads until done; optionally counts its '\n'.
bool pread_slice(int fd, char* dst, u64 off, u64 a, u64 b, bool count_nl, u64* nl) {
  u64 pos = a;
  while (pos < b) {
    const ssize_t k = ::pread(fd, dst + pos, (size_t)std::min<u64>(b - pos, 1ull << 30),
                              (off_t)(off + pos));
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) return false;
    pos += (u64)k;
  }
  *nl = count_nl ? count_newlines(dst + a, b - a) : 0;
  return true;
}

// [off, off + n) of the file into dst, `threads` preads at once (page-cache reads run at
// memcpy speed per core); optionally counts the '\n' bytes read.
u64 pread_parallel(int fd, char* dst, u64 off, u64 n, u32 threads, const std::string& path,
                   bool count_nl) {
  threads = std::max<u32>(1, std::min<u64>(threads, std::max<u64>(1, n >> 20)));
  std::vector<u64> nls(threads, 0);
  std::vector<char> ok(threads, 1);
  auto work = [&](u32 t) {
    ok[t] = pread_slice(fd, dst, off, n * t / threads, n * (t + 1) / threads, count_nl, &nls[t]);
  };
  if (threads == 1) {
    work(0);
  } else {
    std::vector<std::thread> th;
    for (u32 t = 0; t < threads; ++t) th.emplace_back(work, t);
    for (auto& x : th) x.join();
  }
  u64 total = 0;
  for (u32 t = 0; t < threads; ++t) {
    if (!ok[t]) throw Error("short read: " + path);
    total += nls[t];
  }
  return total;
}

// The streamed source's readers: threads - 1 workers that live as long as the source, plus
// the caller, split every read into equal slices.  A piece of a large file is one 16 MiB
// read; starting and joining threads for each cost ~20 % of the read time (measured with
// pread_parallel on a 10 GiB file: 14-15 GB/s).
class ReadPool {
 public:
  explicit ReadPool(u32 threads) : n_(std::max<u32>(threads, 1)) {
    for (u32 t = 1; t < n_; ++t) th_.emplace_back([this, t] { loop(t); });
  }
  ~ReadPool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& x : th_) x.join();
  }
  ReadPool(const ReadPool&) = delete;
  ReadPool& operator=(const ReadPool&) = delete;

  // Reads [off, off + n) into dst; returns its '\n' count (false ok: a short read).
  u64 read(int fd, char* dst, u64 off, u64 n, bool* ok) {
    const u32 parts = (u32)std::max<u64>(1, std::min<u64>(n_, n >> 20));
    {
      std::lock_guard<std::mutex> lk(mu_);
      job_ = {fd, dst, off, n, parts};
      nls_.assign(n_, 0);
      ok_.assign(n_, 1);
      pending_ = n_ - 1;
      ++gen_;
    }
    cv_.notify_all();
    run(0);
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [&] { return pending_ == 0; });
    u64 total = 0;
    *ok = true;
    for (u32 t = 0; t < n_; ++t) {
      total += nls_[t];
      *ok = *ok && ok_[t];
    }
    return total;
  }

 private:
  struct Job {
    int fd = -1;
    char* dst = nullptr;
    u64 off = 0, n = 0;
    u32 parts = 1;
  };
  void run(u32 t) {
    if (t >= job_.parts) return;
    const u64 a = job_.n * t / job_.parts, b = job_.n * (t + 1) / job_.parts;
    u64 nl = 0;
    ok_[t] = pread_slice(job_.fd, job_.dst, job_.off, a, b, true, &nl);
    nls_[t] = nl;
  }
  void loop(u32 t) {
    u64 seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
      }
      run(t);
      std::lock_guard<std::mutex> lk(mu_);
      if (--pending_ == 0) done_cv_.notify_one();
    }
  }
  const u32 n_;
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  Job job_;
  std::vector<u64> nls_;
  std::vector<char> ok_;
  u32 pending_ = 0;
  u64 gen_ = 0;
  bool stop_ = false;
};

// A file as line-aligned chunks (TextSource): each chunk is the carried-over partial line
// of the previous read, then parallel preads, cut after its last '\n'.
// [begin, end) restricts it to one byte range of the file (a rank's shard, file_shards).
class FileTextSource final : public TextSource {
 public:
  FileTextSource(const std::string& path, u32 threads, u64 begin = 0, u64 end = ~0ull)
      : path_(path), fd_(path) {
    const u64 fsize = fd_.size();
    end = std::min<u64>(end, fsize);
    LOCUST_CHECK_ARG(begin <= end, "file range beyond the end of " + path);
    pos_ = begin_ = begin;
    size_ = end;
    threads_ = io_threads(threads, end - begin);
    if (threads_ > 1) pool_.reset(new ReadPool(threads_));
  }
  u64 size() const override { return size_ - begin_; }
  u64 lines() const override { return lines_; }
  u64 next(char* dst, u64 cap) override {
    if (pos_ >= size_ && carry_.empty()) return 0;
    LOCUST_CHECK_ARG(carry_.size() < cap, "a line longer than the stream chunk in " + path_);
    std::memcpy(dst, carry_.data(), carry_.size());
    u64 n = carry_.size();
    u64 nl = count_newlines(carry_.data(), carry_.size());
    carry_.clear();
    const u64 want = std::min<u64>(cap - n, size_ - pos_);
    if (want && pool_) {
      bool ok = true;
      nl += pool_->read(fd_.fd, dst + n, pos_, want, &ok);
      if (!ok) throw Error("short read: " + path_);
    } else if (want) {
      nl += pread_parallel(fd_.fd, dst + n, pos_, want, 1, path_, true);
    }
    pos_ += want;
    n += want;
    if (pos_ < size_) {  // keep whole lines: the tail waits for the next chunk
      const void* p = memrchr(dst, '\n', (size_t)n);
      if (!p) throw Error("a line longer than the stream chunk (" + std::to_string(cap) +
                          " B) in " + path_);
      const u64 cut = (u64)(static_cast<const char*>(p) - dst) + 1;
      carry_.assign(dst + cut, dst + n);
      nl -= count_newlines(dst + cut, n - cut);  // (none: cut is after the last)
      n = cut;
    } else if (n && dst[n - 1] != '\n') {
      ++nl;  // the final line without its newline
    }
    lines_ += nl;
    return n;
  }

 private:
  std::string path_;
  Fd fd_;
  u64 size_ = 0, pos_ = 0, lines_ = 0;  // size_: the range's end offset in the file
  u64 begin_ = 0;
  u32 threads_ = 1;
  std::string carry_;
  std::unique_ptr<ReadPool> pool_;
};

}  // namespace

std::unique_ptr<TextSource> open_file_source(const std::string& path, u32 threads) {
  return std::unique_ptr<TextSource>(new FileTextSource(path, threads));
}

std::unique_ptr<TextSource> open_file_range_source(const std::string& path, u64 begin, u64 end,
                                                   u32 threads) {
  return std::unique_ptr<TextSource>(new FileTextSource(path, threads, begin, end));
}

namespace {

// The first line start at or after byte `off` of an open file of n bytes: off itself when
// off == 0 or byte off-1 is a '\n', else the byte after the next '\n' (n when none).  Reads
// only from off-1 up to that newline.
u64 line_start_at_fd(int fd, u64 n, u64 off, std::vector<char>* buf, const std::string& path) {
  if (off == 0) return 0;
  if (off >= n) return n;
  u64 at = off - 1;
  while (at < n) {
    const u64 len = std::min<u64>(buf->size(), n - at);
    const ssize_t got = ::pread(fd, buf->data(), (size_t)len, (off_t)at);
    if (got < 0 && errno == EINTR) continue;
    if (got <= 0) throw Error("short read: " + path);
    const void* nl = std::memchr(buf->data(), '\n', (size_t)got);
    if (nl) return at + (u64)(static_cast<const char*>(nl) - buf->data()) + 1;
    at += (u64)got;
  }
  return n;
}

}  // namespace

// Cut k of P lies at the start of the first line that begins at or after byte size*k/P
// (the reference's per-node line ranges, main.cu:369-374, as byte ranges).  Only small
// windows around the cuts are read -- never the whole file.
std::vector<FileRange> file_shards(const std::string& path, int parts) {
  LOCUST_CHECK_ARG(parts >= 1, "parts must be >= 1");
  Fd f(path);
  const u64 n = f.size();
  std::vector<u64> cut((size_t)parts + 1, n);
  cut[0] = 0;
  std::vector<char> buf(64 << 10);
  for (int k = 1; k < parts; ++k)
    cut[(size_t)k] = std::max(cut[(size_t)k - 1],
                              line_start_at_fd(f.fd, n, n * (u64)k / (u64)parts, &buf, path));
  std::vector<FileRange> out((size_t)parts);
  for (int k = 0; k < parts; ++k) out[(size_t)k] = {cut[(size_t)k], cut[(size_t)k + 1] - cut[(size_t)k]};
  return out;
}

u64 line_start_at(const std::string& path, u64 off) {
  Fd f(path);
  std::vector<char> buf(64 << 10);
  return line_start_at_fd(f.fd, f.size(), off, &buf, path);
}

LineWindow byte_window(const std::string& path, u64 begin, u64 end) {
  Fd f(path);
  const u64 n = f.size();
  std::vector<char> buf(64 << 10);
  LineWindow w;
  w.begin = line_start_at_fd(f.fd, n, begin, &buf, path);
  w.end = std::max(w.begin, end >= n ? n : line_start_at_fd(f.fd, n, end, &buf, path));
  return w;  // (lines: counted by whoever reads the range)
}

u64 read_file_range_into(const std::string& path, char* dst, u64 off, u64 n, u64* lines,
                         u32 threads) {
  Fd f(path);
  LOCUST_CHECK_ARG(off + n <= f.size(), "file range beyond the end of " + path);
  u64 nl = n ? pread_parallel(f.fd, dst, off, n, io_threads(threads, n), path, true) : 0;
  if (n && dst[n - 1] != '\n') ++nl;
  if (lines) *lines = nl;
  return n;
}

u64 file_size(const std::string& path) { return Fd(path).size(); }

// ---------------- per-file caches: directory and file identity ----------------
namespace {
u64 fnv1a(u64 h, const void* p, size_t n) {
  const unsigned char* b = static_cast<const unsigned char*>(p);
  for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 1099511628211ull;
  return h;
}

// LOCUST_CACHE_DIR, else $XDG_CACHE_HOME/locust, else ~/.cache/locust ("" when none).
std::string cache_dir() {
  if (const char* d = std::getenv("LOCUST_CACHE_DIR"); d && *d) return d;
  if (const char* x = std::getenv("XDG_CACHE_HOME"); x && *x) return std::string(x) + "/locust";
  if (const char* h = std::getenv("HOME"); h && *h) return std::string(h) + "/.cache/locust";
  return "";
}

// FNV-1a of a file's identity: real path, size, mtime, inode, device (false: no such file).
bool file_identity_hash(const std::string& input, u64* h) {
  struct stat st;
  char real[4096];
  if (::stat(input.c_str(), &st) != 0 || !::realpath(input.c_str(), real)) return false;
  *h = fnv1a(1469598103934665603ull, real, std::strlen(real));
  const u64 id[5] = {(u64)st.st_size, (u64)st.st_mtim.tv_sec, (u64)st.st_mtim.tv_nsec,
                     (u64)st.st_ino, (u64)st.st_dev};
  *h = fnv1a(*h, id, sizeof(id));
  return true;
}

// Best-effort atomic write of a cache file (directory mode 0700, one level up too).
void save_cache_file(const std::string& path, const std::vector<char>& bytes) {
  const size_t slash = path.rfind('/');
  if (slash != std::string::npos) {
    const std::string dir = path.substr(0, slash);
    const size_t up = dir.rfind('/');
    if (up != std::string::npos && up > 0) (void)::mkdir(dir.substr(0, up).c_str(), 0700);
    (void)::mkdir(dir.c_str(), 0700);
  }
  const std::string tmp = path + "." + std::to_string((long long)::getpid()) + ".tmp";
  std::FILE* f = std::fopen(tmp.c_str(), "wb");
  if (!f) return;
  bool ok = bytes.empty() || std::fwrite(bytes.data(), 1, bytes.size(), f) == bytes.size();
  ok = std::fclose(f) == 0 && ok;
  if (!ok || std::rename(tmp.c_str(), path.c_str()) != 0) (void)::unlink(tmp.c_str());
}

// ---- sparse line index (find_line_window) ----
// nl_before[i] = newlines in [0, i * kLixBlock): a contiguous prefix of the file's blocks,
// grown by every scan that passes them; complete: a scan reached EOF and `total` is the
// file's line count (a final line without '\n' counts).
constexpr u64 kLixBlock = 8ull << 20;
constexpr char kLixMagic[8] = {'L', 'C', 'S', 'T', 'L', 'I', 'X', '1'};
struct LineIndex {
  std::vector<u64> nl_before;
  bool complete = false;
  u64 total = 0;
};

bool load_line_index(const std::string& path, u64 file_bytes, LineIndex* lix) {
  if (path.empty()) return false;
  std::FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) return false;
  char magic[8];
  u64 head[4] = {};  // block bytes, file bytes, complete, total
  u64 m = 0;
  bool ok = std::fread(magic, 8, 1, f) == 1 && std::memcmp(magic, kLixMagic, 8) == 0 &&
            std::fread(head, sizeof(head), 1, f) == 1 && head[0] == kLixBlock &&
            head[1] == file_bytes && std::fread(&m, sizeof(m), 1, f) == 1 && m >= 1 &&
            (m - 1) * kLixBlock < std::max<u64>(file_bytes, 1);
  if (ok) {
    lix->nl_before.resize(m);
    ok = std::fread(lix->nl_before.data(), sizeof(u64), m, f) == m && lix->nl_before[0] == 0;
    for (u64 i = 1; ok && i < m; ++i) ok = lix->nl_before[i] >= lix->nl_before[i - 1];
    lix->complete = head[2] != 0;
    lix->total = head[3];
  }
  std::fclose(f);
  if (!ok) *lix = LineIndex();
  return ok;
}

void save_line_index(const std::string& path, u64 file_bytes, const LineIndex& lix) {
  if (path.empty() || lix.nl_before.empty()) return;
  std::vector<char> b(8 + 4 * 8 + 8 + lix.nl_before.size() * 8);
  char* p = b.data();
  std::memcpy(p, kLixMagic, 8);
  const u64 head[4] = {kLixBlock, file_bytes, lix.complete ? 1ull : 0ull, lix.total};
  std::memcpy(p + 8, head, sizeof(head));
  const u64 m = lix.nl_before.size();
  std::memcpy(p + 40, &m, 8);
  std::memcpy(p + 48, lix.nl_before.data(), m * 8);
  save_cache_file(path, b);
}
}  // namespace

std::string line_index_cache_path(const std::string& input) {
  if (const char* e = std::getenv("LOCUST_LINE_CACHE"))
    if (e[0] == '0') return "";
  const std::string dir = cache_dir();
  u64 h = 0;
  if (dir.empty() || !file_identity_hash(input, &h)) return "";
  char name[64];
  std::snprintf(name, sizeof(name), "/lines-%016llx.bin", (unsigned long long)h);
  return dir + name;
}

// Line k starts after the k-th '\n' (line 0 at byte 0).  The scan starts at the last block
// of the cached sparse line index that lies before the first newline it needs (so a window
// deep in a file costs one block, not the file's prefix, once any scan has passed there),
// runs T threads x 8 MiB blocks per round (never the whole file in memory), and records the
// newline count at every block start it passes.
LineWindow find_line_window(const std::string& path, i64 line_start, i64 line_end, u32 threads) {
  Fd f(path);
  const u64 n = f.size();
  const u64 s = (u64)std::max<i64>(line_start, 0);
  bool open_end = line_end < 0;
  const u64 e = open_end ? ~0ull : std::max<u64>((u64)line_end, s);
  constexpr u64 kNone = ~0ull;
  constexpr u64 B = kLixBlock;
  const std::string cpath = line_index_cache_path(path);
  LineIndex lix;
  load_line_index(cpath, n, &lix);
  const u64 m0 = lix.nl_before.size();
  const bool complete0 = lix.complete;
  LineWindow w;
  if (lix.complete) {  // the line count is known: clamp the window to it
    if (s >= lix.total) {
      w.begin = w.end = n;
      return w;
    }
    if (!open_end && e >= lix.total) open_end = true;
  }
  u64 at[2] = {s == 0 ? 0 : kNone, open_end ? kNone : (e == 0 ? 0 : kNone)};
  const u64 want[2] = {s, e};
  // first block: the last indexed block start with fewer newlines before it than the first
  // newline still wanted (only EOF wanted: the last indexed block)
  const u64 first_want = at[0] == kNone ? s : (at[1] == kNone && !open_end ? e : kNone);
  u64 blk0 = 0;
  if (m0) {
    if (first_want == kNone) {
      blk0 = m0 - 1;
    } else {
      const auto it = std::lower_bound(lix.nl_before.begin(), lix.nl_before.end(), first_want);
      blk0 = (u64)(it - lix.nl_before.begin()) - 1;  // nl_before[0] == 0 < first_want
    }
  }
  const u32 T = std::max<u32>(1, io_threads(threads, n));
  std::vector<std::vector<char>> buf(T, std::vector<char>(B));
  std::vector<u64> nls(T), got(T);
  std::vector<char> ok(T, 1);
  u64 base = blk0 * B;
  u64 seen = m0 ? lix.nl_before[blk0] : 0;  // newlines before `base`
  u64 after_nl = kNone;                     // offset just after the last newline seen
  auto done = [&] {
    return at[0] != kNone && (open_end ? lix.complete : at[1] != kNone);
  };
  while (base < n && !done()) {
    // Blocks to read this round: T, or only the one the index says holds the next wanted
    // newline.  Line s found and line e not yet: first jump over the window's bytes to the
    // last indexed block before line e's newline (they need no scan).
    u32 Tr = T;
    const u64 next_want = at[0] == kNone ? s : (at[1] == kNone && !open_end ? e : kNone);
    if (next_want != kNone && !lix.nl_before.empty()) {
      const auto it = std::lower_bound(lix.nl_before.begin(), lix.nl_before.end(), next_want);
      const u64 jb = (u64)(it - lix.nl_before.begin()) - 1;  // nl_before[0] == 0 < next_want
      if (jb * B > base) {
        base = jb * B;
        seen = lix.nl_before[jb];
      }
      if (jb * B == base && jb + 1 < lix.nl_before.size()) Tr = 1;  // it lies in this block
    }
    auto work = [&](u32 t) {
      const u64 a = base + (u64)t * B;
      got[t] = a < n && t < Tr ? std::min<u64>(B, n - a) : 0;
      nls[t] = 0;
      if (got[t]) ok[t] = pread_slice(f.fd, buf[t].data(), a, 0, got[t], true, &nls[t]);
    };
    if (Tr == 1) {
      work(0);
    } else {
      std::vector<std::thread> th;
      for (u32 t = 1; t < Tr; ++t) th.emplace_back(work, t);
      work(0);
      for (auto& x : th) x.join();
    }
    for (u32 t = 0; t < Tr && got[t]; ++t) {
      if (!ok[t]) throw Error("short read: " + path);
      const char* blk = buf[t].data();
      const u64 blk_off = base + (u64)t * B;
      if (blk_off / B == lix.nl_before.size()) lix.nl_before.push_back(seen);
      for (int k = 0; k < 2; ++k) {
        if (at[k] != kNone || (k == 1 && open_end) || seen + nls[t] < want[k]) continue;
        const char* p = blk;  // the (want - seen)-th newline of this block ends line want - 1
        for (u64 left = want[k] - seen;; --left) {
          const char* nl = static_cast<const char*>(memchr(p, '\n', (size_t)(blk + got[t] - p)));
          if (left == 1) {
            at[k] = blk_off + (u64)(nl - blk) + 1;
            break;
          }
          p = nl + 1;
        }
      }
      if (nls[t]) {
        const void* r = memrchr(blk, '\n', (size_t)got[t]);
        after_nl = blk_off + (u64)(static_cast<const char*>(r) - blk) + 1;
      }
      seen += nls[t];
    }
    base += (u64)Tr * B;
  }
  if (base >= n && !lix.complete) {  // the scan reached EOF: the file's line count
    // a final line without a newline counts; bytes after the scan's start with no newline
    // among them are such a line
    const u64 last_nl_end = after_nl != kNone ? after_nl : blk0 * B;
    lix.complete = true;
    lix.total = seen + (n > last_nl_end ? 1 : 0);
  }
  if (lix.nl_before.size() > m0 || lix.complete != complete0) save_line_index(cpath, n, lix);
  if (at[0] != kNone && at[1] != kNone && !open_end) {
    w.begin = at[0];
    w.end = std::max(at[0], at[1]);
    w.lines = e - s;
    return w;
  }
  // the window runs to EOF (the line count is known now)
  const u64 total = lix.total;
  if (s >= total) {
    w.begin = w.end = n;
    return w;
  }
  w.begin = at[0];  // (found: line s < total starts after the s-th newline, or at 0)
  w.end = n;
  w.lines = std::min(total, e) - s;
  return w;
}

u64 read_file_into(const std::string& path, char* dst, u64 cap, u64* lines, u32 threads) {
  Fd f(path);
  const u64 n = f.size();
  LOCUST_CHECK_ARG(n <= cap, "file larger than its buffer: " + path);
  u64 nl = n ? pread_parallel(f.fd, dst, 0, n, io_threads(threads, n), path, true) : 0;
  if (n && dst[n - 1] != '\n') ++nl;
  if (lines) *lines = nl;
  return n;
}

LoadedText load_lines(const std::string& path, i64 line_start, i64 line_end, bool ref_compat) {
  LoadedText lt;
  lt.window = line_start >= 0;
  if (!lt.window) {
    // whole file: straight into the result's storage
    Fd f(path);
    const u64 n = f.size();
    lt.storage.resize(n);
    lt.storage.reserve(n + 64);
    u64 nl = n ? pread_parallel(f.fd, lt.storage.data(), 0, n, io_threads(0, n), path, true) : 0;
    const bool open_end = n && lt.storage[n - 1] != '\n';
    lt.file_lines = nl + (open_end ? 1 : 0);
    u64 keep = n, lines = lt.file_lines;
    if (ref_compat && lines) {  // B1: whole-file mode drops the last line
      const char* d = lt.storage.data();
      const u64 end = open_end ? n : n - 1;  // the last line's terminator (or EOF)
      const void* p = end ? memrchr(d, '\n', (size_t)end) : nullptr;
      keep = p ? (u64)(static_cast<const char*>(p) - d) + 1 : 0;
      --lines;
    }
    lt.storage.resize(keep);
    lt.input.data = lt.storage.data();
    lt.input.bytes = keep;
    lt.input.num_lines = lines;
    lt.input.first_line = 0;
    return lt;
  }
  // window [first, last): read 8 MiB blocks up to the window's end, keep only its bytes
  std::FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) throw Error("cannot open input file: " + path);
  const u64 first = (u64)line_start;
  const u64 last = line_end < 0 ? ~0ull : (u64)std::max<i64>(line_end, line_start);
  std::vector<char> buf(8u << 20);
  u64 line = 0;          // current line number
  bool at_start = true;  // the next byte starts a line
  bool more = false;     // bytes remain after the window's last line (not at EOF)
  for (;;) {
    const size_t k = std::fread(buf.data(), 1, buf.size(), f);
    if (k == 0) break;
    if (line >= last) {  // the window ended exactly at the previous block's end
      more = true;
      break;
    }
    const char* p = buf.data();
    const char* end = p + k;
    while (p < end && line < last) {
      const char* nl = static_cast<const char*>(memchr(p, '\n', (size_t)(end - p)));
      const char* stop = nl ? nl + 1 : end;
      if (line >= first) lt.storage.insert(lt.storage.end(), p, stop);
      at_start = nl != nullptr;
      if (nl) ++line;
      p = stop;
    }
    if (line >= last && p < end) {
      more = true;
      break;
    }
  }
  std::fclose(f);
  if (!at_start) ++line;  // a final line without its newline
  lt.file_lines = line;   // lines scanned (the whole file when the window reaches EOF)
  u64 got = line > first ? std::min(line, last) - first : 0;
  // Reference quirk (main.cu:62-63): a window that reaches EOF reports
  // line_num - line_start lines, i.e. loses the last line.
  if (ref_compat && line_end >= 0 && !more && got) {
    const char* d = lt.storage.data();
    const u64 n = lt.storage.size();
    const u64 end = d[n - 1] == '\n' ? n - 1 : n;
    const void* q = end ? memrchr(d, '\n', (size_t)end) : nullptr;
    lt.storage.resize(q ? (u64)(static_cast<const char*>(q) - d) + 1 : 0);
    --got;
  }
  lt.storage.reserve(lt.storage.size() + 64);
  lt.input.data = lt.storage.data();
  lt.input.bytes = lt.storage.size();
  lt.input.num_lines = got;
  lt.input.first_line = std::min<u64>(first, line);
  return lt;
}

std::string key_to_string(const PackedKey& k) {
  char buf[kKeyBytes + 1];
  int n = unpack_key(k.w, buf);
  return std::string(buf, (size_t)n);
}

// ---------------- spill ----------------
namespace {
constexpr char kMagic[8] = {'L', 'C', 'S', 'T', 'S', 'P', 'L', '1'};
constexpr char kKivMagic[8] = {'L', 'C', 'S', 'T', 'K', 'I', 'V', '1'};
struct SpillHeader {
  char magic[8];
  u32 version;
  u32 key_words;
  u64 count;
  u64 reserved;
};
static_assert(sizeof(SpillHeader) == 32, "spill header 32 B");

void append_u64(std::string* s, u64 v) {
  char tmp[24];
  int n = 0;
  do {
    tmp[n++] = (char)('0' + v % 10);
    v /= 10;
  } while (v);
  while (n) s->push_back(tmp[--n]);
}

// One reference record from a packed key: NUL-padded key[30], int value, int count.
KeyIntValuePair to_kiv(const u64* w, i64 value, i64 count, const std::string& path) {
  KeyIntValuePair r;
  std::memset(&r, 0, sizeof(r));
  char buf[kKeyBytes + 1];
  const int n = unpack_key(w, buf);
  if (n > kMaxKeyLen) throw Error("key longer than KeyIntValuePair::key[30] holds: " + path);
  if (value < INT32_MIN || value > INT32_MAX || count < INT32_MIN || count > INT32_MAX)
    throw Error("value beyond KeyIntValuePair's int fields: " + path);
  std::memcpy(r.key, buf, (size_t)n);
  r.value = (int)value;
  r.count = (int)count;
  return r;
}

void write_kiv_file(const std::string& path, const std::vector<KeyIntValuePair>& recs) {
  std::FILE* f = std::fopen(path.c_str(), "wb");
  if (!f) throw Error("cannot write kiv file: " + path);
  SpillHeader h{};
  std::memcpy(h.magic, kKivMagic, 8);
  h.version = 1;
  h.key_words = (u32)sizeof(KeyIntValuePair);  // record size
  h.count = recs.size();
  std::fwrite(&h, sizeof(h), 1, f);
  if (!recs.empty()) std::fwrite(recs.data(), sizeof(KeyIntValuePair), recs.size(), f);
  if (std::fclose(f) != 0) throw Error("error closing kiv file: " + path);
}
}  // namespace

void write_kiv_results(const std::string& path, const WordCountResult& r) {
  const EntryList& e = r.entries;
  std::vector<KeyIntValuePair> v;
  v.reserve(e.size());
  EntryVals vals(r);
  for (const WordCountEntry x : e) v.push_back(to_kiv(x.key.w, (i64)vals.next(x), (i64)x.count, path));
  write_kiv_file(path, v);
}

std::vector<KivRecord> read_kiv(const std::string& path) {
  std::FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) throw Error("cannot open kiv file: " + path);
  SpillHeader h{};
  const bool ok = std::fread(&h, sizeof(h), 1, f) == 1 && std::memcmp(h.magic, kKivMagic, 8) == 0 &&
                  h.version == 1 && h.key_words == sizeof(KeyIntValuePair);
  std::vector<KeyIntValuePair> raw(ok ? h.count : 0);
  const bool full = ok && (raw.empty() ||
                           std::fread(raw.data(), sizeof(KeyIntValuePair), raw.size(), f) == raw.size());
  std::fclose(f);
  if (!ok) throw Error("not a kiv file: " + path);
  if (!full) throw Error("truncated kiv file: " + path);
  std::vector<KivRecord> out(raw.size());
  for (size_t i = 0; i < raw.size(); ++i) {
    const int n = (int)strnlen(raw[i].key, sizeof(raw[i].key));  // bounded (reference bug B11)
    pack_key(raw[i].key, n, out[i].key.w);
    out[i].value = raw[i].value;
    out[i].count = raw[i].count;
  }
  return out;
}

namespace {
constexpr char kIdxMagic[8] = {'L', 'C', 'S', 'T', 'I', 'D', 'X', '1'};
constexpr u64 kIndexSamples = 256;  // samples per spill (<= 16 KiB of index), every >= 16th record
struct IndexHeader {
  char magic[8];
  u32 version, flags;  // flags: 1 sorted, 2 distinct
  u64 records, total_count, spill_bytes, nsamples, stride, reserved;
};
static_assert(sizeof(IndexHeader) == 64, "index header 64 B");
struct IndexRecord {
  u64 key[kKeyWords];
  u64 record, offset, count_before, reserved;
};
static_assert(sizeof(IndexRecord) == 64, "index record 64 B");

// Index bookkeeping while a spill is written record by record.
struct IndexBuilder {
  SpillIndex* idx;
  const KeyCount* prev = nullptr;
  u64 i = 0, cum = 0;
  IndexBuilder(SpillIndex* x, u64 n) : idx(x) {
    if (!idx) return;
    *idx = SpillIndex();
    idx->sorted = idx->distinct = true;
    idx->records = n;
    idx->stride = std::max<u64>(16, div_up(n, kIndexSamples));
  }
  void add(const KeyCount& r, u64 offset) {
    if (!idx) return;
    if (prev) {
      const int c = key_compare(prev->w, r.w);
      if (c > 0) idx->sorted = idx->distinct = false;
      if (c == 0) idx->distinct = false;
    }
    if (i % idx->stride == 0) {
      SpillSample smp;
      for (int w = 0; w < kKeyWords; ++w) smp.key.w[w] = r.w[w];
      smp.record = i;
      smp.offset = offset;
      smp.count_before = cum;
      idx->samples.push_back(smp);
    }
    cum += r.count;
    prev = &r;
    ++i;
  }
  void finish(u64 bytes) {
    if (!idx) return;
    idx->records = i;
    idx->total_count = cum;
    idx->spill_bytes = bytes;
  }
};
}  // namespace

void write_spill(const std::string& path, const std::vector<KeyCount>& recs, SpillFormat fmt,
                 SpillIndex* idx) {
  std::vector<KeyCount> live;  // the reference skips empty keys (main.cu:118)
  const std::vector<KeyCount>* src = &recs;
  for (const auto& r : recs)
    if (!r.w[0]) {
      live.reserve(recs.size());
      for (const auto& x : recs)
        if (x.w[0]) live.push_back(x);
      src = &live;
      break;
    }
  IndexBuilder ib(idx, src->size());
  if (fmt == SpillFormat::kKiv) {
    std::vector<KeyIntValuePair> v;
    v.reserve(src->size());
    u64 off = sizeof(SpillHeader);
    for (const auto& r : *src) {
      v.push_back(to_kiv(r.w, (i64)r.count, 0, path));
      ib.add(r, off);
      off += sizeof(KeyIntValuePair);
    }
    write_kiv_file(path, v);
    ib.finish(off);
    return;
  }
  std::FILE* f = std::fopen(path.c_str(), "wb");
  if (!f) throw Error("cannot write spill file: " + path);
  u64 bytes = 0;
  if (fmt == SpillFormat::kBinary) {
    SpillHeader h{};
    std::memcpy(h.magic, kMagic, 8);
    h.version = 1;
    h.key_words = kKeyWords;
    h.count = src->size();
    std::fwrite(&h, sizeof(h), 1, f);
    if (!src->empty()) std::fwrite(src->data(), sizeof(KeyCount), src->size(), f);
    bytes = sizeof(h);
    for (const auto& r : *src) {
      ib.add(r, bytes);
      bytes += sizeof(KeyCount);
    }
  } else {
    std::string s;
    s.reserve(std::min<size_t>(src->size(), 1u << 20) * 16);
    char buf[kKeyBytes + 1];
    for (const auto& r : *src) {
      ib.add(r, bytes + s.size());
      const int n = unpack_key(r.w, buf);
      s.append(buf, (size_t)n);
      s.append(" \t");
      append_u64(&s, r.count);
      s.push_back('\n');
      if (s.size() >= (8u << 20)) {  // bounded buffer: spills of any size
        write_all(f, s);
        bytes += s.size();
        s.clear();
      }
    }
    write_all(f, s);
    bytes += s.size();
  }
  if (std::fclose(f) != 0) throw Error("error closing spill file: " + path);
  ib.finish(bytes);
}

std::string spill_index_path(const std::string& spill) { return spill + ".idx"; }

void write_spill_index(const std::string& path, const SpillIndex& idx) {
  std::FILE* f = std::fopen(path.c_str(), "wb");
  if (!f) throw Error("cannot write spill index: " + path);
  IndexHeader h{};
  std::memcpy(h.magic, kIdxMagic, 8);
  h.version = 1;
  h.flags = (idx.sorted ? 1u : 0u) | (idx.distinct ? 2u : 0u);
  h.records = idx.records;
  h.total_count = idx.total_count;
  h.spill_bytes = idx.spill_bytes;
  h.nsamples = idx.samples.size();
  h.stride = idx.stride;
  std::fwrite(&h, sizeof(h), 1, f);
  for (const SpillSample& x : idx.samples) {
    IndexRecord r{};
    for (int w = 0; w < kKeyWords; ++w) r.key[w] = x.key.w[w];
    r.record = x.record;
    r.offset = x.offset;
    r.count_before = x.count_before;
    std::fwrite(&r, sizeof(r), 1, f);
  }
  if (std::fclose(f) != 0) throw Error("error closing spill index: " + path);
}

bool read_spill_index(const std::string& spill, SpillIndex* idx) {
  std::FILE* f = std::fopen(spill_index_path(spill).c_str(), "rb");
  if (!f) return false;
  IndexHeader h{};
  bool ok = std::fread(&h, sizeof(h), 1, f) == 1 && std::memcmp(h.magic, kIdxMagic, 8) == 0 &&
            h.version == 1 && h.nsamples <= (1u << 24) && h.stride >= 1;
  std::vector<IndexRecord> v(ok ? h.nsamples : 0);
  ok = ok && (v.empty() || std::fread(v.data(), sizeof(IndexRecord), v.size(), f) == v.size());
  std::fclose(f);
  u64 size = 0;
  try {
    size = file_size(spill);
  } catch (const std::exception&) {
    return false;
  }
  if (!ok || size != h.spill_bytes) return false;  // absent, damaged or stale
  *idx = SpillIndex();
  idx->sorted = (h.flags & 1u) != 0;
  idx->distinct = (h.flags & 2u) != 0;
  idx->records = h.records;
  idx->total_count = h.total_count;
  idx->spill_bytes = h.spill_bytes;
  idx->stride = h.stride;
  idx->samples.resize(v.size());
  for (size_t i = 0; i < v.size(); ++i) {
    for (int w = 0; w < kKeyWords; ++w) idx->samples[i].key.w[w] = v[i].key[w];
    idx->samples[i].record = v[i].record;
    idx->samples[i].offset = v[i].offset;
    idx->samples[i].count_before = v[i].count_before;
  }
  return true;
}

SpillReader::SpillReader(const std::string& path) : path_(path), buf_(1u << 20) {
  f_ = std::fopen(path.c_str(), "rb");
  if (!f_) throw Error("cannot open spill file: " + path);
  size_ = file_size(path);
  char m[sizeof(SpillHeader)] = {};
  const size_t got = std::fread(m, 1, sizeof(m), f_);
  if (got == sizeof(SpillHeader) && std::memcmp(m, kKivMagic, 8) == 0) {
    SpillHeader h;
    std::memcpy(&h, m, sizeof(h));
    if (h.version != 1 || h.key_words != sizeof(KeyIntValuePair))
      throw Error("not a kiv file: " + path);
    if (size_ < sizeof(h) + h.count * sizeof(KeyIntValuePair)) throw Error("truncated kiv file: " + path);
    fmt_ = SpillFormat::kKiv;
    first_ = sizeof(h);
    size_ = sizeof(h) + h.count * sizeof(KeyIntValuePair);
  } else if (got == sizeof(SpillHeader) && std::memcmp(m, kMagic, 8) == 0) {
    SpillHeader h;
    std::memcpy(&h, m, sizeof(h));
    if (h.version != 1 || h.key_words != kKeyWords) throw Error("unsupported spill file: " + path);
    if (size_ < sizeof(h) + h.count * sizeof(KeyCount)) throw Error("truncated spill: " + path);
    fmt_ = SpillFormat::kBinary;
    first_ = sizeof(h);
    size_ = sizeof(h) + h.count * sizeof(KeyCount);
  } else {
    fmt_ = SpillFormat::kText;
    first_ = 0;
  }
  seek(first_);
}

SpillReader::~SpillReader() {
  if (f_) std::fclose(f_);
}

void SpillReader::seek(u64 offset) {
  LOCUST_CHECK_ARG(offset >= first_ && offset <= size_, "spill offset out of range: " + path_);
  if (std::fseek(f_, (long)offset, SEEK_SET) != 0) throw Error("cannot seek in " + path_);
  pos_ = offset;
  at_ = len_ = 0;
}

bool SpillReader::fill() {  // keeps the unread tail, appends the next read
  if (at_ > 0) {
    std::memmove(buf_.data(), buf_.data() + at_, len_ - at_);
    pos_ += at_;
    len_ -= at_;
    at_ = 0;
  }
  if (len_ == buf_.size()) buf_.resize(buf_.size() * 2);  // a text line longer than the buffer
  const u64 end_of_data = size_;
  const u64 file_at = pos_ + len_;
  if (file_at >= end_of_data) return false;
  const size_t want = (size_t)std::min<u64>(buf_.size() - len_, end_of_data - file_at);
  const size_t k = std::fread(buf_.data() + len_, 1, want, f_);
  if (k == 0) throw Error("short read: " + path_);
  len_ += k;
  return true;
}

bool SpillReader::next(KeyCount* rec, u64* offset) {
  if (fmt_ != SpillFormat::kText) {
    const size_t rs = 40;
    while (len_ - at_ < rs)
      if (!fill()) {
        if (len_ != at_) throw Error("truncated spill: " + path_);
        return false;
      }
    if (offset) *offset = pos_ + at_;
    const char* p = buf_.data() + at_;
    if (fmt_ == SpillFormat::kBinary) {
      std::memcpy(rec, p, sizeof(KeyCount));
    } else {
      KeyIntValuePair k;
      std::memcpy(&k, p, sizeof(k));
      pack_key(k.key, (int)strnlen(k.key, sizeof(k.key)), rec->w);  // bounded (B11)
      if (k.value < 0) throw Error("negative count in kiv spill: " + path_);
      rec->count = (u64)k.value;  // value = the record's count (map output)
    }
    at_ += rs;
    return true;
  }
  // text: "<key> \t<count>\n"; the reference's key keeps a trailing space (B8: stripped)
  for (;;) {
    const char* p = buf_.data() + at_;
    const char* e = buf_.data() + len_;
    const char* nl = static_cast<const char*>(memchr(p, '\n', (size_t)(e - p)));
    if (!nl && fill()) continue;
    if (!nl) nl = e;  // a final line without '\n'
    if (nl == p) {
      if (p == e) return false;
      ++at_;  // an empty line
      continue;
    }
    if (offset) *offset = pos_ + at_;
    const char* tab = static_cast<const char*>(memchr(p, '\t', (size_t)(nl - p)));
    const char* key_end = tab ? tab : nl;
    if (key_end > p && key_end[-1] == ' ') --key_end;
    pack_key(p, (int)(key_end - p), rec->w);
    u64 cnt = 1;
    if (tab) {
      cnt = 0;
      const char* q = tab + 1;
      while (q < nl && (*q == ' ' || *q == '\t')) ++q;
      for (; q < nl && *q >= '0' && *q <= '9'; ++q) cnt = cnt * 10 + (u64)(*q - '0');
    }
    rec->count = cnt;
    at_ = (size_t)(nl - buf_.data()) + (nl < e ? 1 : 0);
    return true;
  }
}

std::vector<KeyCount> read_spill(const std::string& path) {
  SpillReader rd(path);
  std::vector<KeyCount> recs;
  if (rd.format() != SpillFormat::kText) recs.reserve((rd.bytes() - rd.first_record_offset()) / 40);
  KeyCount r;
  while (rd.next(&r)) recs.push_back(r);
  return recs;
}

std::vector<KeyCount> tokens_to_records(const std::vector<PackedKey>& toks) {
  std::vector<KeyCount> recs(toks.size());
  for (size_t i = 0; i < toks.size(); ++i) {
    for (int w = 0; w < kKeyWords; ++w) recs[i].w[w] = toks[i].w[w];
    recs[i].count = 1;
  }
  return recs;
}

std::vector<KeyCount> entries_to_records(const EntryList& e) {
  std::vector<KeyCount> recs;
  recs.reserve(e.size());
  for (const WordCountEntry x : e) {
    KeyCount r;
    for (int w = 0; w < kKeyWords; ++w) r.w[w] = x.key.w[w];
    r.count = x.count;
    recs.push_back(r);
  }
  return recs;
}

// ---------------- partition-map cache ----------------
namespace {
constexpr char kPmcMagic[8] = {'L', 'C', 'S', 'T', 'P', 'M', 'C', '1'};
}  // namespace

std::string partmap_cache_path(const std::string& input, const JobConfig& cfg) {
  if (const char* e = std::getenv("LOCUST_PART_CACHE"))
    if (e[0] == '0') return "";
  const std::string dir = cache_dir();
  u64 h = 0;
  if (dir.empty() || !file_identity_hash(input, &h)) return "";
  const int tok[4] = {cfg.emits_per_line, cfg.max_key_len, (int)cfg.map_path, (int)cfg.sort_path};
  h = fnv1a(h, tok, sizeof(tok));
  h = fnv1a(h, cfg.delimiters.data(), cfg.delimiters.size());
  char name[64];
  std::snprintf(name, sizeof(name), "/partmap-%016llx.bin", (unsigned long long)h);
  return dir + name;
}

bool load_partmap_cache(const std::string& path, std::vector<u64>* lo) {
  if (path.empty()) return false;
  std::FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) return false;
  char magic[8];
  u32 n = 0;
  bool ok = std::fread(magic, 8, 1, f) == 1 && std::memcmp(magic, kPmcMagic, 8) == 0 &&
            std::fread(&n, sizeof(n), 1, f) == 1 && n == (u32)kDictParts + 1;
  if (ok) {
    lo->resize(n);
    ok = std::fread(lo->data(), sizeof(u64), n, f) == n;
  }
  std::fclose(f);
  return ok;
}

void save_partmap_cache(const std::string& path, const std::vector<u64>& lo) {
  if (path.empty() || lo.size() != (size_t)kDictParts + 1) return;
  const u32 n = (u32)lo.size();
  std::vector<char> b(8 + sizeof(n) + n * sizeof(u64));
  std::memcpy(b.data(), kPmcMagic, 8);
  std::memcpy(b.data() + 8, &n, sizeof(n));
  std::memcpy(b.data() + 8 + sizeof(n), lo.data(), n * sizeof(u64));
  save_cache_file(path, b);
}

// ---------------- output ----------------
void format_gpu_output(const WordCountResult& r, std::string* out) {
  const EntryList& e = r.entries;
  out->reserve(out->size() + e.size() * 48);
  char buf[kKeyBytes + 1];
  EntryVals vals(r);
  for (const WordCountEntry x : e) {
    const u64 val = vals.next(x);
    int n = unpack_key(x.key.w, buf);
    if (n == 0) continue;
    out->append("print key: ");
    out->append(buf, (size_t)n);
    out->append(" \t val: ");
    append_u64(out, val);
    out->append(" \t count: ");
    append_u64(out, x.count);
    out->push_back('\n');
  }
}

void format_cpu_output(const WordCountResult& r, std::string* out) {
  const EntryList& e = r.entries;
  out->reserve(out->size() + e.size() * 32);
  char buf[kKeyBytes + 1];
  for (const WordCountEntry x : e) {
    int n = unpack_key(x.key.w, buf);
    if (n == 0) continue;
    out->append("print key: ");
    out->append(buf, (size_t)n);
    out->append(" \t value: ");
    append_u64(out, x.count);
    out->push_back('\n');
  }
}

void write_all(std::FILE* f, const std::string& s) {
  if (!s.empty() && std::fwrite(s.data(), 1, s.size(), f) != s.size())
    throw Error("short write");
}

}  // namespace locust
