// Host read throughput of the streaming source (FileTextSource: parallel pread from the
// page cache into a ring of pieces, newline count, whole-line carry) apart from the GPU:
// where a streamed file's ~18-24 GB/s goes (the in-memory 10 GB job runs at 55 GB/s).
//   build/read_probe FILE [threads...]   (pieces of 16 MiB into 4 malloc'd ring slots)
// plus, per thread count, the raw parallel pread of the same pieces without the newline
// count (what the count costs) -- fresh threads per piece, so an upper bound on overhead.
// Build: make read_probe
#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#include "locust/engine.hpp"

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: read_probe FILE [threads...]\n");
    return 2;
  }
  std::vector<unsigned> threads;
  for (int i = 2; i < argc; ++i) threads.push_back((unsigned)std::atoi(argv[i]));
  if (threads.empty()) threads = {0, 1, 2, 4, 8, 16};
  const size_t piece = 16u << 20;
  std::vector<std::vector<char>> ring(4, std::vector<char>(piece + 64));
  for (unsigned t : threads) {
    for (int rep = 0; rep < 2; ++rep) {  // the first pass may still fault the page cache in
      auto src = locust::open_file_source(argv[1], t);
      const auto t0 = std::chrono::steady_clock::now();
      unsigned long long total = 0;
      for (size_t r = 0;; ++r) {
        const unsigned long long n = src->next(ring[r % 4].data(), piece);
        if (!n) break;
        total += n;
      }
      const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      std::printf("threads %2u (%s) pass %d: %.2f GB in %.1f ms = %.1f GB/s, %llu lines\n", t,
                  t ? "fixed" : "auto", rep, total / 1e9, s * 1e3, total / 1e9 / s,
                  (unsigned long long)src->lines());
    }
  }
  const int fd = ::open(argv[1], O_RDONLY | O_CLOEXEC);
  if (fd < 0) return 3;
  const off_t size = ::lseek(fd, 0, SEEK_END);
  for (unsigned t : threads) {
    const unsigned nt = t ? t : 8;
    for (int count = 0; count < 2; ++count) {
      const auto t0 = std::chrono::steady_clock::now();
      unsigned long long nl = 0;
      for (off_t pos = 0, r = 0; pos < size; pos += (off_t)piece, ++r) {
        const size_t n = (size_t)std::min<off_t>((off_t)piece, size - pos);
        char* dst = ring[r % 4].data();
        std::vector<std::thread> th;
        std::vector<unsigned long long> c(nt, 0);
        for (unsigned k = 0; k < nt; ++k)
          th.emplace_back([&, k] {
            const size_t a = n * k / nt, b = n * (k + 1) / nt;
            size_t p = a;
            while (p < b) {
              const ssize_t got = ::pread(fd, dst + p, b - p, pos + (off_t)p);
              if (got <= 0) break;
              p += (size_t)got;
            }
            if (count) c[k] = (unsigned long long)std::count(dst + a, dst + b, '\n');
          });
        for (auto& x : th) x.join();
        for (auto v : c) nl += v;
      }
      const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      std::printf("raw pread, %2u threads, %s: %.1f ms = %.1f GB/s (%llu newlines)\n", nt,
                  count ? "with count" : "no count  ", s * 1e3, size / 1e9 / s, nl);
    }
  }
  ::close(fd);
  return 0;
}
