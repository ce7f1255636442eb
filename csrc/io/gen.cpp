// Synthetic text generator (see locust/gen.hpp for the shape it reproduces).
#include "locust/gen.hpp"
#include "locust/io.hpp"

#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstring>
#include <thread>
#include <unordered_set>

namespace locust {
namespace {

inline u64 splitmix(u64& x) {
  u64 z = (x += 0x9e3779b97f4a7c15ull);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

// xoshiro256** -- one stream per 1,024-line block.
struct Rng {
  u64 s[4];
  explicit Rng(u64 seed) {
    u64 x = seed;
    for (auto& v : s) v = splitmix(x);
  }
  static u64 rotl(u64 v, int k) { return (v << k) | (v >> (64 - k)); }
  u64 next() {
    const u64 r = rotl(s[1] * 5, 7) * 9;
    const u64 t = s[1] << 17;
    s[2] ^= s[0];
    s[3] ^= s[1];
    s[1] ^= s[2];
    s[0] ^= s[3];
    s[2] ^= t;
    s[3] = rotl(s[3], 45);
    return r;
  }
  u32 below(u32 n) { return (u32)(((next() >> 32) * (u64)n) >> 32); }
  double unit() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
};

// English letter frequencies (per mille), a..z.
constexpr int kLetterFreq[26] = {82, 15, 28, 43, 127, 22, 20, 61, 70, 2,  8,  40, 24,
                                 67, 75, 19, 1,  60, 63, 91, 28, 10, 24, 2,  20, 1};

struct Model {
  std::vector<char> chars;     // the words back to back
  std::vector<u32> off;        // word r = chars[off[r] .. off[r] + len[r])
  std::vector<u8> len;
  // Walker alias table over word ranks (Zipf weights); coin thresholds in 1/65536.
  std::vector<u32> coin;
  std::vector<u32> alias;
};

Model build_model(const GenSpec& spec) {
  Model m;
  const std::vector<std::string> words = gen_vocabulary(spec.vocab, spec.seed);
  const u32 v = (u32)words.size();
  for (const auto& w : words) {
    m.off.push_back((u32)m.chars.size());
    m.len.push_back((u8)w.size());
    m.chars.insert(m.chars.end(), w.begin(), w.end());
  }
  std::vector<double> w(v);
  double sum = 0;
  for (u32 r = 0; r < v; ++r) sum += (w[r] = 1.0 / std::pow((double)r + 1.0, spec.zipf_s));
  m.coin.assign(v, 65536);
  m.alias.resize(v);
  for (u32 r = 0; r < v; ++r) m.alias[r] = r;
  std::vector<u32> small, large;
  std::vector<double> sc(v);
  for (u32 r = 0; r < v; ++r) {
    sc[r] = w[r] * v / sum;
    (sc[r] < 1.0 ? small : large).push_back(r);
  }
  while (!small.empty() && !large.empty()) {
    const u32 a = small.back(), b = large.back();
    small.pop_back();
    m.coin[a] = (u32)(sc[a] * 65536.0);
    m.alias[a] = b;
    sc[b] -= 1.0 - sc[a];
    if (sc[b] < 1.0) {
      large.pop_back();
      small.push_back(b);
    }
  }
  return m;
}

// Separator table indexed by 6 random bits: ' ' 86%, ", " 8%, ". " 3%, "; ", ": ", "-".
struct SepTable {
  const char* s[64];
  u8 n[64];
  SepTable() {
    for (int i = 0; i < 64; ++i) {
      const char* x = i < 55 ? " " : i < 60 ? ", " : i < 62 ? ". " : i < 63 ? "; " : "-";
      s[i] = x;
      n[i] = (u8)std::strlen(x);
    }
  }
};
const SepTable kSep;

// Lines [block * 1024, block * 1024 + nlines) of the text, appended to `out`.
void gen_block(const Model& m, const GenSpec& spec, u64 block, u64 nlines, std::string& out) {
  u64 sx = spec.seed ^ (block * 0xd1342543de82ef95ull);
  Rng g(splitmix(sx));
  out.clear();
  out.resize(nlines * ((u64)spec.max_line_chars + 2));
  char* o = &out[0];
  char* const base = o;
  const u32 width = std::max<u32>(spec.max_line_chars, 8);
  const u32 v = (u32)m.coin.size();
  for (u64 l = 0; l < nlines; ++l) {
    const u64 h = g.next();
    char* const line = o;
    if ((h & 31) != 0) {  // ~3% blank lines
      if (((h >> 5) & 15) == 0) {  // verse indentation
        const int ind = 2 + (int)((h >> 9) & 1);
        for (int k = 0; k < ind; ++k) *o++ = ' ';
      }
      const u32 want = 1 + (u32)(((h >> 10) & 0xffff) * 12 >> 16);
      for (u32 k = 0; k < want; ++k) {
        const u64 r = g.next();
        u32 id = (u32)(((r & 0xffffffffull) * v) >> 32);
        if (((r >> 32) & 0xffff) >= m.coin[id]) id = m.alias[id];
        const u32 wl = m.len[id];
        const u32 sc = (u32)(r >> 58);
        const u32 sn = k ? kSep.n[sc] : 0;
        if ((u32)(o - line) + sn + wl + 2 > width) break;
        for (u32 q = 0; q < sn; ++q) *o++ = kSep.s[sc][q];
        char* const w = o;
        std::memcpy(o, &m.chars[m.off[id]], wl);
        o += wl;
        const u32 caps = (u32)((r >> 48) & 0x3ff);  // 1/1024 units
        if (caps < 2) {
          for (char* c = w; c < o; ++c) *c = (char)std::toupper((unsigned char)*c);
        } else if (caps < (k == 0 ? 512u : 51u)) {
          *w = (char)std::toupper((unsigned char)*w);
        }
        const u32 bang = (u32)((r >> 42) & 63);  // '!' / '?' are not delimiters
        if (bang == 0) *o++ = '!';
        else if (bang == 1) *o++ = '?';
      }
      const u32 e = (u32)((h >> 32) & 127);
      if ((u32)(o - line) + 1 <= width) {
        if (e < 38) *o++ = '.';
        else if (e < 51) *o++ = ',';
        else if (e < 55) *o++ = '?';
      }
    }
    *o++ = '\n';
  }
  out.resize((size_t)(o - base));
}

u32 gen_threads(const GenSpec& s) {
  const u32 hw = std::max(1u, std::thread::hardware_concurrency());
  return s.threads ? s.threads : std::min<u32>(hw, 16);  // the GPU box's CPU share is 16
}

// Runs `sink(block_text, block_lines)` in block order until it returns false or the
// spec's line target is reached.  Blocks are generated in parallel rounds.
template <class Sink>
void generate(const GenSpec& spec, Sink&& sink) {
  const Model m = build_model(spec);
  const u32 T = gen_threads(spec);
  const u64 round = (u64)T * 16;
  const bool by_lines = spec.lines > 0;
  const u64 nblocks = by_lines ? div_up(spec.lines, kGenBlockLines) : ~0ull;
  std::vector<std::string> blk(round);
  for (u64 b0 = 0; b0 < nblocks; b0 += round) {
    const u64 nb = std::min<u64>(round, nblocks - b0);
    auto lines_of = [&](u64 j) {
      const u64 b = b0 + j;
      return by_lines && b == nblocks - 1 ? spec.lines - b * kGenBlockLines : kGenBlockLines;
    };
    std::vector<std::thread> th;
    for (u32 t = 0; t < T; ++t)
      th.emplace_back([&, t] {
        for (u64 j = t; j < nb; j += T) gen_block(m, spec, spec.first_block + b0 + j, lines_of(j), blk[j]);
      });
    for (auto& x : th) x.join();
    for (u64 j = 0; j < nb; ++j)
      if (!sink(blk[j], lines_of(j))) return;
  }
}

}  // namespace

std::vector<std::string> gen_vocabulary(u32 vocab, u64 seed) {
  LOCUST_CHECK_ARG(vocab >= 1, "vocab must be >= 1");
  int cum[26];
  int acc = 0;
  for (int i = 0; i < 26; ++i) cum[i] = (acc += kLetterFreq[i]);
  std::vector<std::string> words;
  words.reserve(vocab);
  std::unordered_set<std::string> seen;
  u64 sx = seed * 0x2545f4914f6cdd1dull + 17;
  Rng g(splitmix(sx));
  for (u32 r = 0; words.size() < vocab; ++r) {
    // frequent words are short (Hamlet: "the", "and", "to", "of", "I"); rare ones long
    const double base = 1.6 + 0.55 * std::log2((double)words.size() + 2.0);
    const double noise = (g.unit() + g.unit() + g.unit() - 1.5) * 2.0;
    const int len = std::max(1, std::min(14, (int)std::lround(base + noise)));
    std::string w((size_t)len, 'a');
    for (auto& ch : w) {
      const int x = (int)g.below((u32)acc);
      int i = 0;
      while (cum[i] <= x) ++i;
      ch = (char)('a' + i);
    }
    if (seen.insert(w).second) words.push_back(std::move(w));
  }
  return words;
}

u64 gen_text(const GenSpec& spec, std::string* out) {
  LOCUST_CHECK_ARG(spec.lines > 0 || spec.bytes > 0, "set lines or bytes");
  u64 lines = 0;
  const u64 start = out->size();
  generate(spec, [&](const std::string& b, u64 nl) {
    if (spec.lines > 0 || out->size() - start + b.size() <= spec.bytes) {
      *out += b;
      lines += nl;
      return spec.lines > 0 || out->size() - start < spec.bytes;
    }
    // partial block: keep the full lines that fit
    const u64 room = spec.bytes - (out->size() - start);
    const size_t cut = b.rfind('\n', room ? room - 1 : 0);
    if (room && cut != std::string::npos) {
      out->append(b, 0, cut + 1);
      lines += count_newlines(b.data(), cut + 1);
    }
    return false;
  });
  return lines;
}

u64 gen_text_into(const GenSpec& spec, char* buf, u64 cap, u64* lines_out) {
  LOCUST_CHECK_ARG(spec.lines > 0 || spec.bytes > 0, "set lines or bytes");
  const u64 limit = spec.lines > 0 ? cap : std::min(cap, spec.bytes);
  u64 pos = 0, lines = 0;
  bool full = false;
  generate(spec, [&](const std::string& b, u64 nl) {
    if (pos + b.size() <= limit) {
      std::memcpy(buf + pos, b.data(), b.size());
      pos += b.size();
      lines += nl;
      return spec.lines > 0 || pos < limit;
    }
    const u64 room = limit - pos;
    const size_t cut = room ? b.rfind('\n', room - 1) : std::string::npos;
    if (cut != std::string::npos) {
      std::memcpy(buf + pos, b.data(), cut + 1);
      pos += cut + 1;
      lines += count_newlines(b.data(), cut + 1);
    }
    full = true;
    return false;
  });
  if (full && spec.lines > 0)
    throw Error("gen_text_into: buffer of " + std::to_string(cap) + " B too small for " +
                std::to_string(spec.lines) + " lines");
  if (lines_out) *lines_out = lines;
  return pos;
}

}  // namespace locust
