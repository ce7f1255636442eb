// Host/device string library.
//
// Behavioural twins of the reference's util.cu helpers (/root/reference/MapReduce/src/
// util.cu:3-139), written header-only so device code needs no relocatable device code
// (the reference needed CUDA_SEPARABLE_COMPILATION, CMakeLists.txt:19).  Differences
// from the reference, by design:
//   * d_strcmp honours its length bound (the reference ignores `len`, util.cu:11-20);
//   * d_strcpy_bounded never writes past the destination field (reference B11);
//   * the non-reentrant my_strtok (util.cu:29-52) is dropped: its `static` buffer is
//     unsafe on a GPU and the reference never calls it.
// d_strtok_r has exactly the BSD strtok_r semantics of util.cu:54-89: leading delimiter
// runs are skipped, the token is NUL-terminated in place, *last points past it (or is
// NULL at end of string).
#pragma once

#include "locust/kv.hpp"

namespace locust {

LOCUST_HD inline int d_strlen(const char* s) {
  const char* p = s;
  while (*p) ++p;
  return (int)(p - s);
}

// strcmp on at most `len` bytes.  Returns -1/0/1; compares as *unsigned* bytes, the
// order used by the reference's GPU sort comparator (KeyValue.h:23-28).
LOCUST_HD inline int d_strcmp(const char* a, const char* b, unsigned len = 0xffffffffu) {
  for (unsigned i = 0; i < len; ++i) {
    unsigned char ca = (unsigned char)a[i], cb = (unsigned char)b[i];
    if (ca != cb) return ca < cb ? -1 : 1;
    if (ca == 0) return 0;
  }
  return 0;
}

// Copies at most cap-1 chars and always NUL-terminates (cap >= 1).  Returns the number
// of characters of src that did NOT fit (0 when the copy is complete).
LOCUST_HD inline int d_strcpy_bounded(char* dst, const char* src, int cap) {
  int i = 0;
  for (; i < cap - 1 && src[i]; ++i) dst[i] = src[i];
  dst[i] = 0;
  int dropped = 0;
  while (src[i + dropped]) ++dropped;
  return dropped;
}

LOCUST_HD inline bool d_is_delim(char c, const char* delim) {
  for (const char* d = delim; *d; ++d)
    if (*d == c) return true;
  return false;
}

// BSD strtok_r.  s == NULL continues from *last.
LOCUST_HD inline char* d_strtok_r(char* s, const char* delim, char** last) {
  if (s == nullptr) {
    s = *last;
    if (s == nullptr) return nullptr;
  }
  char c = *s;
  // skip leading delimiters
  while (c != 0 && d_is_delim(c, delim)) c = *++s;
  if (c == 0) {
    *last = nullptr;
    return nullptr;
  }
  char* tok = s;
  for (;;) {
    c = *++s;
    if (c == 0) {
      *last = nullptr;
      return tok;
    }
    if (d_is_delim(c, delim)) {
      *s = 0;
      *last = s + 1;
      return tok;
    }
  }
}

LOCUST_HD inline void d_reverse(char* str, int length) {
  for (int a = 0, b = length - 1; a < b; ++a, --b) {
    char t = str[a];
    str[a] = str[b];
    str[b] = t;
  }
}

// itoa in any base 2..36 (reference my_itoa, util.cu:106-139).  Handles INT_MIN.
LOCUST_HD inline char* d_itoa(int num, char* str, int base) {
  int i = 0;
  bool neg = false;
  unsigned int u = (unsigned int)num;
  if (num == 0) {
    str[0] = '0';
    str[1] = 0;
    return str;
  }
  if (num < 0 && base == 10) {
    neg = true;
    u = 0u - (unsigned int)num;
  }
  while (u != 0) {
    unsigned int rem = u % (unsigned)base;
    str[i++] = (char)(rem > 9 ? (rem - 10) + 'a' : rem + '0');
    u /= (unsigned)base;
  }
  if (neg) str[i++] = '-';
  str[i] = 0;
  d_reverse(str, i);
  return str;
}

// 256-bit delimiter set for the byte-parallel tokenizers: bit c of mask[c>>6].
struct DelimMask {
  uint64_t m[4];
};

inline DelimMask make_delim_mask(const char* delim) {
  DelimMask dm{{0, 0, 0, 0}};
  for (const char* d = delim; *d; ++d) {
    unsigned c = (unsigned char)*d;
    dm.m[c >> 6] |= 1ull << (c & 63);
  }
  return dm;
}

LOCUST_HD inline bool mask_is_delim(const DelimMask& dm, unsigned c) {
  return (dm.m[c >> 6] >> (c & 63)) & 1ull;
}

// The reference tokenizer's delimiter set (main.cu:138,150).
constexpr const char* kDefaultDelims = " ,.-;:'()\"\t";

}  // namespace locust
