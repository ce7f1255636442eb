// Key/value data model.
//
// Reference records (/root/reference/MapReduce/src/KeyValue.h:6-18):
//   KeyValuePair    : char key[100]; char value[100]; int ind;       -> 204 B input record
//   KeyIntValuePair : char key[30]; (2 B pad) int value; int count;  -> 40 B map/reduce record
// Both layouts are reproduced byte-for-byte here (static_asserts below).  KeyIntValuePair
// is a real external format: the kiv stage-1 spill and the --export-kiv result file
// (io.hpp write_spill / write_kiv_results).
//
// Internally the GPU pipeline never sorts 40-B structs with a byte comparator (the
// reference's thrust::sort + KIVComparator, KeyValue.h:20-33).  A key is packed into
// kKeyWords big-endian u64 words, NUL padded:  numeric order of (w0,w1,w2,w3) ==
// unsigned-byte lexicographic order of the C string, and shorter keys sort first exactly
// like strcmp.  Keys are stored structure-of-arrays (one u64 array per word) so radix
// passes and boundary compares read coalesced 8-B words.
#pragma once

#include <cstddef>
#include <cstdint>
#include <cstring>

#ifndef LOCUST_HD
#if defined(__HIPCC__)
#define LOCUST_HD __host__ __device__
#else
#define LOCUST_HD
#endif
#endif

namespace locust {

constexpr int kKeyWords = 4;                 // packed key width in u64 words
constexpr int kKeyBytes = 8 * kKeyWords;     // 32 bytes
constexpr int kRefKeyField = 30;             // KeyIntValuePair::key[30]
constexpr int kMaxKeyLen = kRefKeyField - 1; // 29 chars + NUL fit the 40-B record
constexpr int kRefLineField = 100;           // KeyValuePair::value[100]

struct KeyValuePair {  // reference input record (KeyValue.h:6-11)
  char key[100];
  char value[100];
  int ind;
};

struct KeyIntValuePair {  // reference map/reduce record (KeyValue.h:13-18)
  char key[kRefKeyField];
  int value;
  int count;
};

static_assert(sizeof(KeyValuePair) == 204, "KeyValuePair must stay 204 B");
static_assert(offsetof(KeyValuePair, ind) == 200, "KeyValuePair.ind at 200");
static_assert(sizeof(KeyIntValuePair) == 40, "KeyIntValuePair must stay 40 B");
static_assert(offsetof(KeyIntValuePair, value) == 32, "KeyIntValuePair.value at 32");
static_assert(offsetof(KeyIntValuePair, count) == 36, "KeyIntValuePair.count at 36");

// One packed key (AoS form; used on the host and for shuffle records).
struct PackedKey {
  uint64_t w[kKeyWords];
};

// Shuffle / combine record: packed key plus an occurrence count (40 B, 8-B aligned).
struct KeyCount {
  uint64_t w[kKeyWords];
  uint64_t count;
};
static_assert(sizeof(KeyCount) == 40, "KeyCount must stay 40 B");

// Pack up to kKeyBytes bytes of s[0..len) into big-endian words.
LOCUST_HD inline void pack_key(const char* s, int len, uint64_t* w) {
  for (int j = 0; j < kKeyWords; ++j) w[j] = 0;
  if (len > kKeyBytes) len = kKeyBytes;
  for (int i = 0; i < len; ++i)
    w[i >> 3] |= (uint64_t)(unsigned char)s[i] << (56 - 8 * (i & 7));
}

// Unpack into a NUL-terminated string; returns its length.  `out` needs kKeyBytes+1 bytes.
LOCUST_HD inline int unpack_key(const uint64_t* w, char* out) {
  int n = 0;
  for (int i = 0; i < kKeyBytes; ++i) {
    char c = (char)(w[i >> 3] >> (56 - 8 * (i & 7)));
    if (c == 0) break;
    out[n++] = c;
  }
  out[n] = 0;
  return n;
}

// Compact result record (the host drain format of the ordered kernels and the shuffle's
// shared output): 8-B words
//   [count << kCompactCountShift | nw] [key word 0] ... [key word nw - 1]
// where nw (1-4) counts the key's words up to its last non-zero one (the rest are NUL
// padding).  English and synthetic keys are mostly <= 8 or <= 16 bytes: 16-24 B per entry
// instead of 40 B across PCIe.  The 40-B KeyIntValuePair stays the kiv file format.
constexpr int kCompactCountShift = 8;
constexpr int kCompactMaxWords = 1 + kKeyWords;
LOCUST_HD inline uint32_t key_words_used(const uint64_t* w) {
  return w[3] ? 4u : w[2] ? 3u : w[1] ? 2u : 1u;
}
LOCUST_HD inline uint32_t compact_nw(uint64_t header) { return (uint32_t)(header & 7u); }
LOCUST_HD inline uint64_t compact_header(uint64_t count, uint32_t nw) {
  return (count << kCompactCountShift) | nw;
}
// Decodes the record at p; returns its length in words.
LOCUST_HD inline uint32_t decode_compact(const uint64_t* p, PackedKey* key, uint64_t* count) {
  const uint32_t nw = compact_nw(p[0]);
  *count = p[0] >> kCompactCountShift;
  for (int j = 0; j < kKeyWords; ++j) key->w[j] = (uint32_t)j < nw ? p[1 + j] : 0ull;
  return 1 + nw;
}

LOCUST_HD inline int key_compare(const uint64_t* a, const uint64_t* b) {
  for (int j = 0; j < kKeyWords; ++j) {
    if (a[j] != b[j]) return a[j] < b[j] ? -1 : 1;
  }
  return 0;
}

LOCUST_HD inline bool key_less(const PackedKey& a, const PackedKey& b) {
  return key_compare(a.w, b.w) < 0;
}

}  // namespace locust
