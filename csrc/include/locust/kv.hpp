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
// shared output): a run of 8-B words.  kb = the key's bytes up to its
// last non-zero one (1-32; the rest of the packed key is NUL padding).
//   short (count < 2^24): word 0 = [key bytes 0-3 : 32][count : 24][0 : 1][kb : 6][0 : 1]
//                         then ceil((kb - 4) / 8) words of key bytes 4, 5, ... (big-endian)
//   long:                 word 0 = [count : 56][0 : 1][kb : 6][1 : 1]
//                         then ceil(kb / 8) packed key words
// (bit 0 first).  English and synthetic keys of 5-12 bytes take 16 B instead of 40 B, and
// keys of up to 4 bytes one word.  The 40-B KeyIntValuePair stays the kiv file format.
constexpr uint64_t kCompactShortMax = (1ull << 24) - 1;
constexpr int kCompactMaxWords = 1 + kKeyWords;
LOCUST_HD inline uint32_t key_words_used(const uint64_t* w) {
  return w[3] ? 4u : w[2] ? 3u : w[1] ? 2u : 1u;
}
// Bytes of a packed key up to its last non-zero one (0 for the empty key).
LOCUST_HD inline uint32_t key_bytes_used(const uint64_t* w) {
  const uint32_t nw = key_words_used(w);
  const uint64_t last = nw == 4 ? w[3] : nw == 3 ? w[2] : nw == 2 ? w[1] : w[0];
  return last ? 8u * nw - ((uint32_t)__builtin_ctzll(last) >> 3) : 0u;
}
LOCUST_HD inline uint32_t compact_words_for(uint32_t kb, uint64_t count) {
  return count <= kCompactShortMax ? 1u + (kb > 4u ? (kb + 3u) >> 3 : 0u) : 1u + ((kb + 7u) >> 3);
}
LOCUST_HD inline uint32_t compact_words(const uint64_t* w, uint64_t count) {
  return compact_words_for(key_bytes_used(w), count);
}
// Words of the record starting with header word h.
LOCUST_HD inline uint32_t compact_record_words(uint64_t h) {
  const uint32_t kb = (uint32_t)(h >> 1) & 63u;
  return (h & 1u) ? 1u + ((kb + 7u) >> 3) : 1u + (kb > 4u ? (kb + 3u) >> 3 : 0u);
}
// All words of a key's record into o[0..kCompactMaxWords) (static indices: callers keep o
// in registers); returns how many of them the record uses.
LOCUST_HD inline uint32_t compact_record(const uint64_t* w, uint64_t count, uint64_t* o) {
  const uint32_t kb = key_bytes_used(w);
  if (count <= kCompactShortMax) {
    o[0] = ((w[0] >> 32) << 32) | (count << 8) | ((uint64_t)kb << 1);
    o[1] = (w[0] << 32) | (w[1] >> 32);
    o[2] = (w[1] << 32) | (w[2] >> 32);
    o[3] = (w[2] << 32) | (w[3] >> 32);
    o[4] = w[3] << 32;
  } else {
    o[0] = (count << 8) | ((uint64_t)kb << 1) | 1u;
    o[1] = w[0];
    o[2] = w[1];
    o[3] = w[2];
    o[4] = w[3];
  }
  return compact_words_for(kb, count);
}
// Decodes the record at p; returns its length in words.
LOCUST_HD inline uint32_t decode_compact(const uint64_t* p, PackedKey* key, uint64_t* count) {
  const uint64_t h = p[0];
  const uint32_t n = compact_record_words(h);
  if (h & 1u) {
    *count = h >> 8;
    for (uint32_t j = 0; j < (uint32_t)kKeyWords; ++j) key->w[j] = j + 1 < n ? p[1 + j] : 0ull;
  } else {
    *count = (h >> 8) & kCompactShortMax;
    // key word j = [bytes 8j..8j+3 : the previous word's low half][bytes 8j+4.. : this
    // extra word's high half]
    uint64_t hi = h >> 32;
    for (uint32_t j = 0; j < (uint32_t)kKeyWords; ++j) {
      const uint64_t e = j + 1 < n ? p[1 + j] : 0ull;
      key->w[j] = (hi << 32) | (e >> 32);
      hi = e & 0xFFFFFFFFull;
    }
  }
  return n;
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
