// keys.hpp — the word-key contract shared by host (CPU oracle, merge, formatter)
// and device (map / reduce kernels).  Compiled by hipcc and by g++.
//
// Reference parity: the reference identifies a word by a byte-at-a-time *prefix*
// test (`compare`, /root/reference/main.cu:57-67) over NUL-terminated 30-byte
// buffers (main.cu:16-22).  Here a word is identified EXACTLY by a packed
// 128-bit key so every equality test is two 64-bit integer compares:
//
//   k0 = the first min(len, 8) bytes, little-endian packed, zero-padded
//   k1 = len                                   when len <= 8  (exact, no hash)
//        TAG | fnv1a64(word) & HASH_MASK       when len >  8
//
// Words of <= 8 bytes (the vast majority of natural text) are therefore keyed
// with no hashing at all; longer words collide only if they share their first
// 8 bytes AND a 62-bit FNV-1a tail hash.  k1 is never 0 (0 marks an empty
// slot) and never ~0 (PENDING marks a slot being claimed).
//
// Delimiters are exactly the reference's set {' ', '\r', '\n'} (main.cu:188);
// TAB and every other byte, NUL included, are word bytes.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define WC_HD __host__ __device__ __forceinline__
#else
#define WC_HD inline
#endif

namespace wc {

constexpr uint64_t FNV_OFFSET = 0xcbf29ce484222325ull;
constexpr uint64_t FNV_PRIME = 0x100000001b3ull;
constexpr uint64_t K1_TAG = 1ull << 63;
constexpr uint64_t K1_HASH_MASK = (1ull << 62) - 1;
constexpr uint64_t K1_EMPTY = 0;
constexpr uint64_t K1_PENDING = ~0ull;

WC_HD bool is_delim(uint32_t c) { return c == 0x20u || c == 0x0Du || c == 0x0Au; }

// Per-byte "is delimiter" for 8 packed bytes -> 8-bit mask (exact SWAR zero test).
WC_HD uint64_t delim_mask8(uint64_t x) {
  constexpr uint64_t ONES = 0x0101010101010101ull, LOW7 = 0x7F7F7F7F7F7F7F7Full;
  auto zero_bytes = [](uint64_t y) { return ~(((y & LOW7) + LOW7) | y) & 0x8080808080808080ull; };
  const uint64_t m = zero_bytes(x ^ (0x20 * ONES)) | zero_bytes(x ^ (0x0D * ONES)) | zero_bytes(x ^ (0x0A * ONES));
  return ((m >> 7) * 0x0102040810204080ull) >> 56;
}

WC_HD uint64_t fnv1a_step(uint64_t h, uint32_t byte) { return (h ^ (uint64_t)(byte & 0xFFu)) * FNV_PRIME; }

// murmur3 fmix64 finalizer: FNV's low bits are weak, placement needs all 64.
WC_HD uint64_t fmix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return k;
}

// Long-word tail hash: word-wise FNV-1a-64 over the 8-byte little-endian
// chunks that follow k0 (last chunk zero-padded), folded with the length and
// finalised with fmix64.  Chunk-at-a-time so the map kernel hashes straight
// from registers (one fold per 8 bytes instead of one per byte).
WC_HD uint64_t tail_fold(uint64_t h, uint64_t chunk) { return (h ^ chunk) * FNV_PRIME; }
WC_HD uint64_t make_k1(uint64_t len, uint64_t h) {
  return len <= 8 ? len : (K1_TAG | (fmix64(h ^ len) & K1_HASH_MASK));
}

// Placement hash of the packed key: (k0 ^ rotl(k1, 56)) through a two-multiply
// xor-shift mixer (splitmix64-style finaliser).  Two full 64-bit multiplies —
// the map computes it once per token, so it is kept cheaper than a byte-wise
// FNV.  Bits [2, 2+log2 B) select the shuffle / table bucket (they live inside
// the 32-bit LDS tag, so a flush recovers the bucket without rehashing), bits
// [32, ..) the slot group inside a table, the top bits the merge owner rank.
WC_HD uint64_t place_hash(uint64_t k0, uint64_t k1) {
  uint64_t h = (k0 ^ ((k1 << 56) | (k1 >> 8))) * 0x9E3779B97F4A7C15ull;
  h ^= h >> 29;
  h *= 0xBF58476D1CE4E5B9ull;
  return h ^ (h >> 32);
}

// Nested: the bucket under 2B buckets is b or b + B for bucket b under B.
WC_HD uint32_t bucket_of(uint64_t ph, uint32_t log2_buckets) {
  return (uint32_t)(ph >> 2) & ((1u << log2_buckets) - 1u);
}

// Host helper: key of an explicit byte string.
WC_HD void key_of(const uint8_t* w, uint64_t len, uint64_t* k0, uint64_t* k1) {
  uint64_t a = 0, h = FNV_OFFSET, chunk = 0;
  for (uint64_t i = 0; i < len; ++i) {
    if (i < 8) {
      a |= (uint64_t)w[i] << (8 * i);
    } else {
      chunk |= (uint64_t)w[i] << (8 * (i & 7));
      if ((i & 7) == 7) {
        h = tail_fold(h, chunk);
        chunk = 0;
      }
    }
  }
  if (len > 8 && (len & 7)) h = tail_fold(h, chunk);
  *k0 = a;
  *k1 = make_k1(len, h);
}

// Short words (len <= 8) are recoverable from the key alone.
WC_HD bool key_is_short(uint64_t k1) { return k1 <= 8; }

}  // namespace wc
