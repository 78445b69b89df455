// keys.hpp — the word-key contract shared by host (CPU oracle, merge, formatter)
// and device (map / reduce kernels).  Compiled by hipcc and by g++.
//
// Reference parity: the reference identifies a word by a byte-at-a-time *prefix*
// test (`compare`, /root/reference/main.cu:57-67) over NUL-terminated 30-byte
// buffers (main.cu:16-22).  Here a word is identified by a packed 128-bit key,
// so every equality test is two 64-bit integer compares:
//
//   k0 = the first min(len, 8) bytes, little-endian packed, zero-padded
//   k1 = len                                   len <= 8   SHORT  (exact)
//        bytes [8, len) packed | len << 56     9..15      MEDIUM (exact)
//        TAG | hash62(bytes [8, len), len)     len >= 16  LONG   (hashed)
//
// Words of <= 15 bytes — all but a vanishing fraction of natural text — are
// keyed exactly with no hashing at all.  LONG keys can collide (same first 8
// bytes, same 62-bit tail hash), so they never meet by key alone: every LONG
// token reaches the key table as its own record and is merged only after a
// byte comparison with the table's stored copy of the word (reduce.hip
// wc_long_merge, merge.hip wc_mrow_insert); two colliding words keep two slots.
// k1 is never 0 (empty slot) and never ~0 (PENDING: bit 62 of a LONG k1 is 0).
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

// LONG-word tail hash: word-wise FNV-1a-64 over the 8-byte little-endian
// chunks that follow k0 (last chunk zero-padded), folded with the length and
// finalised with fmix64.  Chunk-at-a-time so the map kernel hashes straight
// from registers (one fold per 8 bytes instead of one per byte).  `mask` keeps
// all 62 bits in production; the collision tests truncate it (Options::k1_hash_bits).
constexpr uint32_t KEY_INLINE_MAX = 15;  // longest word keyed exactly (SHORT / MEDIUM)
WC_HD uint64_t tail_fold(uint64_t h, uint64_t chunk) { return (h ^ chunk) * FNV_PRIME; }
WC_HD uint64_t long_k1(uint64_t len, uint64_t h, uint64_t mask = K1_HASH_MASK) {
  return K1_TAG | (fmix64(h ^ len) & mask);
}
WC_HD uint64_t medium_k1(uint64_t tail, uint64_t len) { return tail | (len << 56); }  // tail = bytes [8, len)
WC_HD uint64_t k1_hash_mask(uint32_t bits) { return bits >= 62 || bits == 0 ? K1_HASH_MASK : ((1ull << bits) - 1); }

// Placement hash of the packed key (32 bits, four 32-bit multiplies — the map
// computes it once per token; a 24-bit-multiply variant measured no faster in
// the map and spread keys worse: reduce +25 % at 1M words): the middle words are pre-mixed by odd-constant
// multiplies, then lowbias32.  Bits [0, log2 B) select the shuffle / table
// bucket, bits [20, 29) the map combiner group, the high bits the merge owner;
// the reduce slice group is taken from a multiplied copy so it stays spread
// when the bucket bits are many.
WC_HD uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  return x ^ (x >> 16);
}
WC_HD uint32_t place_hash(uint64_t k0, uint64_t k1) {
  const uint32_t a = (uint32_t)k0, b = (uint32_t)(k0 >> 32), c = (uint32_t)k1 ^ (uint32_t)(k1 >> 32);
  return mix32(a ^ (b * 0x9E3779B1u) ^ (c * 0x85EBCA77u));
}

// Length of a short word implied by its k0: bytes up to the highest nonzero one
// (0 for k0 = 0).  Equals the length iff the word's last byte is not 0x00.
WC_HD uint32_t implied_len(uint64_t k0) { return k0 ? (71u - (uint32_t)__builtin_clzll(k0)) >> 3 : 0u; }
// k1 of a 16-byte single-occurrence record (kernels.hpp Rec16): t = the word's
// bytes [8, 12) zero-padded, 0 for a word of <= 8 bytes; the length is implied
// by the highest nonzero byte (the record holds words whose last byte is not 0).
WC_HD uint64_t rec16_k1(uint64_t k0, uint32_t t) {
  return t ? medium_k1(t, 9u + ((31u - (uint32_t)__builtin_clz(t)) >> 3)) : implied_len(k0);
}

// Merge owner of a key among W ranks: the high bits of its placement hash
// (bucket bits are the low ones), dist/merge.cpp and its Python mirror
// (cuda_mapreduce_amd/parallel/dist.py _owner).
WC_HD uint32_t owner_of(uint32_t ph, uint32_t W) { return (uint32_t)(((uint64_t)ph * W) >> 32); }

// Nested: the bucket under 2B buckets is b or b + B for bucket b under B.
WC_HD uint32_t bucket_of(uint32_t ph, uint32_t log2_buckets) { return ph & ((1u << log2_buckets) - 1u); }

// Host helper: key of an explicit byte string.
WC_HD void key_of(const uint8_t* w, uint64_t len, uint64_t* k0, uint64_t* k1, uint64_t mask = K1_HASH_MASK) {
  uint64_t a = 0, h = FNV_OFFSET, chunk = 0, first_tail = 0;
  for (uint64_t i = 0; i < len; ++i) {
    if (i < 8) {
      a |= (uint64_t)w[i] << (8 * i);
    } else {
      chunk |= (uint64_t)w[i] << (8 * (i & 7));
      if ((i & 7) == 7) {
        if (i == 15) first_tail = chunk;
        h = tail_fold(h, chunk);
        chunk = 0;
      }
    }
  }
  if (len > 8 && len <= KEY_INLINE_MAX) first_tail = chunk;
  if (len > 8 && (len & 7)) h = tail_fold(h, chunk);
  *k0 = a;
  *k1 = len <= 8 ? len : (len <= KEY_INLINE_MAX ? medium_k1(first_tail, len) : long_k1(len, h, mask));
}

WC_HD bool key_is_short(uint64_t k1) { return k1 <= 8; }
WC_HD bool key_is_hashed(uint64_t k1) { return (k1 >> 63) != 0; }  // LONG: bytes live in the key arena
WC_HD uint32_t inline_len(uint64_t k1) { return k1 <= 8 ? (uint32_t)k1 : (uint32_t)(k1 >> 56); }
// Bytes of an inline (SHORT / MEDIUM) key: out must hold 15 bytes; returns the length.
WC_HD uint32_t inline_bytes(uint64_t k0, uint64_t k1, uint8_t* out) {
  const uint32_t len = inline_len(k1);
  for (uint32_t i = 0; i < len; ++i) out[i] = (uint8_t)((i < 8 ? k0 >> (8 * i) : k1 >> (8 * (i - 8))) & 0xFF);
  return len;
}

// First-occurrence order (sort.hip): log-scale value bin of a first offset k —
// k itself below 2^M, else 2^M bins per octave (monotone) — over FO_LOGBINS
// bins, and the most mantissa bits M that keep every key < 2^key_bits inside
// them.  The reducer histograms its keys with the same function.
constexpr uint32_t FO_LOGBINS = 16384;
WC_HD uint32_t fo_logbin(uint64_t k, uint32_t M) {
  if (k < (1ull << M)) return (uint32_t)k;
  const uint32_t e = 63u - (uint32_t)__builtin_clzll(k);  // >= M
  const uint32_t lb = ((e - M + 1u) << M) | (uint32_t)((k >> (e - M)) & ((1ull << M) - 1));
  return lb < FO_LOGBINS - 1 ? lb : FO_LOGBINS - 1;
}
WC_HD uint32_t fo_mbits(uint32_t key_bits) {
  uint32_t M = 12;
  while (M > 4 && ((uint64_t)(key_bits > M ? key_bits - M + 1 : 1) << M) > (uint64_t)FO_LOGBINS) --M;
  return M;
}

}  // namespace wc
