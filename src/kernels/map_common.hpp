// map_common.hpp — building blocks of the map kernel (map.hip): text loads,
// delimiter masks, word keys from an LDS text buffer, the shuffle-record write
// and the phase clock of the diagnostic build.
#pragma once
#include "kernels.hpp"
#include "keys.hpp"

namespace wc {
namespace dev {

constexpr int MAP_WAVES = MAP_THREADS / 64;
#ifndef WC_MAP_LIST
#define WC_MAP_LIST 512
#endif
constexpr int MAP_LIST = WC_MAP_LIST;            // token-list entries per wave per round (u16)
constexpr uint32_t MAP_LONG = 31u;               // list length field: >= 31 bytes or past the lane window
static_assert(64 * MAP_BPL <= 2048, "list entries hold 11-bit unit-relative positions");

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));

// Bytes [p, p+8) and [p+8, p+16) of an 8-byte-aligned LDS text buffer from
// ALIGNED reads and funnel shifts (an unaligned 16-byte read stalls the LDS
// pipe: SQ_LDS_UNALIGNED_STALL was a third of its busy cycles).  The buffer
// must be readable 24 bytes past p & ~7.
#ifndef WC_WIN_ALIGNBYTE
#define WC_WIN_ALIGNBYTE 1
#endif
__device__ __forceinline__ void window16(const uint8_t* buf, uint32_t p, uint64_t& w0, uint64_t& w1) {
#if WC_WIN_ALIGNBYTE
  // five dwords from the 4-byte-aligned address below p (two ds_read2_b32 +
  // one ds_read_b32: no unaligned LDS access) and four v_alignbyte_b32 funnels
  // by p & 3 — 5 VALU per window instead of 11 for the 8-byte-aligned
  // 64-bit-shift form (which needs a dword select for shifts >= 4)
  const uint32_t* q = reinterpret_cast<const uint32_t*>(buf + (p & ~3u));
  const uint32_t d0 = q[0], d1 = q[1], d2 = q[2], d3 = q[3], d4 = q[4];
  const uint32_t sh = p;  // v_alignbyte_b32 reads only bits [1:0] of the byte shift
  const uint32_t a = __builtin_amdgcn_alignbyte(d1, d0, sh), b = __builtin_amdgcn_alignbyte(d2, d1, sh);
  const uint32_t c = __builtin_amdgcn_alignbyte(d3, d2, sh), d = __builtin_amdgcn_alignbyte(d4, d3, sh);
  w0 = (uint64_t)a | ((uint64_t)b << 32);
  w1 = (uint64_t)c | ((uint64_t)d << 32);
#else
  const uint64_t* q = reinterpret_cast<const uint64_t*>(buf + (p & ~7u));
  const uint64_t d0 = q[0], d1 = q[1], d2 = q[2];
  const uint32_t sh = (p & 7u) * 8u;
  // (x << 1) << (63 - sh) == x << (64 - sh) without the undefined shift by 64 at sh = 0
  w0 = (d0 >> sh) | ((d1 << 1) << (63 - sh));
  w1 = (d1 >> sh) | ((d2 << 1) << (63 - sh));
#endif
}

// Bytes [p, p+8) of the LDS text buffer: three dwords from the 4-byte-aligned
// address below p and two v_alignbyte_b32 funnels.
__device__ __forceinline__ uint64_t window8(const uint8_t* buf, uint32_t p) {
  const uint32_t* q = reinterpret_cast<const uint32_t*>(buf + (p & ~3u));
  const uint32_t d0 = q[0], d1 = q[1], d2 = q[2];
  const uint32_t sh = p;  // bits [1:0] only (v_alignbyte_b32)
  return (uint64_t)__builtin_amdgcn_alignbyte(d1, d0, sh) | ((uint64_t)__builtin_amdgcn_alignbyte(d2, d1, sh) << 32);
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Per-byte delimiter bits of a dword (bit i = byte i is ' ', '\r' or '\n'):
// exact SWAR zero-byte tests (no false positives), 32-bit operations only.
__device__ __forceinline__ uint32_t delim_bits4(uint32_t x) {
  auto zb = [](uint32_t y) { return ~(((y & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | y) & 0x80808080u; };
  const uint32_t m = zb(x ^ 0x20202020u) | zb(x ^ 0x0D0D0D0Du) | zb(x ^ 0x0A0A0A0Au);
  return (((m >> 7) * 0x00204081u) >> 21) & 0xFu;
}

// v_ffbl_b32 as the hardware defines it: index of the lowest set bit, all ones
// for 0.  __builtin_ctz is zero-undefined, so it lowers to the bare v_ffbl_b32
// (no select for 0); callers keep only the low 5 bits of the result or shift
// it out of a 16-bit entry, which is the same for 31 and all ones.  (An inline
// asm v_ffbl made the waitcnt pass drain LDS before every use: an lgkmcnt(0)
// per token-list iteration.)
__device__ __forceinline__ uint32_t ffbl_raw(uint32_t x) { return (uint32_t)__builtin_ctz(x); }

// Wave-wide inclusive prefix sum (wave64) by DPP: four in-row shifts (16-lane
// rows), then row 15 / row 31 broadcasts — six v_add_u32_dpp, no LDS, no
// ballots.  The map scans its two token-class counts PACKED in one word
// (class counts <= 32 per lane, <= 2048 per wave: no carry between halves).
// (The ballot form below costs five ballots + mbcnt pairs per value: ~4x the
// VALU cycles at two values per unit, ~5 % of the map's VALU.)
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true);  // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, true);  // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, true);  // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, true);  // row_shr:8
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false); // row_bcast:15 -> rows 1, 3
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false); // row_bcast:31 -> rows 2, 3
  return x;
}

// Wave-wide exclusive prefix sum of a small per-lane value v < 32 (bit
// decomposition over ballots: no cross-lane shuffles); total = wave sum.
__device__ __forceinline__ uint32_t wave_excl_small(uint32_t v, uint32_t& total) {
  uint32_t ex = 0, tot = 0;
#pragma unroll
  for (int b = 0; b < 5; ++b) {
    const uint64_t m = __ballot((v >> b) & 1u);
    const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    ex += below << b;
    tot += (uint32_t)__popcll(m) << b;
  }
  total = tot;
  return ex;
}

// Phase clock for the diagnostic build (ST = true): accumulates s_memtime
// deltas per wave; the real kernel (ST = false) compiles it away.
template <bool ST>
struct PhaseClock {
  unsigned long long* acc = nullptr;  // block accumulators in LDS (lane 0 of each wave adds)
  uint64_t t = 0;
  __device__ __forceinline__ void start(unsigned long long* lds_acc) {
    if (ST) {
      acc = lds_acc;
      t = __builtin_amdgcn_s_memtime();
    }
  }
  __device__ __forceinline__ void lap(int phase) {
    if (ST) {
      const uint64_t n = __builtin_amdgcn_s_memtime();
      if (__lane_id() == 0) atomicAdd(&acc[phase], (unsigned long long)(n - t));
      t = n;
    }
  }
};

// Profiling builds only (-DWC_EMIT_ABLATE=1, results NOT valid): no record
// stores (staged or direct; the cursor atomics stay).
#ifndef WC_EMIT_ABLATE
#define WC_EMIT_ABLATE 0
#endif

// Record format of a key with count cnt: 16-byte Rec16 (one occurrence of a
// word of <= 12 bytes whose last byte is nonzero, so keys.hpp implied_len of
// k0 / of the tail word gives the length back — inline keys have zero bytes
// past the length) or 24-byte Rec.
__device__ __forceinline__ bool rec16_fits(uint64_t k0, uint64_t k1, uint64_t cnt) {
  if (cnt != 1) return false;
  if (k1 - 1 < 8) return ((k0 >> (8 * (k1 - 1))) & 0xFFu) != 0;
  const uint64_t len = k1 >> 56;  // MEDIUM: 9..15; LONG: >= 0x80
  return len - 9 < 4 && ((k1 >> (8 * (len - 9))) & 0xFFu) != 0;
}

// rec16_fits for one occurrence of an inline word of known length n (k1 its
// MEDIUM key word when n > 8): n <= 8 with k0 >> 8 (n - 1) != 0, or 9..12
// with the tail's byte n - 9 nonzero.  Shifts are masked, so n = 0 of an
// empty lane is harmless.
__device__ __forceinline__ bool rec16_inline(uint64_t k0, uint64_t k1, uint32_t n) {
  if (n - 1u < 8u) return (k0 >> ((8u * n - 8u) & 63u)) != 0;
  return n - 9u < 4u && ((uint32_t)k1 >> ((8u * n - 72u) & 31u)) != 0;
}

__device__ __forceinline__ Rec16 make_rec16(uint64_t k0, uint64_t k1, uint32_t off) {
  return Rec16{(uint32_t)k0, (uint32_t)(k0 >> 32), k1 > 8 ? (uint32_t)k1 : 0u, off};
}

// This block's record sub-regions: bucket b's run starts at (b * sub) records
// from the block base (b * sub < 2^25: 32-bit index math).  lim: the last
// record index of the block's area (nb * sub - 1).
struct RecOut {
  Rec16* b16;
  Rec* b24;
  uint32_t sub, lim;
};
__device__ __forceinline__ RecOut rec_out(const MapArgs& a) {
  const uint64_t first = ((uint64_t)blockIdx.x << a.log2_rec_buckets) * a.rec.subcap;
  return RecOut{a.rec.recs16 + first, a.rec.recs + first, a.rec.subcap,
                (a.rec.subcap << a.log2_rec_buckets) - 1u};
}

// Record cursors in LDS: cur[b] (Rec16) and cur[MAX_REC_BUCKETS + b] (Rec)
// start at b * sub, so a cursor atomic returns the record's index in the
// block's area directly (no select of a packed half, no multiply).  A bucket
// that outgrows its sub-region writes on into the next bucket's — the block
// end sees it (cursor - b * sub > sub), raises FLAG_REGION_OVF and the host
// re-runs the pass, discarding its records; indices are clamped to the block's
// area, so nothing is written outside it.
__device__ __forceinline__ void cursors_init(uint32_t* cur, uint32_t* lcur, uint32_t nb, uint32_t sub) {
  for (uint32_t b = threadIdx.x; b < nb; b += blockDim.x) {
    cur[b] = b * sub;
    cur[MAX_REC_BUCKETS + b] = b * sub;
  }
  if (lcur)
    for (uint32_t w = threadIdx.x; w < (nb + 1) / 2; w += blockDim.x) lcur[w] = 0;
}

// Store one record at area index idx.  The block's store bases are
// wave-uniform (SGPRs) and a record's byte offset fits 32 bits, so the stores
// take the SGPR-base + 32-bit VGPR-offset form.
__device__ __forceinline__ void put_rec16(const RecOut& o, uint32_t idx, const Rec16& r) {
  if (WC_EMIT_ABLATE) return;
  idx = min(idx, o.lim);
  *reinterpret_cast<Rec16*>(reinterpret_cast<uint8_t*>(o.b16) + idx * (uint32_t)sizeof(Rec16)) = r;
}
__device__ __forceinline__ void put_rec24(const RecOut& o, uint32_t idx, uint64_t k0, uint64_t k1, uint64_t cnt,
                                          uint32_t off) {
  if (WC_EMIT_ABLATE) return;
  idx = min(idx, o.lim);
  Rec r;
  r.k0 = k0;
  r.k1 = k1;
  r.co = (cnt << 32) | off;
  *reinterpret_cast<Rec*>(reinterpret_cast<uint8_t*>(o.b24) + __umul24(idx, (uint32_t)sizeof(Rec))) = r;
}

// LONG-word record cursors: 16-bit counts, two buckets per LDS word (bucket b
// in half b & 1 of word b >> 1), counting down from the top of the 24-byte
// sub-region.  A count reaching the sub-region size raises the block's
// overflow word (ovf) at once — a count past 0xFFFF would carry into its
// neighbour — and the block end checks 24-byte + LONG counts against it.
// The deferred-LONG pass calls this directly (every key there is hashed): no
// Rec16 / 24-byte paths in the unit loop's register budget.
__device__ __forceinline__ void emit_long(uint32_t* lcur, uint32_t* ovf, const RecOut& o, uint32_t b, uint64_t k0,
                                          uint64_t k1, uint64_t cnt, uint32_t off) {
  const uint32_t sh = 16u * (b & 1u);
  const uint32_t c = (atomicAdd(&lcur[b >> 1], 1u << sh) >> sh) & 0xFFFFu;
  if (c >= o.sub) *ovf = 1u;
  put_rec24(o, b * o.sub + (o.sub - 1u) - min(c, o.sub - 1u), k0, k1, cnt, off);
}

// Append one record (key, count, first offset) to bucket b's sub-region (the
// hot-table flush: any kind).  LD: LONG records top-down (emit_long).
template <bool LD>
__device__ __forceinline__ void emit_record(uint32_t* cur, uint32_t* lcur, uint32_t* ovf, const RecOut& o, uint32_t b,
                                            uint64_t k0, uint64_t k1, uint64_t cnt, uint32_t off) {
  if (rec16_fits(k0, k1, cnt)) put_rec16(o, atomicAdd(&cur[b], 1u), make_rec16(k0, k1, off));
  else if (LD && key_is_hashed(k1)) emit_long(lcur, ovf, o, b, k0, k1, cnt, off);
  else put_rec24(o, atomicAdd(&cur[MAX_REC_BUCKETS + b], 1u), k0, k1, cnt, off);
}

// Two single-occurrence records of one lane (either may be absent; n1 / n2:
// the words' lengths, x1 / y1 their key words): both cursor atomics are
// issued before either store waits for its index.
__device__ __forceinline__ void emit_two(uint32_t* cur, const RecOut& o, bool d1, uint32_t b1, uint64_t x0,
                                         uint64_t x1, uint32_t o1, uint32_t n1, bool d2, uint32_t b2, uint64_t y0,
                                         uint64_t y1, uint32_t o2, uint32_t n2) {
  const bool s1 = rec16_inline(x0, x1, n1), s2 = rec16_inline(y0, y1, n2);
  uint32_t p1 = 0, p2 = 0;
  if (d1) p1 = atomicAdd(&cur[(s1 ? 0u : (uint32_t)MAX_REC_BUCKETS) + b1], 1u);
  if (d2) p2 = atomicAdd(&cur[(s2 ? 0u : (uint32_t)MAX_REC_BUCKETS) + b2], 1u);
  if (d1) {
    if (s1) put_rec16(o, p1, make_rec16(x0, x1, o1));
    else put_rec24(o, p1, x0, x1, 1, o1);
  }
  if (d2) {
    if (s2) put_rec16(o, p2, make_rec16(y0, y1, o2));
    else put_rec24(o, p2, y0, y1, 1, o2);
  }
}

// emit_two for words of 1..7 bytes (k1 = the length): a Rec16 (tail word 0)
// unless the word's last byte is 0x00 — one 64-bit shift and compare per word.
__device__ __forceinline__ void emit_two_short(uint32_t* cur, const RecOut& o, bool d1, uint32_t b1, uint64_t x0,
                                               uint32_t o1, uint32_t n1, bool d2, uint32_t b2, uint64_t y0,
                                               uint32_t o2, uint32_t n2) {
  const bool s1 = (x0 >> ((8u * n1 - 8u) & 63u)) != 0, s2 = (y0 >> ((8u * n2 - 8u) & 63u)) != 0;
  uint32_t p1 = 0, p2 = 0;
  if (d1) p1 = atomicAdd(&cur[(s1 ? 0u : (uint32_t)MAX_REC_BUCKETS) + b1], 1u);
  if (d2) p2 = atomicAdd(&cur[(s2 ? 0u : (uint32_t)MAX_REC_BUCKETS) + b2], 1u);
  if (d1) {
    if (s1) put_rec16(o, p1, Rec16{(uint32_t)x0, (uint32_t)(x0 >> 32), 0u, o1});
    else put_rec24(o, p1, x0, n1, 1, o1);
  }
  if (d2) {
    if (s2) put_rec16(o, p2, Rec16{(uint32_t)y0, (uint32_t)(y0 >> 32), 0u, o2});
    else put_rec24(o, p2, y0, n2, 1, o2);
  }
}

// Key of a LONG token (>= 16 bytes) of known length 16..30 from its LDS
// windows: k0 = the first 8 bytes, then the tail's 8-byte chunks folded
// (keys.hpp key_of: full chunks, then the zero-padded partial one).  Two
// window16 reads instead of a byte loop.
__device__ __forceinline__ void key_long_known(const uint8_t* buf, uint32_t p, uint32_t len, uint64_t k1_mask,
                                               uint64_t& k0, uint64_t& k1) {
  uint64_t w0, w1, w2, w3;
  window16(buf, p, w0, w1);
  window16(buf, p + 16, w2, w3);
  k0 = w0;
  uint64_t h = tail_fold(FNV_OFFSET, w1);
  auto lo = [](uint64_t x, uint32_t n) { return n >= 8 ? x : (x & ((1ull << (8 * n)) - 1ull)); };
  if (len > 16) h = tail_fold(h, lo(w2, len - 16));
  if (len > 24) h = tail_fold(h, lo(w3, len - 24));
  k1 = long_k1(len, h, k1_mask);
}

// Key of a token of unknown length (>= 31 bytes): 8 bytes per step with a
// SWAR delimiter test, from the LDS buffer (buf_len bytes) and then global
// memory (past avail_len reads as a delimiter).  Returns the length.
__device__ __forceinline__ uint64_t key_long_scan(const uint8_t* buf, uint32_t buf_len, const MapArgs& a, uint32_t pos,
                                                  uint64_t g, uint64_t& k0, uint64_t& k1) {
  uint64_t len = 0, h = FNV_OFFSET, tail = 0;
  k0 = 0;
  for (uint32_t j = 0;; ++j) {
    uint64_t x;
    if (pos + len + 16 <= buf_len) {
      uint64_t y;
      window16(buf, (uint32_t)(pos + len), x, y);
    } else if (g + len + 8 <= a.avail_len) {
      __builtin_memcpy(&x, a.text + g + len, 8);
    } else {
      x = 0;
      for (int i = 0; i < 8; ++i) x |= (uint64_t)(g + len + i < a.avail_len ? a.text[g + len + i] : 0x20) << (8 * i);
    }
    const uint64_t m = delim_mask8(x);
    const uint32_t r = m ? (uint32_t)__ffsll((unsigned long long)m) - 1u : 8u;  // word bytes in this block
    const uint64_t part = r == 8 ? x : (x & ((1ull << (8 * r)) - 1ull));
    if (j == 0) k0 = part;
    else if (r) h = tail_fold(h, part);
    if (j == 1) tail = part;
    len += r;
    if (r < 8) break;
  }
  k1 = len <= 8 ? len : (len <= KEY_INLINE_MAX ? medium_k1(tail, len) : long_k1(len, h, a.k1_mask));
  return len;
}

#ifndef WC_TEXT_NT
#define WC_TEXT_NT 0  // non-temporal text loads (A/B)
#endif
// 32 text bytes at global offset g as two 16-B vectors (' ' past avail).
__device__ __forceinline__ void load32(const MapArgs& a, uint64_t g, uint4& v0, uint4& v1) {
  if (g + MAP_BPL <= a.avail_len) {
    const uint4* src = reinterpret_cast<const uint4*>(a.text + g);
    if (WC_TEXT_NT) {
      typedef uint32_t u4 __attribute__((ext_vector_type(4)));
      const u4* s4 = reinterpret_cast<const u4*>(src);
      const u4 x = __builtin_nontemporal_load(s4), y = __builtin_nontemporal_load(s4 + 1);
      v0 = make_uint4(x.x, x.y, x.z, x.w);
      v1 = make_uint4(y.x, y.y, y.z, y.w);
    } else {
      v0 = src[0];
      v1 = src[1];
    }
  } else {
    uint32_t w[8];
    for (int k = 0; k < 8; ++k) {
      uint32_t x = 0;
      for (int b = 0; b < 4; ++b) {
        const uint64_t i = g + 4 * k + b;
        x |= (uint32_t)(i < a.avail_len ? a.text[i] : 0x20) << (8 * b);
      }
      w[k] = x;
    }
    v0 = make_uint4(w[0], w[1], w[2], w[3]);
    v1 = make_uint4(w[4], w[5], w[6], w[7]);
  }
}

__device__ __forceinline__ uint4 load16(const MapArgs& a, uint64_t g) {
  if (g + 16 <= a.avail_len) return *reinterpret_cast<const uint4*>(a.text + g);
  uint32_t w[4];
  for (int k = 0; k < 4; ++k) {
    uint32_t x = 0;
    for (int b = 0; b < 4; ++b) {
      const uint64_t i = g + 4 * k + b;
      x |= (uint32_t)(i < a.avail_len ? a.text[i] : 0x20) << (8 * b);
    }
    w[k] = x;
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}

}  // namespace dev
}  // namespace wc
