// map_common.hpp — building blocks shared by the map kernels (map.hip: block-
// synchronous tiles; map_dec.hip: wave-decoupled units): delimiter masks, keys
// from an LDS text buffer, the LDS combiner (probe / claim / count) and the
// shuffle-write flush.  Functions touching the combiner take the kernel's LDS
// struct as a template parameter; it must provide key, cnt, off, bcur,
// occupied, sticky, flush_kept and used, plus the slot-state accessors
// bucket(s, log2_buckets) (-1 = empty), key_at(s) and evict(s) of its layout.
#pragma once
#include "kernels.hpp"
#include "keys.hpp"

namespace wc {
namespace dev {

constexpr int MAP_WAVES = MAP_THREADS / 64;
#ifndef WC_MAP_LIST
#define WC_MAP_LIST 256
#endif
constexpr int MAP_LIST = WC_MAP_LIST;            // token-list entries per wave per round (u16)
constexpr int MAP_GS = 8;                        // slots per probe group
constexpr int MAP_NGROUPS = MAP_SLOTS / MAP_GS;  // 256
constexpr int MAP_SPT = MAP_SLOTS / MAP_THREADS; // table slots per thread in a flush
#ifndef WC_MAP_PROMOTE
#define WC_MAP_PROMOTE 5
#endif
#ifndef WC_MAP_STICKY_CAP
#define WC_MAP_STICKY_CAP (MAP_SLOTS * 3 / 16)
#endif
constexpr uint32_t MAP_PROMOTE = WC_MAP_PROMOTE;     // tokens in one flush window that keep a key resident
constexpr int MAP_STICKY_CAP = WC_MAP_STICKY_CAP;    // keys kept per flush and block (0 = off)
constexpr uint32_t MAP_LONG = 31u;               // list length field: >= 31 bytes or past the lane window
constexpr int MAP_WAVE_BYTES = 64 * MAP_BPL;     // text bytes owned by one wave (list positions are relative)
static_assert(MAP_WAVE_BYTES <= 2048, "list entries hold 11-bit wave-relative positions");
static_assert(MAP_SLOTS % MAP_THREADS == 0, "flush assumes whole slots per thread");
static_assert(MAP_TILE <= 65536, "list entries hold 16-bit tile positions");
static_assert((MAP_NGROUPS & (MAP_NGROUPS - 1)) == 0, "group count must be a power of two");

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));


__device__ __forceinline__ uint32_t map_tag(uint64_t ph) { return ((uint32_t)ph & ~1u) | 2u; }  // never 0
__device__ __forceinline__ uint32_t map_group(uint64_t ph) { return (uint32_t)(ph >> 32) & (MAP_NGROUPS - 1); }

// 8 bytes of the LDS tile starting at byte p (dynamic indexing of a register
// window would be lowered to scratch).  Default: ONE unaligned ds_read_b64
// (gfx950 runs HSA queues in unaligned-access mode, and the compiler emits it
// for a byte-aligned memcpy); WC_TILE8_ALIGNED=1: two aligned reads + shift.
#ifndef WC_TILE8_ALIGNED
#define WC_TILE8_ALIGNED 0
#endif
__device__ __forceinline__ uint64_t tile8(const uint8_t* tile, uint32_t p) {
  if (!WC_TILE8_ALIGNED) {
    uint64_t v;
    __builtin_memcpy(&v, tile + p, 8);
    return v;
  }
  const uint64_t* q = reinterpret_cast<const uint64_t*>(tile + (p & ~7u));
  const uint32_t sh = (p & 7) * 8;
  const uint64_t lo = q[0], hi = q[1];
  return sh ? ((lo >> sh) | (hi << (64 - sh))) : lo;
}

__device__ __forceinline__ uint64_t low_bytes(uint64_t v, uint32_t n) {
  return n >= 8 ? v : (v & ((1ull << (8 * n)) - 1ull));
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <class LDS>
__device__ __forceinline__ void clear_slots(LDS& L) {
#pragma unroll
  for (int k = 0; k < MAP_SPT; ++k) {
    const int s = threadIdx.x + k * MAP_THREADS;
    L.evict(s);
    L.cnt[s] = 0;
    L.off[s] = 0xFFFFFFFFu;
  }
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

// Block barrier; the diagnostic build books the time before it to `phase`
// and the wait itself to MS_BARRIER.
template <bool ST>
__device__ __forceinline__ void bsync(PhaseClock<ST>& clk, int phase) {
  clk.lap(phase);
  __syncthreads();
  clk.lap(MS_BARRIER);
}

// Append one record (key, count, first offset) to bucket b's sub-region of this
// block: a 16-byte record for short keys (k1 = length <= 8), else 24 bytes.
// L.bcur[b] packs both cursors (short count | long count << 16).
template <class LDS>
__device__ __forceinline__ void emit_record(LDS& L, const MapArgs& a, uint32_t b, uint64_t k0, uint64_t k1,
                                            uint64_t cnt, uint32_t off) {
  const uint64_t sub = a.rec.subcap;
  const uint64_t at = ((uint64_t)blockIdx.x << a.log2_rec_buckets | b) * sub;
  const bool shortk = k1 <= 8 && cnt <= REC16_MAX_COUNT;
  const uint32_t packed = atomicAdd(&L.bcur[b], shortk ? 1u : 0x10000u);
  const uint32_t pos = shortk ? (packed & 0xFFFFu) : (packed >> 16);
  if (pos < sub) {
    if (shortk) {
      Rec16 r;
      r.k0 = k0;
      r.w = (uint64_t)off | (k1 << 32) | (cnt << 36);
      a.rec.recs16[at + pos] = r;
    } else {
      Rec r;
      r.k0 = k0;
      r.k1 = k1;
      r.co = (cnt << 32) | off;
      a.rec.recs[at + pos] = r;
    }
  } else {
    atomicOr(&a.flags[FLAG_REGION_OVF], 1u);
  }
}

// Shuffle write of the combiner table: every counted slot is appended to its
// bucket's sub-region of this block (emit_record) — one pass, one LDS atomic
// per record, no histogram / scan / directory.  A slot that counted
// MAP_PROMOTE tokens in this window KEEPS its key (count and first offset
// restart from zero) while the block's keep budget lasts, so hot keys stay
// resident and adapt to the text: a key that cools down is evicted at the next
// flush.  `final` evicts every slot.  Two block barriers (occupancy / budget |
// trailing, only when inserts follow immediately); `between` runs on thread 0
// between them.
struct NoHook {
  __device__ void operator()() const {}
};
template <bool ST, class LDS, class Hook = NoHook>
__device__ void flush_table(LDS& L, const MapArgs& a, PhaseClock<ST>& clk, bool trailing_sync, bool final = false,
                            Hook between = Hook()) {
  const int tid = threadIdx.x, lane = tid & 63;
  uint32_t kept = 0, emitted = 0;
#pragma unroll
  for (int j = 0; j < MAP_SPT; ++j) {
    const int s = tid + j * MAP_THREADS;
    const int b = L.bucket(s, a.log2_rec_buckets);
    if (b < 0) continue;
    bool keep = false;
    if (a.ablate != 5) {  // 5 (profiling): flush = clear only
      const uint32_t c = L.cnt[s];
      keep = !final && c >= MAP_PROMOTE && L.sticky < (uint32_t)MAP_STICKY_CAP &&
             atomicAdd(&L.sticky, 1u) < (uint32_t)MAP_STICKY_CAP;
      if (c) {
        const u64x2 kk = L.key_at(s);
        emit_record(L, a, (uint32_t)b, kk.x, kk.y, c, L.off[s]);
        ++emitted;
      }
    }
    L.cnt[s] = 0;  // own slot: no barrier needed before resetting it
    L.off[s] = 0xFFFFFFFFu;
    if (keep) ++kept;
    else L.evict(s);
  }
  for (int o = 32; o > 0; o >>= 1) {
    kept += __shfl_down(kept, o);
    emitted += __shfl_down(emitted, o);
  }
  if (lane == 0 && (kept | emitted)) {
    atomicAdd(&L.flush_kept, kept);
    atomicAdd(&L.used, (unsigned long long)emitted);
  }
  bsync(clk, MS_FL_WRITE);
  if (tid == 0) {
    L.occupied = L.flush_kept;
    L.flush_kept = 0;
    L.sticky = 0;
    between();
  }
  if (trailing_sync) bsync(clk, MS_FL_WRITE);
}

// Block epilogue: this block's per-bucket record counts for the reducer.
template <class LDS>
__device__ __forceinline__ void publish_bucket_counts(LDS& L, const MapArgs& a) {
  const uint32_t nb = 1u << a.log2_rec_buckets;
  for (uint32_t b = threadIdx.x; b < nb; b += MAP_THREADS) a.rec.count[(size_t)blockIdx.x * nb + b] = L.bcur[b];
}

// Key of a token that does not end inside the 64-byte lane window: byte loop
// over the LDS text buffer `buf` (buf_len bytes readable), then global memory.
__device__ __forceinline__ void key_slow(const uint8_t* buf, uint32_t buf_len, const MapArgs& a, uint64_t pos,
                                         uint64_t g, uint64_t& k0, uint64_t& k1) {
  uint64_t len = 0, h = FNV_OFFSET, chunk = 0;
  k0 = 0;
  for (;;) {
    uint32_t c;
    if (pos < (uint64_t)buf_len) c = buf[pos];
    else if (g < a.avail_len) c = a.text[g];
    else break;
    if (is_delim(c)) break;
    if (len < 8) {
      k0 |= (uint64_t)c << (8 * len);
    } else {
      chunk |= (uint64_t)c << (8 * (len & 7));
      if ((len & 7) == 7) {
        h = tail_fold(h, chunk);
        chunk = 0;
      }
    }
    ++len, ++pos, ++g;
  }
  if (len > 8 && (len & 7)) h = tail_fold(h, chunk);
  k1 = make_k1(len, h);
}

// Key of the token at buffer position p with known length (< 31) or MAP_LONG;
// buf[0] is global text offset t0.
__device__ __forceinline__ void token_key(const uint8_t* buf, uint32_t buf_len, const MapArgs& a, uint64_t t0,
                                          uint32_t p, uint32_t len, uint64_t& k0, uint64_t& k1) {
  if (len != MAP_LONG) {
    k0 = low_bytes(tile8(buf, p), len);
    if (len <= 8) {
      k1 = len;
    } else {
      uint64_t h = FNV_OFFSET;
      for (uint32_t c = 8; c < len; c += 8) h = tail_fold(h, low_bytes(tile8(buf, p + c), len - c));
      k1 = make_k1(len, h);
    }
  } else {
    key_slow(buf, buf_len, a, p, t0 + p, k0, k1);
  }
}

// Key from the token's first 8-byte window w (already read at p).
__device__ __forceinline__ void finish_key(const uint8_t* buf, uint32_t buf_len, const MapArgs& a, uint64_t t0,
                                           uint64_t w, uint32_t p, uint32_t len, uint64_t& k0, uint64_t& k1) {
  if (len != MAP_LONG) {
    k0 = low_bytes(w, len);
    if (len <= 8) {
      k1 = len;
    } else {
      uint64_t h = FNV_OFFSET;
      for (uint32_t c = 8; c < len; c += 8) h = tail_fold(h, low_bytes(tile8(buf, p + c), len - c));
      k1 = make_k1(len, h);
    }
  } else {
    key_slow(buf, buf_len, a, p, t0 + p, k0, k1);
  }
}

// Keys of a lane's two tokens of a step: both first windows are read before
// either key is finished, so short words cost ONE LDS round trip for both.
// Lanes without a token read harmless in-buffer bytes (p = 0) and get 0 keys.
__device__ __forceinline__ void token_keys2(const uint8_t* buf, uint32_t buf_len, const MapArgs& a, uint64_t t0,
                                            bool h1, uint32_t p1, uint32_t len1, bool h2, uint32_t p2, uint32_t len2,
                                            uint64_t& a0, uint64_t& a1, uint64_t& b0, uint64_t& b1) {
  const uint64_t w1 = tile8(buf, p1), w2 = tile8(buf, p2);
  a0 = a1 = b0 = b1 = 0;
  if (h1) finish_key(buf, buf_len, a, t0, w1, p1, len1, a0, a1);
  if (h2) finish_key(buf, buf_len, a, t0, w2, p2, len2, b0, b1);
}

// Combiner slot of (k0, k1) — claiming one if the key is absent and `admit` —
// or -1 when MAP_MAX_GROUP_PROBES groups are full (or the key is absent and
// !admit).  Claim = ONE CAS of the tag; the
// claimer then writes k0 before k1 (LDS executes one wave's writes in order,
// and the reader loads the 16-byte key in one instruction), so a reader that
// sees the new k1 also sees the new k0; one that sees the tag before the key
// does not match and may claim a duplicate slot, which the reducer merges.
template <class LDS>
__device__ __forceinline__ int combiner_slot(LDS& L, uint64_t ph, uint64_t k0, uint64_t k1, bool& claimed,
                                             bool admit = true) {
  const uint32_t tag = map_tag(ph);
  uint32_t g = map_group(ph);
  claimed = false;
  for (int steps = 0; steps < MAP_MAX_GROUP_PROBES;) {
    asm volatile("" ::: "memory");
    const u32x4 ta = *reinterpret_cast<const u32x4*>(&L.tag[g * MAP_GS]);
    const u32x4 tb = *reinterpret_cast<const u32x4*>(&L.tag[g * MAP_GS + 4]);
    uint32_t m = (ta.x == tag ? 1u : 0u) | (ta.y == tag ? 2u : 0u) | (ta.z == tag ? 4u : 0u) |
                 (ta.w == tag ? 8u : 0u) | (tb.x == tag ? 16u : 0u) | (tb.y == tag ? 32u : 0u) |
                 (tb.z == tag ? 64u : 0u) | (tb.w == tag ? 128u : 0u);
    while (m) {
      const uint32_t i = __ffs(m) - 1;
      m &= m - 1;
      const u64x2 kk = L.key[g * MAP_GS + i];
      if (kk.x == k0 && kk.y == k1) return (int)(g * MAP_GS + i);
    }
    const uint32_t e = (ta.x == 0 ? 1u : 0u) | (ta.y == 0 ? 2u : 0u) | (ta.z == 0 ? 4u : 0u) |
                       (ta.w == 0 ? 8u : 0u) | (tb.x == 0 ? 16u : 0u) | (tb.y == 0 ? 32u : 0u) |
                       (tb.z == 0 ? 64u : 0u) | (tb.w == 0 ? 128u : 0u);
    if (!e) {
      ++steps;
      g = (g + 1) & (MAP_NGROUPS - 1);
      continue;
    }
    if (!admit) return -1;
    const uint32_t s = g * MAP_GS + (__ffs(e) - 1);
    if (atomicCAS(&L.tag[s], 0u, tag) == 0u) {
      L.key[s].x = k0;
      asm volatile("" ::: "memory");
      L.key[s].y = k1;
      claimed = true;
      return (int)s;
    }
    // lost the slot to another lane: re-read this group
  }
  return -1;
}

// Count one token; false if its probe sequence is full.
template <class LDS>
__device__ __forceinline__ bool combine(LDS& L, uint64_t k0, uint64_t k1, uint32_t off, bool& claimed) {
  const int s = combiner_slot(L, place_hash(k0, k1), k0, k1, claimed);
  if (s < 0) return false;
  atomicAdd(&L.cnt[s], 1u);  // results unused: no-return ds_add / ds_min
  atomicMin(&L.off[s], off);
  return true;
}

// 32 text bytes at global offset g as two 16-B vectors (' ' past avail).
__device__ __forceinline__ void load32(const MapArgs& a, uint64_t g, uint4& v0, uint4& v1) {
  if (g + MAP_BPL <= a.avail_len) {
    const uint4* src = reinterpret_cast<const uint4*>(a.text + g);
    v0 = src[0];
    v1 = src[1];
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
