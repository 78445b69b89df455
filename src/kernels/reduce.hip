// reduce.hip — the REDUCE stage and the running key table.
//
// Reference: reducer (/root/reference/main.cu:69-108) is run by ONE GPU thread
// (reduceKernel, main.cu:119-123) doing a linear scan of at most 10 output
// keys per pair with a prefix compare.  Here:
//
//  wc_reduce_buckets  one 1024-thread block per table bucket (one per CU).
//                     The bucket's 4096-slot slice of the running table is
//                     loaded into LDS (144 KiB with tags), the bucket's
//                     contiguous record run of every map block is streamed
//                     (RED_UNROLL x 64 records in flight per wave) and merged
//                     with LDS atomics (count +=, first = min), and the slice
//                     is written back.  LONG words (>= 16 bytes, hashed keys)
//                     are merged only after a byte comparison with the stored
//                     copy of the word (exact equality, keys.hpp), in line with
//                     every other record (a second, lean pass over the 24-byte
//                     runs): a new LONG word is claimed by the first lane that
//                     meets it, in parallel across the block, and references
//                     its occurrence in the chunk until the block end copies
//                     all the pass's new words to the key arena (keys outlive
//                     streamed chunks) with one arena allocation per block.
//                     If a slice overflows it is NOT written back;
//                     the host splits the table and re-runs only the
//                     overflowed buckets.
//  wc_table_split     B -> 2B buckets (rehash into new slices).
//  wc_table_compact   occupied slots -> dense columns (per-bucket block scan).
#include "kernels.hpp"

#include "bounds.hpp"
#include "map_common.hpp"  // wave_incl_sum (DPP wave scan)
#include "lds_table.hpp"
#include "common/hip_util.hpp"

// Diagnostic build (-DWC_RED_STAMPS=1, tools/variants.sh; run with WC_MAP_STAMPS=1):
// per-block LDS counters of records, slow-path lanes / waves, claim-loop
// iterations, CAS failures, PENDING re-reads, claims and s_memtime wave time.
#ifndef WC_RED_STAMPS
#define WC_RED_STAMPS 0
#endif

namespace wc {
namespace dev {

// Profiling builds only (tools/variants.sh -DWC_RED_ABLATE=N; results NOT
// valid): 1 record loads only, 2 + hashes and both probe reads, 3 everything
// but the hit atomics.
#ifndef WC_RED_ABLATE
#define WC_RED_ABLATE 0
#endif

#ifndef WC_RED_UNROLL
#define WC_RED_UNROLL 4
#endif
constexpr int RED_UNROLL = WC_RED_UNROLL;  // 16-byte records in flight per lane
#ifndef WC_RED_UNROLL_24
#define WC_RED_UNROLL_24 2
#endif
constexpr int RED_UNROLL_24 = WC_RED_UNROLL_24;  // 24-byte records in flight per lane (VGPR budget)
constexpr uint32_t SREF_POISON = 0xFFFFFFFFu;  // sref_len of a LONG slot whose bytes did not fit the arena
constexpr uint32_t LONGQ = 2048;  // LONG record indices queued per bucket pass (more: the runs are re-scanned)

struct RedLds {
  SlotGroup grp[TAB_GROUPS];  // first: 16-B aligned group reads
  uint64_t cnt[TAB_SLOTS];
  uint64_t first[TAB_SLOTS];
  uint32_t longq[LONGQ];  // record indices of this pass's LONG records
  uint32_t nlong;
  uint32_t occupied;
  uint32_t overflow;
  uint32_t runcnt[RED_MAX_RUNS];  // packed record counts of this bucket's run in every map block
  uint16_t runlong[RED_MAX_RUNS]; // LONG records of this bucket's sub-region in every map block (Records::count_long)
  unsigned long long st[RED_STAMP_N];  // diagnostic counters (WC_RED_STAMPS builds only)
};
static_assert(sizeof(RedLds) <= 160 * 1024, "one reduce block per CU");

// A bucket with occupancy 0 has UNDEFINED slice contents (Engine::reset zeroes
// only the occupancy): it starts empty without reading the slice.
__device__ __forceinline__ void load_slice(RedLds& L, const TableView& t, uint32_t b, bool empty = false) {
  const size_t base = (size_t)b * TAB_SLOTS;
  if (empty || t.occupancy[b] == 0) {
    for (int s = threadIdx.x; s < TAB_SLOTS; s += blockDim.x) {
      SlotGroup& G = L.grp[s >> 2];
      G.k0[s & 3] = 0;
      G.k1[s & 3] = K1_EMPTY;
      G.tag[s & 3] = TAG_EMPTY;
      L.cnt[s] = 0;
      L.first[s] = ~0ull;
    }
    return;
  }
  for (int s = threadIdx.x; s < TAB_SLOTS; s += blockDim.x) {
    const uint64_t k0 = t.k0[base + s], k1 = t.k1[base + s];
    SlotGroup& G = L.grp[s >> 2];
    G.k0[s & 3] = k0;
    G.k1[s & 3] = k1;
    G.tag[s & 3] = k1 == K1_EMPTY ? TAG_EMPTY : make_tag(place_hash(k0, k1));
    L.cnt[s] = t.cnt[base + s];
    L.first[s] = t.first[base + s];
  }
}

__device__ __forceinline__ void store_slice(const RedLds& L, const TableView& t, uint32_t b) {
  const size_t base = (size_t)b * TAB_SLOTS;
  for (int s = threadIdx.x; s < TAB_SLOTS; s += blockDim.x) {
    const bool occ = slot_tag(L.grp, s) > TAG_PENDING;
    t.k0[base + s] = slot_k0(L.grp, s);
    t.k1[base + s] = occ ? slot_k1(L.grp, s) : K1_EMPTY;
    t.cnt[base + s] = L.cnt[s];
    t.first[base + s] = L.first[s];
  }
}

// Copy len bytes text[o..) -> arena[p..): 16-byte pieces, then the tail in
// 8/4/2/1-byte pieces (never past len: neighbouring words are written concurrently).
__device__ __forceinline__ void copy_bytes(uint8_t* dst, const uint8_t* src, uint64_t len) {
  uint64_t c = 0;
  for (; c + 16 <= len; c += 16) {
    uint64_t w[2];
    __builtin_memcpy(w, src + c, 16);
    __builtin_memcpy(dst + c, w, 16);
  }
  if (len - c >= 8) { uint64_t w; __builtin_memcpy(&w, src + c, 8); __builtin_memcpy(dst + c, &w, 8); c += 8; }
  if (len - c >= 4) { uint32_t w; __builtin_memcpy(&w, src + c, 4); __builtin_memcpy(dst + c, &w, 4); c += 4; }
  if (len - c >= 2) { uint16_t w; __builtin_memcpy(&w, src + c, 2); __builtin_memcpy(dst + c, &w, 2); c += 2; }
  if (len - c >= 1) dst[c] = src[c];
}

// Count + first offset into slot s.
__device__ __forceinline__ void add_to_slot(RedLds& L, int s, uint64_t cnt, uint64_t first) {
  atomicAdd(reinterpret_cast<unsigned long long*>(&L.cnt[s]), (unsigned long long)cnt);
  atomicMin(reinterpret_cast<unsigned long long*>(&L.first[s]), (unsigned long long)first);
}

// A key not found in its home group: full probe, claiming a slot if new.
// Out of line: one copy keeps the unrolled batch loop small (inlining measured no faster).
__device__ __noinline__ uint32_t merge_slow(RedLds& L, uint32_t ph, uint64_t k0, uint64_t k1, uint64_t cnt,
                                            uint64_t first) {
  bool claimed;
  const int s = lds_find_or_claim(L.grp, TAB_GROUPS, ph, k0, k1, TAB_MAX_GROUP_PROBES, claimed, true,
                                  WC_RED_STAMPS ? L.st : nullptr);
  if (WC_RED_STAMPS) atomicAdd(&L.st[RS_SLOW_LANES], 1ull);
  if (s < 0) {
    L.overflow = 1;
    return 0;
  }
  add_to_slot(L, s, cnt, first);
  return claimed ? 1u : 0u;
}

// What the LONG-word merge reads, passed BY VALUE to the out-of-line
// merge_long (a reference to ReduceArgs would make the kernel keep its
// argument block in scratch memory and reload fields from it in the hot loop).
struct LongCtx {
  const uint8_t* text;
  uint64_t avail_len;
  const uint8_t* arena;
  uint64_t* sref_off;  // this bucket's slice of the table's arena references
  uint32_t* sref_len;
};
// sref_off of a slot claimed during the current pass: the word's bytes are
// still in the chunk text (copied to the key arena at the block end, one
// arena allocation per block instead of one contended atomic per new word).
constexpr uint64_t SREF_TEXT = 1ull << 63;

__device__ __forceinline__ uint64_t word_len(const uint8_t* text, uint64_t avail_len, uint64_t o) {
  uint64_t len = 0;
  while (o + len + 16 <= avail_len) {
    uint64_t w[2];
    __builtin_memcpy(w, text + o + len, 16);
    const uint32_t m = (uint32_t)(delim_mask8(w[0]) | (delim_mask8(w[1]) << 8));
    if (m) return len + (uint64_t)(__ffs(m) - 1);
    len += 16;
  }
  while (o + len < avail_len && !is_delim(text[o + len])) ++len;
  return len;
}

// Is the word at text offset o exactly the stored word (sref so, len)?  The
// stored copy is 8-byte aligned in the arena, or (SREF_TEXT) the claiming
// record's occurrence in this chunk's text; then the byte after the word
// must end it (a delimiter or the end of the readable text).
__device__ __forceinline__ bool long_equal(const LongCtx& c, uint64_t o, uint64_t so, uint32_t len) {
  if (o + len > c.avail_len) return false;
  const bool in_text = (so & SREF_TEXT) != 0;
  const uint8_t* ref = in_text ? c.text + (so & ~SREF_TEXT) : c.arena + so;
  uint32_t i = 0;
  for (; i + 8 <= len; i += 8) {
    uint64_t u, v;
    __builtin_memcpy(&u, c.text + o + i, 8);
    __builtin_memcpy(&v, ref + i, 8);
    if (u != v) return false;
  }
  for (; i < len; ++i)
    if (c.text[o + i] != ref[i]) return false;
  return o + len == c.avail_len || is_delim(c.text[o + len]);
}

// The first 64 bytes at text offset o as eight words, loaded together (one
// memory round trip; past the readable text they read as delimiters), and the
// length of the word there (64: the word is longer).
__device__ __forceinline__ uint32_t load_word64(const LongCtx& c, uint64_t o, uint64_t (&w)[8]) {
  if (o + 64 <= c.avail_len) {
#pragma unroll
    for (int i = 0; i < 8; ++i) __builtin_memcpy(&w[i], c.text + o + 8 * i, 8);
  } else {  // the last 64 bytes of the readable text (rare): byte by byte
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = 0x2020202020202020ull;
#pragma unroll 1
    for (uint32_t k = 0; k < 64 && o + k < c.avail_len; ++k) {
      const uint64_t x = c.text[o + k];
#pragma unroll
      for (int i = 0; i < 8; ++i)
        if ((int)(k >> 3) == i) w[i] = (w[i] & ~(0xFFull << (8 * (k & 7)))) | (x << (8 * (k & 7)));
    }
  }
  uint32_t len = 64;
#pragma unroll
  for (int i = 7; i >= 0; --i) {
    const uint64_t m = delim_mask8(w[i]);
    if (m) len = 8 * i + (uint32_t)__ffsll((unsigned long long)m) - 1;
  }
  return len;
}

// The record's word (first 64 bytes in w, length wlen < 64) == the stored
// word (sref so, sl)?  The stored copy's words are loaded together.
__device__ __forceinline__ bool long_equal64(const LongCtx& c, const uint64_t (&w)[8], uint32_t wlen, uint64_t so,
                                             uint32_t sl) {
  if (sl != wlen) return false;
  const bool in_text = (so & SREF_TEXT) != 0;
  const uint8_t* ref = in_text ? c.text + (so & ~SREF_TEXT) : c.arena + so;
  uint64_t r[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    r[i] = 0;
    if (8 * i < (int)sl) __builtin_memcpy(&r[i], ref + 8 * i, 8);  // the word's last 8-byte piece may read past it
  }
  bool eq = true;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    if (8 * i >= (int)sl) continue;
    const uint32_t n = sl - 8 * i;
    const uint64_t m = n >= 8 ? ~0ull : ((1ull << (8 * n)) - 1ull);
    eq &= ((w[i] ^ r[i]) & m) == 0;
  }
  return eq;
}

// A LONG record (hashed key): find the slot whose stored word equals the
// record's word byte for byte, or claim one.  Colliding words (same k0, k1,
// different bytes) keep separate slots, so the probe continues past a slot
// whose bytes differ.  A claim keeps the slot PENDING while the claimer
// writes the slot's reference (SREF_TEXT | its own text offset, and the
// length), then publishes the tag (workgroup release); a reader that matched
// a published tag acquires before reading the reference.  Probers that see
// PENDING re-read the group; the claimer finishes inside its iteration, so
// the lanes of one wave never wait on each other.  Returns 1 for a claim.
// w / wlen: the record's first 64 bytes and length (load_word64), loaded by
// the caller — long_direct issues them one batch ahead.
__device__ __forceinline__ int find_long_w(RedLds& L, const LongCtx& c, uint32_t ph, uint64_t k0, uint64_t k1,
                                           uint64_t off, const uint64_t (&w)[8], uint32_t wlen, bool& claimed) {
  claimed = false;
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  const uint32_t tag = make_tag(ph);
  const uint32_t g1 = group_of(ph, TAB_GROUPS), g2 = group2_of(ph, TAB_GROUPS);
  uint32_t g = g1;
  int steps = 0;
  if (WC_RED_STAMPS) atomicAdd(&L.st[RS_SLOW_LANES], 1ull);
  for (;;) {
    asm volatile("" ::: "memory");
    SlotGroup& G = L.grp[g];
    const u32x4 t = *reinterpret_cast<const u32x4*>(G.tag);
    const uint32_t tv[4] = {t.x, t.y, t.z, t.w};
    bool pending = false;
    int e = -1;
    uint32_t mm = 0;  // slots holding this key (several only for colliding words)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (tv[i] == TAG_PENDING) pending = true;
      else if (tv[i] == TAG_EMPTY) e = e < 0 ? i : e;
      else if (tv[i] == tag && G.k1[i] == k1 && G.k0[i] == k0) mm |= 1u << i;
    }
    if (mm) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    while (mm) {  // one comparison in the loop body (registers), usually one pass
      const int i = __ffs(mm) - 1;
      mm &= mm - 1;
      const int s = 4 * (int)g + i;
      const uint32_t sl = c.sref_len[s];
      const uint64_t so = c.sref_off[s];
      if (sl == SREF_POISON || (wlen < 64 ? long_equal64(c, w, wlen, so, sl) : long_equal(c, off, so, sl))) return s;
    }
    if (WC_RED_STAMPS) atomicAdd(&L.st[RS_PROBE_ITERS], 1ull);
    if (pending) continue;  // a claim is being published in this group: look again
    if (e >= 0) {
      if (atomicCAS(&G.tag[e], TAG_EMPTY, TAG_PENDING) != TAG_EMPTY) continue;  // lost the race: re-read
      const int s = 4 * (int)g + e;
      G.k0[e] = k0;
      G.k1[e] = k1;
      const uint64_t len = wlen < 64 ? wlen : word_len(c.text, c.avail_len, off);
      c.sref_off[s] = SREF_TEXT | off;
      c.sref_len[s] = len < SREF_POISON ? (uint32_t)len : SREF_POISON;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __hip_atomic_store(&G.tag[e], tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      if (WC_RED_STAMPS) atomicAdd(&L.st[RS_CLAIMS], 1ull);
      claimed = true;
      return s;
    }
    if (++steps >= TAB_MAX_GROUP_PROBES) {
      L.overflow = 1;
      return -1;
    }
    g = probe_group(g1, g2, (uint32_t)steps, TAB_GROUPS);
  }
}

__device__ __forceinline__ int find_long(RedLds& L, const LongCtx& c, uint32_t ph, uint64_t k0, uint64_t k1, uint64_t off,
                                         bool& claimed) {
  uint64_t w[8];  // the record's bytes, before the probe needs them (their loads overlap it)
  const uint32_t wlen = load_word64(c, off, w);
  return find_long_w(L, c, ph, k0, k1, off, w, wlen, claimed);
}

// A wave's LONG records after find_long (slot s, or -1 for none / no room),
// EVERY lane of the wave converged here: the records of the first valid
// lane's slot — a frequent LONG word — add once, summed in registers (one
// pair of LDS atomics instead of one per lane on the same address); the
// others add for themselves.  Each record is counted exactly once: by its own
// lane (s != the lead slot) or inside the lead's sum (s == the lead slot);
// lanes with s < 0 hold no record (the sum takes 0 / ~0 from them).
__device__ __forceinline__ void wave_add_long(RedLds& L, int s, uint64_t cnt, uint64_t first) {
  const int lane = threadIdx.x & 63;
  const uint64_t valid = __ballot(s >= 0);
  if (!valid) return;
  const int lead = __ffsll((unsigned long long)valid) - 1;
  const int ls = __builtin_amdgcn_readlane(s, lead);
  const bool same = s == ls;
  if (s >= 0 && !same) add_to_slot(L, s, cnt, first);
  if (__popcll(__ballot(same)) == 1) {
    if (lane == lead) add_to_slot(L, ls, cnt, first);
    return;
  }
  uint64_t c = same ? cnt : 0ull, f = same ? first : ~0ull;
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t clo = (uint32_t)__shfl_xor((int)(uint32_t)c, o), chi = (uint32_t)__shfl_xor((int)(uint32_t)(c >> 32), o);
    const uint32_t flo = (uint32_t)__shfl_xor((int)(uint32_t)f, o), fhi = (uint32_t)__shfl_xor((int)(uint32_t)(f >> 32), o);
    c += (uint64_t)clo | ((uint64_t)chi << 32);
    const uint64_t g = (uint64_t)flo | ((uint64_t)fhi << 32);
    f = g < f ? g : f;
  }
  if (lane == lead) add_to_slot(L, ls, c, f);
}

// Block end of a bucket pass: the LONG words claimed during the pass still
// reference the chunk text; one arena allocation for all of them (a block
// scan of their 8-byte-rounded lengths, ONE global atomic), then every thread
// copies its slots' words and rewrites their references.
__device__ void settle_new_long(RedLds& L, const ReduceArgs& a, uint32_t b) {
  __shared__ uint32_t wbytes[RED_THREADS / 64];
  __shared__ unsigned long long base;
  const size_t sbase = (size_t)b * TAB_SLOTS;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  static_assert(TAB_SLOTS == 4 * RED_THREADS, "settle: 4 slots per thread");
  uint32_t need[4], mine = 0;
  // the four slots' references loaded together (one device round trip, not one per slot)
  uint64_t so[4];
  uint32_t sl[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    so[j] = a.tab.sref_off[sbase + 4 * tid + j];
    sl[j] = a.tab.sref_len[sbase + 4 * tid + j];
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int s = 4 * tid + j;
    need[j] = 0;
    if (slot_tag(L.grp, s) > TAG_PENDING && key_is_hashed(slot_k1(L.grp, s)) && (so[j] & SREF_TEXT)) {
      const uint32_t len = sl[j];
      need[j] = len == SREF_POISON ? 0u : ((len + 7u) & ~7u) | 1u;  // | 1: a new word (even of length 0)
    }
    mine += need[j] & ~1u;
  }
  uint32_t incl = mine;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(incl, o);
    if (lane >= o) incl += y;
  }
  if (lane == 63) wbytes[wave] = incl;
  __syncthreads();
  uint32_t before = 0, total = 0;
  for (int w = 0; w < RED_THREADS / 64; ++w) {
    before += w < wave ? wbytes[w] : 0u;
    total += wbytes[w];
  }
  if (tid == 0) base = total ? atomicAdd(a.arena.cursor, (unsigned long long)total) : 0ull;
  __syncthreads();
  const bool ovf = base + total > a.arena.cap;
  if (ovf && tid == 0) atomicOr(&a.flags[FLAG_ARENA_OVF], 1u);
  uint64_t p = base + before + incl - mine;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (!need[j]) continue;
    const int s = 4 * tid + j;
    const uint64_t to = so[j] & ~SREF_TEXT;
    const uint32_t len = sl[j];
    if (ovf) {
      a.tab.sref_off[sbase + s] = 0;
      a.tab.sref_len[sbase + s] = SREF_POISON;
      continue;
    }
    copy_bytes(a.arena.bytes + p, a.text + to, len);
    a.tab.sref_off[sbase + s] = p;
    p += need[j] & ~1u;
  }
}

// Records [k, k + U * 64) of one run, three phases so a lane keeps all its
// records' LDS traffic in flight together: (1) load the records, hash them,
// read the tags of the first two groups of every record's probe sequence (one
// LDS round trip for all); (2) read k1 / k0 of the first slot whose tag
// matches (a second round trip); (3) a key match counts with two LDS atomics.
// A record with no matching slot in those groups — a new key, a key placed
// further along its sequence, a tag collision — takes merge_slow.  LONG keys
// (hashed, 24-byte runs only) are left to long_stream.
template <bool R16, int U, class RecT>
__device__ __forceinline__ void merge_batch(RedLds& L, const ReduceArgs& a, uint32_t b, const RecT (&rr)[U],
                                            const bool (&valid)[U], const uint32_t (&idx)[U], uint32_t shift,
                                            uint32_t& claims) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  const int lane = threadIdx.x & 63;
  uint64_t k0[U], k1[R16 ? 1 : U];  // Rec16: k1 is recomputed from k0 and the tail word (VGPR budget)
  uint32_t ph[U], slot[U];
  auto key1 = [&](int u) -> uint64_t {
    if constexpr (R16) return rec16_k1(k0[u], rr[u].t);
    else return k1[u];
  };
  bool mine[U];
  u32x4 tg[U], tg2[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if constexpr (R16) {
      k0[u] = rr[u].lo | ((uint64_t)rr[u].hi << 32);
    } else {
      k0[u] = rr[u].k0;
      k1[u] = rr[u].k1;
    }
    if (WC_RED_ABLATE == 1) {
      if (k0[u] == 0x9E3779B97F4A7C15ull) L.overflow = 2;  // never true: keeps the load
      continue;
    }
    ph[u] = place_hash(k0[u], key1(u));
    mine[u] = valid[u] && (!shift || bucket_of(ph[u], a.tab.log2_buckets) == b);
    if (!R16 && mine[u] && key_is_hashed(key1(u))) {  // LONG: queued for merge_long after the streams
      const uint32_t q = atomicAdd(&L.nlong, 1u);
      if (q < LONGQ) L.longq[q] = idx[u];
      mine[u] = false;
    }
    tg[u] = *reinterpret_cast<const u32x4*>(L.grp[group_of(ph[u], TAB_GROUPS)].tag);
    tg2[u] = *reinterpret_cast<const u32x4*>(L.grp[group2_of(ph[u], TAB_GROUPS)].tag);
  }
  if (WC_RED_ABLATE == 1) return;
  uint64_t c1[U], c0[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint32_t tag = make_tag(ph[u]);
    const uint32_t m = (tg[u].x == tag ? 1u : 0u) | (tg[u].y == tag ? 2u : 0u) | (tg[u].z == tag ? 4u : 0u) |
                       (tg[u].w == tag ? 8u : 0u) | (tg2[u].x == tag ? 16u : 0u) | (tg2[u].y == tag ? 32u : 0u) |
                       (tg2[u].z == tag ? 64u : 0u) | (tg2[u].w == tag ? 128u : 0u);
    const uint32_t f = (uint32_t)__ffs(m) - 1u;  // first candidate (g1 before g2)
    slot[u] = m ? 4 * (f < 4 ? group_of(ph[u], TAB_GROUPS) : group2_of(ph[u], TAB_GROUPS)) + (f & 3) : 0xFFFFFFFFu;
    const uint32_t s = m ? slot[u] : 0u;
    c1[u] = slot_k1(L.grp, (int)s);
    c0[u] = slot_k0(L.grp, (int)s);
  }
  if (WC_RED_ABLATE == 2) {
    uint64_t x = 0;
#pragma unroll
    for (int u = 0; u < U; ++u) x ^= c0[u] ^ c1[u];
    if (x == 0x9E3779B97F4A7C15ull) L.overflow = 2;  // never true
    return;
  }
  if (WC_RED_STAMPS) {
    uint32_t nrec = 0;
    for (int u = 0; u < U; ++u) nrec += (uint32_t)__popcll(__ballot(valid[u]));
    if (lane == 0) atomicAdd(&L.st[RS_RECORDS], (unsigned long long)nrec);
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if (WC_RED_STAMPS) {
      const bool slow = mine[u] && !(slot[u] != 0xFFFFFFFFu && c1[u] == key1(u) && c0[u] == k0[u]);
      if (__ballot(slow) && lane == 0) atomicAdd(&L.st[RS_SLOW_WAVES], 1ull);
    }
    if (!mine[u]) continue;
    uint64_t cnt;
    uint32_t off;
    if constexpr (R16) {
      cnt = 1;
      off = rr[u].off;
    } else {
      cnt = rr[u].co >> 32;
      off = (uint32_t)rr[u].co;
    }
    const uint64_t first = a.chunk_base + off;
    if (slot[u] != 0xFFFFFFFFu && c1[u] == key1(u) && c0[u] == k0[u]) {
      if (WC_RED_ABLATE != 3) add_to_slot(L, (int)slot[u], cnt, first);
    } else {
      claims += merge_slow(L, ph[u], k0[u], key1(u), cnt, first);
    }
  }
}

// One record kind's stream over this wave's runs (map blocks p = wave,
// wave + nwaves, ...; run p = sub-region (p, rb), its length in L.runcnt),
// flattened: batches of U x 64 CONSECUTIVE records of the concatenated runs,
// so batches are full however short the runs are (at 1M words a run holds
// ~270 12-byte records: per-run batches were half empty, and a wave's time is
// its batch count x the per-batch LDS round trips).  Each batch is loaded one
// batch AHEAD of its merge.  Lane j holds run j's exclusive prefix P and
// index adjustment ADJ = first record index of run j - P; a record at stream
// position t of run j sits at t + ADJ_j.
template <bool R16, int U, class RecT>
__device__ __forceinline__ void merge_stream(RedLds& L, const ReduceArgs& a, uint32_t b, const RecT* recs, uint32_t p0,
                                             uint32_t pstride, uint32_t nrb, uint32_t rb, uint32_t sub, uint32_t shift,
                                             uint32_t& claims, uint32_t p_end = ~0u) {
  constexpr uint32_t B = U * 64;
  const uint32_t lane = threadIdx.x & 63;
  // runs p0, p0 + pstride, ... below p_end (pstride >= 16: <= 64 runs, RED_MAX_RUNS)
  const uint32_t pe = min(p_end, a.map_blocks);
  const uint32_t nj = p0 < pe ? (pe - p0 + pstride - 1) / pstride : 0u;
  uint32_t c = 0;
  if (lane < nj) {
    const uint32_t packed = L.runcnt[p0 + lane * pstride];
    c = min(R16 ? (packed & 0xFFFFu) : (packed >> 16), sub);
  }
  const uint32_t incl = wave_incl_sum(c);  // DPP: no bpermute lane addresses held across the stream
  const uint32_t N = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
  if (N == 0) return;
  const uint32_t P = incl - c;
  const uint32_t C0 = (p0 * nrb + rb) * sub, D = pstride * nrb * sub;  // < record capacity < 2^32
  const uint32_t ADJ = C0 + lane * D - P;                               // modular: t + ADJ is exact
  uint32_t jlo = 0;  // run holding the current batch start (wave-uniform)
  auto locate = [&](uint32_t T0, uint32_t (&idx)[U], bool (&valid)[U]) {
    while (jlo + 1 < nj && (uint32_t)__builtin_amdgcn_readlane((int)P, (int)(jlo + 1)) <= T0) ++jlo;
    const uint32_t adj = (uint32_t)__builtin_amdgcn_readlane((int)ADJ, (int)jlo);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t t = T0 + u * 64 + lane;
      idx[u] = t + adj;
      valid[u] = t < N;
    }
    for (uint32_t jj = jlo + 1; jj < nj; ++jj) {  // runs starting inside this batch (usually 0-2)
      const uint32_t pj = (uint32_t)__builtin_amdgcn_readlane((int)P, (int)jj);
      if (pj >= T0 + B) break;
      const uint32_t aj = (uint32_t)__builtin_amdgcn_readlane((int)ADJ, (int)jj);
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (T0 + u * 64 + lane >= pj) idx[u] = T0 + u * 64 + lane + aj;
    }
  };
  auto load = [&](RecT (&rr)[U], const uint32_t (&idx)[U], const bool (&valid)[U]) {
#pragma unroll
    for (int u = 0; u < U; ++u) rr[u] = recs[valid[u] ? idx[u] : C0];  // C0: inside the store
  };
  RecT ra[U], rb2[U];
  uint32_t ia[U], ib[U];
  bool va[U], vb[U];
  locate(0, ia, va);
  load(ra, ia, va);
  for (uint32_t T0 = 0;; T0 += 2 * B) {  // unrolled by two: the register sets swap roles without copies
    const bool more = T0 + B < N;
    if (more) {
      locate(T0 + B, ib, vb);
      load(rb2, ib, vb);
    }
    merge_batch<R16, U>(L, a, b, ra, va, ia, shift, claims);
    if (!more) return;
    const bool more2 = T0 + 2 * B < N;
    if (more2) {
      locate(T0 + 2 * B, ia, va);
      load(ra, ia, va);
    }
    merge_batch<R16, U>(L, a, b, rb2, vb, ib, shift, claims);
    if (!more2) return;
  }
}

// The LONG records of this wave's runs (map blocks p0, p0 + pstride, ...): each
// run fills its 24-byte sub-region from the top down (Records::count_long), so
// they stream straight in, one record per lane, batches of 64 concatenated
// across runs (as merge_stream: lane j holds run j's prefix P_j and the index
// of its record 0, TOP_j, so stream position t of run j is record TOP_j + P_j - t).
// The next batch's records and their first 64 text bytes are loaded before
// this batch's slots are resolved: the random text read — the LONG merge's
// cost — overlaps the probe and the byte comparison of the batch before.
__device__ __forceinline__ void long_direct(RedLds& L, const ReduceArgs& a, const LongCtx& c, uint32_t b, uint32_t p0,
                                            uint32_t pstride, uint32_t nrb, uint32_t rb, uint32_t sub, uint32_t shift,
                                            uint32_t& claims, uint32_t p_end = ~0u) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t pe = min(p_end, a.map_blocks);
  const uint32_t nj = p0 < pe ? (pe - p0 + pstride - 1) / pstride : 0u;  // <= 64 (pstride >= 16)
  const uint32_t cnt = lane < nj ? (uint32_t)L.runlong[p0 + lane * pstride] : 0u;
  const uint32_t incl = wave_incl_sum(cnt);
  const uint32_t N = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
  if (N == 0) return;
  const uint32_t P = incl - cnt;
  const uint32_t TOP = ((p0 + lane * pstride) * nrb + rb + 1) * sub - 1 + P;  // modular: TOP_j - t is exact
  const uint32_t SAFE = rb * sub;                                            // an index inside the store
  uint32_t jlo = 0;
  auto locate = [&](uint32_t T0, uint32_t& idx, bool& valid) {
    while (jlo + 1 < nj && (uint32_t)__builtin_amdgcn_readlane((int)P, (int)(jlo + 1)) <= T0) ++jlo;
    const uint32_t t = T0 + lane;
    idx = (uint32_t)__builtin_amdgcn_readlane((int)TOP, (int)jlo) - t;
    for (uint32_t jj = jlo + 1; jj < nj; ++jj) {  // runs starting inside this batch
      const uint32_t pj = (uint32_t)__builtin_amdgcn_readlane((int)P, (int)jj);
      if (pj >= T0 + 64) break;
      if (t >= pj) idx = (uint32_t)__builtin_amdgcn_readlane((int)TOP, (int)jj) - t;
    }
    valid = t < N;
  };
  auto load = [&](uint32_t idx, bool valid, Rec& r, uint64_t (&w)[8], uint32_t& wlen) {
    r = a.rec.recs[valid ? idx : SAFE];
    wlen = 0;
    if (valid) wlen = load_word64(c, (uint32_t)r.co, w);
  };
  auto merge = [&](const Rec& r, const uint64_t (&w)[8], uint32_t wlen, bool valid) {
    const uint32_t ph = place_hash(r.k0, r.k1), off = (uint32_t)r.co;
    int s = -1;
    if (valid && (!shift || bucket_of(ph, a.tab.log2_buckets) == b)) {
      bool cl;
      s = find_long_w(L, c, ph, r.k0, r.k1, off, w, wlen, cl);
      claims += cl ? 1u : 0u;
    }
    wave_add_long(L, s, r.co >> 32, a.chunk_base + off);
  };
  Rec ra, rb2;
  uint64_t wa[8], wb[8];
  uint32_t la, lb, ia, ib;
  bool va, vb;
  locate(0, ia, va);
  load(ia, va, ra, wa, la);
  for (uint32_t T0 = 0;; T0 += 128) {  // unrolled by two: the register sets swap roles without copies
    const bool more = T0 + 64 < N;
    if (more) {
      locate(T0 + 64, ib, vb);
      load(ib, vb, rb2, wb, lb);
    }
    merge(ra, wa, la, va);
    if (!more) return;
    const bool more2 = T0 + 128 < N;
    if (more2) {
      locate(T0 + 128, ia, va);
      load(ia, va, ra, wa, la);
    }
    merge(rb2, wb, lb, vb);
    if (!more2) return;
  }
}

// LONG records of this pass: the queued ones (every thread of the block takes
// entries), or — more than LONGQ in this bucket — a second, lean pass over the
// wave's 24-byte runs.  One record per lane per step, few live registers
// around the out-of-line merge_long, whose byte comparison reads global memory
// anyway.
__device__ __forceinline__ void long_queue(RedLds& L, const ReduceArgs& a, const LongCtx& c, uint32_t n,
                                           uint32_t& claims) {
  const uint32_t lane = threadIdx.x & 63;
  for (uint32_t i0 = threadIdx.x - lane; i0 < n; i0 += RED_THREADS) {  // wave-uniform: lanes stay converged
    const uint32_t i = i0 + lane;
    int s = -1;
    uint64_t cnt = 0, first = ~0ull;
    if (i < n) {
      const Rec r = a.rec.recs[L.longq[i]];
      const uint32_t off = (uint32_t)r.co;
      bool cl;
      s = find_long(L, c, place_hash(r.k0, r.k1), r.k0, r.k1, off, cl);
      claims += cl ? 1u : 0u;
      cnt = r.co >> 32;
      first = a.chunk_base + off;
    }
    wave_add_long(L, s, cnt, first);
  }
}

__device__ __forceinline__ void long_stream(RedLds& L, const ReduceArgs& a, const LongCtx& c, uint32_t b, uint32_t wave,
                                            uint32_t p0, uint32_t pstride, uint32_t nrb, uint32_t rb, uint32_t sub,
                                            uint32_t shift, uint32_t& claims) {
  // the queue is unused on this path: each wave compacts its LONG records'
  // indices into its 128-entry share of it and merges them 64 at a time (full
  // lanes: a wave's 24-byte runs mix LONG with medium words and hot flushes)
  static_assert(LONGQ >= 128 * (RED_THREADS / 64), "long_stream: 128 queue entries per wave");
  const uint32_t lane = threadIdx.x & 63;
  uint32_t* wl = L.longq + wave * 128;
  auto wsync = [] {  // this wave's LDS writes visible to its other lanes
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };
  auto merge_first = [&](uint32_t k) {  // wl[0, k), one per lane
    const uint64_t t0 = WC_RED_STAMPS ? __builtin_amdgcn_s_memtime() : 0;
    wsync();
    int s = -1;
    uint64_t cnt = 0, first = ~0ull;
    if (lane < k) {
      const Rec r = a.rec.recs[wl[lane]];
      const uint32_t off = (uint32_t)r.co;
      bool cl;
      s = find_long(L, c, place_hash(r.k0, r.k1), r.k0, r.k1, off, cl);
      claims += cl ? 1u : 0u;
      cnt = r.co >> 32;
      first = a.chunk_base + off;
    }
    wave_add_long(L, s, cnt, first);
    wsync();
    if (WC_RED_STAMPS && lane == 0) atomicAdd(&L.st[RS_T_SLOW], (unsigned long long)(__builtin_amdgcn_s_memtime() - t0));
  };
  uint32_t cnt = 0;  // wave-uniform
  for (uint32_t p = p0; p < a.map_blocks; p += pstride) {
    const uint32_t n = min(L.runcnt[p] >> 16, sub);
    const uint32_t base = ((uint32_t)p * nrb + rb) * sub;
    for (uint32_t i0 = 0; i0 < n; i0 += 64) {
      const uint32_t i = i0 + lane;
      bool isl = false;
      if (i < n) {
        const Rec r = a.rec.recs[base + i];
        isl = key_is_hashed(r.k1) && (!shift || bucket_of(place_hash(r.k0, r.k1), a.tab.log2_buckets) == b);
      }
      const uint64_t m = __ballot(isl);
      if (isl) wl[cnt + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u))] = base + i;
      cnt += (uint32_t)__popcll(m);
      if (cnt >= 64) {
        merge_first(64);
        const uint32_t rest = cnt - 64, moved = lane < rest ? wl[64 + lane] : 0u;
        wsync();
        if (lane < rest) wl[lane] = moved;
        cnt = rest;
      }
    }
  }
  if (cnt) merge_first(cnt);
}

// Split reduce, merge step: LONG rows are matched by key and then by bytes
// (colliding words keep separate slots); the references of both sides point at
// the chunk text (SREF_TEXT) or the key arena.
__device__ __forceinline__ bool refs_equal(const LongCtx& c, uint64_t so1, uint32_t l1, uint64_t so2, uint32_t l2) {
  if (l1 == SREF_POISON || l2 == SREF_POISON) return true;  // bytes lost (arena overflow): the key decides
  if (l1 != l2) return false;
  const uint8_t* p1 = (so1 & SREF_TEXT) ? c.text + (so1 & ~SREF_TEXT) : c.arena + so1;
  const uint8_t* p2 = (so2 & SREF_TEXT) ? c.text + (so2 & ~SREF_TEXT) : c.arena + so2;
  uint32_t i = 0;
  for (; i + 8 <= l1; i += 8) {
    uint64_t u, v;
    __builtin_memcpy(&u, p1 + i, 8);
    __builtin_memcpy(&v, p2 + i, 8);
    if (u != v) return false;
  }
  for (; i < l1; ++i)
    if (p1[i] != p2[i]) return false;
  return true;
}

__device__ __noinline__ void merge_long_row(RedLds& L, const LongCtx c, uint64_t k0, uint64_t k1, uint64_t cnt,
                                            uint64_t first, uint64_t so, uint32_t sl) {
  const uint32_t ph = place_hash(k0, k1), tag = make_tag(ph);
  const uint32_t g1 = group_of(ph, TAB_GROUPS), g2 = group2_of(ph, TAB_GROUPS);
  uint32_t g = g1;
  int steps = 0;
  for (;;) {
    asm volatile("" ::: "memory");
    SlotGroup& G = L.grp[g];
    const uint32_t tv[4] = {G.tag[0], G.tag[1], G.tag[2], G.tag[3]};
    bool pending = false;
    int e = -1;
    uint32_t mm = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (tv[i] == TAG_PENDING) pending = true;
      else if (tv[i] == TAG_EMPTY) e = e < 0 ? i : e;
      else if (tv[i] == tag && G.k1[i] == k1 && G.k0[i] == k0) mm |= 1u << i;
    }
    if (mm) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    while (mm) {
      const int i = __ffs(mm) - 1;
      mm &= mm - 1;
      const int s = 4 * (int)g + i;
      if (refs_equal(c, so, sl, c.sref_off[s], c.sref_len[s])) {
        add_to_slot(L, s, cnt, first);
        return;
      }
    }
    if (pending) continue;
    if (e >= 0) {
      if (atomicCAS(&G.tag[e], TAG_EMPTY, TAG_PENDING) != TAG_EMPTY) continue;
      const int s = 4 * (int)g + e;
      G.k0[e] = k0;
      G.k1[e] = k1;
      c.sref_off[s] = so;
      c.sref_len[s] = sl;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __hip_atomic_store(&G.tag[e], tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      add_to_slot(L, s, cnt, first);
      return;
    }
    if (++steps >= TAB_MAX_GROUP_PROBES) {
      L.overflow = 1;
      return;
    }
    g = probe_group(g1, g2, (uint32_t)steps, TAB_GROUPS);
  }
}


// Split reduce: this quarter's partial is published (or it overflowed); count
// the bucket's arrivals — true for the last quarter, which then sees every
// other quarter's partial (agent-scope release by each arrival, acquire by the
// last; the counter is reset for the next launch).
// One agent-scope acq_rel atomic per block (MI355X_MICROARCH.md: one lane per
// storing workgroup, behind a workgroup barrier; the other waves load after a
// barrier that lane joins) — a fence per wave wrote the XCD's L2 back 16 times
// per block (reduce 214 -> 395 us).
__device__ bool split_arrive_last(RedLds& L, const ReduceArgs& a, uint32_t b, uint32_t pieces) {
  __shared__ uint32_t last;
  // every storing wave waits for its own partial-row stores before the barrier
  // behind which one lane signals (MI355X_MICROARCH.md hand-off table, row 1)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t old = __hip_atomic_fetch_add(&a.part.done[b], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    last = old + 1 == pieces ? 1u : 0u;
    if (last) a.part.done[b] = 0;
  }
  __syncthreads();
  if (!last) return false;
  return a.bucket_overflow[b] == 0;  // a quarter overflowed: the host splits the table and re-runs the bucket
}

// Exclusive block-wide prefix of one value per thread (every thread calls).
__device__ __forceinline__ uint32_t block_scan_excl(uint32_t v, uint32_t& total) {
  __shared__ uint32_t ws[RED_THREADS / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t incl = v;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(incl, o);
    if (lane >= o) incl += y;
  }
  if (lane == 63) ws[wave] = incl;
  __syncthreads();
  uint32_t before = 0;
  total = 0;
  for (int w = 0; w < RED_THREADS / 64; ++w) {
    before += w < wave ? ws[w] : 0u;
    total += ws[w];
  }
  __syncthreads();  // ws is reused by the next call
  return before + incl - v;
}

// The last piece of a bucket inserts the other pieces' partial rows (the
// first piece's include the running slice) into its own table — inline keys
// by key, LONG words by key and bytes — and recounts the occupancy.  slots: the
// other pieces' partial slots (np <= 1024, in LDS: L.longq[0, np), which this
// overwrites past 1024).  False on overflow.
__device__ bool merge_partials(RedLds& L, const ReduceArgs& a, const LongCtx& c, uint32_t b, const uint32_t* slots,
                               uint32_t np) {
  const int tid = threadIdx.x;
  uint32_t* pn = L.longq + 1024;  // row prefix of the partials: pn[k], pn[np] = total
  {
    const uint32_t n = (uint32_t)tid < np ? a.part.n[slots[tid]] : 0u;
    uint32_t tot;
    const uint32_t ex = block_scan_excl(n, tot);
    if ((uint32_t)tid < np) pn[tid] = ex;
    if (tid == 0) pn[np] = tot;
  }
  __syncthreads();
  const uint32_t total = pn[np];
  const ReduceArgs::Parts& P = a.part;
#ifndef WC_MERGE_R
#define WC_MERGE_R 4
#endif
  constexpr int R = WC_MERGE_R;  // rows per thread per round, loaded together
  for (uint32_t r0 = 0; r0 < total; r0 += R * RED_THREADS) {
    uint64_t k0[R], k1[R], cnt[R], first[R];
    size_t at[R];
    bool v[R];
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const uint32_t i = r0 + j * RED_THREADS + tid;
      v[j] = i < total;
      uint32_t lo = 0, hi = np ? np - 1 : 0;  // the partial holding row i: largest k with pn[k] <= i
      while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (pn[mid] <= i) lo = mid;
        else hi = mid - 1;
      }
      at[j] = (size_t)slots[lo] * TAB_SLOTS + (i - pn[lo]);
      if (v[j]) {
        k0[j] = P.k0[at[j]];
        k1[j] = P.k1[at[j]];
        cnt[j] = P.cnt[at[j]];
        first[j] = P.first[at[j]];
      }
    }
#pragma unroll
    for (int j = 0; j < R; ++j) {
      if (!v[j]) continue;
      if (key_is_hashed(k1[j])) {
        merge_long_row(L, c, k0[j], k1[j], cnt[j], first[j], P.soff[at[j]], P.slen[at[j]]);
      } else {
        bool claimed;
        const int s = lds_find_or_claim(L.grp, TAB_GROUPS, place_hash(k0[j], k1[j]), k0[j], k1[j],
                                        TAB_MAX_GROUP_PROBES, claimed, true);
        if (s < 0) L.overflow = 1;
        else add_to_slot(L, s, cnt[j], first[j]);
      }
    }
  }
  __syncthreads();
  if (tid == 0) L.occupied = 0;
  __syncthreads();
  uint32_t occ = 0;
  for (int s = tid; s < TAB_SLOTS; s += RED_THREADS) occ += slot_tag(L.grp, s) > TAG_PENDING ? 1u : 0u;
  for (int o = 32; o > 0; o >>= 1) occ += __shfl_down(occ, o);
  if ((tid & 63) == 0 && occ) atomicAdd(&L.occupied, occ);
  __syncthreads();
  if (L.overflow || L.occupied > (uint32_t)TAB_MAX_OCC) {
    if (tid == 0) {
      a.bucket_overflow[b] = 1;
      atomicOr(&a.flags[FLAG_TABLE_OVF], 1u);
    }
    return false;
  }
  return true;
}

// The finalize's first-occurrence bins come from this exact histogram of the
// stored keys' log-bins (sort.hip wc_fo_bin).
__device__ __forceinline__ void add_fo_hist(const RedLds& L, const ReduceArgs& a) {
  if (!a.fo_hist) return;
  for (int s = threadIdx.x; s < TAB_SLOTS; s += RED_THREADS)
    if (slot_tag(L.grp, s) > TAG_PENDING) atomicAdd(&a.fo_hist[fo_logbin(L.first[s], a.fo_m)], 1u);
}

// The last pass before a bitmap-rank order: the stored keys' bits (atomic ORs
// without return, overlapped with the rest of the reduce) and their count.
__device__ __forceinline__ void add_bm_bits(const RedLds& L, const ReduceArgs& a) {
  if (!a.bm) return;
  // the thread's TAB_SLOTS / RED_THREADS slots: every returning OR issued before
  // any result is looked at (one device round trip, not one per slot: in a
  // loop that tested each OR before the next, the bits took ~33 us of a v1m /
  // long30 bucket's ~450 us, profiles/r6_session.md §11)
  constexpr int PER = TAB_SLOTS / RED_THREADS;
  bool range = false;
  unsigned long long m[PER], old[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int s = threadIdx.x + j * RED_THREADS;
    m[j] = 0;
    old[j] = 0;
    if (slot_tag(L.grp, s) <= TAG_PENDING) continue;
    const uint64_t p = L.first[s] >> a.bm_shift;
    if (p >= a.bm_pos_end) {
      range = true;
      continue;
    }
    m[j] = 1ull << (p & 63);
    old[j] = __hip_atomic_fetch_or(&a.bm[p >> 6], m[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_add(&a.bm_lines[p >> 9], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
#pragma unroll
  for (int j = 0; j < PER; ++j)
    if (old[j] & m[j]) range = true;
  if (range) atomicOr(a.bm_ctl, 1ull << 63);  // the order's redo flag (out of bounds, or a shared position)
  if (threadIdx.x == 0 && L.occupied) atomicAdd(a.bm_ctl, (unsigned long long)L.occupied);
}

// Split reduce: a quarter's occupied slots -> its part rows (slot order, a
// block scan places them; LONG rows carry their arena / text reference).
__device__ void write_partial(const RedLds& L, const ReduceArgs& a, const LongCtx& c, uint32_t pb) {
  __shared__ uint32_t wsum[RED_THREADS / 64];
  static_assert(TAB_SLOTS == 4 * RED_THREADS, "partial: 4 slots per thread");
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  bool occ[4];
  uint32_t n = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    occ[j] = slot_tag(L.grp, 4 * tid + j) > TAG_PENDING;
    n += occ[j] ? 1u : 0u;
  }
  uint32_t incl = n;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(incl, o);
    if (lane >= o) incl += y;
  }
  if (lane == 63) wsum[wave] = incl;
  __syncthreads();
  uint32_t before = 0, total = 0;
  for (int w = 0; w < RED_THREADS / 64; ++w) {
    before += w < wave ? wsum[w] : 0u;
    total += wsum[w];
  }
  size_t o = (size_t)pb * TAB_SLOTS + before + incl - n;
  const ReduceArgs::Parts& P = a.part;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (!occ[j]) continue;
    const int s = 4 * tid + j;
    const uint64_t k1 = slot_k1(L.grp, s);
    P.k0[o] = slot_k0(L.grp, s);
    P.k1[o] = k1;
    P.cnt[o] = L.cnt[s];
    P.first[o] = L.first[s];
    if (key_is_hashed(k1)) {
      P.soff[o] = c.sref_off[s];
      P.slen[o] = c.sref_len[s];
    }
    ++o;
  }
  if (tid == 0) P.n[pb] = total;
}

// Exclusive block-wide prefix of a 64-bit value per thread (every thread calls).
__device__ __forceinline__ uint64_t block_scan_excl64(uint64_t v, uint64_t& total) {
  __shared__ uint64_t ws[RED_THREADS / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint64_t incl = v;
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t y = __shfl_up(incl, o);
    if (lane >= o) incl += y;
  }
  if (lane == 63) ws[wave] = incl;
  __syncthreads();
  uint64_t before = 0;
  total = 0;
  for (int w = 0; w < RED_THREADS / 64; ++w) {
    before += w < wave ? ws[w] : 0ull;
    total += ws[w];
  }
  __syncthreads();
  return before + incl - v;
}

// The reduce's dispatch plan (ReduceArgs::bucket_w; profiles/r5_session.md §4):
// every block derives the same plan from the map's per-bucket weights.
// bucket b gets floor(w_b (G - B) / W) + 1 pieces (<= RED_SPLIT_MAX_Q): the
// G - B extra blocks go to the buckets by weight share, so only a bucket above
// W / (G - B) is split.  (Splitting every bucket above 1.5x the mean at
// long30_v1m — 512 buckets, 2 dispatch rounds on 256 CUs — pushed the pieces
// past 2 x CUs into a third round: 446.9 vs 451.0 GB/s, profiles/r5_session.md §12.)
// Pieces are dispatched heaviest first (8 classes of a quarter of the mean
// piece each, then bucket order): with more pieces than CUs the heavy ones no
// longer start in the last wave (at 30 % LONG vocabulary one bucket at 2.4x
// the mean did).  Block i -> (bucket, piece, pieces, the block index of the
// bucket's piece 0 = its partial slots); false: no piece.
__device__ __forceinline__ bool lpt_piece(const ReduceArgs& a, uint32_t& b, uint32_t& q, uint32_t& nq, uint32_t& base) {
  __shared__ uint32_t pl[4];
  const uint32_t tid = threadIdx.x, nb = 1u << a.tab.log2_buckets, i = blockIdx.x, G = gridDim.x;
  // a bucket's weight stays below 2^32 (<= 1024 map blocks x 65535 records x
  // RED_WLONG per run), the sum over 512 buckets does not: 64-bit total, and
  // every bucket weighs >= 1, so W > 0
  const uint64_t w = tid < nb ? (uint64_t)a.bucket_w[tid] + 1u : 0u;
  uint64_t W;
  (void)block_scan_excl64(w, W);
  uint32_t n = tid < nb ? 1u : 0u;
  if (tid < nb) n = (uint32_t)min<uint64_t>(RED_SPLIT_MAX_Q, w * (G - nb) / W + 1);
  uint32_t P;
  (void)block_scan_excl(n, P);
  if (P > G) {  // no room for the extra pieces: one per bucket, order only
    n = tid < nb ? 1u : 0u;
    P = nb;
  }
  // class of the piece weight in quarters of the mean piece (7: >= 1.75x), heaviest first
  const uint32_t cls = tid < nb ? (uint32_t)min<uint64_t>(7, 4ull * w * P / (W * n)) : 0u;
  // pieces before b inside its class: two 64-bit scans of 16-bit per-class counters
  const uint64_t v = (uint64_t)n << (16 * (cls & 3));
  uint64_t tlo, thi;
  const uint64_t plo = block_scan_excl64(cls < 4 ? v : 0ull, tlo);
  const uint64_t phi = block_scan_excl64(cls >= 4 ? v : 0ull, thi);
  uint32_t before = 0;  // pieces of the heavier classes
  for (uint32_t k = 7; k > cls; --k) before += (uint32_t)(((k < 4 ? tlo : thi) >> (16 * (k & 3))) & 0xFFFFu);
  const uint32_t mine = (uint32_t)(((cls < 4 ? plo : phi) >> (16 * (cls & 3))) & 0xFFFFu);
  const uint32_t first = before + mine;
  if (tid == 0) pl[0] = ~0u;
  __syncthreads();
  if (tid < nb && first <= i && i < first + n) {
    pl[0] = tid;
    pl[1] = i - first;
    pl[2] = n;
    pl[3] = first;
  }
  __syncthreads();
  if (pl[0] == ~0u) return false;
  b = pl[0];
  q = pl[1];
  nq = pl[2];
  base = pl[3];
  return true;
}

// LD: the pass's map wrote LONG records top-down (MapArgs::long_direct) and
// they stream through long_direct; otherwise they sit in the 24-byte runs and
// merge_batch queues them (an instance without long_direct's code).
template <bool LD>
__global__ void __launch_bounds__(RED_THREADS) wc_reduce_buckets(ReduceArgs a) {
  __shared__ RedLds L;
  if (a.flags[FLAG_REGION_OVF]) return;  // shuffle output incomplete: host re-runs the chunk
  // block b + B q: bucket b, quarter q (split reduce, a.nq > 1) of the map blocks' runs;
  // with bucket weights, the dispatch plan's piece instead (lpt_piece)
  uint32_t b = blockIdx.x & ((1u << a.tab.log2_buckets) - 1u), q = blockIdx.x >> a.tab.log2_buckets;
  uint32_t nq = a.nq, pbase = b, pstep = 1u << a.tab.log2_buckets;  // partial slot of quarter q': pbase + q' pstep
  if (a.bucket_w) {
    uint32_t base;
    if (!lpt_piece(a, b, q, nq, base)) return;
    b = __builtin_amdgcn_readfirstlane(b);
    q = __builtin_amdgcn_readfirstlane(q);
    nq = __builtin_amdgcn_readfirstlane(nq);
    pbase = __builtin_amdgcn_readfirstlane(base);
    pstep = 1;
  }
  if (a.bucket_enable && !a.bucket_enable[b]) return;
  const int tid = threadIdx.x, wave = tid >> 6, nwaves = RED_THREADS / 64;
  const bool split = nq > 1;
  load_slice(L, a.tab, b, q != 0);  // quarters q > 0 start empty
  {
    const uint32_t rb0 = b & ((1u << a.log2_rec_buckets) - 1u), nrb0 = 1u << a.log2_rec_buckets;
    for (uint32_t p = tid; p < a.map_blocks; p += RED_THREADS) {
      L.runcnt[p] = a.rec.count[(size_t)p * nrb0 + rb0];
      if (LD) L.runlong[p] = (uint16_t)a.rec.count_long[(size_t)p * nrb0 + rb0];
    }
  }
  if (tid == 0) {
    L.occupied = q == 0 ? a.tab.occupancy[b] : 0u;
    L.overflow = 0;
    L.nlong = 0;
  }
  if (WC_RED_STAMPS && tid < RED_STAMP_N) L.st[tid] = 0;
  __syncthreads();
  const uint64_t t_start = WC_RED_STAMPS ? __builtin_amdgcn_s_memtime() : 0;
  const uint64_t rt_start = WC_RED_STAMPS ? __builtin_amdgcn_s_memrealtime() : 0;  // 100 MHz, one clock for every XCD

  const uint32_t shift = a.tab.log2_buckets - a.log2_rec_buckets;  // table buckets per record bucket (log2)
  const uint32_t rb = b & ((1u << a.log2_rec_buckets) - 1u);       // buckets nest on the low bits
  const uint32_t nrb = 1u << a.log2_rec_buckets;
  const uint64_t sub = a.rec.subcap;
  // one contiguous run per map block: sub-region (p, rb) of the record store;
  // the wave streams the 16-byte records of its runs, then the 24-byte ones
  uint32_t claims = 0;
  const uint32_t p0 = q + nq * wave, pstride = nq * nwaves;  // this wave's runs
  merge_stream<true, RED_UNROLL>(L, a, b, a.rec.recs16, p0, pstride, nrb, rb, (uint32_t)sub, shift, claims);
  merge_stream<false, RED_UNROLL_24>(L, a, b, a.rec.recs, p0, pstride, nrb, rb, (uint32_t)sub, shift, claims);
  __syncthreads();  // every LONG record is queued (or counted past the queue)
  if (WC_RED_STAMPS && (tid & 63) == 0)
    atomicAdd(&L.st[RS_T_STREAMS], (unsigned long long)(__builtin_amdgcn_s_memtime() - t_start));
  if (WC_RED_STAMPS && tid == 0) {
    L.st[RS_NLONG] = L.nlong;
    L.st[RS_LONG_STREAMED] = L.nlong > LONGQ ? 1 : 0;
  }
  // LONG words' arena references: the slice's (q = 0) or the quarter's own scratch
  const size_t sbase = (size_t)b * TAB_SLOTS, qbase = (size_t)blockIdx.x * TAB_SLOTS;
  const LongCtx lc{a.text, a.avail_len, a.arena.bytes, q == 0 ? a.tab.sref_off + sbase : a.part.qsoff + qbase,
                   q == 0 ? a.tab.sref_len + sbase : a.part.qslen + qbase};
  if (L.nlong) {  // LONG records inside the 24-byte runs (none since the map fills LONG ones top-down)
    if (L.nlong <= LONGQ) long_queue(L, a, lc, L.nlong, claims);
    else long_stream(L, a, lc, b, wave, p0, pstride, nrb, rb, (uint32_t)sub, shift, claims);
  }
  if constexpr (LD) long_direct(L, a, lc, b, p0, pstride, nrb, rb, (uint32_t)sub, shift, claims);
  for (int o = 32; o > 0; o >>= 1) claims += __shfl_down(claims, o);
  if ((tid & 63) == 0 && claims) atomicAdd(&L.occupied, claims);
  if (WC_RED_STAMPS && (tid & 63) == 0)
    atomicAdd(&L.st[RS_T_RUNS], (unsigned long long)(__builtin_amdgcn_s_memtime() - t_start));
  __syncthreads();
  if (tid == 0 && L.occupied > (uint32_t)TAB_MAX_OCC) L.overflow = 1;  // too full: split and re-run
  __syncthreads();
  if (L.overflow && tid == 0) {
    a.bucket_overflow[b] = 1;
    atomicOr(&a.flags[FLAG_TABLE_OVF], 1u);
  }
  bool store = !L.overflow;
  const uint64_t rt_streams = WC_RED_STAMPS ? __builtin_amdgcn_s_memrealtime() : 0;
  uint64_t rt_arrive = rt_streams;
  if (split) {
    // every quarter publishes its partial table; the last to arrive merges the
    // others into its own LDS table and stores the bucket
    if (!L.overflow) write_partial(L, a, lc, blockIdx.x);
    store = split_arrive_last(L, a, b, nq);
    if (WC_RED_STAMPS) rt_arrive = __builtin_amdgcn_s_memrealtime();
    if (store) {
      if (tid == 0) {  // the other quarters' partial slots
        uint32_t k = 0;
        for (uint32_t qq = 0; qq < nq; ++qq)
          if (qq != q) L.longq[k++] = pbase + pstep * qq;
        L.nlong = k;  // scratch: the slot count
      }
      __syncthreads();
      store = merge_partials(L, a, lc, b, L.longq, L.nlong);
    }
    if (store && q != 0) {  // the merged table's LONG references: quarter scratch -> the slice
      for (int s = tid; s < TAB_SLOTS; s += RED_THREADS) {
        if (slot_tag(L.grp, s) > TAG_PENDING && key_is_hashed(slot_k1(L.grp, s))) {
          a.tab.sref_off[sbase + s] = lc.sref_off[s];
          a.tab.sref_len[sbase + s] = lc.sref_len[s];
        }
      }
      __syncthreads();
    }
  }
  const uint64_t rt_merged = WC_RED_STAMPS ? __builtin_amdgcn_s_memrealtime() : 0;
  uint64_t rt_stored = rt_merged;
  if (store) {
    settle_new_long(L, a, b);
    store_slice(L, a.tab, b);
    if (WC_RED_STAMPS) rt_stored = __builtin_amdgcn_s_memrealtime();
    add_fo_hist(L, a);
    add_bm_bits(L, a);
    if (tid == 0) {
      a.tab.occupancy[b] = L.occupied;
      atomicMax(&a.flags[FLAG_MAX_OCC], L.occupied);
    }
  }
  if (WC_RED_STAMPS && a.stamps) {
    if ((tid & 63) == 0) atomicAdd(&L.st[RS_T_WAVE], (unsigned long long)(__builtin_amdgcn_s_memtime() - t_start));
    __syncthreads();
    if (tid == 0) {
      L.st[RS_BLOCKS] = 1;
      L.st[RS_T_BLKMAX] = 0;
      atomicMax(&a.stamps[RS_T_BLKMAX], (unsigned long long)(__builtin_amdgcn_s_memtime() - t_start));
    }
    __syncthreads();
    if (tid < RED_STAMP_N) atomicAdd(&a.stamps[tid], L.st[tid]);
    if (a.blk && tid == 0) {  // where the reduce's time goes, block by block
      const uint32_t nrb0 = 1u << a.log2_rec_buckets;
      unsigned long long n16 = 0, n24 = 0, nl = L.st[RS_NLONG];
      for (uint32_t p = q; p < a.map_blocks; p += nq) {
        n16 += L.runcnt[p] & 0xFFFFu;
        n24 += L.runcnt[p] >> 16;
        if (LD) nl += L.runlong[p];  // top-down LONG records (inside the 24-byte count)
      }
      (void)nrb0;
      unsigned long long* r = a.blk + (size_t)RED_BLK_WORDS * blockIdx.x;
      r[0] = b | ((unsigned long long)q << 32);
      r[1] = rt_start;
      r[2] = __builtin_amdgcn_s_memrealtime();
      r[3] = n16 | (n24 << 32);
      r[4] = nl;
      r[5] = rt_streams;
      r[6] = rt_arrive;
      r[7] = rt_merged;
      r[8] = rt_stored;
    }
  }
}


// Rehash parent slice (new_b mod B) of `src` into slice new_b of `dst` (2B
// buckets).  Source slots hold distinct words, so every one claims a fresh
// slot (colliding LONG keys stay apart).
__global__ void __launch_bounds__(RED_THREADS) wc_table_split(TableView src, TableView dst) {
  __shared__ RedLds L;
  const uint32_t nb = blockIdx.x, ob = nb & ((1u << src.log2_buckets) - 1u);
  for (int s = threadIdx.x; s < TAB_SLOTS; s += blockDim.x) {
    L.grp[s >> 2].tag[s & 3] = TAG_EMPTY;
    L.cnt[s] = 0;
    L.first[s] = ~0ull;
  }
  if (threadIdx.x == 0) L.occupied = 0;
  __syncthreads();
  const size_t obase = (size_t)ob * TAB_SLOTS, nbase = (size_t)nb * TAB_SLOTS;
  const bool parent_empty = src.occupancy[ob] == 0;  // contents undefined (see load_slice)
  for (int s = threadIdx.x; s < TAB_SLOTS && !parent_empty; s += blockDim.x) {
    const uint64_t k1 = src.k1[obase + s];
    if (k1 == K1_EMPTY) continue;
    const uint64_t k0 = src.k0[obase + s];
    const uint32_t ph = place_hash(k0, k1);
    if (bucket_of(ph, dst.log2_buckets) != nb) continue;
    bool claimed;
    const int d = lds_find_or_claim(L.grp, TAB_GROUPS, ph, k0, k1, TAB_GROUPS, claimed, false);
    // d >= 0 always: a child receives at most the parent's occupancy.
    L.cnt[d] = src.cnt[obase + s];
    L.first[d] = src.first[obase + s];
    dst.sref_off[nbase + d] = src.sref_off[obase + s];
    dst.sref_len[nbase + d] = src.sref_len[obase + s];
    atomicAdd(&L.occupied, 1u);
  }
  __syncthreads();
  store_slice(L, dst, nb);
  if (threadIdx.x == 0) dst.occupancy[nb] = L.occupied;
}

// Debug (WC_CHECK_TABLE=1, Engine::Impl::check_table): the running table's
// invariants — a bucket with occupancy > 0 holds exactly that many keys (k1 !=
// K1_EMPTY: the compaction, the order and the gather size their output from
// the occupancy) and every key hashes to its own bucket.  err = {1 + the first
// bad bucket (0: none), keys found, its occupancy, misplaced keys}.
__global__ void __launch_bounds__(1024) wc_check_table(TableView t, unsigned long long* err) {
  __shared__ uint32_t cnt, bad;
  const uint32_t b = blockIdx.x;
  const uint32_t occ = t.occupancy[b];
  if (occ == 0) return;  // contents undefined (see load_slice)
  if (threadIdx.x == 0) cnt = bad = 0;
  __syncthreads();
  const size_t base = (size_t)b * TAB_SLOTS;
  for (int s = threadIdx.x; s < TAB_SLOTS; s += blockDim.x) {
    const uint64_t k1 = t.k1[base + s];
    if (k1 == K1_EMPTY) continue;
    atomicAdd(&cnt, 1u);
    if (bucket_of(place_hash(t.k0[base + s], k1), t.log2_buckets) != b) atomicAdd(&bad, 1u);
  }
  __syncthreads();
  if (threadIdx.x == 0 && (cnt != occ || bad)) {
    if (atomicCAS(&err[0], 0ull, (unsigned long long)b + 1) == 0ull) {
      err[1] = cnt;
      err[2] = occ;
      err[3] = bad;
    }
  }
}

__global__ void wc_table_clear(TableView t, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    t.k1[i] = K1_EMPTY;
    t.cnt[i] = 0;
    t.first[i] = ~0ull;
    if (i < ((size_t)1 << t.log2_buckets)) t.occupancy[i] = 0;
  }
}

// One 1024-thread block per bucket: thread t owns slots [4t, 4t+4) of the
// slice; a block scan of the occupied counts places them at bucket_off[b] + rank
// (bucket order, slot order inside a bucket).  No global atomics: the previous
// one-counter-per-wave form serialised ~16k waves on one address (~200 us).
__global__ void __launch_bounds__(1024) wc_table_compact(TableView t, const uint64_t* bucket_off, uint64_t* k0,
                                                         uint64_t* k1, uint64_t* cnt, uint64_t* first,
                                                         uint64_t* sref_off, uint32_t* sref_len, Bounds bnd) {
  static_assert(TAB_SLOTS == 4 * 1024, "compact: 4 slots per thread");
  __shared__ uint32_t wsum[16];
  const uint32_t b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const size_t base = (size_t)b * TAB_SLOTS + 4 * tid;
  if (t.occupancy[b] == 0) return;  // contents undefined (see load_slice); no keys
  uint64_t kk1[4];
  uint32_t n = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    kk1[j] = t.k1[base + j];
    n += kk1[j] != K1_EMPTY;
  }
  uint32_t incl = n;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(incl, o);
    if (lane >= o) incl += y;
  }
  if (lane == 63) wsum[wave] = incl;
  __syncthreads();
  uint32_t before = 0;
  for (uint32_t w = 0; w < wave; ++w) before += wsum[w];
  uint64_t o = bucket_off[b] + before + incl - n;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (kk1[j] == K1_EMPTY) continue;
    const size_t i = base + j;
    const bool h = key_is_hashed(kk1[j]);
    if (!bounds_ok(bnd, BND_COMPACT, o)) break;
    k0[o] = t.k0[i];
    k1[o] = kk1[j];
    cnt[o] = t.cnt[i];
    first[o] = t.first[i];
    sref_off[o] = h ? t.sref_off[i] : 0;
    sref_len[o] = h ? t.sref_len[i] : 0;
    ++o;
  }
}

// As wc_table_compact, but only (first offset, global slot index) per key.
__global__ void __launch_bounds__(1024) wc_table_keys(TableView t, const uint64_t* bucket_off, uint64_t* keys,
                                                      uint32_t* slots, Bounds bnd) {
  __shared__ uint32_t wsum[16];
  const uint32_t b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const size_t base = (size_t)b * TAB_SLOTS + 4 * tid;
  if (t.occupancy[b] == 0) return;  // contents undefined (see load_slice); no keys
  bool occ[4];
  uint32_t n = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    occ[j] = t.k1[base + j] != K1_EMPTY;
    n += occ[j];
  }
  uint32_t incl = n;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(incl, o);
    if (lane >= o) incl += y;
  }
  if (lane == 63) wsum[wave] = incl;
  __syncthreads();
  uint32_t before = 0;
  for (uint32_t w = 0; w < wave; ++w) before += wsum[w];
  uint64_t o = bucket_off[b] + before + incl - n;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (!occ[j]) continue;
    if (!bounds_ok(bnd, BND_TABLE_KEYS, o)) break;
    keys[o] = t.first[base + j];
    slots[o] = (uint32_t)(base + j);
    ++o;
  }
}

// One block: bucket_off = exclusive scan of occupancy, *n = the total.
__global__ void __launch_bounds__(1024) wc_bucket_offsets(const uint32_t* occ, uint32_t nb, uint64_t* off,
                                                          uint64_t* n) {
  __shared__ uint64_t wsum[16];
  __shared__ uint64_t carry;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid == 0) carry = 0;
  __syncthreads();
  for (uint32_t c = 0; c < nb; c += 1024) {
    const uint32_t b = c + tid;
    const uint64_t v = b < nb ? occ[b] : 0;
    uint64_t incl = v;
    for (int o = 1; o < 64; o <<= 1) {
      const uint64_t y = __shfl_up(incl, o);
      if ((int)lane >= o) incl += y;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    uint64_t before = carry;
    for (uint32_t w = 0; w < wave; ++w) before += wsum[w];
    if (b < nb) off[b] = before + incl - v;
    __syncthreads();
    if (tid == 0) {
      uint64_t t = 0;
      for (int w = 0; w < 16; ++w) t += wsum[w];
      carry += t;
    }
    __syncthreads();
  }
  if (tid == 0) *n = carry;
}

// Sorted (first, slot) pairs -> the six key columns, read from the table.
__global__ void wc_gather_table(TableView t, const uint64_t* keys, const uint32_t* slots, uint64_t n,
                                const uint64_t* dn, uint64_t* ok0, uint64_t* ok1, uint64_t* ocnt, uint64_t* ofirst,
                                uint64_t* osoff, uint32_t* oslen, Bounds bnd) {
  if (dn) n = *dn;
  const Bounds tab{bnd.err, (uint64_t)TAB_SLOTS << t.log2_buckets};
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t j = slots[i];
    if (!bounds_ok(bnd, BND_GATHER_TABLE, i) || !bounds_ok(tab, BND_GATHER_TABLE, j)) continue;
    const uint64_t k1 = t.k1[j];
    const bool h = key_is_hashed(k1);
    ok0[i] = t.k0[j];
    ok1[i] = k1;
    ocnt[i] = t.cnt[j];
    ofirst[i] = keys[i];
    osoff[i] = h ? t.sref_off[j] : 0;
    oslen[i] = h ? t.sref_len[j] : 0;
  }
}

}  // namespace dev

void launch_table_keys(const TableView& t, const uint64_t* bucket_off, uint64_t* keys, uint32_t* slots, hipStream_t s,
                       const Bounds& bnd) {
  hipLaunchKernelGGL(dev::wc_table_keys, dim3(1u << t.log2_buckets), dim3(1024), 0, s, t, bucket_off, keys, slots, bnd);
}
void launch_gather_table(const TableView& t, const uint64_t* keys, const uint32_t* slots, uint64_t n, uint64_t* ok0,
                         uint64_t* ok1, uint64_t* ocnt, uint64_t* ofirst, uint64_t* osoff, uint32_t* oslen,
                         hipStream_t s, const uint64_t* dn, const Bounds& bnd) {
  if (!n) return;
  uint64_t g = (n + 255) / 256;
  g = g > 4096 ? 4096 : g;
  hipLaunchKernelGGL(dev::wc_gather_table, dim3((unsigned)g), dim3(256), 0, s, t, keys, slots, n, dn, ok0, ok1, ocnt,
                     ofirst, osoff, oslen, bnd);
}
void launch_bucket_offsets(const uint32_t* occupancy, uint32_t nb, uint64_t* bucket_off, uint64_t* n, hipStream_t s) {
  hipLaunchKernelGGL(dev::wc_bucket_offsets, dim3(1), dim3(1024), 0, s, occupancy, nb, bucket_off, n);
}

void launch_reduce(const ReduceArgs& a, hipStream_t s, uint32_t extra) {
  WC_CHECK(a.nq >= 1 && a.nq <= RED_SPLIT_MAX_Q, "reduce: 1..RED_SPLIT_MAX_Q blocks per bucket");
  const uint32_t grid = (1u << a.tab.log2_buckets) * a.nq + (a.bucket_w ? extra : 0u);
  WC_CHECK(!a.bucket_w || (a.nq == 1 && a.tab.log2_buckets == a.log2_rec_buckets && !a.bucket_enable &&
                           (1u << a.tab.log2_buckets) <= (uint32_t)MAX_REC_BUCKETS && grid <= a.part_slots &&
                           (1u << a.tab.log2_buckets) <= (uint32_t)RED_THREADS),
           "reduce dispatch plan: one record bucket per table bucket, <= MAX_REC_BUCKETS, a partial slot per block");
  if (a.long_direct) hipLaunchKernelGGL(dev::wc_reduce_buckets<true>, dim3(grid), dim3(RED_THREADS), 0, s, a);
  else hipLaunchKernelGGL(dev::wc_reduce_buckets<false>, dim3(grid), dim3(RED_THREADS), 0, s, a);
}


void launch_table_split(const TableView& src, const TableView& dst, hipStream_t s) {
  hipLaunchKernelGGL(dev::wc_table_split, dim3(1u << dst.log2_buckets), dim3(RED_THREADS), 0, s, src, dst);
}

void launch_check_table(const TableView& t, unsigned long long* err, hipStream_t s) {
  hipLaunchKernelGGL(dev::wc_check_table, dim3(1u << t.log2_buckets), dim3(1024), 0, s, t, err);
}

void launch_table_clear(const TableView& t, hipStream_t s) {
  const size_t n = ((size_t)1 << t.log2_buckets) * TAB_SLOTS;
  hipLaunchKernelGGL(dev::wc_table_clear, dim3(1024), dim3(256), 0, s, t, n);
}

void launch_table_compact(const TableView& t, const uint64_t* bucket_off, uint64_t* k0, uint64_t* k1, uint64_t* cnt,
                          uint64_t* first, uint64_t* sref_off, uint32_t* sref_len, hipStream_t s, const Bounds& bnd) {
  hipLaunchKernelGGL(dev::wc_table_compact, dim3(1u << t.log2_buckets), dim3(1024), 0, s, t, bucket_off, k0, k1, cnt,
                     first, sref_off, sref_len, bnd);
}

const char* bounds_kernel_name(uint32_t k) {
  static const char* names[BND_KERNELS] = {"none",           "wc_fo_sort",    "wc_bm_place",      "wc_bm_emit",
                                           "wc_gather_cols", "wc_table_keys", "wc_gather_table", "wc_table_compact"};
  return k < BND_KERNELS ? names[k] : "unknown";
}

}  // namespace wc
