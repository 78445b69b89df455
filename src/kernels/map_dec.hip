// map_dec.hip — wc_map_decoupled: the MAP stage with wave-decoupled text units.
//
// Same tokenizer, keys, combiner and shuffle write as map.hip (the building
// blocks live in map_common.hpp), but without block-wide tiles: each of the 16
// waves of a block owns a private LDS buffer holding one 2 KiB text UNIT (+64 B
// halo), grabs its next unit from the block's LDS cursor and prefetches it into
// registers while tokenizing the current one.  Waves therefore never wait for
// each other at a tile boundary (map.hip's phase clock: ~25 % of wave time was
// spent at per-tile barriers).  The only block-wide synchronisation is the
// combiner flush.  The table admits new keys until DEC_ADMIT_AT slots are
// occupied; after that a token whose key is absent (or whose probe sequence is
// full) becomes a record of its own, written straight to the shuffle store, so
// no token ever waits for a flush.  Flushes only REFRESH the table: after
// DEC_REFRESH direct records the wave that notices sets a flag, every wave stops
// after its current step (its position in the unit is kept in registers), the
// block emits every counted slot, keys that were hot in the window stay
// resident (see flush_table; at most MAP_STICKY_CAP, so DEC_ADMIT_AT leaves room
// for keys that turn hot later) and the waves resume.  On Zipf text this cuts
// flushes ~8x against flushing whenever the table is half full (tail keys are
// singletons within a window anyway), and fewer probes per token.
#include "map_common.hpp"

namespace wc {
namespace dev {

constexpr int DEC_UNIT = 64 * MAP_BPL;  // text bytes per wave unit (2 KiB)
constexpr int DEC_HALO = 64;            // bytes past the unit kept in LDS
constexpr int DEC_BUF = DEC_UNIT + DEC_HALO + 16;  // +16: tile8() reads one word past
constexpr uint32_t DEC_NONE = 0xFFFFFFFFu;
#ifndef WC_DEC_TPL
#define WC_DEC_TPL 2
#endif
constexpr uint32_t DEC_TPL = WC_DEC_TPL;  // list entries per lane per step (1 or 2)
constexpr uint32_t DEC_STEP = 64 * DEC_TPL;
#ifndef WC_DEC_KEYS2
#define WC_DEC_KEYS2 1  // both tokens' key windows in one LDS round trip
#endif
#ifndef WC_DEC_ADMIT_EIGHTHS
#define WC_DEC_ADMIT_EIGHTHS 2
#endif
#ifndef WC_DEC_REFRESH
#define WC_DEC_REFRESH 16384
#endif
constexpr uint32_t DEC_ADMIT_AT = MAP_SLOTS * WC_DEC_ADMIT_EIGHTHS / 8;  // occupancy that stops new claims
static_assert(DEC_ADMIT_AT >= MAP_STICKY_CAP + 128, "room for new keys after every refresh");
constexpr uint32_t DEC_REFRESH = WC_DEC_REFRESH;  // direct records that request a flush (table refresh)
static_assert(DEC_UNIT <= 2048, "list entries hold 11-bit unit-relative positions");

// WC_DEC_GROUPED=1: tags and keys of a probe group side by side (one LDS round
// trip per hit instead of two).  Measured: +2 % at 500 words, -7 % at 10k-100k
// (7 VGPRs spill at the 128-register budget), so the split layout is the default.
#ifndef WC_DEC_GROUPED
#define WC_DEC_GROUPED 0
#endif
constexpr int DEC_NGROUPS = MAP_SLOTS / 4;
constexpr int DEC_MAX_PROBES = 8;  // groups probed before a token becomes a direct record

// One probe group: four tags and their four keys together (80 B), read with
// five ds_read_b128 issued back to back — a hit costs ONE dependent LDS round
// trip (tags-then-key was two).
struct alignas(16) DecGroup {
  uint32_t tag[4];  // 0 = empty; else map_tag(place_hash)
  u64x2 key[4];
};

struct DecLds {
#if WC_DEC_GROUPED
  DecGroup grp[DEC_NGROUPS];
#else
  u64x2 key[MAP_SLOTS];
  uint32_t tag[MAP_SLOTS];  // group g = tag[8g, 8g+8); 0 = empty
#endif
  uint32_t cnt[MAP_SLOTS];
  uint32_t off[MAP_SLOTS];
  uint16_t list[MAP_WAVES][MAP_LIST];
  uint32_t bcur[MAX_REC_BUCKETS];  // records appended to each bucket's sub-region (persistent)
  uint8_t buf[MAP_WAVES][DEC_BUF];
  uint32_t occupied, sticky, flush_kept;
  uint32_t flush_req, done_waves, next_unit, direct;
  unsigned long long used;
  unsigned long long tokens;
#if WC_DEC_GROUPED
  __device__ uint32_t& tag_at(int s) { return grp[s >> 2].tag[s & 3]; }
  __device__ uint32_t tag_at(int s) const { return grp[s >> 2].tag[s & 3]; }
  __device__ u64x2 key_at(int s) const { return grp[s >> 2].key[s & 3]; }
  __device__ void evict(int s) {
    grp[s >> 2].tag[s & 3] = 0;
    grp[s >> 2].key[s & 3].y = K1_EMPTY;
  }
#else
  __device__ uint32_t tag_at(int s) const { return tag[s]; }
  __device__ u64x2 key_at(int s) const { return key[s]; }
  __device__ void evict(int s) {
    tag[s] = 0;
    key[s].y = K1_EMPTY;
  }
#endif
  // slot state (flush_table): the bucket bits of place_hash live in the tag
  __device__ int bucket(int s, uint32_t log2_nb) const {
    const uint32_t t = tag_at(s);
    return t ? (int)((t >> 2) & ((1u << log2_nb) - 1u)) : -1;
  }
};
static_assert(sizeof(DecLds) + 8 * MAP_STAMP_N <= 160 * 1024, "one decoupled map block per CU");

#if WC_DEC_GROUPED
// Slot of (k0, k1) in the grouped table — claiming one if the key is absent and
// `admit` — or -1 (absent and not admitted, or DEC_MAX_PROBES full groups).
// Claim = ONE CAS of the tag; the claimer then writes k0 before k1 (one
// wave's LDS writes execute in order, a reader loads each 16-byte key in one
// instruction), so a reader that sees the new k1 also sees the new k0; one
// that reads the tag before the key does not match and may claim a duplicate
// slot, which the reducer merges.  The winner's writes come before this
// iteration's re-read, so lanes of the same wave that lost the CAS see them.
__device__ __forceinline__ int dec_slot(DecLds& L, uint64_t ph, uint64_t k0, uint64_t k1, bool& claimed, bool admit) {
  const uint32_t tag = map_tag(ph);
  uint32_t g = (uint32_t)(ph >> 32) & (DEC_NGROUPS - 1);
  claimed = false;
  for (int steps = 0; steps < DEC_MAX_PROBES;) {
    asm volatile("" ::: "memory");
    const DecGroup& G = L.grp[g];
    const u32x4 t = *reinterpret_cast<const u32x4*>(G.tag);
    const u64x2 q0 = G.key[0], q1 = G.key[1], q2 = G.key[2], q3 = G.key[3];
    const bool h0 = t.x == tag && q0.y == k1 && q0.x == k0;
    const bool h1 = t.y == tag && q1.y == k1 && q1.x == k0;
    const bool h2 = t.z == tag && q2.y == k1 && q2.x == k0;
    const bool h3 = t.w == tag && q3.y == k1 && q3.x == k0;
    if (h0 | h1 | h2 | h3) return 4 * (int)g + (h0 ? 0 : (h1 ? 1 : (h2 ? 2 : 3)));
    const int e = t.x == 0 ? 0 : (t.y == 0 ? 1 : (t.z == 0 ? 2 : (t.w == 0 ? 3 : -1)));
    if (e >= 0 && !admit) return -1;
    bool won = false;
    if (e >= 0) won = atomicCAS(&L.tag_at(4 * (int)g + e), 0u, tag) == 0u;
    if (won) {
      L.grp[g].key[e].x = k0;
      asm volatile("" ::: "memory");
      L.grp[g].key[e].y = k1;
      claimed = true;
      return 4 * (int)g + e;
    }
    if (e < 0) {
      ++steps;
      g = (g + 1) & (DEC_NGROUPS - 1);
    }  // else: lost the slot to another lane, re-read the group
  }
  return -1;
}
#endif

// Count one token in the combiner or, when its key is absent and the table
// admits no new keys (or its probe sequence is full), append it straight to
// the shuffle records as (key, 1, offset).  Returns true for a direct record.
__device__ __forceinline__ bool combine_or_emit(DecLds& L, const MapArgs& a, uint64_t k0, uint64_t k1, uint32_t off,
                                                bool admit, bool& claimed) {
  const uint64_t ph = place_hash(k0, k1);
#if WC_DEC_GROUPED
  const int s = dec_slot(L, ph, k0, k1, claimed, admit);
#else
  const int s = combiner_slot(L, ph, k0, k1, claimed, admit);
#endif
  if (s >= 0) {
    atomicAdd(&L.cnt[s], 1u);  // results unused: no-return ds_add / ds_min
    atomicMin(&L.off[s], off);
    return false;
  }
  if (a.ablate != 7)  // 7 (profiling): direct records dropped
    emit_record(L, a, ((uint32_t)ph >> 2) & ((1u << a.log2_rec_buckets) - 1u), k0, k1, 1, off);
  return true;
}

template <bool ST>
__global__ void __launch_bounds__(MAP_THREADS, 4) wc_map_decoupled(MapArgs a) {
  __shared__ DecLds L;
  __shared__ unsigned long long st_acc[ST ? MAP_STAMP_N : 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (ST && tid < MAP_STAMP_N) st_acc[tid] = 0;
  clear_slots(L);
  for (uint32_t b = tid; b < MAX_REC_BUCKETS; b += MAP_THREADS) L.bcur[b] = 0;
  const uint64_t nunits = (a.chunk_len + DEC_UNIT - 1) / DEC_UNIT;
  const uint64_t per = (nunits + gridDim.x - 1) / gridDim.x;
  const uint64_t u_begin = min((uint64_t)blockIdx.x * per, nunits), u_end = min(u_begin + per, nunits);
  if (tid == 0) {
    L.occupied = 0;
    L.sticky = 0;
    L.tokens = 0;
    L.flush_kept = 0;
    L.used = 0;
    L.flush_req = 0;
    L.done_waves = 0;
    L.next_unit = 0;
    L.direct = 0;
  }
  __syncthreads();

  uint8_t* buf = L.buf[wave];
  uint16_t* list = L.list[wave];
  uint32_t my_tokens = 0;
  uint64_t sink = 0;
  auto grab = [&]() -> uint32_t {
    uint32_t v = 0;
    if (lane == 0) v = atomicAdd(&L.next_unit, 1u);
    v = __builtin_amdgcn_readfirstlane(v);
    return u_begin + v < u_end ? (uint32_t)(u_begin + v) : DEC_NONE;
  };
  // next unit's 32 B per lane (+ halo, + the byte before it) in registers
  uint4 p0 = make_uint4(0, 0, 0, 0), p1 = p0, ph16 = p0;
  uint32_t pprev = 0x20;
  auto prefetch = [&](uint32_t u) {
    if (u == DEC_NONE) return;
    const uint64_t u0 = (uint64_t)u * DEC_UNIT;
    load32(a, u0 + (uint64_t)lane * MAP_BPL, p0, p1);
    if (lane < DEC_HALO / 16) ph16 = load16(a, u0 + DEC_UNIT + (uint64_t)lane * 16);
    if (lane == 0) pprev = (u0 == 0 && a.prev_byte >= 0) ? (uint32_t)a.prev_byte : a.text[(int64_t)u0 - 1];
  };
  PhaseClock<ST> clk;
  clk.start(st_acc);
  const uint64_t t_begin = clk.t;

  uint32_t u = grab();
  prefetch(u);
  uint32_t nu = u == DEC_NONE ? DEC_NONE : grab();
  bool need_unit = true;  // commit the prefetched unit, then build its masks
  uint64_t dm = 0;
  uint32_t starts = 0, bits = 0, k = 0, wave_total = 0, base = 0, round_n = 0, j = 0, prevb = 0x20;
  uint64_t u0 = 0;
  bool counted = false;
  uint32_t occ_seen = 0;  // wave's latest view of L.occupied (claims stop at DEC_ADMIT_AT)
  const uint32_t pbase = lane * MAP_BPL;

  for (;;) {
    // ---------------- work phase: until a flush is requested or no unit is left ----------------
    while (u != DEC_NONE &&
           !__builtin_amdgcn_readfirstlane(__hip_atomic_load(&L.flush_req, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP))) {
      if (need_unit) {
        need_unit = false;
        u0 = (uint64_t)u * DEC_UNIT;
        wave_sync();  // the previous unit's reads are done
        reinterpret_cast<uint4*>(&buf[pbase])[0] = p0;
        reinterpret_cast<uint4*>(&buf[pbase])[1] = p1;
        if (lane < DEC_HALO / 16) *reinterpret_cast<uint4*>(&buf[DEC_UNIT + lane * 16]) = ph16;
        const uint32_t pv = __shfl(pprev, 0);
        wave_sync();
        prefetch(nu);
        clk.lap(MS_COMMIT);
        dm = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint4 v = reinterpret_cast<const uint4*>(&buf[pbase])[q];
          dm |= delim_mask8((uint64_t)v.x | ((uint64_t)v.y << 32)) << (16 * q);
          dm |= delim_mask8((uint64_t)v.z | ((uint64_t)v.w << 32)) << (16 * q + 8);
        }
        prevb = lane == 0 ? pv : buf[pbase - 1];
        starts = (uint32_t)(~dm & ((dm << 1) | (is_delim(prevb) ? 1ull : 0ull)));
        const uint64_t lane_base = u0 + pbase;
        if (lane_base >= a.chunk_len) {
          starts = 0;
        } else if (lane_base + MAP_BPL > a.chunk_len) {
          starts &= (1u << (uint32_t)(a.chunk_len - lane_base)) - 1u;
        }
        const uint32_t ntok = __popc(starts);
        my_tokens += ntok;
        uint32_t incl = ntok;
        for (int o = 1; o < 64; o <<= 1) {
          const uint32_t y = __shfl_up(incl, o);
          if (lane >= o) incl += y;
        }
        wave_total = __builtin_amdgcn_readfirstlane(__shfl(incl, 63));
        bits = starts;
        k = incl - ntok;
        base = 0;
        round_n = 0;
        j = 0;
        clk.lap(MS_MASK);
        if (a.ablate == 2) {
          sink ^= dm;
          base = wave_total;
        }
      }
      if (j >= round_n) {
        if (base >= wave_total) {  // unit done: move to the prefetched one
          u = nu;
          if (u == DEC_NONE) break;
          nu = grab();
          need_unit = true;
          continue;
        }
        const uint32_t lim = base + MAP_LIST;
        while (bits && k < lim) {
          const uint32_t i = __ffs(bits) - 1;
          bits &= bits - 1;
          const uint64_t rest = dm >> i;
          const uint32_t len = rest ? min((uint32_t)__ffsll((unsigned long long)rest) - 1, MAP_LONG) : MAP_LONG;
          list[k - base] = (uint16_t)((pbase + i) | (len << 11));
          ++k;
        }
        wave_sync();
        round_n = min(wave_total - base, (uint32_t)MAP_LIST);
        j = 0;
        clk.lap(MS_LIST);
      }
      // ---- one step: two list entries per lane ----
      const bool h1 = j + lane < round_n, h2 = DEC_TPL > 1 && j + 64 + lane < round_n;
      const uint32_t e1 = h1 ? list[j + lane] : 0u, e2 = h2 ? list[j + 64 + lane] : 0u;
      const uint32_t q1 = e1 & 0x7FFu, q2 = e2 & 0x7FFu;
      uint64_t a0, a1, b0, b1;
#if WC_DEC_KEYS2
      token_keys2(buf, DEC_UNIT + DEC_HALO, a, u0, h1, q1, e1 >> 11, h2, q2, e2 >> 11, a0, a1, b0, b1);
#else
      a0 = a1 = b0 = b1 = 0;
      if (h1) token_key(buf, DEC_UNIT + DEC_HALO, a, u0, q1, e1 >> 11, a0, a1);
      if (h2) token_key(buf, DEC_UNIT + DEC_HALO, a, u0, q2, e2 >> 11, b0, b1);
#endif
      if (ST) {
        asm volatile("" ::"v"(a0), "v"(a1), "v"(b0), "v"(b1));
      }
      clk.lap(MS_KEYS);
      j += DEC_STEP;
      if (j >= round_n) {
        wave_sync();  // entries read before the next round overwrites them
        base += MAP_LIST;
      }
      if (a.ablate == 1) {
        sink ^= place_hash(a0, a1) + place_hash(b0, b1);
        continue;
      }
      const bool admit = occ_seen < DEC_ADMIT_AT;
      bool c1 = false, c2 = false, d1 = false, d2 = false;
      if (h1) d1 = combine_or_emit(L, a, a0, a1, (uint32_t)(u0 + q1), admit, c1);
      if (h2) d2 = combine_or_emit(L, a, b0, b1, (uint32_t)(u0 + q2), admit, c2);
      const uint32_t claims = (uint32_t)__popcll(__ballot(c1)) + (uint32_t)__popcll(__ballot(c2));
      const uint32_t direct = (uint32_t)__popcll(__ballot(d1)) + (uint32_t)__popcll(__ballot(d2));
      if (claims | direct) {
        uint32_t occ = 0, dir = 0;
        if (lane == 0) {
          if (claims) occ = atomicAdd(&L.occupied, claims) + claims;
          if (direct) dir = atomicAdd(&L.direct, direct) + direct;
          if (dir > DEC_REFRESH) atomicOr(&L.flush_req, 1u);
        }
        if (claims) occ_seen = __builtin_amdgcn_readfirstlane(occ);
      }
      clk.lap(MS_COMBINE);
    }
    if (u == DEC_NONE && !counted) {
      counted = true;
      if (lane == 0) atomicAdd(&L.done_waves, 1u);
    }
    // ---------------- barrier phase: flush (if requested), retries ----------------
    __syncthreads();
    clk.lap(MS_RETRY);
    const bool fr = L.flush_req != 0;
    const bool all_done = L.done_waves == (uint32_t)MAP_WAVES;
    if (!fr && all_done) break;
    if (fr) {
      if constexpr (ST) {
        if (tid == 0) st_acc[MS_NFLUSH] += 1;
      }
      // cleared between the flush's barriers: every thread has read flush_req
      // (first barrier) and none resumes before the trailing one
      flush_table(L, a, clk, true, false, [&]() {
        L.flush_req = 0;
        L.used += L.direct;
        L.direct = 0;
      });
      occ_seen = L.occupied;
      clk.lap(MS_FLUSH);
    }
  }
  clk.lap(MS_TOP);
  if (tid == 0) L.used += L.direct;
  if (L.occupied) flush_table(L, a, clk, false, true);  // final: sticky slots too
  clk.lap(MS_FLUSH);
  if constexpr (ST) {
    if (lane == 0) atomicAdd(&st_acc[MS_TOTAL], (unsigned long long)(clk.t - t_begin));
    if (tid == 0) {  // block duration (load balance across the grid; the host divides by the grid)
      atomicAdd(&a.stamps[MS_BLKSUM], (unsigned long long)(clk.t - t_begin));
      atomicMax(&a.stamps[MS_BLKMAX], (unsigned long long)(clk.t - t_begin));
    }
  }

  uint64_t t = my_tokens;
  for (int o = 32; o > 0; o >>= 1) t += __shfl_down(t, o);
  if (lane == 0) atomicAdd(&L.tokens, (unsigned long long)t);
  if (sink == 0x9E3779B97F4A7C15ull) atomicOr(&a.flags[FLAG_COUNT - 1], 0u);  // never true
  __syncthreads();
  if constexpr (ST) {
    if (tid < MAP_STAMP_N) atomicAdd(&a.stamps[tid], st_acc[tid]);
  }
  if (tid == 0) {
    atomicAdd(a.tokens, L.tokens);
    atomicAdd(a.rec.cursor, L.used);
  }
  publish_bucket_counts(L, a);
}

}  // namespace dev

void launch_map_decoupled(const MapArgs& a, uint32_t map_blocks, hipStream_t s) {
  if (a.stamps) hipLaunchKernelGGL(dev::wc_map_decoupled<true>, dim3(map_blocks), dim3(MAP_THREADS), 0, s, a);
  else hipLaunchKernelGGL(dev::wc_map_decoupled<false>, dim3(map_blocks), dim3(MAP_THREADS), 0, s, a);
}

}  // namespace wc
