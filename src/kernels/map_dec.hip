// map_dec.hip — wc_map_decoupled: the MAP stage with wave-decoupled text units.
//
// Same tokenizer, keys, combiner and shuffle write as map.hip (the building
// blocks live in map_common.hpp), but without block-wide tiles: each of the 16
// waves of a block owns a private LDS buffer holding one 2 KiB text UNIT (+64 B
// halo), grabs its next unit from the block's LDS cursor and prefetches it into
// registers while tokenizing the current one.  Waves therefore never wait for
// each other at a tile boundary (map.hip's phase clock: ~25 % of wave time was
// spent at per-tile barriers).  The only block-wide synchronisation is the
// combiner flush: when the shared table passes DEC_FLUSH_AT occupied slots (or a
// probe sequence is full), the wave that notices sets a flag, every wave stops
// after its current step (its position in the unit is kept in registers), the
// block flushes, failed tokens are retried and the waves resume.
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
#ifndef WC_DEC_FLUSH_EIGHTHS
#define WC_DEC_FLUSH_EIGHTHS 4
#endif
constexpr uint32_t DEC_FLUSH_AT = MAP_SLOTS * WC_DEC_FLUSH_EIGHTHS / 8;  // occupancy that requests a flush
static_assert(DEC_UNIT <= 2048, "list entries hold 11-bit unit-relative positions");

struct DecLds {
  u64x2 key[MAP_SLOTS];
  uint32_t tag[MAP_SLOTS];
  uint32_t cnt[MAP_SLOTS];
  uint32_t off[MAP_SLOTS];
  uint16_t list[MAP_WAVES][MAP_LIST];
  uint32_t bcur[MAX_REC_BUCKETS];  // records appended to each bucket's sub-region (persistent)
  uint32_t fail[MAP_THREADS];  // bit i of word t: token at unit byte 32 (t % 64) + i of wave t / 64 must be retried
  uint8_t buf[MAP_WAVES][DEC_BUF];
  uint32_t occupied, sticky, flush_kept;
  uint32_t flush_req, done_waves, next_unit;
  unsigned long long used;
  unsigned long long tokens;
};
static_assert(sizeof(DecLds) + 8 * MAP_STAMP_N <= 160 * 1024, "one decoupled map block per CU");

template <bool ST>
__global__ void __launch_bounds__(MAP_THREADS, 4) wc_map_decoupled(MapArgs a) {
  __shared__ DecLds L;
  __shared__ unsigned long long st_acc[ST ? MAP_STAMP_N : 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (ST && tid < MAP_STAMP_N) st_acc[tid] = 0;
  clear_slots(L);
  L.fail[tid] = 0;
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
      uint64_t a0 = 0, a1 = 0, b0 = 0, b1 = 0;
      if (h1) token_key(buf, DEC_UNIT + DEC_HALO, a, u0, q1, e1 >> 11, a0, a1);
      if (h2) token_key(buf, DEC_UNIT + DEC_HALO, a, u0, q2, e2 >> 11, b0, b1);
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
      bool c1 = false, c2 = false, f = false;
      if (h1 && !combine(L, a0, a1, (uint32_t)(u0 + q1), c1)) {
        atomicOr(&L.fail[wave * 64 + (q1 >> 5)], 1u << (q1 & 31));
        f = true;
      }
      if (h2 && !combine(L, b0, b1, (uint32_t)(u0 + q2), c2)) {
        atomicOr(&L.fail[wave * 64 + (q2 >> 5)], 1u << (q2 & 31));
        f = true;
      }
      const uint32_t claims = (uint32_t)__popcll(__ballot(c1)) + (uint32_t)__popcll(__ballot(c2));
      const bool anyf = __ballot(f) != 0;
      if (lane == 0) {
        const uint32_t occ = claims ? atomicAdd(&L.occupied, claims) + claims : 0u;
        if (anyf || occ > DEC_FLUSH_AT) atomicOr(&L.flush_req, 1u);
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
      flush_table(L, a, clk, true);  // every thread has read flush_req before its first barrier
      if (tid == 0) L.flush_req = 0;
      clk.lap(MS_FLUSH);
      // owners retry the tokens whose probe sequence was full (the unit is still in buf)
      uint32_t todo = L.fail[tid];
      L.fail[tid] = 0;
      uint32_t claims = 0;
      bool f = false;
      while (todo) {
        const uint32_t i = __ffs(todo) - 1;
        todo &= todo - 1;
        const uint64_t rest = dm >> i;
        const uint32_t len = rest ? min((uint32_t)__ffsll((unsigned long long)rest) - 1, MAP_LONG) : MAP_LONG;
        uint64_t k0, k1;
        token_key(buf, DEC_UNIT + DEC_HALO, a, u0, pbase + i, len, k0, k1);
        bool c = false;
        if (!combine(L, k0, k1, (uint32_t)(u0 + pbase + i), c)) {
          atomicOr(&L.fail[tid], 1u << i);
          f = true;
        }
        claims += c;
      }
      if (claims) atomicAdd(&L.occupied, claims);
      if (f) atomicOr(&L.flush_req, 1u);  // retried again after the next flush
      __syncthreads();
      clk.lap(MS_RETRY);
    }
  }
  clk.lap(MS_TOP);
  if (L.occupied) flush_table(L, a, clk, false, true);  // final: sticky slots too
  clk.lap(MS_FLUSH);
  if constexpr (ST) {
    if (lane == 0) atomicAdd(&st_acc[MS_TOTAL], (unsigned long long)(clk.t - t_begin));
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
