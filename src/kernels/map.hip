// map.hip — wc_map_tokenize: the MAP stage (+ combiner + shuffle write).
//
// Reference: mapKernel (/root/reference/main.cu:109-117) runs one thread per
// pre-split input record and only copies words the HOST tokenizer
// (main.cu:181-206) already found.  Here the GPU does the whole map:
//
//  1. A persistent grid of 2 blocks/CU walks 16 KiB text tiles.  The next
//     tile (+256 B halo) is prefetched into registers while the current one is
//     tokenized, then committed to LDS.
//  2. Each lane owns 32 bytes and builds a 64-bit delimiter mask over its
//     bytes and its neighbour's (SWAR zero-byte test against {0x20,0x0D,0x0A}).
//     Token starts are  ~d & (d << 1 | carry-in)  restricted to the owned 32
//     bytes, so a token straddling lanes / tiles / chunks / GPU shards is owned
//     by the unit holding its FIRST byte.
//  3. Load balance: a wave scan of the per-lane token counts compacts the
//     wave's tokens into an LDS list of (position, length) entries, and the 64
//     lanes then take list entries two at a time — every lane keys and combines
//     the same number of tokens, instead of each lane walking its own (uneven)
//     tokens while the rest of the wave idles.
//  4. Keys (keys.hpp) come from two aligned ds_read_b64 per 8 bytes; words
//     longer than the lane window fall back to a byte loop (LDS halo, then
//     global memory).
//  5. Combiner: 2048-slot LDS hash table, 8-slot groups.  A probe reads the
//     group's eight 32-bit tags (two ds_read_b128) and then only the matching
//     slot's 16-byte key.  Claims are ONE CAS on the tag (duplicates are
//     allowed: the reducer merges them), count / first-offset updates are
//     no-return LDS atomics, occupancy is counted once per wave.
//  6. A token whose probe sequence is full is marked in a per-tile failure
//     bitmap; the block flushes and the owning lanes retry those tokens.
//  7. Flush = shuffle write: occupied slots are counting-sorted by shuffle
//     bucket (LDS histogram + block scan) and written as ONE contiguous chunk
//     (coalesced) plus a bucket-offset directory entry; the reducer of bucket
//     b reads its run of every chunk.
#include "map_common.hpp"

namespace wc {
namespace dev {

struct MapLds {
  u64x2 key[MAP_SLOTS];    // {k0, k1}; k1 = K1_EMPTY after a flush, so a stale key never matches
  uint32_t tag[MAP_SLOTS];  // group g = tag[8g, 8g+8); 0 = empty
  uint32_t cnt[MAP_SLOTS];
  uint32_t off[MAP_SLOTS];
  uint16_t list[MAP_WAVES][MAP_LIST];  // token rounds: wave-relative position | min(length, 31) << 11
  uint32_t bcur[MAX_REC_BUCKETS];  // records appended to each bucket's sub-region (persistent)
  uint32_t fail[MAP_THREADS];  // bit i of word t: token at tile byte 32 t + i must be retried
  uint8_t tile[MAP_TILE + MAP_HALO + 16];  // +16: tile8() reads one word past
  uint32_t occupied;
  uint32_t flush_kept;  // flush: sticky slots kept (-> occupied)
  uint32_t sticky;  // slots promoted to sticky (budget counter)
  uint32_t occ_before, last_new;  // adaptive flush: keys added by the last tile
  uint32_t prev;
  unsigned long long used;  // records emitted by this block (stats)
  unsigned long long tokens;
  // slot state (flush_table): the bucket bits of place_hash live in the tag
  __device__ int bucket(int s, uint32_t log2_nb) const {
    const uint32_t t = tag[s];
    return t ? (int)((t >> 2) & ((1u << log2_nb) - 1u)) : -1;
  }
  __device__ void evict(int s) {
    tag[s] = 0;
    key[s].y = K1_EMPTY;
  }
  __device__ u64x2 key_at(int s) const { return key[s]; }
};
static_assert(sizeof(MapLds) <= 160 * 1024 / MAP_BLOCKS_PER_CU, "map blocks per CU must fit its LDS");

template <bool ST>
__global__ void __launch_bounds__(MAP_THREADS, 4) wc_map_tokenize(MapArgs a) {  // 2nd arg: waves per SIMD
  __shared__ MapLds L;
  __shared__ unsigned long long st_acc[ST ? MAP_STAMP_N : 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (ST && tid < MAP_STAMP_N) st_acc[tid] = 0;
  clear_slots(L);
  L.fail[tid] = 0;
  for (uint32_t b = tid; b < MAX_REC_BUCKETS; b += MAP_THREADS) L.bcur[b] = 0;
  if (tid == 0) {
    L.occupied = 0;
    L.sticky = 0;
    L.last_new = 0;
    L.tokens = 0;
    L.flush_kept = 0;
    L.used = 0;
  }

  const uint64_t ntiles = (a.chunk_len + MAP_TILE - 1) / MAP_TILE;
  uint32_t my_tokens = 0;
  uint64_t sink = 0;  // keeps ablated work alive

  // Software pipeline: the next tile's 32 B per lane (+ halo) are loaded into
  // registers while the current tile is being tokenized.
  uint4 p0 = make_uint4(0, 0, 0, 0), p1 = p0, ph16 = p0;
  uint32_t pprev = 0x20;
  auto prefetch = [&](uint64_t tile) {
    if (tile >= ntiles) return;
    const uint64_t t0 = tile * MAP_TILE;
    load32(a, t0 + (uint64_t)tid * MAP_BPL, p0, p1);
    if (tid < MAP_HALO / 16) ph16 = load16(a, t0 + MAP_TILE + (uint64_t)tid * 16);
    if (tid == 0) pprev = (t0 == 0 && a.prev_byte >= 0) ? (uint32_t)a.prev_byte : a.text[(int64_t)t0 - 1];
  };
  prefetch(blockIdx.x);
  PhaseClock<ST> clk;
  clk.start(st_acc);
  const uint64_t t_begin = clk.t;

  for (uint64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const uint64_t t0 = tile * MAP_TILE;
    __syncthreads();  // previous tile fully consumed
    clk.lap(MS_TOP);
    // Flush only if the keys the last tile added would not fit again: Zipf
    // text with a small vocabulary keeps its table across many tiles, large
    // vocabularies flush before every tile instead of overflowing mid-tile.
    if (L.occupied + L.last_new > MAP_FILL_MAX) {
      if constexpr (ST) {
        if (tid == 0) st_acc[MS_NFLUSH] += 1;
      }
      flush_table(L, a, clk, false);  // the commit barrier follows
    }
    clk.lap(MS_FLUSH);
    if (tid == 0) L.occ_before = L.occupied;
    // ---- commit the prefetched tile to LDS, start loading the next ----
    reinterpret_cast<uint4*>(&L.tile[tid * MAP_BPL])[0] = p0;
    reinterpret_cast<uint4*>(&L.tile[tid * MAP_BPL])[1] = p1;
    if (tid < MAP_HALO / 16) *reinterpret_cast<uint4*>(&L.tile[MAP_TILE + tid * 16]) = ph16;
    if (tid == 0) L.prev = pprev;
    __syncthreads();
    prefetch(tile + gridDim.x);
    clk.lap(MS_COMMIT);

    // ---- 64-byte window (own 32 B + next lane's), delimiter / start masks ----
    uint64_t dm = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint4 v = reinterpret_cast<const uint4*>(&L.tile[tid * MAP_BPL])[j];
      dm |= delim_mask8((uint64_t)v.x | ((uint64_t)v.y << 32)) << (16 * j);
      dm |= delim_mask8((uint64_t)v.z | ((uint64_t)v.w << 32)) << (16 * j + 8);
    }
    const uint32_t prevb = (tid == 0) ? L.prev : L.tile[tid * MAP_BPL - 1];
    uint32_t starts = (uint32_t)(~dm & ((dm << 1) | (is_delim(prevb) ? 1ull : 0ull)));
    const uint64_t lane_base = t0 + (uint64_t)tid * MAP_BPL;
    if (lane_base >= a.chunk_len) {
      starts = 0;
    } else if (lane_base + MAP_BPL > a.chunk_len) {
      starts &= (1u << (uint32_t)(a.chunk_len - lane_base)) - 1u;
    }
    const uint32_t ntok = __popc(starts);
    my_tokens += ntok;
    uint64_t t_tok = 0;
    if constexpr (ST) t_tok = __builtin_amdgcn_s_memtime();
    clk.lap(MS_MASK);
    if (a.ablate == 2) {
      sink ^= dm;
      continue;
    }

    // ---- compact the wave's tokens into list rounds of MAP_LIST entries ----
    uint32_t incl = ntok;
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(incl, o);
      if (lane >= o) incl += y;
    }
    const uint32_t wave_total = __shfl(incl, 63), excl = incl - ntok;
    const uint32_t pbase = tid * MAP_BPL;
    uint16_t* list = L.list[wave];
    const uint32_t wbase = wave * MAP_WAVE_BYTES;
    bool any_fail = false;
    uint32_t bits = starts, k = excl;  // this lane's next token and its wave index
    for (uint32_t base = 0; base < wave_total; base += MAP_LIST) {
      const uint32_t lim = base + MAP_LIST;
      while (bits && k < lim) {
        const uint32_t i = __ffs(bits) - 1;
        bits &= bits - 1;
        const uint64_t rest = dm >> i;
        const uint32_t len = rest ? min((uint32_t)__ffsll((unsigned long long)rest) - 1, MAP_LONG) : MAP_LONG;
        list[k - base] = (uint16_t)((pbase + i - wbase) | (len << 11));
        ++k;
      }
      wave_sync();
      clk.lap(MS_LIST);
      const uint32_t n = min(wave_total - base, (uint32_t)MAP_LIST);
      for (uint32_t j = 0; j < n; j += 128) {
      const bool h1 = j + lane < n, h2 = j + 64 + lane < n;
      const uint32_t e1 = h1 ? list[j + lane] : 0u, e2 = h2 ? list[j + 64 + lane] : 0u;
      const uint32_t q1 = wbase + (e1 & 0x7FFu), q2 = wbase + (e2 & 0x7FFu);
      uint64_t a0 = 0, a1 = 0, b0 = 0, b1 = 0;
      if (h1) token_key(L.tile, MAP_TILE + MAP_HALO, a, t0, q1, e1 >> 11, a0, a1);
      if (h2) token_key(L.tile, MAP_TILE + MAP_HALO, a, t0, q2, e2 >> 11, b0, b1);
      if (ST) {  // force the keys before the keys/combine boundary stamp
        asm volatile("" ::"v"(a0), "v"(a1), "v"(b0), "v"(b1));
      }
      clk.lap(MS_KEYS);
      if (a.ablate == 1) {
        sink ^= place_hash(a0, a1) + place_hash(b0, b1);
        continue;
      }
      bool c1 = false, c2 = false;
      if (h1 && !combine(L, a0, a1, (uint32_t)(t0 + q1), c1)) {
        atomicOr(&L.fail[q1 >> 5], 1u << (q1 & 31));
        any_fail = true;
      }
      if (h2 && !combine(L, b0, b1, (uint32_t)(t0 + q2), c2)) {
        atomicOr(&L.fail[q2 >> 5], 1u << (q2 & 31));
        any_fail = true;
      }
      const uint32_t claims = (uint32_t)__popcll(__ballot(c1)) + (uint32_t)__popcll(__ballot(c2));
      if (lane == 0 && claims) atomicAdd(&L.occupied, claims);
      clk.lap(MS_COMBINE);
      }
      wave_sync();  // entries read before the next round overwrites them
    }

    if constexpr (ST) {  // spread of the waves' token-phase times (diagnostic)
      const uint64_t dt = __builtin_amdgcn_s_memtime() - t_tok;
      if (lane == 0) {
        atomicAdd(&st_acc[MS_TOKSUM], (unsigned long long)dt);
        atomicMax(&st_acc[MS_TOKMAX_TILE], (unsigned long long)dt);
      }
    }
    // ---- probe sequences that were full: flush, then the owners retry ----
    // (a second retry in one tile also evicts the sticky slots: always progresses)
    for (uint32_t attempt = 0; __syncthreads_or(any_fail); ++attempt) {
      clk.lap(MS_RETRY);
      if constexpr (ST) {
        if (tid == 0) st_acc[MS_NRETRY] += 1;
      }
      flush_table(L, a, clk, true, attempt > 0);
      clk.lap(MS_FLUSH);
      uint32_t todo = L.fail[tid];
      L.fail[tid] = 0;
      any_fail = false;
      uint32_t claims = 0;
      while (todo) {
        const uint32_t i = __ffs(todo) - 1;
        todo &= todo - 1;
        const uint64_t rest = dm >> i;
        const uint32_t len = rest ? min((uint32_t)__ffsll((unsigned long long)rest) - 1, MAP_LONG) : MAP_LONG;
        uint64_t k0, k1;
        token_key(L.tile, MAP_TILE + MAP_HALO, a, t0, pbase + i, len, k0, k1);
        bool c = false;
        if (!combine(L, k0, k1, (uint32_t)(t0 + pbase + i), c)) {
          atomicOr(&L.fail[tid], 1u << i);
          any_fail = true;
        }
        claims += c;
      }
      if (claims) atomicAdd(&L.occupied, claims);
    }
    clk.lap(MS_RETRY);
    if (tid == 0) L.last_new = L.occupied > L.occ_before ? L.occupied - L.occ_before : L.occupied;
    if constexpr (ST) {
      if (tid == 0) {  // all waves passed __syncthreads_or: the tile's max is final
        st_acc[MS_TOKMAX] += st_acc[MS_TOKMAX_TILE];
        st_acc[MS_TOKMAX_TILE] = 0;
      }
    }
  }
  __syncthreads();
  clk.lap(MS_TOP);
  if (L.occupied) flush_table(L, a, clk, false, true);  // final: sticky slots too
  clk.lap(MS_FLUSH);
  if constexpr (ST) {
    if (lane == 0) atomicAdd(&st_acc[MS_TOTAL], (unsigned long long)(clk.t - t_begin));
  }

  // block totals -> one global atomic
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
    atomicAdd(a.rec.cursor, L.used);  // stats: records after the combiner
  }
  publish_bucket_counts(L, a);
}

}  // namespace dev

void launch_map(const MapArgs& a, uint32_t map_blocks, hipStream_t s) {
  if (a.stamps) hipLaunchKernelGGL(dev::wc_map_tokenize<true>, dim3(map_blocks), dim3(MAP_THREADS), 0, s, a);
  else hipLaunchKernelGGL(dev::wc_map_tokenize<false>, dim3(map_blocks), dim3(MAP_THREADS), 0, s, a);
}

}  // namespace wc
