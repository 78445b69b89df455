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
#include "kernels.hpp"
#include "keys.hpp"

namespace wc {
namespace dev {

constexpr int MAP_WAVES = MAP_THREADS / 64;
constexpr int MAP_LIST = 256;                    // token-list entries per wave per round (u16)
constexpr int MAP_GS = 8;                        // slots per probe group
constexpr int MAP_NGROUPS = MAP_SLOTS / MAP_GS;  // 256
constexpr int MAP_SPT = MAP_SLOTS / MAP_THREADS; // table slots per thread in a flush
constexpr uint32_t MAP_STICKY = 0x80000000u;     // cnt flag: hot slot, kept across flushes
#ifndef WC_MAP_PROMOTE
#define WC_MAP_PROMOTE 5
#endif
#ifndef WC_MAP_STICKY_CAP
#define WC_MAP_STICKY_CAP (MAP_SLOTS / 4)
#endif
constexpr uint32_t MAP_PROMOTE = WC_MAP_PROMOTE;     // tokens in one window that make a slot sticky
constexpr int MAP_STICKY_CAP = WC_MAP_STICKY_CAP;    // sticky budget per block (0 = off)
constexpr uint32_t MAP_LONG = 31u;               // list length field: >= 31 bytes or past the lane window
constexpr int MAP_WAVE_BYTES = 64 * MAP_BPL;     // text bytes owned by one wave (list positions are relative)
static_assert(MAP_WAVE_BYTES <= 2048, "list entries hold 11-bit wave-relative positions");
static_assert(MAP_SLOTS % MAP_THREADS == 0, "flush assumes whole slots per thread");
static_assert(MAP_TILE <= 65536, "list entries hold 16-bit tile positions");
static_assert((MAP_NGROUPS & (MAP_NGROUPS - 1)) == 0, "group count must be a power of two");

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));

struct MapLds {
  u64x2 key[MAP_SLOTS];    // {k0, k1}; k1 = K1_EMPTY after a flush, so a stale key never matches
  uint32_t tag[MAP_SLOTS];  // group g = tag[8g, 8g+8); 0 = empty
  uint32_t cnt[MAP_SLOTS];
  uint32_t off[MAP_SLOTS];
  uint16_t list[MAP_WAVES][MAP_LIST];  // token rounds: wave-relative position | min(length, 31) << 11
  uint32_t boff[MAX_REC_BUCKETS + 4];  // flush: bucket counts -> exclusive offsets (+ total); 0 between flushes
  uint32_t fail[MAP_THREADS];  // bit i of word t: token at tile byte 32 t + i must be retried
  uint8_t tile[MAP_TILE + MAP_HALO + 16];  // +16: tile8() reads one word past
  uint32_t wsum[MAP_WAVES];
  uint32_t occupied;
  uint32_t sticky;  // slots promoted to sticky (budget counter)
  uint32_t occ_before, last_new;  // adaptive flush: keys added by the last tile
  uint32_t prev;
  uint32_t flush_ok;
  uint32_t nflush;  // directory entries written by this block
  uint64_t used;    // records written into this block's region
  uint64_t flush_base;
  unsigned long long tokens;
};
static_assert(sizeof(MapLds) <= 160 * 1024 / MAP_BLOCKS_PER_CU, "map blocks per CU must fit its LDS");

__device__ __forceinline__ uint32_t map_tag(uint64_t ph) { return ((uint32_t)ph & ~1u) | 2u; }  // never 0
__device__ __forceinline__ uint32_t map_group(uint64_t ph) { return (uint32_t)(ph >> 32) & (MAP_NGROUPS - 1); }

// Per-byte "is delimiter" for 8 packed bytes -> 8-bit mask (exact SWAR zero test).
__device__ __forceinline__ uint64_t delim_mask8(uint64_t x) {
  constexpr uint64_t ONES = 0x0101010101010101ull, LOW7 = 0x7F7F7F7F7F7F7F7Full;
  auto zero_bytes = [](uint64_t y) { return ~(((y & LOW7) + LOW7) | y) & 0x8080808080808080ull; };
  const uint64_t m = zero_bytes(x ^ (0x20 * ONES)) | zero_bytes(x ^ (0x0D * ONES)) | zero_bytes(x ^ (0x0A * ONES));
  return ((m >> 7) * 0x0102040810204080ull) >> 56;
}

// 8 bytes of the LDS tile starting at byte p: two aligned ds_read_b64 + funnel
// shift (dynamic indexing of a register window would be lowered to scratch).
__device__ __forceinline__ uint64_t tile8(const uint8_t* tile, uint32_t p) {
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

__device__ __forceinline__ void clear_slots(MapLds& L) {
#pragma unroll
  for (int k = 0; k < MAP_SPT; ++k) {
    const int s = threadIdx.x + k * MAP_THREADS;
    L.tag[s] = 0;
    L.key[s].y = K1_EMPTY;
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

// Shuffle write of the combiner table: one contiguous bucket-sorted chunk.
// Four block barriers: bucket histogram | wave sums of the scan | offsets +
// region | records written (then the histogram is re-zeroed).  trailing_sync
// adds a fifth when inserts follow immediately (retry path).
template <bool ST>
__device__ void flush_table(MapLds& L, const MapArgs& a, PhaseClock<ST>& clk, bool trailing_sync, bool final = false) {
  static_assert(MAX_REC_BUCKETS < MAP_THREADS, "one bucket per thread in the scan");
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint32_t nb = 1u << a.log2_rec_buckets;
  uint32_t sb[MAP_SPT], sr[MAP_SPT], kept = 0;
  if (a.ablate != 5) {  // 5 (profiling): flush = clear only
#pragma unroll
    for (int j = 0; j < MAP_SPT; ++j) {
      const int s = tid + j * MAP_THREADS;
      sb[j] = 0xFFFFFFFFu;
      const uint32_t tag = L.tag[s];
      if (tag != 0) {
        // Sticky slots (hot keys) stay and keep counting until the block's
        // final flush; a slot that counted MAP_PROMOTE tokens in this window
        // becomes sticky while the sticky budget lasts.
        const uint32_t c = L.cnt[s];
        bool stick = (c & MAP_STICKY) != 0;
        if (!final && !stick && c >= MAP_PROMOTE && L.sticky < (uint32_t)MAP_STICKY_CAP &&
            atomicAdd(&L.sticky, 1u) < (uint32_t)MAP_STICKY_CAP) {
          L.cnt[s] = c | MAP_STICKY;
          stick = true;
        }
        if (stick && !final) {
          ++kept;
        } else {
          sb[j] = (tag >> 2) & (nb - 1u);  // == bucket_of(place_hash): bucket bits live in the tag
          sr[j] = atomicAdd(&L.boff[sb[j]], 1u);
        }
      }
    }
    bsync(clk, MS_FL_HIST);
    // exclusive scan of boff[0, nb): one bucket per thread
    const uint32_t v = (uint32_t)tid < nb ? L.boff[tid] : 0u;
    uint32_t x = v;
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(x, o);
      if (lane >= o) x += y;
    }
    if (lane == 63) L.wsum[wave] = x;
    bsync(clk, MS_FL_SCAN);
    uint32_t before = 0, total = 0;
#pragma unroll
    for (int w = 0; w < MAP_WAVES; ++w) {
      const uint32_t ws = L.wsum[w];
      before += w < wave ? ws : 0u;
      total += ws;
    }
    if ((uint32_t)tid <= nb) L.boff[tid] = before + x - v;  // boff[nb] = total
    if (tid == 0) {
      uint32_t ok = 0;
      L.occupied = 0;
      if (total) {
        // block-private record region: no global cursor contention
        const uint64_t region = a.rec.cap / gridDim.x;
        const uint64_t base = (uint64_t)blockIdx.x * region + L.used;
        const uint32_t j = L.nflush;
        ok = (L.used + total <= region && j < a.rec.dir_per_block) ? 1u : 0u;
        L.used += total;
        if (ok) {
          L.nflush = j + 1;
          a.rec.dir_base[(size_t)blockIdx.x * a.rec.dir_per_block + j] = base;
        } else {
          atomicOr(&a.flags[FLAG_REGION_OVF], 1u);
        }
        L.flush_base = base;
      }
      L.flush_ok = ok;
    }
    bsync(clk, MS_FL_SCAN);
    if (L.flush_ok) {
      const uint32_t j = L.nflush - 1;
      const size_t row = (size_t)gridDim.x * a.rec.dir_per_block;
      if (a.ablate != 3 && (uint32_t)tid <= nb)
        a.rec.dir_off[(size_t)tid * row + (size_t)blockIdx.x * a.rec.dir_per_block + j] = L.boff[tid];
      const uint64_t base = L.flush_base;
#pragma unroll
      for (int k = 0; k < MAP_SPT; ++k) {
        if (sb[k] == 0xFFFFFFFFu) continue;
        const int s = tid + k * MAP_THREADS;
        const u64x2 kk = L.key[s];
        Rec r;
        r.k0 = kk.x;
        r.k1 = kk.y;
        r.co = ((uint64_t)(L.cnt[s] & ~MAP_STICKY) << 32) | L.off[s];
        a.rec.recs[base + L.boff[sb[k]] + sr[k]] = r;
      }
    }
    if (kept) atomicAdd(&L.occupied, kept);
#pragma unroll
    for (int k = 0; k < MAP_SPT; ++k) {  // own emitted slots only: no barrier needed before
      if (sb[k] == 0xFFFFFFFFu) continue;
      const int s = tid + k * MAP_THREADS;
      L.tag[s] = 0;
      L.key[s].y = K1_EMPTY;
      L.cnt[s] = 0;
      L.off[s] = 0xFFFFFFFFu;
    }
  } else {
    if (tid == 0) L.occupied = 0;
    clear_slots(L);
  }
  if (final && tid == 0) L.sticky = 0;
  bsync(clk, MS_FL_WRITE);  // every thread done reading boff (and the slots cleared)
  if ((uint32_t)tid <= nb) L.boff[tid] = 0;
  if (trailing_sync) bsync(clk, MS_FL_WRITE);
}

// Key of a token that does not end inside the 64-byte lane window.
__device__ __forceinline__ void key_slow(const MapLds& L, const MapArgs& a, uint64_t pos, uint64_t g, uint64_t& k0,
                                      uint64_t& k1) {
  uint64_t len = 0, h = FNV_OFFSET, chunk = 0;
  k0 = 0;
  for (;;) {
    uint32_t c;
    if (pos < (uint64_t)(MAP_TILE + MAP_HALO)) c = L.tile[pos];
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

// Key of the token at tile position p with known length (< 31) or MAP_LONG.
__device__ __forceinline__ void token_key(const MapLds& L, const MapArgs& a, uint64_t t0, uint32_t p, uint32_t len,
                                          uint64_t& k0, uint64_t& k1) {
  if (len != MAP_LONG) {
    k0 = low_bytes(tile8(L.tile, p), len);
    if (len <= 8) {
      k1 = len;
    } else {
      uint64_t h = FNV_OFFSET;
      for (uint32_t c = 8; c < len; c += 8) h = tail_fold(h, low_bytes(tile8(L.tile, p + c), len - c));
      k1 = make_k1(len, h);
    }
  } else {
    key_slow(L, a, p, t0 + p, k0, k1);
  }
}

// Combiner slot of (k0, k1) — claiming one if the key is absent — or -1 when
// MAP_MAX_GROUP_PROBES groups are full.  Claim = ONE CAS of the tag; the
// claimer then writes k0 before k1 (LDS executes one wave's writes in order,
// and the reader loads the 16-byte key in one instruction), so a reader that
// sees the new k1 also sees the new k0; one that sees the tag before the key
// does not match and may claim a duplicate slot, which the reducer merges.
__device__ __forceinline__ int combiner_slot(MapLds& L, uint64_t ph, uint64_t k0, uint64_t k1, bool& claimed) {
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
__device__ __forceinline__ bool combine(MapLds& L, uint64_t k0, uint64_t k1, uint32_t off, bool& claimed) {
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

template <bool ST>
__global__ void __launch_bounds__(MAP_THREADS, 4) wc_map_tokenize(MapArgs a) {  // 2nd arg: waves per SIMD
  __shared__ MapLds L;
  __shared__ unsigned long long st_acc[ST ? MAP_STAMP_N : 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (ST && tid < MAP_STAMP_N) st_acc[tid] = 0;
  clear_slots(L);
  L.fail[tid] = 0;
  for (uint32_t b = tid; b < MAX_REC_BUCKETS + 4; b += MAP_THREADS) L.boff[b] = 0;
  if (tid == 0) {
    L.occupied = 0;
    L.sticky = 0;
    L.last_new = 0;
    L.tokens = 0;
    L.nflush = 0;
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
      if (h1) token_key(L, a, t0, q1, e1 >> 11, a0, a1);
      if (h2) token_key(L, a, t0, q2, e2 >> 11, b0, b1);
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
        token_key(L, a, t0, pbase + i, len, k0, k1);
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
    atomicAdd(a.rec.cursor, (unsigned long long)L.used);  // stats: records after the combiner
    a.rec.dir_count[blockIdx.x] = L.nflush;
  }
}

}  // namespace dev

void launch_map(const MapArgs& a, uint32_t map_blocks, hipStream_t s) {
  if (a.stamps) hipLaunchKernelGGL(dev::wc_map_tokenize<true>, dim3(map_blocks), dim3(MAP_THREADS), 0, s, a);
  else hipLaunchKernelGGL(dev::wc_map_tokenize<false>, dim3(map_blocks), dim3(MAP_THREADS), 0, s, a);
}

}  // namespace wc
