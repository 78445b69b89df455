// map_v4.hip — previous map kernel, kept for A/B measurement: the MAP stage (+ combiner + shuffle write).
//
// Reference: mapKernel (/root/reference/main.cu:109-117) runs one thread per
// pre-split input record and only copies words the HOST tokenizer
// (main.cu:181-206) already found.  Here the GPU does the whole map:
//
//  1. A persistent grid of ~2 blocks/CU walks 16 KiB text tiles.  Each tile
//     (+256 B halo) is staged global -> LDS with 16-B loads.
//  2. Each lane owns 32 bytes and holds a 64-byte register window (its bytes
//     + the next lane's, four aligned ds_read_b128).  A SWAR packed-byte
//     compare against {0x20,0x0D,0x0A} gives a 64-bit delimiter mask; token
//     starts are  ~d & (d << 1 | carry-in)  restricted to the owned 32 bytes,
//     so a token straddling lanes / tiles / chunks is owned by the unit
//     holding its FIRST byte.
//  3. A token that ends inside the window is keyed from registers: k0 by a
//     funnel shift + mask, and (> 8 bytes) the tail hash one 8-byte chunk at a
//     time.  Only tokens longer than the window take a byte loop (LDS halo,
//     then global).
//  4. Keys are combined in a group-probed LDS hash table (lds_table.hpp): the
//     MapReduce combiner, kept across tiles while it is sparse, so Zipf text
//     collapses to one record per hot word per block.  A token that finds no
//     slot makes the block flush and retry it (no singleton fallback).
//  5. Flush = shuffle write: occupied slots are counting-sorted by shuffle
//     bucket (LDS histogram + block scan) and written as ONE contiguous chunk
//     (coalesced) plus a bucket-offset directory entry; the reducer of bucket
//     b reads its run of every chunk.
#include "kernels.hpp"
#include "lds_table.hpp"

namespace wc {
namespace dev {
namespace v4 {

constexpr int MAP_SPT = MAP_SLOTS / MAP_THREADS;  // table slots per thread in a flush
static_assert(MAP_SLOTS % MAP_THREADS == 0, "flush assumes whole slots per thread");

struct MapLds {
  SlotGroup grp[MAP_GROUPS];  // first: 16-B aligned for the ds_read_b128 group reads
  uint32_t cnt[MAP_SLOTS];
  uint32_t off[MAP_SLOTS];
  uint32_t boff[MAX_REC_BUCKETS + 4];  // bucket counts -> exclusive offsets (+ total)
  uint8_t tile[MAP_TILE + MAP_HALO + 16];  // +16: tile8() reads one word past
  uint32_t wsum[MAP_THREADS / 64];
  uint32_t occupied;
  uint32_t occ_before, last_new;  // adaptive flush: keys added by the last tile
  uint32_t prev;
  uint32_t flush_ok;
  uint32_t nflush;  // directory entries written by this block
  uint64_t used;    // records written into this block's region
  uint64_t flush_base;
  unsigned long long tokens;
};

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

// Exclusive scan of a[0..n) in place (n <= MAX_REC_BUCKETS); a[n] = total.
__device__ void block_exclusive_scan(uint32_t* a, uint32_t n, uint32_t* wsum) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr int PER = (MAX_REC_BUCKETS + MAP_THREADS - 1) / MAP_THREADS;
  uint32_t v[PER], s = 0;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const uint32_t i = tid * PER + k;
    v[k] = i < n ? a[i] : 0;
    s += v[k];
  }
  uint32_t x = s;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[wave] = x;
  __syncthreads();
  uint32_t before = 0, total = 0;
  for (int w = 0; w < MAP_THREADS / 64; ++w) {
    before += w < wave ? wsum[w] : 0;
    total += wsum[w];
  }
  uint32_t run = before + x - s;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const uint32_t i = tid * PER + k;
    if (i < n) a[i] = run;
    run += v[k];
  }
  if (tid == 0) a[n] = total;
  __syncthreads();
}

// Shuffle write of the combiner table: one contiguous bucket-sorted chunk.
__device__ void flush_table(MapLds& L, const MapArgs& a) {
  const int tid = threadIdx.x;
  const uint32_t nb = 1u << a.log2_rec_buckets;
  if (a.ablate == 5) {  // profiling: clear only
    for (int s = tid; s < MAP_SLOTS; s += MAP_THREADS) {
      L.grp[s >> 2].tag[s & 3] = TAG_EMPTY;
      L.grp[s >> 2].k1[s & 3] = K1_EMPTY;
    }
    __syncthreads();
    if (tid == 0) L.occupied = 0;
    __syncthreads();
    return;
  }
  for (uint32_t b = tid; b <= nb; b += MAP_THREADS) L.boff[b] = 0;
  __syncthreads();
  uint32_t sb[MAP_SPT], sr[MAP_SPT];
#pragma unroll
  for (int j = 0; j < MAP_SPT; ++j) {
    const int s = tid + j * MAP_THREADS;
    sb[j] = 0xFFFFFFFFu;
    const uint32_t tag = slot_tag(L.grp, s);
    if (tag > TAG_PENDING) {
      sb[j] = (tag >> 2) & (nb - 1u);  // == bucket_of(place_hash): bucket bits live in the tag
      sr[j] = atomicAdd(&L.boff[sb[j]], 1u);
    }
  }
  __syncthreads();
  block_exclusive_scan(L.boff, nb, L.wsum);
  const uint32_t n = L.boff[nb];
  if (tid == 0) {
    uint32_t ok = 0;
    if (n) {
      // block-private record region: no global cursor contention
      const uint64_t region = a.rec.cap / gridDim.x;
      const uint64_t base = (uint64_t)blockIdx.x * region + L.used;
      const uint32_t j = L.nflush;
      ok = (L.used + n <= region && j < a.rec.dir_per_block) ? 1u : 0u;
      L.used += n;
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
  __syncthreads();
  if (L.flush_ok) {
    const uint32_t j = L.nflush - 1;
    const size_t row = (size_t)gridDim.x * a.rec.dir_per_block;
    if (a.ablate != 3)
      for (uint32_t b = tid; b <= nb; b += MAP_THREADS)
        a.rec.dir_off[b * row + (size_t)blockIdx.x * a.rec.dir_per_block + j] = L.boff[b];
    const uint64_t base = L.flush_base;
#pragma unroll
    for (int k = 0; k < MAP_SPT; ++k) {
      if (sb[k] == 0xFFFFFFFFu) continue;
      const int s = tid + k * MAP_THREADS;
      Rec r;
      r.k0 = slot_k0(L.grp, s);
      r.k1 = slot_k1(L.grp, s);
      r.co = ((uint64_t)L.cnt[s] << 32) | L.off[s];
      a.rec.recs[base + L.boff[sb[k]] + sr[k]] = r;
    }
  }
#pragma unroll
  for (int k = 0; k < MAP_SPT; ++k) {
    const int s = tid + k * MAP_THREADS;
    L.grp[s >> 2].tag[s & 3] = TAG_EMPTY;
    L.grp[s >> 2].k1[s & 3] = K1_EMPTY;
    L.cnt[s] = 0;
    L.off[s] = 0xFFFFFFFFu;
  }
  __syncthreads();
  if (tid == 0) L.occupied = 0;
  __syncthreads();
}

// Key of a token that does not end inside the register window.
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

// Key of the token starting at tile position p, given the lane's 64-bit
// delimiter window mask `rest` shifted to the token start.
struct TokKey {
  uint64_t k0, k1, ph;
  uint32_t off;
};

__device__ __forceinline__ TokKey token_key(const MapLds& L, const MapArgs& a, uint64_t t0, uint32_t p,
                                            uint64_t rest) {
  TokKey t;
  if (rest != 0) {
    const uint32_t len = (uint32_t)__ffsll((unsigned long long)rest) - 1;  // ends inside the window
    t.k0 = low_bytes(tile8(L.tile, p), len);
    if (len <= 8) {
      t.k1 = len;
    } else {
      uint64_t h = FNV_OFFSET;
      for (uint32_t c = 8; c < len; c += 8) h = tail_fold(h, low_bytes(tile8(L.tile, p + c), len - c));
      t.k1 = make_k1(len, h);
    }
  } else {
    key_slow(L, a, p, t0 + p, t.k0, t.k1);
  }
  t.off = (uint32_t)(t0 + p);
  t.ph = place_hash(t.k0, t.k1);
  return t;
}

// Combiner insert.  The map's table may hold the same key in two slots (each
// becomes a record and the reducer sums them), so a claim is ONE CAS from
// EMPTY straight to the final tag; the claimer then writes k0/k1.  A reader
// that sees the tag before the keys simply does not match (k1 was cleared to
// 0 at the last flush, so stale keys never match) and probes on — at worst it
// claims a duplicate slot.  Returns the slot, or -1 if `max_groups` groups
// were full.
__device__ __forceinline__ int combiner_slot(SlotGroup* groups, const TokKey& t) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
  const uint32_t tag = make_tag(t.ph);
  uint32_t g = group_of(t.ph, MAP_GROUPS);
  for (int steps = 0; steps < MAP_MAX_GROUP_PROBES;) {
    asm volatile("" ::: "memory");
    SlotGroup& G = groups[g];
    const u32x4 tg = *reinterpret_cast<const u32x4*>(G.tag);
    const u64x2 a1 = *reinterpret_cast<const u64x2*>(&G.k1[0]);
    const u64x2 b1 = *reinterpret_cast<const u64x2*>(&G.k1[2]);
    const u64x2 a0 = *reinterpret_cast<const u64x2*>(&G.k0[0]);
    const u64x2 b0 = *reinterpret_cast<const u64x2*>(&G.k0[2]);
    const bool h0 = tg.x == tag && a1.x == t.k1 && a0.x == t.k0;
    const bool h1 = tg.y == tag && a1.y == t.k1 && a0.y == t.k0;
    const bool h2 = tg.z == tag && b1.x == t.k1 && b0.x == t.k0;
    const bool h3 = tg.w == tag && b1.y == t.k1 && b0.y == t.k0;
    if (h0 | h1 | h2 | h3) return 4 * (int)g + (h0 ? 0 : (h1 ? 1 : (h2 ? 2 : 3)));
    const int e = tg.x == TAG_EMPTY ? 0 : (tg.y == TAG_EMPTY ? 1 : (tg.z == TAG_EMPTY ? 2 : (tg.w == TAG_EMPTY ? 3 : -1)));
    if (e < 0) {
      ++steps;
      g = (g + 1) & (MAP_GROUPS - 1);
      continue;
    }
    if (atomicCAS(&G.tag[e], TAG_EMPTY, tag) == TAG_EMPTY) {
      G.k0[e] = t.k0;
      G.k1[e] = t.k1;
      return 4 * (int)g + e;
    }
    // lost the slot to another lane: re-read this group
  }
  return -1;
}

// Count token t into the combiner; returns false if its neighbourhood is full.
__device__ __forceinline__ bool combine(MapLds& L, const TokKey& t) {
  const int s = combiner_slot(L.grp, t);
  if (s < 0) return false;
  const uint32_t c = atomicAdd(&L.cnt[s], 1u);
  atomicMin(&L.off[s], t.off);
  if (c == 0) atomicAdd(&L.occupied, 1u);
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

__global__ void __launch_bounds__(MAP_THREADS, 4) wc_map_tokenize_v4(MapArgs a) {  // 2 blocks / CU
  __shared__ MapLds L;
  const int tid = threadIdx.x;
  for (int s = tid; s < MAP_SLOTS; s += MAP_THREADS) {
    L.grp[s >> 2].tag[s & 3] = TAG_EMPTY;
    L.grp[s >> 2].k1[s & 3] = K1_EMPTY;
    L.cnt[s] = 0;
    L.off[s] = 0xFFFFFFFFu;
  }
  if (tid == 0) {
    L.occupied = 0;
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

  for (uint64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const uint64_t t0 = tile * MAP_TILE;
    __syncthreads();  // previous tile fully consumed
    // Flush only if the keys the last tile added would not fit again: Zipf
    // text with a small vocabulary keeps its table across many tiles, large
    // vocabularies flush before every tile instead of overflowing mid-tile.
    if (L.occupied + L.last_new > MAP_FILL_MAX) flush_table(L, a);
    if (tid == 0) L.occ_before = L.occupied;
    // ---- commit the prefetched tile to LDS, start loading the next ----
    reinterpret_cast<uint4*>(&L.tile[tid * MAP_BPL])[0] = p0;
    reinterpret_cast<uint4*>(&L.tile[tid * MAP_BPL])[1] = p1;
    if (tid < MAP_HALO / 16) *reinterpret_cast<uint4*>(&L.tile[MAP_TILE + tid * 16]) = ph16;
    if (tid == 0) L.prev = pprev;
    __syncthreads();
    prefetch(tile + gridDim.x);

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
    my_tokens += __popc(starts);
    if (a.ablate == 2) {
      sink ^= dm;
      continue;
    }

    // ---- tokens: two per iteration so their LDS round trips overlap ----
    const uint32_t pbase = tid * MAP_BPL;
    uint32_t todo = starts;
    for (;;) {
      uint32_t failed = 0;
      while (todo) {
        const uint32_t i1 = __ffs(todo) - 1;
        todo &= todo - 1;
        const bool two = todo != 0;
        const uint32_t i2 = two ? (uint32_t)__ffs(todo) - 1 : i1;
        todo &= two ? todo - 1 : todo;
        const TokKey ta = token_key(L, a, t0, pbase + i1, dm >> i1);
        const TokKey tb = token_key(L, a, t0, pbase + i2, dm >> i2);
        if (a.ablate == 1) {
          sink ^= ta.ph + tb.ph;
          continue;
        }
        if (!combine(L, ta)) failed |= 1u << i1;
        if (two && !combine(L, tb)) failed |= 1u << i2;
      }
      todo = failed;
      if (!__syncthreads_or(todo != 0)) break;
      flush_table(L, a);  // neighbourhood full: flush, then retry those tokens
    }
    if (tid == 0) L.last_new = L.occupied > L.occ_before ? L.occupied - L.occ_before : L.occupied;
  }
  __syncthreads();
  if (L.occupied) flush_table(L, a);

  // block totals -> one global atomic
  uint64_t t = my_tokens;
  for (int o = 32; o > 0; o >>= 1) t += __shfl_down(t, o);
  if ((tid & 63) == 0) atomicAdd(&L.tokens, (unsigned long long)t);
  if (sink == 0x9E3779B97F4A7C15ull) atomicOr(&a.flags[FLAG_COUNT - 1], 0u);  // never true
  __syncthreads();
  if (tid == 0) {
    atomicAdd(a.tokens, L.tokens);
    atomicAdd(a.rec.cursor, (unsigned long long)L.used);  // stats: records after the combiner
    a.rec.dir_count[blockIdx.x] = L.nflush;
  }
}

}  // namespace v4
}  // namespace dev

// A/B baseline (WC_MAP_V4=1): the previous lane-serial map kernel.
void launch_map_v4(const MapArgs& a, uint32_t map_blocks, hipStream_t s) {
  hipLaunchKernelGGL(dev::v4::wc_map_tokenize_v4, dim3(map_blocks), dim3(MAP_THREADS), 0, s, a);
}

}  // namespace wc
