// map.hip — wc_map_tokenize: the MAP stage (+ combiner + shuffle write).
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
//  4. Keys are combined in an LDS open-addressing table (the MapReduce
//     combiner), kept across tiles while it is sparse, so Zipf text collapses
//     to one record per hot word per block.  Probing is bounded: a key that
//     finds no slot within MAP_MAX_PROBE ships as a singleton record.
//  5. Flush = shuffle write: each record goes to partition
//     bucket_of(place_hash) in a per-(bucket, block) region, so the reducer
//     reads its bucket contiguously and no global atomics are needed.
#include "kernels.hpp"
#include "lds_table.hpp"

namespace wc {
namespace dev {

struct MapLds {
  uint64_t k0[MAP_SLOTS];
  uint64_t k1[MAP_SLOTS];
  uint32_t cnt[MAP_SLOTS];
  uint32_t off[MAP_SLOTS];
  uint32_t cursor[MAX_REC_BUCKETS];
  uint8_t tile[MAP_TILE + MAP_HALO];
  uint32_t occupied;
  uint32_t prev;
  unsigned long long tokens;
};

// Per-byte "is delimiter" for 8 packed bytes -> 8-bit mask (exact SWAR zero test).
__device__ __forceinline__ uint64_t delim_mask8(uint64_t x) {
  constexpr uint64_t ONES = 0x0101010101010101ull, LOW7 = 0x7F7F7F7F7F7F7F7Full;
  auto zero_bytes = [](uint64_t y) { return ~(((y & LOW7) + LOW7) | y) & 0x8080808080808080ull; };
  const uint64_t m = zero_bytes(x ^ (0x20 * ONES)) | zero_bytes(x ^ (0x0D * ONES)) | zero_bytes(x ^ (0x0A * ONES));
  return ((m >> 7) * 0x0102040810204080ull) >> 56;
}

// 8 bytes starting at byte b (0..63) of the 64-byte window w[0..7] (zero past it).
__device__ __forceinline__ uint64_t window8(const uint64_t (&w)[8], uint32_t b) {
  const uint32_t q = b >> 3, sh = (b & 7) * 8;
  uint64_t lo = 0, hi = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    lo = (q == (uint32_t)j) ? w[j] : lo;
    hi = (q + 1 == (uint32_t)j) ? w[j] : hi;
  }
  return sh ? ((lo >> sh) | (hi << (64 - sh))) : lo;
}

__device__ __forceinline__ uint64_t low_bytes(uint64_t v, uint32_t n) {
  return n >= 8 ? v : (v & ((1ull << (8 * n)) - 1ull));
}

__device__ __forceinline__ void emit_record(MapLds& L, const MapArgs& a, uint64_t k0, uint64_t k1, uint32_t cnt,
                                            uint32_t off) {
  const uint32_t b = bucket_of(place_hash(k0, k1), a.log2_rec_buckets);
  const uint32_t pos = atomicAdd(&L.cursor[b], 1u);
  if (pos < a.rec.cap) {
    const size_t r = ((size_t)b * gridDim.x + blockIdx.x) * a.rec.cap + pos;
    a.rec.k0[r] = k0;
    a.rec.k1[r] = k1;
    a.rec.co[r] = ((uint64_t)cnt << 32) | off;
  }
}

__device__ __forceinline__ void flush_table(MapLds& L, const MapArgs& a) {
  for (int s = threadIdx.x; s < MAP_SLOTS; s += MAP_THREADS) {
    const uint64_t k1 = L.k1[s];
    if (k1 != K1_EMPTY) {
      emit_record(L, a, L.k0[s], k1, L.cnt[s], L.off[s]);
      L.k1[s] = K1_EMPTY;
      L.cnt[s] = 0;
      L.off[s] = 0xFFFFFFFFu;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) L.occupied = 0;
  __syncthreads();
}

// Key of a token that does not end inside the register window.
__device__ __noinline__ void key_slow(const MapLds& L, const MapArgs& a, uint64_t pos, uint64_t g, uint64_t& k0,
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

__global__ void __launch_bounds__(MAP_THREADS) wc_map_tokenize(MapArgs a) {
  __shared__ MapLds L;
  const int tid = threadIdx.x;
  for (int s = tid; s < MAP_SLOTS; s += MAP_THREADS) {
    L.k1[s] = K1_EMPTY;
    L.cnt[s] = 0;
    L.off[s] = 0xFFFFFFFFu;
  }
  const uint32_t nb = 1u << a.log2_rec_buckets;
  for (uint32_t b = tid; b < nb; b += MAP_THREADS) L.cursor[b] = 0;
  if (tid == 0) {
    L.occupied = 0;
    L.tokens = 0;
  }

  const uint64_t ntiles = (a.chunk_len + MAP_TILE - 1) / MAP_TILE;
  uint32_t my_tokens = 0;

  for (uint64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const uint64_t t0 = tile * MAP_TILE;
    __syncthreads();  // previous tile fully consumed
    if (L.occupied > MAP_FLUSH_AT) flush_table(L, a);
    // ---- stage tile + halo into LDS (16-B loads; ' ' past avail_len) ----
    {
      const uint64_t g = t0 + (uint64_t)tid * MAP_BPL;
      uint4* dst = reinterpret_cast<uint4*>(&L.tile[tid * MAP_BPL]);
      if (g + MAP_BPL <= a.avail_len) {
        const uint4* src = reinterpret_cast<const uint4*>(a.text + g);
        const uint4 v0 = src[0], v1 = src[1];
        dst[0] = v0;
        dst[1] = v1;
      } else {
        for (int i = 0; i < MAP_BPL; ++i) L.tile[tid * MAP_BPL + i] = (g + i < a.avail_len) ? a.text[g + i] : 0x20;
      }
      if (tid < MAP_HALO / 16) {
        const uint64_t h = t0 + MAP_TILE + (uint64_t)tid * 16;
        uint4* hd = reinterpret_cast<uint4*>(&L.tile[MAP_TILE + tid * 16]);
        if (h + 16 <= a.avail_len) {
          *hd = *reinterpret_cast<const uint4*>(a.text + h);
        } else {
          for (int i = 0; i < 16; ++i) L.tile[MAP_TILE + tid * 16 + i] = (h + i < a.avail_len) ? a.text[h + i] : 0x20;
        }
      }
      if (tid == 0) L.prev = (t0 == 0 && a.prev_byte >= 0) ? (uint32_t)a.prev_byte : a.text[(int64_t)t0 - 1];
    }
    __syncthreads();

    // ---- 64-byte register window, delimiter / start masks ----
    uint64_t w[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint4 v = reinterpret_cast<const uint4*>(&L.tile[tid * MAP_BPL])[j];
      w[2 * j] = (uint64_t)v.x | ((uint64_t)v.y << 32);
      w[2 * j + 1] = (uint64_t)v.z | ((uint64_t)v.w << 32);
    }
    uint64_t dm = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) dm |= delim_mask8(w[j]) << (8 * j);
    const uint32_t prevb = (tid == 0) ? L.prev : L.tile[tid * MAP_BPL - 1];
    uint32_t starts = (uint32_t)(~dm & ((dm << 1) | (is_delim(prevb) ? 1ull : 0ull)));
    const uint64_t lane_base = t0 + (uint64_t)tid * MAP_BPL;
    if (lane_base >= a.chunk_len) {
      starts = 0;
    } else if (lane_base + MAP_BPL > a.chunk_len) {
      starts &= (1u << (uint32_t)(a.chunk_len - lane_base)) - 1u;
    }
    my_tokens += __popc(starts);

    while (starts) {
      const uint32_t i = __ffs(starts) - 1;
      starts &= starts - 1;
      const uint64_t rest = dm >> i;
      uint64_t k0, k1;
      if (rest != 0) {
        const uint32_t len = (uint32_t)__ffsll((unsigned long long)rest) - 1;  // ends inside the window
        k0 = low_bytes(window8(w, i), len);
        if (len <= 8) {
          k1 = len;
        } else {
          uint64_t h = FNV_OFFSET;
          for (uint32_t c = 8; c < len; c += 8) h = tail_fold(h, low_bytes(window8(w, i + c), len - c));
          k1 = make_k1(len, h);
        }
      } else {
        key_slow(L, a, (uint64_t)tid * MAP_BPL + i, lane_base + i, k0, k1);
      }
      const uint32_t off = (uint32_t)(lane_base + i);
      bool claimed;
      const int s = lds_find_or_claim(L.k0, L.k1, MAP_SLOTS - 1, k0, k1,
                                      (uint32_t)place_hash(k0, k1) & (MAP_SLOTS - 1), MAP_MAX_PROBE, claimed);
      if (s >= 0) {
        atomicAdd(&L.cnt[s], 1u);
        atomicMin(&L.off[s], off);
        if (claimed) atomicAdd(&L.occupied, 1u);
      } else {
        emit_record(L, a, k0, k1, 1u, off);  // crowded neighbourhood: ship the singleton
      }
    }
  }
  __syncthreads();
  flush_table(L, a);

  unsigned long long recs = 0;
  for (uint32_t b = tid; b < nb; b += MAP_THREADS) {
    const uint32_t c = L.cursor[b];
    recs += c;
    a.rec.region_count[(size_t)b * gridDim.x + blockIdx.x] = c < a.rec.cap ? c : a.rec.cap;
    if (c > a.rec.cap) atomicOr(&a.flags[FLAG_REGION_OVF], 1u);
  }
  // block totals -> one global atomic each
  uint64_t t = my_tokens;
  for (int o = 32; o > 0; o >>= 1) {
    t += __shfl_down(t, o);
    recs += __shfl_down(recs, o);
  }
  if ((tid & 63) == 0) atomicAdd(&L.tokens, (unsigned long long)t);
  if ((tid & 63) == 0 && recs) atomicAdd(a.records, recs);
  __syncthreads();
  if (tid == 0) atomicAdd(a.tokens, L.tokens);
}

}  // namespace dev

void launch_map(const MapArgs& a, uint32_t map_blocks, hipStream_t s) {
  hipLaunchKernelGGL(dev::wc_map_tokenize, dim3(map_blocks), dim3(MAP_THREADS), 0, s, a);
}

}  // namespace wc
