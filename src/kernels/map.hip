// map.hip — wc_map_tokenize: the MAP stage (+ combiner + shuffle write).
//
// Reference: mapKernel (/root/reference/main.cu:109-117) runs one thread per
// pre-split input record and only copies words the HOST tokenizer
// (main.cu:181-206) already found.  Here the GPU does the whole map:
//
//  1. A persistent grid of ~2 blocks/CU walks 16 KiB text tiles.  Each tile
//     (+256 B halo) is staged global -> LDS with 16-B loads.
//  2. Each lane owns 32 bytes.  A SWAR packed-byte compare against
//     {0x20,0x0D,0x0A} gives a 32-bit delimiter mask per lane; token starts
//     are  ~d & (d << 1 | carry-in)  where carry-in is the neighbouring lane's
//     last byte (so tokens straddling lanes / tiles / chunks are owned by the
//     unit holding their FIRST byte, and finished through LDS halo or global).
//  3. Words of <= 8 bytes inside the lane are keyed straight from registers
//     (funnel shift + mask: no byte loop, no hash); longer / straddling words
//     take a byte loop that also computes FNV-1a-64.
//  4. Keys are combined in an LDS open-addressing table (the MapReduce
//     combiner), kept across tiles until it fills, so skewed (Zipf) text
//     collapses to one record per hot word per block.
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
};

// Per-byte "is delimiter" for 8 packed bytes -> 8-bit mask (exact SWAR zero test).
__device__ __forceinline__ uint32_t delim_mask8(uint64_t x) {
  constexpr uint64_t ONES = 0x0101010101010101ull, LOW7 = 0x7F7F7F7F7F7F7F7Full;
  auto zero_bytes = [](uint64_t y) { return ~(((y & LOW7) + LOW7) | y) & 0x8080808080808080ull; };
  const uint64_t m = zero_bytes(x ^ (0x20 * ONES)) | zero_bytes(x ^ (0x0D * ONES)) | zero_bytes(x ^ (0x0A * ONES));
  return (uint32_t)(((m >> 7) * 0x0102040810204080ull) >> 56);
}

__device__ __forceinline__ uint64_t sel4(uint32_t i, uint64_t a, uint64_t b, uint64_t c, uint64_t d) {
  return i == 0 ? a : (i == 1 ? b : (i == 2 ? c : d));
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
  if (tid == 0) L.occupied = 0;

  const uint64_t ntiles = (a.chunk_len + MAP_TILE - 1) / MAP_TILE;
  uint64_t my_tokens = 0;

  for (uint64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const uint64_t t0 = tile * MAP_TILE;
    __syncthreads();  // previous tile fully consumed (slow-path LDS reads)
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

    // ---- per-lane delimiter / start masks ----
    const uint4 v0 = reinterpret_cast<const uint4*>(&L.tile[tid * MAP_BPL])[0];
    const uint4 v1 = reinterpret_cast<const uint4*>(&L.tile[tid * MAP_BPL])[1];
    const uint64_t q0 = (uint64_t)v0.x | ((uint64_t)v0.y << 32);
    const uint64_t q1 = (uint64_t)v0.z | ((uint64_t)v0.w << 32);
    const uint64_t q2 = (uint64_t)v1.x | ((uint64_t)v1.y << 32);
    const uint64_t q3 = (uint64_t)v1.z | ((uint64_t)v1.w << 32);
    const uint32_t dm = delim_mask8(q0) | (delim_mask8(q1) << 8) | (delim_mask8(q2) << 16) | (delim_mask8(q3) << 24);
    const uint32_t prevb = (tid == 0) ? L.prev : L.tile[tid * MAP_BPL - 1];
    uint32_t starts = ~dm & ((dm << 1) | (is_delim(prevb) ? 1u : 0u));
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
      const uint32_t rest = dm >> i;
      uint64_t k0, k1;
      if (rest != 0 && __ffs(rest) - 1 <= 8) {
        // fast path: short word fully inside this lane's 32 bytes
        const uint32_t len = __ffs(rest) - 1;
        const uint32_t lo = i >> 3, sh = (i & 7) * 8;
        const uint64_t w0 = sel4(lo, q0, q1, q2, q3);
        const uint64_t w1 = sel4(lo, q1, q2, q3, 0ull);
        const uint64_t v = sh ? ((w0 >> sh) | (w1 << (64 - sh))) : w0;
        k0 = (len == 8) ? v : (v & ((1ull << (8 * len)) - 1ull));
        k1 = len;
      } else {
        // long or lane-straddling word: byte loop through LDS, then global
        uint64_t pos = (uint64_t)tid * MAP_BPL + i, g = lane_base + i, len = 0, h = FNV_OFFSET;
        k0 = 0;
        for (;;) {
          uint32_t c;
          if (pos < (uint64_t)(MAP_TILE + MAP_HALO)) c = L.tile[pos];
          else if (g < a.avail_len) c = a.text[g];
          else break;
          if (is_delim(c)) break;
          if (len < 8) k0 |= (uint64_t)c << (8 * len);
          h = fnv1a_step(h, c);
          ++len, ++pos, ++g;
        }
        k1 = make_k1(len, h);
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
        emit_record(L, a, k0, k1, 1u, off);  // table saturated: ship the singleton
      }
    }
    __syncthreads();
    if (L.occupied >= MAP_FLUSH_AT) flush_table(L, a);
  }
  __syncthreads();
  flush_table(L, a);

  for (uint32_t b = tid; b < nb; b += MAP_THREADS) {
    const uint32_t c = L.cursor[b];
    a.rec.region_count[(size_t)b * gridDim.x + blockIdx.x] = c < a.rec.cap ? c : a.rec.cap;
    if (c > a.rec.cap) atomicOr(&a.flags[FLAG_REGION_OVF], 1u);
  }
  // block token total -> one global atomic
  __shared__ unsigned long long blk_tokens;
  if (tid == 0) blk_tokens = 0;
  __syncthreads();
  uint64_t w = my_tokens;
  for (int o = 32; o > 0; o >>= 1) w += __shfl_down(w, o);
  if ((tid & 63) == 0) atomicAdd(&blk_tokens, (unsigned long long)w);
  __syncthreads();
  if (tid == 0) atomicAdd(a.tokens, blk_tokens);
}

}  // namespace dev

void launch_map(const MapArgs& a, uint32_t map_blocks, hipStream_t s) {
  hipLaunchKernelGGL(dev::wc_map_tokenize, dim3(map_blocks), dim3(MAP_THREADS), 0, s, a);
}

}  // namespace wc
