// sort.hip — stable LSD radix sort of (u64 key, u32 value) pairs + small
// column kernels used by finalisation and the multi-GPU merge.
//
// Used for: first-occurrence output order (the reference gets that order for
// free from its serial append, /root/reference/main.cu:97-104) and the
// deterministic dictionary union of the cross-GPU merge.
//
// Per digit pass (<= 11 bits): wc_radix_hist (LDS histogram per 2048-item tile, plus
// the pass's per-digit totals) -> wc_radix_scan (one block per digit: base of
// the digit + exclusive scan of its row of tile counts; the v8 single-block
// scan of the whole digit-major array took 195 us at 1M keys, this ~5 us) ->
// wc_radix_scatter (stable
// in-tile ranking with 64-lane ballots: lanes with equal digits are matched
// with 8 ballots, ranked with popcount, waves combined through LDS).
#include <algorithm>
#include <utility>

#include "../common/hip_util.hpp"
#include "kernels.hpp"
#include "lds_table.hpp"

namespace wc {
namespace dev {

constexpr int RS_THREADS = 256;
// Tiles of ROUNDS x 256 items per block: 2048 for large sorts, 512 below
// 2^19 items so a 1e5-key sort still spreads over ~200 blocks (A/B: +1.3 % at
// 100k words; 2048 wins at 1M).
constexpr int RS_ROUNDS_BIG = 8, RS_ROUNDS_SMALL = 2;
constexpr uint64_t RS_SMALL_N = 1ull << 19;
__host__ __device__ constexpr int rs_rounds(uint64_t n) { return n < RS_SMALL_N ? RS_ROUNDS_SMALL : RS_ROUNDS_BIG; }
constexpr int RS_WAVES = RS_THREADS / 64;
#ifndef WC_RS_DB
#define WC_RS_DB 8
#endif
constexpr int RS_MAX_DB = WC_RS_DB;              // digit bits per pass (11-bit digits measured slower: the
                                                  // per-round LDS work on 2048 bins outweighs one pass fewer)
constexpr int RS_BINS = 1 << RS_MAX_DB;

// dn (nullable): the item count lives on the device and n is only an upper
// bound: the tiles in use, ceil(*dn / tile), are spread grid-stride over a
// grid sized from the host's estimate (hist rows keep the stride nb of n).
__device__ __forceinline__ uint32_t rs_tiles(uint64_t n, const uint64_t* dn, uint64_t tile) {
  return (uint32_t)(((dn ? *dn : n) + tile - 1) / tile);
}

template <int RS_ROUNDS>
__global__ void __launch_bounds__(RS_THREADS) wc_radix_hist(const uint64_t* keys, uint64_t n, const uint64_t* dn,
                                                            int shift, int db, uint32_t* hist, uint32_t nblocks,
                                                            uint32_t* totals) {
  __shared__ uint32_t h[RS_BINS];
  constexpr uint64_t TILE = RS_THREADS * RS_ROUNDS;
  const uint32_t nd = 1u << db, dmask = nd - 1;
  const uint32_t ntiles = rs_tiles(n, dn, TILE);
  if (dn) n = *dn;
  for (uint32_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    for (uint32_t d = threadIdx.x; d < nd; d += RS_THREADS) h[d] = 0;
    __syncthreads();
    const uint64_t base = (uint64_t)tile * TILE;
    for (int r = 0; r < RS_ROUNDS; ++r) {
      const uint64_t i = base + (uint64_t)r * RS_THREADS + threadIdx.x;
      if (i < n) atomicAdd(&h[(keys[i] >> shift) & dmask], 1u);
    }
    __syncthreads();
    for (uint32_t d = threadIdx.x; d < nd; d += RS_THREADS) {
      hist[(size_t)d * nblocks + tile] = h[d];
      if (h[d]) atomicAdd(&totals[d], h[d]);
    }
    __syncthreads();  // h is cleared for the next tile
  }
}

// Block d: hist row d (tile counts of digit d, nb words) -> exclusive offsets,
// starting at the total of all smaller digits.
__global__ void __launch_bounds__(256) wc_radix_scan(uint32_t* hist, uint32_t stride, const uint32_t* totals,
                                                     uint64_t n, const uint64_t* dn, uint64_t tile_items) {
  __shared__ uint32_t wsum[4];
  const uint32_t d = blockIdx.x;
  const uint32_t nb = rs_tiles(n, dn, tile_items);  // tiles in use
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // base of digit d: sum of totals[0, d)
  uint32_t x = 0;
  for (uint32_t t = tid; t < d; t += 256) x += totals[t];
  for (int o = 32; o > 0; o >>= 1) x += __shfl_down(x, o);
  if (lane == 0) wsum[wave] = x;
  __syncthreads();
  uint32_t run = wsum[0] + wsum[1] + wsum[2] + wsum[3];
  __syncthreads();
  uint32_t* row = hist + (size_t)d * stride;
  for (uint32_t c = 0; c < nb; c += 1024) {  // 4 consecutive words per thread
    const uint32_t b = c + 4 * tid;
    uint32_t v[4], t = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      v[k] = b + k < nb ? row[b + k] : 0u;
      t += v[k];
    }
    uint32_t incl = t;
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(incl, o);
      if (lane >= o) incl += y;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    uint32_t pre = run + incl - t, chunk = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      pre += w < wave ? wsum[w] : 0u;
      chunk += wsum[w];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (b + k < nb) row[b + k] = pre;
      pre += v[k];
    }
    run += chunk;
    __syncthreads();  // wsum reused by the next chunk
  }
}

template <int RS_ROUNDS>
__global__ void __launch_bounds__(RS_THREADS) wc_radix_scatter(const uint64_t* keys, const uint32_t* vals,
                                                               uint64_t* okeys, uint32_t* ovals, uint64_t n,
                                                               const uint64_t* dn, int shift, int db,
                                                               const uint32_t* hist, uint32_t nblocks) {
  __shared__ uint32_t run[RS_BINS];             // next output slot per digit
  __shared__ uint32_t wcnt[RS_WAVES][RS_BINS];  // per-wave digit counts, then offsets
  constexpr uint64_t TILE = RS_THREADS * RS_ROUNDS;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint32_t nd = 1u << db, dmask = nd - 1;
  const uint32_t ntiles = rs_tiles(n, dn, TILE);
  if (dn) n = *dn;
  const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  for (uint32_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    for (uint32_t d = tid; d < nd; d += RS_THREADS) run[d] = hist[(size_t)d * nblocks + tile];
    const uint64_t base = (uint64_t)tile * TILE;
    for (int r = 0; r < RS_ROUNDS; ++r) {
      for (int w = 0; w < RS_WAVES; ++w)
        for (uint32_t d = tid; d < nd; d += RS_THREADS) wcnt[w][d] = 0;
      __syncthreads();
      const uint64_t i = base + (uint64_t)r * RS_THREADS + tid;
      const bool valid = i < n;
      const uint64_t k = valid ? keys[i] : 0;
      const uint32_t d = (uint32_t)(k >> shift) & dmask;
      uint64_t peers = __ballot(valid);
      for (int bit = 0; bit < db; ++bit) {  // lanes with equal digits
        const uint64_t bb = __ballot((d >> bit) & 1);
        peers &= ((d >> bit) & 1) ? bb : ~bb;
      }
      const uint32_t rank = (uint32_t)__popcll(peers & lt);
      if (valid && rank == 0) wcnt[wave][d] = (uint32_t)__popcll(peers);
      __syncthreads();
      for (uint32_t e = tid; e < nd; e += RS_THREADS) {
        uint32_t acc = run[e];
        for (int w = 0; w < RS_WAVES; ++w) {
          const uint32_t c = wcnt[w][e];
          wcnt[w][e] = acc;
          acc += c;
        }
        run[e] = acc;
      }
      __syncthreads();
      if (valid) {
        const uint32_t dst = wcnt[wave][d] + rank;
        okeys[dst] = k;
        ovals[dst] = vals[i];
      }
      __syncthreads();
    }
  }
}

// out.col[i] = in.col[perm[i]] for all six key-table columns (one launch).
__global__ void wc_gather_cols(const uint64_t* k0, const uint64_t* k1, const uint64_t* cnt, const uint64_t* first,
                               const uint64_t* soff, const uint32_t* slen, const uint32_t* perm, uint64_t* ok0,
                               uint64_t* ok1, uint64_t* ocnt, uint64_t* ofirst, uint64_t* osoff, uint32_t* oslen,
                               uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t j = perm[i];
    ok0[i] = k0[j];
    ok1[i] = k1[j];
    ocnt[i] = cnt[j];
    ofirst[i] = first[j];
    osoff[i] = soff[j];
    oslen[i] = slen[j];
  }
}

__global__ void wc_iota_u32(uint32_t* v, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    v[i] = (uint32_t)i;
}
__global__ void wc_fill_u64(uint64_t* p, uint64_t v, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    p[i] = v;
}
inline dim3 grid_for(uint64_t n) {
  uint64_t g = (n + 255) / 256;
  if (g < 1) g = 1;
  if (g > 2048) g = 2048;
  return dim3((unsigned)g);
}

}  // namespace dev

constexpr int RS_MAX_PASSES = 8;  // 64-bit keys

size_t radix_hist_words(uint64_t n, uint64_t n_hint) {
  const uint64_t tile = (uint64_t)dev::RS_THREADS * dev::rs_rounds(n_hint ? n_hint : n);
  const uint64_t nb = (n + tile - 1) / tile;
  return (size_t)dev::RS_BINS * (nb ? nb : 1) + (size_t)dev::RS_BINS * RS_MAX_PASSES;  // tile counts + digit totals
}

// 8-bit digits (11-bit ones measured slower: the per-round LDS work on 2048
// bins outweighs one pass fewer).
void radix_sort_pairs(uint64_t* keys, uint32_t* vals, uint64_t* tmp_keys, uint32_t* tmp_vals, uint32_t* hist,
                      uint64_t n, int bits, hipStream_t s, bool* in_tmp, const uint64_t* dn, uint64_t n_hint) {
  if (in_tmp) *in_tmp = false;
  if (n <= 1 || bits <= 0) return;
  const uint64_t est = dn && n_hint ? std::min(n, n_hint) : n;  // expected items (tile size, grid)
  const bool small = dev::rs_rounds(n_hint ? n_hint : n) == dev::RS_ROUNDS_SMALL;
  const uint64_t tile = (uint64_t)dev::RS_THREADS * (small ? dev::RS_ROUNDS_SMALL : dev::RS_ROUNDS_BIG);
  const uint32_t nb = (uint32_t)((n + tile - 1) / tile);  // hist row stride (upper bound)
  const uint32_t grid = dn ? (uint32_t)std::min<uint64_t>(nb, (est + est / 4 + tile - 1) / tile + 1) : nb;
  const int passes = (bits + dev::RS_MAX_DB - 1) / dev::RS_MAX_DB;
  const int db = (bits + passes - 1) / passes;
  uint32_t* totals = hist + (size_t)dev::RS_BINS * nb;  // [passes][2^db]
  WC_HIP_CHECK(hipMemsetAsync(totals, 0, (size_t)dev::RS_BINS * passes * sizeof(uint32_t), s));
  uint64_t *ki = keys, *ko = tmp_keys;
  uint32_t *vi = vals, *vo = tmp_vals;
  for (int p = 0; p < passes; ++p) {
    const int shift = db * p;
    uint32_t* tot = totals + (size_t)dev::RS_BINS * p;
    if (small)
      hipLaunchKernelGGL(dev::wc_radix_hist<dev::RS_ROUNDS_SMALL>, dim3(grid), dim3(dev::RS_THREADS), 0, s, ki, n, dn,
                         shift, db, hist, nb, tot);
    else
      hipLaunchKernelGGL(dev::wc_radix_hist<dev::RS_ROUNDS_BIG>, dim3(grid), dim3(dev::RS_THREADS), 0, s, ki, n, dn,
                         shift, db, hist, nb, tot);
    hipLaunchKernelGGL(dev::wc_radix_scan, dim3(1u << db), dim3(256), 0, s, hist, nb, tot, n, dn, tile);
    if (small)
      hipLaunchKernelGGL(dev::wc_radix_scatter<dev::RS_ROUNDS_SMALL>, dim3(grid), dim3(dev::RS_THREADS), 0, s, ki, vi,
                         ko, vo, n, dn, shift, db, hist, nb);
    else
      hipLaunchKernelGGL(dev::wc_radix_scatter<dev::RS_ROUNDS_BIG>, dim3(grid), dim3(dev::RS_THREADS), 0, s, ki, vi,
                         ko, vo, n, dn, shift, db, hist, nb);
    std::swap(ki, ko);
    std::swap(vi, vo);
  }
  if (ki != keys && in_tmp) {  // odd pass count: the caller takes the result from tmp
    *in_tmp = true;
  } else if (ki != keys) {
    WC_CHECK(dn == nullptr, "radix_sort_pairs: a device-side count needs in_tmp");
    WC_HIP_CHECK(hipMemcpyAsync(keys, ki, n * sizeof(uint64_t), hipMemcpyDeviceToDevice, s));
    WC_HIP_CHECK(hipMemcpyAsync(vals, vi, n * sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
  }
}

void launch_gather_cols(const uint64_t* k0, const uint64_t* k1, const uint64_t* cnt, const uint64_t* first,
                        const uint64_t* soff, const uint32_t* slen, const uint32_t* perm, uint64_t* ok0, uint64_t* ok1,
                        uint64_t* ocnt, uint64_t* ofirst, uint64_t* osoff, uint32_t* oslen, uint64_t n, hipStream_t s) {
  if (n)
    hipLaunchKernelGGL(dev::wc_gather_cols, dev::grid_for(n), dim3(256), 0, s, k0, k1, cnt, first, soff, slen, perm,
                       ok0, ok1, ocnt, ofirst, osoff, oslen, n);
}

void launch_iota_u32(uint32_t* v, uint64_t n, hipStream_t s) {
  if (n) hipLaunchKernelGGL(dev::wc_iota_u32, dev::grid_for(n), dim3(256), 0, s, v, n);
}
void launch_fill_u64(uint64_t* p, uint64_t v, uint64_t n, hipStream_t s) {
  if (n) hipLaunchKernelGGL(dev::wc_fill_u64, dev::grid_for(n), dim3(256), 0, s, p, v, n);
}
}  // namespace wc
