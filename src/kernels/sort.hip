// sort.hip — stable LSD radix sort of (u64 key, u32 value) pairs + small
// column kernels used by finalisation and the multi-GPU merge.
//
// Used for: first-occurrence output order (the reference gets that order for
// free from its serial append, /root/reference/main.cu:97-104) and the
// sort-based-reduce A/B (tools/sort_vs_hash.py).
//
// Onesweep form: ONE histogram launch counts the digits of every pass
// (wc_os_hist: per-block LDS histograms, one global add per digit), then ONE
// launch per 8-bit digit pass (wc_os_pass).  A pass block takes the next tile
// of 8192 items from a counter (tiles start in order, so a block only ever
// waits on tiles already running), ranks its items stably in LDS (64-lane
// ballots match equal digits), publishes its per-digit tile count, and finds
// the count of every earlier tile by decoupled look-back: a flag/count word per
// (tile, digit) that is AGGREGATE (this tile only) or INCLUSIVE (all tiles up to
// it) — summing aggregates backwards until the first inclusive word.  Items go
// straight to their final slot of the pass.  A 32-bit key sort is 5 launches
// (round 2: 12 — histogram, scan and scatter per pass).  Tiles of 8192 items
// (1024-thread blocks) keep the look-back to a dozen hops at 1e5 keys.
#include <algorithm>
#include <utility>

#include "../common/hip_util.hpp"
#include "kernels.hpp"
#include "lds_table.hpp"

namespace wc {
namespace dev {

constexpr int OS_THREADS = 1024;                      // pass blocks: 16 waves
constexpr int OS_WAVES = OS_THREADS / 64;
constexpr int OS_ROUNDS = 8;                          // items per lane
constexpr uint32_t OS_WAVE_ITEMS = 64 * OS_ROUNDS;    // a wave's contiguous segment of its tile
constexpr uint32_t OS_TILE = OS_THREADS * OS_ROUNDS;  // 8192 items per tile
constexpr int OS_HIST_THREADS = 256;
constexpr int OS_DB = 8;                              // digit bits per pass
constexpr int OS_BINS = 1 << OS_DB;
constexpr int OS_MAX_PASSES = 8;                      // 64-bit keys
constexpr uint32_t OS_AGG = 1u << 30, OS_INC = 2u << 30, OS_VAL = (1u << 30) - 1u;

__host__ __device__ inline uint32_t os_tiles(uint64_t n) { return (uint32_t)((n + OS_TILE - 1) / OS_TILE); }

// Digit counts of all passes: ghist[p * 256 + d] = items whose digit p is d.
__global__ void __launch_bounds__(OS_HIST_THREADS) wc_os_hist(const uint64_t* keys, uint64_t n, const uint64_t* dn,
                                                              int passes, uint32_t* ghist) {
  __shared__ uint32_t h[OS_MAX_PASSES][OS_BINS];
  for (int i = threadIdx.x; i < OS_MAX_PASSES * OS_BINS; i += OS_HIST_THREADS) (&h[0][0])[i] = 0;
  __syncthreads();
  if (dn) n = *dn;
  for (uint64_t i = blockIdx.x * (uint64_t)OS_HIST_THREADS + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * OS_HIST_THREADS) {
    const uint64_t k = keys[i];
    for (int p = 0; p < passes; ++p) atomicAdd(&h[p][(k >> (OS_DB * p)) & (OS_BINS - 1)], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < passes * OS_BINS; i += OS_HIST_THREADS) {
    const uint32_t c = (&h[0][0])[i];
    if (c) atomicAdd(&ghist[i], c);
  }
}

// One digit pass.  ghist: this pass's 256 digit totals; ctr: tile counter;
// look: [tiles][256] flag/count words (zeroed).  Item order inside a tile is
// wave-major (wave w owns items [512 w, 512 w + 512), lane-contiguous per
// round), so a wave's running per-digit counters give every item its stable
// rank among its wave's items; a block scan over the waves completes it.
__global__ void __launch_bounds__(OS_THREADS) wc_os_pass(const uint64_t* keys, const uint32_t* vals, uint64_t* okeys,
                                                         uint32_t* ovals, uint64_t n, const uint64_t* dn, int shift,
                                                         const uint32_t* ghist, uint32_t* ctr, uint32_t* look) {
  __shared__ uint32_t wcnt[OS_WAVES][OS_BINS];  // per-wave running digit counts, then the wave's offsets
  __shared__ uint32_t base[OS_BINS];            // first output slot of each digit in this tile
  __shared__ uint32_t wsum[4];
  __shared__ uint32_t s_tile;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (dn) n = *dn;
  const uint32_t ntiles = os_tiles(n);
  if (tid == 0) s_tile = atomicAdd(ctr, 1u);
  __syncthreads();
  const uint32_t tile = s_tile;
  if (tile >= ntiles) return;  // block-uniform: a grid sized for an upper bound of n
  for (int i = tid; i < OS_WAVES * OS_BINS; i += OS_THREADS) (&wcnt[0][0])[i] = 0;
  __syncthreads();
  const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  const uint64_t w0 = (uint64_t)tile * OS_TILE + (uint64_t)wave * OS_WAVE_ITEMS;
  uint64_t k[OS_ROUNDS];
  uint32_t v[OS_ROUNDS], pos[OS_ROUNDS];
#pragma unroll
  for (int r = 0; r < OS_ROUNDS; ++r) {
    const uint64_t i = w0 + (uint64_t)r * 64 + lane;
    const bool valid = i < n;
    k[r] = valid ? keys[i] : 0;
    v[r] = valid ? vals[i] : 0;
  }
#pragma unroll
  for (int r = 0; r < OS_ROUNDS; ++r) {
    const bool valid = w0 + (uint64_t)r * 64 + lane < n;
    const uint32_t d = (uint32_t)(k[r] >> shift) & (OS_BINS - 1);
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (int bit = 0; bit < OS_DB; ++bit) {  // lanes with equal digits
      const uint64_t bb = __ballot((d >> bit) & 1);
      peers &= ((d >> bit) & 1) ? bb : ~bb;
    }
    const uint32_t rank = (uint32_t)__popcll(peers & lt);
    const int leader = valid ? __ffsll((unsigned long long)peers) - 1 : lane;
    uint32_t old = 0;
    if (valid && rank == 0) {  // one leader per digit per round: the wave's counter, no atomics
      old = wcnt[wave][d];
      wcnt[wave][d] = old + (uint32_t)__popcll(peers);
    }
    old = (uint32_t)__shfl((int)old, leader);
    pos[r] = valid ? old + rank : 0xFFFFFFFFu;
    __builtin_amdgcn_wave_barrier();
  }
  __syncthreads();
  // digit d = tid < 256: the waves' offsets (exclusive over waves) and the tile total
  uint32_t acc = 0;
  if (tid < OS_BINS) {
#pragma unroll
    for (int w = 0; w < OS_WAVES; ++w) {
      const uint32_t c = wcnt[w][tid];
      wcnt[w][tid] = acc;
      acc += c;
    }
    // exclusive scan of the digit totals (thread d owns digit d)
    const uint32_t tot = ghist[tid];
    uint32_t incl = tot;
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(incl, o);
      if (lane >= o) incl += y;
    }
    if (lane == 63) wsum[wave] = incl;
    // decoupled look-back for digit d over the tiles before this one
    uint32_t* my = look + (size_t)tile * OS_BINS + tid;
    uint32_t excl = 0;
    if (tile == 0) {
      __hip_atomic_store(my, OS_INC | acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      __hip_atomic_store(my, OS_AGG | acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      // the flags of up to OS_LB predecessors are loaded together (one round
      // trip, not one per tile), then consumed newest first: aggregates add up
      // until the first inclusive word; an unpublished tile (0) is re-read
      constexpr int OS_LB = 16;
      int t = (int)tile - 1;
      for (;;) {
        uint32_t f[OS_LB];
#pragma unroll
        for (int q = 0; q < OS_LB; ++q)
          f[q] = t - q >= 0 ? __hip_atomic_load(look + (size_t)(t - q) * OS_BINS + tid, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT)
                            : OS_INC;  // never reached: tile 0 is inclusive
        int used = OS_LB;
        bool done = false;
#pragma unroll
        for (int q = 0; q < OS_LB; ++q) {
          if (done || used < OS_LB) continue;
          if (f[q] == 0) {
            used = q;  // tile t - q started earlier (tiles are taken in order) and publishes soon
          } else {
            excl += f[q] & OS_VAL;
            done = (f[q] & OS_INC) != 0;
          }
        }
        if (done) break;
        t -= used;
        if (used < OS_LB) __builtin_amdgcn_s_sleep(1);
      }
      __hip_atomic_store(my, OS_INC | (excl + acc), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    base[tid] = incl - tot + excl;  // + the digit's base (the waves before: added below)
  }
  __syncthreads();
  if (tid < OS_BINS) {
    uint32_t before = 0;
    for (int w = 0; w < wave; ++w) before += wsum[w];
    base[tid] += before;
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < OS_ROUNDS; ++r) {
    if (pos[r] == 0xFFFFFFFFu) continue;
    const uint32_t d = (uint32_t)(k[r] >> shift) & (OS_BINS - 1);
    const uint32_t dst = base[d] + wcnt[wave][d] + pos[r];
    okeys[dst] = k[r];
    ovals[dst] = v[r];
  }
}

// out.col[i] = in.col[perm[i]] for all six key-table columns (one launch).
__global__ void wc_gather_cols(const uint64_t* k0, const uint64_t* k1, const uint64_t* cnt, const uint64_t* first,
                               const uint64_t* soff, const uint32_t* slen, const uint32_t* perm, uint64_t* ok0,
                               uint64_t* ok1, uint64_t* ocnt, uint64_t* ofirst, uint64_t* osoff, uint32_t* oslen,
                               uint64_t n, const uint64_t* dn) {
  if (dn) n = *dn;
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

// Workspace (32-bit words): digit totals [8][256] | tile counters [8] (+ pad)
// | look-back words [passes][tiles][256] — zeroed by one memset per sort.
size_t radix_hist_words(uint64_t n, uint64_t /*n_hint*/) {
  const uint64_t tiles = dev::os_tiles(n ? n : 1);
  return (size_t)dev::OS_MAX_PASSES * dev::OS_BINS + 64 + (size_t)dev::OS_MAX_PASSES * tiles * dev::OS_BINS;
}

void radix_sort_pairs(uint64_t* keys, uint32_t* vals, uint64_t* tmp_keys, uint32_t* tmp_vals, uint32_t* hist,
                      uint64_t n, int bits, hipStream_t s, bool* in_tmp, const uint64_t* dn, uint64_t n_hint) {
  if (in_tmp) *in_tmp = false;
  if (n <= 1 || bits <= 0) return;
  WC_CHECK(n < (1ull << 30), "radix_sort_pairs: at most 2^30 items (look-back counts are 30-bit)");
  const int passes = std::min((bits + dev::OS_DB - 1) / dev::OS_DB, dev::OS_MAX_PASSES);
  const uint32_t tiles = dev::os_tiles(n);  // upper bound with a device-side count
  uint32_t* ghist = hist;
  uint32_t* ctr = hist + dev::OS_MAX_PASSES * dev::OS_BINS;
  uint32_t* look = ctr + 64;
  const size_t zero_words = (size_t)dev::OS_MAX_PASSES * dev::OS_BINS + 64 + (size_t)passes * tiles * dev::OS_BINS;
  WC_HIP_CHECK(hipMemsetAsync(hist, 0, zero_words * sizeof(uint32_t), s));
  // histogram grid: ~2048 items per block (est: the expected device-side count)
  const uint64_t est = dn && n_hint ? std::min(n, n_hint) : n;
  const uint32_t hgrid = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(4096, (est + 2047) / 2048));
  hipLaunchKernelGGL(dev::wc_os_hist, dim3(hgrid), dim3(dev::OS_HIST_THREADS), 0, s, keys, n, dn, passes, ghist);
  // one block per tile of the bound n (with a device-side count the blocks past it exit at once)
  const uint32_t grid = tiles;
  uint64_t *ki = keys, *ko = tmp_keys;
  uint32_t *vi = vals, *vo = tmp_vals;
  for (int p = 0; p < passes; ++p) {
    hipLaunchKernelGGL(dev::wc_os_pass, dim3(grid), dim3(dev::OS_THREADS), 0, s, ki, vi, ko, vo, n, dn, dev::OS_DB * p,
                       ghist + (size_t)p * dev::OS_BINS, ctr + p, look + (size_t)p * tiles * dev::OS_BINS);
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
                        uint64_t* ocnt, uint64_t* ofirst, uint64_t* osoff, uint32_t* oslen, uint64_t n, hipStream_t s,
                        const uint64_t* dn) {
  if (n)
    hipLaunchKernelGGL(dev::wc_gather_cols, dev::grid_for(n), dim3(256), 0, s, k0, k1, cnt, first, soff, slen, perm,
                       ok0, ok1, ocnt, ofirst, osoff, oslen, n, dn);
}

void launch_iota_u32(uint32_t* v, uint64_t n, hipStream_t s) {
  if (n) hipLaunchKernelGGL(dev::wc_iota_u32, dev::grid_for(n), dim3(256), 0, s, v, n);
}
void launch_fill_u64(uint64_t* p, uint64_t v, uint64_t n, hipStream_t s) {
  if (n) hipLaunchKernelGGL(dev::wc_fill_u64, dev::grid_for(n), dim3(256), 0, s, p, v, n);
}
}  // namespace wc
