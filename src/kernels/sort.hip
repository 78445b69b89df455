// sort.hip — the first-occurrence output order (the reference gets that order
// for free from its serial append, /root/reference/main.cu:97-104): the
// three-launch sample sort (up to 400k keys), ranks from a bitmap of first
// offsets (above), the stable LSD radix sort of (u64 key, u32 value) pairs
// (fallbacks; also the sort-based-reduce A/B, tools/sort_vs_hash.py), and small
// column kernels used by finalisation and the multi-GPU merge.
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
#include <cstdlib>
#include <utility>

#include "../common/hip_util.hpp"
#include "kernels.hpp"
#include "bounds.hpp"
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

// ---- first-occurrence order: sample sort of UNIQUE keys, three launches ----
// The keys are first offsets, distinct per word, so no stability is needed.
// Sorting networks cost ~400-600 cycles per dependent phase on one CU
// (tools/probe/clock_probe.hip: a 4096-key LDS bitonic sort takes 34 us, a
// one-wave 512-key register sort 11 us), so no step here sorts with one:
//   wc_fo_split  one block: a FO_SAMPLE-key sample (strided over the key
//                column, or every occupied slot of windows spread over the
//                table) histogrammed over log-scale value bins (exact below
//                2^M, then 2^M bins per octave); a block scan turns the
//                histogram into a monotone map log-bin -> one of FO_BINS bins
//                holding ~1/FO_BINS of the sample each;
//   wc_fo_bin    one block per 4096 source rows (a table bucket): every row ->
//                its bin through the map (in LDS), the block's rows written to
//                its own segment in bin order as 48-byte entries carrying the
//                whole row, and per bin the block's count and local offset
//                (bin-major matrices) — no global atomics;
//   wc_fo_sort   one block per bin: its output offset = the sum of its column
//                of local offsets, its rows gathered from every block's segment
//                into LDS, each row's rank in the bin counted directly (small
//                bins) or after a counting sort into value sub-buckets (larger
//                ones), the six output columns written from the entries.
// A bin above its LDS capacity (a pathological value distribution) raises *ovf
// and the caller redoes the order with the radix sort.
#ifndef WC_FO_ROWS
#define WC_FO_ROWS 2048
#endif
// Bins per order: 512 up to FO_SMALL_KEYS keys, FO_BINS (the maximum, LDS
// sizing) above — bins average <= 800 rows either way (one wave sorts 2048).
constexpr int FO_BINS = 2048, FO_BINS_SMALL = 512, FO_ROWS = WC_FO_ROWS, FO_SAMPLE = 4096;
constexpr uint64_t FO_SMALL_KEYS = 400000;
static_assert(FO_BINS % 1024 == 0 && FO_BINS_SMALL % (2 * 64) == 0 && FO_BINS_SMALL <= 1024,
              "fo bins: whole wc_fo_bin scan passes, whole wc_fo_sort blocks");
constexpr int FO_RPT = FO_ROWS / 1024;  // wc_fo_bin rows per thread
static_assert(FO_ROWS % 1024 == 0 && TAB_SLOTS % FO_ROWS == 0, "fo_bin: whole rows per thread, blocks inside a bucket");

// WC_FO_STAMPS (debug API): per kernel K, [16 K + p] = the max over blocks of
// the 100 MHz wall time from the block's start to its phase p.
__device__ unsigned long long* fo_stamps = nullptr;
struct FoClock {
  uint64_t t0;
  int k;
  __device__ FoClock(int kernel) : t0(wall_clock64()), k(kernel) {}
  __device__ void at(int p) {
    if (fo_stamps && threadIdx.x == 0) atomicMax(&fo_stamps[16 * k + p], (unsigned long long)(wall_clock64() - t0));
  }
};

struct alignas(16) FoEntry {
  uint64_t first, k0, k1, cnt, soff;
  uint32_t slen, pad;
};
static_assert(sizeof(FoEntry) == 48, "48-byte entries");

// Block-wide exclusive scan of `n` (a multiple of T, or < T) LDS counters in
// place, T threads; returns the total.  `ws`: T / 64 words of scratch.
template <int T>
__device__ __forceinline__ uint32_t lds_exclusive_scan(uint32_t* c, int n, uint32_t* ws) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int per = n >= T ? n / T : (tid < n ? 1 : 0);  // n < T: one counter on the first n threads
  uint32_t own = 0;
  if (per % 4 == 0) {  // 16-byte reads: 4x fewer LDS trips and bank conflicts
    for (int i = 0; i < per; i += 4) {
      const uint4 q = *reinterpret_cast<const uint4*>(&c[tid * per + i]);
      own += q.x + q.y + q.z + q.w;
    }
  } else {
    for (int i = 0; i < per; ++i) own += c[tid * per + i];
  }
  uint32_t x = own;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  if (lane == 63) ws[wave] = x;
  __syncthreads();
  uint32_t before = 0, total = 0;
  for (int w = 0; w < T / 64; ++w) {
    before += w < wave ? ws[w] : 0u;
    total += ws[w];
  }
  uint32_t run = before + x - own;
  if (per % 4 == 0) {
    for (int i = 0; i < per; i += 4) {
      uint4 q = *reinterpret_cast<const uint4*>(&c[tid * per + i]);
      const uint32_t a = run, b2 = a + q.x, c2 = b2 + q.y, d2 = c2 + q.z;
      run = d2 + q.w;
      q = make_uint4(a, b2, c2, d2);
      *reinterpret_cast<uint4*>(&c[tid * per + i]) = q;
    }
  } else {
    for (int i = 0; i < per; ++i) {
      const uint32_t v = c[tid * per + i];
      c[tid * per + i] = run;
      run += v;
    }
  }
  __syncthreads();
  return total;
}

__global__ void __launch_bounds__(1024) wc_fo_split(OrderSrc src, uint32_t M, uint32_t nb, uint16_t* map, uint32_t* ctl) {
  FoClock clk(0);
  __shared__ alignas(16) uint32_t hist[FO_LOGBINS];
  __shared__ uint32_t ws[16];
  __shared__ uint32_t nvalid;
  const uint32_t tid = threadIdx.x;
  if (tid == 0) {
    ctl[0] = 0;  // the overflow word
    nvalid = 0;
  }
  for (int i = tid; i < FO_LOGBINS; i += 1024) hist[i] = 0;
  __syncthreads();
  clk.at(1);
  constexpr int R = FO_SAMPLE / 1024;
  if (src.table) {
    // 1024 windows of 16 slots spread over the table, one per thread, their
    // first offsets read whole (16-byte loads; an empty slot of an occupied
    // bucket holds ~0 — the reducer's slice initialisation — and a stray value
    // could only skew the sample, never the order): every occupied slot in
    // them is a sample — a sparse table still yields a uniform sample —
    // thinned to ~0.9 FO_SAMPLE when they hold more.  (One slot per window
    // would bias it: slot order inside a group is claim order.)
    const uint64_t cap = (uint64_t)1 << (src.t.log2_buckets + TAB_SLOTS_LOG2);
    const uint64_t p = ((uint64_t)tid * cap / 1024) & ~15ull;
    uint64_t f[16];
    uint32_t vm = 0;
    if (src.t.occupancy[p >> TAB_SLOTS_LOG2] != 0) {
      const ulonglong2* w = reinterpret_cast<const ulonglong2*>(src.t.first + p);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const ulonglong2 q = w[j];
        f[2 * j] = q.x;
        f[2 * j + 1] = q.y;
      }
#pragma unroll
      for (int j = 0; j < 16; ++j) vm |= (f[j] != ~0ull ? 1u : 0u) << j;
    }
    atomicAdd(&nvalid, (uint32_t)__popc(vm));
    __syncthreads();
    const uint32_t V = nvalid;
    const uint32_t keep = V <= (uint32_t)FO_SAMPLE ? 0xFFFFFFFFu
                                                    : (uint32_t)(0.9 * (double)FO_SAMPLE / V * 4294967296.0);
#pragma unroll
    for (int j = 0; j < 16; ++j)
      if ((vm >> j) & 1u)
        if (keep == 0xFFFFFFFFu || (uint32_t)(((tid << 4) + j) * 0x9E3779B1u) < keep)
          atomicAdd(&hist[fo_logbin(f[j], M)], 1u);
  } else {
    const uint64_t n = src.dn ? *src.dn : src.n;
    const uint64_t m = n < (uint64_t)FO_SAMPLE ? n : (uint64_t)FO_SAMPLE;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint32_t i = (uint32_t)r * 1024 + tid;
      if (i < m) atomicAdd(&hist[fo_logbin(src.first[i * n / m], M)], 1u);
    }
  }
  __syncthreads();
  clk.at(2);
  const uint32_t V = lds_exclusive_scan<1024>(hist, FO_LOGBINS, ws);
  clk.at(3);
  // log-bin -> bin: the sample share below it, in nb equal parts (monotone:
  // a float scaling, no integer division)
  const float inv = V ? (float)nb / (float)V : 0.0f;
  for (int i = tid; i < FO_LOGBINS; i += 1024)
    map[i] = (uint16_t)min(nb - 1, (uint32_t)((float)hist[i] * inv));
  clk.at(4);
}

// Block k: source rows [FO_ROWS k, FO_ROWS (k + 1)) (table: slots of bucket FO_ROWS k / TAB_SLOTS).
// cntm / loffm are bin-major: [bin * nblk + k].
// Exact log-bin histogram of a column source's keys (the merged table): LDS
// counts per block, one global add per nonzero bin; hist zeroed by the caller
// (wc_fo_sort zeroes it again after its use).  Replaces the one-block sample.
constexpr int FO_HIST_ROWS = 4096;  // rows per block
__global__ void __launch_bounds__(1024) wc_fo_hist(OrderSrc src, uint32_t M, uint32_t* hist) {
  __shared__ uint32_t lh[FO_LOGBINS];
  const uint32_t tid = threadIdx.x;
  for (int i = tid; i < FO_LOGBINS; i += 1024) lh[i] = 0;
  __syncthreads();
  const uint64_t n = src.dn ? *src.dn : src.n;
  for (uint64_t i = (uint64_t)blockIdx.x * FO_HIST_ROWS + tid; i < n; i += (uint64_t)gridDim.x * FO_HIST_ROWS)
    for (uint32_t r = 0; r < FO_HIST_ROWS && i + r < n; r += 1024) atomicAdd(&lh[fo_logbin(src.first[i + r], M)], 1u);
  __syncthreads();
  for (int i = tid; i < FO_LOGBINS; i += 1024)
    if (lh[i]) atomicAdd(&hist[i], lh[i]);
}

// phist (nullable): the reducer's histogram of every key's log-bin — each
// block then builds the log-bin -> bin map itself (no wc_fo_split launch).
__global__ void __launch_bounds__(1024) wc_fo_bin(OrderSrc src, uint32_t M, uint32_t nb, const uint16_t* map,
                                                  const uint32_t* phist, uint32_t* cntm, uint32_t* loffm, FoEntry* seg,
                                                  uint32_t* ctl) {
  FoClock clk(1);
  __shared__ uint16_t lmap[FO_LOGBINS];
  __shared__ alignas(16) uint32_t lh[FO_LOGBINS];
  __shared__ uint32_t lc[FO_BINS], ws[16];
  const uint32_t tid = threadIdx.x, k = blockIdx.x, nblk = gridDim.x;
  const uint64_t i0 = (uint64_t)k * FO_ROWS;
  uint64_t lim;
  if (src.table) lim = src.t.occupancy[i0 >> TAB_SLOTS_LOG2] ? i0 + FO_ROWS : i0;  // an empty bucket's slots are undefined
  else lim = src.dn ? *src.dn : src.n;
  // rows first (their loads overlap the map copy)
  FoEntry e[FO_RPT];
  bool ok[FO_RPT];
#pragma unroll
  for (int r = 0; r < FO_RPT; ++r) {
    const uint64_t i = i0 + (uint64_t)r * 1024 + tid;
    ok[r] = i < lim;
    if (src.table) {
      const uint64_t k1 = ok[r] ? src.t.k1[i] : K1_EMPTY;
      ok[r] = k1 != K1_EMPTY;
      if (ok[r]) {
        const bool h = key_is_hashed(k1);
        e[r].first = src.t.first[i];
        e[r].k0 = src.t.k0[i];
        e[r].k1 = k1;
        e[r].cnt = src.t.cnt[i];
        e[r].soff = h ? src.t.sref_off[i] : 0;
        e[r].slen = h ? src.t.sref_len[i] : 0;
      }
    } else if (ok[r]) {
      e[r].first = src.first[i];
      e[r].k0 = src.k0[i];
      e[r].k1 = src.k1[i];
      e[r].cnt = src.cnt[i];
      e[r].soff = src.soff[i];
      e[r].slen = src.slen[i];
    }
    e[r].pad = 0;
  }
  if (phist) {  // the map from the exact histogram (as wc_fo_split does from its sample)
    const uint4* g = reinterpret_cast<const uint4*>(phist);
    uint4* l = reinterpret_cast<uint4*>(lh);
    for (int i = tid; i < FO_LOGBINS / 4; i += 1024) l[i] = g[i];
    if (k == 0 && tid == 0) ctl[0] = 0;  // the overflow word (wc_fo_sort runs after every block)
    __syncthreads();
    const uint32_t V = lds_exclusive_scan<1024>(lh, FO_LOGBINS, ws);
    const float inv = V ? (float)nb / (float)V : 0.0f;
    for (int i = tid; i < FO_LOGBINS; i += 1024)
      lmap[i] = (uint16_t)min(nb - 1, (uint32_t)((float)lh[i] * inv));
  } else {
    const uint4* g = reinterpret_cast<const uint4*>(map);
    uint4* l = reinterpret_cast<uint4*>(lmap);
    for (int i = tid; i < FO_LOGBINS * 2 / 16; i += 1024) l[i] = g[i];
  }
  for (uint32_t b = tid; b < nb; b += 1024) lc[b] = 0;
  __syncthreads();
  clk.at(1);
  uint32_t bb[FO_RPT], lp[FO_RPT];
#pragma unroll
  for (int r = 0; r < FO_RPT; ++r) {
    bb[r] = nb;
    if (ok[r]) {
      bb[r] = lmap[fo_logbin(e[r].first, M)];
      lp[r] = atomicAdd(&lc[bb[r]], 1u);
    }
  }
  __syncthreads();
  clk.at(2);
  for (uint32_t b = tid; b < nb; b += 1024) cntm[(size_t)b * nblk + k] = lc[b];
  lds_exclusive_scan<1024>(lc, (int)nb, ws);  // nb < 1024: one bin on each of the first nb threads
  clk.at(3);
  for (uint32_t b = tid; b < nb; b += 1024) loffm[(size_t)b * nblk + k] = lc[b];
  FoEntry* out = seg + i0;
#pragma unroll
  for (int r = 0; r < FO_RPT; ++r)
    if (bb[r] != nb) out[lc[bb[r]] + lp[r]] = e[r];
  clk.at(4);
}

// Per-wave sort of one bin (m <= FO_WAVE_CAP rows), no block barrier: the
// wave gathers its bin's (first, entry) pairs into its LDS region, counting-
// sorts them into FO_WSUB value sub-buckets over [min, max] (a monotone float
// scaling), and each row's rank = its sub-bucket's start + the keys below it
// inside the sub-bucket.  The block's waves each take a bin; bins above the
// wave capacity are sorted afterwards by the whole block (LDS bitonic over
// the block's combined regions, up to FO_BLOCK_CAP rows).
constexpr int FO_SORT_WAVES = 2, FO_WAVE_CAP = 2048, FO_WSUB = 512;
constexpr int FO_BLOCK_CAP = FO_SORT_WAVES * FO_WAVE_CAP * 2;  // 12-byte rows in the 24-byte-per-row regions

struct FoWaveLds {
  alignas(16) uint64_t ka[FO_WAVE_CAP];
  uint64_t kb[FO_WAVE_CAP];
  uint32_t va[FO_WAVE_CAP];
  uint32_t vb[FO_WAVE_CAP];
  uint32_t sub[FO_WSUB];
};

// Bitonic sort of P (a power of two) keys + values in LDS, T threads.
template <int T, bool V>
__device__ __forceinline__ void lds_bitonic(uint64_t* k, uint32_t* v, uint32_t P) {
  for (uint32_t size = 2; size <= P; size <<= 1) {
    for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
      __syncthreads();
      for (uint32_t t = threadIdx.x; t < P / 2; t += T) {
        const uint32_t i = 2 * t - (t & (stride - 1)), j = i + stride;
        const uint64_t a = k[i], b = k[j];
        if ((a > b) == ((i & size) == 0)) {
          k[i] = b;
          k[j] = a;
          if (V) {
            const uint32_t x = v[i];
            v[i] = v[j];
            v[j] = x;
          }
        }
      }
    }
  }
  __syncthreads();
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
  const uint32_t lane = __lane_id();
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o);
    if (lane >= (uint32_t)o) x += y;
  }
  return x;
}

__global__ void __launch_bounds__(64 * FO_SORT_WAVES) wc_fo_sort(OrderDst dst, const uint32_t* cntm,
                                                                 const uint32_t* loffm, const FoEntry* seg,
                                                                 uint32_t nblk, uint32_t nb, uint32_t cap,
                                                                 uint32_t* ctl, uint64_t* nout, uint32_t* zero_hist) {
  constexpr int T = 64 * FO_SORT_WAVES;
  FoClock clk(2);
  if (zero_hist)  // wc_fo_bin is done with it: leave it zeroed for the next wc_fo_hist
    for (uint32_t i = blockIdx.x * T + threadIdx.x; i < FO_LOGBINS; i += gridDim.x * T) zero_hist[i] = 0;
  __shared__ FoWaveLds W[FO_SORT_WAVES];
  __shared__ uint32_t big_m[FO_SORT_WAVES], big_off[FO_SORT_WAVES];
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint32_t b = blockIdx.x * FO_SORT_WAVES + wave;
  const uint32_t* cc = cntm + (size_t)b * nblk;
  const uint32_t* ll = loffm + (size_t)b * nblk;
  FoWaveLds& L = W[wave];
  // this bin's output offset (sum of the blocks' local offsets) and size
  uint32_t off = 0, m = 0;
  for (uint32_t k = lane; k < nblk; k += 64) {
    off += ll[k];
    m += cc[k];
  }
  for (int o = 32; o > 0; o >>= 1) {
    off += __shfl_xor(off, o);
    m += __shfl_xor(m, o);
  }
  if (b == nb - 1 && lane == 0 && nout) *nout = (uint64_t)off + m;
  clk.at(1);
  const auto emit = [&](uint32_t at, uint32_t ei) {
    const FoEntry x = seg[ei];
    const uint64_t j = (uint64_t)off + at;
    if (!bounds_ok(dst.bnd, BND_FO_SORT, j)) return;
    dst.k0[j] = x.k0;
    dst.k1[j] = x.k1;
    dst.cnt[j] = x.cnt;
    dst.first[j] = x.first;
    dst.soff[j] = x.soff;
    dst.slen[j] = x.slen;
  };
  // gather (first, entry index) of every block's run: lane l owns the blocks
  // [G l, G l + G) — all their counts / offsets loaded at once, one wave scan,
  // then all the entry loads (two dependent memory steps, whatever nblk)
  const auto gather = [&](const uint32_t* gcc, const uint32_t* gll, uint64_t* keys, uint32_t* idx) {
    const uint32_t G = (nblk + 63) / 64, k0 = lane * G;
    uint32_t tot = 0;
    for (uint32_t g = 0; g < G; ++g)
      if (k0 + g < nblk) tot += gcc[k0 + g];
    uint32_t at = wave_incl_scan(tot) - tot;
    for (uint32_t g = 0; g < G; ++g) {
      const uint32_t k = k0 + g;
      if (k >= nblk) break;
      const uint32_t c = gcc[k];
      if (!c) continue;
      const size_t e0 = (size_t)k * FO_ROWS + gll[k];
      for (uint32_t i = 0; i < c; ++i) {
        keys[at + i] = seg[e0 + i].first;
        idx[at + i] = (uint32_t)(e0 + i);
      }
      at += c;
    }
  };
  const bool over = m > cap;  // a pathological value distribution: the caller redoes the order
  if (over && lane == 0) ctl[0] = 1;
  const bool big = !over && m > (uint32_t)FO_WAVE_CAP;
  if (m != 0 && !big && !over) {
    gather(cc, ll, L.ka, L.va);
    for (uint32_t i = lane; i < FO_WSUB; i += 64) L.sub[i] = 0;
    wave_sync();
    clk.at(2);
    uint64_t lo = ~0ull, hi = 0;
    for (uint32_t t = lane; t < m; t += 64) {
      lo = min(lo, L.ka[t]);
      hi = max(hi, L.ka[t]);
    }
    for (int o = 32; o > 0; o >>= 1) {
      lo = min(lo, (uint64_t)__shfl_xor((unsigned long long)lo, o));
      hi = max(hi, (uint64_t)__shfl_xor((unsigned long long)hi, o));
    }
    const float scale = (float)FO_WSUB / ((float)(hi - lo) + 1.0f);
    const auto sub_of = [&](uint64_t key) { return min((uint32_t)((float)(key - lo) * scale), (uint32_t)FO_WSUB - 1); };
    for (uint32_t t = lane; t < m; t += 64) atomicAdd(&L.sub[sub_of(L.ka[t])], 1u);
    wave_sync();
    {  // exclusive scan of the sub-bucket counts, FO_WSUB / 64 per lane
      constexpr int PL = FO_WSUB / 64;
      uint32_t c[PL], own = 0;
#pragma unroll
      for (int i = 0; i < PL; ++i) own += c[i] = L.sub[lane * PL + i];
      uint32_t run = wave_incl_scan(own) - own;
#pragma unroll
      for (int i = 0; i < PL; ++i) {
        L.sub[lane * PL + i] = run;
        run += c[i];
      }
    }
    wave_sync();
    for (uint32_t t = lane; t < m; t += 64) {
      const uint64_t key = L.ka[t];
      const uint32_t d = atomicAdd(&L.sub[sub_of(key)], 1u);  // sub[s] advances to its end
      L.kb[d] = key;
      L.vb[d] = L.va[t];
    }
    wave_sync();
    for (uint32_t t = lane; t < m; t += 64) {
      const uint64_t key = L.kb[t];
      const uint32_t sb = sub_of(key);
      const uint32_t end = L.sub[sb], start = sb ? L.sub[sb - 1] : 0u;
      uint32_t rank = start;
      for (uint32_t j = start; j < end; ++j) rank += L.kb[j] < key ? 1u : 0u;
      emit(rank, L.vb[t]);
    }
    clk.at(3);
  }
  // bins above the wave capacity: the whole block, one at a time
  if (lane == 0) {
    big_m[wave] = big ? m : 0u;
    big_off[wave] = off;
  }
  __syncthreads();
  uint64_t* sk = reinterpret_cast<uint64_t*>(&W[0]);                                  // FO_BLOCK_CAP keys
  uint32_t* sv = reinterpret_cast<uint32_t*>(sk + FO_BLOCK_CAP);                      // + values
  static_assert(sizeof(W) >= (size_t)FO_BLOCK_CAP * 12, "block path fits the wave regions");
  for (int w = 0; w < FO_SORT_WAVES; ++w) {
    const uint32_t bm = big_m[w];
    if (bm == 0) continue;
    const uint32_t bb = blockIdx.x * FO_SORT_WAVES + w;
    const uint32_t* bcc = cntm + (size_t)bb * nblk;
    const uint32_t* bll = loffm + (size_t)bb * nblk;
    if (wave == 0) gather(bcc, bll, sk, sv);  // by one wave
    uint32_t P = 64;
    while (P < bm) P <<= 1;
    __syncthreads();
    for (uint32_t i = bm + tid; i < P; i += T) sk[i] = ~0ull;
    lds_bitonic<T, true>(sk, sv, P);
    const uint32_t boff = big_off[w];
    for (uint32_t i = tid; i < bm; i += T) {
      const FoEntry x = seg[sv[i]];
      const uint64_t j = (uint64_t)boff + i;
      if (!bounds_ok(dst.bnd, BND_FO_SORT, j)) continue;
      dst.k0[j] = x.k0;
      dst.k1[j] = x.k1;
      dst.cnt[j] = x.cnt;
      dst.first[j] = x.first;
      dst.soff[j] = x.soff;
      dst.slen[j] = x.slen;
    }
    __syncthreads();
  }
  clk.at(4);
}

// out.col[i] = in.col[perm[i]] for all six key-table columns (one launch).
__global__ void wc_gather_cols(const uint64_t* k0, const uint64_t* k1, const uint64_t* cnt, const uint64_t* first,
                               const uint64_t* soff, const uint32_t* slen, const uint32_t* perm, uint64_t* ok0,
                               uint64_t* ok1, uint64_t* ocnt, uint64_t* ofirst, uint64_t* osoff, uint32_t* oslen,
                               uint64_t n, const uint64_t* dn, Bounds bnd) {
  if (dn) n = *dn;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t j = perm[i];
    if (!bounds_ok(bnd, BND_GATHER_COLS, i) || !bounds_ok(bnd, BND_GATHER_COLS, j)) continue;
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

// ---- first-occurrence order above 400k keys: ranks from a bitmap of first offsets ----
// Distinct words have distinct first offsets, and two token starts are >= 2
// bytes apart (a delimiter between them), so first >> 1 indexes a bitmap
// without collisions: 1 GiB of text is a 64 MiB bitmap.  A key's output row is
// the number of set bits before its position — no comparison sort at all:
//   wc_bm_set     set each key's bit (an atomic OR; a bit already set = two
//                 keys at one position: the redo flag), add 1 to its 512-bit
//                 line's counter, and count the keys into the control word
//   wc_bm_count   per line its counter (4 bytes, not the 64-byte line: 4 MiB
//                 read at 1M lines instead of 64 MiB), the lines' exclusive
//                 prefix inside each 256-line block + block totals
//   wc_bm_scan    one block: the block totals' exclusive scan and the key
//                 count; fewer set bits than keys (two keys at one position)
//                 or a key beyond the bound raises the overflow word, and the
//                 caller redoes the order with the radix sort; the control word
//                 is zeroed again for the next call
//   wc_bm_place   row = block prefix + line prefix + popcount of the line's
//                 bits below the key: the key's six columns go to that row as
//                 ONE 64-byte record (a whole memory sector: six scattered
//                 8-byte column stores measured 160 us at 1M keys, 6 partial
//                 lines each)
//   wc_bm_emit    records -> the six columns in row order (coalesced), and the
//                 row's bitmap word and line counter zeroed: every set bit has
//                 a row, so the bitmap is left all-zero for the next call
// The radix path it replaces (4 digit passes + histogram + table keys +
// gather) measured 200 us at 1M keys (profiles/r4_session3.md §7).
constexpr uint32_t BM_LINE_BITS = 512;
constexpr uint32_t BM_BLOCK_LINES = 256;
constexpr uint64_t BM_BLOCK_WORDS = BM_BLOCK_LINES * BM_LINE_BITS / 64;
constexpr uint64_t BM_BLOCK_CNT_WORDS = BM_BLOCK_LINES / 2;  // the block's u32 line counters, in u64 words
// control word: redo (a key beyond the bound, or two keys at one position) | the key count
constexpr uint64_t BM_RANGE = 1ull << 63;
struct alignas(64) BmRow {
  uint64_t k0, k1, cnt, first, soff;
  uint32_t slen, pad0;
  uint64_t pad1, pad2;
};
static_assert(sizeof(BmRow) == 64, "one memory sector per row");

// A row of the source: false for an empty table slot (or an empty bucket,
// whose slots are undefined).
__device__ inline bool bm_row(const OrderSrc& src, uint64_t i, uint64_t& first) {
  if (src.table) {
    if (src.t.occupancy[i >> TAB_SLOTS_LOG2] == 0 || src.t.k1[i] == K1_EMPTY) return false;
    first = src.t.first[i];
  } else {
    first = src.first[i];
  }
  return true;
}
__device__ inline uint64_t bm_rows(const OrderSrc& src, uint64_t rows) {
  return !src.table && src.dn ? *src.dn : rows;
}

__global__ void __launch_bounds__(256) wc_bm_set(OrderSrc src, uint64_t rows, unsigned long long* bm, uint32_t* lc,
                                                 uint32_t shift, uint64_t pos_end, unsigned long long* ctl) {
  __shared__ uint32_t wn[4];
  rows = bm_rows(src, rows);
  uint32_t n = 0;
  bool range = false;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < rows; i += (uint64_t)gridDim.x * 256) {
    uint64_t f;
    if (!bm_row(src, i, f)) continue;
    const uint64_t p = f >> shift;
    ++n;
    if (p >= pos_end) {  // beyond the bound the caller gave (place skips it too)
      range = true;
      continue;
    }
    // random 8-byte writes dominate: 1M keys over a 64 MiB bitmap measured 68 us
    // with 64- or 32-bit, agent- or workgroup-scope ORs, with or without the
    // return, and 52 us as plain (inexact) stores (tools/bm_probe.py)
    const unsigned long long m = 1ull << (p & 63);
    if (__hip_atomic_fetch_or(&bm[p >> 6], m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & m) range = true;
    __hip_atomic_fetch_add(&lc[p / BM_LINE_BITS], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  for (int o = 32; o > 0; o >>= 1) n += __shfl_xor(n, o);
  range = __any(range);
  if ((threadIdx.x & 63) == 0) wn[threadIdx.x >> 6] = n;
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint64_t t = (uint64_t)wn[0] + wn[1] + wn[2] + wn[3];
    if (t) atomicAdd(ctl, (unsigned long long)t);
  }
  if (range && (threadIdx.x & 63) == 0) atomicOr(ctl, (unsigned long long)BM_RANGE);
}

__global__ void __launch_bounds__(BM_BLOCK_LINES) wc_bm_count(const uint32_t* lc, uint64_t lines, uint32_t* linepre,
                                                              uint32_t* blocktot) {
  __shared__ uint32_t wsum[BM_BLOCK_LINES / 64];
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint64_t line = (uint64_t)blockIdx.x * BM_BLOCK_LINES + tid;
  const uint32_t c = line < lines ? lc[line] : 0u;
  uint32_t incl = c;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(incl, o);
    if ((int)lane >= o) incl += y;
  }
  if (lane == 63) wsum[wave] = incl;
  __syncthreads();
  uint32_t before = 0, tot = 0;
#pragma unroll
  for (uint32_t w = 0; w < BM_BLOCK_LINES / 64; ++w) {
    before += w < wave ? wsum[w] : 0;
    tot += wsum[w];
  }
  if (line < lines) linepre[line] = before + incl - c;
  if (tid == 0) blocktot[blockIdx.x] = tot;
}

// One block: blockpre = exclusive scan of blocktot, *n = the total; the
// overflow word from the control word, which is zeroed for the next call.
__global__ void __launch_bounds__(1024) wc_bm_scan(const uint32_t* blocktot, uint32_t nblk, uint64_t* blockpre,
                                                   uint64_t* n, unsigned long long* ctl, uint32_t* ovf) {
  constexpr int PER = 8;
  __shared__ uint64_t wsum[16];
  __shared__ uint64_t carry;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid == 0) carry = 0;
  __syncthreads();
  for (uint32_t c = 0; c < nblk; c += 1024 * PER) {
    uint32_t v[PER];
    uint64_t s = 0;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const uint32_t b = c + tid * PER + j;
      v[j] = b < nblk ? blocktot[b] : 0;
      s += v[j];
    }
    uint64_t incl = s;
    for (int o = 1; o < 64; o <<= 1) {
      const uint64_t y = __shfl_up(incl, o);
      if ((int)lane >= o) incl += y;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    uint64_t before = carry;
    for (uint32_t w = 0; w < wave; ++w) before += wsum[w];
    uint64_t o = before + incl - s;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const uint32_t b = c + tid * PER + j;
      if (b < nblk) blockpre[b] = o;
      o += v[j];
    }
    __syncthreads();
    if (tid == 0) {
      uint64_t t = 0;
      for (int w = 0; w < 16; ++w) t += wsum[w];
      carry += t;
    }
    __syncthreads();
  }
  if (tid == 0) {
    const unsigned long long k = *ctl;
    *n = carry;
    *ovf = (k & BM_RANGE) || (k & ~BM_RANGE) != carry ? 1u : 0u;
    *ctl = 0;
  }
}

__global__ void __launch_bounds__(256) wc_bm_place(OrderSrc src, uint64_t rows, const unsigned long long* bm,
                                                   uint32_t shift, uint64_t pos_end, const uint32_t* linepre,
                                                   const uint64_t* blockpre, BmRow* out, Bounds bnd) {
  rows = bm_rows(src, rows);
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < rows; i += (uint64_t)gridDim.x * 256) {
    uint64_t f;
    // a table slot's words loaded at once, not behind its occupancy / k1 tests
    // (one round trip; i < rows stays inside the table, stale slots go unused)
    uint64_t tk0 = 0, tk1 = 0, tcnt = 0;
    if (src.table) {
      const uint32_t occ = src.t.occupancy[i >> TAB_SLOTS_LOG2];
      tk1 = src.t.k1[i];
      f = src.t.first[i];
      tk0 = src.t.k0[i];
      tcnt = src.t.cnt[i];
      if (occ == 0 || tk1 == K1_EMPTY) continue;
    } else {
      f = src.first[i];
    }
    const uint64_t p = f >> shift;
    if (p >= pos_end) continue;
    const uint64_t line = p / BM_LINE_BITS;
    const ulonglong2* q = reinterpret_cast<const ulonglong2*>(bm + line * (BM_LINE_BITS / 64));
    const uint32_t wi = (uint32_t)(p >> 6) & 7, b = (uint32_t)p & 63;
    const unsigned long long below = (1ull << b) - 1;
    uint32_t r = 0;
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
      const ulonglong2 v = q[k];
      r += 2 * k < wi ? __popcll(v.x) : 2 * k == wi ? __popcll(v.x & below) : 0;
      r += 2 * k + 1 < wi ? __popcll(v.y) : 2 * k + 1 == wi ? __popcll(v.y & below) : 0;
    }
    const uint64_t o = blockpre[line / BM_BLOCK_LINES] + linepre[line] + r;
    if (!bounds_ok(bnd, BND_BM_PLACE, o)) continue;
    ulonglong2 w[4];
    if (src.table) {
      const bool h = key_is_hashed(tk1);
      w[0] = make_ulonglong2(tk0, tk1);
      w[1] = make_ulonglong2(tcnt, f);
      w[2] = make_ulonglong2(h ? src.t.sref_off[i] : 0, h ? src.t.sref_len[i] : 0);
    } else {
      w[0] = make_ulonglong2(src.k0[i], src.k1[i]);
      w[1] = make_ulonglong2(src.cnt[i], f);
      w[2] = make_ulonglong2(src.soff[i], src.slen[i]);
    }
    w[3] = make_ulonglong2(0, 0);
    ulonglong2* d = reinterpret_cast<ulonglong2*>(out + o);
#pragma unroll
    for (int k = 0; k < 4; ++k) d[k] = w[k];
  }
}

// With two keys at one position (the redo flag) the line counters count more
// keys than set bits, so some rows below *n were never placed: their stale
// contents are cleared only inside the bitmap's bounds (ranks of distinct
// positions stay distinct, so every set bit still has its own placed row).
__global__ void __launch_bounds__(256) wc_bm_emit(const BmRow* in, const uint64_t* n, OrderDst dst,
                                                  unsigned long long* bm, uint32_t* lc, uint32_t shift,
                                                  uint64_t pos_end) {
  uint64_t rows = *n;
  if (rows > dst.bnd.cap) {  // more set bits than rows: record once, emit what fits
    if (blockIdx.x == 0 && threadIdx.x == 0) (void)bounds_ok(dst.bnd, BND_BM_EMIT, rows - 1);
    rows = dst.bnd.cap;
  }
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < rows; i += (uint64_t)gridDim.x * 256) {
    const ulonglong2* q = reinterpret_cast<const ulonglong2*>(in + i);
    const ulonglong2 a = q[0], b = q[1], c = q[2];
    dst.k0[i] = a.x;
    dst.k1[i] = a.y;
    dst.cnt[i] = b.x;
    dst.first[i] = b.y;
    dst.soff[i] = c.x;
    dst.slen[i] = (uint32_t)c.y;
    const uint64_t p = b.y >> shift;
    if (p < pos_end) {
      bm[p >> 6] = 0;
      lc[p / BM_LINE_BITS] = 0;
    }
  }
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


static uint32_t fo_blocks(const OrderSrc& src, uint64_t bound) {
  return src.table ? (1u << src.t.log2_buckets) * (TAB_SLOTS / dev::FO_ROWS)
                   : (uint32_t)std::max<uint64_t>(1, (bound + dev::FO_ROWS - 1) / dev::FO_ROWS);
}
void first_order_stamps(unsigned long long* d) {
  WC_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(dev::fo_stamps), &d, sizeof d));
}

static uint32_t fo_nbins(uint64_t bound) { return bound <= dev::FO_SMALL_KEYS ? dev::FO_BINS_SMALL : dev::FO_BINS; }

size_t first_order_ws_bytes(const OrderSrc& src, uint64_t bound) {
  const size_t nblk = fo_blocks(src, bound);
  return 64 * 1024 + 2 * (size_t)fo_nbins(bound) * nblk * 4 + 256 + nblk * dev::FO_ROWS * sizeof(dev::FoEntry);
}

uint32_t* first_order(const OrderSrc& src, const OrderDst& dst, uint64_t bound, uint32_t key_bits, void* ws,
                      uint64_t* nout, hipStream_t s, const uint32_t* key_hist, uint32_t key_hist_m,
                      uint32_t* hist_ws, uint32_t hist_ready_m) {
  WC_CHECK(bound <= FO_MAX_KEYS, "first_order: key bound above FO_MAX_KEYS (use the radix sort)");
  const uint32_t nblk = fo_blocks(src, bound), M = fo_mbits(key_bits), nb = fo_nbins(bound);
  uint8_t* p = static_cast<uint8_t*>(ws);
  uint16_t* map = reinterpret_cast<uint16_t*>(p);  // FO_LOGBINS entries (32 KiB)
  uint32_t* ctl = reinterpret_cast<uint32_t*>(p + 48 * 1024);
  uint32_t* cntm = reinterpret_cast<uint32_t*>(p + 64 * 1024);
  uint32_t* loffm = cntm + (size_t)nb * nblk;
  const size_t mat = 2 * (size_t)nb * nblk * 4;
  dev::FoEntry* seg = reinterpret_cast<dev::FoEntry*>(p + 64 * 1024 + (mat + 255) / 256 * 256);
  const uint32_t* phist = key_hist && key_hist_m == M ? key_hist : nullptr;
  uint32_t* zero_hist = nullptr;
  if (!phist && hist_ws && hist_ready_m == M) {  // a producer of the keys already histogrammed them into hist_ws
    phist = zero_hist = hist_ws;
  } else if (!phist && hist_ws) {  // the exact histogram of the keys, many blocks (not the one-block sample)
    const uint32_t hb = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(256, (bound + dev::FO_HIST_ROWS - 1) / dev::FO_HIST_ROWS));
    hipLaunchKernelGGL(dev::wc_fo_hist, dim3(hb), dim3(1024), 0, s, src, M, hist_ws);
    phist = zero_hist = hist_ws;
  }
  if (!phist) hipLaunchKernelGGL(dev::wc_fo_split, dim3(1), dim3(1024), 0, s, src, M, nb, map, ctl);
  hipLaunchKernelGGL(dev::wc_fo_bin, dim3(nblk), dim3(1024), 0, s, src, M, nb, map, phist, cntm, loffm, seg, ctl);
  uint32_t cap = dev::FO_BLOCK_CAP;
  if (const char* e = std::getenv("WC_FO_CAP")) cap = std::min<uint32_t>(cap, (uint32_t)std::atoi(e));  // tests
  hipLaunchKernelGGL(dev::wc_fo_sort, dim3(nb / dev::FO_SORT_WAVES), dim3(64 * dev::FO_SORT_WAVES), 0, s, dst, cntm,
                     loffm, seg, nblk, nb, cap, ctl, nout, zero_hist);
  return ctl;
}

void launch_gather_cols(const uint64_t* k0, const uint64_t* k1, const uint64_t* cnt, const uint64_t* first,
                        const uint64_t* soff, const uint32_t* slen, const uint32_t* perm, uint64_t* ok0, uint64_t* ok1,
                        uint64_t* ocnt, uint64_t* ofirst, uint64_t* osoff, uint32_t* oslen, uint64_t n, hipStream_t s,
                        const uint64_t* dn, const Bounds& bnd) {
  if (n)
    hipLaunchKernelGGL(dev::wc_gather_cols, dev::grid_for(n), dim3(256), 0, s, k0, k1, cnt, first, soff, slen, perm,
                       ok0, ok1, ocnt, ofirst, osoff, oslen, n, dn, bnd);
}

void launch_iota_u32(uint32_t* v, uint64_t n, hipStream_t s) {
  if (n) hipLaunchKernelGGL(dev::wc_iota_u32, dev::grid_for(n), dim3(256), 0, s, v, n);
}
void launch_fill_u64(uint64_t* p, uint64_t v, uint64_t n, hipStream_t s) {
  if (n) hipLaunchKernelGGL(dev::wc_fill_u64, dev::grid_for(n), dim3(256), 0, s, p, v, n);
}

static uint64_t bm_lines(uint64_t key_end, uint32_t shift) {
  return ((key_end >> shift) + dev::BM_LINE_BITS) / dev::BM_LINE_BITS;  // positions [0, (key_end >> shift) + 1)
}
static uint64_t bm_blocks(uint64_t key_end, uint32_t shift) {
  return (bm_lines(key_end, shift) + dev::BM_BLOCK_LINES - 1) / dev::BM_BLOCK_LINES;
}
// + 8 words: the control word (key count | range flag) after the bitmap
// bitmap | line counters | 8 control words
size_t bitmap_order_words(uint64_t key_end, uint32_t shift) {
  return bm_blocks(key_end, shift) * (dev::BM_BLOCK_WORDS + dev::BM_BLOCK_CNT_WORDS) + 8;
}
uint32_t* bitmap_order_linecnt(unsigned long long* bm, uint64_t key_end, uint32_t shift) {
  return reinterpret_cast<uint32_t*>(bm + bm_blocks(key_end, shift) * dev::BM_BLOCK_WORDS);
}
size_t bitmap_order_ws_bytes(uint64_t bound, uint64_t key_end, uint32_t shift) {
  return 256 + (bm_lines(key_end, shift) * 4 + 255) / 256 * 256 + bm_blocks(key_end, shift) * 12 + 512 +
         std::max<uint64_t>(bound, 1) * sizeof(dev::BmRow) + 64;
}

unsigned long long* bitmap_order_ctl(unsigned long long* bm, uint64_t key_end, uint32_t shift) {
  return bm + bm_blocks(key_end, shift) * (dev::BM_BLOCK_WORDS + dev::BM_BLOCK_CNT_WORDS);
}

uint32_t* bitmap_order(const OrderSrc& src, const OrderDst& dst, uint64_t bound, uint64_t key_end, uint32_t shift,
                       unsigned long long* bm, void* ws, uint64_t* nout, hipStream_t s, bool bits_set) {
  const uint64_t lines = bm_lines(key_end, shift), blocks = bm_blocks(key_end, shift);
  WC_CHECK(blocks < (1ull << 31), "bitmap_order: key bound too large");
  uint8_t* p = static_cast<uint8_t*>(ws);
  uint32_t* ovf = reinterpret_cast<uint32_t*>(p);
  uint64_t* n = nout ? nout : reinterpret_cast<uint64_t*>(p + 64);
  uint32_t* linepre = reinterpret_cast<uint32_t*>(p + 256);
  uint8_t* q = p + 256 + (lines * 4 + 255) / 256 * 256;
  uint64_t* blockpre = reinterpret_cast<uint64_t*>(q);
  q += (blocks * 8 + 255) / 256 * 256;
  uint32_t* blocktot = reinterpret_cast<uint32_t*>(q);
  q += (blocks * 4 + 255) / 256 * 256;
  dev::BmRow* rows_buf = reinterpret_cast<dev::BmRow*>((reinterpret_cast<uintptr_t>(q) + 63) & ~uintptr_t(63));
  unsigned long long* ctl = bitmap_order_ctl(bm, key_end, shift);
  uint32_t* lc = bitmap_order_linecnt(bm, key_end, shift);
  const uint64_t pos_end = (key_end >> shift) + 1;
  const uint64_t rows = src.table ? ((uint64_t)1 << src.t.log2_buckets) * TAB_SLOTS : bound;
  const dim3 g((unsigned)std::max<uint64_t>(1, std::min<uint64_t>(4096, (rows + 255) / 256)));
  if (!bits_set) hipLaunchKernelGGL(dev::wc_bm_set, g, dim3(256), 0, s, src, rows, bm, lc, shift, pos_end, ctl);
  hipLaunchKernelGGL(dev::wc_bm_count, dim3((unsigned)blocks), dim3(dev::BM_BLOCK_LINES), 0, s, lc, lines, linepre,
                     blocktot);
  hipLaunchKernelGGL(dev::wc_bm_scan, dim3(1), dim3(1024), 0, s, blocktot, (uint32_t)blocks, blockpre, n, ctl, ovf);
  hipLaunchKernelGGL(dev::wc_bm_place, g, dim3(256), 0, s, src, rows, bm, shift, pos_end, linepre, blockpre, rows_buf,
                     dst.bnd);
  const dim3 ge((unsigned)std::max<uint64_t>(1, std::min<uint64_t>(4096, (bound + 255) / 256)));
  hipLaunchKernelGGL(dev::wc_bm_emit, ge, dim3(256), 0, s, rows_buf, n, dst, bm, lc, shift, pos_end);
  return ovf;
}
}  // namespace wc
