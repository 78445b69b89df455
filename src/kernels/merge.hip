// merge.hip — device kernels of the cross-GPU merge protocols.
//
// Shuffle merge (default): every key goes to its owner rank (high bits of the
// placement hash) — owner partition + pack (wc_owner_count / wc_owner_scatter),
// RCCL all-to-all, owner-side merge in a global open-addressing table whose
// slots are claimed by the row id of the first inserter (wc_mrow_insert: keys are
// read from the immutable received rows, so no key publication race), owner
// compaction (wc_mrow_compact), and rank-0 conversion to key columns
// (wc_mrow_to_cols).
//
// Dense merge (merge_mode 1) runs the same owner partition / exchange / merge
// to build the dictionary, then numbers each owner's keys (wc_row_ids), returns
// the ids to the senders, and scatters local counts into dense vectors by id
// (wc_scatter_ids) for the reduce-scatter.
#include <algorithm>

#include "../common/hip_util.hpp"
#include "kernels.hpp"
#include "keys.hpp"
#include "lds_table.hpp"

namespace wc {
namespace dev {

inline dim3 mgrid(uint64_t n) {
  uint64_t g = (n + 255) / 256;
  return dim3((unsigned)(g < 1 ? 1 : (g > 4096 ? 4096 : g)));
}

// Byte equality of two LONG-word payloads, 8 bytes per compare (unaligned
// loads), the tail in one masked compare of the bytes that remain.
__device__ __forceinline__ bool mem_equal(const uint8_t* x, const uint8_t* y, uint64_t len) {
  uint64_t c = 0;
  for (; c + 8 <= len; c += 8) {
    uint64_t u, v;
    __builtin_memcpy(&u, x + c, 8);
    __builtin_memcpy(&v, y + c, 8);
    if (u != v) return false;
  }
  if (c == len) return true;
  uint64_t u = 0, v = 0;
  for (uint64_t i = c; i < len; ++i) {
    u |= (uint64_t)x[i] << (8 * (i - c));
    v |= (uint64_t)y[i] << (8 * (i - c));
  }
  return u == v;
}

constexpr int OWN_MAX = 64;       // ranks supported by the shuffle merge
constexpr int OWN_ROWS_PER_BLOCK = 1024;


// Wave-aggregated LDS counter adds: lanes with owner `o` (OWN_MAX = none) add 1
// to ctr[2 o] and `bytes` to ctr[2 o + 1] — two LDS atomics per distinct owner
// in the wave (<= W), not two per lane (a W = 1 or 2 merge would serialise 64
// lanes on one address).  Returns this lane's rank among the row adds to its
// counter; `boff` = its offset among the byte adds.
__device__ __forceinline__ unsigned long long wave_owner_add(unsigned long long* ctr, uint32_t o, uint32_t bytes,
                                                             unsigned long long& boff) {
  const int lane = (int)__lane_id();
  const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  uint64_t pending = __ballot(o != (uint32_t)OWN_MAX);
  const bool any_bytes = __ballot(bytes != 0) != 0;
  unsigned long long mine = 0;
  boff = 0;
  while (pending) {
    const int leader = __ffsll((unsigned long long)pending) - 1;
    const uint32_t po = (uint32_t)__shfl((int)o, leader);
    const bool in = o == po;
    const uint64_t m = __ballot(in);
    uint32_t incl = 0, total = 0;  // inclusive wave scan of this owner's byte counts
    if (any_bytes) {
      incl = in ? bytes : 0u;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)incl, d);
        if (lane >= d) incl += y;
      }
      total = (uint32_t)__shfl((int)incl, 63);
    }
    unsigned long long b = 0, bb = 0;
    if (lane == leader) {
      b = atomicAdd(&ctr[2 * po], (unsigned long long)__popcll(m));
      if (total) bb = atomicAdd(&ctr[2 * po + 1], (unsigned long long)total);
    }
    b = __shfl(b, leader);
    bb = __shfl(bb, leader);
    if (in) {
      mine = b + (unsigned long long)__popcll(m & lt);
      boff = bb + incl - bytes;
    }
    pending &= ~m;
  }
  return mine;
}

// counts[2o] += rows owned by o, counts[2o+1] += their long-word bytes (each
// word rounded up to 8 bytes: payloads stay 8-byte aligned, copied and compared
// a word at a time); rows [0, n) or [0, *dn) (device-side count, n the bound);
// pass_flags (nullable): counts[2W + 1] |= 1 if the pass needs a re-run (shuffle
// region / table overflow), |= 2 if the key arena overflowed (every
// rank then fails the job together instead of one rank throwing alone).
__global__ void __launch_bounds__(256) wc_owner_count(const uint64_t* k0, const uint64_t* k1, const uint32_t* slen,
                                                      uint64_t n, const uint64_t* dn, const uint32_t* pass_flags,
                                                      uint32_t W, unsigned long long* counts, uint32_t count_bias) {
  __shared__ unsigned long long h[2 * OWN_MAX];
  for (uint32_t i = threadIdx.x; i < 2 * W; i += blockDim.x) h[i] = 0;
  if (dn) n = *dn;
  // the row count counted here, next to the owner counts: every rank checks
  // every rank's count against its owner-count sum from the gathered matrix
  // (count_bias: fault injection, WC_MERGE_FAULT_COUNT).  Both come from the
  // same rows [0, n), so this guards the owner counting and the gathered
  // matrix only — it cannot see a compaction that wrote fewer rows than the
  // occupancy promised (WC_CHECK_TABLE and the finalize's bounds guard do)
  if (blockIdx.x == 0 && threadIdx.x == 0) counts[2 * W + 2] = n + count_bias;
  if (pass_flags && blockIdx.x == 0 && threadIdx.x == 0) {
    const uint32_t rerun = pass_flags[FLAG_REGION_OVF] | pass_flags[FLAG_TABLE_OVF];
    const unsigned long long f = (rerun ? 1ull : 0ull) | (pass_flags[FLAG_ARENA_OVF] ? 2ull : 0ull);
    if (f) atomicOr(&counts[2 * W + 1], f);
  }
  __syncthreads();
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i0 = blockIdx.x * (uint64_t)blockDim.x; i0 < n; i0 += stride) {  // whole waves call the wave op
    const uint64_t i = i0 + threadIdx.x;
    uint32_t o = OWN_MAX, nb = 0;
    if (i < n) {
      o = owner_of(place_hash(k0[i], k1[i]), W);
      if (key_is_hashed(k1[i])) nb = (slen[i] + 7u) & ~7u;
    }
    unsigned long long bo;
    (void)wave_owner_add(h, o, nb, bo);
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < 2 * W; i += blockDim.x)
    if (h[i]) atomicAdd(&counts[i], h[i]);
}

// Pack rows (and long-word bytes) contiguously by owner.  Each block reserves
// one range per owner (one global atomic per owner per block), then places its
// rows with LDS atomics.  counts = wc_owner_count output; cursor zeroed (distinct
// words: blocks add to the cursor while others read the counts).  A long word
// is copied in 8-byte words: its arena copy is 8-byte aligned and rounded up
// (reduce.hip settle_new_long), and its payload slot is rounded the same way.
// Planned mode (reg_rows > 0, dist/merge.cpp merge_cols_planned): owner o's
// rows go to the fixed region [o reg_rows, (o + 1) reg_rows) and its bytes to
// [o reg_bytes, ...), counts unused; a row past its region (rows or bytes) is
// dropped and sets bit 2 of *ovf (the job redoes the merge with the exact plan).  Rows
// [0, n) or [0, *dn) with n the bound.
__global__ void __launch_bounds__(256) wc_owner_scatter(const uint64_t* k0, const uint64_t* k1, const uint64_t* cnt,
                                                        const uint64_t* first, const uint64_t* soff,
                                                        const uint32_t* slen, const uint8_t* arena, uint64_t n,
                                                        const uint64_t* dn, uint32_t W,
                                                        const unsigned long long* counts, unsigned long long* cursor,
                                                        MRow* rows, uint8_t* bytes, uint32_t* send_pos,
                                                        uint64_t reg_rows, uint64_t reg_bytes, uint32_t* ovf,
                                                        const uint32_t* pass_flags, const uint32_t* occ,
                                                        unsigned long long* nvalid, MergeSelf self) {
  __shared__ unsigned long long base[2 * OWN_MAX], h[2 * OWN_MAX];
  __shared__ uint32_t nv;
  constexpr int PER = OWN_ROWS_PER_BLOCK / 256;
  const uint64_t r0 = (uint64_t)blockIdx.x * OWN_ROWS_PER_BLOCK;
  if (pass_flags && blockIdx.x == 0 && threadIdx.x == 0) {  // planned: this rank's pass flags into its flag word
    const uint32_t rerun = pass_flags[FLAG_REGION_OVF] | pass_flags[FLAG_TABLE_OVF];
    const uint32_t f = (rerun ? 1u : 0u) | (pass_flags[FLAG_ARENA_OVF] ? 2u : 0u);
    if (f) atomicOr(ovf, f);
  }
  if (self.base && blockIdx.x == 0) {  // planned: the fixed-region words (no host copies in the zeroing launch)
    for (uint32_t p = threadIdx.x; p <= W; p += blockDim.x) {
      self.base[p] = p * reg_rows;
      self.base[W + 1 + p] = p * reg_bytes;
      self.seg[p] = p * reg_rows;
    }
    if (threadIdx.x == 0) self.quad[2] = self.max_end;
  }
  if (dn) n = *dn;
  if (r0 >= n) return;
  const bool fixed = reg_rows != 0;
  for (uint32_t i = threadIdx.x; i < 2 * W; i += blockDim.x) h[i] = 0;
  if (threadIdx.x == 0) nv = 0;
  __syncthreads();
  // a table source: one occupancy word per 4096-slot bucket (a block's 1024 rows share it)
  const bool live = !occ || occ[r0 >> TAB_SLOTS_LOG2] != 0;
  uint32_t own[PER], mine = 0;
  unsigned long long lr[PER], lb[PER];
  // every row's key, count and first offset loaded at once (one round trip,
  // not gated on the occupancy word or on k1; an empty bucket's slots hold
  // stale values that are never used)
  uint64_t rk0[PER], rk1[PER], rc[PER], rf[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const uint64_t i = min(r0 + threadIdx.x + (uint64_t)j * 256, n - 1);
    rk0[j] = k0[i];
    rk1[j] = k1[i];
    rc[j] = cnt[i];
    rf[j] = first[i];
  }
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const uint64_t i = r0 + threadIdx.x + (uint64_t)j * 256;
    own[j] = OWN_MAX;
    uint32_t nb = 0;
    if (i < n) {
      if (live && (!occ || rk1[j] != K1_EMPTY)) {
        own[j] = owner_of(place_hash(rk0[j], rk1[j]), W);
        if (key_is_hashed(rk1[j])) nb = (slen[i] + 7u) & ~7u;
        ++mine;
      } else if (send_pos) {
        send_pos[i] = 0xFFFFFFFFu;  // an empty slot: no id comes back for it
      }
    }
    lr[j] = wave_owner_add(h, own[j], nb, lb[j]);
  }
  if (nvalid) {
    for (int o = 32; o > 0; o >>= 1) mine += __shfl_xor(mine, o);
    if ((threadIdx.x & 63) == 0 && mine) atomicAdd(&nv, mine);
  }
  __syncthreads();
  if (nvalid && threadIdx.x == 0 && nv) atomicAdd(nvalid, (unsigned long long)nv);
  if (threadIdx.x == 0) {
    unsigned long long br = 0, bb = 0;  // exclusive prefix of the global per-owner totals (or the regions)
    for (uint32_t o = 0; o < W; ++o) {
      if (fixed) {
        br = o * reg_rows;
        bb = o * reg_bytes;
      }
      base[2 * o] = br + (h[2 * o] ? atomicAdd(&cursor[2 * o], h[2 * o]) : 0);
      base[2 * o + 1] = bb + (h[2 * o + 1] ? atomicAdd(&cursor[2 * o + 1], h[2 * o + 1]) : 0);
      if (!fixed) {
        br += counts[2 * o];
        bb += counts[2 * o + 1];
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    if (own[j] == OWN_MAX) continue;
    const uint64_t i = r0 + threadIdx.x + (uint64_t)j * 256;
    const uint32_t o = own[j];
    if (fixed) {  // the row and its bytes must fit the owner's regions
      const uint64_t rp = base[2 * o] + lr[j] - o * reg_rows;
      const uint64_t bp = base[2 * o + 1] + lb[j] - o * reg_bytes;
      const uint64_t nb = key_is_hashed(rk1[j]) ? ((slen[i] + 7u) & ~7u) : 0u;
      if (rp >= reg_rows || bp + nb > reg_bytes) {
        atomicOr(ovf, 4u);  // wc_merge_check's capacity bit
        if (send_pos) send_pos[i] = 0xFFFFFFFFu;
        continue;
      }
    }
    MRow r;
    r.k0 = rk0[j];
    r.k1 = rk1[j];
    r.cnt = rc[j];
    r.first = rf[j];
    r.aoff = 0;
    r.alen = 0;
    const bool mine = o == self.rank;  // planned: straight into this rank's receive regions
    if (key_is_hashed(r.k1)) {
      const unsigned long long bpos = base[2 * o + 1] + lb[j];
      const uint64_t* src = reinterpret_cast<const uint64_t*>(arena + soff[i]);
      uint64_t* dst = reinterpret_cast<uint64_t*>((mine ? self.bytes : bytes) + bpos);
      for (uint32_t c = 0; c < (slen[i] + 7u) / 8u; ++c) dst[c] = src[c];
      unsigned long long bb = fixed ? o * reg_bytes : 0;  // offset inside owner o's byte payload
      for (uint32_t q = 0; !fixed && q < o; ++q) bb += counts[2 * q + 1];
      r.aoff = (uint32_t)(bpos - bb);
      r.alen = slen[i];
    }
    (mine ? self.rows : rows)[base[2 * o] + lr[j]] = r;
    if (send_pos) send_pos[i] = (uint32_t)(base[2 * o] + lr[j]);
  }
}

// Source rank of received row r (rbase: exclusive prefix of rows per source).
__device__ __forceinline__ uint32_t source_of(const uint64_t* rbase, uint32_t W, uint64_t r) {
  uint32_t src = 0;
  while (src + 1 < W && rbase[src + 1] <= r) ++src;
  return src;
}

// Owner-side merge: a slot belongs to the first row that CAS-es its id in;
// later rows of the same key compare against that row (immutable input) and add
// their counts with device-scope atomics.  The claiming row's own count and
// first offset are folded in by wc_mrow_compact (which reads that row anyway):
// a key seen once costs one atomic, not three — device-scope atomics resolve
// past the per-XCD L2s and bound this kernel.  LONG keys (hashed) also compare the
// word bytes of the two rows, so colliding words take different slots.  T is a
// power of two >= 2 R.
__global__ void __launch_bounds__(256) wc_mrow_insert(const MRow* rows, uint64_t R, const uint8_t* bytes,
                                                      const uint64_t* rbase, const uint64_t* bbase, uint32_t W,
                                                      uint32_t* state, unsigned long long* cnt,
                                                      unsigned long long* first, uint64_t T, uint32_t* row_slot) {
  for (uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; r < R; r += (uint64_t)gridDim.x * blockDim.x) {
    const MRow me = rows[r];
    if (me.k1 == K1_EMPTY) {  // padding of a planned exchange's fixed region
      if (row_slot) row_slot[r] = 0xFFFFFFFFu;
      continue;
    }
    const bool hashed = key_is_hashed(me.k1);
    const uint8_t* mb = hashed ? bytes + bbase[source_of(rbase, W, r)] + me.aoff : nullptr;
    uint64_t slot = place_hash(me.k0, me.k1) & (T - 1);
    bool claimed = false;
    // bounded: a planned merge sizes T from the learned merged-row cap, so a
    // job with more distinct keys than T can fill it; the compaction then
    // counts > cap merged rows and every rank redoes the merge exactly
    for (uint64_t probes = 0;; ++probes) {
      if (probes >= T) {
        slot = ~0ull;
        break;
      }
      // CAS first: most probes find their slot empty, and a load before the CAS
      // would add a round trip to every claim
      const uint32_t s = atomicCAS(&state[slot], 0u, (uint32_t)r + 1u);
      if (s == 0) {
        claimed = true;
        break;
      }
      const MRow& o = rows[s - 1];
      if (o.k0 == me.k0 && o.k1 == me.k1 &&
          (!hashed || (o.alen == me.alen && mem_equal(bytes + bbase[source_of(rbase, W, s - 1)] + o.aoff, mb, me.alen))))
        break;  // same word
      slot = (slot + 1) & (T - 1);
    }
    if (slot == ~0ull) {  // table full (see above): the row is dropped, the merge redone
      if (row_slot) row_slot[r] = 0xFFFFFFFFu;
      continue;
    }
    if (!claimed) {
      atomicAdd(&cnt[slot], (unsigned long long)me.cnt);
      atomicMin(&first[slot], (unsigned long long)me.first);
    }
    if (row_slot) row_slot[r] = (uint32_t)slot;
  }
}

// Occupied slots -> merged rows; aoff becomes absolute in the received byte
// buffer (rbase/bbase: exclusive prefixes of rows / bytes received per source).
// count = the claiming row's + the later rows' sum, first = min of both.
constexpr int MCOMPACT_PER = 4;  // slots per thread (256-thread blocks: 1024 slots per block)
__global__ void __launch_bounds__(256) wc_mrow_compact(const MRow* rows, const uint32_t* state,
                                                       const unsigned long long* cnt,
                                                       const unsigned long long* first, uint64_t T,
                                                       const uint64_t* rbase, const uint64_t* bbase, uint32_t W,
                                                       MRow* out, unsigned long long* out_n, uint32_t* slot_id,
                                                       uint64_t out_cap) {
  __shared__ unsigned long long blk;
  __shared__ uint32_t bcount;
  const int lane = (int)__lane_id();
  const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  const uint64_t s0 = (uint64_t)blockIdx.x * 256 * MCOMPACT_PER;
  if (threadIdx.x == 0) bcount = 0;
  __syncthreads();
  uint32_t local[MCOMPACT_PER];
#pragma unroll
  for (int j = 0; j < MCOMPACT_PER; ++j) {  // wave-aggregated ranks: one LDS atomic per wave and j
    const uint64_t sl = s0 + threadIdx.x + (uint64_t)j * 256;
    const bool occ = sl < T && state[sl] != 0u;
    const uint64_t m = __ballot(occ);
    uint32_t b = 0;
    if (lane == 0 && m) b = atomicAdd(&bcount, (uint32_t)__popcll(m));
    b = (uint32_t)__shfl((int)b, 0);
    local[j] = occ ? b + (uint32_t)__popcll(m & lt) : 0xFFFFFFFFu;
  }
  __syncthreads();
  if (threadIdx.x == 0) blk = bcount ? atomicAdd(out_n, (unsigned long long)bcount) : 0;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < MCOMPACT_PER; ++j) {
    if (local[j] == 0xFFFFFFFFu) continue;
    const uint64_t sl = s0 + threadIdx.x + (uint64_t)j * 256;
    const uint64_t r = state[sl] - 1u;
    const uint32_t src = source_of(rbase, W, r);
    MRow m = rows[r];
    m.cnt += cnt[sl];
    const unsigned long long f = first[sl];
    if (f < m.first) m.first = f;
    if (m.alen) m.aoff = (uint32_t)(bbase[src] + m.aoff);
    if (blk + local[j] < out_cap) out[blk + local[j]] = m;  // past it: counted in out_n (the caller's overflow check)
    if (slot_id) slot_id[sl] = (uint32_t)(blk + local[j]);
  }
}

// Planned merge (dist/merge.cpp merge_cols_planned), owner side: the insert
// and the compaction in one launch.  A slot belongs to the first row that
// CAS-es its id in (as wc_mrow_insert); the claiming rows of a block take
// their merged-row indices with one device atomic, write their key and
// long-word reference there, and publish the index in slot_idx.  Every row —
// claimer or a later row of the same key, which waits for the published index
// — adds its count and its inverted first offset (atomicMax of ~first) to the
// merged row with device atomics: the caller zeroed both words, so no order is
// needed between a claimer's stores and another row's adds, and no fence.
// A waiting row's claimer published before its own wave could wait (claim,
// publish, then wait, in that order per wave), so the waits cannot cycle.
// Indices past `cap` are counted in *out_n (the merge is redone), not written.
__global__ void __launch_bounds__(256) wc_mrow_insert_emit(const MRow* rows, uint64_t R, const uint8_t* bytes,
                                                           const uint64_t* rbase, const uint64_t* bbase, uint32_t W,
                                                           uint32_t* state, uint32_t* slot_idx, uint64_t T, MRow* out,
                                                           unsigned long long* out_n, uint64_t cap, uint32_t* ids,
                                                           uint32_t* ids_self, uint32_t self, uint64_t reg) {
  __shared__ uint32_t bcount;
  __shared__ unsigned long long bbase_idx;
  const int lane = (int)__lane_id();
  const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t r0 = blockIdx.x * (uint64_t)blockDim.x; r0 < R; r0 += stride) {  // whole blocks iterate together
    const uint64_t r = r0 + threadIdx.x;
    if (threadIdx.x == 0) bcount = 0;
    MRow me{};
    bool live = false;
    if (r < R) {
      me = rows[r];
      live = me.k1 != K1_EMPTY;  // else padding of a fixed region
    }
    uint64_t slot = ~0ull;
    bool claimed = false;
    uint32_t src = 0;
    if (live) {
      const bool hashed = key_is_hashed(me.k1);
      src = source_of(rbase, W, r);
      const uint8_t* mb = hashed ? bytes + bbase[src] + me.aoff : nullptr;
      slot = place_hash(me.k0, me.k1) & (T - 1);
      for (uint64_t probes = 0;; ++probes) {
        if (probes >= T) {  // table full: the row is dropped, the count past cap redoes the merge
          slot = ~0ull;
          break;
        }
        const uint32_t s = atomicCAS(&state[slot], 0u, (uint32_t)r + 1u);
        if (s == 0) {
          claimed = true;
          break;
        }
        const MRow& o = rows[s - 1];
        if (o.k0 == me.k0 && o.k1 == me.k1 &&
            (!hashed || (o.alen == me.alen && mem_equal(bytes + bbase[source_of(rbase, W, s - 1)] + o.aoff, mb, me.alen))))
          break;  // same word
        slot = (slot + 1) & (T - 1);
      }
    }
    __syncthreads();  // bcount reset seen
    const uint64_t cm = __ballot(claimed);
    uint32_t wb = 0;
    if (lane == 0 && cm) wb = atomicAdd(&bcount, (uint32_t)__popcll(cm));
    wb = (uint32_t)__shfl((int)wb, 0);
    __syncthreads();
    if (threadIdx.x == 0) bbase_idx = bcount ? atomicAdd(out_n, (unsigned long long)bcount) : 0;
    __syncthreads();
    uint64_t idx = ~0ull;
    if (claimed) {
      idx = bbase_idx + wb + (uint64_t)__popcll(cm & lt);
      if (idx < cap) {
        MRow* o = out + idx;
        o->k0 = me.k0;
        o->k1 = me.k1;
        o->aoff = me.alen ? (uint32_t)(bbase[src] + me.aoff) : 0u;
        o->alen = me.alen;
      }
      __hip_atomic_store(&slot_idx[slot], (uint32_t)idx + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // every claim of the block published before any of its rows waits: as an
    // if / else the compiler may run the waiting lanes of a wave first, with the
    // claiming lanes of the same wave (a region boundary: two sources) masked off
    __syncthreads();
    if (!claimed && slot != ~0ull) {  // a later row of a claimed key: wait for its index
      uint32_t v;
      while ((v = __hip_atomic_load(&slot_idx[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == 0u)
        __builtin_amdgcn_s_sleep(1);
      idx = v - 1u;
    }
    if (idx < cap) {
      atomicAdd(reinterpret_cast<unsigned long long*>(&out[idx].cnt), (unsigned long long)me.cnt);
      atomicMax(reinterpret_cast<unsigned long long*>(&out[idx].first), (unsigned long long)~me.first);
    }
    if (ids && r < R) {
      uint32_t* d = ids_self && r / reg == self ? ids_self : ids;
      d[r] = idx == ~0ull ? 0xFFFFFFFFu : (uint32_t)idx;
    }
    // no wave claims in the next round before every wave of this one is done
    // waiting: a claim made behind a waiting wave's barrier could be the one it waits for
    __syncthreads();
  }
}

// Dense merge: global id of received row r = this owner's id base + the compact
// index of the slot the row merged into.
// id base = the merged rows of the owners before this one, from the all-gathered
// (rows, bytes) pairs `owns` (no host round trip).
// Padding rows (row_slot all ones, planned exchange) get no id.
__global__ void wc_row_ids(const uint32_t* row_slot, const uint32_t* slot_id, uint64_t R,
                           const unsigned long long* owns, uint32_t rank, uint32_t* ids, uint32_t* ids_self,
                           uint32_t self, uint64_t reg) {
  uint64_t id_base = 0;
  for (uint32_t p = 0; p < rank; ++p) id_base += owns[2 * p];
  for (uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; r < R; r += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t sl = row_slot[r];
    // this rank's own region (planned): straight to the returned-id buffer
    uint32_t* d = ids_self && r / reg == self ? ids_self : ids;
    d[r] = sl == 0xFFFFFFFFu ? 0xFFFFFFFFu : (uint32_t)(id_base + slot_id[sl]);
  }
}

// Dense merge: local key i (sent as row send_pos[i], whose owner-local index
// came back in ids_back) stores its count and first offset at its global id =
// the owner's base (merged rows of the owners before it, from the all-gathered
// (rows, bytes) pairs `owns`) + the index; the owner of send row j is the
// segment of the send layout (`seg`: W + 1 row starts) holding j.  Ids of one
// rank's keys are distinct, so plain stores.
// Planned exchange (pad > 0): ids are padded (owner o's keys at [o pad,
// o pad + its count)), so the base of owner o is o pad; rows [0, n) or
// [0, *dn) with n the bound.
__global__ void __launch_bounds__(256) wc_scatter_ids(const uint32_t* send_pos, const uint32_t* ids_back,
                                                      const uint64_t* seg, const unsigned long long* owns, uint32_t W,
                                                      const uint64_t* cnt, const uint64_t* first, uint64_t n,
                                                      const uint64_t* dn, uint64_t pad, uint64_t* dcnt,
                                                      uint64_t* dfirst) {
  __shared__ uint64_t lseg[MERGE_MAX_RANKS + 1], lbase[MERGE_MAX_RANKS];
  if (dn) n = *dn;
  if (threadIdx.x == 0) {
    uint64_t b = 0;
    for (uint32_t o = 0; o < W; ++o) {
      lbase[o] = pad ? o * pad : b;
      if (!pad) b += owns[2 * o];
    }
  }
  for (uint32_t o = threadIdx.x; o <= W; o += blockDim.x) lseg[o] = seg[o];
  __syncthreads();
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t j = send_pos[i];
    if (j == 0xFFFFFFFFu) continue;  // a row dropped from an overflowing planned region
    if (pad && ids_back[j] >= pad) continue;  // past the padded id range: the job redoes the merge
    uint32_t lo = 0, hi = W - 1;  // the last owner whose segment starts at or before j
    while (lo < hi) {
      const uint32_t mid = (lo + hi + 1) >> 1;
      if (lseg[mid] <= j) lo = mid;
      else hi = mid - 1;
    }
    const uint64_t g = lbase[lo] + ids_back[j];
    dcnt[g] = cnt[i];
    dfirst[g] = first[i];
  }
}

// Gathered merged rows (grouped by owner) -> key columns; sref_off is made
// absolute in the gathered byte buffer.  cnt / first may be null (the dense
// merge takes them from its reduced vectors).
__global__ void wc_mrow_to_cols(const MRow* rows, uint64_t n, const uint64_t* dn, const uint64_t* rbase,
                                const uint64_t* bbase, uint32_t W, uint64_t* k0, uint64_t* k1, uint64_t* cnt,
                                uint64_t* first, uint64_t* soff, uint32_t* slen) {
  if (dn) n = *dn;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t o = 0;
    while (o + 1 < W && rbase[o + 1] <= i) ++o;
    const MRow m = rows[i];
    k0[i] = m.k0;
    k1[i] = m.k1;
    if (cnt) cnt[i] = m.cnt;
    if (first) first[i] = m.first;
    soff[i] = m.alen ? bbase[o] + m.aoff : 0;
    slen[i] = m.alen;
  }
}

// Planned merge (dist/merge.cpp merge_cols_planned): the decision from every
// rank's all-gathered word quad (merged rows, flags, max first offset, -):
// flags bit 0 = a rank's last pass needs recovery, bit 1 = its key arena
// overflowed, bit 2 = rows or bytes past a fixed region (set by its scatter);
// bit 2 also for merged rows past reg_merged and for a first offset above the
// bound the host sized the order's key width from (max_end).  Every rank reads
// the same gathered words, so every rank decides the same.
__global__ void wc_merge_check(const unsigned long long* owns, uint32_t W, uint64_t reg_merged, uint64_t max_end,
                               uint32_t* flags) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  uint32_t f = 0;
  for (uint32_t o = 0; o < W; ++o) {
    const unsigned long long* v = owns + 4 * (size_t)o;
    f |= (uint32_t)(v[1] & 7u);
    if (v[0] > reg_merged || v[2] > max_end) f |= 4u;
  }
  if (f) atomicOr(flags, f);
}

// Planned merge, rank 0: the gathered merged rows sit in fixed regions of
// reg_merged rows per owner, owner o's first owns[4 o] rows valid (k1 != 0);
// they become dense key columns at the exclusive prefix of the owners' counts,
// the long-word references made absolute in the gathered byte buffer (owner o's
// payload at o * byte_stride); dense merge: counts / first offsets from the
// reduced padded vectors (id o * reg_merged + j), else from the rows (first
// offset inverted, as wc_mrow_insert_emit leaves it).
// *out_n = the key count.
// HIST: one 1024-thread block per CU, an LDS histogram per block flushed with
// one global add per nonzero bin (a device atomic per row measured 16 us at
// 100k rows, against 5 us without the histogram).
template <bool HIST>
__global__ void __launch_bounds__(HIST ? 1024 : 256) wc_mrow_regions_to_cols(const MRow* rows, uint32_t W, uint64_t reg_merged,
                                                              const unsigned long long* owns, uint64_t byte_stride,
                                                              const uint64_t* dcnt, const uint64_t* dfirst,
                                                              uint64_t* k0, uint64_t* k1, uint64_t* cnt,
                                                              uint64_t* first, uint64_t* soff, uint32_t* slen,
                                                              unsigned long long* out_n, uint32_t* check_flags,
                                                              uint64_t max_end, uint32_t* hist, uint32_t hist_m) {
  __shared__ uint64_t pre[MERGE_MAX_RANKS + 1];
  __shared__ uint32_t lh[HIST ? FO_LOGBINS : 1];
  if (HIST)
    for (uint32_t i = threadIdx.x; i < FO_LOGBINS; i += blockDim.x) lh[i] = 0;
  if (check_flags && blockIdx.x == 0 && threadIdx.x == 64) {  // wc_merge_check, in another wave of block 0
    uint32_t f = 0;
    for (uint32_t o = 0; o < W; ++o) {
      const unsigned long long* v = owns + 4 * (size_t)o;
      f |= (uint32_t)(v[1] & 7u);
      if (v[0] > reg_merged || v[2] > max_end) f |= 4u;
    }
    if (f) atomicOr(check_flags, f);
  }
  if (threadIdx.x == 0) {
    uint64_t b = 0;
    for (uint32_t o = 0; o < W; ++o) {
      pre[o] = b;
      b += min((uint64_t)owns[4 * o], reg_merged);
    }
    pre[W] = b;
    if (blockIdx.x == 0) *out_n = b;
  }
  __syncthreads();
  const uint64_t N = (uint64_t)W * reg_merged;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < N; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t o = (uint32_t)(i / reg_merged);
    const uint64_t j = i - (uint64_t)o * reg_merged;
    if (j >= pre[o + 1] - pre[o]) continue;
    const MRow m = rows[i];
    const uint64_t at = pre[o] + j;
    k0[at] = m.k0;
    k1[at] = m.k1;
    cnt[at] = dcnt ? dcnt[i] : m.cnt;
    const uint64_t f = dfirst ? dfirst[i] : ~m.first;  // stored inverted by wc_mrow_insert_emit
    first[at] = f;
    soff[at] = m.alen ? o * byte_stride + m.aoff : 0;
    slen[at] = m.alen;
    if (HIST) atomicAdd(&lh[fo_logbin(f, hist_m)], 1u);  // the order's exact key histogram (no wc_fo_hist launch)
  }
  if (HIST) {
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < FO_LOGBINS; i += blockDim.x)
      if (lh[i]) atomicAdd(&hist[i], lh[i]);
  }
}

}  // namespace dev

void launch_merge_check(const unsigned long long* owns, uint32_t W, uint64_t reg_merged, uint64_t max_end,
                        uint32_t* flags, hipStream_t s) {
  WC_CHECK(W >= 1 && W <= MERGE_MAX_RANKS, "merge_check: 1..64 ranks");
  hipLaunchKernelGGL(dev::wc_merge_check, dim3(1), dim3(64), 0, s, owns, W, reg_merged, max_end, flags);
}
void launch_mrow_regions_to_cols(const MRow* rows, uint32_t W, uint64_t reg_merged, const unsigned long long* owns,
                                 uint64_t byte_stride, const uint64_t* dcnt, const uint64_t* dfirst, uint64_t* k0,
                                 uint64_t* k1, uint64_t* cnt, uint64_t* first, uint64_t* soff, uint32_t* slen,
                                 unsigned long long* out_n, hipStream_t s, uint32_t* check_flags, uint64_t max_end,
                                 uint32_t* hist, uint32_t hist_m) {
  WC_CHECK(W >= 1 && W <= MERGE_MAX_RANKS, "regions_to_cols: 1..64 ranks");
  if (hist) {
    const uint64_t g = std::min<uint64_t>(256, ((uint64_t)W * reg_merged + 1023) / 1024);
    hipLaunchKernelGGL(dev::wc_mrow_regions_to_cols<true>, dim3((unsigned)std::max<uint64_t>(1, g)), dim3(1024), 0, s,
                       rows, W, reg_merged, owns, byte_stride, dcnt, dfirst, k0, k1, cnt, first, soff, slen, out_n,
                       check_flags, max_end, hist, hist_m);
  } else {
    hipLaunchKernelGGL(dev::wc_mrow_regions_to_cols<false>, dev::mgrid((uint64_t)W * reg_merged), dim3(256), 0, s,
                       rows, W, reg_merged, owns, byte_stride, dcnt, dfirst, k0, k1, cnt, first, soff, slen, out_n,
                       check_flags, max_end, hist, hist_m);
  }
}

void launch_owner_count(const uint64_t* k0, const uint64_t* k1, const uint32_t* slen, uint64_t n, const uint64_t* dn,
                        const uint32_t* pass_flags, uint32_t W, unsigned long long* counts, hipStream_t s,
                        uint32_t count_bias) {
  // with a device-side count the grid is sized for the bound (grid-stride inside)
  hipLaunchKernelGGL(dev::wc_owner_count, dev::mgrid(n ? n : 1), dim3(256), 0, s, k0, k1, slen, n, dn, pass_flags, W,
                     counts, count_bias);
}
void launch_owner_scatter(const uint64_t* k0, const uint64_t* k1, const uint64_t* cnt, const uint64_t* first,
                          const uint64_t* soff, const uint32_t* slen, const uint8_t* arena, uint64_t n, uint32_t W,
                          const unsigned long long* counts, unsigned long long* cursor, MRow* rows, uint8_t* bytes,
                          uint32_t* send_pos, hipStream_t s, const uint64_t* dn, uint64_t reg_rows, uint64_t reg_bytes,
                          uint32_t* ovf, const uint32_t* pass_flags, const uint32_t* occ, unsigned long long* nvalid,
                          const MergeSelf* self) {
  const MergeSelf me = self ? *self : MergeSelf{~0u, nullptr, nullptr, nullptr, nullptr, nullptr, 0};
  static_assert(TAB_SLOTS % dev::OWN_ROWS_PER_BLOCK == 0, "a scatter block stays inside one table bucket");
  const uint64_t blocks = (n + dev::OWN_ROWS_PER_BLOCK - 1) / dev::OWN_ROWS_PER_BLOCK;
  if (n)
    hipLaunchKernelGGL(dev::wc_owner_scatter, dim3((unsigned)blocks), dim3(256), 0, s, k0, k1, cnt, first, soff, slen,
                       arena, n, dn, W, counts, cursor, rows, bytes, send_pos, reg_rows, reg_bytes, ovf, pass_flags,
                       occ, nvalid, me);
}
void launch_mrow_insert(const MRow* rows, uint64_t R, const uint8_t* bytes, const uint64_t* rbase,
                        const uint64_t* bbase, uint32_t W, uint32_t* state, unsigned long long* cnt,
                        unsigned long long* first, uint64_t T, uint32_t* row_slot, hipStream_t s) {
  if (R)
    hipLaunchKernelGGL(dev::wc_mrow_insert, dev::mgrid(R), dim3(256), 0, s, rows, R, bytes, rbase, bbase, W, state, cnt,
                       first, T, row_slot);
}
void launch_mrow_compact(const MRow* rows, const uint32_t* state, const unsigned long long* cnt,
                         const unsigned long long* first, uint64_t T, const uint64_t* rbase, const uint64_t* bbase,
                         uint32_t W, MRow* out, unsigned long long* out_n, uint32_t* slot_id, hipStream_t s,
                         uint64_t out_cap) {
  const uint64_t blocks = (T + 256 * dev::MCOMPACT_PER - 1) / (256 * dev::MCOMPACT_PER);
  hipLaunchKernelGGL(dev::wc_mrow_compact, dim3((unsigned)blocks), dim3(256), 0, s, rows, state, cnt, first, T, rbase,
                     bbase, W, out, out_n, slot_id, out_cap);
}
void launch_mrow_insert_emit(const MRow* rows, uint64_t R, const uint8_t* bytes, const uint64_t* rbase,
                             const uint64_t* bbase, uint32_t W, uint32_t* state, uint32_t* slot_idx, uint64_t T,
                             MRow* out, unsigned long long* out_n, uint64_t cap, uint32_t* ids, uint32_t* ids_self,
                             uint32_t self, uint64_t reg, hipStream_t s) {
  WC_CHECK(R < 0xFFFFFFFFull && T <= 0xFFFFFFFFull && (T & (T - 1)) == 0, "insert_emit: 32-bit row ids, T a power of two");
  WC_CHECK(!ids_self || reg > 0, "insert_emit: a region size with ids_self");
  if (R)
    hipLaunchKernelGGL(dev::wc_mrow_insert_emit, dev::mgrid(R), dim3(256), 0, s, rows, R, bytes, rbase, bbase, W, state,
                       slot_idx, T, out, out_n, cap, ids, ids_self, self, reg);
}
void launch_mrow_to_cols(const MRow* rows, uint64_t n, const uint64_t* rbase, const uint64_t* bbase, uint32_t W,
                         uint64_t* k0, uint64_t* k1, uint64_t* cnt, uint64_t* first, uint64_t* soff, uint32_t* slen,
                         hipStream_t s, const uint64_t* dn) {
  if (n)
    hipLaunchKernelGGL(dev::wc_mrow_to_cols, dev::mgrid(n), dim3(256), 0, s, rows, n, dn, rbase, bbase, W, k0, k1, cnt,
                       first, soff, slen);
}

void launch_row_ids(const uint32_t* row_slot, const uint32_t* slot_id, uint64_t R, const unsigned long long* owns,
                    uint32_t rank, uint32_t* ids, hipStream_t s, uint32_t* ids_self, uint32_t self, uint64_t reg) {
  WC_CHECK(!ids_self || reg > 0, "row_ids: a region size with ids_self");
  if (R)
    hipLaunchKernelGGL(dev::wc_row_ids, dev::mgrid(R), dim3(256), 0, s, row_slot, slot_id, R, owns, rank, ids, ids_self,
                       self, reg);
}
void launch_scatter_ids(const uint32_t* send_pos, const uint32_t* ids_back, const uint64_t* seg,
                        const unsigned long long* owns, uint32_t W, const uint64_t* cnt, const uint64_t* first,
                        uint64_t n, uint64_t* dcnt, uint64_t* dfirst, hipStream_t s, const uint64_t* dn, uint64_t pad) {
  WC_CHECK(W >= 1 && W <= MERGE_MAX_RANKS, "scatter_ids: 1..64 ranks");
  if (n)
    hipLaunchKernelGGL(dev::wc_scatter_ids, dev::mgrid(n), dim3(256), 0, s, send_pos, ids_back, seg, owns, W, cnt,
                       first, n, dn, pad, dcnt, dfirst);
}
}  // namespace wc
