// map.hip — the MAP stage: hot-key sampling, hot-table build, and wc_map
// (tokenize -> key -> LDS hot table | shuffle record).
//
// Reference: mapKernel / mapper (/root/reference/main.cu:37-54, 109-117) copy
// one pre-split line's words per thread with <= 9 threads active; the host
// tokenizes (main.cu:181-206).  Here the GPU tokenizes and pre-aggregates in
// three launches per sampled chunk:
//
//  wc_hot_sample  every map block tokenizes HOT_SAMPLE units spread over its
//                 range, counts their words in an LDS table and writes them,
//                 split by table partition (GPP = 8 groups each), to its own
//                 stage cells;
//  wc_hot_merge   one block per partition sums the cells in LDS, keeps the
//                 partition's most frequent words as candidates and places
//                 them into ITS groups of the pass's table image
//                 (place_partition): a 2-choice table of 2-slot groups (4096
//                 slots of 64-bit signatures, a two-word word's side word in
//                 its group's second slot), both groups of a word in its
//                 partition;
//  wc_map         persistent, ONE 1024-thread block (16 waves) per CU over a
//                 contiguous range of 2 KiB text units.  The block copies
//                 the image into its LDS (every block flushes its slots with
//                 full keys, so exactness never rests on it).  Each wave grabs its
//                 next unit from an LDS cursor and prefetches it into registers (32 B per lane) while
//                 tokenizing the current one from its private LDS copy:
//                 SWAR delimiter masks -> token starts `~d & (d << 1 | c)` ->
//                 ballot-bit prefix sum -> a list of (position, length)
//                 entries -> per step two tokens per lane: exact inline key
//                 from two 8-byte windows (keys.hpp), 32-bit placement hash,
//                 both candidate groups read in ONE LDS round trip; a hit is
//                 two no-return LDS atomics (count, min first offset), a miss
//                 is a shuffle record (key, 1, offset) appended to the
//                 (block, bucket) sub-region of its reduce bucket.  The table
//                 is READ-ONLY while tokens stream: no claims, no refresh
//                 barriers, no divergent slow path.  A token belongs to the
//                 unit holding its first byte (lanes, units, chunks and GPU
//                 shards all use this rule).  The block ends by emitting every
//                 counted hot slot as one record.
//
// Signatures: a word of <= 7 bytes is its own 64-bit signature (bytes | len
// << 56, one compare) and takes one slot of a 2-slot group; 8..15-byte words
// use len << 56 | low 7 bytes of (k0 ^ tail) and take a WHOLE group: the
// signature in its first slot, k0 (the `side` word) in the second, so the
// token's one 16-byte probe read confirms it.  LONG words of 16..64 bytes are
// hot-table words too (0xFF << 56 | a key hash; side = the length | the
// candidate's index << 32): a hit needs the token's bytes to equal the
// candidate's 64-byte copy of the word, so exactness never rests on the hash;
// every other LONG token is a record whose bytes the reducer compares.  A
// side word never equals a short signature (a short signature's top byte is
// its length 1..7; two-word words whose k0 has a top byte < 8 are not placed).

#include <type_traits>

#include "common/hip_util.hpp"
#include "map_common.hpp"
#include "zero_list.hpp"

namespace wc {
namespace dev {

constexpr int UNIT = 64 * MAP_BPL;     // text bytes per wave unit (2 KiB)
constexpr int HALO = 64;               // bytes past the unit kept in LDS
// + one 24-byte window read past the halo, rounded to 16 bytes: every wave's
// buffer starts 16-byte aligned, so the unit commit's ds_write_b128 are aligned
// (2136-byte buffers put odd waves at 8 mod 16: SQ_LDS_UNALIGNED_STALL 3.0e7 / GiB)
constexpr int BUF = (UNIT + HALO + 24 + 15) / 16 * 16;
constexpr int MAP_DEF_CAP = 248;       // deferred LONG entries per wave and round (>= 128 + UNIT / 17)
constexpr int MAP_DEF_CAP_Q = 256;     // the same, queue layout (no LONG cursors in its LDS)
constexpr uint32_t NONE = 0xFFFFFFFFu;
constexpr int GS = HOT_GROUP_SLOTS;    // slots per group
constexpr int NG = HOT_GROUPS;         // groups
#ifndef WC_HOT_SAMPLE
#define WC_HOT_SAMPLE 4  // 8: +0.3-1 % at v100k but long30_v1m 388 -> 245 GB/s (profiles/r4_session3.md §13)
#endif
constexpr uint32_t HOT_SAMPLE = WC_HOT_SAMPLE;  // units sampled per map block
constexpr int SAMPLE_PROBES = 8;
// The table's groups come in HOT_PARTS partitions of GPP consecutive groups
// (a partition = the top bits of g1); a word's two groups lie in ONE partition
// (g2 = g1 ^ 1..GPP-1), and the partition's wc_hot_merge block, which holds
// all of that partition's sampled words, places them itself (place_partition).
static_assert((NG & (NG - 1)) == 0, "table geometry: 2^k groups");
constexpr uint32_t GPP = NG / HOT_PARTS;  // groups per partition
static_assert(GPP >= 2 && GPP <= 16 && (GPP & (GPP - 1)) == 0 && GPP * HOT_PARTS == NG,
              "table geometry: 2..16 groups per hot-word partition");
// The sampling table keeps 4096 slots whatever the map table holds.
constexpr int SAMPLE_SLOTS = 4096, SNG = SAMPLE_SLOTS / GS;
static_assert(UNIT <= 2048, "list entries hold 11-bit unit-relative positions");

// Profiling builds only (tools/variants.sh -DWC_MAP_ABLATE=N; results are NOT
// valid): 5 text stream + LDS commit only, 4 + delimiter masks and token
// starts, 6 + the token list, 7 + the steps' entry reads, 1 + key windows,
// 2 + keys and hashes, 3 + table probes and hit counts (misses dropped);
// 8 / 9: the partial short / general step of each round dropped.
#ifndef WC_MAP_ABLATE
#define WC_MAP_ABLATE 0
#endif

constexpr uint64_t LOW7 = 0x00FFFFFFFFFFFFFFull;
__device__ __forceinline__ bool two_word(uint64_t sig) { return (sig >> 56) >= 8; }

__device__ __forceinline__ void sig_key(uint64_t sig, uint64_t side, uint64_t& k0, uint64_t& k1) {
  const uint64_t top = sig >> 56;
  if (top < 8) {
    k0 = sig & LOW7;
    k1 = top;
  } else {
    k0 = side;
    k1 = top == 8 ? 8ull : (((sig ^ side) & LOW7) | (top << 56));
  }
}

// Inline key of a token of known length 1..15 from its windows w0 = bytes
// [p, p+8) and w1 = [p+8, p+16), and its table signature.
__device__ __forceinline__ void inline_key(uint64_t w0, uint64_t w1, uint32_t len, uint64_t& k0, uint64_t& k1,
                                           uint64_t& sig) {
  // k0: the first min(len, 8) bytes — a shift pair by 64 - 8 min(len, 8) in
  // [0, 56] (len 0 of an empty lane clamps to 1: no shift by 64)
  const uint32_t s0 = 64u - 8u * min(max(len, 1u), 8u);
  k0 = (w0 << s0) >> s0;
  const uint32_t tl = len > 8 ? len - 8 : 0u;
  const uint64_t t = w1 & ((1ull << (8 * tl)) - 1ull);
  const uint64_t lt = (uint64_t)len << 56;
  k1 = len <= 8 ? (uint64_t)len : (t | lt);
  sig = (len <= 7 ? k0 : ((t ^ k0) & LOW7)) | lt;
}

// inline_key for a token of 8 or more bytes (the map's other-class steps):
// k0 is the first window whole; len 8..15 -> exact key, longer -> garbage
// (LONG tokens are deferred, never keyed here).
__device__ __forceinline__ void inline_key_long8(uint64_t w0, uint64_t w1, uint32_t len, uint64_t& k0, uint64_t& k1,
                                                 uint64_t& sig) {
  k0 = w0;
  const uint64_t t = len > 8 ? w1 & (~0ull >> ((128u - 8u * len) & 63u)) : 0ull;  // the first len - 8 bytes
  const uint64_t lt = (uint64_t)len << 56;
  k1 = len == 8 ? 8ull : (t | lt);
  sig = ((t ^ k0) & LOW7) | lt;
}

// Slot i of group g.  4-slot groups: slots 0-1 of every group form the first
// half of the table, slots 2-3 the second, so each 16-byte probe read of a
// group half lands on bank quad (g mod 16) — all 16 quads — instead of only
// even / odd.  2-slot groups: one 16-byte read per group, slots 2g, 2g + 1.
__device__ __forceinline__ uint32_t slot_of(uint32_t g, uint32_t i) {
  if (GS == 2) return 2 * g + i;
  return (i < 2 ? 0u : MAP_SLOTS / 2) + 2 * g + (i & 1);
}

// The two candidate groups of a key (2-choice placement; g2 != g1: the xor
// term is odd; both in g1's partition: the xor term is < GPP).
__device__ __forceinline__ void hot_groups(uint32_t ph, uint32_t& g1, uint32_t& g2) {
  g1 = (ph >> 20) & (NG - 1);
  g2 = g1 ^ (((ph >> 8) & (GPP - 1)) | 1u);
}
__device__ __forceinline__ uint32_t hot_partition(uint32_t ph) { return ((ph >> 20) & (NG - 1)) / GPP; }
// The same as byte offsets of the groups in the signature image (16 * g):
// right shifts, ands and one bitop3 — all full-rate VALU on gfx950, where the
// left shifts / max / shift-or forms are half rate (profiles/r4_session3.md §2).
__device__ __forceinline__ void hot_group_offs(uint32_t ph, uint32_t& o1, uint32_t& o2) {
  o1 = (ph >> 16) & ((NG - 1) << 4);
  o2 = o1 ^ (((ph >> 4) & ((GPP - 1) << 4)) | 16u);
}

// 64-bit fingerprint of a sampled word (never 0): keys the global sample table.
__device__ __forceinline__ uint64_t sample_fp(uint64_t sig, uint64_t side) {
  return fmix64(sig ^ (side * 0x9E3779B97F4A7C15ull)) | 1ull;
}

// Hot LONG words (16..HOT_LONG_MAX bytes, hashed keys).  Their signature has
// top byte 0xFF — an inline signature's top byte is its length (<= 15), so the
// two never meet — and 56 bits of a hash of the key; placement and lookup
// both take the groups from the signature alone.  A signature match is only a
// candidate: the token's bytes are compared with the slot's 64-byte copy of
// the word (HotArgs::long_bytes), so colliding words never merge.
constexpr uint64_t LONG_SIG_TOP = 0xFFull << 56;
__device__ __forceinline__ bool is_long_sig(uint64_t sig) { return (sig >> 56) == 0xFF; }
__device__ __forceinline__ uint64_t long_signature(uint64_t k0, uint64_t k1) {
  return LONG_SIG_TOP | (fmix64(k0 ^ (k1 * 0x9E3779B97F4A7C15ull)) & LOW7);
}
__device__ __forceinline__ uint32_t long_group_hash(uint64_t sig) {
  return mix32((uint32_t)sig ^ (uint32_t)(sig >> 32));
}

// Key of a word of known length 16..64 at p of an LDS text buffer (readable
// to p + len + 12): k0 = first 8 bytes, the tail folded in 8-byte chunks
// (keys.hpp key_of).
__device__ __forceinline__ void key_long_len(const uint8_t* buf, uint32_t p, uint32_t len, uint64_t mask, uint64_t& k0,
                                             uint64_t& k1) {
  k0 = window8(buf, p);
  uint64_t h = FNV_OFFSET;
  for (uint32_t c = 8; c < len; c += 8) {
    uint64_t x = window8(buf, p + c);
    if (len - c < 8) x &= (1ull << (8 * (len - c))) - 1ull;
    h = tail_fold(h, x);
  }
  k1 = long_k1(len, h, mask);
}

// The same from a slot's zero-padded 64-byte line (global, 8-byte words).
__device__ __forceinline__ void key_long_line(const uint8_t* line, uint32_t len, uint64_t mask, uint64_t& k0,
                                              uint64_t& k1) {
  const uint64_t* w = reinterpret_cast<const uint64_t*>(line);
  k0 = w[0];
  uint64_t h = FNV_OFFSET;
  for (uint32_t c = 8; c < len; c += 8) h = tail_fold(h, w[c / 8]);  // padding bytes are zero
  k1 = long_k1(len, h, mask);
}

// The same with the whole 64-byte line loaded in one round trip (four 16-byte
// loads, then the compares): the top-down LONG layout's instance only — its
// extra registers spilled the main loop of the LONG-free one (-2.5 % at v100k,
// profiles/r3_session2.md §5), which keeps the loop above.
__device__ __forceinline__ bool long_line_equal_1rt(const uint8_t* buf, uint32_t p, const uint8_t* line, uint32_t len) {
  const uint4* l4 = reinterpret_cast<const uint4*>(line);
  const uint4 v0 = l4[0], v1 = l4[1], v2 = l4[2], v3 = l4[3];
  const uint64_t w[8] = {v0.x | (uint64_t)v0.y << 32, v0.z | (uint64_t)v0.w << 32, v1.x | (uint64_t)v1.y << 32,
                         v1.z | (uint64_t)v1.w << 32, v2.x | (uint64_t)v2.y << 32, v2.z | (uint64_t)v2.w << 32,
                         v3.x | (uint64_t)v3.y << 32, v3.z | (uint64_t)v3.w << 32};
  bool eq = true;
#pragma unroll
  for (uint32_t i = 0; i < 8; ++i) {
    const uint32_t c = 8 * i;
    if (c >= len) break;
    uint64_t x = window8(buf, p + c);
    if (len - c < 8) x &= (1ull << (8 * (len - c))) - 1ull;
    eq &= x == w[i];
  }
  return eq;
}

#ifndef WC_LONG_1RT
#define WC_LONG_1RT 1  // A/B
#endif

// Token bytes [p, p + len) of the LDS buffer == the slot's line?
__device__ __forceinline__ bool long_line_equal(const uint8_t* buf, uint32_t p, const uint8_t* line, uint32_t len) {
  const uint64_t* w = reinterpret_cast<const uint64_t*>(line);
  bool eq = true;
  for (uint32_t c = 0; c < len; c += 8) {
    uint64_t x = window8(buf, p + c);
    if (len - c < 8) x &= (1ull << (8 * (len - c))) - 1ull;
    eq &= x == w[c / 8];
  }
  return eq;
}

// Delimiter bits of 16 bytes.
__device__ __forceinline__ uint32_t delim_bits16(const uint4& v) {
  return delim_bits4(v.x) | (delim_bits4(v.y) << 4) | (delim_bits4(v.z) << 8) | (delim_bits4(v.w) << 12);
}

// Delimiter bits of the first 32 halo bytes (lanes 0 and 1 hold them in h16),
// wave-uniform.
__device__ __forceinline__ uint32_t halo_bits(const uint4& h16) {
  const uint32_t hb = __lane_id() < 2 ? delim_bits16(h16) : 0u;
  return (uint32_t)__builtin_amdgcn_readlane((int)hb, 0) | ((uint32_t)__builtin_amdgcn_readlane((int)hb, 1) << 16);
}

// Delimiter bits of the lane's 32 bytes (registers) and of the following 32
// (neighbour lane by a DPP wave shift; lane 63: the halo bits), and the lane's
// token starts.  Registers only: no LDS round trip.
__device__ __forceinline__ void unit_masks(const uint4& p0, const uint4& p1, uint32_t hbits, uint32_t pv,
                                           uint64_t u0, uint32_t pbase, uint64_t chunk_len, uint64_t& dm,
                                           uint32_t& starts) {
  const int lane = (int)__lane_id();
  const uint32_t mine = delim_bits16(p0) | (delim_bits16(p1) << 16);
  const uint32_t next = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)mine, 0x130, 0xF, 0xF, false);  // wave_shl:1
  const uint32_t prev = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)mine, 0x138, 0xF, 0xF, false);  // wave_shr:1
  dm = (uint64_t)mine | ((uint64_t)(lane == 63 ? hbits : next) << 32);
  const uint32_t carry = lane == 0 ? (is_delim(pv) ? 1u : 0u) : (prev >> 31);  // last byte of the lane below
  starts = ~mine & ((mine << 1) | carry);
  const uint64_t lane_base = u0 + pbase;
  if (lane_base >= chunk_len) starts = 0;
  else if (lane_base + MAP_BPL > chunk_len) starts &= (1u << (uint32_t)(chunk_len - lane_base)) - 1u;
}

// Unit range of map block `blk` (units of UNIT bytes).
__device__ __forceinline__ void unit_range(uint64_t chunk_len, uint32_t grid, uint32_t blk, uint64_t& ub,
                                           uint64_t& ue) {
  const uint64_t nunits = (chunk_len + UNIT - 1) / UNIT;
  const uint64_t per = (nunits + grid - 1) / grid;
  ub = min((uint64_t)blk * per, nunits);
  ue = min(ub + per, nunits);
}

// Diagnostic phase clock of the two per-job setup kernels (WC_MAP_STAMPS=1:
// hot_setup_stamps): [16 k + p] = the max over blocks of the 100 MHz wall time
// from the block's start to its phase p (k 0: wc_hot_sample, 1: wc_hot_merge).
__device__ unsigned long long* hot_stamps = nullptr;
struct HotClock {
  uint64_t t0;
  int k;
  __device__ HotClock(int kernel) : t0(hot_stamps ? __builtin_amdgcn_s_memrealtime() : 0), k(kernel) {}
  __device__ void at(int p) {
    if (hot_stamps && threadIdx.x == 0)
      atomicMax(&hot_stamps[16 * k + p], (unsigned long long)(__builtin_amdgcn_s_memrealtime() - t0));
  }
};

// ------------------------------------------------------------------ sampling
struct SampleLds {
  uint64_t fp[SAMPLE_SLOTS];  // 0 empty, else the word's fingerprint
  uint64_t sig[SAMPLE_SLOTS];
  uint64_t side[SAMPLE_SLOTS];
  uint32_t cnt[SAMPLE_SLOTS];
  uint32_t pn[HOT_PARTS];  // words of this block in each fingerprint partition
  alignas(16) uint8_t buf[MAP_WAVES][BUF];
};
static_assert(sizeof(SampleLds) <= 160 * 1024, "one sample block per CU");

// Each wave takes sampled units (stride over the block's range) and counts
// their words per lane in the block's LDS table; the block then writes its
// words, split by fingerprint partition, to its own stage cells with plain
// stores (a cell holds HOT_STAGE_CAP words; the rest of a crowded cell is
// dropped — the table is only an accelerator, exactness never depends on it).
// The round-2 form added every block's words into one global fingerprint table
// with device CAS + add: the Zipf head's slots took one atomic pair from each
// of the 256 blocks in turn, two thirds of a 35 us launch.
// SUBW waves share each sampled unit, each counting every SUBW-th word of
// every lane (a lane holds ~5 words of its 32 bytes and counts them one after
// another: one wave per unit took 8 us for that loop, with 12 of 16 waves idle).
constexpr int SUBW = MAP_WAVES / (int)HOT_SAMPLE;
static_assert(SUBW >= 1 && MAP_WAVES % (int)HOT_SAMPLE == 0, "sampling: whole waves per sampled unit");
__global__ void __launch_bounds__(MAP_THREADS) wc_hot_sample(MapArgs a, HotArgs h, ZeroList z) {
  __shared__ SampleLds L;
  HotClock clk(0);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint32_t sub = (uint32_t)wave % SUBW;
  uint64_t ub, ue;
  unit_range(a.chunk_len, gridDim.x, blockIdx.x, ub, ue);
  const uint64_t nu = ue - ub;
  const uint64_t ns = min<uint64_t>(nu, HOT_SAMPLE);
  uint8_t* buf = L.buf[wave];
  const uint32_t pbase = lane * MAP_BPL;
  // this wave's unit loaded first: its HBM latency overlaps the zeroing below
  const uint64_t i = (uint64_t)wave / SUBW;  // < HOT_SAMPLE: one unit per wave group
  const bool act = i < ns;
  const uint64_t u0 = act ? (ub + i * nu / ns) * UNIT : 0;
  uint4 p0 = make_uint4(0, 0, 0, 0), p1 = p0, h16 = make_uint4(0x20202020u, 0x20202020u, 0x20202020u, 0x20202020u);
  uint32_t pv = 0x20;
  if (act) {
    load32(a, u0 + pbase, p0, p1);
    if (lane < HALO / 16) h16 = load16(a, u0 + UNIT + lane * 16);
    pv = (u0 == 0 && a.prev_byte >= 0) ? (uint32_t)a.prev_byte : a.text[(int64_t)u0 - 1];
  }
  // the pass's zeroing (counters, table occupancy after a reset, ...): nothing
  // here or in wc_hot_merge touches those regions; the map and reduce that read
  // them run after both launches
  apply_zero_list(z, blockIdx.x * (uint64_t)MAP_THREADS + tid, (uint64_t)gridDim.x * MAP_THREADS, blockIdx.x == 0,
                  MAP_THREADS);
  for (int s = tid; s < SAMPLE_SLOTS; s += MAP_THREADS) {
    L.fp[s] = 0;
    L.cnt[s] = 0;
  }
  if (tid < HOT_PARTS) L.pn[tid] = 0;
  __syncthreads();
  clk.at(1);  // zero list + LDS init
  if (act) {
    reinterpret_cast<uint4*>(&buf[pbase])[0] = p0;
    reinterpret_cast<uint4*>(&buf[pbase])[1] = p1;
    if (lane < HALO / 16) *reinterpret_cast<uint4*>(&buf[UNIT + lane * 16]) = h16;
    wave_sync();
    uint64_t dm;
    uint32_t bits;
    unit_masks(p0, p1, halo_bits(h16), pv, u0, pbase, a.chunk_len, dm, bits);
    clk.at(4);  // diagnostic: wave 0's unit loaded and masked
    for (uint32_t k = 0; bits; ++k) {
      const uint32_t b = __ffs(bits) - 1;
      bits &= bits - 1;
      if (k % SUBW != sub) continue;  // another wave of the group counts this word
      const uint64_t rest = dm >> b;
      const uint32_t p = pbase + b;
      uint32_t len;
      if (rest) {
        len = (uint32_t)__ffsll((unsigned long long)rest) - 1;
      } else {  // the word runs past the lane's 64-byte window: its end in the unit's LDS copy + halo
        uint32_t q = pbase + 64;
        while (q < (uint32_t)(UNIT + HALO) && !is_delim(buf[q])) ++q;
        if (q >= (uint32_t)(UNIT + HALO)) continue;  // past the halo: not a candidate
        len = q - p;
      }
      if (len > HOT_LONG_MAX) continue;
      uint64_t k0, k1, sg, sd, f;
      uint32_t g;
      if (len <= KEY_INLINE_MAX) {
        uint64_t w0, w1;
        window16(buf, p, w0, w1);
        inline_key(w0, w1, len, k0, k1, sg);
        sd = two_word(sg) ? k0 : 0ull;
        const uint32_t ph = place_hash(k0, k1);
        // the fingerprint's top byte is the word's table partition: its merge block places it
        f = (sample_fp(sg, sd) & ~(0xFFull << 56)) | ((uint64_t)hot_partition(ph) << 56);
        g = (ph >> 20) & (SNG - 1);
      } else {  // LONG: side = this occurrence's chunk offset | length (the placement copies its bytes)
        key_long_len(buf, p, len, a.k1_mask, k0, k1);
        sg = long_signature(k0, k1);
        sd = (u0 + p) | ((uint64_t)len << 32);
        f = (sample_fp(sg, k0) & ~(0xFFull << 56)) | ((uint64_t)hot_partition(long_group_hash(sg)) << 56);
        g = (uint32_t)(f >> 20) & (SNG - 1);
      }
      for (int st = 0; st < SAMPLE_PROBES * GS; ++st) {
        const uint32_t s = GS * g + (st & (GS - 1));
        uint64_t cur = L.fp[s];
        if (cur == 0) {
          cur = atomicCAS(reinterpret_cast<unsigned long long*>(&L.fp[s]), 0ull, (unsigned long long)f);
          if (cur == 0) {  // claimed: the claimer stores the key (read after the block barrier)
            L.sig[s] = sg;
            L.side[s] = sd;
            cur = f;
          }
        }
        if (cur == f) {
          atomicAdd(&L.cnt[s], 1u);
          break;
        }
        if ((st & (GS - 1)) == GS - 1) g = (g + 1) & (SNG - 1);
      }
    }
    wave_sync();
    clk.at(5);  // diagnostic: wave 0's unit's words counted
  }
  __syncthreads();
  clk.at(2);  // the sampled units counted
  const size_t cell0 = (size_t)blockIdx.x * HOT_STAGE_CAP;  // + partition * maxb * HOT_STAGE_CAP
  for (int s = tid; s < SAMPLE_SLOTS; s += MAP_THREADS) {
    const uint32_t c = L.cnt[s];
    if (!c) continue;
    const uint64_t f = L.fp[s];
    const uint32_t part = (uint32_t)(f >> 56);  // the word's table partition (HOT_PARTS = 256)
    const uint32_t at = atomicAdd(&L.pn[part], 1u);
    if (at >= (uint32_t)HOT_STAGE_CAP) continue;
    HotEnt e;
    e.sig = L.sig[s];
    e.side = L.side[s];
    e.cnt = c;
    e.pad = 0;
    e.fp = f;
    h.stage[(size_t)part * h.maxb * HOT_STAGE_CAP + cell0 + at] = e;
  }
  __syncthreads();
  if (tid < HOT_PARTS) h.stage_n[(size_t)tid * h.maxb + blockIdx.x] = min(L.pn[tid], (uint32_t)HOT_STAGE_CAP);
  clk.at(3);  // stage cells written
}

// ------------------------------------------------------------------ selection
// Selection threshold over a count histogram of HOT_SEL_BINS bins in LDS:
// t = the smallest count >= 1 whose words (counted >= t) number <= limit (the
// last bin when even that holds more), cum = the words counted >= t
// (wave_count_threshold below).
constexpr int SEL_BINS = HOT_SEL_BINS;
// hist[bin] += 1 for every lane with `valid`, one LDS atomic per distinct bin
// of the wave: sampled counts crowd the low bins, and 64 lanes adding to one
// LDS word serialise on its bank (called by whole waves, lanes converged).
__device__ __forceinline__ void hist_add_wave(uint32_t* hist, uint32_t bin, bool valid) {
  uint64_t todo = __ballot(valid);
  while (todo) {
    const uint32_t b = (uint32_t)__builtin_amdgcn_readlane((int)bin, (int)(__ffsll((unsigned long long)todo) - 1));
    const uint64_t same = __ballot(valid && bin == b) & todo;
    if (__lane_id() == (uint32_t)(__ffsll((unsigned long long)todo) - 1)) atomicAdd(&hist[b], (uint32_t)__popcll(same));
    todo &= ~same;
  }
}
// ------------------------------------------------------------------ hot-table image
// The partition's words into its GPP groups (2 GPP slots) of the table image,
// by ONE wave of the partition's wc_hot_merge block: lane i holds candidate i;
// in count order (ties by index) each word takes a free slot of the emptier of
// its two groups (a two-slot word — two-word inline or LONG: signature + side
// word — an empty group), else moves a one-slot occupant of one of its groups
// to that occupant's other group when it has room and takes its slot, else
// stays out.  Uniform control flow, the group states in one scalar word (2
// bits per group: 0..2 occupants, 3 = a two-slot word), the slot owners one
// per lane.  Every map block copies the finished image (no per-block build);
// CPU model: tools/hot_place_sim.cpp mode 11 (SIM_REPAIR=1): 29.5 % of v100k
// tokens missed vs 31.2 % for the per-block placement it replaces
// (profiles/r6_session.md).
static_assert(HOT_PART_TOP <= 64 && 2 * GPP <= 64, "partition placement: one wave");
static_assert(HOT_PARTS == 256, "a sampled word's partition rides in its fingerprint's top byte");
__device__ void place_partition(const HotArgs& h, uint32_t part, uint32_t n, const uint32_t* oc, const uint64_t* osig,
                                const uint64_t* oside, uint32_t* ord) {
  const uint32_t lane = __lane_id();
  const bool have = lane < n;
  const uint32_t c = have ? oc[lane] : 0u;
  const uint64_t sg = have ? osig[lane] : 0ull, sd = have ? oside[lane] : 0ull;
  // local groups (0..GPP-1) and kind; a two-word word whose side word k0 has a
  // top byte < 8 could equal a short signature in the image: it stays out
  uint32_t g1 = 0, g2 = 0;
  const bool lng = is_long_sig(sg);
  bool ok = have && c != 0;
  if (ok) {
    if (lng) {
      hot_groups(long_group_hash(sg), g1, g2);
    } else {
      uint64_t k0, k1;
      sig_key(sg, sd, k0, k1);
      hot_groups(place_hash(k0, k1), g1, g2);
      if (two_word(sg) && (sd >> 59) == 0) ok = false;
    }
  }
  // one word per candidate for the scalar loop: a | b << 4 | two-slot << 8 |
  // placeable << 9 | its lane << 10
  const uint32_t info = (g1 & (GPP - 1)) | ((g2 & (GPP - 1)) << 4) | ((lng || two_word(sg)) ? 1u << 8 : 0u) |
                        (ok ? 1u << 9 : 0u) | (lane << 10);
  // rank in count order (ties: lower index first); lane r of `sinfo` then
  // holds the info of the rank-r candidate, so step r reads it with one readlane
  uint32_t rank = 0;
  for (uint32_t j = 0; j < n; ++j) {
    const uint32_t cj = (uint32_t)__builtin_amdgcn_readlane((int)c, (int)j);
    rank += (cj > c || (cj == c && j < lane)) ? 1u : 0u;
  }
  if (have) ord[rank] = info;
  wave_sync();
  const uint32_t sinfo = have ? ord[lane] : 0u;
  uint32_t st = 0;           // group states, 2 bits each (uniform)
  uint64_t alt = 0;          // slot s: its one-slot occupant's other group (4 bits each, uniform)
  uint32_t owner = 0xFFu;    // lane s < 2 GPP: the candidate (lane) in slot s (0xFF: empty)
  static_assert(2 * GPP * 4 <= 64, "placement: 4 bits of `alt` per slot");
  constexpr uint32_t FULL = (uint32_t)(0xAAAAAAAAull & ((1ull << (2 * GPP)) - 1ull));  // every group at 2 or 3: bit 1 of each field
  auto gst = [&](uint32_t g) { return (st >> (2 * g)) & 3u; };
  auto set_alt = [&](uint32_t s, uint32_t g) { alt = (alt & ~(0xFull << (4 * s))) | ((uint64_t)g << (4 * s)); };
  for (uint32_t r = 0; r < n; ++r) {
    if ((st & FULL) == FULL) break;  // no free slot left: no word (or move) can be placed any more
    const uint32_t ii = (uint32_t)__builtin_amdgcn_readlane((int)sinfo, (int)r);
    if (!(ii & (1u << 9))) continue;
    const uint32_t i = ii >> 10, ai = ii & 15u, bi = (ii >> 4) & 15u;
    const uint32_t sa = gst(ai), sb = gst(bi);
    if (ii & (1u << 8)) {  // an empty group, g1 first
      const uint32_t g = sa == 0 ? ai : (sb == 0 ? bi : 0xFFu);
      if (g == 0xFFu) continue;
      st |= 3u << (2 * g);
      if ((lane >> 1) == g) owner = i;
      continue;
    }
    const uint32_t fa = sa == 3 ? 0u : 2u - sa, fb = sb == 3 ? 0u : 2u - sb;
    if (fa | fb) {  // a free slot of the emptier group (slots fill first, then second)
      const uint32_t g = fb > fa ? bi : ai, s = 2 * g + gst(g);
      if (lane == s) owner = i;
      set_alt(s, g == ai ? bi : ai);
      st += 1u << (2 * g);
      continue;
    }
    // both full: move a one-slot occupant to its other group if that has room
    for (int k = 0; k < 4; ++k) {
      const uint32_t g = k < 2 ? ai : bi, s = 2 * g + (k & 1);
      if (gst(g) == 3) continue;
      const uint32_t ag = (uint32_t)(alt >> (4 * s)) & 15u, sag = gst(ag);
      if (sag >= 2) continue;
      const uint32_t o = (uint32_t)__builtin_amdgcn_readlane((int)owner, (int)s), s2 = 2 * ag + sag;
      if (lane == s2) owner = o;
      set_alt(s2, g);
      st += 1u << (2 * ag);
      if (lane == s) owner = i;
      set_alt(s, g == ai ? bi : ai);
      break;
    }
  }
  // the partition's 2 GPP image slots: a two-slot word's signature and side
  // word, one-slot words' signatures, 0 = empty
  const uint32_t o = owner & 63u;  // (the whole wave shuffles: every source lane active)
  const uint64_t osg = __shfl(sg, (int)o), osd = __shfl(sd, (int)o);
  if (lane < 2 * GPP) {
    const uint32_t g = lane >> 1;
    const uint64_t v = owner == 0xFFu ? 0ull : ((gst(g) == 3 && (lane & 1)) ? osd : osg);
    h.image[slot_of(part * GPP + g, lane & 1)] = v;
  }
}

// One block per fingerprint partition: every map block's stage cell of the
// partition is summed into an LDS table, then the HOT_PART_TOP most frequent
// words (ties at the threshold while room remains) become the partition's
// candidates.  Two dependent global steps in all (the cells' word counts, then
// every thread's cell entries at once): a loop that issued one load per
// iteration behind LDS atomics took 24 us.
constexpr int MERGE_SLOTS = 4096;
constexpr int MERGE_CELLS_PER_THREAD = 1024 / HOT_STAGE_CAP;  // cells covered by one pass of the block
static_assert(1024 % HOT_STAGE_CAP == 0, "merge: whole cells per pass");
struct HotMergeLds {
  uint64_t fp[MERGE_SLOTS];
  uint64_t sig[MERGE_SLOTS];
  uint64_t side[MERGE_SLOTS];
  uint32_t cnt[MERGE_SLOTS];
  alignas(16) uint32_t hist[SEL_BINS];
  uint32_t nout, nties;
  // the partition's candidates (place_partition): count, signature, side word
  uint32_t oc[HOT_PART_TOP];
  uint64_t osig[HOT_PART_TOP], oside[HOT_PART_TOP];
  uint32_t ord[HOT_PART_TOP];  // place_partition: candidates' info in count order
};
__device__ __forceinline__ void merge_insert(HotMergeLds& L, const HotEnt& e) {
  uint32_t s = (uint32_t)(e.fp >> 20) & (MERGE_SLOTS - 1);
  for (int k = 0; k < 64; ++k) {  // bounded: a word that finds no slot is dropped
    uint64_t cur = L.fp[s];
    if (cur == 0) {
      cur = atomicCAS(reinterpret_cast<unsigned long long*>(&L.fp[s]), 0ull, (unsigned long long)e.fp);
      if (cur == 0) {  // claimed: the claimer stores the key (read after the block barrier)
        L.sig[s] = e.sig;
        L.side[s] = e.side;
        cur = e.fp;
      }
    }
    if (cur == e.fp) {
      atomicAdd(&L.cnt[s], e.cnt);
      return;
    }
    s = (s + 1) & (MERGE_SLOTS - 1);
  }
}
// The threshold by one wave, no block barrier (every wave may call it and gets
// the same result): SEL_BINS = 4 bins per lane, a shuffle suffix scan.  (A
// block-wide scan over 4096 bins took 4 us of the merge's ~20.)
static_assert(SEL_BINS == 4 * 64, "wave threshold: 4 bins per lane");
__device__ __forceinline__ void wave_count_threshold(const uint32_t* hist, uint32_t limit, uint32_t& t_out,
                                                     uint32_t& cum_out) {
  const uint32_t lane = __lane_id();
  const uint4 b = reinterpret_cast<const uint4*>(hist)[lane];
  const uint32_t own = b.x + b.y + b.z + b.w;
  uint32_t x = own;  // words counted >= bin 4 lane (inclusive suffix over the lanes)
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_down(x, o);
    if (lane + o < 64) x += y;
  }
  // words counted >= each of this lane's bins; the first bin >= 1 at or under the limit
  const uint32_t s0 = x, s1 = s0 - b.x, s2 = s1 - b.y, s3 = s2 - b.z;
  const uint32_t i0 = 4 * lane;
  uint32_t t = SEL_BINS, cum = 0;
  if (s3 <= limit && i0 + 3 >= 1) { t = i0 + 3; cum = s3; }
  if (s2 <= limit && i0 + 2 >= 1) { t = i0 + 2; cum = s2; }
  if (s1 <= limit && i0 + 1 >= 1) { t = i0 + 1; cum = s1; }
  if (s0 <= limit && i0 >= 1) { t = i0; cum = s0; }
  // the smallest such bin over the wave (suffixes only shrink with the bin)
  const uint64_t has = __ballot(t < SEL_BINS);
  if (has) {
    const int l = __ffsll((unsigned long long)has) - 1;
    t_out = (uint32_t)__builtin_amdgcn_readlane((int)t, l);
    cum_out = (uint32_t)__builtin_amdgcn_readlane((int)cum, l);
  } else {  // even the last bin holds more than the limit
    t_out = SEL_BINS - 1;
    cum_out = (uint32_t)__builtin_amdgcn_readlane((int)s3, 63);
  }
}

__global__ void __launch_bounds__(1024) wc_hot_merge(HotArgs h) {
  __shared__ HotMergeLds L;
  HotClock clk(1);
  const int tid = threadIdx.x;
  const uint32_t part = blockIdx.x;
  for (int s = tid; s < MERGE_SLOTS; s += 1024) {
    L.fp[s] = 0;
    L.cnt[s] = 0;
  }
  for (int i = tid; i < SEL_BINS; i += 1024) L.hist[i] = 0;
  if (tid == 0) L.nout = L.nties = 0;
  __syncthreads();
  clk.at(1);  // LDS init
  const size_t row = (size_t)part * h.maxb;
  // thread tid: entry (tid % CAP) of the cells tid / CAP + k * CELLS (all loads of a thread issued together)
  const uint32_t e = tid % HOT_STAGE_CAP, c0 = tid / HOT_STAGE_CAP;
  for (uint32_t base = 0; base < h.nblk; base += 4 * MERGE_CELLS_PER_THREAD) {
    uint32_t n[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t blk = base + c0 + k * MERGE_CELLS_PER_THREAD;
      n[k] = blk < h.nblk ? h.stage_n[row + blk] : 0u;
    }
    HotEnt x[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t blk = base + c0 + k * MERGE_CELLS_PER_THREAD;
      if (e < n[k]) x[k] = h.stage[(row + blk) * HOT_STAGE_CAP + e];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (e < n[k]) merge_insert(L, x[k]);
  }
  __syncthreads();
  clk.at(2);  // stage cells summed
  for (int s = tid; s < MERGE_SLOTS; s += 1024) hist_add_wave(L.hist, min(L.cnt[s], (uint32_t)SEL_BINS - 1), L.cnt[s] != 0);
  __syncthreads();
  uint32_t t, cum;
  clk.at(3);  // histogram
  wave_count_threshold(L.hist, HOT_PART_TOP, t, cum);
  clk.at(4);  // threshold
  const uint32_t ties = t > 1 ? HOT_PART_TOP - min(cum, (uint32_t)HOT_PART_TOP) : 0u;
  for (int s = tid; s < MERGE_SLOTS; s += 1024) {
    const uint32_t c = L.cnt[s];
    if (!c || c + 1 < t) continue;
    if (c < t && atomicAdd(&L.nties, 1u) >= ties) continue;
    const uint32_t o = atomicAdd(&L.nout, 1u);
    if (o >= (uint32_t)HOT_PART_TOP) continue;
    const size_t at = (size_t)part * HOT_PART_TOP + o;
    const uint64_t sg = L.sig[s];
    uint64_t sd = L.side[s];
    if (is_long_sig(sg)) {  // the sampled occurrence's bytes (zero-padded) -> the candidate's line
      const uint32_t len = (uint32_t)(sd >> 32), from = (uint32_t)sd;
      sd = len | ((uint64_t)at << 32);
      uint64_t* line = reinterpret_cast<uint64_t*>(h.long_bytes + at * 64);
      for (uint32_t c8 = 0; c8 < 64; c8 += 8) {
        uint64_t x = 0;
        for (uint32_t j = 0; j < 8 && c8 + j < len; ++j) x |= (uint64_t)h.text[(size_t)from + c8 + j] << (8 * j);
        line[c8 / 8] = x;
      }
    }
    h.cand_cnt[at] = c;
    h.cand_sig[at] = sg;
    h.cand_side[at] = sd;
    L.oc[o] = c;
    L.osig[o] = sg;
    L.oside[o] = sd;
  }
  __syncthreads();
  clk.at(5);  // candidates written
  if (tid == 0) h.cand_n[part] = min(L.nout, (uint32_t)HOT_PART_TOP);
#ifndef WC_PLACE_ABLATE
#define WC_PLACE_ABLATE 0  // profiling builds only (results invalid): 1 = no placement (empty image)
#endif
  if (WC_PLACE_ABLATE) {
    if (tid < 2 * GPP) h.image[slot_of(part * GPP + tid / 2, tid & 1)] = 0;
    return;
  }
  if (tid < 64) place_partition(h, part, min(L.nout, (uint32_t)HOT_PART_TOP), L.oc, L.osig, L.oside, L.ord);
  clk.at(6);  // placed
}

// ------------------------------------------------------------------ map
// cnt / off first: every per-token LDS address (the two hit atomics at 4 s
// and 16 KiB + 4 s, the probe reads at 32 KiB + 16 g) is one VGPR plus an
// immediate ds offset (< 64 KiB) — no VALU add per token
// LD: the top-down LONG layout's LDS (its 16-bit LONG cursors take what the
// deferred lists give up); the queue layout keeps round 4's layout exactly.
template <bool LD>
struct alignas(16) MapLds {
  uint32_t cnt[MAP_SLOTS];
  uint32_t off[MAP_SLOTS];              // chunk-relative first offset in the block
  alignas(16) uint64_t sig[MAP_SLOTS];  // hot table image (read-only while tokens stream); 0 = empty
  uint16_t list[MAP_WAVES][MAP_LIST];
  uint16_t dlist[MAP_WAVES][LD ? MAP_DEF_CAP : MAP_DEF_CAP_Q];  // deferred LONG entries of a round: pos | (len - 16) << 11 | prev << 15
  uint32_t bcur[2 * MAX_REC_BUCKETS];   // record cursors (map_common.hpp cursors_init): Rec16 | Rec per bucket
  uint32_t lcur[LD ? MAX_REC_BUCKETS / 2 : 1];  // LONG-record counts, 16 bits per bucket (map_common.hpp emit_long)
  uint32_t lovf;                        // a LONG count reached its sub-region
  uint32_t nltok;                       // LONG-word tokens of this block (MapArgs::long_tokens)
  alignas(16) uint8_t buf[MAP_WAVES][2][BUF];  // two unit slots per wave: the current unit and the one before
  uint32_t next_unit;
  unsigned long long used, tokens;
};
static_assert(sizeof(MapLds<true>) + 8 * MAP_STAMP_N <= 160 * 1024, "one map block per CU");
static_assert(sizeof(MapLds<false>) + 8 * MAP_STAMP_N <= 160 * 1024, "one map block per CU");
static_assert(MAP_DEF_CAP >= 128 + UNIT / 17, "a round defers at most 127 carried + UNIT / 17 LONG tokens");
static_assert(GS == 2, "pair-packed two-word words: 2-slot groups");

// Hot-table slot of a one-slot word's signature in its candidate groups g1 (a)
// and g2 (b), or -1: a compare + select chain straight to the slot index (a
// word sits in at most one slot; the old match-mask / ffs / slot decode took
// twice the VALU).
// Slot results are BYTE offsets of the slot's counter (4 * slot = 8 * group +
// 4 * i, from the groups' image offsets o = 16 * group: o / 2 + 4 i).
__device__ __forceinline__ int sig_slot4(const u64x2& a, const u64x2& b, uint64_t sig, uint32_t o1, uint32_t o2) {
  const int c1 = (int)(o1 >> 1), c2 = (int)(o2 >> 1);
  int s = b.y == sig ? c2 + 4 : -1;
  s = b.x == sig ? c2 : s;
  s = a.y == sig ? c1 + 4 : s;
  return a.x == sig ? c1 : s;
}

// Hot-table slot of an inline token (signature sig, k0): a one-slot word
// (sig's top byte < 8) in any of the four slots; a two-word word only in a
// group's first slot with k0 in the second.  -1: not in the table.
__device__ __forceinline__ int pair_slot(const u64x2& a, const u64x2& b, uint64_t sig, uint64_t k0, uint32_t o1,
                                         uint32_t o2) {
  const int s = b.x == sig && b.y == k0 ? (int)(o2 >> 1) : -1;
  return a.x == sig && a.y == k0 ? (int)(o1 >> 1) : s;
}
__device__ __forceinline__ int inline_slot(const u64x2& a, const u64x2& b, uint64_t sig, uint64_t k0, uint32_t o1,
                                           uint32_t o2) {
  return two_word(sig) ? pair_slot(a, b, sig, k0, o1, o2) : sig_slot4(a, b, sig, o1, o2);
}

// LDS word at byte offset o of an array (the hot table's count / offset arrays).
__device__ __forceinline__ uint32_t* at_byte(uint32_t* base, int o) {
  return reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(base) + o);
}

template <bool ST, bool LD>
__global__ void __launch_bounds__(MAP_THREADS, MAP_WAVES / 4) wc_map(MapArgs a, HotArgs h) {
  __shared__ MapLds<LD> L;
  __shared__ unsigned long long st_acc[ST ? MAP_STAMP_N : 1];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: per-wave LDS bases in SGPRs
  if (ST && tid < MAP_STAMP_N) st_acc[tid] = 0;
  // the pass's hot table image (wc_hot_merge built it once for every block)
  static_assert(MAP_SLOTS % 2 == 0, "image copy: 16-byte pieces");
  for (int i = tid; i < MAP_SLOTS / 2; i += MAP_THREADS)
    reinterpret_cast<u64x2*>(L.sig)[i] = reinterpret_cast<const u64x2*>(h.image)[i];
  for (int s = tid; s < MAP_SLOTS; s += MAP_THREADS) {
    L.cnt[s] = 0;
    L.off[s] = 0xFFFFFFFFu;
  }
  cursors_init(L.bcur, LD ? L.lcur : nullptr, 1u << a.log2_rec_buckets, a.rec.subcap);
  uint64_t u_begin, u_end;
  unit_range(a.chunk_len, gridDim.x, blockIdx.x, u_begin, u_end);
  if (tid == 0) {
    L.next_unit = 0;
    L.used = L.tokens = 0;
    L.lovf = 0;
    L.nltok = 0;
  }
  __syncthreads();

  const uint32_t bmask = (1u << a.log2_rec_buckets) - 1u;
  const uint32_t nb = 1u << a.log2_rec_buckets;
  const RecOut rout = rec_out(a);
  uint8_t* const bufw = &L.buf[wave][0][0];  // both unit slots: slot s at s * BUF
  uint16_t* list = L.list[wave];
  uint16_t* dlist = L.dlist[wave];
  uint32_t my_tokens = 0, my_direct = 0;
  uint64_t sink = 0;  // profiling builds: keeps ablated work alive
  auto grab = [&]() -> uint32_t {
    uint32_t v = 0;
    if (lane == 0) v = atomicAdd(&L.next_unit, 1u);
    v = __builtin_amdgcn_readfirstlane(v);
    return u_begin + v < u_end ? (uint32_t)(u_begin + v) : NONE;
  };
  // next unit's 32 B per lane (+ halo, + the byte before it) in registers
  uint4 p0 = make_uint4(0, 0, 0, 0), p1 = p0, ph16 = p0;
  uint32_t pprev = 0x20;
  auto prefetch = [&](uint32_t u) {
    if (u == NONE) return;
    const uint64_t g0 = (uint64_t)u * UNIT;
    load32(a, g0 + (uint64_t)lane * MAP_BPL, p0, p1);
    if (lane < HALO / 16) ph16 = load16(a, g0 + UNIT + (uint64_t)lane * 16);
    if (lane == 0) pprev = (g0 == 0 && a.prev_byte >= 0) ? (uint32_t)a.prev_byte : a.text[(int64_t)g0 - 1];
  };
  PhaseClock<ST> clk;
  clk.start(st_acc);
  const uint64_t t_begin = clk.t;
  const uint64_t rt_begin = ST ? __builtin_amdgcn_s_memrealtime() : 0;  // 100 MHz, one clock for every XCD
  const uint32_t pbase = lane * MAP_BPL;
  uint32_t ndef = 0;  // deferred LONG entries of the current round (dlist[0, ndef))
  // Unit slots: the current unit's text at byte cbo of bufw, the previous
  // unit's (entries carried over from its round) at pbo; their chunk offsets.
  uint32_t cbo = 0, pbo = BUF;
  uint64_t cu0 = 0, pu0 = 0;

  // LONG words of the round (>= 16 bytes): keys from LDS windows (16..30
  // bytes) or an 8-byte SWAR scan (>= 31), one record each; 64 per pass, both
  // unit slots still in LDS.
  auto run_deferred = [&]() {
    // the pass's LONG share picks the next pass's record layout: an LDS count of
    // the round's LONG tokens (ndef is wave-uniform; no register held across the loop)
    if (lane == 0 && ndef) atomicAdd(&L.nltok, ndef);
    wave_sync();
    for (uint32_t c = 0; c < ndef; c += 64) {
      const bool hv = c + lane < ndef;
      const uint32_t e = hv ? dlist[c + lane] : 0u;
      const uint32_t q = e & 0x7FFu, n = ((e >> 11) & 0xFu) + 16u;
      const bool old = (e >> 15) != 0;
      const uint8_t* buf = bufw + (old ? pbo : cbo);
      const uint64_t u0 = old ? pu0 : cu0;
      if (hv) {
        uint64_t k0, k1;
        uint32_t len = n;
        if (n < MAP_LONG) key_long_known(buf, q, n, a.k1_mask, k0, k1);  // 16..30 bytes: length known
        else len = (uint32_t)min<uint64_t>(key_long_scan(buf, UNIT + HALO, a, q, u0 + q, k0, k1), 0xFFFFFFFFull);
        // a hot LONG word: the signature in a group's first slot, then the
        // length and the bytes against the candidate's copy (side word = the
        // length | the candidate index << 32, in the group's second slot)
        int slot = -1;
        if (len <= HOT_LONG_MAX) {
          const uint64_t sg = long_signature(k0, k1);
          uint32_t g1, g2;
          hot_groups(long_group_hash(sg), g1, g2);
          const u64x2* S = reinterpret_cast<const u64x2*>(L.sig);
          const u64x2 x1 = S[g1], x2 = S[g2];
          const bool m1 = x1.x == sg, m2 = x2.x == sg;
          if (m1 || m2) {
            const uint64_t sd = m1 ? x1.y : x2.y;
            const uint8_t* line = h.long_bytes + (sd >> 32) * 64;
            bool eq;
            if constexpr (LD && WC_LONG_1RT) eq = (uint32_t)sd == len && long_line_equal_1rt(buf, q, line, len);
            else eq = (uint32_t)sd == len && long_line_equal(buf, q, line, len);
            if (eq) slot = (int)(2 * (m1 ? g1 : g2));
          }
        }
        if (slot >= 0) {
          atomicAdd(&L.cnt[slot], 1u);
          atomicMin(&L.off[slot], (uint32_t)(u0 + q));
        } else {
          const uint32_t bk = place_hash(k0, k1) & bmask;
          if constexpr (LD) emit_long(L.lcur, &L.lovf, rout, bk, k0, k1, 1, (uint32_t)(u0 + q));
          else put_rec24(rout, atomicAdd(&L.bcur[MAX_REC_BUCKETS + bk], 1u), k0, k1, 1, (uint32_t)(u0 + q));
        }
      }
    }
    if (ST) my_direct += ndef;
    ndef = 0;
    wave_sync();
  };

  // Carried entries: a round runs only FULL steps (128 entries) of each token
  // class; the remainder (< 128 entries) waits in the list for the next
  // round, whose unit goes to the other slot, so every step but the block's
  // last ones is full.  A remainder holding entries carried from the round
  // before (two units back: that slot is about to be overwritten) or of the
  // wave's last unit runs at once.  Carried entries go to the front of their
  // class in the next list; an entry below a step's `cut` index reads the
  // previous slot and offsets.
  uint32_t cs = 0, cs_from = 0, co = 0, co_from = 0;  // carried short / other entries and where they wait
  uint32_t pr1 = 0, pr2 = 0;  // a plain full step's entries, read one step ahead
  uint32_t u = grab();
  prefetch(u);
  uint32_t nu = u == NONE ? NONE : grab();
  while (u != NONE) {
    // ---- commit the prefetched unit into the free slot, masks and token count ----
    pbo = cbo;
    cbo = BUF - cbo;
    pu0 = cu0;
    cu0 = (uint64_t)u * UNIT;
    const uint64_t u0 = cu0;
    uint8_t* const buf = bufw + cbo;
    wave_sync();  // the previous unit's reads are done
    reinterpret_cast<uint4*>(&buf[pbase])[0] = p0;
    reinterpret_cast<uint4*>(&buf[pbase])[1] = p1;
    if (lane < HALO / 16) *reinterpret_cast<uint4*>(&buf[UNIT + lane * 16]) = ph16;
    const uint32_t pv = (uint32_t)__builtin_amdgcn_readlane((int)pprev, 0);
    const uint4 c0 = p0, c1 = p1;
    const uint32_t hb = halo_bits(ph16);
    prefetch(nu);  // the LDS copy is first read by the steps, behind the list round's wave_sync
    clk.lap(MS_COMMIT);
    if (WC_MAP_ABLATE == 5) {  // stream + commit only
      sink ^= c0.x ^ c1.w ^ hb ^ pv;
      u = nu;
      nu = u == NONE ? NONE : grab();
      continue;
    }
    uint64_t dm;
    uint32_t bits;
    unit_masks(c0, c1, hb, pv, u0, pbase, a.chunk_len, dm, bits);
    my_tokens += __popc(bits);
    if (WC_MAP_ABLATE == 4) {  // + masks and token starts, no list / steps
      sink ^= dm ^ wave_incl_sum(bits);
      u = nu;
      nu = u == NONE ? NONE : grab();
      continue;
    }
    const uint32_t dlo = (uint32_t)dm, dhi = (uint32_t)(dm >> 32);
    // delimiter bits from the token start on (i < 32: one funnel shift); none
    // within 31 bytes -> MAP_LONG: ffbl of 0 is all ones, and the u16 entry
    // keeps 5 length bits, so (ffbl << 11) needs no clamp
    static_assert(MAP_LONG == 31, "list entries: 11 position bits + 5 length bits");
    // One step: two list entries [j, hi) per lane, both probed in one LDS round
    // trip; a tail of <= 64 entries takes the one-entry step.  General form:
    // any length (two-word signatures are confirmed by their group's side
    // word, LONG words deferred to the round end).
    auto step = [&](uint32_t j, uint32_t hi, uint32_t cut, auto two_c, auto mixed_c, auto any_c, auto full_c) {
      // ANY: entries of any length (the > MAP_LIST rounds); otherwise the
      // other class only (8 bytes or longer: k0 is the first window as read)
      constexpr bool TWO = decltype(two_c)::value, MIXED = decltype(mixed_c)::value, ANY = decltype(any_c)::value;
      constexpr bool FULL = decltype(full_c)::value;  // j + 128 <= hi: every lane holds two entries
      static_assert(!FULL || TWO, "full steps take two entries per lane");
      const bool h1 = FULL || j + lane < hi, h2 = TWO && (FULL || j + 64 + lane < hi);
      // unconditional (see step_short); a plain full step's entries were read by the step before it
      constexpr bool PRE = FULL && !MIXED;
      const uint32_t r1 = PRE ? pr1 : list[j + lane], r2 = PRE ? pr2 : TWO ? list[j + 64 + lane] : 0u;
      const uint32_t e1 = h1 ? r1 : 0u, e2 = h2 ? r2 : 0u;
      if (WC_MAP_ABLATE == 7) {
        sink ^= e1 ^ e2;
        return;
      }
      const uint32_t q1 = e1 & 0x7FFu, q2 = e2 & 0x7FFu, n1 = e1 >> 11, n2 = e2 >> 11;
      const bool old1 = MIXED && j + lane < cut, old2 = MIXED && TWO && j + 64 + lane < cut;  // carried entries
      uint64_t w10, w11, w20 = 0, w21 = 0;
      window16(bufw, q1 + (old1 ? pbo : cbo), w10, w11);
      if (TWO) window16(bufw, q2 + (old2 ? pbo : cbo), w20, w21);
      if (PRE) {  // the next step's entries, beside this step's windows (past the list: inside MapLds, unused)
        pr1 = list[j + 128 + lane];
        pr2 = list[j + 192 + lane];
      }
      if (WC_MAP_ABLATE == 1) {
        sink ^= w10 ^ w21;
        return;
      }
      const bool in1 = h1 && n1 <= KEY_INLINE_MAX, in2 = h2 && n2 <= KEY_INLINE_MAX;
      uint64_t a0, a1, as, b0 = 0, b1 = 0, bs = 0;
      if (ANY) {
        inline_key(w10, w11, n1, a0, a1, as);
        if (TWO) inline_key(w20, w21, n2, b0, b1, bs);
      } else {
        inline_key_long8(w10, w11, n1, a0, a1, as);
        if (TWO) inline_key_long8(w20, w21, n2, b0, b1, bs);
      }
      const uint32_t ha = place_hash(a0, a1), hb = TWO ? place_hash(b0, b1) : 0u;
      uint32_t ga1, ga2, gb1 = 0, gb2 = 0;  // group byte offsets in the image
      hot_group_offs(ha, ga1, ga2);
      if (TWO) hot_group_offs(hb, gb1, gb2);
      clk.lap(MS_KEYS);
      if (WC_MAP_ABLATE == 2) {
        sink ^= as ^ bs ^ ga2 ^ gb2;
        return;
      }
      const uint8_t* S = reinterpret_cast<const uint8_t*>(L.sig);
      int s1 = -1, s2 = -1;  // counter byte offsets
      {  // both slots of a group in one 16-byte read
        // (other class, 8..15 bytes: always a two-word signature — only the pair match)
        const u64x2 xa0 = *reinterpret_cast<const u64x2*>(S + ga1), xa1 = *reinterpret_cast<const u64x2*>(S + ga2);
        if (TWO) {
          const u64x2 xb0 = *reinterpret_cast<const u64x2*>(S + gb1), xb1 = *reinterpret_cast<const u64x2*>(S + gb2);
          s2 = in2 ? (ANY ? inline_slot(xb0, xb1, bs, b0, gb1, gb2) : pair_slot(xb0, xb1, bs, b0, gb1, gb2)) : -1;
        }
        s1 = in1 ? (ANY ? inline_slot(xa0, xa1, as, a0, ga1, ga2) : pair_slot(xa0, xa1, as, a0, ga1, ga2)) : -1;
      }
      clk.lap(MS_PROBE);
      const uint32_t o1 = (uint32_t)(old1 ? pu0 : cu0) + q1, o2 = (uint32_t)(old2 ? pu0 : cu0) + q2;
      if (s1 >= 0) {
        atomicAdd(at_byte(L.cnt, s1), 1u);  // results unused: no-return ds_add / ds_min
        atomicMin(at_byte(L.off, s1), o1);
      }
      if (TWO && s2 >= 0) {
        atomicAdd(at_byte(L.cnt, s2), 1u);
        atomicMin(at_byte(L.off, s2), o2);
      }
      if (WC_MAP_ABLATE == 3) return;
      // misses of inline words become records now; LONG words wait for the round end
      const bool d1 = in1 && s1 < 0, d2 = TWO && in2 && s2 < 0;
      emit_two(L.bcur, rout, d1, ha & bmask, a0, a1, o1, n1, d2, hb & bmask, b0, b1, o2, n2);
      const bool f1 = h1 && !in1, f2 = TWO && h2 && !in2;
      const uint64_t mf1 = __ballot(f1), mf2 = TWO ? __ballot(f2) : 0ull;
      if (mf1 | mf2) {  // LONG entries (length field 16..31) to the round's deferred list
        const uint32_t r1 =
            __builtin_amdgcn_mbcnt_hi((uint32_t)(mf1 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mf1, 0u));
        const uint32_t r2 =
            __builtin_amdgcn_mbcnt_hi((uint32_t)(mf2 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mf2, 0u));
        const uint32_t n1c = (uint32_t)__popcll(mf1);
        if (f1) dlist[ndef + r1] = (uint16_t)(q1 | ((n1 - 16u) << 11) | (old1 ? 0x8000u : 0u));
        if (f2) dlist[ndef + n1c + r2] = (uint16_t)(q2 | ((n2 - 16u) << 11) | (old2 ? 0x8000u : 0u));
        ndef += n1c + (uint32_t)__popcll(mf2);
      }
      if constexpr (ST) {
        my_direct += (uint32_t)(__popcll(__ballot(d1)) + (TWO ? __popcll(__ballot(d2)) : 0));
        const uint32_t nh = (uint32_t)(__popcll(__ballot(s1 >= 0)) + __popcll(__ballot(s2 >= 0)));
        if (lane == 0) {
          atomicAdd(&st_acc[MS_N_HIT], (unsigned long long)nh);
          atomicAdd(&st_acc[MS_N_DEFER], (unsigned long long)__popcll(mf1 | mf2));
        }
      }
      clk.lap(MS_EMIT);
    };
    // Short step: entries of words of <= 7 bytes only — the signature IS the
    // key (bytes | len << 56): one 8-byte window (three LDS dwords, two
    // funnels), no tail, no side-word confirmation, and every miss a 16-byte
    // record candidate.  3 of 4 tokens of English-like text take it.
    auto step_short = [&](uint32_t j, uint32_t hi, uint32_t cut, auto two_c, auto mixed_c, auto full_c) {
      constexpr bool TWO = decltype(two_c)::value, MIXED = decltype(mixed_c)::value;
      constexpr bool FULL = decltype(full_c)::value;  // j + 128 <= hi
      static_assert(!FULL || TWO, "full steps take two entries per lane");
      const bool h1 = FULL || j + lane < hi, h2 = TWO && (FULL || j + 64 + lane < hi);
      // unconditional entry reads (no exec-mask branch): past `hi` they read a
      // later entry, the next wave's list or the deferred lists — inside MapLds, and masked by h1 / h2
      constexpr bool PRE = FULL && !MIXED;  // entries read by the step before (see step)
      const uint32_t r1 = PRE ? pr1 : list[j + lane], r2 = PRE ? pr2 : TWO ? list[j + 64 + lane] : 0u;
      const uint32_t e1 = h1 ? r1 : 0u, e2 = h2 ? r2 : 0u;
      if (WC_MAP_ABLATE == 7) {
        sink ^= e1 ^ e2;
        return;
      }
      const uint32_t q1 = e1 & 0x7FFu, q2 = e2 & 0x7FFu, n1 = e1 >> 11, n2 = e2 >> 11;
      const bool old1 = MIXED && j + lane < cut, old2 = MIXED && TWO && j + 64 + lane < cut;  // carried entries
      const uint64_t w1 = window8(bufw, q1 + (old1 ? pbo : cbo)), w2 = TWO ? window8(bufw, q2 + (old2 ? pbo : cbo)) : 0ull;
      if (PRE) {
        pr1 = list[j + 128 + lane];
        pr2 = list[j + 192 + lane];
      }
      if (WC_MAP_ABLATE == 1) {
        sink ^= w1 ^ w2;
        return;
      }
      // k0: the first n bytes — the mask -1 >> (64 - 8 n), with 8 n taken from
      // the entry's length field by a right shift and an and (full-rate ops; an
      // empty lane's n = 0 shifts by (64 & 63) = 0: garbage, masked by h)
      const uint32_t sa = (64u - ((e1 >> 8) & 0xF8u)) & 63u, sb = (64u - ((e2 >> 8) & 0xF8u)) & 63u;
      const uint64_t a0 = w1 & (~0ull >> sa), b0 = TWO ? w2 & (~0ull >> sb) : 0ull;
      const uint64_t as = a0 | ((uint64_t)n1 << 56), bs = b0 | ((uint64_t)n2 << 56);
      const uint32_t ha = place_hash(a0, n1), hb = TWO ? place_hash(b0, n2) : 0u;
      uint32_t ga1, ga2, gb1 = 0, gb2 = 0;  // group byte offsets in the image
      hot_group_offs(ha, ga1, ga2);
      if (TWO) hot_group_offs(hb, gb1, gb2);
      clk.lap(MS_KEYS);
      if (WC_MAP_ABLATE == 2) {
        sink ^= as ^ bs ^ ga2 ^ gb2;
        return;
      }
      const uint8_t* S = reinterpret_cast<const uint8_t*>(L.sig);
      int s1 = -1, s2 = -1;  // counter byte offsets
      {  // a pair's side word never equals a short signature: plain 4-slot match
        // (an empty lane's signature has top byte 0, like a LONG group's side word: masked by h)
        const u64x2 xa0 = *reinterpret_cast<const u64x2*>(S + ga1), xa1 = *reinterpret_cast<const u64x2*>(S + ga2);
        if (TWO) {
          const u64x2 xb0 = *reinterpret_cast<const u64x2*>(S + gb1), xb1 = *reinterpret_cast<const u64x2*>(S + gb2);
          const int m2 = sig_slot4(xb0, xb1, bs, gb1, gb2);
          s2 = h2 ? m2 : -1;
        }
        const int m1 = sig_slot4(xa0, xa1, as, ga1, ga2);
        s1 = h1 ? m1 : -1;
      }
      clk.lap(MS_PROBE);
      const uint32_t o1 = (uint32_t)(old1 ? pu0 : cu0) + q1, o2 = (uint32_t)(old2 ? pu0 : cu0) + q2;
      if (s1 >= 0) {
        atomicAdd(at_byte(L.cnt, s1), 1u);
        atomicMin(at_byte(L.off, s1), o1);
      }
      if (TWO && s2 >= 0) {
        atomicAdd(at_byte(L.cnt, s2), 1u);
        atomicMin(at_byte(L.off, s2), o2);
      }
      if (WC_MAP_ABLATE == 3) return;
      const bool d1 = h1 && s1 < 0, d2 = TWO && h2 && s2 < 0;
      emit_two_short(L.bcur, rout, d1, ha & bmask, a0, o1, n1, d2, hb & bmask, b0, o2, n2);
      if constexpr (ST) {
        my_direct += (uint32_t)(__popcll(__ballot(d1)) + (TWO ? __popcll(__ballot(d2)) : 0));
        const uint32_t nh = (uint32_t)(__popcll(__ballot(s1 >= 0)) + __popcll(__ballot(s2 >= 0)));
        if (lane == 0) atomicAdd(&st_acc[MS_N_HIT], (unsigned long long)nh);
      }
      clk.lap(MS_EMIT);
    };
    // short token starts: a delimiter within the next 7 bytes (dm bits i+1..i+7)
    const uint64_t s1m = dm >> 1, s2m = s1m | (s1m >> 1), s4m = s2m | (s2m >> 2);
    const uint32_t near7 = (uint32_t)(s4m | (s4m >> 3));
    const uint32_t sbits = bits & near7, obits = bits & ~near7;
    // both class counts in one packed DPP scan (short | other << 16)
    const uint32_t cnt2 = (uint32_t)__popc(sbits) | ((uint32_t)__popc(obits) << 16);
    const uint32_t inc2 = wave_incl_sum(cnt2), exc2 = inc2 - cnt2;
    const uint32_t tot2 = (uint32_t)__builtin_amdgcn_readlane((int)inc2, 63);
    const uint32_t ks0 = exc2 & 0xFFFFu, ko0 = exc2 >> 16;
    const uint32_t tot_s = tot2 & 0xFFFFu, tot_o = tot2 >> 16;
    const uint32_t wave_total = tot_s + tot_o;
    clk.lap(MS_MASK);
    const bool last = nu == NONE;  // the wave's last unit: nothing is carried past it
    if (cs + co + wave_total <= (uint32_t)MAP_LIST) {
      // one list round: short entries at [0, ns) — the cs carried ones first —
      // the others at [ns, no_end) — the co carried ones first; one loop per
      // class (no per-entry class select: 9 instead of 16 VALU per entry)
      const uint32_t ns = cs + tot_s, ob0 = ns, no_end = ns + co + tot_o;
      {  // carried entries to the front of their class (read before any write: one wave, in order)
        const uint32_t c0 = list[cs_from + lane], c1 = list[cs_from + 64 + lane];
        const uint32_t d0 = list[co_from + lane], d1 = list[co_from + 64 + lane];
        wave_sync();
        if (lane < cs) list[lane] = (uint16_t)c0;
        if (lane + 64 < cs) list[64 + lane] = (uint16_t)c1;
        if (lane < co) list[ob0 + lane] = (uint16_t)d0;
        if (lane + 64 < co) list[ob0 + 64 + lane] = (uint16_t)d1;
      }
      uint32_t ks = cs + ks0, ko = ob0 + co + ko0, sb = sbits, ob = obits;
      // the lane's byte base, opaque: the entry's position q = base | i also
      // feeds alignbit (which reads q's low 5 bits = i), so the entry is one
      // lshl_or (known low zero bits would fold q back to i and add an or3)
      uint32_t pb = pbase;
      asm volatile("" : "+v"(pb));
      while (sb) {
        const uint32_t q = pb | (uint32_t)(__ffs(sb) - 1);
        sb &= sb - 1;
        list[ks++] = (uint16_t)(q | (ffbl_raw(__builtin_amdgcn_alignbit(dhi, dlo, q)) << 11));
      }
      while (ob) {
        const uint32_t q = pb | (uint32_t)(__ffs(ob) - 1);
        ob &= ob - 1;
        list[ko++] = (uint16_t)(q | (ffbl_raw(__builtin_amdgcn_alignbit(dhi, dlo, q)) << 11));
      }
      wave_sync();
      clk.lap(MS_LIST);
      if (WC_MAP_ABLATE == 6) {  // + the token list, no steps
        sink ^= list[lane];
        wave_sync();
        cs = co = 0;
        u = nu;
        nu = u == NONE ? NONE : grab();
        continue;
      }
      // full steps; a remainder waits for the next round unless it holds
      // carried entries (their slot is overwritten next) or this is the last unit
      // (explicit loops: the same steps behind a lambda made the kernel spill ~80 VGPRs)
      // (only a round's first step of a class can hold carried entries: MIXED
      // steps select slot and offsets per entry, the others need not)
      constexpr std::true_type T{}, M{};
      constexpr std::false_type F{}, P{};
      uint32_t j = 0;
      if (cs && ns >= 128) {
        step_short(0u, ns, cs, T, M, T);
        j = 128;
      }
      pr1 = list[j + lane];
      pr2 = list[j + 64 + lane];
      for (; j + 128 <= ns; j += 128) step_short(j, ns, 0u, T, P, T);
      if (j < ns && (j < cs || last)) {
        if (j < cs) step_short(j, ns, cs, T, M, F);
        else if (j + 64 < ns) step_short(j, ns, 0u, T, P, F);
        else step_short(j, ns, 0u, F, P, F);
        j = ns;
      }
      cs_from = j;
      cs = ns - j;
      const uint32_t ocut = ob0 + co;
      j = ob0;
      if (co && no_end >= ob0 + 128) {
        step(j, no_end, ocut, T, M, F, T);
        j += 128;
      }
      pr1 = list[j + lane];
      pr2 = list[j + 64 + lane];
      for (; j + 128 <= no_end; j += 128) step(j, no_end, 0u, T, P, F, T);
      if (j < no_end && (j < ocut || last)) {
        if (j < ocut) step(j, no_end, ocut, T, M, F, F);
        else if (j + 64 < no_end) step(j, no_end, 0u, T, P, F, F);
        else step(j, no_end, 0u, F, P, F, F);
        j = no_end;
      }
      co_from = j;
      co = no_end - j;
      if (ndef) {
        run_deferred();
        clk.lap(MS_SLOW);
      }
      wave_sync();  // entries read before the next unit's list overwrites them
    } else {
      // more than MAP_LIST tokens with the carried ones (runs of 1-byte
      // words): the carried entries first, then rounds of MAP_LIST entries of
      // the unit in stream order, every entry on the general step
      // all carried: the cut past them (one general step per class, < 128 entries each)
      if (cs) step_short(cs_from, cs_from + cs, MAP_LIST, std::true_type{}, std::true_type{}, std::false_type{});
      if (co) step(co_from, co_from + co, MAP_LIST, std::true_type{}, std::true_type{}, std::false_type{}, std::false_type{});
      cs = co = 0;
      if (ndef) {
        run_deferred();
        clk.lap(MS_SLOW);
      }
      wave_sync();
      uint32_t k = ks0 + ko0;  // the lane's first entry among all tokens of the unit
      for (uint32_t base = 0; base < wave_total; base += MAP_LIST) {
        const uint32_t lim = base + MAP_LIST;
        while (bits && k < lim) {
          const uint32_t i = __ffs(bits) - 1;
          bits &= bits - 1;
          const uint32_t rest = __builtin_amdgcn_alignbit(dhi, dlo, i);
          list[k - base] = (uint16_t)((pbase + i) | (ffbl_raw(rest) << 11));
          ++k;
        }
        wave_sync();
        const uint32_t round_n = min(wave_total - base, (uint32_t)MAP_LIST);
        clk.lap(MS_LIST);
        uint32_t j = 0;
        for (; j + 64 < round_n; j += 128) step(j, round_n, 0u, std::true_type{}, std::false_type{}, std::true_type{}, std::false_type{});
        if (j < round_n) step(j, round_n, 0u, std::false_type{}, std::false_type{}, std::true_type{}, std::false_type{});
        if (ndef) {
          run_deferred();
          clk.lap(MS_SLOW);
        }
        wave_sync();  // entries read before the next round overwrites them
      }
    }
    u = nu;
    nu = u == NONE ? NONE : grab();
  }
  __syncthreads();
  clk.lap(MS_WAIT);
  // block end: every counted hot slot becomes one record of its bucket (a
  // two-word or LONG word counts in its group's first slot; its side word is
  // the second)
  for (int s = tid; s < MAP_SLOTS; s += MAP_THREADS) {
    const uint32_t c = L.cnt[s];
    if (!c) continue;
    uint64_t k0, k1;
    const uint64_t sg = L.sig[s];
    const uint64_t sd = (two_word(sg) || is_long_sig(sg)) ? L.sig[s | 1] : 0ull;
    if (is_long_sig(sg)) key_long_line(h.long_bytes + (sd >> 32) * 64, (uint32_t)sd, a.k1_mask, k0, k1);
    else sig_key(sg, sd, k0, k1);
    emit_record<LD>(L.bcur, L.lcur, &L.lovf, rout, place_hash(k0, k1) & bmask, k0, k1, c, L.off[s]);
  }
  clk.lap(MS_FLUSH);
  if constexpr (ST) {
    if (lane == 0) atomicAdd(&st_acc[MS_TOTAL], (unsigned long long)(clk.t - t_begin));
    if (lane == 0) atomicAdd(&st_acc[MS_N_DIRECT], (unsigned long long)my_direct);
    if (tid == 0) {  // block duration (load balance across the grid)
      atomicAdd(&a.stamps[MS_BLKSUM], (unsigned long long)(clk.t - t_begin));
      atomicMax(&a.stamps[MS_BLKMAX], (unsigned long long)(clk.t - t_begin));
      if (a.blk) {  // where the imbalance comes from: start skew, XCC, units taken
        unsigned long long* r = a.blk + 4 * (size_t)blockIdx.x;
        r[0] = rt_begin;
        r[1] = __builtin_amdgcn_s_memrealtime();
        r[2] = (unsigned long long)(__builtin_amdgcn_s_getreg((3 << 11) | 20) & 15);  // HW_REG_XCC_ID [3:0]
        r[3] = L.next_unit;
      }
    }
  }
  if (WC_MAP_ABLATE && sink == 0x9E3779B97F4A7C15ull) atomicOr(&a.flags[FLAG_COUNT - 1], 0u);  // never true
  // records of the block = the sum of its bucket cursors (no per-step counting)
  __syncthreads();  // every flush's cursor add is in
  uint64_t t = my_tokens, e = 0;
  for (uint32_t b = tid; b < nb; b += MAP_THREADS) {
    const uint32_t sub = rout.sub, c16 = L.bcur[b] - b * sub, c24 = L.bcur[MAX_REC_BUCKETS + b] - b * sub;
    const uint32_t cl = LD ? (L.lcur[b >> 1] >> (16u * (b & 1u))) & 0xFFFFu : 0u;
    // overran into the next sub-region (24-byte records grow up, LONG ones down)
    if (c16 > sub || c24 + cl > sub || (LD && L.lovf)) atomicOr(&a.flags[FLAG_REGION_OVF], 1u);
    const uint32_t n16 = min(c16, sub), n24 = min(c24, sub), nl = min(cl, sub);
    a.rec.count[(size_t)blockIdx.x * nb + b] = n16 | (n24 << 16);  // packed for the reducer (sub <= 0xFFFF)
    a.rec.count_long[(size_t)blockIdx.x * nb + b] = nl;
    if (a.bucket_w && (n16 | n24 | nl)) atomicAdd(&a.bucket_w[b], n16 + RED_W24 * n24 + RED_WLONG * nl);  // dispatch plan
    e += n16 + n24 + nl;
  }
  for (int o = 32; o > 0; o >>= 1) {
    t += __shfl_down(t, o);
    e += __shfl_down(e, o);
  }
  if (lane == 0) {
    atomicAdd(&L.tokens, (unsigned long long)t);
    atomicAdd(&L.used, (unsigned long long)e);
  }
  __syncthreads();
  if constexpr (ST) {
    if (tid < MS_BLKSUM) atomicAdd(&a.stamps[tid], st_acc[tid]);
  }
  if (tid == 0) {
    atomicAdd(a.tokens, L.tokens);
    atomicAdd(a.rec.cursor, L.used);
    if (L.nltok && a.long_tokens) atomicAdd(a.long_tokens, (unsigned long long)L.nltok);
  }
}

}  // namespace dev

void hot_setup_stamps(unsigned long long* d) {
  WC_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(dev::hot_stamps), &d, sizeof d));
}

void launch_map(const MapArgs& a, const HotArgs& h, uint32_t map_blocks, hipStream_t s, bool sample,
                const ZeroList& z) {
  if (sample) {  // the zeroing rides in the sampling launch
    hipLaunchKernelGGL(dev::wc_hot_sample, dim3(map_blocks), dim3(MAP_THREADS), 0, s, a, h, z);
    hipLaunchKernelGGL(dev::wc_hot_merge, dim3(HOT_PARTS), dim3(1024), 0, s, h);
  } else {
    launch_zero_regions(z, s);
  }
  if (a.stamps) {
    if (a.long_direct) hipLaunchKernelGGL((dev::wc_map<true, true>), dim3(map_blocks), dim3(MAP_THREADS), 0, s, a, h);
    else hipLaunchKernelGGL((dev::wc_map<true, false>), dim3(map_blocks), dim3(MAP_THREADS), 0, s, a, h);
  } else {
    if (a.long_direct) hipLaunchKernelGGL((dev::wc_map<false, true>), dim3(map_blocks), dim3(MAP_THREADS), 0, s, a, h);
    else hipLaunchKernelGGL((dev::wc_map<false, false>), dim3(map_blocks), dim3(MAP_THREADS), 0, s, a, h);
  }
}

}  // namespace wc
