// kernels.hpp — host-side launch interface of every hand-written CDNA4 kernel.
//
// Pipeline per chunk (SURVEY §2.2 replacement column):
//   wc_map            text -> token keys -> LDS pre-aggregation -> bucketed records
//   wc_reduce_buckets records -> per-bucket LDS hash table -> running key table
//   wc_table_split    running table B -> 2B buckets (grows with the vocabulary)
//   wc_table_compact  running table -> dense key list
//   wc_radix_*        LSD radix sort (first-occurrence order, merge dictionary)
//   wc_synth_text     device-side synthetic text generator
// Reference counterparts: mapKernel (/root/reference/main.cu:109-117) and the
// single-thread reduceKernel (main.cu:119-123).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace wc {

// ---- geometry (gfx950: wave64, 256 CUs, 160 KiB LDS per CU) -------------------
#ifndef WC_MAP_THREADS
#define WC_MAP_THREADS 1024
#endif
#ifndef WC_MAP_BLOCKS_PER_CU
#define WC_MAP_BLOCKS_PER_CU 1
#endif
#ifndef WC_MAP_SLOTS
#define WC_MAP_SLOTS 4096
#endif
constexpr int MAP_THREADS = WC_MAP_THREADS;          // 16 waves, one block per CU
constexpr int MAP_BLOCKS_PER_CU = WC_MAP_BLOCKS_PER_CU;
constexpr int MAP_BPL = 32;                          // text bytes per lane
constexpr int MAP_TILE = 1024 * MAP_BPL;             // 32 KiB: chunk-length granule of the engine (16 wave units)
static_assert(MAP_THREADS % 256 == 0 && MAP_THREADS <= 1024, "map block: the same wave count on every SIMD");
constexpr int MAP_SLOTS = WC_MAP_SLOTS;              // LDS combiner slots (groups of 4)
constexpr int MAX_REC_BUCKETS_LOG2 = 9;              // shuffle partitions <= 512
constexpr int MAX_REC_BUCKETS = 1 << MAX_REC_BUCKETS_LOG2;

constexpr int RED_THREADS = 1024;                    // 16 waves, one block per CU
constexpr int RED_MAX_RUNS = 1024;                   // map blocks per pass (the reducer stages their run counts in LDS)
constexpr int TAB_SLOTS_LOG2 = 12;
constexpr int TAB_SLOTS = 1 << TAB_SLOTS_LOG2;       // 4096 slots x 32 B = 128 KiB LDS
constexpr int TAB_MAX_OCC = TAB_SLOTS * 7 / 8;       // overflow -> split the table
constexpr int TAB_SPLIT_AT = TAB_SLOTS * 5 / 8;      // proactive split threshold
constexpr int TAB_GROUPS = TAB_SLOTS / 4;
constexpr int TAB_MAX_GROUP_PROBES = 64;

// ---- flags word indices ------------------------------------------------------
enum : int { FLAG_REGION_OVF = 0, FLAG_ARENA_OVF = 1, FLAG_TABLE_OVF = 2, FLAG_MAX_OCC = 3, FLAG_COUNT = 4 };

// One shuffle record: key words and (count << 32 | chunk-relative first offset).
struct Rec {
  uint64_t k0, k1, co;
};
// One occurrence of an inline word of <= 12 bytes whose last byte is nonzero:
// 16 bytes, count 1, one aligned dwordx4.  k0 = lo | hi << 32 (the first 8
// bytes), t = bytes [8, 12) zero-padded; the length is implied by the highest
// nonzero byte (of t if t != 0, else of k0: keys.hpp implied_len), so
// k1 = t ? t | len << 56 : len.  Every other record — counted hot-slot
// flushes, 13..15-byte and LONG words included — is a 24-byte Rec.
struct Rec16 {
  uint32_t lo, hi, t, off;  // off: chunk-relative offset
};
static_assert(sizeof(Rec16) == 16, "Rec16 layout");

// Shuffle output.  Two record stores (single occurrences of <= 12-byte words as
// 16-B Rec16, everything else as 24-B Rec), each split into one sub-region of
// `subcap` records per (map block p, shuffle bucket b):
//   recs16[(p * nb + b) * subcap + i],  i < count[p * nb + b] & 0xFFFF
//   recs  [(p * nb + b) * subcap + i],  i < count[p * nb + b] >> 16
// The map appends records to its bucket's sub-region through a per-bucket LDS
// cursor (no histogram, no scan, no directory) and the reducer of bucket b
// reads one contiguous run per map block.  A full sub-region sets FLAG_REGION_OVF and
// the host re-runs the chunk in halves.
struct Records {
  Rec* recs;                   // 24-byte records
  Rec16* recs16;               // single occurrences of <= 12-byte words
  unsigned long long* cursor;  // records emitted (stats)
  uint64_t cap;                // record capacity of each store
  uint32_t* count;             // [map_blocks * nb] Rec16 (low 16 bits) | Rec (high 16) records appended
  uint32_t subcap;             // records per sub-region, <= 65535 (cap / (map_blocks * nb) of the pass)
  // LONG-word records (hashed keys: their bytes are compared in the reduce)
  // fill the same 24-byte sub-region from its TOP down — recs[(p nb + b + 1)
  // subcap - 1 - i], i < count_long[p nb + b] — so the reducer streams them
  // directly instead of re-scanning the 24-byte runs for them
  uint32_t* count_long;        // [map_blocks * nb]
};

// Running key table: n_buckets x TAB_SLOTS open-addressing slices.
struct TableView {
  uint64_t* k0;
  uint64_t* k1;
  uint64_t* cnt;
  uint64_t* first;     // global byte offset of the first occurrence
  uint64_t* sref_off;  // arena offset of the word bytes (long words only)
  uint32_t* sref_len;
  uint32_t* occupancy;  // [n_buckets]
  uint32_t log2_buckets;
};

struct Arena {
  uint8_t* bytes;
  unsigned long long* cursor;
  uint64_t cap;
};

struct MapArgs {
  const uint8_t* text;  // chunk start (16-B aligned)
  uint64_t chunk_len;   // tokens owned: those starting in [0, chunk_len)
  uint64_t avail_len;   // bytes readable from text (>= chunk_len), for straddling tokens
  int32_t prev_byte;    // byte before the chunk; -1 = read text[-1]
  uint32_t log2_rec_buckets;
  Records rec;
  uint32_t* flags;
  unsigned long long* tokens;   // += tokens owned by this chunk
  uint64_t k1_mask;            // LONG-key hash bits kept (K1_HASH_MASK; collision tests truncate)
  unsigned long long* stamps;  // diagnostic build: per-phase s_memtime sums (MAP_STAMP_N), nullptr = off
  unsigned long long* blk;     // diagnostic: per map block {start, end (s_memrealtime), XCC id, units}, nullable
  // nullable (zeroed per pass): per shuffle bucket, += the reduce-cost weight of
  // every map block's run (Rec16 records + RED_W24 x 24-byte records) — the
  // balanced reduce's plan (ReduceArgs::bucket_w)
  uint32_t* bucket_w;
  // LONG-word records (hashed keys): true = into the top of their 24-byte
  // sub-region (Records::count_long, streamed by the reduce's long_direct);
  // false = appended to the 24-byte run like any 24-byte record (the reduce
  // queues them while it streams).  The engine picks per pass from the LONG
  // token share of the pass before (Engine::Impl::long_direct); every pass's reduce
  // runs the same mode (ReduceArgs::long_direct).
  bool long_direct = false;
  unsigned long long* long_tokens = nullptr;  // nullable: += LONG-word tokens of the pass (hot hits included)
};
// Reduce cost of a record relative to a Rec16 one in the dispatch plan: a
// LONG word's byte comparison (a random 64-byte text read) costs ~10-20x a
// Rec16 merge (profiles/r5_session.md §4)
constexpr uint32_t RED_W24 = 2;     // a 24-byte inline-key record (a counted hot slot, a 13..15-byte word)
constexpr uint32_t RED_WLONG = 16;  // a LONG-word record
// Hot-key sampling workspace (map.hip).  Two launches, no device-scope
// atomics and nothing to zero: wc_hot_sample writes every map block's sampled
// words, split by fingerprint into HOT_PARTS partitions, to its own stage
// cells; wc_hot_merge (one block per partition) sums them in LDS and keeps the
// partition's HOT_PART_TOP most frequent words as candidates.  Every wc_map
// block then selects the HOT_K most frequent candidates and places them in its
// own LDS table (blocks need not agree: each flushes its slots with full keys).
struct HotEnt {  // one sampled word (32 B)
  uint64_t sig, side;
  uint32_t cnt, pad;
  uint64_t fp;  // 64-bit fingerprint, never 0; its top byte is the partition
};
struct HotArgs {
  HotEnt* stage;           // [HOT_PARTS][maxb][HOT_STAGE_CAP] per (partition, map block)
  uint32_t* stage_n;       // [HOT_PARTS][maxb] entries written (every cell written by its block)
  uint32_t* cand_cnt;      // [HOT_PARTS][HOT_PART_TOP] candidates of each partition (SoA)
  uint64_t* cand_sig;
  uint64_t* cand_side;     // side word; LONG words: the length | candidate index << 32
  uint32_t* cand_n;        // [HOT_PARTS]
  uint32_t maxb;           // stage stride: the engine's map grid
  uint32_t nblk;           // map blocks of the sampling pass (<= maxb)
  // Hot LONG words (16..HOT_LONG_MAX bytes): wc_hot_merge copies each LONG
  // candidate's bytes (zero-padded) into the candidate's 64-byte line; the map
  // verifies every hit against it byte for byte (persists while the candidates
  // are reused)
  uint8_t* long_bytes;     // [HOT_PARTS * HOT_PART_TOP * 64]
  const uint8_t* text;     // the sampling pass's chunk text (the merge reads the sampled occurrence)
  // The hot table image, built ONCE per sampled pass — each wc_hot_merge block
  // places its partition's words into its partition's groups — and copied
  // into every map block's LDS; persists while the candidates are reused.
  uint64_t* image;         // [MAP_SLOTS] signatures (0 = empty slot)
};
constexpr uint32_t HOT_LONG_MAX = 64;
constexpr int HOT_PARTS = 256;       // table partitions (one wc_hot_merge block each; a fingerprint's top byte)
#ifndef WC_HOT_STAGE_CAP
#define WC_HOT_STAGE_CAP 8
#endif
constexpr int HOT_STAGE_CAP = WC_HOT_STAGE_CAP;  // words per (partition, map block) cell; more are dropped (a heuristic)
constexpr int HOT_PART_TOP = 32;     // candidates kept per partition (the HOT_K words average 14)
// Map hot-table geometry: 2-choice groups of HOT_GROUP_SLOTS signatures.  Two
// slots per group (4 candidate compares and two 16-byte probe reads per token)
// holds 7/8 of the slots at the hit rate that 4-slot groups (8 compares, four
// reads) reach at 3/4 (profiles/r2_plumbing.md: greedy 2-choice placement
// simulated on Zipf(1.0)).
#ifndef WC_HOT_GS
#define WC_HOT_GS 2
#endif
constexpr int HOT_GROUP_SLOTS = WC_HOT_GS;
constexpr int HOT_GROUPS = MAP_SLOTS / HOT_GROUP_SLOTS;
static_assert(HOT_GROUP_SLOTS == 2 || HOT_GROUP_SLOTS == 4, "hot-table groups of 2 or 4 slots");
constexpr int HOT_SEL_BINS = 256;  // sampled-count histogram bins (counts clamp to the last: a partition holds < 1 word sampled 255+ times on Zipf(1.0) at 100k words)

// In-kernel phase stamps of the map (diagnostic build, WC_MAP_STAMPS=1): shares
// of wave lifetime per phase, then counters.
enum : int { MS_COMMIT = 0, MS_MASK, MS_LIST, MS_KEYS, MS_PROBE, MS_SLOW, MS_EMIT, MS_WAIT, MS_FLUSH, MS_TOTAL,
             MS_N_HIT, MS_N_DEFER, MS_N_DIRECT,
             MS_BLKSUM, MS_BLKMAX, MAP_STAMP_N };

struct ReduceArgs {
  Records rec;
  uint32_t map_blocks;  // grid of the map pass that wrote `rec`
  uint32_t log2_rec_buckets;
  TableView tab;
  const uint8_t* text;  // the same chunk, for copying new long words
  uint64_t avail_len;
  uint64_t chunk_base;  // global offset of text[0]
  Arena arena;
  uint32_t* flags;
  uint32_t* bucket_overflow;      // [n_buckets] set when a slice overflowed
  const uint8_t* bucket_enable;   // nullptr = all
  unsigned long long* stamps;     // [RED_STAMP_N] diagnostic counters (WC_RED_STAMPS builds), nullable
  // diagnostic (WC_RED_STAMPS builds, nullable): per reduce block RED_BLK_WORDS words
  // {bucket | quarter << 32, start, end (s_memrealtime), Rec16 | Rec records << 32 of its runs, LONG records}
  unsigned long long* blk;
  uint32_t* fo_hist;              // [FO_LOGBINS] += every stored key's fo_logbin(first, fo_m) (nullable)
  uint32_t fo_m;
  // The last pass before a bitmap-rank order (nullable): every stored key sets
  // its bit and its bucket's key count goes to the control word — the order
  // then skips its own bit-set launch (sort.hip bitmap_order, bits_set)
  unsigned long long* bm;
  uint32_t* bm_lines;  // per 512-bit line: keys set in it
  unsigned long long* bm_ctl;
  uint64_t bm_pos_end;
  uint32_t bm_shift;
  // Split reduce (nq > 1: fewer table buckets than CUs).  Block b + B q (q < nq)
  // merges the runs of map blocks p = q mod nq into a partial table of bucket b
  // (q = 0 starting from the running slice, the others empty) and writes its
  // occupied rows to part slot (b + B q); the last quarter of a bucket to finish
  // merges the other partials into its own table and stores the slice.
  uint32_t nq;
  // Dispatch plan (nullable: one block per bucket / the uniform split above):
  // the map's per-bucket weights (MapArgs::bucket_w; record buckets == table
  // buckets >= CUs, nq = 1).  Heavy buckets are split into quarters and the
  // pieces dispatched heaviest first (reduce.hip lpt_piece); a piece's partial
  // slot is its block index.
  const uint32_t* bucket_w;
  struct Parts {
    uint64_t *k0, *k1, *cnt, *first, *soff;  // [(b + B q) * TAB_SLOTS + i] rows
    uint32_t* slen;
    uint32_t* n;                              // [b + B q] rows written
    uint64_t* qsoff;                          // [(b + B q) * TAB_SLOTS + slot] arena references of quarters q > 0
    uint32_t* qslen;
    uint32_t* done;                           // [b] quarters arrived (zeroed; the last resets it)
  } part;
  uint32_t part_slots;  // partial-table slots allocated (the dispatch plan needs one per block)
  bool long_direct = false;  // the pass's map wrote LONG records top-down (MapArgs::long_direct)
};
// Most reduce blocks per bucket (split reduce: fewer table buckets than CUs).
constexpr uint32_t RED_SPLIT_MAX_Q = 16;
constexpr uint32_t RED_PLAN_EXTRA = 64;  // dispatch plan: blocks for split heavy buckets past one per bucket
// Reduce diagnostic counters (src/kernels/reduce.hip built with -DWC_RED_STAMPS=1).
constexpr int RED_BLK_WORDS = 9;  // bucket | q, start, end, n16 | n24, LONG, streams end, arrival, merged, stored
enum : int { RS_RECORDS = 0, RS_SLOW_LANES, RS_SLOW_WAVES, RS_PROBE_ITERS, RS_CAS_FAIL, RS_PENDING, RS_CLAIMS,
             RS_T_WAVE, RS_T_SLOW, RS_T_RUNS, RS_BLOCKS, RS_T_BLKMAX, RS_T_STREAMS, RS_NLONG, RS_LONG_STREAMED,
             RED_STAMP_N };

struct SynthVocab {
  const uint8_t* bytes;
  const uint32_t* off;
  const uint8_t* len;
  const uint32_t* cdf;  // cumulative P(rank <= i) scaled to 2^32
  uint32_t n;
};

// ---- launchers (all stream-ordered, no host sync) ----------------------------
// wc_hot_sample + wc_hot_merge + wc_map;
// sample = false: wc_map alone, on the hot-table image an earlier pass of the job built.
struct ZeroList;
// z: the pass's zeroing, applied before the map (inside the sampling launch when `sample`)
void launch_map(const MapArgs& a, const HotArgs& h, uint32_t map_blocks, hipStream_t s, bool sample,
                const ZeroList& z);
// diagnostic: phase clock of wc_hot_sample / wc_hot_merge into d (32 words, nullptr: off)
void hot_setup_stamps(unsigned long long* d);
// extra: with ReduceArgs::bucket_w, blocks past one per bucket for the dispatch
// plan's split heavy buckets (reduce.hip lpt_piece)
// Bounds guard on the finalize's row writers (profiles/r5_fault_hunt.md): a
// write at or past `cap` rows is skipped and the first one recorded in *err as
// (kernel id << 56 | row); the engine fails naming the kernel and the row at
// the finalize's wait (Engine::Impl::check_bounds) instead of faulting the GPU.
// err == nullptr: unchecked.
enum BoundsKernel : uint32_t {
  BND_NONE = 0,
  BND_FO_SORT,       // sort.hip wc_fo_sort: output rows
  BND_BM_PLACE,      // sort.hip wc_bm_place: record rows
  BND_BM_EMIT,       // sort.hip wc_bm_emit: output rows
  BND_GATHER_COLS,   // sort.hip wc_gather_cols: output rows and source rows
  BND_TABLE_KEYS,    // reduce.hip wc_table_keys: (first, slot) rows
  BND_GATHER_TABLE,  // reduce.hip wc_gather_table: output rows and table slots
  BND_COMPACT,       // reduce.hip wc_table_compact: output rows
  BND_KERNELS
};
struct Bounds {
  unsigned long long* err = nullptr;
  uint64_t cap = ~0ull;
};
const char* bounds_kernel_name(uint32_t k);

void launch_reduce(const ReduceArgs& a, hipStream_t s, uint32_t extra = 0);
void launch_table_split(const TableView& src, const TableView& dst, hipStream_t s);
void launch_table_clear(const TableView& t, hipStream_t s);
// debug: err (4 words, zeroed) <- the first bucket breaking the table's invariants (reduce.hip wc_check_table)
void launch_check_table(const TableView& t, unsigned long long* err, hipStream_t s);
// Writes occupied entries densely in bucket order; bucket_off[b] = exclusive
// prefix of the per-bucket occupancy (device array of 2^log2_buckets).
void launch_table_compact(const TableView& t, const uint64_t* bucket_off, uint64_t* k0, uint64_t* k1, uint64_t* cnt,
                          uint64_t* first, uint64_t* sref_off, uint32_t* sref_len, hipStream_t s,
                          const Bounds& bnd = {});

// LSD radix sort of (key, value) by the low `bits` bits of key; stable.
// tmp_* must hold n items; hist must hold radix_hist_words(n) words.  With
// in_tmp, an odd pass count leaves the result in tmp_* (*in_tmp = true)
// instead of copying it back.
// dn: the item count on the device; n is then an upper bound (buffers, hist
// stride) and n_hint the expected count (tile size, grid).
size_t radix_hist_words(uint64_t n, uint64_t n_hint = 0);
void radix_sort_pairs(uint64_t* keys, uint32_t* vals, uint64_t* tmp_keys, uint32_t* tmp_vals, uint32_t* hist,
                      uint64_t n, int bits, hipStream_t s, bool* in_tmp = nullptr, const uint64_t* dn = nullptr,
                      uint64_t n_hint = 0);
// Local finalize without the column copy: occupied slots -> (first offset,
// global slot index) pairs at host-computed bucket offsets; after the sort,
// the six output columns are gathered straight from the table.
void launch_table_keys(const TableView& t, const uint64_t* bucket_off, uint64_t* keys, uint32_t* slots, hipStream_t s,
                       const Bounds& bnd = {});
void launch_gather_table(const TableView& t, const uint64_t* keys, const uint32_t* slots, uint64_t n, uint64_t* ok0,
                         uint64_t* ok1, uint64_t* ocnt, uint64_t* ofirst, uint64_t* osoff, uint32_t* oslen,
                         hipStream_t s, const uint64_t* dn = nullptr, const Bounds& bnd = {});
// Exclusive scan of the bucket occupancy on the device: bucket_off[b] and the
// key count *n (the speculative finalize: no host round trip after the pass).
void launch_bucket_offsets(const uint32_t* occupancy, uint32_t nb, uint64_t* bucket_off, uint64_t* n, hipStream_t s);

// First-occurrence order (sort.hip: a three-launch sample sort of UNIQUE
// keys): rows ordered by first offset, the six output columns written straight
// from the source — the table's slots (`table`: the single-GPU finalize) or
// key columns (the merged table, n rows or *dn with n the bound).  `bound` >=
// the key count; keys < 2^key_bits set the log-bin resolution (a larger key is
// still ordered); ws = first_order_ws_bytes(src, bound) bytes; *nout (if
// given) = the key count.  Returns a device word that is nonzero after the stream if a bin
// overflowed: the output is then invalid and the caller redoes it with
// radix_sort_pairs (~1e-4 per call for hash-ordered sources).
struct OrderSrc {
  bool table;
  TableView t;
  const uint64_t *k0, *k1, *cnt, *first, *soff;
  const uint32_t* slen;
  uint64_t n;
  const uint64_t* dn;
};
struct OrderDst {
  uint64_t *k0, *k1, *cnt, *first, *soff;
  uint32_t* slen;
  Bounds bnd;  // the columns' row capacity (the bitmap order's record rows too)
};
#ifndef WC_FO_MAX_KEYS
#define WC_FO_MAX_KEYS 1600000
#endif
constexpr uint64_t FO_MAX_KEYS = WC_FO_MAX_KEYS;  // 512 / 2048 bins average <= 800 rows (one wave sorts up to 2048)
size_t first_order_ws_bytes(const OrderSrc& src, uint64_t bound);
void first_order_stamps(unsigned long long* d);  // debug: phase clocks of the three kernels (nullptr: off)
// key_hist (nullable): a histogram over fo_logbin(first, key_hist_m) of exactly
// the source's keys (the reducer builds one for the table): used when
// key_hist_m matches the resolution of key_bits, replacing the sample launch.
// Otherwise hist_ws (nullable: a zeroed FO_LOGBINS-word buffer, left zeroed)
// receives the exact histogram from a many-block launch; without either, a
// one-block sample (wc_fo_split) sets the bins.
// hist_ready_m (nonzero): hist_ws already holds that exact histogram at
// resolution hist_ready_m (the planned merge's regions -> columns launch builds
// it); used when it matches, and left zeroed as usual.
uint32_t* first_order(const OrderSrc& src, const OrderDst& dst, uint64_t bound, uint32_t key_bits, void* ws,
                      uint64_t* nout, hipStream_t s, const uint32_t* key_hist = nullptr, uint32_t key_hist_m = 0,
                      uint32_t* hist_ws = nullptr, uint32_t hist_ready_m = 0);

// First-occurrence order by ranks from a bitmap over first >> shift (sort.hip:
// five launches, no comparison sort; the engine uses it above 400k keys).
// Positions must be distinct (shift 1: two token starts are >= 2 bytes apart)
// and first < key_end.  bm: bitmap_order_words(key_end, shift) words, all zero
// on entry and left all zero (a control word follows the bitmap).  bound >= the
// key count (a column source: its row bound, *src.dn the count when set; a
// table source reads every slot).  ws: bitmap_order_ws_bytes(bound, ...).
// *nout (if given) = the key count.  Returns a device word that is nonzero
// after the stream if two keys shared a position or one lay beyond key_end:
// the output is then invalid (redo with radix_sort_pairs).
size_t bitmap_order_words(uint64_t key_end, uint32_t shift);
size_t bitmap_order_ws_bytes(uint64_t bound, uint64_t key_end, uint32_t shift);
// bits_set: the reduce already set every key's bit and added the key count
// (ReduceArgs::bm); bitmap_order_ctl: that control word's address.
uint32_t* bitmap_order(const OrderSrc& src, const OrderDst& dst, uint64_t bound, uint64_t key_end, uint32_t shift,
                       unsigned long long* bm, void* ws, uint64_t* nout, hipStream_t s, bool bits_set = false);
unsigned long long* bitmap_order_ctl(unsigned long long* bm, uint64_t key_end, uint32_t shift);
uint32_t* bitmap_order_linecnt(unsigned long long* bm, uint64_t key_end, uint32_t shift);  // per 512-bit line

// out[i] = in[perm[i]] for the six key-table columns (one launch).
void launch_gather_cols(const uint64_t* k0, const uint64_t* k1, const uint64_t* cnt, const uint64_t* first,
                        const uint64_t* soff, const uint32_t* slen, const uint32_t* perm, uint64_t* ok0, uint64_t* ok1,
                        uint64_t* ocnt, uint64_t* ofirst, uint64_t* osoff, uint32_t* oslen, uint64_t n, hipStream_t s,
                        const uint64_t* dn = nullptr, const Bounds& bnd = {});
void launch_iota_u32(uint32_t* v, uint64_t n, hipStream_t s);

// util.hip: fill several device regions (+ a few small copies, e.g. host words
// from page-locked memory into device buffers) / copy several small device
// regions into page-locked host memory, one launch each (sizes in 32-bit words).
// (18 fills: a pass's own <= 5 + a planned merge's <= 12, folded into the
// job's sampling launch — dist/merge.cpp merge_cols_planned)
constexpr int ZERO_MAX_REGIONS = 18, ZERO_MAX_COPIES = 4, PUB_MAX_REGIONS = 8;
[[noreturn]] void launch_list_overflow(const char* what);  // util.hip: fails the job (a caller bug)
struct ZeroList {
  uint32_t* ptr[ZERO_MAX_REGIONS];
  uint64_t words[ZERO_MAX_REGIONS];
  uint32_t val[ZERO_MAX_REGIONS];  // the 32-bit fill pattern (0: zeroing)
  int n;
  const uint32_t* csrc[ZERO_MAX_COPIES];  // small copies (device or page-locked host source)
  uint32_t* cdst[ZERO_MAX_COPIES];
  uint32_t cwords[ZERO_MAX_COPIES];
  int nc;
  void add(void* p, uint64_t bytes, uint32_t pattern = 0) {
    if (n >= ZERO_MAX_REGIONS) launch_list_overflow("ZeroList: more than ZERO_MAX_REGIONS fills");
    ptr[n] = static_cast<uint32_t*>(p);
    val[n] = pattern;
    words[n++] = bytes / 4;
  }
  void copy(void* dst, const void* src, uint64_t bytes) {
    if (nc >= ZERO_MAX_COPIES) launch_list_overflow("ZeroList: more than ZERO_MAX_COPIES copies");
    cdst[nc] = static_cast<uint32_t*>(dst);
    csrc[nc] = static_cast<const uint32_t*>(src);
    cwords[nc++] = (uint32_t)(bytes / 4);
  }
  void append_fills(const ZeroList& o) {
    for (int i = 0; i < o.n; ++i) add(o.ptr[i], o.words[i] * 4, o.val[i]);
  }
};
// the same fills (regions, sizes, patterns, in order) and no copies in either
inline bool same_fills(const ZeroList& a, const ZeroList& b) {
  if (a.n != b.n || a.nc != 0 || b.nc != 0) return false;
  for (int i = 0; i < a.n; ++i)
    if (a.ptr[i] != b.ptr[i] || a.words[i] != b.words[i] || a.val[i] != b.val[i]) return false;
  return true;
}
struct PubList {
  const uint32_t* src[PUB_MAX_REGIONS];
  uint32_t* dst[PUB_MAX_REGIONS];
  uint32_t words[PUB_MAX_REGIONS];
  int n;
  uint32_t* seq_dst;  // nullable: written last (system-scope release) with seq, for a host spin-wait
  uint32_t seq;
  void add(void* host_dst, const void* dev_src, uint64_t bytes) {
    if (n >= PUB_MAX_REGIONS) launch_list_overflow("PubList: more than PUB_MAX_REGIONS regions");
    dst[n] = static_cast<uint32_t*>(host_dst);
    src[n] = static_cast<const uint32_t*>(dev_src);
    words[n++] = (uint32_t)(bytes / 4);
  }
};
void launch_zero_regions(const ZeroList& z, hipStream_t s);
void launch_publish(const PubList& c, hipStream_t s);

void launch_synth(uint8_t* out, uint64_t n, uint64_t first_segment, uint64_t seed, const SynthVocab& v,
                  hipStream_t s);

// Merge-protocol helpers (dist/merge.cpp).
// Dense scatter: dst_cnt[id[i]] += cnt[i] (ids unique per rank, so plain stores), dst_first min.
void launch_fill_u64(uint64_t* p, uint64_t v, uint64_t n, hipStream_t s);
// merge.hip
// ---- shuffle / dense merge (src/kernels/merge.hip) ----
struct MRow {  // one key row on the wire (40 B)
  uint64_t k0, k1, cnt, first;
  uint32_t aoff, alen;  // long word: bytes [aoff, aoff + alen) of the accompanying byte payload
};
static_assert(sizeof(MRow) == 40, "MRow layout");
constexpr uint32_t MERGE_MAX_RANKS = 64;
// Shuffle merge: below this many rows in total every rank sends straight to
// rank 0, which merges alone.  Rank 0 then inserts all W x V rows instead of
// V / W x W; the owner path costs one more exchange + host sync (~50 us at one
// rank, tools/merge_cost.py) — the insert + compact of ~2.5e5 rows.
constexpr uint64_t MERGE_ROOT_MAX_ROWS = 1ull << 18;
// counts of rows [0, n) — or [0, *dn) with n a bound — (pass_flags) the pass's recovery flags at 2W + 1,
// and the row count itself (+ count_bias, a fault-injection switch) at 2W + 2
void launch_owner_count(const uint64_t* k0, const uint64_t* k1, const uint32_t* slen, uint64_t n, const uint64_t* dn,
                        const uint32_t* pass_flags, uint32_t W, unsigned long long* counts, hipStream_t s,
                        uint32_t count_bias = 0);
// send_pos (nullable): row index of each local key; dn: device-side row count
// (n the bound); reg_rows > 0: planned mode — owner o's rows / bytes in fixed
// regions of reg_rows rows / reg_bytes bytes (counts unused), overflow -> *ovf
// bit 2, and pass_flags (nullable) -> *ovf bits 0 / 1 (rerun / arena overflow)
struct MergeSelf {
  uint32_t rank;
  MRow* rows;      // the receive row buffer
  uint8_t* bytes;  // the receive byte buffer
  // planned-merge words the scatter's block 0 writes (nullable): region bases
  // per source (rows p * reg_rows | bytes p * reg_bytes, p <= W), send-row
  // starts per owner, and this rank's max first offset into quad[2]
  uint64_t* base;
  uint64_t* seg;
  unsigned long long* quad;
  uint64_t max_end;
};
void launch_owner_scatter(const uint64_t* k0, const uint64_t* k1, const uint64_t* cnt, const uint64_t* first,
                          const uint64_t* soff, const uint32_t* slen, const uint8_t* arena, uint64_t n, uint32_t W,
                          const unsigned long long* counts, unsigned long long* cursor, MRow* rows, uint8_t* bytes,
                          uint32_t* send_pos, hipStream_t s, const uint64_t* dn = nullptr, uint64_t reg_rows = 0,
                          uint64_t reg_bytes = 0, uint32_t* ovf = nullptr, const uint32_t* pass_flags = nullptr,
                          const uint32_t* occ = nullptr, unsigned long long* nvalid = nullptr,
                          const MergeSelf* self = nullptr);
// occ (nullable): the columns are the running table's (n = its capacity): slot
// i is a row iff occ[i >> TAB_SLOTS_LOG2] != 0 and k1[i] != K1_EMPTY (an empty
// slot's send_pos is all ones); nvalid (nullable, zeroed) += the rows seen.
// self (nullable, planned mode): this rank's own rows and bytes go straight to
// its receive regions (same offsets as in the send layout) — nothing to send
// to itself in the exchange.
// Planned merge: the decision flags from every rank's gathered word quad
// (merged rows, flags, max first offset, -) (merge.hip).
void launch_merge_check(const unsigned long long* owns, uint32_t W, uint64_t reg_merged, uint64_t max_end,
                        uint32_t* flags, hipStream_t s);
// check_flags (nullable): wc_merge_check folded in (max_end its bound); hist
// (nullable, zeroed): += fo_logbin(first, hist_m) of every row written.
void launch_mrow_regions_to_cols(const MRow* rows, uint32_t W, uint64_t reg_merged, const unsigned long long* owns,
                                 uint64_t byte_stride, const uint64_t* dcnt, const uint64_t* dfirst, uint64_t* k0,
                                 uint64_t* k1, uint64_t* cnt, uint64_t* first, uint64_t* soff, uint32_t* slen,
                                 unsigned long long* out_n, hipStream_t s, uint32_t* check_flags = nullptr,
                                 uint64_t max_end = 0, uint32_t* hist = nullptr, uint32_t hist_m = 0);
void launch_mrow_insert(const MRow* rows, uint64_t R, const uint8_t* bytes, const uint64_t* rbase,
                        const uint64_t* bbase, uint32_t W, uint32_t* state, unsigned long long* cnt,
                        unsigned long long* first, uint64_t T, uint32_t* row_slot, hipStream_t s);  // row_slot nullable
void launch_mrow_compact(const MRow* rows, const uint32_t* state, const unsigned long long* cnt,
                         const unsigned long long* first, uint64_t T, const uint64_t* rbase, const uint64_t* bbase,
                         uint32_t W, MRow* out, unsigned long long* out_n, uint32_t* slot_id, hipStream_t s,
                         uint64_t out_cap = ~0ull);  // slot_id nullable; rows past out_cap are counted, not written
// Planned merge, owner side: insert + emit of the merged rows in one launch
// (no compaction).  `out` rows [0, cap) must read count 0 / first word 0 (the
// first offset is stored inverted: atomicMax of ~first); rows past cap are
// counted in *out_n, not written.  ids (dense, nullable): each received row's
// owner-local id (rows of region `self` of `reg` rows -> ids_self).
void launch_mrow_insert_emit(const MRow* rows, uint64_t R, const uint8_t* bytes, const uint64_t* rbase,
                             const uint64_t* bbase, uint32_t W, uint32_t* state, uint32_t* slot_idx, uint64_t T,
                             MRow* out, unsigned long long* out_n, uint64_t cap, uint32_t* ids, uint32_t* ids_self,
                             uint32_t self, uint64_t reg, hipStream_t s);
void launch_mrow_to_cols(const MRow* rows, uint64_t n, const uint64_t* rbase, const uint64_t* bbase, uint32_t W,
                         uint64_t* k0, uint64_t* k1, uint64_t* cnt, uint64_t* first, uint64_t* soff, uint32_t* slen,
                         hipStream_t s, const uint64_t* dn = nullptr);  // dn: device-side row count (n a bound)
void launch_row_ids(const uint32_t* row_slot, const uint32_t* slot_id, uint64_t R, const unsigned long long* owns,
                    uint32_t rank, uint32_t* ids, hipStream_t s,  // owns: all-gathered (rows, bytes) per owner
                    uint32_t* ids_self = nullptr, uint32_t self = 0, uint64_t reg = 0);  // rows of region self -> ids_self
void launch_scatter_ids(const uint32_t* send_pos, const uint32_t* ids_back, const uint64_t* seg,
                        const unsigned long long* owns, uint32_t W, const uint64_t* cnt, const uint64_t* first,
                        uint64_t n, uint64_t* dcnt, uint64_t* dfirst, hipStream_t s, const uint64_t* dn = nullptr,
                        uint64_t pad = 0);  // ids_back: owner-local; pad > 0: padded ids (owner base o * pad)

// ---- stream-ordered loopback communicator (src/kernels/comm.hip, dist/comm.cpp) ----
constexpr int LB_MAX_RANKS = 64, LB_RING = 16, LB_XFER_PARTS = 64;
enum : uint32_t { LB_ALLGATHER = 0, LB_ALLTOALLV = 1, LB_BROADCAST = 2, LB_REDUCE_SCATTER = 3 };
struct LbMeta {  // one rank's buffers for one collective (page-locked; read by the peers' transfer kernels)
  uint64_t send, recv;
  uint64_t soff[LB_MAX_RANKS];    // alltoallv: where this rank's bytes for rank q start in `send`
  uint64_t roff[LB_MAX_RANKS];    // alltoallv: where rank q's bytes land in `recv`
  uint64_t rbytes[LB_MAX_RANKS];  // alltoallv: bytes received from rank q
};
struct LbShared {  // page-locked, shared by the ranks of one loopback group
  uint32_t aborted;                     // a rank failed: queued transfers skip their copies
  LbMeta meta[LB_RING * LB_MAX_RANKS];  // [slot * world + rank]
};
struct LbXfer {
  const LbShared* shared;
  uint32_t kind, world, rank, slot, op, root;
  uint64_t count;  // allgather / broadcast: bytes per rank; reduce-scatter: u64 elements per rank
};
void launch_loopback_xfer(const LbXfer& x, hipStream_t s);

}  // namespace wc
