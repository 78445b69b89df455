// engine_impl.hpp — private state of wc::Engine (shared with dist/merge.cpp).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <map>
#include <memory>
#include <vector>

#include "../common/hip_util.hpp"
#include "../io/numa.hpp"
#include "../io/synth_host.hpp"
#include "../kernels/kernels.hpp"
#include "../kernels/keys.hpp"
#include "wc/wc.hpp"

namespace wc {

// Device counters block, zeroed per map/reduce pass.
struct DevCounters {
  uint32_t flags[FLAG_COUNT];
  unsigned long long tokens;
  unsigned long long records;
  unsigned long long long_tokens;  // LONG-word tokens of the pass (MapArgs::long_tokens)
};

// Running table storage (own allocation: it grows by splitting).
struct TableStore {
  void* mem = nullptr;
  TableView v{};
  ~TableStore();
  void alloc(uint32_t log2_buckets);
  size_t slots() const { return ((size_t)1 << v.log2_buckets) * TAB_SLOTS; }
};

// Dense key columns (compact output, merge input/output).
struct KeyCols {
  uint64_t *k0 = nullptr, *k1 = nullptr, *cnt = nullptr, *first = nullptr, *sref_off = nullptr;
  uint32_t* sref_len = nullptr;
  uint64_t n = 0;
  // non-null: the row count lives on the device (n is its bound) until the
  // finalize's last wait publishes it (the merge's rank-0 gather: no host round trip)
  unsigned long long* dn = nullptr;
  // non-null: the columns ARE the running table (the planned merge scatters
  // straight from it): row i is a slot, valid iff occ[i >> TAB_SLOTS_LOG2] != 0
  // and k1[i] != K1_EMPTY; n = the table's capacity
  const uint32_t* occ = nullptr;
};

struct Engine::Impl {
  Options opt;
  Stats st;
  int dev = 0;
  hipStream_t s = nullptr, copy_s = nullptr;
  uint32_t map_blocks = 0;
  bool sync_debug = false;  // WC_SYNC_DEBUG: sync + log after every kernel
  uint64_t k1_mask = K1_HASH_MASK;  // Options::k1_hash_bits (collision tests)
  unsigned long long* d_stamps = nullptr;  // WC_MAP_STAMPS: map phase clock sums
  unsigned long long* d_blk = nullptr;     // WC_MAP_STAMPS: per-block timing of the last map pass
  unsigned long long* d_red_stamps = nullptr;  // WC_MAP_STAMPS: reduce counters (WC_RED_STAMPS builds)
  unsigned long long* d_hot_stamps = nullptr;  // WC_MAP_STAMPS: setup kernels' phase clock (hot_setup_stamps)
  unsigned long long* d_red_blk = nullptr;     // WC_MAP_STAMPS: per reduce block profile (RED_BLK_WORDS each)
  size_t red_blk_n = 0;
  // the profile buffer when the next reduce grid fits it (its last launch's blocks are printed at teardown)
  unsigned long long* red_blk() {
    if (!d_red_blk || ((size_t)table().log2_buckets >= 63)) return nullptr;
    const size_t grid = ((size_t)1 << table().log2_buckets) * red_q();
    if (grid > red_blk_n) return nullptr;
    red_blk_grid = grid;
    return d_red_blk;
  }
  size_t red_blk_grid = 0;
  uint32_t fin_seq = 0;
  bool red_plan = true;
  // LONG-word records top-down + streamed by the reduce (MapArgs::long_direct):
  // chosen per pass from the LONG share of the pass before (LONG tokens > 1/64
  // of its records; the first pass of an engine: off); both modes are exact for any
  // text — the instances without the LONG stream run the LONG-free headline
  // text ~1 % faster (profiles/r5_session.md §5).  WC_LONG_DIRECT=0|1 forces.
  bool long_direct = false;
  int long_direct_force = -1;
  bool pass_ld = false;  // the mode of the pass in flight (its map, its reduce and any re-run of it)
  // WC_CHECK_TABLE=1 (debug): after every reduce and split the table's
  // invariants are checked on the device and a violation fails the job naming
  // the stage (engine.cpp check_table)
  unsigned long long* d_tab_err = nullptr;
  // the finalize writers' bounds guard (kernels.hpp Bounds): one word, zero
  // unless a writer met a row past its buffer; checked at every finalize
  unsigned long long* d_bounds = nullptr;
  uint64_t fault_occ_under = 0;  // WC_FAULT_OCC_UNDER (tests): host key count short by this many
  Bounds bounds(uint64_t cap) const { return Bounds{d_bounds, cap}; }
  void check_bounds(uint64_t word, const char* where);
  void check_table(const char* where);             // the balanced reduce (WC_RED_PLAN=0: the uniform split)
  uint32_t* d_bucket_w = nullptr;   // its per-bucket weights (the map adds them)  // sequence word of the merged finalize's last publish (h_fin + 32)
  uint64_t blocks_stamped = 0;             // map blocks launched with stamps (block-duration mean)

  // shuffle records
  uint64_t rec_total = 0;
  Records rec{};       // full-capacity views
  Records pass_rec{};  // views of the current map/reduce pass
  DeviceArena rec_mem;

  // counters + pinned mirror
  DevCounters* d_ctr = nullptr;
  DevCounters* h_ctr = nullptr;

  TableStore tab[2];
  int cur = 0;
  uint32_t* d_bucket_ovf = nullptr;
  uint8_t* d_bucket_en = nullptr;
  // hot-key sampling workspace of the map (HotArgs)
  DeviceArena hot_mem;
  HotArgs hot{};
  // Hot-table reuse inside a job (never across jobs: reset() drops it): a pass
  // keeps the image its job's last sampling pass built while its miss share
  // (records / tokens) stays within hot_resample_slack of that pass's, and
  // samples again every hot_resample_every passes (WC_HOT_RESAMPLE_EVERY, 0 =
  // sample every pass).
  bool hot_valid = false;
  double hot_miss_ref = 0, hot_miss_last = 0;
  uint32_t hot_age = 0, hot_resample_every = 16;
  double hot_resample_slack = 1.15;
  bool pass_sampled = false;  // the pass in flight built its own image

  // key arena (bytes of LONG words, >= 16 bytes)
  uint8_t* d_arena = nullptr;
  unsigned long long* d_arena_cursor = nullptr;

  // resident text (synth_device) and, separately, the streaming staging pair
  DeviceArena text_mem;
  uint8_t* d_text = nullptr;
  uint64_t text_cap = 0;
  DeviceArena stage_mem;
  DeviceArena giant_mem;  // a word longer than a stream piece, counted as its own pass
  uint64_t stage_cap = 0;
  uint8_t* d_stage[2] = {nullptr, nullptr};
  std::vector<PinnedBuffer> pinned;
  const uint8_t* registered = nullptr;  // caller pool page-locked by count_pinned_replay
  hipEvent_t ev_h2d[2] = {}, ev_done[2] = {};

  // synthetic vocabulary on device
  uint64_t vocab_key = ~0ull;
  DeviceArena vocab_mem;
  SynthVocab d_vocab{};

  // finalisation workspace
  DeviceArena fin_mem;   // compact output
  PinnedBuffer h_boff;   // per-bucket compaction offsets (H2D without a sync)
  PinnedBuffer h_occ;    // bucket occupancy + key-arena cursor, copied with every pass's counters
  bool occ_valid = false;  // h_occ matches the table (no split / clear since the last pass)
  bool occ_copied = false;  // the current pass enqueued its occupancy copy
  DeviceArena merge_mem; // merge buffers (merged columns live here)
  DeviceArena merge_small;  // merge metadata (count matrices)
  PinnedBuffer h_merge;     // merge host words for async H2D copies (no sync before they go out of scope)
  PinnedBuffer h_plan;      // speculative merge: gathered owner-count matrix + key count + sequence word
  PinnedBuffer h_fin;       // the merged key count (KeyCols::dn) published before the finalize's last wait
  uint32_t plan_seq = 0;
  DeviceArena sort_mem;  // first-occurrence sort + sorted columns
  KeyCols cols;        // local (compact) or merged, sorted by first after finalize
  uint8_t* cols_arena = nullptr;   // arena the sref_* of cols point into
  uint64_t cols_arena_bytes = 0;
  uint64_t max_end = 0;  // max global byte offset seen (sort key width)
  uint32_t* d_fo_hist = nullptr;  // [FO_LOGBINS] log-bin histogram of the table's first offsets (each reduce)
  uint32_t fo_hist_m = 0;         // its resolution (fo_mbits of the pass's key width)
  bool fo_hist_ok = false;        // it describes the current table (a pass ran since the reset)
  uint32_t* d_fo_hist_cols = nullptr;  // [FO_LOGBINS] zeroed: exact histogram of merged columns (first_order)
  uint32_t cols_hist_m = 0;  // nonzero: the planned merge filled d_fo_hist_cols for cols at this resolution
  uint32_t key_bits() const {  // first offsets are < max_end < 2^key_bits
    uint32_t b = 1;
    while (b < 64 && (max_end >> b) != 0) ++b;
    return b;
  }

  explicit Impl(const Options& o);
  ~Impl();

  TableView& table() { return tab[cur].v; }
  void ensure_text(uint64_t n);
  void ensure_staging(uint64_t chunk);

  // One chunk: map + reduce with overflow recovery (synchronous).  With
  // `last`, the pass is only launched and left PENDING: a local finalize runs
  // behind it speculatively and checks its counters at its own single sync;
  // anything else first settles it (complete_pass).
  void process_chunk(const uint8_t* text, uint64_t len, uint64_t avail, uint64_t base, int prev, bool last = false);
  // Asynchronous part (map + reduce + counters D2H) and the completion check;
  // complete_pass returns false when the pass needed recovery (re-runs / splits).
  void launch_pass(const uint8_t* text, uint64_t len, uint64_t avail, uint64_t base, int prev, uint32_t log2_rb,
                   uint32_t blocks, bool copy_occupancy = true, bool defer_publish = false);
  // The pass's counter publish (pinned copies of counters + occupancy), held
  // back by a speculative last pass: the local finalize folds it into its own
  // publish launch (one launch, ~4.5 us, fewer per job); anything else that
  // takes the pending pass launches it first (flush_pass_publish).
  PubList pass_pub{};
  bool pass_pub_pending = false;
  void flush_pass_publish();
  bool complete_pass(const uint8_t* text, uint64_t len, uint64_t avail, uint64_t base, int prev, uint32_t log2_rb,
                     uint32_t blocks, bool synced = false);  // synced: the stream has drained (publish waited)
  struct PendingPass {
    bool active = false;
    const uint8_t* text = nullptr;
    uint64_t len = 0, avail = 0, base = 0;
    int prev = -1;
    uint32_t rb = 0, blocks = 0;
  } pend;
  // Planned merge (dist/merge.cpp merge_cols_planned): fixed exchange regions
  // learned from the last exact merge of the same shape — identical on every
  // rank, since they come from all-gathered counts — so the merged finalize
  // needs no host round trip; its decision flags arrive with the last wait.
  struct MergeCaps {
    bool valid = false;
    int world = 0;
    uint32_t mode = 0;
    uint64_t rows = 0, bytes = 0, merged = 0;  // per (rank -> owner) region / per owner in the gather
    uint64_t gmax_end = 0;                     // the sort key width of the last exact merge
  } merge_caps;
  // WC_HOST_CLOCK=1 (diagnostics): host time between a job's milestones
  // (each credited with the time since the previous milestone), summed over
  // jobs and printed at teardown — where the GPU's idle gap between jobs goes
  enum { HC_START, HC_RESET, HC_PRELAUNCH, HC_MAPPED, HC_WAIT, HC_WAITED, HC_DONE, HC_N };
  bool host_clock = false;
  double hc_prev = 0, hc_sum[HC_N] = {};
  uint64_t hc_jobs = 0;
  void hc_mark(int i);
  // The last planned merge's zeroing list: the next job's last pass applies it
  // inside its sampling launch (merge_zero_pre), and the planned merge skips
  // its own zeroing launch when its list is the same (one launch fewer per job)
  ZeroList merge_zero_last{};
  bool merge_zero_last_valid = false;
  bool merge_zero_pre = false;
  uint64_t merge_zero_gen = 0;  // the arenas' generations the list points into (a reallocation voids it)
  uint64_t merge_arena_gen() const {
    return merge_mem.generation() * 0x9E3779B97F4A7C15ull ^ merge_small.generation() * 0xC2B2AE3D27D4EB4Full ^
           fin_mem.generation();
  }
  bool planned_active = false;      // a planned merge is in flight: check its flags after the last wait
  PendingPass planned_pass;         // the pass it ran behind (completed after the last wait)
  uint32_t* d_merge_flags = nullptr;  // device word of the planned merge's flags (merge_small)
  uint64_t* d_local_n = nullptr;      // the planned merge's local key count (device, published at the end)
  // Engine::reset() only marks the table empty; the next pass's zeroing kernel
  // (or apply_reset, before anything else reads the table) clears it.
  bool reset_pending = false;
  bool copy_used = false;  // copy_s carried H2D copies since the last reset
  void apply_reset();
  bool speculate = true;  // WC_NO_SPECULATE=1: every pass synchronous
  uint64_t last_keys = 0;  // keys of the previous finalize (sort size hint)
  PinnedBuffer h_spec;     // speculative finalize: key count + arena cursor + publish sequence word
  bool spin_wait = true;   // WC_SPIN_WAIT=0: wait for the finalize with a stream sync instead
  uint32_t spec_seq = 0;
  PinnedBuffer h_pass_seq;  // sequence word of the last pass's publish launch
  uint32_t pass_seq = 0;
  void wait_published(const uint32_t* seq, uint32_t want);
  void settle();           // complete a pending pass
  // Stage events (device time per stage of the last job, Stats::map_ms ...):
  // mark(tag) records an event on s; the interval from the previous mark to
  // this one is charged to the stage `tag` closes.
  enum : int { EV_PASS = 0, EV_MAP, EV_REDUCE, EV_FIN, EV_MERGE0, EV_MERGE1, EV_FIN_END };
  bool stage_events = true;
  std::vector<hipEvent_t> ev_pool;
  std::vector<int> ev_tag;
  size_t ev_n = 0;
  bool fin_end_marked = false;
  void mark(int tag);
  void collect_stage_times();
  uint32_t blocks_for(uint64_t len) const;
  // Shuffle partitions track the running table (one reduce block reads only
  // its own partition) up to MAX_REC_BUCKETS.
  uint32_t rec_shift = 0;  // WC_REC_SHIFT (sweeps only): shuffle partitions = table buckets >> shift
  uint32_t n_cu = 0;         // compute units: reduce blocks per pass
  NumaNode numa;             // the GPU's host NUMA node: pinned staging + reader threads bound there
  uint32_t red_q_force = 0;  // WC_RED_Q (sweeps only): reduce blocks per bucket
  uint32_t part_blocks = 0;  // split-reduce partial tables allocated
  ReduceArgs::Parts part{};
  DeviceArena part_mem;
  // reduce blocks per table bucket: the split reduce fills the CUs when the
  // table has fewer buckets than CUs
  uint32_t red_q() {
    const uint32_t B = 1u << table().log2_buckets;
    uint32_t q = red_q_force ? red_q_force : std::max<uint32_t>(1, n_cu / B);
    q = std::min<uint32_t>(q, RED_SPLIT_MAX_Q);
    while (q > 1 && (uint64_t)q * B > part_blocks) --q;
    return q;
  }
  uint32_t rec_buckets_log2() {
    const uint32_t tb = table().log2_buckets;
    return std::min<uint32_t>(std::max(opt.log2_rec_buckets, tb) - std::min(rec_shift, tb), MAX_REC_BUCKETS_LOG2);
  }
  void split_table();

  uint64_t finalize(Comm* comm, bool all_ranks);  // compact [+ merge] + order by first
  void enqueue_occupancy();                 // async D2H of occupancy + arena cursor into h_occ
  void add_occupancy(PubList& c);           // the same as regions of a publish launch
  uint64_t host_occupancy(uint64_t*& boff, uint64_t& arena_used);  // h_occ (sync only if stale) -> offsets, n
  void compact_local();                     // table -> cols (unsorted)
  void finalize_local_sorted();             // table -> cols ordered by first (no merge: no column copy)
  bool finalize_local_speculative();        // same behind a pending pass; false: redo after its recovery
  void sort_cols_by_first(bool radix = false);  // cols ordered by first occurrence
  // First-occurrence order: the three-launch sample sort (first_order) up to
  // FO_MAX_KEYS keys, the onesweep radix sort above it, after a sample-sort
  // overflow, or always with WC_FIRST_ORDER=radix.
  bool order_radix = false;
  // The sample sort up to 400k keys; above, the radix sort: the 2048-bin sample
  // sort (first_order handles up to FO_MAX_KEYS) measured no faster at 1M keys
  // — fo_bin 73 + fo_sort 138 us vs 200 us of radix passes + gather
  // (profiles/r4_session3.md §7)
  bool sample_order(uint64_t bound) const { return !order_radix && !order_bitmap && bound <= 400000; }
  // Above it the bitmap ranks (bitmap_order: first >> 1 positions, a 64 MiB
  // bitmap per GiB of text) while the bitmap stays within 128 bytes per key;
  // WC_FIRST_ORDER=bitmap takes it at every size.
  bool order_bitmap = false;
  bool bitmap_order_ok(uint64_t bound) const {
    return !order_radix && (order_bitmap || (bound > 400000 && (max_end >> 4) <= 128 * bound));
  }
  unsigned long long* d_bm = nullptr;  // bitmap_order's bitmap: all zero between calls
  size_t bm_words = 0;
  unsigned long long* ensure_bitmap();  // sized for max_end
  // The pending last pass's reduce set the bitmap's bits (ReduceArgs::bm): the
  // speculative finalize's bitmap order consumes them; any other path clears them.
  bool bm_in_reduce = false;
  void drop_reduce_bits();
  uint64_t spec_hint();  // the speculative finalize's key-count hint (sizes its order)
  uint32_t* fo_ovf = nullptr;  // overflow word of the sample sort sort_cols_by_first left in flight
  KeyCols cols_unsorted;       // its input, kept for a radix redo
  bool order_redo = false;     // the speculative finalize's sample sort overflowed (Stats::order_path 4)
  KeyTable download_cols();
};

// Multi-rank merge (dist/merge.cpp): replaces im.cols / cols_arena with the
// merged global table — on rank 0, or on every rank if all_ranks (the dense
// protocol always leaves it on every rank).
void merge_cols(Engine::Impl& im, Comm& comm, bool all_ranks);
// The same behind a pending last pass (compaction + owner plan without a
// settle, one host wait); false: some rank's pass needs recovery — the caller
// settles, compacts and runs merge_cols (every rank takes the same branch).
bool merge_cols_speculative(Engine::Impl& im, Comm& comm, bool all_ranks);
// The planned merge behind the pending pass (no host round trip; needs
// MergeCaps of this shape): false = not applicable, nothing enqueued.
bool merge_cols_planned_speculative(Engine::Impl& im, Comm& comm, bool all_ranks);

}  // namespace wc
