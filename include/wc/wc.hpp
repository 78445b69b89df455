// wc.hpp — public C++ API of the MI355X-native MapReduce word-count engine.
//
// Capability parity with the reference (/root/reference/main.cu): count
// whitespace-delimited words of a text and report `word<TAB>count` in
// first-occurrence order plus the total (main.cu:208-218).  Semantics are the
// reference's on its safe envelope, without its limits.
#pragma once
#include <stdint.h>

#include <memory>
#include <string>
#include <vector>

namespace wc {

// Final result: one row per distinct word, ordered by first occurrence.
struct KeyTable {
  std::vector<std::string> words;
  std::vector<uint64_t> counts;
  std::vector<uint64_t> first_off;  // global byte offset of the first occurrence
  uint64_t total = 0;               // sum of counts == number of tokens
  size_t size() const { return words.size(); }
};

struct Stats {
  uint64_t bytes = 0;     // text bytes ingested
  uint64_t tokens = 0;    // words counted (device counter)
  uint64_t keys = 0;      // distinct words (local, before merge)
  uint64_t records = 0;   // shuffle records after the LDS combiner
  uint64_t long_tokens = 0;   // LONG-word (>= 16-byte, hashed-key) tokens
  uint32_t long_direct = 0;   // the last pass wrote LONG records top-down (Engine::Impl::long_direct)
  uint32_t chunks = 0;    // map/reduce chunk passes
  uint32_t map_reruns = 0;     // shuffle-region overflow -> chunk halved
  uint32_t table_splits = 0;   // running table grew B -> 2B
  uint32_t log2_buckets = 0;   // final table buckets
  // first-occurrence order of the last finalize: 1 = sample sort, 2 = radix
  // sort, 3 = sample sort overflowed and redone by the radix sort, 4 = the
  // speculative finalize's sample sort (sized by the previous job) overflowed
  // and the exact-count one did not, 5 = bitmap ranks (above 400k keys),
  // 6 = the bitmap saw a shared position and the radix sort redid the order
  uint32_t order_path = 0;
  // cross-GPU merges of the engine's life run planned (fixed exchange regions,
  // no host round trip) / redone exactly after a planned one overflowed
  uint32_t merges_planned = 0, merge_redos = 0;
  // Wire traffic of the last merge, this rank's side (what a W-GPU xGMI run
  // would move; profiles/r5_merge_rank_cost.md): collectives issued, bytes sent
  // to peers in all of them, and the sum over collectives of the largest
  // amount sent to ONE peer (each peer pair has its own xGMI link, so that is
  // the link-bound part of a point-to-point exchange); bytes received by rank 0
  // in the gather.
  uint32_t merge_collectives = 0;
  uint64_t merge_sent_bytes = 0, merge_peer_bytes = 0, merge_root_recv_bytes = 0;
  // Host wall clock of the last job's API calls (count_*, finalize / result).
  double host_count_ms = 0, host_finalize_ms = 0;
  // Device time of the last job's stages, from events on the engine stream
  // (WC_STAGE_EVENTS=0 turns them off): map = zeroing + hot-word sampling +
  // wc_map of every pass; reduce = wc_reduce_buckets + counter publish;
  // finalize = compaction, first-occurrence sort, gather; merge = the
  // cross-GPU protocol (kernels + RCCL); idle = stream gaps between them (host
  // turn-arounds, H2D waits).  device_ms = their sum: first pass start to
  // finalize end.
  double map_ms = 0, reduce_ms = 0, finalize_ms = 0, merge_ms = 0, idle_ms = 0, device_ms = 0;
};

struct Options {
  int device = 0;
  uint64_t chunk_bytes = 1ull << 30;   // device chunk (<= 4 GiB: records carry u32 offsets)
  // 64 buckets to start: the map appends each record to its bucket's run, and
  // fewer runs keep their line tails in L2 (256 -> 64 buckets: wc_map -18 % at
  // 100k words); the reduce then runs several blocks per bucket (split reduce).
  uint32_t log2_rec_buckets = 6;       // shuffle partitions
  uint32_t log2_tab_buckets = 6;       // initial running-table buckets (x4096 slots)
  uint32_t max_log2_tab_buckets = 16;
  uint64_t min_records = 1ull << 21;   // floor of shuffle record capacity per chunk
  double records_per_byte = 0.25;      // shuffle record capacity per chunk byte
  uint64_t arena_bytes = 256ull << 20; // key arena for >8-byte words
  uint32_t map_blocks = 0;             // 0 = 2 per CU
  // pinned host ring depth (host-staged path): 2 suffices — piece k + 2 is
  // read into piece k's buffer only after pass k (which waited for its H2D)
  // completed — and each buffer costs ~15 ms of pinning per 64 MiB at start-up
  uint32_t staging_buffers = 2;
  // Streaming sources (files, host buffers) move through the pinned ring in
  // pieces of min(chunk_bytes, stream_chunk_bytes): small pieces start the
  // pipeline sooner and keep the page-locked ring cheap to allocate (4 GiB
  // file, whole CLI: 3.5 GB/s at 1 GiB pieces, 11 GB/s at 64 MiB).
  uint64_t stream_chunk_bytes = 64ull << 20;
  // Cross-GPU merge: 0 = shuffle (all-to-all of each key to its hash owner, owner-side
  // merge, gather to rank 0); 1 = dense (dictionary union on every rank, reduce-scatter of
  // dense count vectors + all-gather).
  uint32_t merge_mode = 0;
  // Tests only: keep this many bits of the LONG-word (>= 16 bytes) tail hash
  // (0 = all 62) to force key collisions; equality stays exact (bytes compared).
  uint32_t k1_hash_bits = 0;
};

// Synthetic text spec (see src/kernels/synth.hpp).
struct SynthSpec {
  uint64_t seed = 1;
  uint32_t vocab = 100000;
  double zipf_s = 1.0;
  // Share of the vocabulary drawn as LONG words of 16..64 bytes (hashed keys,
  // byte-compared downstream); 0 = the English-like length profile only.
  double long_frac = 0.0;
};

// Supplies host text chunks for the streaming (host-staged) path.
class ChunkSource {
 public:
  virtual ~ChunkSource() = default;
  // Fill up to `cap` bytes; return bytes written (0 = end).  The engine cuts
  // chunks at the last delimiter and carries the remainder forward.
  virtual uint64_t read(uint8_t* dst, uint64_t cap) = 0;
};

class Comm;  // dist/comm.hpp

class Engine {
 public:
  explicit Engine(const Options& opt);
  ~Engine();
  Engine(const Engine&) = delete;
  Engine& operator=(const Engine&) = delete;

  const Options& options() const;
  Stats& stats();
  void reset();  // empty the running table (keeps allocations)
  // Stage timing marks (Stats::device_ms; default on, WC_STAGE_EVENTS=0 off):
  // each costs the GPU ~4.5 us between two kernels, so timed loops turn them off
  void set_stage_events(bool on);

  // Text already resident in HBM (16-B aligned).  Tokens owned by this call are
  // those starting in [0, n); bytes in [n, avail) may be read to finish them.
  void count_device(const uint8_t* d_text, uint64_t n, uint64_t avail, uint64_t global_base, int prev_byte = ' ');
  // Host text: staged through a pinned ring, H2D overlapped with compute.
  void count_host(const uint8_t* h_text, uint64_t n, uint64_t global_base);
  // Streaming source (files larger than HBM, replayed synthetic chunks).
  void count_source(ChunkSource& src, uint64_t global_base);
  // Host-staged benchmark path: `total` bytes replayed from a host pool of
  // whole chunks (each ending with a delimiter), page-locked once and DMA'd
  // straight into HBM with H2D of chunk k+1 overlapping compute of chunk k.
  // `pinned`: the pool is already page-locked (hipHostMalloc, e.g. a HostPool).
  void count_pinned_replay(const uint8_t* pool, uint64_t pool_bytes, uint64_t total, uint64_t global_base,
                           bool pinned = false);

  // Device-resident synthetic text: allocates (or reuses) a buffer of n bytes
  // holding segments [first_segment, ...) of the spec's stream.
  const uint8_t* synth_device(uint64_t n, uint64_t first_segment, const SynthSpec& spec);

  // Merge with other ranks (comm may be null), order by first occurrence and
  // download.  Only rank 0 receives rows unless all_ranks.
  KeyTable result(Comm* comm = nullptr, bool all_ranks = false);

  // Device-side finalisation only (no download): returns distinct keys.  Used
  // by the benchmark to time the full pipeline to an ordered device table.
  uint64_t finalize_device(Comm* comm = nullptr);

  struct Impl;

 private:
  std::unique_ptr<Impl> p_;
};

// ---- host components ----------------------------------------------------------
namespace cpu {
// Single-thread oracle (BASELINE config 1): hash map keyed by the word bytes.
KeyTable count(const uint8_t* text, uint64_t n, uint64_t global_base = 0);
// Exact counts of n bytes of the synthetic stream starting at segment
// `first_segment`, offsets from global_base; `threads` workers (0 = all):
// the full-scale benchmark oracle (words come from the generator's own walk).
KeyTable count_synth(uint64_t n, uint64_t first_segment, const SynthSpec& spec, uint64_t global_base, int threads);
// The reference program's exact quirks (prefix compare, 99-byte fgets records,
// blank line stops input, ...) for differential tests.
// `echo` (optional) receives what the reference echoes: every record it reads,
// up to and including the short record that ends its input.
KeyTable count_reference_compat(const uint8_t* text, uint64_t n, std::string* echo = nullptr);
}  // namespace cpu

// Page-locked host buffer holding a synthetic replay pool (host-staged
// benchmark config): generated in place by `threads` threads, no pageable copy.
class HostPool {
 public:
  // device >= 0: the pool's pages and its generator threads on that GPU's NUMA
  // node (src/io/numa.hpp); numa_node() reports it (-1: unknown / unbound).
  HostPool(uint64_t n, uint64_t first_segment, const SynthSpec& spec, int threads, int device = -1);
  ~HostPool();
  HostPool(const HostPool&) = delete;
  HostPool& operator=(const HostPool&) = delete;
  const uint8_t* data() const { return p_; }
  uint64_t size() const { return n_; }
  double build_seconds() const { return secs_; }
  int numa_node() const { return node_; }

 private:
  uint8_t* p_ = nullptr;
  uint64_t n_ = 0;
  double secs_ = 0;
  int node_ = -1;
};

// Host copy of the synthetic stream (bit-identical to the device generator).
std::vector<uint8_t> synth_host(uint64_t n, uint64_t first_segment, const SynthSpec& spec);

// Reference-identical output framing (/root/reference/main.cu:166-218).
std::string format_output(const KeyTable& t, const uint8_t* echo, uint64_t echo_len, bool echo_input,
                          bool list_rows, uint64_t top_k = 0);

}  // namespace wc
