/* wc.h — C ABI of libwc (used by the Python package through ctypes).
 * Every function returning int returns 0 on success and -1 on error; the
 * message is available from wc_last_error() (thread-local). */
#ifndef WC_C_API_H
#define WC_C_API_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct wc_engine wc_engine;
typedef struct wc_result wc_result;
typedef struct wc_comm wc_comm;

typedef struct wc_options {
  int32_t device;
  uint32_t log2_rec_buckets;
  uint32_t log2_tab_buckets;
  uint32_t max_log2_tab_buckets;
  uint32_t map_blocks;
  uint32_t staging_buffers;
  uint64_t chunk_bytes;
  uint64_t arena_bytes;
  uint64_t min_records;
  double records_per_byte;
  uint32_t merge_mode; /* 0 shuffle (all-to-all by key owner), 1 dense reduce-scatter */
  uint32_t k1_hash_bits; /* tests: LONG-word hash bits kept (0 = all) to force collisions */
} wc_options;

const char* wc_last_error(void);
const char* wc_version(void);
int wc_device_count(void);
/* Host-only test hook: bytes [begin, end) of a file through the parallel reader, `piece` bytes per read. */
int wc_debug_read_file(const char* path, uint64_t begin, uint64_t end, uint64_t piece, uint8_t* dst, uint64_t* got);
/* Kernel test hook: stable LSD radix sort of n u64 keys (low `bits` bits) on
 * `device`; returns the sorted keys and the permutation (host arrays). */
int wc_debug_radix_sort(int device, const uint64_t* keys, uint64_t n, int bits, uint64_t* sorted, uint32_t* perm);
int wc_bench_radix_sort(int device, const uint64_t* keys, uint64_t n, int bits, int reps, double* ms);
int wc_debug_first_order(int device, const uint64_t* keys, uint64_t n, int reps, uint64_t* sorted, uint32_t* perm,
                         int* overflow, double* ms);
/* The same for method 0 (first_order, the sample sort) or 1 (bitmap_order over
 * the keys themselves: distinct keys, a bitmap of max key + 1 bits); *residue =
 * nonzero bitmap words left afterwards (0: the bitmap was cleared). */
int wc_debug_order(int device, int method, const uint64_t* keys, uint64_t n, int reps, uint64_t* sorted,
                   uint32_t* perm, int* overflow, double* ms, uint64_t* residue);
void wc_default_options(wc_options* o);

wc_engine* wc_engine_create(const wc_options* o);
void wc_engine_destroy(wc_engine* e);
int wc_engine_reset(wc_engine* e);
int wc_engine_set_stage_events(wc_engine* e, int on);
/* reset + count the resident text + finalize on the device, in one call */
int wc_job_resident(wc_engine* e, uint64_t n, uint64_t base, wc_comm* c, uint64_t* n_keys);
int wc_count_host(wc_engine* e, const uint8_t* text, uint64_t n, uint64_t global_base);
int wc_count_file(wc_engine* e, const char* path, uint64_t begin, uint64_t end, uint64_t global_base);
/* Checkpointed count of [begin, end) of a file (rank `rank` of `world`): intervals of
   `interval` bytes, each finalised and folded into a host table saved with the next offset to
   `ckpt` (empty: no file).  `resume` continues from an existing checkpoint.  e == NULL counts
   on the CPU oracle.  Returns this rank's table (first-occurrence order) or NULL on error. */
wc_result* wc_count_file_checkpointed(wc_engine* e, const char* path, uint64_t begin, uint64_t end, int rank,
                                      int world, const char* ckpt, uint64_t interval, int resume);
/* Fold `src` into `dst` (counts add, first offset = min, first-occurrence order). */
int wc_result_merge(wc_result* dst, const wc_result* src);
int wc_count_replay(wc_engine* e, const uint8_t* pool, uint64_t pool_bytes, uint64_t total, uint64_t global_base);
/* Host-staged benchmark path: pool page-locked once, chunks DMA'd directly. */
int wc_count_pinned_replay(wc_engine* e, const uint8_t* pool, uint64_t pool_bytes, uint64_t total, uint64_t global_base);
/* Page-locked synthetic replay pool generated in place on `threads` threads (host-staged config);
 * device >= 0: pages and generator threads on that GPU's NUMA node. */
typedef struct wc_pool wc_pool;
wc_pool* wc_pool_create(uint64_t n, uint64_t first_segment, uint64_t seed, uint32_t vocab, double zipf_s,
                        double long_frac, int threads, int device);
void wc_pool_destroy(wc_pool* p);
double wc_pool_build_seconds(const wc_pool* p);
int wc_pool_numa_node(const wc_pool* p); /* -1: unknown / unbound */
int wc_count_pool(wc_engine* e, const wc_pool* p, uint64_t total, uint64_t global_base);
/* Generate synthetic text into the engine's device text buffer (long_frac: share of the
 * vocabulary drawn as 16..64-byte words) ... */
int wc_synth_device(wc_engine* e, uint64_t n, uint64_t first_segment, uint64_t seed, uint32_t vocab, double zipf_s,
                    double long_frac);
/* ... and count [0, n) of it. */
int wc_count_resident(wc_engine* e, uint64_t n, uint64_t global_base);
int wc_finalize_device(wc_engine* e, wc_comm* comm, uint64_t* n_keys);
wc_result* wc_engine_result(wc_engine* e, wc_comm* comm, int all_ranks);
/* JSON object with the engine's Stats. Returns required length. */
int wc_engine_stats_json(wc_engine* e, char* buf, int cap);
int wc_engine_sync(wc_engine* e);

/* results */
uint64_t wc_result_size(const wc_result* r);
uint64_t wc_result_total(const wc_result* r);
uint64_t wc_result_bytes(const wc_result* r);
void wc_result_export(const wc_result* r, uint64_t* counts, uint64_t* first_off, uint64_t* word_off, char* bytes);
void wc_result_free(wc_result* r);
/* reference output framing; *out must be released with wc_free */
int wc_format(const wc_result* r, const uint8_t* echo, uint64_t echo_len, int echo_input, int list_rows,
              uint64_t top_k, char** out, uint64_t* out_len);
void wc_free(void* p);

/* CPU paths */
wc_result* wc_cpu_count(const uint8_t* text, uint64_t n, uint64_t global_base);
wc_result* wc_cpu_count_compat(const uint8_t* text, uint64_t n);
/* Exact counts of n bytes of the synthetic stream from segment first_segment (offsets from
   global_base), computed from the generator's word walk on `threads` CPU threads (0 = all). */
wc_result* wc_cpu_count_synth(uint64_t n, uint64_t first_segment, uint64_t seed, uint32_t vocab, double zipf_s,
                              double long_frac, uint64_t global_base, int threads);
int wc_synth_host(uint8_t* out, uint64_t n, uint64_t first_segment, uint64_t seed, uint32_t vocab, double zipf_s);
/* The same on `threads` threads, written in place. */
int wc_synth_host_mt(uint8_t* out, uint64_t n, uint64_t first_segment, uint64_t seed, uint32_t vocab, double zipf_s,
                     double long_frac, int threads);
int wc_shard_range_mem(const uint8_t* text, uint64_t n, int rank, int world, uint64_t* begin, uint64_t* end);
int wc_shard_range_file(const char* path, int rank, int world, uint64_t* begin, uint64_t* end);

/* communicators */
int wc_rccl_unique_id(char out[128]);
wc_comm* wc_comm_rccl_create(const char* unique_id, int rank, int size, int device);
void wc_comm_destroy(wc_comm* c);
/* Control plane over the communicator itself (no second runtime in the process):
 * a barrier, and recv[r * bytes ...] = rank r's `bytes` host bytes. */
int wc_comm_barrier(wc_comm* c);
int wc_comm_allgather_host(wc_comm* c, const void* send, uint64_t bytes, void* recv);
/* N virtual ranks on `devices` (one thread each) count shards of `text` and
 * merge through the loopback communicator; returns rank 0's result.  With
 * all_ranks every rank receives the merged table and must match rank 0's.
 * resident: shards are copied to HBM first and counted in place (the last
 * pass stays pending: the speculative merged finalize). */
wc_result* wc_loopback_count(const uint8_t* text, uint64_t n, int ranks, const int* devices, const wc_options* o,
                             int all_ranks, int resident, const uint8_t* warm, uint64_t warm_n);
/* warm (nullable): every rank first runs a job on its shard of `warm` (the merge
 * learns its caps there), then the job on `text` — a planned merge. */

#ifdef __cplusplus
}
#endif
#endif
