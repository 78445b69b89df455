// capi.cpp — C ABI over the C++ engine (ctypes binding of the Python package).
#include <atomic>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <exception>
#include <memory>
#include <thread>

#include "common/hip_util.hpp"
#include "dist/comm.hpp"
#include "io/checkpoint.hpp"
#include "io/numa.hpp"
#include "io/source.hpp"
#include "io/synth_host.hpp"
#include "kernels/kernels.hpp"
#include "kernels/keys.hpp"
#include "wc/wc.h"
#include "wc/wc.hpp"

struct wc_engine {
  std::unique_ptr<wc::Engine> e;
  uint64_t resident = 0;  // bytes of synthetic text resident on device
  const uint8_t* d_text = nullptr;
};
struct wc_result {
  wc::KeyTable t;
};
struct wc_comm {
  std::unique_ptr<wc::Comm> c;
  int device = 0;
  hipStream_t s = nullptr;   // control-plane collectives (barrier, host all-gather)
  void* scratch = nullptr;   // device staging of wc_comm_allgather_host
  size_t scratch_bytes = 0;
  ~wc_comm() {
    (void)hipSetDevice(device);
    if (scratch) (void)hipFree(scratch);
    if (s) (void)hipStreamDestroy(s);
  }
  hipStream_t stream() {
    if (!s) {
      WC_HIP_CHECK(hipSetDevice(device));
      WC_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    }
    return s;
  }
};

namespace {
thread_local std::string g_err;

template <class F>
int guard(F&& f) {
  try {
    f();
    return 0;
  } catch (const std::exception& ex) {
    g_err = ex.what();
    return -1;
  }
}

wc::Options to_opts(const wc_options* o) {
  wc::Options x;
  if (!o) return x;
  x.device = o->device;
  x.log2_rec_buckets = o->log2_rec_buckets;
  x.log2_tab_buckets = o->log2_tab_buckets;
  x.max_log2_tab_buckets = o->max_log2_tab_buckets;
  x.map_blocks = o->map_blocks;
  x.staging_buffers = o->staging_buffers;
  x.chunk_bytes = o->chunk_bytes;
  x.arena_bytes = o->arena_bytes;
  x.min_records = o->min_records;
  x.records_per_byte = o->records_per_byte;
  x.merge_mode = o->merge_mode;
  x.k1_hash_bits = o->k1_hash_bits;
  return x;
}

wc::SynthSpec spec_of(uint64_t seed, uint32_t vocab, double s, double long_frac) {
  wc::SynthSpec sp;
  sp.seed = seed;
  sp.vocab = vocab;
  sp.zipf_s = s;
  sp.long_frac = long_frac;
  return sp;
}
}  // namespace

extern "C" {

const char* wc_last_error(void) { return g_err.c_str(); }
const char* wc_version(void) { return "wc-mi355x 0.1.0"; }

// Stream-ordering check of the loopback communicator (tests): two ranks on
// `device`, rank 1's stream held by a wait on a page-locked flag.  Both ranks
// enqueue an allgather of 64 u64 from their own threads; the calls must
// return while rank 1's stream is held (no host wait inside a collective) and
// rank 0's stream must still be waiting (nothing is complete before every
// rank's stream gets there).  Then the flag is released and both results are
// checked.  *returned = 1 if both calls returned while held, *pending = 1 if
// rank 0's stream was still busy then, *correct = 1 if both gathers are right.
int wc_debug_loopback_async(int device, int* returned, int* pending, int* correct) {
  return guard([&] {
    WC_HIP_CHECK(hipSetDevice(device));
    auto comms = wc::make_loopback_comms(2);
    hipStream_t st[2];
    for (auto& x : st) WC_HIP_CHECK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
    uint32_t* hold = nullptr;
    WC_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&hold), 64, hipHostMallocCoherent));
    *hold = 0;
    uint64_t* d = nullptr;
    WC_HIP_CHECK(hipMalloc(&d, 2 * 192 * 8));
    std::vector<uint64_t> h(2 * 192);
    for (int r = 0; r < 2; ++r)
      for (int i = 0; i < 64; ++i) h[(size_t)r * 192 + i] = (uint64_t)r * 1000003u + (uint64_t)i * 7u;
    WC_HIP_CHECK(hipMemcpy(d, h.data(), h.size() * 8, hipMemcpyHostToDevice));
    WC_HIP_CHECK(hipStreamWaitValue32(st[1], hold, 1, hipStreamWaitValueGte, 0xFFFFFFFFu));
    std::atomic<int> back{0};
    std::vector<std::thread> th;
    for (int r = 0; r < 2; ++r)
      th.emplace_back([&, r] {
        comms[r]->allgather(d + (size_t)r * 192, d + (size_t)r * 192 + 64, 64 * 8, st[r]);
        ++back;
      });
    const double t0 = wc::now_seconds();
    while (back.load() < 2 && wc::now_seconds() - t0 < 10.0) std::this_thread::yield();
    *returned = back.load() == 2;
    *pending = hipStreamQuery(st[0]) == hipErrorNotReady;
    __atomic_store_n(hold, 1u, __ATOMIC_SEQ_CST);
    for (auto& t : th) t.join();
    for (auto& x : st) WC_HIP_CHECK(hipStreamSynchronize(x));
    WC_HIP_CHECK(hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost));
    bool ok = true;
    for (int r = 0; r < 2; ++r)
      for (int q = 0; q < 2; ++q)
        for (int i = 0; i < 64; ++i) ok &= h[(size_t)r * 192 + 64 + (size_t)q * 64 + i] == (uint64_t)q * 1000003u + (uint64_t)i * 7u;
    *correct = ok;
    WC_HIP_CHECK(hipFree(d));
    WC_HIP_CHECK(hipHostFree(hold));
    for (auto& x : st) WC_HIP_CHECK(hipStreamDestroy(x));
  });
}

// Raw host side of the file path: the file read with pread_parallel (the
// FileSource reader) in pieces of `piece` bytes into one page-locked buffer
// bound to `device`'s NUMA node, nothing copied to the GPU: the ceiling the
// file-streaming count is measured against (tools/file_path.sh).
// Host-only test hook: read bytes [begin, end) of a file through FileSource
// (the parallel reader pool) in pieces of `piece` bytes into dst.
int wc_debug_read_file(const char* path, uint64_t begin, uint64_t end, uint64_t piece, uint8_t* dst, uint64_t* got) {
  return guard([&] {
    wc::FileSource src(path, begin, end);
    uint64_t n = 0;
    for (;;) {
      const uint64_t k = src.read(dst + n, std::min<uint64_t>(piece, end - begin - n));
      if (k == 0) break;
      n += k;
    }
    *got = n;
  });
}

int wc_file_read_bench(const char* path, uint64_t piece, int device, double* gbps, uint64_t* bytes) {
  return guard([&] {
    const wc::NumaNode nn = device >= 0 ? wc::numa_of_device(device) : wc::NumaNode{};
    wc::ScopedAffinity bind(nn.cpus);
    const uint64_t n = wc::file_size(path);
    wc::PinnedBuffer buf(std::max<uint64_t>(piece, 1));
    wc::FileSource src(path, 0, n);
    const double t0 = wc::now_seconds();
    uint64_t got = 0;
    for (;;) {
      const uint64_t k = src.read(buf.data(), piece);
      if (!k) break;
      got += k;
    }
    *gbps = (double)got / (wc::now_seconds() - t0) / 1e9;
    *bytes = got;
  });
}

// Process-wide communicator counters: collectives enqueued, host waits.
void wc_debug_comm_counters(uint64_t* collectives, uint64_t* host_waits) {
  *collectives = wc::Comm::collectives_total();
  *host_waits = wc::Comm::host_waits_total();
}

// Merge owner of a word among W ranks (keys.hpp owner_of of its placement
// hash): the native rule the Python merge mirror is tested against.
uint32_t wc_key_owner(const uint8_t* word, uint64_t len, uint32_t W) {
  uint64_t k0, k1;
  wc::key_of(word, len, &k0, &k1);
  return wc::owner_of(wc::place_hash(k0, k1), W ? W : 1);
}

int wc_debug_radix_sort(int device, const uint64_t* keys, uint64_t n, int bits, uint64_t* sorted, uint32_t* perm) {
  return guard([&] {
    WC_HIP_CHECK(hipSetDevice(device));
    hipStream_t s = nullptr;
    uint8_t* mem = nullptr;
    const size_t nn = n ? n : 1, hw = wc::radix_hist_words(n);
    const size_t bytes = nn * (8 + 8 + 4 + 4) + hw * 4 + 1024;
    WC_HIP_CHECK(hipMalloc(&mem, bytes));
    uint64_t* k = reinterpret_cast<uint64_t*>(mem);
    uint64_t* tk = k + nn;
    uint32_t* v = reinterpret_cast<uint32_t*>(tk + nn);
    uint32_t* tv = v + nn;
    uint32_t* hist = tv + nn;
    WC_HIP_CHECK(hipMemcpy(k, keys, n * 8, hipMemcpyHostToDevice));
    wc::launch_iota_u32(v, n, s);
    wc::radix_sort_pairs(k, v, tk, tv, hist, n, bits, s);
    WC_HIP_CHECK(hipMemcpy(sorted, k, n * 8, hipMemcpyDeviceToHost));
    WC_HIP_CHECK(hipMemcpy(perm, v, n * 4, hipMemcpyDeviceToHost));
    WC_HIP_CHECK(hipFree(mem));
  });
}

// Device time of radix_sort_pairs on n given keys (+ iota values), averaged
// over `reps` sorts of the same input: the sort-based-reduce A/B
// (tools/sort_vs_hash.py) prices one full sort of a pass's records.
int wc_bench_radix_sort(int device, const uint64_t* keys, uint64_t n, int bits, int reps, double* ms) {
  return guard([&] {
    WC_HIP_CHECK(hipSetDevice(device));
    hipStream_t s = nullptr;
    uint8_t* mem = nullptr;
    const size_t nn = n ? n : 1, hw = wc::radix_hist_words(n);
    WC_HIP_CHECK(hipMalloc(&mem, nn * (8 + 8 + 8 + 4 + 4) + hw * 4 + 1024));
    uint64_t* src = reinterpret_cast<uint64_t*>(mem);
    uint64_t* k = src + nn;
    uint64_t* tk = k + nn;
    uint32_t* v = reinterpret_cast<uint32_t*>(tk + nn);
    uint32_t* tv = v + nn;
    uint32_t* hist = tv + nn;
    WC_HIP_CHECK(hipMemcpy(src, keys, n * 8, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    WC_HIP_CHECK(hipEventCreate(&e0));
    WC_HIP_CHECK(hipEventCreate(&e1));
    float total = 0;
    for (int r = 0; r < reps; ++r) {
      WC_HIP_CHECK(hipMemcpyAsync(k, src, n * 8, hipMemcpyDeviceToDevice, s));
      wc::launch_iota_u32(v, n, s);
      WC_HIP_CHECK(hipEventRecord(e0, s));
      bool in_tmp = false;
      wc::radix_sort_pairs(k, v, tk, tv, hist, n, bits, s, &in_tmp);
      WC_HIP_CHECK(hipEventRecord(e1, s));
      WC_HIP_CHECK(hipEventSynchronize(e1));
      float t = 0;
      WC_HIP_CHECK(hipEventElapsedTime(&t, e0, e1));
      if (r > 0 || reps == 1) total += t;  // first rep warms up
    }
    *ms = total / (reps > 1 ? reps - 1 : 1);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    WC_HIP_CHECK(hipFree(mem));
  });
}

// first_order (the three-launch sample sort) on n UNIQUE given keys as a key
// column source: sorted keys, the permutation (source row of each output row)
// and the overflow word; *ms = device time averaged over `reps` (> 1: the
// first rep warms up).  Tests + tools/sort_bench.py.
// method 0: first_order (the sample sort); 1: bitmap_order over the keys
// themselves (shift 0; keys must be distinct, the bitmap spans [0, max key]);
// *residue = nonzero bitmap words left after the calls (must be 0).
int wc_debug_order(int device, int method, const uint64_t* keys, uint64_t n, int reps, uint64_t* sorted,
                   uint32_t* perm, int* overflow, double* ms, uint64_t* residue) {
  return guard([&] {
    WC_HIP_CHECK(hipSetDevice(device));
    hipStream_t s = nullptr;
    const size_t nn = n ? n : 1;
    wc::OrderSrc src{};
    src.table = false;
    src.n = n;
    uint64_t kmax = 0;
    for (uint64_t i = 0; i < n; ++i) kmax = std::max(kmax, keys[i]);
    const size_t ws = method == 1 ? wc::bitmap_order_ws_bytes(nn, kmax + 1, 0) : wc::first_order_ws_bytes(src, n);
    unsigned long long* bm = nullptr;
    const size_t bm_words = method == 1 ? wc::bitmap_order_words(kmax + 1, 0) : 0;
    if (bm_words) {
      WC_HIP_CHECK(hipMalloc(&bm, bm_words * 8));
      WC_HIP_CHECK(hipMemset(bm, 0, bm_words * 8));
    }
    uint8_t* mem = nullptr;
    WC_HIP_CHECK(hipMalloc(&mem, nn * (8 * 5 + 4) * 2 + ws + 4096));
    uint8_t* p = mem;
    auto take = [&](size_t b) {
      uint8_t* r = p;
      p += (b + 255) / 256 * 256;
      return r;
    };
    uint64_t* in[5];
    for (auto& c : in) c = reinterpret_cast<uint64_t*>(take(nn * 8));
    uint32_t* in_len = reinterpret_cast<uint32_t*>(take(nn * 4));
    wc::OrderDst d{};
    d.k0 = reinterpret_cast<uint64_t*>(take(nn * 8));
    d.k1 = reinterpret_cast<uint64_t*>(take(nn * 8));
    d.cnt = reinterpret_cast<uint64_t*>(take(nn * 8));
    d.first = reinterpret_cast<uint64_t*>(take(nn * 8));
    d.soff = reinterpret_cast<uint64_t*>(take(nn * 8));
    d.slen = reinterpret_cast<uint32_t*>(take(nn * 4));
    void* w = take(ws);
    std::vector<uint64_t> idx(nn);
    for (uint64_t i = 0; i < n; ++i) idx[i] = i;
    uint32_t kb = 1;
    while (kb < 64 && (kmax >> kb) != 0) ++kb;
    WC_HIP_CHECK(hipMemcpy(in[0], idx.data(), n * 8, hipMemcpyHostToDevice));  // k0 = the source row
    WC_HIP_CHECK(hipMemset(in[1], 0, nn * 8));
    WC_HIP_CHECK(hipMemset(in[2], 0, nn * 8));
    WC_HIP_CHECK(hipMemcpy(in[3], keys, n * 8, hipMemcpyHostToDevice));
    WC_HIP_CHECK(hipMemset(in[4], 0, nn * 8));
    WC_HIP_CHECK(hipMemset(in_len, 0, nn * 4));
    src.k0 = in[0];
    src.k1 = in[1];
    src.cnt = in[2];
    src.first = in[3];
    src.soff = in[4];
    src.slen = in_len;
    hipEvent_t e0, e1;
    WC_HIP_CHECK(hipEventCreate(&e0));
    WC_HIP_CHECK(hipEventCreate(&e1));
    float total = 0;
    uint32_t* ovf = nullptr;
    unsigned long long* d_st = nullptr;
    const bool stamps = std::getenv("WC_FO_STAMPS") != nullptr;
    if (stamps) {
      WC_HIP_CHECK(hipMalloc(&d_st, 48 * 8));
      WC_HIP_CHECK(hipMemset(d_st, 0, 48 * 8));
      wc::first_order_stamps(d_st);
    }
    for (int r = 0; r < std::max(reps, 1); ++r) {
      WC_HIP_CHECK(hipEventRecord(e0, s));
      if (stamps && r == 1) WC_HIP_CHECK(hipMemsetAsync(d_st, 0, 48 * 8, s));  // warm reps only
      if (n && method == 1) ovf = wc::bitmap_order(src, d, n, kmax + 1, 0, bm, w, nullptr, s);
      else if (n) ovf = wc::first_order(src, d, n, kb, w, nullptr, s);
      WC_HIP_CHECK(hipEventRecord(e1, s));
      WC_HIP_CHECK(hipEventSynchronize(e1));
      float t = 0;
      WC_HIP_CHECK(hipEventElapsedTime(&t, e0, e1));
      if (r > 0 || reps <= 1) total += t;
    }
    *ms = total / (reps > 1 ? reps - 1 : 1);
    if (stamps) {  // max over reps and blocks, 100 MHz ticks -> us
      unsigned long long h[48];
      WC_HIP_CHECK(hipMemcpy(h, d_st, sizeof h, hipMemcpyDeviceToHost));
      wc::first_order_stamps(nullptr);
      WC_HIP_CHECK(hipFree(d_st));
      const char* nm[3] = {"split", "bin", "sort"};
      for (int k = 0; k < 3; ++k) {
        std::fprintf(stderr, "fo %-5s n=%llu phase us:", nm[k], (unsigned long long)n);
        for (int p = 1; p < 6; ++p) std::fprintf(stderr, " %.2f", h[16 * k + p] / 100.0);
        std::fprintf(stderr, "\n");
      }
    }
    uint32_t o = 0;
    if (ovf) WC_HIP_CHECK(hipMemcpy(&o, ovf, 4, hipMemcpyDeviceToHost));
    *overflow = (int)o;
    std::vector<uint64_t> k0(nn);
    WC_HIP_CHECK(hipMemcpy(sorted, d.first, n * 8, hipMemcpyDeviceToHost));
    WC_HIP_CHECK(hipMemcpy(k0.data(), d.k0, n * 8, hipMemcpyDeviceToHost));
    for (uint64_t i = 0; i < n; ++i) perm[i] = (uint32_t)k0[i];
    *residue = 0;
    if (bm) {
      std::vector<uint64_t> h(bm_words);
      WC_HIP_CHECK(hipMemcpy(h.data(), bm, bm_words * 8, hipMemcpyDeviceToHost));
      for (uint64_t x : h) *residue += x != 0;
      WC_HIP_CHECK(hipFree(bm));
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    WC_HIP_CHECK(hipFree(mem));
  });
}

int wc_debug_first_order(int device, const uint64_t* keys, uint64_t n, int reps, uint64_t* sorted, uint32_t* perm,
                         int* overflow, double* ms) {
  uint64_t residue = 0;
  return wc_debug_order(device, 0, keys, n, reps, sorted, perm, overflow, ms, &residue);
}

int wc_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

void wc_default_options(wc_options* o) {
  const wc::Options d;
  o->device = d.device;
  o->log2_rec_buckets = d.log2_rec_buckets;
  o->log2_tab_buckets = d.log2_tab_buckets;
  o->max_log2_tab_buckets = d.max_log2_tab_buckets;
  o->map_blocks = d.map_blocks;
  o->staging_buffers = d.staging_buffers;
  o->chunk_bytes = d.chunk_bytes;
  o->arena_bytes = d.arena_bytes;
  o->min_records = d.min_records;
  o->records_per_byte = d.records_per_byte;
  o->merge_mode = d.merge_mode;
  o->k1_hash_bits = d.k1_hash_bits;
}

wc_engine* wc_engine_create(const wc_options* o) {
  wc_engine* e = nullptr;
  if (guard([&] {
        e = new wc_engine;
        e->e.reset(new wc::Engine(to_opts(o)));
      }) != 0) {
    delete e;
    return nullptr;
  }
  return e;
}

void wc_engine_destroy(wc_engine* e) { delete e; }

int wc_engine_reset(wc_engine* e) { return guard([&] { e->e->reset(); }); }
int wc_engine_set_stage_events(wc_engine* e, int on) { return guard([&] { e->e->set_stage_events(on != 0); }); }

int wc_count_host(wc_engine* e, const uint8_t* text, uint64_t n, uint64_t base) {
  return guard([&] { e->e->count_host(text, n, base); });
}

int wc_count_file(wc_engine* e, const char* path, uint64_t begin, uint64_t end, uint64_t base) {
  return guard([&] {
    wc::FileSource src(path, begin, end);
    e->e->count_source(src, base);
  });
}

wc_result* wc_count_file_checkpointed(wc_engine* e, const char* path, uint64_t begin, uint64_t end, int rank,
                                      int world, const char* ckpt, uint64_t interval, int resume) {
  wc_result* r = nullptr;
  const int rc = guard([&] {
    const std::string file(path), base(ckpt ? ckpt : "");
    const std::string cpath = base.empty() ? std::string() : wc::checkpoint_path(base, rank, world);
    wc::Checkpoint k = wc::open_checkpoint(cpath, resume != 0 && !cpath.empty(), file, wc::file_size(file), begin, end,
                                           rank, world);
    wc::run_checkpointed(file, k, interval, cpath, [&](const uint8_t* q, uint64_t n, uint64_t gbase) {
      if (!e) return wc::cpu::count(q, n, gbase);
      e->e->count_host(q, n, gbase);
      wc::KeyTable kt = e->e->result(nullptr, false);
      e->e->reset();
      return kt;
    });
    r = new wc_result{std::move(k.table)};
  });
  return rc == 0 ? r : nullptr;
}

int wc_result_merge(wc_result* dst, const wc_result* src) { return guard([&] { wc::merge_tables(dst->t, src->t); }); }

int wc_count_replay(wc_engine* e, const uint8_t* pool, uint64_t pool_bytes, uint64_t total, uint64_t base) {
  return guard([&] {
    wc::ReplaySource src(pool, pool_bytes, total);
    e->e->count_source(src, base);
  });
}

int wc_count_pinned_replay(wc_engine* e, const uint8_t* pool, uint64_t pool_bytes, uint64_t total, uint64_t base) {
  return guard([&] { e->e->count_pinned_replay(pool, pool_bytes, total, base); });
}

int wc_synth_device(wc_engine* e, uint64_t n, uint64_t first_segment, uint64_t seed, uint32_t vocab, double s,
                    double long_frac) {
  return guard([&] {
    e->d_text = e->e->synth_device(n, first_segment, spec_of(seed, vocab, s, long_frac));
    e->resident = n;
  });
}

int wc_count_resident(wc_engine* e, uint64_t n, uint64_t base) {
  return guard([&] {
    WC_CHECK(e->d_text && n <= e->resident, "no resident text of that size (call wc_synth_device first)");
    e->e->count_device(e->d_text, n, e->resident, base, ' ');
  });
}

int wc_finalize_device(wc_engine* e, wc_comm* c, uint64_t* n_keys) {
  return guard([&] { *n_keys = e->e->finalize_device(c ? c->c.get() : nullptr); });
}

// One whole job on the resident text in one call: reset + count + finalize
// (the three calls' Python round trips were GPU idle time between jobs).
int wc_job_resident(wc_engine* e, uint64_t n, uint64_t base, wc_comm* c, uint64_t* n_keys) {
  return guard([&] {
    WC_CHECK(e->d_text && n <= e->resident, "no resident text of that size (call wc_synth_device first)");
    e->e->reset();
    e->e->count_device(e->d_text, n, e->resident, base, ' ');
    *n_keys = e->e->finalize_device(c ? c->c.get() : nullptr);
  });
}

wc_result* wc_engine_result(wc_engine* e, wc_comm* c, int all_ranks) {
  wc_result* r = new wc_result;
  if (guard([&] { r->t = e->e->result(c ? c->c.get() : nullptr, all_ranks != 0); }) != 0) {
    delete r;
    return nullptr;
  }
  return r;
}

int wc_engine_stats_json(wc_engine* e, char* buf, int cap) {
  const wc::Stats& s = e->e->stats();
  char tmp[2048];
  const int k = snprintf(tmp, sizeof tmp,
                         "{\"bytes\": %llu, \"tokens\": %llu, \"keys\": %llu, \"records\": %llu, "
                         "\"long_tokens\": %llu, \"long_direct\": %u, \"chunks\": %u, "
                         "\"map_reruns\": %u, \"table_splits\": %u, \"log2_buckets\": %u, \"order_path\": %u, "
                         "\"merges_planned\": %u, \"merge_redos\": %u, "
                         "\"device_ms\": {\"map\": %.4f, \"reduce\": %.4f, \"finalize\": %.4f, \"merge\": %.4f, "
                         "\"idle\": %.4f, \"total\": %.4f}, "
                         "\"host_ms\": {\"count\": %.4f, \"finalize\": %.4f}}",
                         (unsigned long long)s.bytes, (unsigned long long)s.tokens, (unsigned long long)s.keys,
                         (unsigned long long)s.records, (unsigned long long)s.long_tokens, s.long_direct, s.chunks,
                         s.map_reruns, s.table_splits, s.log2_buckets, s.order_path,
                         s.merges_planned, s.merge_redos,
                         s.map_ms,
                         s.reduce_ms, s.finalize_ms, s.merge_ms, s.idle_ms, s.device_ms, s.host_count_ms,
                         s.host_finalize_ms);
  if (buf && cap > 0) {
    std::strncpy(buf, tmp, (size_t)cap - 1);
    buf[cap - 1] = 0;
  }
  return k;
}

int wc_engine_sync(wc_engine* e) {
  return guard([&] {
    WC_HIP_CHECK(hipSetDevice(e->e->options().device));
    WC_HIP_CHECK(hipDeviceSynchronize());
  });
}

uint64_t wc_result_size(const wc_result* r) { return r->t.size(); }
uint64_t wc_result_total(const wc_result* r) { return r->t.total; }
uint64_t wc_result_bytes(const wc_result* r) {
  uint64_t b = 0;
  for (const auto& w : r->t.words) b += w.size();
  return b;
}

void wc_result_export(const wc_result* r, uint64_t* counts, uint64_t* first_off, uint64_t* word_off, char* bytes) {
  uint64_t o = 0;
  for (size_t i = 0; i < r->t.size(); ++i) {
    if (counts) counts[i] = r->t.counts[i];
    if (first_off) first_off[i] = r->t.first_off[i];
    if (word_off) word_off[i] = o;
    if (bytes) std::memcpy(bytes + o, r->t.words[i].data(), r->t.words[i].size());
    o += r->t.words[i].size();
  }
  if (word_off) word_off[r->t.size()] = o;
}

void wc_result_free(wc_result* r) { delete r; }

int wc_format(const wc_result* r, const uint8_t* echo, uint64_t echo_len, int echo_input, int list_rows,
              uint64_t top_k, char** out, uint64_t* out_len) {
  return guard([&] {
    const std::string s = wc::format_output(r->t, echo, echo_len, echo_input != 0, list_rows != 0, top_k);
    char* p = static_cast<char*>(std::malloc(s.size() + 1));
    WC_CHECK(p, "out of memory");
    std::memcpy(p, s.data(), s.size());
    p[s.size()] = 0;
    *out = p;
    *out_len = s.size();
  });
}

void wc_free(void* p) { std::free(p); }

wc_result* wc_cpu_count(const uint8_t* text, uint64_t n, uint64_t base) {
  wc_result* r = new wc_result;
  if (guard([&] { r->t = wc::cpu::count(text, n, base); }) != 0) {
    delete r;
    return nullptr;
  }
  return r;
}

wc_result* wc_cpu_count_compat(const uint8_t* text, uint64_t n) {
  wc_result* r = new wc_result;
  if (guard([&] { r->t = wc::cpu::count_reference_compat(text, n); }) != 0) {
    delete r;
    return nullptr;
  }
  return r;
}

wc_result* wc_cpu_count_synth(uint64_t n, uint64_t first_segment, uint64_t seed, uint32_t vocab, double zs,
                              double long_frac, uint64_t base, int threads) {
  wc_result* r = new wc_result;
  if (guard([&] { r->t = wc::cpu::count_synth(n, first_segment, spec_of(seed, vocab, zs, long_frac), base, threads); }) !=
      0) {
    delete r;
    return nullptr;
  }
  return r;
}

int wc_synth_host(uint8_t* out, uint64_t n, uint64_t first_segment, uint64_t seed, uint32_t vocab, double s) {
  return wc_synth_host_mt(out, n, first_segment, seed, vocab, s, 0.0, 1);
}

int wc_synth_host_mt(uint8_t* out, uint64_t n, uint64_t first_segment, uint64_t seed, uint32_t vocab, double s,
                     double long_frac, int threads) {
  return guard([&] {
    const wc::SynthSpec sp = spec_of(seed, vocab, s, long_frac);
    wc::synth_host_into(out, n, first_segment, sp, wc::build_vocab(sp), threads);
  });
}

struct wc_pool {
  std::unique_ptr<wc::HostPool> p;
};

wc_pool* wc_pool_create(uint64_t n, uint64_t first_segment, uint64_t seed, uint32_t vocab, double s, double long_frac,
                        int threads, int device) {
  wc_pool* r = new wc_pool;
  if (guard([&] {
        r->p.reset(new wc::HostPool(n, first_segment, spec_of(seed, vocab, s, long_frac), threads, device));
      }) != 0) {
    delete r;
    return nullptr;
  }
  return r;
}
void wc_pool_destroy(wc_pool* p) { delete p; }
double wc_pool_build_seconds(const wc_pool* p) { return p ? p->p->build_seconds() : 0.0; }
int wc_pool_numa_node(const wc_pool* p) { return p ? p->p->numa_node() : -1; }

// NUMA resolution against a sysfs tree (tests: a fake root): node of the PCI
// device and up to `cap` of its CPUs; returns the CPU count.
int wc_numa_of_pci(const char* sysfs_root, const char* bus_id, int* node, int* cpus, int cap) {
  const wc::NumaNode n = wc::numa_of_pci(bus_id, sysfs_root);
  *node = n.node;
  for (int i = 0; i < cap && i < (int)n.cpus.size(); ++i) cpus[i] = n.cpus[i];
  return (int)n.cpus.size();
}

// Pinned-memory H2D bandwidth from a pool on NUMA node `node` (-1: the GPU's
// own node, numa_of_device) to `device`: `bytes` copied `reps` times after one
// warm copy.  *node_used = the node the pool was bound to (-1: unbound).
int wc_h2d_bench(int device, int node, uint64_t bytes, int reps, double* gbps, int* node_used) {
  return guard([&] {
    WC_HIP_CHECK(hipSetDevice(device));
    const wc::NumaNode nn = node >= 0 ? wc::numa_node_cpus(node) : wc::numa_of_device(device);
    uint8_t* h = nullptr;
    uint8_t* d = nullptr;
    {
      wc::ScopedAffinity bind(nn.cpus);
      *node_used = bind.active() ? nn.node : -1;
      WC_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&h), bytes,
                                 bind.active() ? hipHostMallocNumaUser : hipHostMallocDefault));
      std::memset(h, 0x20, bytes);
    }
    wc::dev_malloc(&d, bytes);
    hipStream_t s;
    WC_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    WC_HIP_CHECK(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s));
    WC_HIP_CHECK(hipStreamSynchronize(s));
    const double t0 = wc::now_seconds();
    for (int i = 0; i < reps; ++i) WC_HIP_CHECK(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s));
    WC_HIP_CHECK(hipStreamSynchronize(s));
    *gbps = (double)bytes * reps / (wc::now_seconds() - t0) / 1e9;
    WC_HIP_CHECK(hipStreamDestroy(s));
    WC_HIP_CHECK(hipFree(d));
    WC_HIP_CHECK(hipHostFree(h));
  });
}
int wc_count_pool(wc_engine* e, const wc_pool* p, uint64_t total, uint64_t base) {
  return guard([&] { e->e->count_pinned_replay(p->p->data(), p->p->size(), total, base, true); });
}

int wc_shard_range_mem(const uint8_t* text, uint64_t n, int rank, int world, uint64_t* begin, uint64_t* end) {
  return guard([&] {
    const wc::ShardRange r = wc::shard_range_mem(text, n, rank, world);
    *begin = r.begin;
    *end = r.end;
  });
}

int wc_shard_range_file(const char* path, int rank, int world, uint64_t* begin, uint64_t* end) {
  return guard([&] {
    const wc::ShardRange r = wc::shard_range(path, rank, world);
    *begin = r.begin;
    *end = r.end;
  });
}

int wc_rccl_unique_id(char out[128]) {
  return guard([&] {
    const std::string id = wc::rccl_unique_id();
    std::memcpy(out, id.data(), id.size());
  });
}

wc_comm* wc_comm_rccl_create(const char* unique_id, int rank, int size, int device) {
  wc_comm* c = new wc_comm;
  c->device = device;
  if (guard([&] { c->c = wc::make_rccl_comm(std::string(unique_id, wc::RCCL_ID_BYTES), rank, size, device); }) != 0) {
    delete c;
    return nullptr;
  }
  return c;
}

// Control plane of one-process-per-GPU jobs without a second runtime (bench.py):
// a barrier and a small all-gather of host bytes over the job's own RCCL
// communicator, both waited for under its watchdog (WC_COMM_TIMEOUT_S).
int wc_comm_barrier(wc_comm* c) {
  return guard([&] {
    WC_HIP_CHECK(hipSetDevice(c->device));
    c->c->barrier(c->stream());
  });
}

int wc_comm_allgather_host(wc_comm* c, const void* send, uint64_t bytes, void* recv) {
  return guard([&] {
    WC_HIP_CHECK(hipSetDevice(c->device));
    hipStream_t s = c->stream();
    const size_t W = (size_t)c->c->size(), need = bytes * (W + 1);
    if (need > c->scratch_bytes) {
      if (c->scratch) WC_HIP_CHECK(hipFree(c->scratch));
      c->scratch = nullptr;
      WC_HIP_CHECK(hipMalloc(&c->scratch, need));
      c->scratch_bytes = need;
    }
    uint8_t* d_send = static_cast<uint8_t*>(c->scratch);
    uint8_t* d_recv = d_send + bytes;
    WC_HIP_CHECK(hipMemcpyAsync(d_send, send, bytes, hipMemcpyHostToDevice, s));
    c->c->allgather(d_send, d_recv, bytes, s);
    WC_HIP_CHECK(hipMemcpyAsync(recv, d_recv, bytes * W, hipMemcpyDeviceToHost, s));
    c->c->sync(s);
  });
}

void wc_comm_destroy(wc_comm* c) { delete c; }

// Virtual ranks on one GPU (bench.py --virtual-ranks): `ranks` engines in
// threads on `device`, each holding its own resident shard of the synthetic
// stream (rank r: segments [r * nseg, (r + 1) * nseg), global offsets from
// r * bytes), one stream-ordered loopback group, and bench.py's step — reset,
// count the shard, merged finalize on the device — `warmup` + `steps` times,
// the timed loop bracketed by communicator barriers.  out[14 r + i] =
// {wall ms / step, device ms of the last job: map, reduce, finalize, merge,
// idle, tokens, local keys, merges planned, merges redone, merge collectives,
// merge bytes sent to peers, sum over collectives of the largest per-peer
// amount, bytes rank 0 received in the gather} (14 doubles per rank).  Returns rank 0's
// merged table of one more job after timing — the same step ending in
// result(), so it goes the way the timed jobs went (planned merge once the
// first job learned its caps) — for validation.
wc_result* wc_virtual_bench(const wc_options* o, int ranks, int device, uint64_t bytes, uint64_t seed, uint32_t vocab,
                            double zipf, double long_frac, int steps, int warmup, double* out) {
  wc_result* res = new wc_result;
  std::vector<std::string> errs(ranks);
  std::vector<std::unique_ptr<wc::Comm>> comms;
  if (guard([&] { comms = wc::make_loopback_comms(ranks); }) != 0) {
    delete res;
    return nullptr;
  }
  const uint64_t seg = 1024, nseg = bytes / seg;
  // tests only: the LAST rank's validation job counts this many more segments
  // than the timed jobs (the stream stays contiguous: [0, (ranks * nseg + grow) * seg)),
  // so it outgrows the planned merge's learned caps
  const uint64_t grow = std::getenv("WC_VB_GROW_SEGS") ? std::strtoull(std::getenv("WC_VB_GROW_SEGS"), nullptr, 10) : 0;
  std::vector<std::thread> th;
  for (int r = 0; r < ranks; ++r) {
    th.emplace_back([&, r] {
      try {
        wc::Options opt = to_opts(o);
        opt.device = device;
        wc::Engine eng(opt);
        const uint64_t vseg = nseg + (r == ranks - 1 ? grow : 0);  // the validation job's segments
        const uint8_t* d = eng.synth_device(vseg * seg, (uint64_t)r * nseg, spec_of(seed, vocab, zipf, long_frac));
        wc::Comm* c = comms[r].get();
        auto step = [&] {
          eng.reset();
          eng.count_device(d, nseg * seg, nseg * seg, (uint64_t)r * nseg * seg, ' ');
          return eng.finalize_device(c);
        };
        for (int i = 0; i < warmup; ++i) step();
        WC_HIP_CHECK(hipDeviceSynchronize());
        c->barrier(nullptr);
        const double t0 = wc::now_seconds();
        uint64_t keys = 0;
        for (int i = 0; i < steps; ++i) keys = step();
        WC_HIP_CHECK(hipDeviceSynchronize());
        c->barrier(nullptr);
        const double ms = (wc::now_seconds() - t0) * 1e3 / (steps > 0 ? steps : 1);
        const wc::Stats st = eng.stats();
        eng.reset();
        eng.count_device(d, vseg * seg, vseg * seg, (uint64_t)r * nseg * seg, ' ');
        wc::KeyTable t = eng.result(c, false);
        const wc::Stats& st2 = eng.stats();
        double* v = out + 14 * (size_t)r;
        v[0] = ms;
        v[1] = st.map_ms;
        v[2] = st.reduce_ms;
        v[3] = st.finalize_ms;
        v[4] = st.merge_ms;
        v[5] = st.idle_ms;
        v[6] = (double)st.tokens;
        v[7] = (double)keys;
        v[8] = (double)st2.merges_planned;
        v[9] = (double)st2.merge_redos;
        v[10] = (double)st.merge_collectives;
        v[11] = (double)st.merge_sent_bytes;
        v[12] = (double)st.merge_peer_bytes;
        v[13] = (double)st.merge_root_recv_bytes;
        if (r == 0) res->t = std::move(t);
      } catch (const std::exception& ex) {
        errs[r] = ex.what();
        comms[r]->abort(ex.what());
      }
    });
  }
  for (auto& t : th) t.join();
  for (int r = 0; r < ranks; ++r)
    if (!errs[r].empty()) {
      g_err = "rank " + std::to_string(r) + ": " + errs[r];
      delete res;
      return nullptr;
    }
  return res;
}

wc_result* wc_loopback_count(const uint8_t* text, uint64_t n, int ranks, const int* devices, const wc_options* o,
                             int all_ranks, int resident, const uint8_t* warm, uint64_t warm_n) {
  wc_result* out = new wc_result;
  std::vector<std::string> errs(ranks);
  std::vector<wc::KeyTable> tables(ranks);
  std::vector<std::unique_ptr<wc::Comm>> comms;
  if (guard([&] {
        std::vector<int> devs;
        if (devices) devs.assign(devices, devices + ranks);
        comms = wc::make_loopback_comms(ranks, devs);
      }) != 0) {
    delete out;
    return nullptr;
  }
  std::vector<std::thread> th;
  for (int r = 0; r < ranks; ++r) {
    th.emplace_back([&, r] {
      try {
        wc::Options opt = to_opts(o);
        opt.device = devices ? devices[r] : 0;
        wc::Engine eng(opt);
        // one job on (tx, nn): this rank's shard, counted and merged
        auto job = [&](const uint8_t* tx, uint64_t nn) {
          eng.reset();
          const wc::ShardRange sr = wc::shard_range_mem(tx, nn, r, ranks);
          uint8_t* d = nullptr;
          if (sr.end > sr.begin && resident) {
            // HBM-resident shard: the last pass stays pending and the merge runs
            // speculatively behind it (merge_cols_speculative / the planned merge)
            const uint64_t len = sr.end - sr.begin;
            WC_HIP_CHECK(hipSetDevice(opt.device));
            wc::dev_malloc(&d, len + 64);
            WC_HIP_CHECK(hipMemcpy(d, tx + sr.begin, len, hipMemcpyHostToDevice));
            eng.count_device(d, len, len, sr.begin, sr.begin ? tx[sr.begin - 1] : ' ');
          } else if (sr.end > sr.begin) {
            eng.count_host(tx + sr.begin, sr.end - sr.begin, sr.begin);
          }
          wc::KeyTable kt = eng.result(comms[r].get(), all_ranks != 0);
          if (d) (void)hipFree(d);
          return kt;
        };
        // warm (nullable): a first job on other text — the merge learns its caps
        // from it, so the job on `text` runs the planned merge
        if (warm) (void)job(warm, warm_n);
        wc::KeyTable t = job(text, n);
        if (r == 0) {
          out->t = std::move(t);
        } else if (all_ranks) {
          tables[r] = std::move(t);
        }
      } catch (const std::exception& ex) {
        errs[r] = ex.what();
        comms[r]->abort(ex.what());  // peers blocked in a collective fail instead of waiting forever
      }
    });
  }
  for (auto& t : th) t.join();
  for (int r = 0; r < ranks; ++r)
    if (!errs[r].empty()) {
      g_err = "rank " + std::to_string(r) + ": " + errs[r];
      delete out;
      return nullptr;
    }
  for (int r = 1; all_ranks && r < ranks; ++r) {
    const wc::KeyTable& t = tables[r];
    if (t.words != out->t.words || t.counts != out->t.counts || t.first_off != out->t.first_off) {
      g_err = "rank " + std::to_string(r) + ": all_ranks result differs from rank 0";
      delete out;
      return nullptr;
    }
  }
  return out;
}

}  // extern "C"
