// engine.cpp — per-GPU MapReduce pipeline (host orchestration).
//
// Reference: runMapReduce (/root/reference/main.cu:133-162) mallocs, copies,
// launches map then reduce on the legacy default stream, copies back and
// frees, once, for <= 891 bytes of input.  Here:
//  * one preallocated workspace per engine (records, running table, key arena,
//    counters); nothing is allocated on the per-chunk path;
//  * text is processed in HBM-sized chunks (default 1 GiB) — either already
//    resident (count_device), or streamed from host memory / files through a
//    pinned ring where the H2D of chunk k+1 (copy stream) overlaps the
//    map/reduce of chunk k (compute stream);
//  * per chunk ONE host synchronisation reads a 32-byte counter block; shuffle
//    region overflow re-runs the chunk in halves, running-table overflow
//    splits the table (B -> 2B) and re-runs only the overflowed buckets.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "engine_impl.hpp"
#include "../dist/comm.hpp"

namespace wc {

// ---------------------------------------------------------------- TableStore --
TableStore::~TableStore() {
  if (mem) (void)hipFree(mem);
}

void TableStore::alloc(uint32_t log2_buckets) {
  if (mem && v.log2_buckets == log2_buckets) return;
  if (mem) WC_HIP_CHECK(hipFree(mem));
  mem = nullptr;
  const size_t nb = (size_t)1 << log2_buckets, n = nb * TAB_SLOTS;
  const size_t bytes = n * (5 * sizeof(uint64_t) + sizeof(uint32_t)) + nb * sizeof(uint32_t) + 1024;
  dev_malloc(&mem, bytes);
  uint8_t* p = static_cast<uint8_t*>(mem);
  auto take = [&](size_t b) {
    uint8_t* r = p;
    p += (b + 255) / 256 * 256;
    return r;
  };
  v.k0 = reinterpret_cast<uint64_t*>(take(n * 8));
  v.k1 = reinterpret_cast<uint64_t*>(take(n * 8));
  v.cnt = reinterpret_cast<uint64_t*>(take(n * 8));
  v.first = reinterpret_cast<uint64_t*>(take(n * 8));
  v.sref_off = reinterpret_cast<uint64_t*>(take(n * 8));
  v.sref_len = reinterpret_cast<uint32_t*>(take(n * 4));
  v.occupancy = reinterpret_cast<uint32_t*>(take(nb * 4));
  v.log2_buckets = log2_buckets;
}

// ---------------------------------------------------------------------- Impl --
Engine::Impl::Impl(const Options& o) : opt(o) {
  dev = opt.device;
  WC_HIP_CHECK(hipSetDevice(dev));
  WC_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  WC_HIP_CHECK(hipStreamCreateWithFlags(&copy_s, hipStreamNonBlocking));
  n_cu = (uint32_t)device_cu_count(dev);
  numa = numa_of_device(dev);
  map_blocks = opt.map_blocks ? opt.map_blocks : MAP_BLOCKS_PER_CU * n_cu;
  map_blocks = std::min<uint32_t>(map_blocks, RED_MAX_RUNS);
  if (const char* e = std::getenv("WC_SYNC_DEBUG")) sync_debug = std::atoi(e) != 0;
  if (const char* e = std::getenv("WC_NO_SPECULATE")) speculate = std::atoi(e) == 0;
  if (const char* e = std::getenv("WC_SPIN_WAIT")) spin_wait = std::atoi(e) != 0;
  if (const char* e = std::getenv("WC_STAGE_EVENTS")) stage_events = std::atoi(e) != 0;
  if (const char* e = std::getenv("WC_HOST_CLOCK")) host_clock = std::atoi(e) != 0;
  if (const char* e = std::getenv("WC_FIRST_ORDER")) {
    order_radix = std::string(e) == "radix";
    order_bitmap = std::string(e) == "bitmap";
  }
  if (const char* e = std::getenv("WC_HOT_RESAMPLE_EVERY")) hot_resample_every = (uint32_t)std::atoi(e);
  k1_mask = k1_hash_mask(opt.k1_hash_bits);
  if (const char* e = std::getenv("WC_MAP_STAMPS"); e && std::atoi(e)) {
    dev_malloc(&d_stamps, MAP_STAMP_N * 8);
    WC_HIP_CHECK(hipMemset(d_stamps, 0, MAP_STAMP_N * 8));
    dev_malloc(&d_red_stamps, RED_STAMP_N * 8);
    WC_HIP_CHECK(hipMemset(d_red_stamps, 0, RED_STAMP_N * 8));
    dev_malloc(&d_hot_stamps, 32 * 8);
    WC_HIP_CHECK(hipMemset(d_hot_stamps, 0, 32 * 8));
    hot_setup_stamps(d_hot_stamps);
    red_blk_n = 16384;  // reduce grids up to this many blocks are profiled
    dev_malloc(&d_red_blk, red_blk_n * RED_BLK_WORDS * 8);
    WC_HIP_CHECK(hipMemset(d_red_blk, 0, red_blk_n * RED_BLK_WORDS * 8));
    dev_malloc(&d_blk, (size_t)map_blocks * 4 * 8);
    WC_HIP_CHECK(hipMemset(d_blk, 0, (size_t)map_blocks * 4 * 8));
  }

  if (const char* e = std::getenv("WC_REC_SHIFT")) rec_shift = (uint32_t)std::atoi(e);  // sweeps only
  if (const char* e = std::getenv("WC_RED_Q")) red_q_force = (uint32_t)std::atoi(e);    // sweeps only
  if (const char* e = std::getenv("WC_RED_PLAN")) red_plan = std::atoi(e) != 0;  // A/B: 0 = the uniform split
  if (const char* e = std::getenv("WC_LONG_DIRECT")) long_direct_force = std::atoi(e) != 0 ? 1 : 0;  // A/B
  long_direct = long_direct_force == 1;
  if (const char* e = std::getenv("WC_FAULT_OCC_UNDER")) fault_occ_under = std::strtoull(e, nullptr, 10);  // tests
  dev_malloc(&d_bounds, 64);
  WC_HIP_CHECK(hipMemset(d_bounds, 0, 64));
  if (const char* e = std::getenv("WC_CHECK_TABLE"); e && std::atoi(e)) {
    dev_malloc(&d_tab_err, 4 * sizeof(unsigned long long));
    WC_HIP_CHECK(hipMemset(d_tab_err, 0, 4 * sizeof(unsigned long long)));
  }
  {  // split-reduce partial tables: one per reduce block when buckets < CUs,
     // two per block of the balanced reduce (its grid is one block per CU)
    part_blocks = std::max<uint32_t>(n_cu, 256) + MAX_REC_BUCKETS;
    if (red_q_force) part_blocks = std::max<uint32_t>(part_blocks, 512u * red_q_force);  // sweeps: Q above 512 buckets
    const size_t rows = (size_t)part_blocks * TAB_SLOTS;
    part_mem.reserve(rows * (5 * 8 + 4) + part_blocks * 8 + rows * 12 + MAX_REC_BUCKETS * 4 + 16 * 256);
    part.k0 = part_mem.take_n<uint64_t>(rows);
    part.k1 = part_mem.take_n<uint64_t>(rows);
    part.cnt = part_mem.take_n<uint64_t>(rows);
    part.first = part_mem.take_n<uint64_t>(rows);
    part.soff = part_mem.take_n<uint64_t>(rows);
    part.slen = part_mem.take_n<uint32_t>(rows);
    part.n = part_mem.take_n<uint32_t>(part_blocks);
    part.qsoff = part_mem.take_n<uint64_t>(rows);
    part.qslen = part_mem.take_n<uint32_t>(rows);
    const size_t ndone = std::max<size_t>(part_blocks, MAX_REC_BUCKETS);  // indexed by bucket
    part.done = part_mem.take_n<uint32_t>(ndone);
    WC_HIP_CHECK(hipMemset(part.done, 0, ndone * sizeof(uint32_t)));
    dev_malloc(&d_bucket_w, MAX_REC_BUCKETS * sizeof(uint32_t));
  }
  if (const char* e = std::getenv("WC_LOG2_BUCKETS")) {  // sweeps only: shuffle + table bucket count
    opt.log2_rec_buckets = (uint32_t)std::atoi(e);
    opt.log2_tab_buckets = opt.log2_rec_buckets;
  }
  opt.log2_rec_buckets = std::min<uint32_t>(opt.log2_rec_buckets, MAX_REC_BUCKETS_LOG2);
  opt.max_log2_tab_buckets = std::min<uint32_t>(std::max<uint32_t>(opt.max_log2_tab_buckets, 1), 20);
  opt.log2_tab_buckets = std::max(opt.log2_tab_buckets, opt.log2_rec_buckets);
  opt.log2_tab_buckets = std::min(opt.log2_tab_buckets, opt.max_log2_tab_buckets);
  const uint64_t max_chunk = (1ull << 32) - 2 * (uint64_t)MAP_TILE;  // records carry u32 offsets
  opt.chunk_bytes = std::min<uint64_t>(std::max<uint64_t>(opt.chunk_bytes, MAP_TILE), max_chunk);
  opt.chunk_bytes = opt.chunk_bytes / MAP_TILE * MAP_TILE;

  if (const char* e = std::getenv("WC_RECORDS_PER_BYTE")) opt.records_per_byte = std::atof(e);  // sweeps only
  rec_total = std::max<uint64_t>(opt.min_records, (uint64_t)((double)opt.chunk_bytes * opt.records_per_byte));
  rec_total = std::min<uint64_t>(rec_total, 0xFFFFFFFFull);  // record indices are 32-bit in the reducer
  // record store + per-(block, bucket) counts; partitions follow the table up to the max
  const size_t ncount = (size_t)map_blocks * MAX_REC_BUCKETS;
  rec_mem.reserve(rec_total * (sizeof(Rec) + sizeof(Rec16)) + 2 * ncount * 4 + 8192);
  rec.recs = rec_mem.take_n<Rec>(rec_total);
  rec.recs16 = rec_mem.take_n<Rec16>(rec_total);
  rec.cap = rec_total;
  rec.count = rec_mem.take_n<uint32_t>(ncount);
  rec.count_long = rec_mem.take_n<uint32_t>(ncount);

  const size_t stage_n = (size_t)HOT_PARTS * map_blocks;
  hot_mem.reserve(stage_n * HOT_STAGE_CAP * sizeof(HotEnt) + stage_n * 4 +
                  (size_t)HOT_PARTS * HOT_PART_TOP * (20 + 64) + HOT_PARTS * 4 + MAP_SLOTS * 8 + 8192);
  hot.stage = hot_mem.take_n<HotEnt>(stage_n * HOT_STAGE_CAP);
  hot.stage_n = hot_mem.take_n<uint32_t>(stage_n);
  hot.cand_sig = hot_mem.take_n<uint64_t>((size_t)HOT_PARTS * HOT_PART_TOP);
  hot.cand_side = hot_mem.take_n<uint64_t>((size_t)HOT_PARTS * HOT_PART_TOP);
  hot.cand_cnt = hot_mem.take_n<uint32_t>((size_t)HOT_PARTS * HOT_PART_TOP);
  hot.cand_n = hot_mem.take_n<uint32_t>(HOT_PARTS);
  hot.maxb = map_blocks;
  hot.long_bytes = hot_mem.take_n<uint8_t>((size_t)HOT_PARTS * HOT_PART_TOP * 64);
  hot.image = hot_mem.take_n<uint64_t>(MAP_SLOTS);
  dev_malloc(&d_ctr, sizeof(DevCounters));
  WC_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&h_ctr), sizeof(DevCounters), hipHostMallocDefault));
  h_pass_seq.resize(256);
  std::memset(h_pass_seq.data(), 0, h_pass_seq.size());
  const size_t maxb = (size_t)1 << opt.max_log2_tab_buckets;
  dev_malloc(&d_bucket_ovf, maxb * sizeof(uint32_t));
  dev_malloc(&d_bucket_en, maxb);
  dev_malloc(&d_arena, std::max<uint64_t>(opt.arena_bytes, 16));
  dev_malloc(&d_arena_cursor, sizeof(unsigned long long));
  dev_malloc(&d_fo_hist, FO_LOGBINS * sizeof(uint32_t));
  dev_malloc(&d_fo_hist_cols, FO_LOGBINS * sizeof(uint32_t));
  WC_HIP_CHECK(hipMemsetAsync(d_fo_hist_cols, 0, FO_LOGBINS * sizeof(uint32_t), s));
  for (int i = 0; i < 2; ++i) {
    WC_HIP_CHECK(hipEventCreateWithFlags(&ev_h2d[i], hipEventDisableTiming));
    WC_HIP_CHECK(hipEventCreateWithFlags(&ev_done[i], hipEventDisableTiming));
  }
  tab[0].alloc(opt.log2_tab_buckets);
  cur = 0;
  launch_table_clear(table(), s);
  occ_valid = false;
  WC_HIP_CHECK(hipMemsetAsync(d_bucket_ovf, 0, maxb * sizeof(uint32_t), s));
  WC_HIP_CHECK(hipMemsetAsync(d_arena_cursor, 0, sizeof(unsigned long long), s));
  WC_HIP_CHECK(hipStreamSynchronize(s));
}

void Engine::Impl::hc_mark(int i) {
  if (!host_clock) return;
  const double t = now_seconds();
  // the interval since the previous milestone is credited to this one; a job's
  // start closes the caller's own turnaround since the previous job's end
  if (hc_prev > 0) hc_sum[i] += t - hc_prev;
  if (i == HC_DONE) ++hc_jobs;
  hc_prev = t;
}

Engine::Impl::~Impl() {
  (void)hipSetDevice(dev);
  if (host_clock && hc_jobs > 1) {
    const double n = (double)hc_jobs;
    fprintf(stderr,
            "[wc] host clock (us per job, %llu jobs): caller gap %.2f | reset %.2f | ->prelaunch %.2f | "
            "sample+merge+map launches %.2f | ->wait %.2f | wait %.2f | waited->done %.2f\n",
            (unsigned long long)hc_jobs, hc_sum[HC_START] / (n - 1) * 1e6, hc_sum[HC_RESET] / n * 1e6,
            hc_sum[HC_PRELAUNCH] / n * 1e6, hc_sum[HC_MAPPED] / n * 1e6, hc_sum[HC_WAIT] / n * 1e6,
            hc_sum[HC_WAITED] / n * 1e6, hc_sum[HC_DONE] / n * 1e6);
  }
  if (s) (void)hipStreamSynchronize(s);
  if (copy_s) (void)hipStreamSynchronize(copy_s);
  for (int i = 0; i < 2; ++i) {
    if (ev_h2d[i]) (void)hipEventDestroy(ev_h2d[i]);
    if (ev_done[i]) (void)hipEventDestroy(ev_done[i]);
  }
  for (hipEvent_t e : ev_pool) (void)hipEventDestroy(e);
  if (d_ctr) (void)hipFree(d_ctr);
  if (h_ctr) (void)hipHostFree(h_ctr);
  if (d_bucket_ovf) (void)hipFree(d_bucket_ovf);
  if (d_bucket_en) (void)hipFree(d_bucket_en);
  if (d_arena) (void)hipFree(d_arena);
  if (d_arena_cursor) (void)hipFree(d_arena_cursor);
  if (d_fo_hist) (void)hipFree(d_fo_hist);
  if (d_bucket_w) (void)hipFree(d_bucket_w);
  if (d_tab_err) (void)hipFree(d_tab_err);
  if (d_bounds) (void)hipFree(d_bounds);
  if (d_fo_hist_cols) (void)hipFree(d_fo_hist_cols);
  if (d_bm) (void)hipFree(d_bm);
  if (d_stamps) {
    unsigned long long h[MAP_STAMP_N];
    if (hipMemcpy(h, d_stamps, sizeof h, hipMemcpyDeviceToHost) == hipSuccess && h[MS_TOTAL]) {
      static const char* names[MS_TOTAL] = {"commit", "mask", "list", "keys", "probe",
                                            "slow",   "emit", "wait", "flush"};
      fprintf(stderr, "[wc] map phase clock (share of wave lifetime):");
      for (int i = 0; i < MS_TOTAL; ++i) fprintf(stderr, " %s=%.3f", names[i], (double)h[i] / h[MS_TOTAL]);
      fprintf(stderr, "; tokens: hot-table hits %llu, deferred LONG %llu, miss records %llu", h[MS_N_HIT],
              h[MS_N_DEFER], h[MS_N_DIRECT]);
      fprintf(stderr, "; slowest block / mean block = %.3f\n",
              h[MS_BLKSUM] ? (double)h[MS_BLKMAX] * blocks_stamped / (double)h[MS_BLKSUM] : 0.0);
    }
    (void)hipFree(d_stamps);
  }
  if (d_blk) {  // last map pass: block start skew / duration per XCC (100 MHz realtime ticks -> us)
    std::vector<unsigned long long> h((size_t)map_blocks * 4);
    if (hipMemcpy(h.data(), d_blk, h.size() * 8, hipMemcpyDeviceToHost) == hipSuccess && h[1]) {
      unsigned long long t0 = ~0ull, t1 = 0;
      for (uint32_t b = 0; b < map_blocks; ++b) {
        if (!h[4 * b + 1]) continue;
        t0 = std::min(t0, h[4 * b]);
        t1 = std::max(t1, h[4 * b + 1]);
      }
      fprintf(stderr, "[wc] map blocks (last pass): span %.1f us\n", (t1 - t0) / 100.0);
      for (int x = 0; x < 16; ++x) {
        double n = 0, st = 0, stmax = 0, du = 0, dumax = 0, dumin = 1e30, un = 0;
        for (uint32_t b = 0; b < map_blocks; ++b) {
          const unsigned long long* r = &h[4 * (size_t)b];
          if (!r[1] || (int)r[2] != x) continue;
          const double s0 = (r[0] - t0) / 100.0, d = (r[1] - r[0]) / 100.0;
          n += 1, st += s0, stmax = std::max(stmax, s0), du += d, dumax = std::max(dumax, d);
          dumin = std::min(dumin, d), un += (double)r[3];
        }
        if (n)
          fprintf(stderr,
                  "[wc]   xcc %d: %3.0f blocks, start mean %.1f max %.1f us, duration mean %.1f min %.1f max %.1f us, "
                  "unit grabs/block %.0f\n",
                  x, n, st / n, stmax, du / n, dumin, dumax, un / n);
      }
    }
    (void)hipFree(d_blk);
  }
  if (d_hot_stamps) {  // the per-job setup kernels' phases (max over blocks and jobs, us from block start)
    unsigned long long h[32];
    hot_setup_stamps(nullptr);
    if (hipMemcpy(h, d_hot_stamps, sizeof h, hipMemcpyDeviceToHost) == hipSuccess) {
      fprintf(stderr, "[wc] hot setup phases (us, max over blocks): sample init %.2f (unit loaded %.2f, counted %.2f) counted %.2f staged %.2f | "
              "merge init %.2f summed %.2f hist %.2f threshold %.2f candidates %.2f placed %.2f\n",
              h[1] / 100.0, h[4] / 100.0, h[5] / 100.0, h[2] / 100.0, h[3] / 100.0, h[17] / 100.0, h[18] / 100.0, h[19] / 100.0, h[20] / 100.0,
              h[21] / 100.0, h[22] / 100.0);
    }
    (void)hipFree(d_hot_stamps);
  }
  if (d_red_stamps) {
    unsigned long long h[RED_STAMP_N];
    if (hipMemcpy(h, d_red_stamps, sizeof h, hipMemcpyDeviceToHost) == hipSuccess && h[RS_RECORDS]) {
      fprintf(stderr,
              "[wc] reduce counters: records %llu, slow lanes %llu, slow wave-steps %llu, claim-loop iterations %llu, "
              "CAS failures %llu, PENDING re-reads %llu, claims %llu; run phase / wave lifetime = %.3f; blocks %llu, "
              "mean wave lifetime %.0f clk, slowest block %llu clk; record streams / wave lifetime = %.3f, LONG "
              "records %llu (%llu blocks past the LDS queue), LONG merges / wave lifetime = %.3f\n",
              h[RS_RECORDS], h[RS_SLOW_LANES], h[RS_SLOW_WAVES], h[RS_PROBE_ITERS], h[RS_CAS_FAIL], h[RS_PENDING],
              h[RS_CLAIMS], h[RS_T_WAVE] ? (double)h[RS_T_RUNS] / h[RS_T_WAVE] : 0.0, h[RS_BLOCKS],
              h[RS_BLOCKS] ? (double)h[RS_T_WAVE] / (h[RS_BLOCKS] * (RED_THREADS / 64)) : 0.0, h[RS_T_BLKMAX],
              h[RS_T_WAVE] ? (double)h[RS_T_STREAMS] / h[RS_T_WAVE] : 0.0, h[RS_NLONG], h[RS_LONG_STREAMED],
              h[RS_T_WAVE] ? (double)h[RS_T_SLOW] / h[RS_T_WAVE] : 0.0);
    }
    (void)hipFree(d_red_stamps);
  }
  if (d_red_blk && red_blk_grid) {  // the last reduce launch, block by block (100 MHz realtime ticks -> us)
    std::vector<unsigned long long> h(red_blk_grid * RED_BLK_WORDS);
    if (hipMemcpy(h.data(), d_red_blk, h.size() * 8, hipMemcpyDeviceToHost) == hipSuccess) {
      struct B { double start, dur; uint32_t b, q; unsigned long long n16, n24, nl; double streams, arrive, merged, stored; };
      std::vector<B> v;
      unsigned long long t0 = ~0ull, t1 = 0;
      for (size_t i = 0; i < red_blk_grid; ++i) {
        const unsigned long long* r = &h[i * RED_BLK_WORDS];
        if (!r[2]) continue;
        t0 = std::min(t0, r[1]);
        t1 = std::max(t1, r[2]);
        v.push_back(B{(double)r[1], (r[2] - r[1]) / 100.0, (uint32_t)r[0], (uint32_t)(r[0] >> 32), r[3] & 0xFFFFFFFFull,
                      r[3] >> 32, r[4], (r[5] - r[1]) / 100.0, (r[6] - r[1]) / 100.0, (r[7] - r[1]) / 100.0,
                      (r[8] - r[1]) / 100.0});
      }
      if (!v.empty()) {
        double sum = 0;
        for (auto& x : v) sum += x.dur;
        std::sort(v.begin(), v.end(), [](const B& a, const B& b) { return a.dur > b.dur; });
        fprintf(stderr, "[wc] reduce blocks (last launch): %zu blocks, span %.1f us, duration mean %.1f max %.1f us\n",
                v.size(), (t1 - t0) / 100.0, sum / v.size(), v[0].dur);
        const size_t show = std::getenv("WC_RED_BLK_ALL") ? v.size() : 8;  // tools/red_blocks.sh: every block
        for (size_t i = 0; i < v.size() && i < show; ++i)
          fprintf(stderr,
                  "[wc]   #%zu bucket %u q %u: %.1f us from %.1f us, records 16B %llu 24B %llu, LONG %llu; streams end "
                  "%.1f, arrival %.1f, merged %.1f, stored %.1f us\n",
                  i, v[i].b, v[i].q, v[i].dur, (v[i].start - t0) / 100.0, v[i].n16, v[i].n24, v[i].nl, v[i].streams,
                  v[i].arrive, v[i].merged, v[i].stored);
        double m16 = 0, m24 = 0, ml = 0;
        for (auto& x : v) m16 += x.n16, m24 += x.n24, ml += (double)x.nl;
        fprintf(stderr, "[wc]   mean records 16B %.0f 24B %.0f LONG %.0f\n", m16 / v.size(), m24 / v.size(),
                ml / v.size());
      }
    }
  }
  if (d_red_blk) (void)hipFree(d_red_blk);
  if (registered) (void)hipHostUnregister(const_cast<uint8_t*>(registered));
  if (s) (void)hipStreamDestroy(s);
  if (copy_s) (void)hipStreamDestroy(copy_s);
}

void Engine::Impl::ensure_text(uint64_t n) {
  const uint64_t need = (n + 4095) / 4096 * 4096 + 4096;
  if (need > text_cap || !d_text) {
    text_mem.reserve(need);
    d_text = static_cast<uint8_t*>(text_mem.take(need));
    text_cap = need;
  }
}

// Own allocation: the resident text (synth_device, count_resident) stays valid
// while streaming sources use the staging pair, in either order.
void Engine::Impl::ensure_staging(uint64_t chunk) {
  if (d_stage[0] && stage_cap >= chunk && pinned.size() >= 2 && pinned[0].size() >= chunk) return;
  const uint64_t per = (chunk + 4096 + 255) / 256 * 256;  // + read-ahead slack past the chunk
  stage_mem.reserve(2 * per);
  stage_mem.reset();
  d_stage[0] = static_cast<uint8_t*>(stage_mem.take(per));
  d_stage[1] = static_cast<uint8_t*>(stage_mem.take(per));
  stage_cap = chunk;
  pinned.clear();
  ScopedAffinity bind(numa.cpus);  // the staging ring's pages on the GPU's node
  const uint32_t nring = std::max<uint32_t>(2, opt.staging_buffers);
  for (uint32_t i = 0; i < nring; ++i) pinned.emplace_back(chunk);
}

uint32_t Engine::Impl::blocks_for(uint64_t len) const {
  const uint64_t tiles = (len + MAP_TILE - 1) / MAP_TILE;
  return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(map_blocks, tiles));
}

void Engine::Impl::launch_pass(const uint8_t* text, uint64_t len, uint64_t avail, uint64_t base, int prev,
                               uint32_t log2_rb, uint32_t blocks, bool copy_occupancy, bool defer_publish) {
  WC_CHECK((reinterpret_cast<uintptr_t>(text) & 15) == 0, "chunk text must be 16-byte aligned");
  mark(EV_PASS);
  // one zeroing launch: pass counters and, after a reset, the
  // table occupancy and the key-arena cursor
  // reuse the job's hot-table image while it keeps its hit rate (the previous
  // pass's miss share vs that of the pass that sampled it)
  const bool sample = !hot_valid || hot_resample_every == 0 || hot_age >= hot_resample_every ||
                      hot_miss_last > hot_miss_ref * hot_resample_slack;
  pass_sampled = sample;
  // The last pass of a job, with its finalize launched right behind it: the
  // finalize's order is known now.  Unless the sample sort will run, the
  // reducer's key histogram is useless (~1M device atomics at 1M keys); for
  // the bitmap-rank order the reducer sets the keys' bits instead.
  bool want_hist = true;
  unsigned long long* bm = nullptr;
  uint64_t bm_end = 0;
  if (defer_publish) {
    drop_reduce_bits();
    const uint64_t hint = spec_hint();
    if (!sample_order(hint)) {
      want_hist = false;
      if (bitmap_order_ok(hint)) {
        bm_end = std::max(max_end, base + len);
        max_end = bm_end;  // the order's key width (the finalize reads the same value)
        bm = ensure_bitmap();
        bm_in_reduce = true;
      }
    }
  }
  // the reduce's dispatch plan (heavy buckets split, pieces heaviest first)
  // for tables of >= CUs buckets: one record bucket per table bucket (no
  // split since the records were bucketed), its weights from this map.
  // Below CUs buckets the uniform split stays: weight-sized pieces at 2 per CU
  // cost 11 % more block time in partial tables than their balance saved
  // (v100k reduce 0.244 -> 0.307 ms; profiles/r5_session.md §4)
  const uint32_t nbk = 1u << table().log2_buckets;
  const uint32_t plan_grid = nbk + RED_PLAN_EXTRA;
  const bool planned = red_plan && !red_q_force && nbk >= n_cu && log2_rb == table().log2_buckets &&
                       nbk <= (uint32_t)MAX_REC_BUCKETS && plan_grid <= part_blocks;
  const uint32_t plan_extra = plan_grid - nbk;
  ZeroList z{};
  z.add(d_ctr, sizeof(DevCounters));
  if (planned) z.add(d_bucket_w, nbk * sizeof(uint32_t));
  if (want_hist) z.add(d_fo_hist, FO_LOGBINS * sizeof(uint32_t));  // rebuilt by this pass's reduce over the whole table
  {
    uint32_t kb = 1;
    while (kb < 64 && (std::max(max_end, base + len) >> kb) != 0) ++kb;
    fo_hist_m = fo_mbits(kb);
    fo_hist_ok = want_hist;
  }
  if (reset_pending) {
    z.add(table().occupancy, ((size_t)1 << table().log2_buckets) * 4);
    z.add(d_arena_cursor, sizeof(unsigned long long));
    reset_pending = false;
  }
  // the last pass of a job whose finalize will likely run the planned merge
  // again: its zeroing rides here (merge_cols_planned skips its launch if the
  // list it needs is this one)
  // (not under WC_POISON=2: the arenas' reset poisons the regions after this)
  merge_zero_pre = false;
  if (defer_publish && merge_zero_last_valid && merge_caps.valid && merge_zero_gen == merge_arena_gen() &&
      poison_level() < 2) {
    z.append_fills(merge_zero_last);
    merge_zero_pre = true;
  }
  pass_rec = rec;
  pass_rec.cursor = &d_ctr->records;
  pass_rec.subcap = (uint32_t)std::min<uint64_t>(rec.cap / ((uint64_t)blocks << log2_rb), 0xFFFFull);
  WC_CHECK(pass_rec.subcap > 0, "shuffle record capacity below one record per (map block, bucket)");
  MapArgs m{text,     len,          avail,          prev,     log2_rb, pass_rec, d_ctr->flags, &d_ctr->tokens,
            k1_mask,  d_stamps,     d_blk,          planned ? d_bucket_w : nullptr};
  pass_ld = long_direct;
  m.long_direct = pass_ld;
  m.long_tokens = &d_ctr->long_tokens;
  if (d_stamps) blocks_stamped += blocks;
  hot.text = text;
  hot.nblk = blocks;
  hc_mark(HC_PRELAUNCH);
  launch_map(m, hot, blocks, s, sample, z);  // z applied first (inside the sampling launch)
  hc_mark(HC_MAPPED);
  mark(EV_MAP);
  if (sync_debug) {  // WC_SYNC_DEBUG: attribute a device fault to a kernel and a chunk
    const hipError_t e = hipStreamSynchronize(s);
    fprintf(stderr, "[wc] map    base=%llu len=%llu avail=%llu blocks=%u subcap=%u -> %s\n", (unsigned long long)base,
            (unsigned long long)len, (unsigned long long)avail, blocks, pass_rec.subcap, hipGetErrorString(e));
    WC_HIP_CHECK(e);
  }
  ReduceArgs ra{pass_rec, blocks,       log2_rb,       table(), text,
                avail,    base,         Arena{d_arena, d_arena_cursor, opt.arena_bytes},
                d_ctr->flags, d_bucket_ovf, nullptr, d_red_stamps, red_blk(), want_hist ? d_fo_hist : nullptr, fo_hist_m,
                bm, bm ? bitmap_order_linecnt(bm, bm_end, 1) : nullptr, bm ? bitmap_order_ctl(bm, bm_end, 1) : nullptr,
                bm ? (bm_end >> 1) + 1 : 0, 1u, planned ? 1u : red_q(), planned ? d_bucket_w : nullptr, part,
                part_blocks};
  ra.long_direct = pass_ld;
  if (planned && ra.blk) red_blk_grid = nbk + plan_extra;
  launch_reduce(ra, s, plan_extra);
  check_table("the reduce");
  if (sync_debug) {
    const hipError_t e = hipStreamSynchronize(s);
    fprintf(stderr, "[wc] reduce base=%llu buckets=%u -> %s\n", (unsigned long long)base, 1u << table().log2_buckets,
            hipGetErrorString(e));
    WC_HIP_CHECK(e);
  }
  // counters (+ occupancy and arena cursor, read at finalize without a sync of
  // their own) into pinned memory: one launch
  PubList c{};
  c.add(h_ctr, d_ctr, sizeof(DevCounters));
  occ_copied = false;
  if (copy_occupancy) add_occupancy(c);
  if (spin_wait) {  // complete_pass spins on it instead of a stream sync
    c.seq_dst = reinterpret_cast<uint32_t*>(h_pass_seq.data());
    c.seq = ++pass_seq;
  }
  pass_pub = c;
  pass_pub_pending = true;
  if (!defer_publish) flush_pass_publish();
  mark(EV_REDUCE);
}

void Engine::Impl::check_table(const char* where) {
  if (!d_tab_err) return;
  launch_check_table(table(), d_tab_err, s);
  unsigned long long h[4] = {};
  WC_HIP_CHECK(hipMemcpyAsync(h, d_tab_err, sizeof h, hipMemcpyDeviceToHost, s));
  WC_HIP_CHECK(hipStreamSynchronize(s));
  if (h[0])
    fail(std::string("WC_CHECK_TABLE: table invariant broken after ") + where + ": bucket " + std::to_string(h[0] - 1) +
         " of " + std::to_string(1u << table().log2_buckets) + " holds " + std::to_string(h[1]) + " keys, occupancy " +
         std::to_string(h[2]) + ", " + std::to_string(h[3]) + " misplaced");
}

// A finalize writer met a row at or past its buffer's capacity (the word
// published with the finalize's last wait): the row was not written, so the
// output is incomplete — fail, naming the kernel and the row, and re-arm.
void Engine::Impl::check_bounds(uint64_t word, const char* where) {
  if (!word) return;
  WC_HIP_CHECK(hipMemsetAsync(d_bounds, 0, 8, s));
  if (d_bm) WC_HIP_CHECK(hipMemsetAsync(d_bm, 0, bm_words * 8, s));  // rows not emitted left their bits set
  WC_HIP_CHECK(hipStreamSynchronize(s));
  fail(std::string("bounds guard: ") + bounds_kernel_name((uint32_t)(word >> 56)) + " reached row " +
       std::to_string(word & ((1ull << 56) - 1)) + " past its buffer's capacity in " + where +
       " (the key count it was sized for is short; output discarded)");
}

void Engine::Impl::flush_pass_publish() {
  if (!pass_pub_pending) return;
  pass_pub_pending = false;
  launch_publish(pass_pub, s);
}

void Engine::Impl::mark(int tag) {
  if (!stage_events || ev_n >= 8192) return;  // a 1 TB job: ~400 marks
  if (ev_n == ev_pool.size()) {
    // timing only (read by stats() after the job's last wait): no system-scope
    // release at the record.  A record still costs the GPU ~4.5 us between two
    // kernels (its barrier packet; a one-thread stamp kernel measured the same:
    // every dispatch reaches all 8 XCDs), so the bench times its steps with the
    // marks off (set_stage_events) and takes the stage split from one more step.
    hipEvent_t e;
    WC_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
    ev_pool.push_back(e);
    ev_tag.push_back(0);
  }
  WC_HIP_CHECK(hipEventRecord(ev_pool[ev_n], s));
  ev_tag[ev_n++] = tag;
}

// Called once the job's work has completed (stats()): elapsed time between
// consecutive marks, charged to the stage the later mark closes.
void Engine::Impl::collect_stage_times() {
  if (ev_n < 2) return;
  double t[EV_FIN_END + 1] = {};
  for (size_t i = 1; i < ev_n; ++i) {
    float ms = 0;
    if (hipEventElapsedTime(&ms, ev_pool[i - 1], ev_pool[i]) != hipSuccess) {
      (void)hipGetLastError();
      return;  // not complete (a pass still pending): keep the previous values
    }
    t[ev_tag[i]] += ms;
  }
  st.map_ms = t[EV_MAP];
  st.reduce_ms = t[EV_REDUCE];
  st.merge_ms = t[EV_MERGE1];
  st.finalize_ms = t[EV_MERGE0] + t[EV_FIN_END];
  st.idle_ms = t[EV_PASS] + t[EV_FIN];
  st.device_ms = st.map_ms + st.reduce_ms + st.merge_ms + st.finalize_ms + st.idle_ms;
}

void Engine::Impl::drop_reduce_bits() {
  if (!bm_in_reduce) return;
  bm_in_reduce = false;
  WC_HIP_CHECK(hipMemsetAsync(d_bm, 0, bm_words * sizeof(unsigned long long), s));  // bits + control word
}

uint64_t Engine::Impl::spec_hint() {
  const uint64_t cap = ((uint64_t)1 << table().log2_buckets) * TAB_SLOTS;
  return std::min<uint64_t>(cap, last_keys ? last_keys + last_keys / 8 + 1024 : cap / 4);
}

void Engine::Impl::settle() {
  drop_reduce_bits();  // a pending pass completed by anything but the speculative local finalize
  if (!pend.active) return;
  const PendingPass p = pend;
  pend.active = false;
  complete_pass(p.text, p.len, p.avail, p.base, p.prev, p.rb, p.blocks);
}

void Engine::Impl::add_occupancy(PubList& c) {
  occ_copied = true;
  const size_t nb = (size_t)1 << table().log2_buckets;
  if (h_occ.size() < nb * 4 + 8) h_occ.resize(std::max<size_t>(nb * 4 + 8, 4096));
  c.add(h_occ.data() + 8, table().occupancy, nb * 4);
  c.add(h_occ.data(), d_arena_cursor, 8);
}

void Engine::Impl::enqueue_occupancy() {
  PubList c{};
  add_occupancy(c);
  launch_publish(c, s);
}

// Wait for a publish launch's sequence word: a host spin on page-locked memory
// wakes within a microsecond of the kernel's store, where a stream sync waits
// for the completion signal and the runtime's wake-up (~20-30 us of GPU idle
// per job, profiles/r2_plumbing.md).  The stream is polled now and then so a
// device fault still surfaces as an error; the stream sync at the end returns
// at once (everything before the publish launch has completed).
void Engine::Impl::wait_published(const uint32_t* seq, uint32_t want) {
  for (uint64_t it = 1;; ++it) {
    if (__atomic_load_n(seq, __ATOMIC_ACQUIRE) == want) break;
    if ((it & 0xFFFF) == 0) {
      const hipError_t e = hipStreamQuery(s);
      if (e != hipErrorNotReady) {
        WC_HIP_CHECK(e);
        if (__atomic_load_n(seq, __ATOMIC_ACQUIRE) != want) fail("publish launch completed without its sequence word");
        break;
      }
    }
    __builtin_ia32_pause();
  }
}

void Engine::Impl::apply_reset() {
  if (!reset_pending) return;
  ZeroList z{};
  z.add(table().occupancy, ((size_t)1 << table().log2_buckets) * 4);
  z.add(d_arena_cursor, sizeof(unsigned long long));
  launch_zero_regions(z, s);
  reset_pending = false;
}

// Bucket offsets and key count from the occupancy copied with the last pass's
// counters (that pass synced); a stale copy (table split or cleared since) is
// refreshed with one sync.
uint64_t Engine::Impl::host_occupancy(uint64_t*& boff, uint64_t& arena_used) {
  const size_t nb = (size_t)1 << table().log2_buckets;
  if (!occ_valid) {
    enqueue_occupancy();
    WC_HIP_CHECK(hipStreamSynchronize(s));
    occ_valid = true;
  }
  const uint32_t* occ = reinterpret_cast<const uint32_t*>(h_occ.data() + 8);
  std::memcpy(&arena_used, h_occ.data(), 8);
  if (h_boff.size() < nb * 8) h_boff.resize(nb * 8);
  boff = reinterpret_cast<uint64_t*>(h_boff.data());
  uint64_t n = 0;
  for (size_t b = 0; b < nb; ++b) {
    boff[b] = n;
    n += occ[b];
  }
  return n - std::min(n, fault_occ_under);
}

void Engine::Impl::split_table() {
  const uint32_t lg = table().log2_buckets;
  if (lg >= opt.max_log2_tab_buckets)
    fail("vocabulary exceeds the key table (" + std::to_string(((size_t)1 << lg) * TAB_MAX_OCC) +
         " keys); raise max_log2_tab_buckets");
  TableStore& dst = tab[cur ^ 1];
  dst.alloc(lg + 1);
  occ_valid = false;
  launch_table_clear(dst.v, s);
  launch_table_split(table(), dst.v, s);
  cur ^= 1;
  check_table("a table split");
  st.table_splits++;
  WC_LOG(LOG_INFO, "dev %d: key table split %u -> %u buckets", dev, 1u << lg, 2u << lg);
}

bool Engine::Impl::complete_pass(const uint8_t* text, uint64_t len, uint64_t avail, uint64_t base, int prev,
                                 uint32_t log2_rb, uint32_t blocks, bool synced) {
  // the pass's publish launch (counters, occupancy) is what this needs: spin on
  // its sequence word; later work already on the stream keeps running
  if (pass_pub_pending) {  // still held back: launch it now and wait for it
    flush_pass_publish();
    synced = false;
  }
  if (!synced) {
    if (spin_wait) wait_published(reinterpret_cast<const uint32_t*>(h_pass_seq.data()), pass_seq);
    else WC_HIP_CHECK(hipStreamSynchronize(s));
  }
  DevCounters c = *h_ctr;
  if (c.flags[FLAG_REGION_OVF]) {
    // Shuffle regions too small for this chunk's record skew: the reduce was
    // skipped (table untouched), so re-run exactly this chunk, smaller.
    st.map_reruns++;
    WC_LOG(LOG_INFO, "dev %d: shuffle region overflow at base=%llu len=%llu -> re-run in halves", dev,
           (unsigned long long)base, (unsigned long long)len);
    auto run = [&](const uint8_t* t, uint64_t l, uint64_t av, uint64_t b, int pv, uint32_t rb) {
      const uint32_t bl = blocks_for(l);
      launch_pass(t, l, av, b, pv, rb, bl);
      complete_pass(t, l, av, b, pv, rb, bl);
    };
    if (len > (uint64_t)MAP_TILE) {
      const uint64_t h = std::max<uint64_t>(MAP_TILE, (len / 2) / MAP_TILE * MAP_TILE);
      run(text, h, avail, base, prev, log2_rb);
      run(text + h, len - h, avail - h, base + h, -1, log2_rb);
    } else if (log2_rb > 0) {
      run(text, len, avail, base, prev, 0);
    } else {
      fail("shuffle record capacity too small for a single tile");
    }
    return false;
  }
  const uint64_t tokens = c.tokens;
  st.records += c.records;
  st.long_tokens += c.long_tokens;
  st.long_direct = pass_ld ? 1u : 0u;
  // the next pass's LONG-record layout, from this pass's LONG share
  long_direct = long_direct_force >= 0 ? long_direct_force == 1 : c.long_tokens * 64 > c.records;
  {  // hot-table reuse bookkeeping (see launch_pass)
    const double miss = tokens ? (double)c.records / (double)tokens : 0.0;
    if (pass_sampled) {
      hot_valid = true;
      hot_miss_ref = miss;
      hot_age = 0;
    }
    hot_miss_last = miss;
    ++hot_age;
  }
  uint32_t max_occ = c.flags[FLAG_MAX_OCC];
  const bool clean = !c.flags[FLAG_TABLE_OVF];
  while (c.flags[FLAG_TABLE_OVF]) {
    if (c.flags[FLAG_ARENA_OVF]) break;
    const uint32_t lg = table().log2_buckets;
    std::vector<uint32_t> ovf((size_t)1 << lg);
    WC_HIP_CHECK(hipMemcpy(ovf.data(), d_bucket_ovf, ovf.size() * 4, hipMemcpyDeviceToHost));
    split_table();
    std::vector<uint8_t> en(ovf.size() * 2);
    for (size_t b = 0; b < en.size(); ++b) en[b] = ovf[b & (ovf.size() - 1)] ? 1 : 0;  // parent = b mod B
    WC_HIP_CHECK(hipMemcpyAsync(d_bucket_en, en.data(), en.size(), hipMemcpyHostToDevice, s));
    WC_HIP_CHECK(hipMemsetAsync(d_bucket_ovf, 0, en.size() * 4, s));
    WC_HIP_CHECK(hipMemsetAsync(d_ctr, 0, sizeof(DevCounters), s));
    ReduceArgs ra{pass_rec, blocks,       log2_rb,       table(), text,
                  avail,    base,         Arena{d_arena, d_arena_cursor, opt.arena_bytes},
                  d_ctr->flags, d_bucket_ovf, d_bucket_en, d_red_stamps, red_blk(), fo_hist_ok ? d_fo_hist : nullptr, fo_hist_m,
                  nullptr, nullptr, nullptr, 0, 0u, red_q(), nullptr, part, part_blocks};
    ra.long_direct = pass_ld;  // the pass's records: its map's LONG layout
    launch_reduce(ra, s);
    check_table("a split re-run's reduce");
    PubList pc{};
    pc.add(h_ctr, d_ctr, sizeof(DevCounters));
    add_occupancy(pc);
    launch_publish(pc, s);
    WC_HIP_CHECK(hipStreamSynchronize(s));
    c = *h_ctr;
    max_occ = std::max(max_occ, c.flags[FLAG_MAX_OCC]);
  }
  if (c.flags[FLAG_ARENA_OVF])
    fail("key arena exhausted (" + std::to_string(opt.arena_bytes) + " bytes); raise arena_bytes");
  st.tokens += tokens;
  st.chunks++;
  WC_LOG(LOG_DEBUG, "dev %d: chunk base=%llu len=%llu blocks=%u tokens=%llu records=%llu", dev,
         (unsigned long long)base, (unsigned long long)len, blocks, (unsigned long long)tokens,
         (unsigned long long)c.records);
  max_end = std::max(max_end, base + len);
  occ_valid = occ_copied;  // occupancy copies enqueued with this pass's counters completed at its sync
  if (max_occ >= (uint32_t)TAB_SPLIT_AT && table().log2_buckets < opt.max_log2_tab_buckets) split_table();
  return clean;
}

void Engine::Impl::process_chunk(const uint8_t* text, uint64_t len, uint64_t avail, uint64_t base, int prev,
                                 bool last) {
  settle();
  const uint32_t blocks = blocks_for(len);
  const uint32_t rb = rec_buckets_log2();
  if (last && speculate && !sync_debug) {
    launch_pass(text, len, avail, base, prev, rb, blocks, false, true);
    pend = PendingPass{true, text, len, avail, base, prev, rb, blocks};
    occ_valid = false;
    max_end = std::max(max_end, base + len);  // the sort key width of the speculative finalize
    return;
  }
  launch_pass(text, len, avail, base, prev, rb, blocks);
  complete_pass(text, len, avail, base, prev, rb, blocks);
}

unsigned long long* Engine::Impl::ensure_bitmap() {
  const size_t words = bitmap_order_words(max_end, 1);
  if (words > bm_words) {
    if (d_bm) WC_HIP_CHECK(hipFree(d_bm));  // waits for the device: nothing in flight reads it
    d_bm = nullptr;
    const size_t w = words + words / 4;  // room for a growing input
    dev_malloc(&d_bm, w * 8);
    WC_HIP_CHECK(hipMemsetAsync(d_bm, 0, w * 8, s));  // once: every bitmap_order leaves it zeroed
    bm_words = w;
  }
  return d_bm;
}

void Engine::Impl::compact_local() {
  Range r("wc_finalize_compact");
  const TableView& t = table();
  const size_t nb = (size_t)1 << t.log2_buckets;
  uint64_t* boff = nullptr;
  uint64_t arena_used = 0;
  const uint64_t n = host_occupancy(boff, arena_used);
  // columns x2 (sorted copy) + sort scratch + hist
  const size_t per = 5 * 8 + 4;
  fin_mem.reserve(std::max<size_t>(1 << 20, (n + 1) * per + nb * 8 + radix_hist_words(n) * 4 + 64 * 1024));
  fin_mem.reset();
  cols = KeyCols{};
  cols.k0 = fin_mem.take_n<uint64_t>(n + 1);
  cols.k1 = fin_mem.take_n<uint64_t>(n + 1);
  cols.cnt = fin_mem.take_n<uint64_t>(n + 1);
  cols.first = fin_mem.take_n<uint64_t>(n + 1);
  cols.sref_off = fin_mem.take_n<uint64_t>(n + 1);
  cols.sref_len = fin_mem.take_n<uint32_t>(n + 1);
  uint64_t* d_boff = fin_mem.take_n<uint64_t>(nb);
  WC_HIP_CHECK(hipMemcpyAsync(d_boff, boff, nb * 8, hipMemcpyHostToDevice, s));  // pinned: no sync needed
  launch_table_compact(t, d_boff, cols.k0, cols.k1, cols.cnt, cols.first, cols.sref_off, cols.sref_len, s,
                       bounds(n + 1));
  cols.n = n;
  cols_arena = d_arena;
  cols_arena_bytes = std::min<uint64_t>(arena_used, opt.arena_bytes);
  st.keys = n;
  st.log2_buckets = t.log2_buckets;
}

// The local finalize launched right behind a pending pass, with no host round
// trip: bucket offsets and the key count are computed on the device, the sort
// and gather are sized for the table's capacity and run on the device count.
// One sync at the end covers the pass counters too; if the pass needed
// recovery (re-runs / splits) the result is discarded (returns false).
bool Engine::Impl::finalize_local_speculative() {
  Range r("wc_finalize_speculative");
  const PendingPass p = pend;
  pend.active = false;
  const TableView& t = table();
  const size_t nb = (size_t)1 << t.log2_buckets;
  const uint64_t cap = (uint64_t)nb * TAB_SLOTS;
  const uint64_t hint = spec_hint();  // the same hint launch_pass chose the reducer's extras from
  const bool sample = sample_order(hint);  // sized for the hint; a far larger count -> overflow -> redo
  const bool bitmap = !sample && bitmap_order_ok(hint);
  if (!bitmap) drop_reduce_bits();  // (cannot be set: the same hint decided the pass's extras)
  OrderSrc src{};
  src.table = true;
  src.t = t;
  DeviceArena& A = sort_mem;
  A.reserve((cap + 1) * (5 * 8 + 4) + 64 * 1024 +
            (sample   ? first_order_ws_bytes(src, hint)
             : bitmap ? bitmap_order_ws_bytes(cap + 1, max_end, 1)
                      : (cap + 1) * (2 * 8 + 2 * 4) + nb * 8 + radix_hist_words(cap, hint) * 4));
  unsigned long long* bm = bitmap ? ensure_bitmap() : nullptr;
  A.reset();
  uint64_t* d_n = A.take_n<uint64_t>(2);
  KeyCols o;
  o.k0 = A.take_n<uint64_t>(cap + 1);
  o.k1 = A.take_n<uint64_t>(cap + 1);
  o.cnt = A.take_n<uint64_t>(cap + 1);
  o.first = A.take_n<uint64_t>(cap + 1);
  o.sref_off = A.take_n<uint64_t>(cap + 1);
  o.sref_len = A.take_n<uint32_t>(cap + 1);
  uint32_t* ovf = nullptr;
  if (sample) {
    ovf = first_order(src, OrderDst{o.k0, o.k1, o.cnt, o.first, o.sref_off, o.sref_len, bounds(cap + 1)}, hint, key_bits(),
                      A.take_n<uint8_t>(first_order_ws_bytes(src, hint)), d_n, s, fo_hist_ok ? d_fo_hist : nullptr,
                      fo_hist_m);
  } else if (bitmap) {
    ovf = bitmap_order(src, OrderDst{o.k0, o.k1, o.cnt, o.first, o.sref_off, o.sref_len, bounds(cap + 1)}, cap, max_end,
                       1, bm,
                       A.take_n<uint8_t>(bitmap_order_ws_bytes(cap + 1, max_end, 1)), d_n, s, bm_in_reduce);
    bm_in_reduce = false;  // consumed (the order leaves the bitmap zeroed, a failed pass included)
  } else {
    uint64_t* d_boff = A.take_n<uint64_t>(nb);
    uint64_t* keys = A.take_n<uint64_t>(cap + 1);
    uint64_t* tkeys = A.take_n<uint64_t>(cap + 1);
    uint32_t* slots = A.take_n<uint32_t>(cap + 1);
    uint32_t* tslots = A.take_n<uint32_t>(cap + 1);
    uint32_t* hist = A.take_n<uint32_t>(radix_hist_words(cap, hint));
    launch_bucket_offsets(t.occupancy, (uint32_t)nb, d_boff, d_n, s);
    launch_table_keys(t, d_boff, keys, slots, s, bounds(cap + 1));
    int bits = 1;
    while (bits < 64 && (max_end >> bits) != 0) ++bits;
    bool in_tmp = false;
    radix_sort_pairs(keys, slots, tkeys, tslots, hist, cap, bits, s, &in_tmp, d_n, hint);
    launch_gather_table(t, in_tmp ? tkeys : keys, in_tmp ? tslots : slots, cap, o.k0, o.k1, o.cnt, o.first,
                        o.sref_off, o.sref_len, s, d_n, bounds(cap + 1));
  }
  if (h_spec.size() < 32) {
    h_spec.resize(4096);
    std::memset(h_spec.data(), 0, h_spec.size());  // the sequence word starts below every spec_seq
  }
  mark(EV_FIN_END);
  fin_end_marked = true;
  PubList pc{};
  if (pass_pub_pending) {  // the pass's counters ride in this launch (complete_pass below reads them)
    pass_pub_pending = false;
    for (int i = 0; i < pass_pub.n; ++i) pc.add(pass_pub.dst[i], pass_pub.src[i], (uint64_t)pass_pub.words[i] * 4);
  }
  pc.add(h_spec.data(), d_n, 8);
  pc.add(h_spec.data() + 8, d_arena_cursor, 8);
  pc.add(h_spec.data() + 40, d_bounds, 8);
  uint32_t* seq = reinterpret_cast<uint32_t*>(h_spec.data() + 16);
  uint32_t* h_ovf = reinterpret_cast<uint32_t*>(h_spec.data() + 24);
  *h_ovf = 0;
  if (ovf) pc.add(h_ovf, ovf, 4);
  if (spin_wait) {
    pc.seq_dst = seq;
    pc.seq = ++spec_seq;
  }
  launch_publish(pc, s);
  hc_mark(HC_WAIT);
  if (spin_wait) wait_published(seq, spec_seq);
  else WC_HIP_CHECK(hipStreamSynchronize(s));
  hc_mark(HC_WAITED);
  // the pass's counters arrived with this sync: check it (stats, recovery).  A
  // discarded attempt re-arms the bounds word: whatever it recorded belongs to
  // output that is thrown away, not to the redo that publishes it next
  if (!complete_pass(p.text, p.len, p.avail, p.base, p.prev, p.rb, p.blocks, true)) {
    WC_HIP_CHECK(hipMemsetAsync(d_bounds, 0, 8, s));
    return false;
  }
  if (*h_ovf) {  // a sample-sort bin overflowed (far more keys than the hint) / shared bitmap position: redo exactly
    WC_LOG(LOG_INFO, "dev %d: first-occurrence %s order overflowed (hint %llu keys); redoing", dev,
           bitmap ? "bitmap" : "sample", (unsigned long long)hint);
    last_keys = 0;
    order_redo = true;
    WC_HIP_CHECK(hipMemsetAsync(d_bounds, 0, 8, s));
    return false;
  }
  uint64_t bw = 0;
  std::memcpy(&bw, h_spec.data() + 40, 8);
  check_bounds(bw, "the speculative local finalize");
  uint64_t n = 0, arena_used = 0;
  std::memcpy(&n, h_spec.data(), 8);
  std::memcpy(&arena_used, h_spec.data() + 8, 8);
  o.n = n;
  cols = o;
  cols_arena = d_arena;
  cols_arena_bytes = std::min<uint64_t>(arena_used, opt.arena_bytes);
  st.keys = n;
  st.log2_buckets = t.log2_buckets;
  st.order_path = sample ? 1 : bitmap ? 5 : 2;
  last_keys = n;
  return true;
}

void Engine::Impl::finalize_local_sorted() {
  Range r("wc_finalize_local");
  const TableView& t = table();
  const size_t nb = (size_t)1 << t.log2_buckets;
  uint64_t* boff = nullptr;
  uint64_t arena_used = 0;
  const uint64_t n = host_occupancy(boff, arena_used);
  DeviceArena& A = sort_mem;
  KeyCols o;
  auto take_cols = [&] {
    o.k0 = A.take_n<uint64_t>(n + 1);
    o.k1 = A.take_n<uint64_t>(n + 1);
    o.cnt = A.take_n<uint64_t>(n + 1);
    o.first = A.take_n<uint64_t>(n + 1);
    o.sref_off = A.take_n<uint64_t>(n + 1);
    o.sref_len = A.take_n<uint32_t>(n + 1);
    o.n = n;
  };
  st.order_path = 2;
  if (sample_order(n)) {
    OrderSrc src{};
    src.table = true;
    src.t = t;
    A.reserve((n + 1) * (5 * 8 + 4) + first_order_ws_bytes(src, n) + 64 * 1024);
    A.reset();
    take_cols();
    const uint32_t* ovf = first_order(src, OrderDst{o.k0, o.k1, o.cnt, o.first, o.sref_off, o.sref_len, bounds(n + 1)},
                                      n, key_bits(), A.take_n<uint8_t>(first_order_ws_bytes(src, n)), nullptr, s,
                                      fo_hist_ok ? d_fo_hist : nullptr, fo_hist_m);
    if (h_fin.size() < 64) {
      h_fin = PinnedBuffer(64);
      std::memset(h_fin.data(), 0, 64);
    }
    WC_HIP_CHECK(hipMemcpyAsync(h_fin.data() + 8, ovf, 4, hipMemcpyDeviceToHost, s));
    WC_HIP_CHECK(hipStreamSynchronize(s));  // the fallback path: one more wait is fine
    uint32_t bad = 0;
    std::memcpy(&bad, h_fin.data() + 8, 4);
    st.order_path = bad ? 3 : 1;
  } else if (bitmap_order_ok(n)) {
    OrderSrc src{};
    src.table = true;
    src.t = t;
    unsigned long long* bm = ensure_bitmap();
    A.reserve((n + 1) * (5 * 8 + 4) + bitmap_order_ws_bytes(n + 1, max_end, 1) + 64 * 1024);
    A.reset();
    take_cols();
    const uint32_t* ovf = bitmap_order(src, OrderDst{o.k0, o.k1, o.cnt, o.first, o.sref_off, o.sref_len, bounds(n + 1)},
                                       n, max_end, 1, bm, A.take_n<uint8_t>(bitmap_order_ws_bytes(n + 1, max_end, 1)), nullptr, s);
    if (h_fin.size() < 64) {
      h_fin = PinnedBuffer(64);
      std::memset(h_fin.data(), 0, 64);
    }
    WC_HIP_CHECK(hipMemcpyAsync(h_fin.data() + 8, ovf, 4, hipMemcpyDeviceToHost, s));
    WC_HIP_CHECK(hipStreamSynchronize(s));
    uint32_t bad = 0;
    std::memcpy(&bad, h_fin.data() + 8, 4);
    st.order_path = bad ? 6 : 5;
  }
  if (st.order_path != 1 && st.order_path != 5) {
    A.reserve((n + 1) * (2 * 8 + 2 * 4 + 5 * 8 + 4) + nb * 8 + radix_hist_words(n) * 4 + 64 * 1024);
    A.reset();
    uint64_t* d_boff = A.take_n<uint64_t>(nb);
    uint64_t* keys = A.take_n<uint64_t>(n + 1);
    uint64_t* tkeys = A.take_n<uint64_t>(n + 1);
    uint32_t* slots = A.take_n<uint32_t>(n + 1);
    uint32_t* tslots = A.take_n<uint32_t>(n + 1);
    uint32_t* hist = A.take_n<uint32_t>(radix_hist_words(n));
    take_cols();
    WC_HIP_CHECK(hipMemcpyAsync(d_boff, boff, nb * 8, hipMemcpyHostToDevice, s));  // pinned: no sync needed
    launch_table_keys(t, d_boff, keys, slots, s, bounds(n + 1));
    int bits = 1;
    while (bits < 64 && (max_end >> bits) != 0) ++bits;
    bool in_tmp = false;
    radix_sort_pairs(keys, slots, tkeys, tslots, hist, n, bits, s, &in_tmp);
    launch_gather_table(t, in_tmp ? tkeys : keys, in_tmp ? tslots : slots, n, o.k0, o.k1, o.cnt, o.first,
                        o.sref_off, o.sref_len, s, nullptr, bounds(n + 1));
  }
  cols = o;
  cols_arena = d_arena;
  cols_arena_bytes = std::min<uint64_t>(arena_used, opt.arena_bytes);
  st.keys = n;
  st.log2_buckets = t.log2_buckets;
  last_keys = n;
}

void Engine::Impl::sort_cols_by_first(bool radix) {
  Range r("wc_finalize_sort");
  fo_ovf = nullptr;
  const uint64_t n = cols.n;
  if (cols_hist_m && (radix || n == 0 || !sample_order(n))) {  // a histogram the sample sort will not consume
    WC_HIP_CHECK(hipMemsetAsync(d_fo_hist_cols, 0, FO_LOGBINS * sizeof(uint32_t), s));
    cols_hist_m = 0;
  }
  if (n == 0) return;
  // cols.dn: the count is on the device (n its bound) — sort and gather on it
  const uint64_t* dn = reinterpret_cast<const uint64_t*>(cols.dn);
  DeviceArena& A = sort_mem;
  KeyCols o;
  auto take_cols = [&] {
    o.k0 = A.take_n<uint64_t>(n);
    o.k1 = A.take_n<uint64_t>(n);
    o.cnt = A.take_n<uint64_t>(n);
    o.first = A.take_n<uint64_t>(n);
    o.sref_off = A.take_n<uint64_t>(n);
    o.sref_len = A.take_n<uint32_t>(n);
    o.n = n;
    o.dn = cols.dn;
  };
  if (!radix && sample_order(n)) {
    // the overflow word is read at the finalize's last wait (a rare radix redo follows)
    OrderSrc src{};
    src.table = false;
    src.k0 = cols.k0;
    src.k1 = cols.k1;
    src.cnt = cols.cnt;
    src.first = cols.first;
    src.soff = cols.sref_off;
    src.slen = cols.sref_len;
    src.n = n;
    src.dn = dn;
    A.reserve(n * (5 * 8 + 4) + first_order_ws_bytes(src, n) + 64 * 1024);
    A.reset();
    take_cols();
    fo_ovf = first_order(src, OrderDst{o.k0, o.k1, o.cnt, o.first, o.sref_off, o.sref_len, bounds(n)}, n, key_bits(),
                         A.take_n<uint8_t>(first_order_ws_bytes(src, n)), nullptr, s, nullptr, 0, d_fo_hist_cols,
                         cols_hist_m);
    cols_hist_m = 0;
    cols_unsorted = cols;
    cols = o;
    st.order_path = 1;
    return;
  }
  if (!radix && bitmap_order_ok(n)) {  // the same in-flight overflow word as the sample sort
    OrderSrc src{};
    src.table = false;
    src.k0 = cols.k0;
    src.k1 = cols.k1;
    src.cnt = cols.cnt;
    src.first = cols.first;
    src.soff = cols.sref_off;
    src.slen = cols.sref_len;
    src.n = n;
    src.dn = dn;
    unsigned long long* bm = ensure_bitmap();
    A.reserve(n * (5 * 8 + 4) + bitmap_order_ws_bytes(n, max_end, 1) + 64 * 1024);
    A.reset();
    take_cols();
    fo_ovf = bitmap_order(src, OrderDst{o.k0, o.k1, o.cnt, o.first, o.sref_off, o.sref_len, bounds(n)}, n, max_end, 1, bm,
                          A.take_n<uint8_t>(bitmap_order_ws_bytes(n, max_end, 1)), nullptr, s);
    cols_unsorted = cols;
    cols = o;
    st.order_path = 5;
    return;
  }
  A.reserve(n * (2 * 8 + 2 * 4 + 5 * 8 + 4) + radix_hist_words(n) * 4 + 64 * 1024);
  A.reset();
  uint64_t* keys = A.take_n<uint64_t>(n);
  uint64_t* tkeys = A.take_n<uint64_t>(n);
  uint32_t* vals = A.take_n<uint32_t>(n);
  uint32_t* tvals = A.take_n<uint32_t>(n);
  uint32_t* hist = A.take_n<uint32_t>(radix_hist_words(n));
  take_cols();
  WC_HIP_CHECK(hipMemcpyAsync(keys, cols.first, n * 8, hipMemcpyDeviceToDevice, s));
  launch_iota_u32(vals, n, s);
  int bits = 1;
  while (bits < 64 && (max_end >> bits) != 0) ++bits;
  bool in_tmp = false;
  radix_sort_pairs(keys, vals, tkeys, tvals, hist, n, bits, s, &in_tmp, dn, dn ? n : 0);
  launch_gather_cols(cols.k0, cols.k1, cols.cnt, cols.first, cols.sref_off, cols.sref_len, in_tmp ? tvals : vals, o.k0,
                     o.k1, o.cnt, o.first, o.sref_off, o.sref_len, n, s, dn, bounds(n));
  cols = o;
  st.order_path = radix ? 3 : 2;
}

KeyTable Engine::Impl::download_cols() {
  Range r("wc_download");
  const uint64_t n = cols.n;
  std::vector<uint64_t> k0(n), k1(n), cnt(n), first(n), soff(n);
  std::vector<uint32_t> slen(n);
  std::vector<uint8_t> arena(cols_arena_bytes);
  if (n) {
    WC_HIP_CHECK(hipMemcpyAsync(k0.data(), cols.k0, n * 8, hipMemcpyDeviceToHost, s));
    WC_HIP_CHECK(hipMemcpyAsync(k1.data(), cols.k1, n * 8, hipMemcpyDeviceToHost, s));
    WC_HIP_CHECK(hipMemcpyAsync(cnt.data(), cols.cnt, n * 8, hipMemcpyDeviceToHost, s));
    WC_HIP_CHECK(hipMemcpyAsync(first.data(), cols.first, n * 8, hipMemcpyDeviceToHost, s));
    WC_HIP_CHECK(hipMemcpyAsync(soff.data(), cols.sref_off, n * 8, hipMemcpyDeviceToHost, s));
    WC_HIP_CHECK(hipMemcpyAsync(slen.data(), cols.sref_len, n * 4, hipMemcpyDeviceToHost, s));
  }
  if (!arena.empty())
    WC_HIP_CHECK(hipMemcpyAsync(arena.data(), cols_arena, arena.size(), hipMemcpyDeviceToHost, s));
  WC_HIP_CHECK(hipStreamSynchronize(s));
  KeyTable t;
  t.words.resize(n);
  t.counts = std::move(cnt);
  t.first_off = std::move(first);
  for (uint64_t i = 0; i < n; ++i) {
    if (!key_is_hashed(k1[i])) {
      uint8_t w[KEY_INLINE_MAX];
      const uint32_t len = inline_bytes(k0[i], k1[i], w);
      t.words[i].assign(reinterpret_cast<const char*>(w), len);
    } else {
      WC_CHECK(soff[i] + slen[i] <= arena.size(), "arena reference out of range");
      t.words[i].assign(reinterpret_cast<const char*>(arena.data()) + soff[i], slen[i]);
    }
    t.total += t.counts[i];
  }
  return t;
}

// -------------------------------------------------------------------- Engine --
Engine::Engine(const Options& opt) : p_(new Impl(opt)) {}
Engine::~Engine() = default;
const Options& Engine::options() const { return p_->opt; }
Stats& Engine::stats() {
  p_->collect_stage_times();
  return p_->st;
}

void Engine::set_stage_events(bool on) { p_->stage_events = on; }

void Engine::reset() {
  Impl& im = *p_;
  im.hc_mark(Impl::HC_START);
  WC_HIP_CHECK(hipSetDevice(im.dev));
  // zero only the occupancy: a bucket with occupancy 0 is empty whatever its
  // slice holds (reduce / compact / split never read such a slice)
  im.pend.active = false;  // an unchecked pass of the previous job is discarded with it
  im.drop_reduce_bits();
  // WC_STAMPS_PER_JOB=1 (diagnostics): the map / reduce stamp sums printed at
  // teardown cover the last job only (the first job's table growth excluded)
  static const bool stamps_per_job = std::getenv("WC_STAMPS_PER_JOB") && std::atoi(std::getenv("WC_STAMPS_PER_JOB"));
  // WC_MAP_CLOCK=1 (with the stamps build path): the previous job's effective
  // shader clock during the map — s_memtime ticks over 100 MHz realtime ticks,
  // summed over the map blocks (tools/ramp_probe.py: is the short-run ramp the clock?)
  static const bool map_clock = std::getenv("WC_MAP_CLOCK") && std::atoi(std::getenv("WC_MAP_CLOCK"));
  if (map_clock && im.d_stamps && im.d_blk) {
    WC_HIP_CHECK(hipStreamSynchronize(im.s));
    unsigned long long st[MAP_STAMP_N];
    std::vector<unsigned long long> blk((size_t)im.map_blocks * 4);
    WC_HIP_CHECK(hipMemcpy(st, im.d_stamps, sizeof st, hipMemcpyDeviceToHost));
    WC_HIP_CHECK(hipMemcpy(blk.data(), im.d_blk, blk.size() * 8, hipMemcpyDeviceToHost));
    double rt = 0;
    for (size_t i = 0; i < im.map_blocks; ++i) rt += (double)(blk[4 * i + 1] - blk[4 * i]);
    if (rt > 0 && st[MS_BLKSUM])
      fprintf(stderr, "[wc] job map clock %.0f MHz (memtime %.3e / realtime %.3e), mean map block %.1f us\n",
              (double)st[MS_BLKSUM] / rt * 100.0, (double)st[MS_BLKSUM], rt, rt / im.map_blocks / 100.0);
  }
  if (stamps_per_job && im.d_stamps) {
    WC_HIP_CHECK(hipMemsetAsync(im.d_stamps, 0, MAP_STAMP_N * 8, im.s));
    WC_HIP_CHECK(hipMemsetAsync(im.d_red_stamps, 0, RED_STAMP_N * 8, im.s));
    im.blocks_stamped = 0;
  }
  im.pass_pub_pending = false;
  // no API call: the next pass's zeroing launch clears occupancy + arena cursor
  // (apply_reset does it first for anything else that reads the table)
  im.reset_pending = true;
  im.occ_valid = false;
  im.fo_hist_ok = false;
  if (im.copy_used) WC_HIP_CHECK(hipStreamSynchronize(im.copy_s));  // a failed stream may have left copies
  im.copy_used = false;
  const uint32_t planned = im.st.merges_planned, redos = im.st.merge_redos;  // engine-lifetime counters
  im.st = Stats{};
  im.st.merges_planned = planned;
  im.st.merge_redos = redos;
  im.max_end = 0;
  im.ev_n = 0;
  im.hot_valid = false;  // each job samples its own hot words
  im.merge_zero_pre = false;
  im.hc_mark(Impl::HC_RESET);
}

void Engine::count_device(const uint8_t* d_text, uint64_t n, uint64_t avail, uint64_t global_base, int prev_byte) {
  Impl& im = *p_;
  WC_HIP_CHECK(hipSetDevice(im.dev));
  Range r("wc_count_device");
  const double t0 = now_seconds();
  const uint64_t C = im.opt.chunk_bytes;
  for (uint64_t off = 0; off < n; off += C) {
    const uint64_t len = std::min<uint64_t>(C, n - off);
    im.process_chunk(d_text + off, len, avail - off, global_base + off, off == 0 ? prev_byte : -1, off + len >= n);
  }
  im.st.bytes += n;
  im.st.host_count_ms += (now_seconds() - t0) * 1e3;
}

namespace {
struct MemorySource : ChunkSource {
  const uint8_t* p;
  uint64_t n, pos = 0;
  MemorySource(const uint8_t* p_, uint64_t n_) : p(p_), n(n_) {}
  uint64_t read(uint8_t* dst, uint64_t cap) override {
    const uint64_t k = std::min(cap, n - pos);
    // into pinned staging: one thread copies ~5-8 GB/s, split large copies
    const uint64_t t = std::min<uint64_t>(8, std::max<uint64_t>(1, k / (16ull << 20))), per = (k + t - 1) / t;
    std::vector<std::thread> th;
    for (uint64_t i = 1; i < t; ++i) {
      const uint64_t b = i * per, e = std::min(k, b + per);
      if (b < e) th.emplace_back([=] { std::memcpy(dst + b, p + pos + b, e - b); });
    }
    std::memcpy(dst, p + pos, std::min(k, per));
    for (auto& x : th) x.join();
    pos += k;
    return k;
  }
};
}  // namespace

void Engine::count_host(const uint8_t* h_text, uint64_t n, uint64_t global_base) {
  MemorySource src(h_text, n);
  count_source(src, global_base);
}

void Engine::count_source(ChunkSource& src, uint64_t global_base) {
  Impl& im = *p_;
  WC_HIP_CHECK(hipSetDevice(im.dev));
  Range r("wc_count_stream");
  im.settle();
  const double t0 = now_seconds();
  uint64_t stream = im.opt.stream_chunk_bytes;
  if (const char* e = std::getenv("WC_STREAM_CHUNK")) stream = std::strtoull(e, nullptr, 10);  // sweeps only
  const uint64_t C = std::min(im.opt.chunk_bytes, std::max<uint64_t>(1ull << 20, stream / 256 * 256));
  im.ensure_staging(C);
  im.copy_used = true;
  ScopedAffinity bind(im.numa.cpus);  // the source's reader threads (they inherit the mask) on the GPU's node
  std::vector<uint8_t> carry;
  bool eof = false;
  uint64_t offset = global_base;

  // A word longer than a whole piece (no delimiter in C bytes): its bytes are
  // gathered on the host up to the next delimiter and counted as a pass of its
  // own from a device buffer sized to it (SURVEY §5.7 long-word fallback; the
  // map keys it with the byte loop, the reducer copies it to the key arena).
  std::vector<uint8_t> giant;
  auto count_giant = [&](uint64_t base) {
    const uint64_t n = giant.size();
    // records and hot slots carry 32-bit chunk offsets and word lengths; the
    // word's bytes must also fit the key arena — fail clearly, before launching
    WC_CHECK(n <= (1ull << 32) - 2 * (uint64_t)MAP_TILE,
             "a " + std::to_string(n) + "-byte word exceeds the longest supported word (4 GiB - 64 KiB)");
    WC_CHECK(n + 8 <= im.opt.arena_bytes, "a " + std::to_string(n) + "-byte word does not fit the " +
                                              std::to_string(im.opt.arena_bytes) + "-byte key arena (raise arena_bytes)");
    WC_LOG(LOG_INFO, "dev %d: %llu-byte word at %llu exceeds the %llu-byte stream piece: own pass", im.dev,
           (unsigned long long)n, (unsigned long long)base, (unsigned long long)C);
    im.giant_mem.reserve(n + 4096);
    im.giant_mem.reset();
    uint8_t* d = static_cast<uint8_t*>(im.giant_mem.take(n + 4096));
    WC_HIP_CHECK(hipMemcpy(d, giant.data(), n, hipMemcpyHostToDevice));
    const uint32_t blocks = im.blocks_for(n), rb = im.rec_buckets_log2();
    im.launch_pass(d, n, n, base, ' ', rb, blocks);
    im.complete_pass(d, n, n, base, ' ', rb, blocks);
    im.st.bytes += n;
    giant.clear();
  };

  // Fill pinned[k % ring] with carry + fresh bytes, cut at the last delimiter.
  // A piece with no delimiter at all is the start of a giant word: it moves to
  // `giant` (counted by the caller, before the returned piece) and the piece is
  // refilled from the bytes after it.
  auto fill = [&](uint64_t k) -> uint64_t {
    uint8_t* pin = im.pinned[k % im.pinned.size()].data();
    for (;;) {
      uint64_t total = carry.size();
      if (total) std::memcpy(pin, carry.data(), total);
      carry.clear();
      while (!eof && total < C) {
        const uint64_t got = src.read(pin + total, C - total);
        if (got == 0) eof = true;
        total += got;
      }
      if (total == 0 || eof) return total;
      uint64_t cut = total;
      while (cut > 0 && !is_delim(pin[cut - 1])) --cut;
      if (cut > 0) {
        carry.assign(pin + cut, pin + total);
        return cut;
      }
      WC_CHECK(giant.empty(), "one giant word per piece");  // a piece after a giant starts with its delimiter
      giant.assign(pin, pin + total);
      std::vector<uint8_t> tmp(std::min<uint64_t>(C, 16ull << 20));
      while (!eof) {
        const uint64_t got = src.read(tmp.data(), tmp.size());
        if (got == 0) {
          eof = true;
          break;
        }
        uint64_t d = 0;
        while (d < got && !is_delim(tmp[d])) ++d;
        giant.insert(giant.end(), tmp.data(), tmp.data() + d);
        if (d < got) {
          carry.assign(tmp.data() + d, tmp.data() + got);
          break;
        }
      }
    }
  };
  auto issue = [&](uint64_t k, uint64_t len) {
    WC_HIP_CHECK(hipStreamWaitEvent(im.copy_s, im.ev_done[k & 1], 0));
    WC_HIP_CHECK(hipMemcpyAsync(im.d_stage[k & 1], im.pinned[k % im.pinned.size()].data(), len,
                                hipMemcpyHostToDevice, im.copy_s));
    WC_HIP_CHECK(hipEventRecord(im.ev_h2d[k & 1], im.copy_s));
  };
  WC_HIP_CHECK(hipEventRecord(im.ev_done[0], im.s));
  WC_HIP_CHECK(hipEventRecord(im.ev_done[1], im.s));
  uint64_t len = fill(0);
  if (!giant.empty()) {  // the stream starts with a giant word
    const uint64_t n = giant.size();
    count_giant(offset);
    offset += n;
  }
  if (len) issue(0, len);
  // WC_STREAM_TRACE=1 (diagnostics): host seconds in the reads, the launches and
  // the completion waits, printed at the end
  static const bool trace = std::getenv("WC_STREAM_TRACE") && std::atoi(std::getenv("WC_STREAM_TRACE"));
  double t_fill = 0, t_launch = 0, t_wait = 0;
  const double t_pre = now_seconds() - t0;  // staging ring + the first piece's read
  for (uint64_t k = 0; len; ++k) {
    const uint8_t* d = im.d_stage[k & 1];
    const double a0 = trace ? now_seconds() : 0;
    WC_HIP_CHECK(hipStreamWaitEvent(im.s, im.ev_h2d[k & 1], 0));
    const uint32_t blocks = im.blocks_for(len);
    const uint32_t rb = im.rec_buckets_log2();
    im.launch_pass(d, len, len, offset, ' ', rb, blocks);
    const double a1 = trace ? now_seconds() : 0;
    const uint64_t next = fill(k + 1);  // host reads the next chunk while the GPU works
    if (next) issue(k + 1, next);
    const double a2 = trace ? now_seconds() : 0;
    im.complete_pass(d, len, len, offset, ' ', rb, blocks);
    if (trace) {
      t_launch += a1 - a0;
      t_fill += a2 - a1;
      t_wait += now_seconds() - a2;
    }
    WC_HIP_CHECK(hipEventRecord(im.ev_done[k & 1], im.s));
    offset += len;
    im.st.bytes += len;
    if (!giant.empty()) {  // between piece k and piece k + 1 (stream order)
      const uint64_t n = giant.size();
      count_giant(offset);
      offset += n;
    }
    len = next;
  }
  WC_HIP_CHECK(hipStreamSynchronize(im.copy_s));
  im.st.host_count_ms += (now_seconds() - t0) * 1e3;
  if (trace)
    std::fprintf(stderr, "[wc] stream: %.3f s total, before the loop %.3f s, read %.3f s, launch %.3f s, wait %.3f s, %u pieces\n",
                 now_seconds() - t0, t_pre, t_fill, t_launch, t_wait, im.st.chunks);
}

void Engine::count_pinned_replay(const uint8_t* pool, uint64_t pool_bytes, uint64_t total, uint64_t global_base,
                                 bool pinned) {
  Impl& im = *p_;
  WC_HIP_CHECK(hipSetDevice(im.dev));
  Range r("wc_count_pinned_replay");
  im.settle();
  const double t0 = now_seconds();
  const uint64_t C = std::min<uint64_t>(im.opt.chunk_bytes, pool_bytes);
  WC_CHECK(pool_bytes % C == 0, "replay pool must be a whole number of chunks");
  for (uint64_t c = C; c <= pool_bytes; c += C)
    WC_CHECK(is_delim(pool[c - 1]), "every replay chunk must end with a delimiter");
  // Page-lock the caller's pool once: chunks are DMA'd straight from it.
  if (!pinned && im.registered != pool) {
    if (im.registered) (void)hipHostUnregister(const_cast<uint8_t*>(im.registered));
    im.registered = nullptr;
    WC_HIP_CHECK(hipHostRegister(const_cast<uint8_t*>(pool), pool_bytes, hipHostRegisterDefault));
    im.registered = pool;
  }
  im.ensure_staging(C);
  im.copy_used = true;
  WC_HIP_CHECK(hipEventRecord(im.ev_done[0], im.s));
  WC_HIP_CHECK(hipEventRecord(im.ev_done[1], im.s));
  const uint64_t nchunks = (total + C - 1) / C;
  auto issue = [&](uint64_t k) {
    const uint64_t len = std::min<uint64_t>(C, total - k * C);
    WC_HIP_CHECK(hipStreamWaitEvent(im.copy_s, im.ev_done[k & 1], 0));
    WC_HIP_CHECK(hipMemcpyAsync(im.d_stage[k & 1], pool + (k * C) % pool_bytes, len, hipMemcpyHostToDevice,
                                im.copy_s));
    WC_HIP_CHECK(hipEventRecord(im.ev_h2d[k & 1], im.copy_s));
  };
  if (nchunks) issue(0);
  for (uint64_t k = 0; k < nchunks; ++k) {
    const uint64_t len = std::min<uint64_t>(C, total - k * C);
    const uint8_t* d = im.d_stage[k & 1];
    WC_HIP_CHECK(hipStreamWaitEvent(im.s, im.ev_h2d[k & 1], 0));
    const uint32_t blocks = im.blocks_for(len), rb = im.rec_buckets_log2();
    // a truncated last chunk may end mid-word: it is the end of the stream
    im.launch_pass(d, len, len, global_base + k * C, ' ', rb, blocks);
    if (k + 1 < nchunks) issue(k + 1);  // H2D of chunk k+1 overlaps map/reduce of chunk k
    im.complete_pass(d, len, len, global_base + k * C, ' ', rb, blocks);
    WC_HIP_CHECK(hipEventRecord(im.ev_done[k & 1], im.s));
    im.st.bytes += len;
  }
  WC_HIP_CHECK(hipStreamSynchronize(im.copy_s));
  im.st.host_count_ms += (now_seconds() - t0) * 1e3;
}

const uint8_t* Engine::synth_device(uint64_t n, uint64_t first_segment, const SynthSpec& spec) {
  Impl& im = *p_;
  WC_HIP_CHECK(hipSetDevice(im.dev));
  // the generated text is rewritten: a pass still pending on the old text
  // (speculative last pass) must complete first — its recovery would re-read it
  im.settle();
  const uint64_t key = spec.seed * 1000003ull ^ ((uint64_t)spec.vocab << 20) ^ (uint64_t)(spec.zipf_s * 1e6) ^
                       ((uint64_t)(spec.long_frac * 1e6) << 40);
  if (key != im.vocab_key) {
    const HostVocab hv = build_vocab(spec);
    im.vocab_mem.reserve(hv.bytes.size() + hv.off.size() * 9 + hv.cdf.size() * 4 + 4096);
    uint8_t* b = im.vocab_mem.take_n<uint8_t>(hv.bytes.size());
    uint32_t* off = im.vocab_mem.take_n<uint32_t>(hv.off.size());
    uint8_t* len = im.vocab_mem.take_n<uint8_t>(hv.len.size());
    uint32_t* cdf = im.vocab_mem.take_n<uint32_t>(hv.cdf.size());
    WC_HIP_CHECK(hipMemcpy(b, hv.bytes.data(), hv.bytes.size(), hipMemcpyHostToDevice));
    WC_HIP_CHECK(hipMemcpy(off, hv.off.data(), hv.off.size() * 4, hipMemcpyHostToDevice));
    WC_HIP_CHECK(hipMemcpy(len, hv.len.data(), hv.len.size(), hipMemcpyHostToDevice));
    WC_HIP_CHECK(hipMemcpy(cdf, hv.cdf.data(), hv.cdf.size() * 4, hipMemcpyHostToDevice));
    im.d_vocab = SynthVocab{b, off, len, cdf, (uint32_t)hv.off.size()};
    im.vocab_key = key;
  }
  im.ensure_text(n);
  launch_synth(im.d_text, n, first_segment, spec.seed, im.d_vocab, im.s);
  WC_HIP_CHECK(hipStreamSynchronize(im.s));
  return im.d_text;
}

uint64_t Engine::finalize_device(Comm* comm) { return p_->finalize(comm, false); }

uint64_t Engine::Impl::finalize(Comm* comm, bool all_ranks) {
  Impl& im = *this;
  WC_HIP_CHECK(hipSetDevice(im.dev));
  const double t0 = now_seconds();
  // WC_MERGE_ALWAYS=1 (tests): run the merge protocol even with one rank, so
  // the RCCL exchange code is exercised on a one-GPU box
  static const bool merge_always = getenv("WC_MERGE_ALWAYS") && atoi(getenv("WC_MERGE_ALWAYS")) != 0;
  const bool merged = comm && (comm->size() > 1 || merge_always);
  im.apply_reset();  // a reset with no pass since: the table reads empty
  im.mark(EV_FIN);
  im.fin_end_marked = false;
  im.fo_ovf = nullptr;
  im.order_redo = false;
  bool drained = false;
  im.planned_active = false;
  if (!merged) im.merge_zero_last_valid = false;  // a local job: the next pass does not pre-zero merge regions
  if (merged) {
    im.drop_reduce_bits();  // the merged order runs on merged columns
    // planned (no host round trip) when the last exact merge of this shape
    // left its caps, else the speculative exact protocol, else the synchronous one
    const bool spec = im.pend.active && im.speculate && !im.sync_debug &&
                      (merge_cols_planned_speculative(im, *comm, all_ranks) || merge_cols_speculative(im, *comm, all_ranks));
    if (!spec) {
      im.settle();
      im.compact_local();
      im.mark(EV_MERGE0);
      merge_cols(im, *comm, all_ranks);
    }
    im.mark(EV_MERGE1);
    im.sort_cols_by_first();
  } else if (im.pend.active && im.finalize_local_speculative()) {
    drained = im.spin_wait;  // its publish wait saw the whole stream complete
  } else {
    im.fin_end_marked = false;  // a speculative finalize that needed recovery is redone here
    im.settle();
    im.finalize_local_sorted();  // sort (first, slot) pairs, gather the columns from the table once
    if (im.order_redo && im.st.order_path == 1) im.st.order_path = 4;
  }
  if (!im.fin_end_marked) im.mark(EV_FIN_END);
  // the merged count still on the device, the sample sort's overflow word and
  // (planned merge) its decision flags and local key count: published with the last wait
  auto publish_and_wait = [&] {
    if (!drained) {  // the bounds word rides in every finalize's last publish
      if (im.h_fin.size() < 64) {
        im.h_fin = PinnedBuffer(64);
        std::memset(im.h_fin.data(), 0, 64);  // the sequence word starts below every fin_seq
      }
      PubList pc{};
      if (im.pass_pub_pending) {  // the planned merge's pending pass: its counters ride here
        im.pass_pub_pending = false;
        for (int i = 0; i < im.pass_pub.n; ++i)
          pc.add(im.pass_pub.dst[i], im.pass_pub.src[i], (uint64_t)im.pass_pub.words[i] * 4);
      }
      if (im.cols.dn) pc.add(im.h_fin.data(), im.cols.dn, 8);
      pc.add(im.h_fin.data() + 40, im.d_bounds, 8);
      if (im.fo_ovf) pc.add(im.h_fin.data() + 8, im.fo_ovf, 4);
      if (im.planned_active) {
        std::memset(im.h_fin.data() + 16, 0, 16);
        pc.add(im.h_fin.data() + 16, im.d_merge_flags, 4);
        pc.add(im.h_fin.data() + 24, im.d_local_n, 8);
      }
      if (merged && im.spin_wait) {  // a sequence word stored last: the host spins on it (below)
        pc.seq_dst = reinterpret_cast<uint32_t*>(im.h_fin.data() + 32);
        pc.seq = ++im.fin_seq;
      }
      launch_publish(pc, im.s);
      // the merge's last collectives are still in flight: wait under the comm watchdog
      if (merged && im.spin_wait) {
        im.hc_mark(HC_WAIT);
        comm->wait_word(reinterpret_cast<const uint32_t*>(im.h_fin.data() + 32), im.fin_seq, im.s);
        im.hc_mark(HC_WAITED);
        return;
      }
    }
    if (merged) comm->sync(im.s);
    else if (!drained) WC_HIP_CHECK(hipStreamSynchronize(im.s));
  };
  publish_and_wait();
  const auto bounds_word = [&] {
    uint64_t w = 0;
    if (!drained) std::memcpy(&w, im.h_fin.data() + 40, 8);
    return w;
  };
  // the planned merge decides first whether this attempt is redone: a redone
  // attempt's bounds word is discarded with its output (re-armed before the redo)
  const uint64_t bw_first = bounds_word();
  if (!im.planned_active) im.check_bounds(bw_first, merged ? "the merged finalize" : "the local finalize");
  if (im.planned_active) {
    // the planned merge's decisions (the same on every rank: all-gathered words)
    im.planned_active = false;
    uint32_t f = 0;
    uint64_t local_n = 0;
    std::memcpy(&f, im.h_fin.data() + 16, 4);
    std::memcpy(&local_n, im.h_fin.data() + 24, 8);
    if (f & 2) fail("key arena exhausted on a rank (" + std::to_string(im.opt.arena_bytes) + " bytes each); raise arena_bytes");
    const PendingPass p = im.planned_pass;
    const bool clean = im.complete_pass(p.text, p.len, p.avail, p.base, p.prev, p.rb, p.blocks, true);
    im.st.keys = local_n;
    if (clean && !(f & 5)) im.check_bounds(bw_first, "the merged finalize");
    if (!clean || (f & 5)) {
      // a pass needed recovery (1) or a fixed region overflowed (4): every rank
      // redoes the merge exactly (the table is intact) and relearns the caps
      WC_LOG(LOG_INFO, "dev %d: planned merge redone exactly (flags %u)", im.dev, f);
      if (bw_first) WC_HIP_CHECK(hipMemsetAsync(im.d_bounds, 0, 8, im.s));
      im.merge_caps.valid = false;
      im.st.merge_redos++;
      im.fo_ovf = nullptr;
      im.settle();
      im.compact_local();
      im.mark(EV_MERGE0);
      merge_cols(im, *comm, all_ranks);
      im.mark(EV_MERGE1);
      im.sort_cols_by_first();
      im.mark(EV_FIN_END);
      publish_and_wait();
      im.check_bounds(bounds_word(), "the redone merged finalize");
    }
  }
  if (im.fo_ovf) {
    uint32_t bad = 0;
    std::memcpy(&bad, im.h_fin.data() + 8, 4);
    im.fo_ovf = nullptr;
    if (bad) {  // a sample-sort bin overflowed / a shared bitmap position: redo the order with the radix sort
      const bool was_bitmap = im.st.order_path == 5;
      im.cols = im.cols_unsorted;
      im.sort_cols_by_first(true);
      if (was_bitmap) im.st.order_path = 6;
      uint64_t w = 0;
      WC_HIP_CHECK(hipMemcpyAsync(&w, im.d_bounds, 8, hipMemcpyDeviceToHost, im.s));
      WC_HIP_CHECK(hipStreamSynchronize(im.s));
      im.check_bounds(w, "the radix order redo");
    }
  }
  if (im.cols.dn) {
    uint64_t g = 0;
    std::memcpy(&g, im.h_fin.data(), 8);
    WC_CHECK(g <= im.cols.n, "merged key count exceeds its bound");
    im.cols.n = g;
    im.cols.dn = nullptr;
  }
  im.st.host_finalize_ms += (now_seconds() - t0) * 1e3;
  im.hc_mark(HC_DONE);
  WC_LOG(LOG_INFO, "dev %d: finalize %.3f ms (host), %llu keys, %u chunk(s), %llu records, %u re-run(s)", im.dev,
         (now_seconds() - t0) * 1e3, (unsigned long long)im.cols.n, im.st.chunks, (unsigned long long)im.st.records,
         im.st.map_reruns);
  return im.cols.n;
}

KeyTable Engine::result(Comm* comm, bool all_ranks) {
  Impl& im = *p_;
  im.finalize(comm, all_ranks);
  if (comm && comm->size() > 1 && comm->rank() != 0 && !all_ranks) {
    KeyTable t;
    return t;
  }
  return im.download_cols();
}

}  // namespace wc

namespace wc {
HostPool::HostPool(uint64_t n, uint64_t first_segment, const SynthSpec& spec, int threads, int device) : n_(n) {
  const double t0 = now_seconds();
  // bound to the GPU's node: the page-locked pages (placed at allocation by the
  // local-node policy) and the generator threads (they inherit the mask)
  const NumaNode nn = device >= 0 ? numa_of_device(device) : NumaNode{};
  ScopedAffinity bind(nn.cpus);
  node_ = bind.active() ? nn.node : -1;
  WC_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&p_), std::max<uint64_t>(n, 1),
                             bind.active() ? hipHostMallocNumaUser : hipHostMallocDefault));
  synth_host_into(p_, n, first_segment, spec, build_vocab(spec), threads);
  secs_ = now_seconds() - t0;
}
HostPool::~HostPool() {
  if (p_) (void)hipHostFree(p_);
}
}  // namespace wc
