// wordcount — CLI of the MI355X-native MapReduce word count.
//
// Reference CLI: the reference binary ignores argv and always reads ./test.txt
// (/root/reference/main.cu:164-167), printing the framed table of
// main.cu:166-218.  `wordcount` with no arguments does exactly that;
// `wordcount <file>` is the north-star form; everything else is opt-in.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../src/common/hip_util.hpp"
#include "../src/dist/comm.hpp"
#include "../src/io/checkpoint.hpp"
#include "../src/io/source.hpp"
#include "wc/wc.hpp"

namespace {

const char* kUsage =
    "usage: wordcount [FILE] [options]\n"
    "  FILE                    input text (default: test.txt, as the reference)\n"
    "  --gpus N                shard across N GPUs, merged with RCCL (default 1; more\n"
    "                          than the visible GPUs is an error)\n"
    "  --virtual-ranks W       shard across W ranks on GPU 0 (threads), merged with the\n"
    "                          stream-ordered loopback communicator (tests the W-rank\n"
    "                          merge on one GPU; not a multi-GPU run)\n"
    "  --merge shuffle|dense   cross-GPU merge: all-to-all by key owner (default) or\n"
    "                          dictionary union + reduce-scatter / all-gather\n"
    "  --cpu                   single-thread CPU oracle (hash map)\n"
    "  --compat=reference      CPU emulation of the reference program's quirks\n"
    "  --echo | --no-echo      echo the input after 'Input Data:' (default: echo)\n"
    "  --no-list               do not print per-word rows\n"
    "  --top K                 print only the K most frequent words\n"
    "  --synthetic SIZE[:SEED[:VOCAB[:ZIPF[:LONGFRAC]]]]  count generated text instead of FILE\n"
    "  --chunk-bytes N         device chunk size (default 1G)\n"
    "  --host-staged           stream FILE through the pinned host ring (no echo)\n"
    "  --bench-json PATH       write throughput / stage timings as JSON\n"
    "  --bench                 print throughput / stage timings to stderr\n"
    "  --checkpoint PATH       count FILE in intervals; after each, save the running\n"
    "                          table + byte offset to PATH (PATH.r<rank>of<N> per GPU)\n"
    "  --checkpoint-every SIZE interval between checkpoints (default 4G)\n"
    "  --resume                continue from the checkpoint(s) at PATH when present\n";

uint64_t parse_size(const std::string& s) {
  char* end = nullptr;
  const double v = std::strtod(s.c_str(), &end);
  uint64_t mul = 1;
  if (end && *end) {
    switch (*end) {
      case 'k': case 'K': mul = 1ull << 10; break;
      case 'm': case 'M': mul = 1ull << 20; break;
      case 'g': case 'G': mul = 1ull << 30; break;
      case 't': case 'T': mul = 1ull << 40; break;
      default: wc::fail("bad size: " + s);
    }
  }
  return (uint64_t)(v * (double)mul);
}

struct Cli {
  std::string file = "test.txt";
  int gpus = 1;
  int virtual_ranks = 0;
  bool cpu = false, compat = false, echo = true, list = true, host_staged = false;
  uint64_t top = 0, chunk = 1ull << 30;
  uint32_t merge_mode = 0;
  bool synthetic = false;
  uint64_t synth_bytes = 0;
  wc::SynthSpec spec;
  std::string bench_json;
  bool bench = false;
  std::string ckpt;
  uint64_t ckpt_every = 4ull << 30;
  bool resume = false;
};

Cli parse(int argc, char** argv) {
  Cli c;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto need = [&](const char* what) -> std::string {
      if (i + 1 >= argc) wc::fail(std::string("missing value for ") + what);
      return argv[++i];
    };
    if (a == "-h" || a == "--help") {
      std::fputs(kUsage, stdout);
      std::exit(0);
    } else if (a == "--gpus") c.gpus = std::stoi(need("--gpus"));
    else if (a == "--virtual-ranks") c.virtual_ranks = std::stoi(need("--virtual-ranks"));
    else if (a == "--cpu") c.cpu = true;
    else if (a == "--merge") {
      const std::string m = need("--merge");
      if (m == "shuffle") c.merge_mode = 0;
      else if (m == "dense") c.merge_mode = 1;
      else wc::fail("--merge expects shuffle or dense, got " + m);
    }
    else if (a == "--compat=reference") c.compat = true;
    else if (a == "--echo") c.echo = true;
    else if (a == "--no-echo") c.echo = false;
    else if (a == "--no-list") c.list = false;
    else if (a == "--top") c.top = std::stoull(need("--top"));
    else if (a == "--chunk-bytes") c.chunk = parse_size(need("--chunk-bytes"));
    else if (a == "--host-staged") c.host_staged = true;
    else if (a == "--bench-json") c.bench_json = need("--bench-json");
    else if (a == "--bench") c.bench = true;
    else if (a == "--checkpoint") c.ckpt = need("--checkpoint");
    else if (a == "--checkpoint-every") c.ckpt_every = parse_size(need("--checkpoint-every"));
    else if (a == "--resume") c.resume = true;
    else if (a == "--synthetic") {
      std::string v = need("--synthetic");
      std::vector<std::string> f;
      size_t p = 0;
      for (size_t q; (q = v.find(':', p)) != std::string::npos; p = q + 1) f.push_back(v.substr(p, q - p));
      f.push_back(v.substr(p));
      c.synthetic = true;
      c.synth_bytes = parse_size(f[0]);
      if (f.size() > 1) c.spec.seed = std::stoull(f[1]);
      if (f.size() > 2) c.spec.vocab = (uint32_t)std::stoul(f[2]);
      if (f.size() > 3) c.spec.zipf_s = std::stod(f[3]);
      if (f.size() > 4) c.spec.long_frac = std::stod(f[4]);
    } else if (!a.empty() && a[0] == '-') wc::fail("unknown option " + a + "\n" + kUsage);
    else c.file = a;
  }
  if (c.synthetic) c.echo = false;
  if (!c.ckpt.empty() && (c.synthetic || c.compat)) wc::fail("--checkpoint needs a FILE input and the clean semantics");
  if (c.resume && c.ckpt.empty()) wc::fail("--resume needs --checkpoint PATH");
  if (c.gpus < 1) wc::fail("--gpus expects N >= 1");
  if (c.virtual_ranks < 0 || c.virtual_ranks > 64) wc::fail("--virtual-ranks expects 1..64");
  if (c.virtual_ranks && c.gpus != 1) wc::fail("--virtual-ranks runs on one GPU: drop --gpus");
  return c;
}

wc::Checkpoint open_checkpoint(const Cli& c, uint64_t input_size, const wc::ShardRange& sr, int r, int g) {
  return wc::open_checkpoint(wc::checkpoint_path(c.ckpt, r, g), c.resume, c.file, input_size, sr.begin, sr.end, r, g);
}

void add_stats(wc::Stats& a, const wc::Stats& b) {
  a.bytes += b.bytes;
  a.tokens += b.tokens;
  a.keys = std::max(a.keys, b.keys);
  a.records += b.records;
  a.chunks += b.chunks;
  a.map_reruns += b.map_reruns;
  a.table_splits += b.table_splits;
  a.map_ms += b.map_ms;
  a.reduce_ms += b.reduce_ms;
  a.finalize_ms += b.finalize_ms;
  a.merge_ms += b.merge_ms;
  a.idle_ms += b.idle_ms;
  a.device_ms += b.device_ms;
}

void write_out(const std::string& s) { std::fwrite(s.data(), 1, s.size(), stdout); }

int run(const Cli& c) {
  wc::KeyTable t;
  std::string text;  // host copy when echoing / CPU paths
  bool have_text = false;
  const double t0 = wc::now_seconds();
  uint64_t bytes = 0;
  int gpus_used = 0, ranks_used = 0;
  wc::Stats stages;  // GPU path: stage timings (max over ranks) and counters (sums)

  const bool need_host_text = !c.synthetic && (c.echo || c.cpu || c.compat);
  if (!c.synthetic) {
    try {
      if (need_host_text) {
        text = wc::read_file(c.file);
        have_text = true;
      } else {
        (void)wc::file_size(c.file);
      }
    } catch (const wc::Error&) {
      // Reference behaviour for a missing file: empty framing, exit 0 (main.cu:174).
      std::fprintf(stderr, "wordcount: cannot open %s\n", c.file.c_str());
      write_out(wc::format_output(t, nullptr, 0, false, c.list));
      return 0;
    }
  }

  if (c.compat || c.cpu) {
    std::string host = have_text ? text : std::string();
    if (c.synthetic) {
      const std::vector<uint8_t> v = wc::synth_host(c.synth_bytes, 0, c.spec);
      host.assign(v.begin(), v.end());
    }
    const auto* p = reinterpret_cast<const uint8_t*>(host.data());
    if (!c.ckpt.empty()) {
      wc::Checkpoint k = open_checkpoint(c, host.size(), wc::ShardRange{0, host.size()}, 0, 1);
      wc::run_checkpointed(c.file, k, c.ckpt_every, c.ckpt,
                           [](const uint8_t* q, uint64_t n, uint64_t base) { return wc::cpu::count(q, n, base); });
      t = std::move(k.table);
    } else {
      if (c.compat) {
        std::string echoed;
        t = wc::cpu::count_reference_compat(p, host.size(), &echoed);
        if (have_text) text = std::move(echoed);  // the reference echoes only the records it read
      } else {
        t = wc::cpu::count(p, host.size());
      }
    }
    bytes = host.size();
  } else {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess) {  // no GPU driver / device: none visible
      (void)hipGetLastError();
      ndev = 0;
    }
    if (c.gpus > ndev)
      wc::fail(std::to_string(c.gpus) + " GPUs requested, " + std::to_string(ndev) + " visible");
    const bool virt = c.virtual_ranks > 0;
    const int g = virt ? c.virtual_ranks : c.gpus;  // ranks
    gpus_used = virt ? 1 : g;
    std::vector<int> devs(g);
    for (int i = 0; i < g; ++i) devs[i] = virt ? 0 : i;
    std::vector<std::unique_ptr<wc::Comm>> comms;
    if (g > 1) comms = virt ? wc::make_loopback_comms(g) : wc::make_rccl_comms_all(devs);
    std::vector<std::string> errs(g);
    std::vector<wc::KeyTable> rank_tables(g);  // checkpointed runs merge on the host
    std::vector<wc::Stats> rank_stats(g);
    const uint64_t total = c.synthetic ? c.synth_bytes : (have_text ? text.size() : wc::file_size(c.file));
    bytes = total;
    auto worker = [&](int r) {
      try {
        wc::Options o;
        o.device = devs[r];
        o.chunk_bytes = c.chunk;
        o.merge_mode = c.merge_mode;
        wc::Engine eng(o);
        if (!c.ckpt.empty()) {
          // Checkpointed: delimiter-aligned intervals, each finalised on the GPU and
          // folded into the rank's host table; ranks merge on the host below.
          const wc::ShardRange sr = wc::shard_range(c.file, r, g);
          wc::Checkpoint k = open_checkpoint(c, total, sr, r, g);
          wc::run_checkpointed(c.file, k, c.ckpt_every, wc::checkpoint_path(c.ckpt, r, g),
                               [&](const uint8_t* q, uint64_t n, uint64_t base) {
                                 eng.count_host(q, n, base);
                                 wc::KeyTable kt = eng.result(nullptr, false);
                                 add_stats(rank_stats[r], eng.stats());
                                 eng.reset();
                                 return kt;
                               });
          rank_tables[r] = std::move(k.table);
          return;
        } else if (c.synthetic) {
          // shard at segment granularity: every segment ends with a delimiter
          const uint64_t nseg = (total + 1023) / 1024, per = (nseg + g - 1) / g;
          const uint64_t s0 = std::min<uint64_t>(nseg, per * r), s1 = std::min<uint64_t>(nseg, per * (r + 1));
          const uint64_t b0 = s0 * 1024, b1 = std::min<uint64_t>(total, s1 * 1024);
          if (b1 > b0) {
            const uint8_t* d = eng.synth_device(b1 - b0, s0, c.spec);
            eng.count_device(d, b1 - b0, b1 - b0, b0, ' ');
          }
        } else if (have_text && !c.host_staged) {
          const auto* p = reinterpret_cast<const uint8_t*>(text.data());
          const wc::ShardRange sr = wc::shard_range_mem(p, text.size(), r, g);
          if (sr.end > sr.begin) eng.count_host(p + sr.begin, sr.end - sr.begin, sr.begin);
        } else {
          const wc::ShardRange sr = wc::shard_range(c.file, r, g);
          wc::FileSource src(c.file, sr.begin, sr.end);
          eng.count_source(src, sr.begin);
        }
        wc::KeyTable kt = eng.result(g > 1 ? comms[r].get() : nullptr, false);
        rank_stats[r] = eng.stats();
        if (r == 0) t = std::move(kt);
      } catch (const std::exception& ex) {
        errs[r] = ex.what();
        // peers may be blocked in (or heading into) the merge collectives:
        // abort this rank's communicator so they fail fast instead of waiting
        // for the watchdog timeout
        if (g > 1 && comms[r]) comms[r]->abort(ex.what());
      }
    };
    if (g == 1) {
      worker(0);
    } else {
      std::vector<std::thread> th;
      for (int r = 0; r < g; ++r) th.emplace_back(worker, r);
      for (auto& x : th) x.join();
    }
    ranks_used = g;
    for (int r = 0; r < g; ++r)
      if (!errs[r].empty()) wc::fail((virt ? "rank " : "GPU ") + std::to_string(r) + ": " + errs[r]);
    if (!c.ckpt.empty())
      for (int r = 0; r < g; ++r) wc::merge_tables(t, rank_tables[r]);
    for (int r = 0; r < g; ++r) {
      const wc::Stats& x = rank_stats[r];
      // per-rank stage maxima: ranks run concurrently, the slowest sets the pace
      stages.map_ms = std::max(stages.map_ms, x.map_ms);
      stages.reduce_ms = std::max(stages.reduce_ms, x.reduce_ms);
      stages.finalize_ms = std::max(stages.finalize_ms, x.finalize_ms);
      stages.merge_ms = std::max(stages.merge_ms, x.merge_ms);
      stages.device_ms = std::max(stages.device_ms, x.device_ms);
      stages.host_count_ms = std::max(stages.host_count_ms, x.host_count_ms);
      stages.records += x.records;
      stages.chunks += x.chunks;
      stages.map_reruns += x.map_reruns;
      stages.table_splits += x.table_splits;
    }
  }
  const double secs = wc::now_seconds() - t0;
  write_out(wc::format_output(t, have_text ? reinterpret_cast<const uint8_t*>(text.data()) : nullptr,
                              have_text ? text.size() : 0, c.echo && have_text, c.list, c.top));
  const bool gpu_path = !(c.cpu || c.compat);
  char js[1536];
  std::snprintf(js, sizeof(js),
                "{\"bytes\": %llu, \"tokens\": %llu, \"keys\": %zu, \"seconds\": %.6f, \"gb_per_s\": %.3f, "
                "\"words_per_s\": %.1f, \"gpus\": %d, \"ranks\": %d, \"virtual_ranks\": %s, \"path\": \"%s\", "
                "\"count_seconds\": %.6f, \"count_gb_per_s\": %.3f, \"chunk_bytes\": %llu, "
                "\"device_ms\": {\"map\": %.3f, \"reduce\": %.3f, \"finalize\": %.3f, \"merge\": %.3f, "
                "\"total\": %.3f}, "
                "\"chunks\": %u, \"records\": %llu, \"map_reruns\": %u, \"table_splits\": %u}",
                (unsigned long long)bytes, (unsigned long long)t.total, t.size(), secs, bytes / secs / 1e9,
                t.total / secs, gpu_path ? gpus_used : 0, gpu_path ? ranks_used : 0,
                c.virtual_ranks > 0 ? "true" : "false", c.compat ? "compat" : (c.cpu ? "cpu" : "gpu"),
                stages.host_count_ms / 1e3, stages.host_count_ms > 0 ? bytes / (stages.host_count_ms * 1e6) : 0.0,
                (unsigned long long)c.chunk, stages.map_ms, stages.reduce_ms, stages.finalize_ms, stages.merge_ms,
                stages.device_ms,
                stages.chunks, (unsigned long long)stages.records, stages.map_reruns, stages.table_splits);
  if (c.bench) std::fprintf(stderr, "wordcount bench: %s\n", js);
  if (!c.bench_json.empty()) {
    FILE* f = std::fopen(c.bench_json.c_str(), "w");
    if (!f) wc::fail("cannot write " + c.bench_json);
    std::fprintf(f, "%s\n", js);
    std::fclose(f);
  }
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  try {
    return run(parse(argc, argv));
  } catch (const std::exception& ex) {
    std::fprintf(stderr, "wordcount: %s\n", ex.what());
    return 1;
  }
}
