// synth_oracle.cpp — exact counts of the synthetic stream, for validating the
// benchmark at full scale.
//
// The generator (kernels/synth.hpp) places whole vocabulary words separated by
// single delimiters, so the word count of a segment range is known without
// tokenizing anything: synth_walk reports (rank, position) of every word and
// the oracle adds one to that rank.  Segments are split over threads; a
// trailing partial segment is generated and tokenized byte-wise (a word cut by
// the end of the stream is a different, shorter token).
#include <algorithm>
#include <map>
#include <string>
#include <thread>
#include <vector>

#include "../io/synth_host.hpp"
#include "../kernels/synth.hpp"
#include "wc/wc.hpp"

namespace wc {
namespace cpu {

KeyTable count_synth(uint64_t n, uint64_t first_segment, const SynthSpec& spec, uint64_t global_base, int threads) {
  const HostVocab hv = build_vocab(spec);
  const SynthVocab v = hv.view();
  const uint64_t full = n / SYNTH_SEG, tail = n % SYNTH_SEG;
  const int T = std::max(1, std::min<int>(threads > 0 ? threads : (int)std::thread::hardware_concurrency(), 64));
  std::vector<std::vector<uint64_t>> cnt(T), first(T);
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t) {
    th.emplace_back([&, t] {
      cnt[t].assign(v.n, 0);
      first[t].assign(v.n, ~0ull);
      const uint64_t s0 = full * t / T, s1 = full * (t + 1) / T;
      uint64_t* c = cnt[t].data();
      uint64_t* f = first[t].data();
      for (uint64_t s = s0; s < s1; ++s) {
        const uint64_t base = global_base + s * SYNTH_SEG;
        synth_walk(first_segment + s, spec.seed, v, [&](uint32_t w, uint32_t p, bool) {
          if (c[w]++ == 0) f[w] = base + p;  // segments of a thread run in order
        });
      }
    });
  }
  for (auto& x : th) x.join();
  // fold the threads (thread order = offset order, so min == first seen)
  std::vector<uint64_t> C(v.n, 0), F(v.n, ~0ull);
  for (int t = 0; t < T; ++t)
    for (uint32_t w = 0; w < v.n; ++w) {
      C[w] += cnt[t][w];
      F[w] = std::min(F[w], first[t][w]);
    }
  // trailing partial segment: bytes, tokenized
  std::map<std::string, std::pair<uint64_t, uint64_t>> extra;  // word -> (count, first)
  if (tail) {
    uint8_t seg[SYNTH_SEG];
    synth_segment(first_segment + full, spec.seed, v, seg);
    const uint64_t base = global_base + full * SYNTH_SEG;
    uint64_t i = 0;
    while (i < tail) {
      while (i < tail && is_delim(seg[i])) ++i;
      if (i >= tail) break;
      const uint64_t s = i;
      while (i < tail && !is_delim(seg[i])) ++i;
      const std::string w(reinterpret_cast<const char*>(seg) + s, i - s);
      auto it = extra.find(w);
      if (it == extra.end()) extra.emplace(w, std::make_pair(1ull, base + s));
      else it->second.first++;
    }
  }
  struct Row {
    uint64_t first;
    std::string word;
    uint64_t count;
  };
  std::vector<Row> rows;
  std::map<std::string, size_t> vocab_row;
  for (uint32_t w = 0; w < v.n; ++w) {
    if (!C[w]) continue;
    rows.push_back({F[w], std::string(reinterpret_cast<const char*>(v.bytes) + v.off[w], v.len[w]), C[w]});
    if (!extra.empty()) vocab_row.emplace(rows.back().word, rows.size() - 1);
  }
  for (auto& e : extra) {  // a cut word may equal a vocabulary word
    auto it = vocab_row.find(e.first);
    if (it != vocab_row.end()) {
      rows[it->second].count += e.second.first;
      rows[it->second].first = std::min(rows[it->second].first, e.second.second);
    } else {
      rows.push_back({e.second.second, e.first, e.second.first});
    }
  }
  std::sort(rows.begin(), rows.end(), [](const Row& a, const Row& b) { return a.first < b.first; });
  KeyTable kt;
  kt.words.reserve(rows.size());
  for (auto& r : rows) {
    kt.words.push_back(std::move(r.word));
    kt.counts.push_back(r.count);
    kt.first_off.push_back(r.first);
    kt.total += r.count;
  }
  return kt;
}

}  // namespace cpu
}  // namespace wc
