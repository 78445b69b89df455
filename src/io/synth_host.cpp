// synth_host.cpp — vocabulary construction for the synthetic text stream and
// the host copy of the generator (bit-identical to wc_synth_text).
#include "synth_host.hpp"

#include <algorithm>
#include <cmath>
#include <thread>
#include <unordered_set>

#include "../kernels/synth.hpp"

namespace wc {

HostVocab build_vocab(const SynthSpec& spec) {
  HostVocab v;
  const uint32_t n = spec.vocab < 1 ? 1 : spec.vocab;
  std::unordered_set<std::string> seen;
  seen.reserve(n * 2);
  uint64_t st = spec.seed * 0xA24BAED4963EE407ull + 0x9FB21C651E98DF25ull;
  v.off.reserve(n);
  v.len.reserve(n);
  // long_frac: each rank independently becomes a 16..64-byte word (its own
  // stream, so long_frac = 0 leaves the vocabulary bit-identical)
  uint64_t lst = spec.seed * 0xD1B54A32D192ED03ull + 0x8CB92BA72F3D8DD7ull;
  const uint64_t long_cut = (uint64_t)(std::min(std::max(spec.long_frac, 0.0), 1.0) * 18446744073709551615.0);
  for (uint32_t i = 0; i < n; ++i) {
    // Frequent ranks are short words, rare ranks long (English-like); ~10% of
    // the vocabulary is longer than 8 bytes.
    const double lg = std::log2((double)i + 2.0);
    const uint64_t lr = spec.long_frac > 0 ? splitmix64(lst) : ~0ull;
    const bool is_long = spec.long_frac > 0 && (spec.long_frac >= 1.0 || lr < long_cut);
    std::string w;
    for (int attempt = 0;; ++attempt) {
      const uint64_t r = splitmix64(st);
      uint32_t len = 1 + (uint32_t)(lg * 0.45) + (uint32_t)(r % 4) + (uint32_t)attempt / 4;
      if (len > 24) len = 24;
      if (is_long) len = 16 + (uint32_t)((r >> 8) % 49) + (uint32_t)attempt / 4;  // 16..64 (+ retries)
      w.assign(len, 'a');
      uint64_t bits = splitmix64(st);
      for (uint32_t c = 0; c < len; ++c) {
        if (c % 12 == 11) bits = splitmix64(st);
        w[c] = (char)('a' + (bits % 26));
        bits /= 26;
      }
      if ((r >> 20) % 16 == 0) w[0] = (char)(w[0] - 'a' + 'A');  // some capitalised words
      if (seen.insert(w).second) break;
    }
    v.off.push_back((uint32_t)v.bytes.size());
    v.len.push_back((uint8_t)w.size());
    v.bytes.insert(v.bytes.end(), w.begin(), w.end());
  }
  // Zipf(s) CDF scaled to 2^32.
  std::vector<double> p(n);
  double z = 0;
  for (uint32_t i = 0; i < n; ++i) z += p[i] = 1.0 / std::pow((double)i + 1.0, spec.zipf_s);
  v.cdf.resize(n);
  double acc = 0;
  for (uint32_t i = 0; i < n; ++i) {
    acc += p[i] / z;
    double c = acc * 4294967296.0;
    v.cdf[i] = c >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)c;
  }
  v.cdf[n - 1] = 0xFFFFFFFFu;
  return v;
}

SynthVocab HostVocab::view() const {
  SynthVocab s;
  s.bytes = bytes.data();
  s.off = off.data();
  s.len = len.data();
  s.cdf = cdf.data();
  s.n = (uint32_t)off.size();
  return s;
}

void synth_host_into(uint8_t* out, uint64_t n, uint64_t first_segment, const SynthSpec& spec, const HostVocab& v,
                     int threads) {
  const SynthVocab sv = v.view();
  const uint64_t nseg = (n + SYNTH_SEG - 1) / SYNTH_SEG;
  // segments are independent: T threads write disjoint ranges of `out`
  const int T = (int)std::max<uint64_t>(1, std::min<uint64_t>(threads > 0 ? (uint64_t)threads : 1, nseg / 64 + 1));
  auto work = [&](uint64_t s0, uint64_t s1) {
    uint8_t seg[SYNTH_SEG];
    for (uint64_t s = s0; s < s1; ++s) {
      const uint64_t base = s * SYNTH_SEG;
      if (base + SYNTH_SEG <= n) {
        synth_segment(first_segment + s, spec.seed, sv, out + base);
      } else {
        synth_segment(first_segment + s, spec.seed, sv, seg);
        for (uint64_t i = 0; base + i < n; ++i) out[base + i] = seg[i];
      }
    }
  };
  std::vector<std::thread> th;
  for (int t = 1; t < T; ++t) th.emplace_back(work, nseg * t / T, nseg * (t + 1) / T);
  work(0, nseg / T);
  for (auto& x : th) x.join();
}

std::vector<uint8_t> synth_host(uint64_t n, uint64_t first_segment, const SynthSpec& spec) {
  std::vector<uint8_t> out(n);
  synth_host_into(out.data(), n, first_segment, spec, build_vocab(spec), 1);
  return out;
}

}  // namespace wc
