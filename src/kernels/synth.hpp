// synth.hpp — deterministic synthetic text, bit-identical on host and device.
//
// The text is a sequence of SYNTH_SEG-byte segments; segment i depends only on
// (seed, i), so any byte range can be generated independently on any GPU
// (data-parallel shards, host-staged chunks) and re-generated on the host for
// the CPU oracle.  Words are drawn from a Zipf(s) vocabulary (frequent words
// short, rare words long — including >8-byte words that exercise the hashed
// key path), separated by ' ', with '\n' every 8-19 words.  The tail of each
// segment that cannot hold the next word is padded with '\n' (delimiters only).
#pragma once
#include <stdint.h>

#include "kernels.hpp"
#include "keys.hpp"

namespace wc {

constexpr uint32_t SYNTH_SEG = 1024;

WC_HD uint64_t splitmix64(uint64_t& s) {
  uint64_t z = (s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// Walks segment `seg`: calls word(rank, pos) for every word placed at byte
// `pos` of the segment (delimiters between words are one byte: ' ' or '\n'),
// and returns the number of bytes used (the rest is '\n' padding).
template <class Word>
WC_HD uint32_t synth_walk(uint64_t seg, uint64_t seed, const SynthVocab& v, Word&& word) {
  uint64_t st = seed ^ fmix64(seg + 0x632BE59BD9B4E019ull);
  uint32_t pos = 0, in_line = 0;
  uint32_t line_words = 8 + (uint32_t)(splitmix64(st) % 12);
  for (;;) {
    const uint64_t r = splitmix64(st);
    const uint32_t u = (uint32_t)r;
    uint32_t lo = 0, hi = v.n - 1;
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (v.cdf[mid] > u) hi = mid;
      else lo = mid + 1;
    }
    const uint32_t len = v.len[lo];
    if (pos + len + 1 > SYNTH_SEG) break;
    const bool nl = ++in_line >= line_words;
    word(lo, pos, nl);
    pos += len + 1;
    if (nl) {
      in_line = 0;
      line_words = 8 + (uint32_t)((r >> 40) % 12);
    }
  }
  return pos;
}

// Writes exactly SYNTH_SEG bytes to out.
WC_HD void synth_segment(uint64_t seg, uint64_t seed, const SynthVocab& v, uint8_t* out) {
  uint32_t pos = synth_walk(seg, seed, v, [&](uint32_t w, uint32_t p, bool nl) {
    const uint8_t* src = v.bytes + v.off[w];
    const uint32_t len = v.len[w];
    for (uint32_t i = 0; i < len; ++i) out[p + i] = src[i];
    out[p + len] = nl ? '\n' : ' ';
  });
  while (pos < SYNTH_SEG) out[pos++] = '\n';
}

}  // namespace wc
