#pragma once
#include <stdint.h>

#include <string>
#include <vector>

#include "../kernels/kernels.hpp"
#include "wc/wc.hpp"

namespace wc {

struct HostVocab {
  std::vector<uint8_t> bytes;
  std::vector<uint32_t> off;
  std::vector<uint8_t> len;
  std::vector<uint32_t> cdf;
  SynthVocab view() const;  // host pointers
};

HostVocab build_vocab(const SynthSpec& spec);
// n bytes of the stream from segment first_segment into out, on `threads` threads.
void synth_host_into(uint8_t* out, uint64_t n, uint64_t first_segment, const SynthSpec& spec, const HostVocab& v,
                     int threads = 1);

}  // namespace wc
