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
void synth_host_into(uint8_t* out, uint64_t n, uint64_t first_segment, const SynthSpec& spec, const HostVocab& v);

}  // namespace wc
