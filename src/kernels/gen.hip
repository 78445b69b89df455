// gen.hip — wc_synth_text: device-side synthetic text generator.
// One thread builds one 1 KiB segment in LDS, then the block writes its
// 64 KiB out with 16-B coalesced stores.  Used so 1 GB - 256 GB benchmark
// inputs never touch host memory or PCIe.
#include "kernels.hpp"
#include "synth.hpp"

namespace wc {
namespace dev {

constexpr int GEN_THREADS = 64;

__global__ void __launch_bounds__(GEN_THREADS) wc_synth_text(uint8_t* out, uint64_t n, uint64_t first_segment,
                                                             uint64_t seed, SynthVocab v) {
  __shared__ __attribute__((aligned(16))) uint8_t buf[GEN_THREADS * SYNTH_SEG];
  const uint64_t nseg = (n + SYNTH_SEG - 1) / SYNTH_SEG;
  for (uint64_t blk = blockIdx.x; blk * GEN_THREADS < nseg; blk += gridDim.x) {
    const uint64_t seg = blk * GEN_THREADS + threadIdx.x;
    if (seg < nseg) synth_segment(first_segment + seg, seed, v, &buf[threadIdx.x * SYNTH_SEG]);
    __syncthreads();
    const uint64_t base = blk * GEN_THREADS * SYNTH_SEG;
    const uint64_t bytes = (n - base) < (uint64_t)GEN_THREADS * SYNTH_SEG ? (n - base) : (uint64_t)GEN_THREADS * SYNTH_SEG;
    for (uint64_t i = threadIdx.x * 16; i < bytes; i += GEN_THREADS * 16) {
      if (i + 16 <= bytes) {
        *reinterpret_cast<uint4*>(out + base + i) = *reinterpret_cast<const uint4*>(&buf[i]);
      } else {
        for (uint64_t j = i; j < bytes; ++j) out[base + j] = buf[j];
      }
    }
    __syncthreads();
  }
}

}  // namespace dev

void launch_synth(uint8_t* out, uint64_t n, uint64_t first_segment, uint64_t seed, const SynthVocab& v,
                  hipStream_t s) {
  const uint64_t nseg = (n + SYNTH_SEG - 1) / SYNTH_SEG;
  uint64_t blocks = (nseg + dev::GEN_THREADS - 1) / dev::GEN_THREADS;
  if (blocks > 65536) blocks = 65536;
  if (blocks == 0) return;
  hipLaunchKernelGGL(dev::wc_synth_text, dim3((unsigned)blocks), dim3(dev::GEN_THREADS), 0, s, out, n, first_segment,
                     seed, v);
}

}  // namespace wc
