// util.hip — two small launch-count kernels of the pass / finalize plumbing.
//
//  wc_zero_regions  fills up to ZERO_MAX_REGIONS device regions (and does up to
//                   ZERO_MAX_COPIES small copies) in ONE launch:
//                   the per-pass counters + hot-key sampling state, and (after
//                   Engine::reset) the table occupancy and key-arena cursor.  It
//                   replaces four hipMemsetAsync calls whose host-side enqueue
//                   cost (~5-12 us each, profiles/r2_plumbing.md) left the GPU
//                   idle between the previous job's sync and the next map.
//  wc_publish       copies up to PUB_MAX_REGIONS small device regions (pass
//                   counters, bucket occupancy, key count, arena cursor) into
//                   page-locked host memory in ONE launch, instead of one
//                   copy-engine blit per region.
//
// Reference: the reference has neither (main.cu:143-161 copies its two result
// arrays with blocking cudaMemcpy); these exist because the MI355X step is
// ~1.4 ms and a dozen tiny host-enqueued operations per step are a few %.
#include <algorithm>

#include "../common/hip_util.hpp"
#include "kernels.hpp"
#include "zero_list.hpp"

namespace wc {
namespace dev {

__global__ void __launch_bounds__(256) wc_zero_regions(ZeroList z) {
  apply_zero_list(z, blockIdx.x * 256ull + threadIdx.x, (uint64_t)gridDim.x * 256, blockIdx.x == 0, 256);
}

__global__ void __launch_bounds__(256) wc_publish(PubList c) {
  for (int r = 0; r < c.n; ++r) {
    const uint32_t* src = c.src[r];
    uint32_t* dst = c.dst[r];
    for (uint32_t i = threadIdx.x; i < c.words[r]; i += 256) dst[i] = src[i];
  }
  __threadfence_system();
  if (c.seq_dst) {
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(c.seq_dst, c.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

}  // namespace dev

void launch_list_overflow(const char* what) { fail(std::string(what) + " (raise the list's bound)"); }

void launch_zero_regions(const ZeroList& z, hipStream_t s) {
  if (z.n == 0 && z.nc == 0) return;
  WC_CHECK(z.n <= ZERO_MAX_REGIONS && z.nc <= ZERO_MAX_COPIES, "launch_zero_regions: too many regions");
  uint64_t most = 0;
  for (int r = 0; r < z.n; ++r) most = z.words[r] > most ? z.words[r] : most;
  // up to 4 blocks per CU: a merge list fills ~10 MB (owner table, padding rows)
  const uint64_t blocks = std::min<uint64_t>(1024, std::max<uint64_t>(1, (most / 4 + 255) / 256));
  hipLaunchKernelGGL(dev::wc_zero_regions, dim3((unsigned)blocks), dim3(256), 0, s, z);
}

void launch_publish(const PubList& c, hipStream_t s) {
  if (c.n == 0) return;
  WC_CHECK(c.n <= PUB_MAX_REGIONS, "launch_publish: too many regions");
  hipLaunchKernelGGL(dev::wc_publish, dim3(1), dim3(256), 0, s, c);
}

}  // namespace wc
