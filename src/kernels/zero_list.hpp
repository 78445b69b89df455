// zero_list.hpp — device side of ZeroList (kernels.hpp): fills and small copies
// applied by one launch, either wc_zero_regions (util.hip) or folded into the
// head of another kernel that touches none of the regions (wc_hot_sample: a
// pass that samples hot words needs no launch of its own for its zeroing).
#pragma once
#include "kernels.hpp"

namespace wc {
namespace dev {

// Threads [0, nthreads) of the launch, thread `t`; copies by the first block
// (`block0`, threads t < bthreads).
__device__ __forceinline__ void apply_zero_list(const ZeroList& z, uint64_t t, uint64_t nthreads, bool block0,
                                                uint32_t bthreads) {
  for (int r = 0; r < z.n; ++r) {
    uint32_t* p = z.ptr[r];
    const uint64_t words = z.words[r];
    const uint32_t v = z.val[r];
    const uint64_t quads = (reinterpret_cast<uintptr_t>(p) & 15) == 0 ? words / 4 : 0;
    uint4* q = reinterpret_cast<uint4*>(p);
    for (uint64_t i = t; i < quads; i += nthreads) q[i] = make_uint4(v, v, v, v);
    for (uint64_t i = quads * 4 + t; i < words; i += nthreads) p[i] = v;
  }
  if (block0)
    for (int c = 0; c < z.nc; ++c)
      for (uint32_t i = (uint32_t)t; i < z.cwords[c]; i += bthreads) z.cdst[c][i] = z.csrc[c][i];
}

}  // namespace dev
}  // namespace wc
