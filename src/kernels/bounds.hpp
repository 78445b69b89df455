// bounds.hpp — device side of the finalize writers' bounds guard (kernels.hpp
// Bounds): a row index at or past the buffer's capacity is not written; the
// first such index is recorded with its kernel's id for the host to report.
#pragma once
#include <hip/hip_runtime.h>

#include "kernels.hpp"

namespace wc {
namespace dev {

__device__ __forceinline__ bool bounds_ok(const Bounds& g, uint32_t kernel, uint64_t row) {
  if (row < g.cap) return true;
  if (g.err) atomicCAS(g.err, 0ull, ((unsigned long long)kernel << 56) | (row & ((1ull << 56) - 1)));
  return false;
}

}  // namespace dev
}  // namespace wc
