// merge.hip — device kernels of the cross-GPU merge protocol:
// dictionary-union head flags, global-id assignment, dense combine, and a
// single-block exclusive scan.
#include "kernels.hpp"
#include "lds_table.hpp"

namespace wc {
namespace dev {

inline dim3 mgrid(uint64_t n) {
  uint64_t g = (n + 255) / 256;
  return dim3((unsigned)(g < 1 ? 1 : (g > 4096 ? 4096 : g)));
}

// flag[i] = 1 iff sorted entry i is a valid key differing from entry i-1.
__global__ void wc_union_flags(const uint32_t* pos, const uint64_t* K0, const uint64_t* K1, uint32_t* flag,
                               uint64_t m) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < m; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t p = pos[i];
    const bool valid = K1[p] != K1_EMPTY;
    bool head = valid;
    if (valid && i > 0) {
      const uint32_t q = pos[i - 1];
      head = !(K0[q] == K0[p] && K1[q] == K1[p]);
    }
    flag[i] = head ? 1u : 0u;
  }
}

// After an EXCLUSIVE scan of flags in `ex`: id = ex[i] (+ head) - 1.
__global__ void wc_union_assign(const uint32_t* pos, const uint32_t* flag, const uint32_t* ex, const uint64_t* K0,
                                const uint64_t* K1, const uint64_t* SO, const uint32_t* SL, uint64_t m,
                                uint64_t n_max, uint64_t arena_stride, uint32_t* id_of_pos, uint64_t* ok0,
                                uint64_t* ok1, uint64_t* osoff, uint32_t* oslen) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < m; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t p = pos[i];
    if (K1[p] == K1_EMPTY) continue;
    const uint32_t id = ex[i] + flag[i] - 1;
    id_of_pos[p] = id;
    if (flag[i]) {
      ok0[id] = K0[p];
      ok1[id] = K1[p];
      osoff[id] = SO[p] + (p / n_max) * arena_stride;  // owner = lowest rank holding the key
      oslen[id] = SL[p];
    }
  }
}

__global__ void wc_combine_u64(uint64_t* dst, const uint64_t* src, uint64_t n, int op) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t a = dst[i], b = src[i];
    dst[i] = op == 0 ? a + b : (op == 1 ? (a < b ? a : b) : (a > b ? a : b));
  }
}

// Pad: out[i] = i < n ? in[i] : fill.
__global__ void wc_pad_u64(const uint64_t* in, uint64_t n, uint64_t* out, uint64_t m, uint64_t fill) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < m; i += (uint64_t)gridDim.x * blockDim.x)
    out[i] = i < n ? in[i] : fill;
}

__global__ void __launch_bounds__(1024) wc_exclusive_scan_u32(const uint32_t* in, uint32_t* out, uint64_t m,
                                                              uint32_t* total) {
  __shared__ uint32_t wsum[16];
  __shared__ uint32_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (uint64_t base = 0; base < m; base += 1024) {
    const uint64_t i = base + threadIdx.x;
    const uint32_t v = i < m ? in[i] : 0;
    uint32_t x = v;
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(x, o);
      if (lane >= o) x += y;
    }
    if (lane == 63) wsum[wave] = x;
    __syncthreads();
    if (wave == 0) {
      uint32_t s = lane < 16 ? wsum[lane] : 0;
      for (int o = 1; o < 16; o <<= 1) {
        const uint32_t y = __shfl_up(s, o);
        if (lane >= o) s += y;
      }
      if (lane < 16) wsum[lane] = s;
    }
    __syncthreads();
    if (i < m) out[i] = carry + (wave ? wsum[wave - 1] : 0) + x - v;
    __syncthreads();
    if (threadIdx.x == 0) carry += wsum[15];
    __syncthreads();
  }
  if (threadIdx.x == 0) *total = carry;
}

}  // namespace dev

void launch_union_flags(const uint32_t* pos, const uint64_t* K0, const uint64_t* K1, uint32_t* flag, uint64_t m,
                        hipStream_t s) {
  if (m) hipLaunchKernelGGL(dev::wc_union_flags, dev::mgrid(m), dim3(256), 0, s, pos, K0, K1, flag, m);
}
void launch_union_assign(const uint32_t* pos, const uint32_t* flag, const uint32_t* ex, const uint64_t* K0,
                         const uint64_t* K1, const uint64_t* SO, const uint32_t* SL, uint64_t m, uint64_t n_max,
                         uint64_t arena_stride, uint32_t* id_of_pos, uint64_t* ok0, uint64_t* ok1, uint64_t* osoff,
                         uint32_t* oslen, hipStream_t s) {
  if (m)
    hipLaunchKernelGGL(dev::wc_union_assign, dev::mgrid(m), dim3(256), 0, s, pos, flag, ex, K0, K1, SO, SL, m, n_max,
                       arena_stride, id_of_pos, ok0, ok1, osoff, oslen);
}
void launch_combine_u64(uint64_t* dst, const uint64_t* src, uint64_t n, int op, hipStream_t s) {
  if (n) hipLaunchKernelGGL(dev::wc_combine_u64, dev::mgrid(n), dim3(256), 0, s, dst, src, n, op);
}
void launch_pad_u64(const uint64_t* in, uint64_t n, uint64_t* out, uint64_t m, uint64_t fill, hipStream_t s) {
  if (m) hipLaunchKernelGGL(dev::wc_pad_u64, dev::mgrid(m), dim3(256), 0, s, in, n, out, m, fill);
}
void launch_exclusive_scan_u32(const uint32_t* in, uint32_t* out, uint64_t m, uint32_t* total, hipStream_t s) {
  hipLaunchKernelGGL(dev::wc_exclusive_scan_u32, dim3(1), dim3(1024), 0, s, in, out, m, total);
}

}  // namespace wc
