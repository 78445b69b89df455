// comm.hip — the data movement of the stream-ordered loopback communicator
// (src/dist/comm.cpp LoopbackComm): N virtual ranks in one process, every
// collective ENQUEUED on the caller's stream like an RCCL collective (the
// host never waits for the GPU inside a collective).
//
// Each rank publishes its buffers in a page-locked metadata slot and records
// a "ready" event behind its earlier work; its stream then waits for every
// peer's ready event and runs wc_loopback_xfer, which reads the peers' buffer
// addresses from the metadata at run time, and records "done"; the stream
// waits for every peer's done before going on (send buffers are reusable once
// the collective completes on the stream, as with RCCL).  Protocol and its
// host side: src/dist/comm.cpp LoopbackComm.
// The reference has no communication at all.
#include "kernels.hpp"

namespace wc {
namespace dev {

__device__ __forceinline__ void copy_bytes_grid(uint8_t* dst, const uint8_t* src, uint64_t n, uint32_t part,
                                                uint32_t nparts) {
  const uint64_t tid = (uint64_t)part * blockDim.x + threadIdx.x, stride = (uint64_t)nparts * blockDim.x;
  if ((((uintptr_t)dst | (uintptr_t)src) & 15) == 0) {
    const uint64_t n16 = n / 16;
    for (uint64_t i = tid; i < n16; i += stride)
      reinterpret_cast<uint4*>(dst)[i] = reinterpret_cast<const uint4*>(src)[i];
    for (uint64_t i = n16 * 16 + tid; i < n; i += stride) dst[i] = src[i];
  } else if ((((uintptr_t)dst | (uintptr_t)src) & 7) == 0) {
    const uint64_t n8 = n / 8;
    for (uint64_t i = tid; i < n8; i += stride)
      reinterpret_cast<uint64_t*>(dst)[i] = reinterpret_cast<const uint64_t*>(src)[i];
    for (uint64_t i = n8 * 8 + tid; i < n; i += stride) dst[i] = src[i];
  } else {
    for (uint64_t i = tid; i < n; i += stride) dst[i] = src[i];
  }
}

// grid (LB_XFER_PARTS, W): blockIdx.y = the source rank p.
__global__ void __launch_bounds__(256) wc_loopback_xfer(LbXfer x) {
  __shared__ uint64_t sp[LB_MAX_RANKS];  // every rank's send buffer (reduce-scatter)
  __shared__ uint64_t s_src, s_dst, s_n;
  const volatile LbShared* sh = x.shared;
  if (sh->aborted) return;
  const uint32_t p = blockIdx.y;
  const volatile LbMeta& me = sh->meta[x.slot * x.world + x.rank];
  const volatile LbMeta& src = sh->meta[x.slot * x.world + p];
  if (x.kind == LB_REDUCE_SCATTER) {
    if (p != 0) return;
    for (uint32_t q = threadIdx.x; q < x.world; q += blockDim.x) sp[q] = sh->meta[x.slot * x.world + q].send;
    __syncthreads();
    uint64_t* recv = reinterpret_cast<uint64_t*>(me.recv);
    const uint64_t n = x.count, base = (uint64_t)x.rank * n;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
      uint64_t acc = reinterpret_cast<const uint64_t*>(sp[0])[base + i];
      for (uint32_t q = 1; q < x.world; ++q) {
        const uint64_t v = reinterpret_cast<const uint64_t*>(sp[q])[base + i];
        acc = x.op == 0 ? acc + v : (x.op == 1 ? (v < acc ? v : acc) : (v > acc ? v : acc));
      }
      recv[i] = acc;
    }
    return;
  }
  if (threadIdx.x == 0) {
    uint64_t from = 0, to = 0, n = 0;
    switch (x.kind) {
      case LB_ALLGATHER:
        from = src.send;
        to = me.recv + (uint64_t)p * x.count;
        n = x.count;
        break;
      case LB_ALLTOALLV:
        from = src.send + src.soff[x.rank];
        to = me.recv + me.roff[p];
        n = me.rbytes[p];
        break;
      case LB_BROADCAST:
        if (p == x.root && x.rank != x.root) {
          from = src.send;
          to = me.recv;
          n = x.count;
        }
        break;
      default:
        break;
    }
    s_src = from;
    s_dst = to;
    s_n = n;
  }
  __syncthreads();
  if (s_n)
    copy_bytes_grid(reinterpret_cast<uint8_t*>(s_dst), reinterpret_cast<const uint8_t*>(s_src), s_n, blockIdx.x,
                    gridDim.x);
}

}  // namespace dev

void launch_loopback_xfer(const LbXfer& x, hipStream_t s) {
  hipLaunchKernelGGL(dev::wc_loopback_xfer, dim3(LB_XFER_PARTS, x.world), dim3(256), 0, s, x);
}

}  // namespace wc
