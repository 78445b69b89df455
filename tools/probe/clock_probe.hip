// Clock / latency probe for small latency-bound kernels (first-occurrence order work):
// shader clock vs the 100 MHz wall clock, and the cost of a one-wave register
// bitonic sort (shuffles) and of an LDS bitonic sort, measured inside the kernel.
// hipcc --offload-arch=gfx950 -O3 tools/probe/clock_probe.hip -o tools/probe/clock_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int m) {
  const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, m), hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), m);
  return (uint64_t)hi << 32 | lo;
}
template <int R>
__device__ __forceinline__ void wave_sort(uint64_t (&v)[R]) {
  constexpr int N = 64 * R;
  const uint32_t lane = __lane_id();
#pragma unroll
  for (int size = 2; size <= N; size *= 2) {
#pragma unroll
    for (int stride = size / 2; stride > 0; stride /= 2) {
      if (stride >= 64) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const int q = r ^ (stride / 64);
          if (q < r) continue;
          const bool asc = ((r * 64) & size) == 0;
          const uint64_t x = v[r], y = v[q];
          const bool sw = (x > y) == asc;
          v[r] = sw ? y : x;
          v[q] = sw ? x : y;
        }
      } else {
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const uint64_t p = shfl_xor64(v[r], stride);
          const bool asc = (((uint32_t)(r * 64) + lane) & (uint32_t)size) == 0;
          const bool lower = (lane & (uint32_t)stride) == 0;
          const uint64_t mn = v[r] < p ? v[r] : p, mx = v[r] < p ? p : v[r];
          v[r] = lower == asc ? mn : mx;
        }
      }
    }
  }
}

// out[0..): per block 8 stamps: clock64/wall64 at start, after phase 1, after phase 2, end
__global__ void k_freq(uint64_t* out, int iters) {
  uint64_t c0 = clock64(), w0 = wall_clock64();
  uint32_t x = threadIdx.x;
  for (int i = 0; i < iters; ++i) x = x * 1664525u + 1013904223u;
  uint64_t c1 = clock64(), w1 = wall_clock64();
  if (threadIdx.x == 0) { out[0] = c0; out[1] = w0; out[2] = c1; out[3] = w1; out[4] = x; }
}

template <int R>
__global__ void k_wsort(const uint64_t* in, uint64_t* outk, uint64_t* st) {
  uint64_t v[R];
  const uint32_t lane = __lane_id();
  for (int r = 0; r < R; ++r) v[r] = in[r * 64 + lane];
  uint64_t c0 = clock64(), w0 = wall_clock64();
  wave_sort<R>(v);
  uint64_t c1 = clock64(), w1 = wall_clock64();
  for (int r = 0; r < R; ++r) outk[r * 64 + lane] = v[r];
  if (lane == 0) { st[0] = c0; st[1] = w0; st[2] = c1; st[3] = w1; }
}

template <int T>
__global__ void k_lsort(const uint64_t* in, uint64_t* outk, uint64_t* st, int P) {
  __shared__ uint64_t k[8192];
  for (int i = threadIdx.x; i < P; i += T) k[i] = in[i];
  __syncthreads();
  uint64_t c0 = clock64(), w0 = wall_clock64();
  for (uint32_t size = 2; size <= (uint32_t)P; size <<= 1)
    for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
      __syncthreads();
      for (uint32_t t = threadIdx.x; t < (uint32_t)P / 2; t += T) {
        const uint32_t i = 2 * t - (t & (stride - 1)), j = i + stride;
        const uint64_t a = k[i], b = k[j];
        if ((a > b) == ((i & size) == 0)) { k[i] = b; k[j] = a; }
      }
    }
  __syncthreads();
  uint64_t c1 = clock64(), w1 = wall_clock64();
  for (int i = threadIdx.x; i < P; i += T) outk[i] = k[i];
  if (threadIdx.x == 0) { st[0] = c0; st[1] = w0; st[2] = c1; st[3] = w1; }
}

// straight-line code: N unrolled dependent-free VALU steps (~8 B each) — the
// cost of fetching cold instructions
template <int N>
__global__ void k_straight(uint64_t* st, uint32_t seed) {
  uint64_t c0 = clock64(), w0 = wall_clock64();
  uint32_t a = seed + threadIdx.x, b = a ^ 0x55aa, c = a * 3, d = a + 7;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    a = __builtin_amdgcn_alignbyte(a, b, i & 3) + (uint32_t)i;
    b = __builtin_amdgcn_alignbyte(b, c, (i + 1) & 3) ^ (uint32_t)(i * 7);
    c = __builtin_amdgcn_alignbyte(c, d, (i + 2) & 3) + a;
    d = __builtin_amdgcn_alignbyte(d, a, (i + 3) & 3) ^ b;
  }
  uint64_t c1 = clock64(), w1 = wall_clock64();
  if (threadIdx.x == 0) { st[0] = c0; st[1] = w0; st[2] = c1; st[3] = w1; st[4] = a ^ b ^ c ^ d; }
}

template <int N>
__global__ void k_looped(uint64_t* st, uint32_t seed) {
  uint64_t c0 = clock64(), w0 = wall_clock64();
  uint32_t a = seed + threadIdx.x, b = a ^ 0x55aa, c = a * 3, d = a + 7;
#pragma unroll 1
  for (int i = 0; i < N; i += 4) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int ii = i + q;
      a = __builtin_amdgcn_alignbyte(a, b, q & 3) + (uint32_t)ii;
      b = __builtin_amdgcn_alignbyte(b, c, (q + 1) & 3) ^ (uint32_t)(ii * 7);
      c = __builtin_amdgcn_alignbyte(c, d, (q + 2) & 3) + a;
      d = __builtin_amdgcn_alignbyte(d, a, (q + 3) & 3) ^ b;
    }
  }
  uint64_t c1 = clock64(), w1 = wall_clock64();
  if (threadIdx.x == 0) { st[0] = c0; st[1] = w0; st[2] = c1; st[3] = w1; st[4] = a ^ b ^ c ^ d; }
}

// one lane chases `steps` dependent loads: idx = buf[idx]
__global__ void k_chase(const uint64_t* buf, uint64_t start, int steps, uint64_t* st) {
  uint64_t idx = start;
  uint64_t c0 = clock64(), w0 = wall_clock64();
  for (int i = 0; i < steps; ++i) idx = __builtin_nontemporal_load(&buf[idx]);
  uint64_t c1 = clock64(), w1 = wall_clock64();
  st[0] = c0; st[1] = w0; st[2] = c1; st[3] = w1; st[4] = idx;
}
__global__ void k_fill_chain(uint64_t* buf, uint64_t n, uint64_t stride_elems, uint64_t steps) {
  // element j*stride -> (j+1)*stride (mod n), a permuted order to defeat prefetch
  for (uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < steps; j += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t a = (j * 2654435761ull) % steps, b = ((j + 1) * 2654435761ull) % steps;
    buf[(a * stride_elems) % n] = (b * stride_elems) % n;
  }
}

__global__ void k_write(uint64_t* buf, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    buf[i] = i * 3;
}
// st: [0] max(load done - entry), [1] min entry, [2] max entry, [3] max(end - entry)
__global__ void k_read1(const uint64_t* buf, uint64_t* out, unsigned long long* st) {
  const uint64_t t0 = wall_clock64();
  const uint64_t v = buf[blockIdx.x * 256 + threadIdx.x];
  __syncthreads();
  const uint64_t t1 = wall_clock64();
  out[blockIdx.x * 256 + threadIdx.x] = v + 1;
  if (threadIdx.x == 0) {
    atomicMax(&st[0], (unsigned long long)(t1 - t0));
    atomicMin(&st[1], (unsigned long long)t0);
    atomicMax(&st[2], (unsigned long long)t0);
    atomicMax(&st[3], (unsigned long long)(wall_clock64() - t0));
  }
}

// Scattered 12-byte stores: `active` of 64 lanes store per instruction, each to
// a different bucket region (256 regions of this block, sequential within a
// region), `total` records per wave either way.
struct R12 { uint32_t a, b, c; };
__global__ void __launch_bounds__(1024) k_scatter(R12* out, int active, int total, uint64_t* st) {
  __shared__ uint32_t cur[256];
  for (int i = threadIdx.x; i < 256; i += 1024) cur[i] = 0;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63;
  R12* base = out + (size_t)blockIdx.x * 256 * 8192;
  uint32_t x = threadIdx.x * 2654435761u + blockIdx.x;
  const int iters = total / active;
  uint64_t t0 = wall_clock64();
  for (int it = 0; it < iters; ++it) {
    x = x * 1664525u + 1013904223u;
    if ((int)lane < active) {
      const uint32_t b = x >> 24;
      const uint32_t pos = atomicAdd(&cur[b], 1u) & 8191u;
      R12 r{x, x ^ 1u, (uint32_t)it};
      base[(size_t)b * 8192 + pos] = r;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) atomicMax((unsigned long long*)st, (unsigned long long)(wall_clock64() - t0));
}

// busy kernel: keeps every CU at work for a while (clock ramp)
__global__ void k_busy(uint32_t* out, int iters) {
  uint32_t x = threadIdx.x + blockIdx.x;
  for (int i = 0; i < iters; ++i) x = x * 1664525u + 1013904223u;
  if (x == 12345) out[0] = x;
}

static void report(const char* name, const uint64_t* h) {
  const double cyc = (double)(h[2] - h[0]), wall = (double)(h[3] - h[1]);  // wall at 100 MHz
  printf("%-28s clock %9.0f  wall %8.2f us  -> %6.0f MHz shader\n", name, cyc, wall / 100.0, cyc / wall * 100.0);
}

int main() {
  uint64_t *d_in, *d_out, *d_st;
  uint32_t* d_b;
  CK(hipMalloc(&d_in, 8192 * 8));
  CK(hipMalloc(&d_out, 8192 * 8));
  CK(hipMalloc(&d_st, 64 * 8));
  CK(hipMalloc(&d_b, 64));
  std::vector<uint64_t> h(8192);
  uint64_t x = 88172645463325252ull;
  for (auto& v : h) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; v = x >> 20; }
  CK(hipMemcpy(d_in, h.data(), 8192 * 8, hipMemcpyHostToDevice));
  uint64_t st[8];
  for (int rep = 0; rep < 2; ++rep) {
    printf("--- %s\n", rep == 0 ? "idle GPU" : "right after a 20 ms all-CU busy kernel");
    if (rep == 1) hipLaunchKernelGGL(k_busy, dim3(4096), dim3(256), 0, 0, d_b, 2000000);
    hipLaunchKernelGGL(k_freq, dim3(1), dim3(64), 0, 0, d_st, 100000);
    CK(hipMemcpy(st, d_st, 64, hipMemcpyDeviceToHost));
    report("freq loop (100k dep. ops)", st);
    if (rep == 1) hipLaunchKernelGGL(k_busy, dim3(4096), dim3(256), 0, 0, d_b, 2000000);
    hipLaunchKernelGGL(k_wsort<4>, dim3(1), dim3(64), 0, 0, d_in, d_out, d_st);
    CK(hipMemcpy(st, d_st, 64, hipMemcpyDeviceToHost));
    report("wave_sort<4> (256 keys)", st);
    if (rep == 1) hipLaunchKernelGGL(k_busy, dim3(4096), dim3(256), 0, 0, d_b, 2000000);
    hipLaunchKernelGGL(k_wsort<8>, dim3(1), dim3(64), 0, 0, d_in, d_out, d_st);
    CK(hipMemcpy(st, d_st, 64, hipMemcpyDeviceToHost));
    report("wave_sort<8> (512 keys)", st);
    for (int P : {256, 2048, 4096}) {
      if (rep == 1) hipLaunchKernelGGL(k_busy, dim3(4096), dim3(256), 0, 0, d_b, 2000000);
      hipLaunchKernelGGL(k_lsort<1024>, dim3(1), dim3(1024), 0, 0, d_in, d_out, d_st, P);
      CK(hipMemcpy(st, d_st, 64, hipMemcpyDeviceToHost));
      char nm[64];
      snprintf(nm, sizeof nm, "LDS bitonic %d, 1024 thr", P);
      report(nm, st);
    }
    hipLaunchKernelGGL(k_looped<8192>, dim3(1), dim3(64), 0, 0, d_st, 1u);
    CK(hipMemcpy(st, d_st, 64, hipMemcpyDeviceToHost));
    report("looped 8192 steps", st);
    for (int twice = 0; twice < 2; ++twice) {
      hipLaunchKernelGGL(k_straight<2048>, dim3(1), dim3(64), 0, 0, d_st, 1u);
      CK(hipMemcpy(st, d_st, 64, hipMemcpyDeviceToHost));
      report(twice ? "straight 8192 ops (again)" : "straight 8192 ops (cold)", st);
    }
  }
  {
    const uint64_t nbytes = 4ull << 30, n = nbytes / 8;
    uint64_t* big;
    CK(hipMalloc(&big, nbytes));
    const uint64_t strides[] = {8, 512, 8192, 262144, 33554432 + 8};  // 64 B, 4 KiB, 64 KiB, 2 MiB, 256 MiB (elements)
    const char* names[] = {"64 B", "4 KiB", "64 KiB", "2 MiB", "256 MiB"};
    for (int si = 0; si < 5; ++si) {
      const uint64_t steps = 4096;
      hipLaunchKernelGGL(k_fill_chain, dim3(64), dim3(256), 0, 0, big, n, strides[si], steps);
      CK(hipDeviceSynchronize());
      hipLaunchKernelGGL(k_busy, dim3(4096), dim3(256), 0, 0, d_b, 200000);
      for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(k_chase, dim3(1), dim3(1), 0, 0, big, 0ull, 256, d_st);
        CK(hipMemcpy(st, d_st, 64, hipMemcpyDeviceToHost));
        const double cyc = (double)(st[2] - st[0]), wall = (double)(st[3] - st[1]);
        printf("chase stride %-8s %s: %7.0f ns per dependent load\n", names[si], rep ? "warm" : "cold",
               wall * 10.0 / 256);
      }
    }
    CK(hipFree(big));
  }
  {
    uint64_t *a, *o2;
    unsigned long long* dst4;
    CK(hipMalloc(&a, 64 << 20));
    CK(hipMalloc(&o2, 64 << 20));
    CK(hipMalloc(&dst4, 64));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int variant = 0; variant < 4; ++variant) {
      unsigned long long init[4] = {0, ~0ull, 0, 0};
      CK(hipMemcpy(dst4, init, 32, hipMemcpyHostToDevice));
      if (variant == 0) hipLaunchKernelGGL(k_write, dim3(1024), dim3(256), 0, 0, a, (uint64_t)(8 << 20));  // just written
      if (variant == 1) hipLaunchKernelGGL(k_busy, dim3(4096), dim3(256), 0, 0, d_b, 200000);              // data older
      if (variant == 2) { hipLaunchKernelGGL(k_write, dim3(1024), dim3(256), 0, 0, o2, (uint64_t)(8 << 20)); }
      CK(hipEventRecord(e0, 0));
      hipLaunchKernelGGL(k_read1, dim3(512), dim3(256), 0, 0, a, o2 + (variant == 3 ? 0 : (1 << 20)), dst4);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      unsigned long long h4[4];
      CK(hipMemcpy(h4, dst4, 32, hipMemcpyDeviceToHost));
      const char* vn[4] = {"after writer of same buf", "after busy kernel", "after writer of other buf", "repeat"};
      printf("read1 %-26s event %6.2f us | block: load+sync %5.2f us, entry spread %5.2f us, block max %5.2f us\n",
             vn[variant], ms * 1e3, h4[0] / 100.0, (h4[2] - h4[1]) / 100.0, h4[3] / 100.0);
    }
  }
  {
    R12* out;
    CK(hipMalloc(&out, (size_t)256 * 256 * 8192 * sizeof(R12)));
    for (int active : {64, 32, 19, 8}) {
      CK(hipMemset(d_st, 0, 8));
      hipLaunchKernelGGL(k_scatter, dim3(256), dim3(1024), 0, 0, out, active, 4096, d_st);
      CK(hipMemset(d_st, 0, 8));
      hipLaunchKernelGGL(k_scatter, dim3(256), dim3(1024), 0, 0, out, active, 4096, d_st);
      CK(hipMemcpy(st, d_st, 8, hipMemcpyDeviceToHost));
      printf("scatter 12B records, %2d active lanes/instr, 4096 per wave x 16 waves x 256 CUs: %8.1f us\n", active,
             st[0] / 100.0);
    }
    CK(hipFree(out));
  }
  std::vector<uint64_t> o(512);
  hipLaunchKernelGGL(k_wsort<8>, dim3(1), dim3(64), 0, 0, d_in, d_out, d_st);
  CK(hipMemcpy(o.data(), d_out, 512 * 8, hipMemcpyDeviceToHost));
  bool ok = true;
  for (int i = 1; i < 512; ++i) ok &= o[i - 1] <= o[i];
  printf("wave_sort<8> sorted: %s\n", ok ? "yes" : "NO");
  return 0;
}
