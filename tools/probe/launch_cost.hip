// launch_cost.hip — host-side cost of hipLaunchKernelGGL on this box, by
// kernel-argument size and grid, and the GPU's idle gap from a host-seen
// completion to the next kernel's start (the per-job turnaround the engine pays:
// profiles/r6_session.md §4).
//
//   hipcc --offload-arch=gfx950 -O2 -o tools/probe/launch_cost tools/probe/launch_cost.hip
//   ./tools/probe/launch_cost
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                   \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
      std::exit(1);                                                                \
    }                                                                              \
  } while (0)

template <int B>
struct Args {
  unsigned long long w[B / 8];
};

template <int B>
__global__ void k_args(Args<B> a, unsigned long long* out) {
  if (blockIdx.x == 0 && threadIdx.x == 0 && a.w[0] == 12345) out[0] = a.w[B / 8 - 1];
}

// one word stored with system scope: the host spins on it (as wc_publish)
__global__ void k_flag(unsigned* flag, unsigned v) {
  __threadfence_system();
  if (threadIdx.x == 0) __hip_atomic_store(flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void k_stamp(unsigned long long* t) {
  if (threadIdx.x == 0 && blockIdx.x == 0) t[0] = wall_clock64();
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

template <int B>
static void bench_args(hipStream_t s, unsigned long long* out, unsigned grid, unsigned block) {
  Args<B> a{};
  const int N = 2000;
  for (int i = 0; i < 50; ++i) hipLaunchKernelGGL(k_args<B>, dim3(grid), dim3(block), 0, s, a, out);
  CHECK(hipStreamSynchronize(s));
  // host cost per launch while the GPU is busy (launches queue up)
  const double t0 = now_us();
  for (int i = 0; i < N; ++i) hipLaunchKernelGGL(k_args<B>, dim3(grid), dim3(block), 0, s, a, out);
  const double t1 = now_us();
  CHECK(hipStreamSynchronize(s));
  // host cost of one launch into an idle stream (the engine's first launch of a job)
  double idle = 0;
  for (int i = 0; i < 200; ++i) {
    const double u0 = now_us();
    hipLaunchKernelGGL(k_args<B>, dim3(grid), dim3(block), 0, s, a, out);
    idle += now_us() - u0;
    CHECK(hipStreamSynchronize(s));
  }
  printf("kernarg %4d B grid %5u x %4u: back-to-back %.2f us/launch, into an idle stream %.2f us\n", B + 8, grid,
         block, (t1 - t0) / N, idle / 200);
}

int main() {
  hipStream_t s;
  CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  unsigned long long* out;
  CHECK(hipMalloc(&out, 64));
  bench_args<8>(s, out, 1, 64);
  bench_args<256>(s, out, 1, 64);
  bench_args<512>(s, out, 1, 64);
  bench_args<1024>(s, out, 1, 64);
  bench_args<2048>(s, out, 1, 64);
  bench_args<1024>(s, out, 512, 1024);
  // turnaround: GPU writes a flag, host spins, host launches the next kernel;
  // the GPU clock gap between the flag kernel's end and the next kernel's start
  unsigned* flag;
  CHECK(hipHostMalloc(&flag, 64, hipHostMallocDefault));
  unsigned long long* ts;
  CHECK(hipMalloc(&ts, 64));
  double gap = 0, spin = 0;
  const int R = 200;
  int freq_khz = 0;
  CHECK(hipDeviceGetAttribute(&freq_khz, hipDeviceAttributeWallClockRate, 0));
  for (int i = 1; i <= R; ++i) {
    hipLaunchKernelGGL(k_stamp, dim3(1), dim3(64), 0, s, ts);
    hipLaunchKernelGGL(k_flag, dim3(1), dim3(64), 0, s, flag, (unsigned)i);
    const double u0 = now_us();
    while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != (unsigned)i) __builtin_ia32_pause();
    spin += now_us() - u0;
    hipLaunchKernelGGL(k_stamp, dim3(1), dim3(64), 0, s, ts + 1);
    CHECK(hipStreamSynchronize(s));
    unsigned long long h[2];
    CHECK(hipMemcpy(h, ts, 16, hipMemcpyDeviceToHost));
    gap += (double)(h[1] - h[0]) * 1e3 / freq_khz;
  }
  printf("turnaround: stamp -> flag -> host spin -> launch -> stamp: %.2f us on the GPU clock (host spin %.2f us)\n",
         gap / R, spin / R);
  CHECK(hipFree(ts));
  CHECK(hipHostFree(flag));
  CHECK(hipFree(out));
  CHECK(hipStreamDestroy(s));
  return 0;
}
