// LDS bank-conflict probe: the share of LDS cycles lost to
// bank conflicts for the reduce's access pattern — 64 lanes probing RANDOM
// slots of a 4096-slot table — against conflict-free baselines.  Run under
//   rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES -- tools/probe/lds_conflicts
// (tools/lds_probe.sh); conflict share = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE.
// One 1024-thread block per CU, as the reduce.  Layout as RedLds: 80-byte slot
// groups (4 tags, 4 k1, 4 k0), then 8-byte counters and first offsets.
// hipcc --offload-arch=gfx950 -O3 tools/probe/lds_conflicts.hip -o tools/probe/lds_conflicts
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CK(x)                                                     \
  do {                                                            \
    hipError_t e = (x);                                           \
    if (e != hipSuccess) {                                        \
      printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); \
      return 1;                                                   \
    }                                                             \
  } while (0)

constexpr int GROUPS = 1024, SLOTS = 4096, ITERS = 256;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct alignas(16) Group {
  uint32_t tag[4];
  uint64_t k1[4], k0[4];
};
struct Lds {
  Group g[GROUPS];
  unsigned long long cnt[SLOTS], first[SLOTS];
};
// the split layout — tags alone at a 16-byte group stride,
// k1 / k0 in their own 8-byte-stride arrays (same 80 B per group in all)
struct LdsSplit {
  u32x4 tag[GROUPS];
  uint64_t k1[SLOTS], k0[SLOTS];
  unsigned long long cnt[SLOTS], first[SLOTS];
};

__device__ __forceinline__ uint32_t next(uint32_t& x) {  // per-lane LCG
  x = x * 1664525u + 1013904223u;
  return x >> 8;
}

// mode 0: random group tag reads (two per record, as g1 / g2); 1: the same
// reads, consecutive groups per lane (conflict-free layout); 2: random 8-byte
// atomics (count add + first-offset min); 3: the reduce's whole per-record
// pattern (two random tag reads, k1 / k0 of one slot, two atomics).
// Split layout (LdsSplit): 4 random tag reads, 5 consecutive tag reads, 6 the
// whole per-record pattern.
template <int MODE>
__global__ void __launch_bounds__(1024) k_probe_split(uint32_t* out, uint32_t seed) {
  __shared__ LdsSplit L;
  for (int i = threadIdx.x; i < GROUPS; i += 1024) L.tag[i] = u32x4{(uint32_t)i * 4, (uint32_t)i * 4 + 1, (uint32_t)i * 4 + 2, (uint32_t)i * 4 + 3};
  for (int i = threadIdx.x; i < SLOTS; i += 1024) {
    L.k0[i] = L.k1[i] = i >> 2;
    L.cnt[i] = L.first[i] = 0;
  }
  __syncthreads();
  uint32_t x = seed + threadIdx.x * 0x9E3779B9u + blockIdx.x * 7919u, acc = 0;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int it = 0; it < ITERS; ++it) {
    asm volatile("" ::: "memory");
    if (MODE == 4 || MODE == 6) {
      const uint32_t g1 = next(x) & (GROUPS - 1), g2 = next(x) & (GROUPS - 1);
      const u32x4 a = L.tag[g1], b = L.tag[g2];
      acc ^= a.x ^ b.y;
      if (MODE == 6) {
        const uint32_t s = (g1 * 4 + (acc & 3)) & (SLOTS - 1);
        acc ^= (uint32_t)L.k1[s] ^ (uint32_t)L.k0[s];
        atomicAdd(&L.cnt[s], 1ull);
        atomicMin(&L.first[s], (unsigned long long)it);
      }
    } else {
      const uint32_t g = (wave * 64 + lane + it * 2) & (GROUPS - 1);
      const u32x4 a = L.tag[g], b = L.tag[(g + 1) & (GROUPS - 1)];
      acc ^= a.x ^ b.y;
      (void)next(x);
      (void)next(x);
    }
  }
  __syncthreads();
  if (acc == 0x12345678u) out[threadIdx.x] = acc + (uint32_t)L.cnt[threadIdx.x];
}

template <int MODE>
__global__ void __launch_bounds__(1024) k_probe(uint32_t* out, uint32_t seed) {
  __shared__ Lds L;
  for (int i = threadIdx.x; i < GROUPS; i += 1024) {
    for (int j = 0; j < 4; ++j) {
      L.g[i].tag[j] = i * 4 + j;
      L.g[i].k0[j] = L.g[i].k1[j] = i;
    }
  }
  for (int i = threadIdx.x; i < SLOTS; i += 1024) L.cnt[i] = L.first[i] = 0;
  __syncthreads();
  uint32_t x = seed + threadIdx.x * 0x9E3779B9u + blockIdx.x * 7919u, acc = 0;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int it = 0; it < ITERS; ++it) {
    asm volatile("" ::: "memory");
    if (MODE == 0 || MODE == 3) {
      const uint32_t g1 = next(x) & (GROUPS - 1), g2 = next(x) & (GROUPS - 1);
      const u32x4 a = *reinterpret_cast<const u32x4*>(L.g[g1].tag);
      const u32x4 b = *reinterpret_cast<const u32x4*>(L.g[g2].tag);
      acc ^= a.x ^ b.y;
      if (MODE == 3) {
        const uint32_t s = (g1 * 4 + (acc & 3)) & (SLOTS - 1);
        acc ^= (uint32_t)L.g[s >> 2].k1[s & 3] ^ (uint32_t)L.g[s >> 2].k0[s & 3];
        atomicAdd(&L.cnt[s], 1ull);
        atomicMin(&L.first[s], (unsigned long long)it);
      }
    } else if (MODE == 1) {
      const uint32_t g = (wave * 64 + lane + it * 2) & (GROUPS - 1);
      const u32x4 a = *reinterpret_cast<const u32x4*>(L.g[g].tag);
      const u32x4 b = *reinterpret_cast<const u32x4*>(L.g[(g + 1) & (GROUPS - 1)].tag);
      acc ^= a.x ^ b.y;
      (void)next(x);
      (void)next(x);
    } else {
      const uint32_t s = next(x) & (SLOTS - 1);
      atomicAdd(&L.cnt[s], 1ull);
      atomicMin(&L.first[s], (unsigned long long)it);
    }
  }
  __syncthreads();
  if (acc == 0x12345678u) out[threadIdx.x] = acc + (uint32_t)L.cnt[threadIdx.x];
}

int main() {
  uint32_t* out;
  CK(hipMalloc(&out, 4096));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const char* names[7] = {"random tag reads (2 x ds_read_b128 / record)", "consecutive tag reads (conflict-free)",
                          "random 8-byte atomics (add + min)", "reduce pattern (2 tag reads, k1/k0, 2 atomics)",
                          "split layout: random tag reads, 16-B stride", "split layout: consecutive tag reads",
                          "split layout: reduce pattern"};
  for (int m = 0; m < 7; ++m) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventRecord(a));
    switch (m) {
      case 0: hipLaunchKernelGGL(k_probe<0>, dim3(cus), dim3(1024), 0, 0, out, 1u); break;
      case 1: hipLaunchKernelGGL(k_probe<1>, dim3(cus), dim3(1024), 0, 0, out, 1u); break;
      case 2: hipLaunchKernelGGL(k_probe<2>, dim3(cus), dim3(1024), 0, 0, out, 1u); break;
      case 3: hipLaunchKernelGGL(k_probe<3>, dim3(cus), dim3(1024), 0, 0, out, 1u); break;
      case 4: hipLaunchKernelGGL(k_probe_split<4>, dim3(cus), dim3(1024), 0, 0, out, 1u); break;
      case 5: hipLaunchKernelGGL(k_probe_split<5>, dim3(cus), dim3(1024), 0, 0, out, 1u); break;
      default: hipLaunchKernelGGL(k_probe_split<6>, dim3(cus), dim3(1024), 0, 0, out, 1u); break;
    }
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    printf("mode %d (%s): %.1f us\n", m, names[m], ms * 1e3);
  }
  CK(hipFree(out));
  return 0;
}
