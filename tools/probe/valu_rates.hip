// VALU issue-rate probe: wave-instruction throughput of the integer ops the
// map's per-token code is made of (v_mul_lo_u32 vs the 24-bit multiplies, 64-bit
// shifts and compares, v_bitop3, DPP adds), at the map's occupancy (one
// 1024-thread block per CU = 4 waves per SIMD).  Each op runs as 8 independent
// chains (no dependency stalls); cycles per wave-instruction per SIMD =
// elapsed cycles x 4 SIMDs / (waves per CU x instructions per wave).
// hipcc --offload-arch=gfx950 -O3 tools/probe/valu_rates.hip -o tools/probe/valu_rates
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e = (x);                                                          \
    if (e != hipSuccess) {                                                       \
      printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__);                \
      return 1;                                                                  \
    }                                                                            \
  } while (0)

constexpr int ITERS = 512;
constexpr int CH = 8;

#define BODY(ASM)                                                                \
  uint32_t x[CH];                                                                \
  for (int c = 0; c < CH; ++c) x[c] = seed + c * 0x9E3779B9u + threadIdx.x;      \
  const uint32_t k = seed ^ 0x85EBCA77u;                                         \
  for (int i = 0; i < ITERS; ++i) {                                              \
    _Pragma("unroll") for (int c = 0; c < CH; ++c) asm volatile(ASM : "+v"(x[c]) : "v"(k)); \
  }                                                                              \
  uint32_t s = 0;                                                                \
  for (int c = 0; c < CH; ++c) s ^= x[c];                                        \
  if (s == 0x12345678u) out[threadIdx.x] = s;

__global__ void __launch_bounds__(1024) k_add(uint32_t* out, uint32_t seed) { BODY("v_add_u32 %0, %0, %1") }
__global__ void __launch_bounds__(1024) k_mullo(uint32_t* out, uint32_t seed) { BODY("v_mul_lo_u32 %0, %0, %1") }
__global__ void __launch_bounds__(1024) k_mul24(uint32_t* out, uint32_t seed) { BODY("v_mul_u32_u24 %0, %0, %1") }
__global__ void __launch_bounds__(1024) k_mulhi24(uint32_t* out, uint32_t seed) { BODY("v_mul_hi_u32_u24 %0, %0, %1") }
__global__ void __launch_bounds__(1024) k_mad24(uint32_t* out, uint32_t seed) { BODY("v_mad_u32_u24 %0, %0, %1, %0") }
__global__ void __launch_bounds__(1024) k_mulhi(uint32_t* out, uint32_t seed) { BODY("v_mul_hi_u32 %0, %0, %1") }
__global__ void __launch_bounds__(1024) k_bitop3(uint32_t* out, uint32_t seed) { BODY("v_bitop3_b32 %0, %0, %1, %0 bitop3:0x6c") }
__global__ void __launch_bounds__(1024) k_xad(uint32_t* out, uint32_t seed) { BODY("v_xad_u32 %0, %0, %1, %0") }
__global__ void __launch_bounds__(1024) k_alignbit(uint32_t* out, uint32_t seed) { BODY("v_alignbit_b32 %0, %0, %1, 7") }
__global__ void __launch_bounds__(1024) k_bfe(uint32_t* out, uint32_t seed) { BODY("v_bfe_u32 %0, %0, %1, 5") }
__global__ void __launch_bounds__(1024) k_ffbl(uint32_t* out, uint32_t seed) { BODY("v_ffbl_b32 %0, %0") }
__global__ void __launch_bounds__(1024) k_bcnt(uint32_t* out, uint32_t seed) { BODY("v_bcnt_u32_b32 %0, %0, %1") }
__global__ void __launch_bounds__(1024) k_lshlor(uint32_t* out, uint32_t seed) { BODY("v_lshl_or_b32 %0, %0, 3, %1") }
__global__ void __launch_bounds__(1024) k_dppadd(uint32_t* out, uint32_t seed) {
  BODY("v_add_u32_dpp %0, %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf")
}

// 64-bit ops: chains on register pairs
#define BODY64(ASM)                                                              \
  uint64_t x[CH];                                                                \
  for (int c = 0; c < CH; ++c) x[c] = ((uint64_t)seed << 32 | (seed + c)) + threadIdx.x; \
  const uint32_t k = (seed & 31) | 1;                                            \
  for (int i = 0; i < ITERS; ++i) {                                              \
    _Pragma("unroll") for (int c = 0; c < CH; ++c) asm volatile(ASM : "+v"(x[c]) : "v"(k)); \
  }                                                                              \
  uint64_t s = 0;                                                                \
  for (int c = 0; c < CH; ++c) s ^= x[c];                                        \
  if (s == 0x12345678u) out[threadIdx.x] = (uint32_t)s;

__global__ void __launch_bounds__(1024) k_lshr64(uint32_t* out, uint32_t seed) { BODY64("v_lshrrev_b64 %0, %1, %0") }
__global__ void __launch_bounds__(1024) k_add64(uint32_t* out, uint32_t seed) { BODY64("v_lshl_add_u64 %0, %0, 0, %0") }

// v_cmp_eq_u64 into VCC (writes an SGPR pair; one compare per lane)
__global__ void __launch_bounds__(1024) k_cmp64(uint32_t* out, uint32_t seed) {
  uint64_t a[CH];
  for (int c = 0; c < CH; ++c) a[c] = ((uint64_t)seed << 32 | (seed + c)) + threadIdx.x;
  const uint64_t b = seed;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) asm volatile("v_cmp_eq_u64 vcc, %0, %1" ::"v"(a[c]), "v"(b) : "vcc");
  }
  if (a[0] == 0x12345678u) out[threadIdx.x] = 1;
}


__global__ void __launch_bounds__(1024) k_and(uint32_t* out, uint32_t seed) { BODY("v_and_b32 %0, %0, %1") }
__global__ void __launch_bounds__(1024) k_xor(uint32_t* out, uint32_t seed) { BODY("v_xor_b32 %0, %0, %1") }
__global__ void __launch_bounds__(1024) k_lshr(uint32_t* out, uint32_t seed) { BODY("v_lshrrev_b32 %0, %1, %0") }
__global__ void __launch_bounds__(1024) k_lshl(uint32_t* out, uint32_t seed) { BODY("v_lshlrev_b32 %0, %1, %0") }
__global__ void __launch_bounds__(1024) k_lshrimm(uint32_t* out, uint32_t seed) { BODY("v_lshrrev_b32 %0, 3, %0\n v_xor_b32 %0, %0, %1") }
__global__ void __launch_bounds__(1024) k_max(uint32_t* out, uint32_t seed) { BODY("v_max_u32 %0, %0, %1") }
__global__ void __launch_bounds__(1024) k_sub(uint32_t* out, uint32_t seed) { BODY("v_sub_u32 %0, %0, %1") }
__global__ void __launch_bounds__(1024) k_add3(uint32_t* out, uint32_t seed) { BODY("v_add3_u32 %0, %0, %1, %0") }
__global__ void __launch_bounds__(1024) k_or3(uint32_t* out, uint32_t seed) { BODY("v_or3_b32 %0, %0, %1, %0") }
__global__ void __launch_bounds__(1024) k_andor(uint32_t* out, uint32_t seed) { BODY("v_and_or_b32 %0, %0, %1, %0") }
__global__ void __launch_bounds__(1024) k_lshladd(uint32_t* out, uint32_t seed) { BODY("v_lshl_add_u32 %0, %0, 3, %1") }
__global__ void __launch_bounds__(1024) k_perm(uint32_t* out, uint32_t seed) { BODY("v_perm_b32 %0, %0, %1, %0") }
__global__ void __launch_bounds__(1024) k_alignbyte(uint32_t* out, uint32_t seed) { BODY("v_alignbyte_b32 %0, %0, %1, %0") }
__global__ void __launch_bounds__(1024) k_mul24e32(uint32_t* out, uint32_t seed) { BODY("v_mul_u32_u24_e32 %0, %1, %0") }
__global__ void __launch_bounds__(1024) k_xorsdwa(uint32_t* out, uint32_t seed) { BODY("v_xor_b32_sdwa %0, %0, %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD") }
__global__ void __launch_bounds__(1024) k_cmp32(uint32_t* out, uint32_t seed) { BODY("v_cmp_eq_u32 vcc, %0, %1\n v_cndmask_b32 %0, %0, %1, vcc") }
__global__ void __launch_bounds__(1024) k_cnd(uint32_t* out, uint32_t seed) { BODY("v_cndmask_b32 %0, %0, %1, vcc") }
__global__ void __launch_bounds__(1024) k_min3(uint32_t* out, uint32_t seed) { BODY("v_min3_u32 %0, %0, %1, %0") }
__global__ void __launch_bounds__(1024) k_bfi(uint32_t* out, uint32_t seed) { BODY("v_bfi_b32 %0, %0, %1, %0") }
__global__ void __launch_bounds__(1024) k_mov(uint32_t* out, uint32_t seed) { BODY("v_mov_b32 %0, %1") }
__global__ void __launch_bounds__(1024) k_pkadd(uint32_t* out, uint32_t seed) { BODY("v_pk_add_u16 %0, %0, %1") }

typedef void (*Kern)(uint32_t*, uint32_t);

int main() {
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  int clk_khz = 0;
  CK(hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0));
  uint32_t* out;
  CK(hipMalloc(&out, 4096 * 4));
  struct {
    const char* n;
    Kern k;
  } ks[] = {{"v_add_u32", k_add},           {"v_mul_lo_u32", k_mullo},      {"v_mul_u32_u24", k_mul24},
            {"v_mul_hi_u32_u24", k_mulhi24}, {"v_mad_u32_u24", k_mad24},     {"v_mul_hi_u32", k_mulhi},
            {"v_bitop3_b32", k_bitop3},      {"v_xad_u32", k_xad},           {"v_alignbit_b32", k_alignbit},
            {"v_bfe_u32", k_bfe},            {"v_ffbl_b32", k_ffbl},         {"v_bcnt_u32_b32", k_bcnt},
            {"v_lshl_or_b32", k_lshlor},     {"v_add_u32_dpp", k_dppadd},    {"v_lshrrev_b64", k_lshr64},
            {"v_lshl_add_u64", k_add64},     {"v_cmp_eq_u64 (vcc)", k_cmp64},
            {"v_and_b32", k_and}, {"v_xor_b32", k_xor}, {"v_lshrrev_b32 (vgpr)", k_lshr}, {"v_lshlrev_b32 (vgpr)", k_lshl},
            {"lshr imm + xor (2 insts)", k_lshrimm}, {"v_max_u32", k_max}, {"v_sub_u32", k_sub}, {"v_add3_u32", k_add3},
            {"v_or3_b32", k_or3}, {"v_and_or_b32", k_andor}, {"v_lshl_add_u32", k_lshladd}, {"v_perm_b32", k_perm},
            {"v_alignbyte_b32", k_alignbyte}, {"v_mul_u32_u24_e32", k_mul24e32}, {"v_xor_b32_sdwa", k_xorsdwa},
            {"v_cmp_eq_u32+cndmask (2)", k_cmp32}, {"v_cndmask_b32 vcc", k_cnd}, {"v_min3_u32", k_min3},
            {"v_bfi_b32", k_bfi}, {"v_mov_b32", k_mov}, {"v_pk_add_u16", k_pkadd}};
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int blocks = cus * 4;  // 4 passes of one block per CU
  printf("CUs %d, reported clock %d MHz; cycles per wave-instruction per SIMD at 4 waves/SIMD (at 2.4 GHz)\n", cus,
         clk_khz / 1000);
  for (auto& e : ks) {
    hipLaunchKernelGGL(e.k, dim3(blocks), dim3(1024), 0, 0, out, 1u);  // warm
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 3; ++r) {
      CK(hipEventRecord(a));
      hipLaunchKernelGGL(e.k, dim3(blocks), dim3(1024), 0, 0, out, (uint32_t)r + 2);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      if (ms < best) best = ms;
    }
    // per SIMD: blocks/cus blocks x 4 waves each (16 waves per block / 4 SIMDs) x ITERS x CH instructions
    const double insts = (double)blocks / cus * 4.0 * ITERS * CH;
    const double cyc = best * 1e-3 * 2.4e9;
    printf("%-22s %7.3f ms  %5.2f cyc/inst/SIMD\n", e.n, best, cyc / insts);
  }
  return 0;
}
