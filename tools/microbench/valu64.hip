// Per-instruction VALU throughput on gfx950 for the ops in the NTT butterfly.
// Each kernel runs ITER x 8 independent instances of one instruction (inline
// asm so the compiler cannot fold it); rate = lane-ops/s, compared with the
// full-rate 78.6 T lane-ops/s (256 CU x 4 SIMD x 32 lanes x 2.4 GHz).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define ITER 2048
typedef uint64_t u64;

#define KERNEL(name, BODY)                                                        \
  __global__ void name(u64 *out, u64 seed) {                                     \
    u64 x0 = seed + threadIdx.x, x1 = x0 * 3, x2 = x0 * 5, x3 = x0 * 7;            \
    u64 x4 = x0 * 11, x5 = x0 * 13, x6 = x0 * 17, x7 = x0 * 19;                    \
    u64 k = seed | 1;                                                            \
    uint32_t a = (uint32_t)seed;                                                 \
    for (int i = 0; i < ITER; ++i) { BODY(x0) BODY(x1) BODY(x2) BODY(x3) BODY(x4) BODY(x5) BODY(x6) BODY(x7) } \
    out[blockIdx.x * blockDim.x + threadIdx.x] = x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7;  \
  }

#define KERNEL32(name, BODY)                                                      \
  __global__ void name(u64 *out, u64 seed) {                                     \
    uint32_t x0 = seed + threadIdx.x, x1 = x0 * 3, x2 = x0 * 5, x3 = x0 * 7;       \
    uint32_t x4 = x0 * 11, x5 = x0 * 13, x6 = x0 * 17, x7 = x0 * 19;               \
    u64 k = seed | 1;                                                            \
    uint32_t a = (uint32_t)seed;                                                 \
    for (int i = 0; i < ITER; ++i) { BODY(x0) BODY(x1) BODY(x2) BODY(x3) BODY(x4) BODY(x5) BODY(x6) BODY(x7) } \
    out[blockIdx.x * blockDim.x + threadIdx.x] = x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7 ^ k;  \
  }

#define KERNELF(name, BODY)                                                       \
  __global__ void name(u64 *out, u64 seed) {                                     \
    double x0 = 1.0 + threadIdx.x * 1e-3 + seed * 1e-9, x1 = x0 * 1.1, x2 = x0 * 1.2, x3 = x0 * 1.3; \
    double x4 = x0 * 1.4, x5 = x0 * 1.5, x6 = x0 * 1.6, x7 = x0 * 1.7;           \
    double k = 0.9999999;                                                        \
    for (int i = 0; i < ITER; ++i) { BODY(x0) BODY(x1) BODY(x2) BODY(x3) BODY(x4) BODY(x5) BODY(x6) BODY(x7) } \
    out[blockIdx.x * blockDim.x + threadIdx.x] = (u64)(x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7); \
  }

#define B_LSHLADD(x) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(x) : "v"(k));
#define B_MAD(x) asm volatile("v_mad_u64_u32 %0, s[40:41], %1, %1, %0" : "+v"(x) : "v"(a) : "s40", "s41");
#define B_ADDC(x) asm volatile("v_add_co_u32 %0, vcc, %0, %1\n v_addc_co_u32 %0, vcc, %0, %1, vcc" : "+v"(x) : "v"(a) : "vcc");
#define B_ADD32(x) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(a));
#define B_CMP64(x) asm volatile("v_cmp_le_u64 vcc, %0, %1" : : "v"(x), "v"(k) : "vcc"); x += 1;
#define B_MULHI(x) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(x) : "v"(a));
#define B_MULLO(x) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x) : "v"(a));
#define B_NOT(x) asm volatile("v_not_b32 %0, %0" : "+v"(x));
#define B_BFI(x) asm volatile("v_bfi_b32 %0, %0, %1, %0" : "+v"(x) : "v"(a));
#define B_MOV64(x) asm volatile("v_mov_b32 %0, %1" : "=v"(x) : "v"(x));
#define B_PKMOV(x) asm volatile("v_pk_mov_b32 %0, %0, %1 op_sel:[1,1]" : "+v"(x) : "v"(k));
#define B_SUBCO(x) asm volatile("v_sub_co_u32 %0, s[40:41], %0, %1\n v_subb_co_u32 %0, s[40:41], %0, %1, s[40:41]" : "+v"(x) : "v"(a) : "s40", "s41");

#define B_FMAF64(x) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(x) : "v"(k));
#define B_MULF64(x) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(x) : "v"(k));
#define B_ADDF64(x) asm volatile("v_add_f64 %0, %0, %1" : "+v"(x) : "v"(k));
#define B_RNDF64(x) asm volatile("v_rndne_f64 %0, %0" : "+v"(x));
KERNELF(k_fmaf64, B_FMAF64)
KERNELF(k_mulf64, B_MULF64)
KERNELF(k_addf64, B_ADDF64)
KERNELF(k_rndf64, B_RNDF64)
KERNEL(k_lshladd, B_LSHLADD)
KERNEL(k_mad, B_MAD)
KERNEL32(k_addc, B_ADDC)
KERNEL32(k_add32, B_ADD32)
KERNEL(k_cmp64, B_CMP64)
KERNEL32(k_mulhi, B_MULHI)
KERNEL32(k_mullo, B_MULLO)
KERNEL32(k_subco, B_SUBCO)
KERNEL32(k_not, B_NOT)
KERNEL32(k_bfi, B_BFI)
KERNEL32(k_mov, B_MOV64)
KERNEL(k_pkmov, B_PKMOV)

int main() {
  const int threads = 256, blocks = 256 * 8;
  u64 *out; (void)hipMalloc(&out, sizeof(u64) * threads * blocks);
  hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  double lanes = (double)threads * blocks;
  auto run = [&](const char *name, void (*k)(u64 *, u64), double instr_per_body) {
    hipLaunchKernelGGL(k, blocks, threads, 0, 0, out, 12345); (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k, blocks, threads, 0, 0, out, 12345);
    (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1); ms /= 5;
    double rate = lanes * ITER * 8 * instr_per_body / (ms * 1e-3);
    printf("%-26s %8.3f ms %9.2f G instr-lanes/s  = %.3f of full rate (78.6T)\n", name, ms, rate / 1e9, rate / 78.6e12);
  };
  run("v_lshl_add_u64", k_lshladd, 1);
  run("v_mad_u64_u32", k_mad, 1);
  run("v_add_co+v_addc (per instr)", k_addc, 2);
  run("v_add_u32", k_add32, 1);
  run("v_cmp_le_u64 (+1 add64)", k_cmp64, 1);
  run("v_mul_hi_u32", k_mulhi, 1);
  run("v_mul_lo_u32", k_mullo, 1);
  run("v_sub_co+v_subb sgpr (/instr)", k_subco, 2);
  run("v_not_b32", k_not, 1);
  run("v_bfi_b32", k_bfi, 1);
  run("v_mov_b32", k_mov, 1);
  run("v_pk_mov_b32 (2 dwords)", k_pkmov, 1);
  run("v_fma_f64", k_fmaf64, 1);
  run("v_mul_f64", k_mulf64, 1);
  run("v_add_f64", k_addf64, 1);
  run("v_rndne_f64", k_rndf64, 1);
  return 0;
}
