// Microbenchmark: VALU integer / fp64 multiply throughput on gfx950.
// Answers SURVEY.md §7 "integer-multiply ceiling": what v_mul_lo_u32, v_mul_hi_u32,
// v_mad_u64_u32, v_fma_f64 and a full 64-bit Shoup modmul cost per lane.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define ITERS 4096
#define CHAINS 8

__global__ void k_mullo(uint32_t* out, uint32_t seed) {
  uint32_t a[CHAINS];
  for (int c = 0; c < CHAINS; ++c) a[c] = seed + threadIdx.x * 7 + c;
  uint32_t b = seed | 1;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) a[c] = a[c] * b + 0;  // v_mul_lo_u32
  }
  uint32_t s = 0;
  for (int c = 0; c < CHAINS; ++c) s ^= a[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_mulhi(uint32_t* out, uint32_t seed) {
  uint32_t a[CHAINS];
  for (int c = 0; c < CHAINS; ++c) a[c] = seed + threadIdx.x * 7 + c;
  uint32_t b = seed | 0x80000001u;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) a[c] = __umulhi(a[c], b) ^ c;
  }
  uint32_t s = 0;
  for (int c = 0; c < CHAINS; ++c) s ^= a[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_mad64(uint32_t* out, uint32_t seed) {
  uint64_t a[CHAINS];
  for (int c = 0; c < CHAINS; ++c) a[c] = seed + threadIdx.x * 7 + c;
  uint32_t b = seed | 0x80000001u;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) a[c] = (uint64_t)(uint32_t)a[c] * b + (a[c] >> 32);  // v_mad_u64_u32
  }
  uint64_t s = 0;
  for (int c = 0; c < CHAINS; ++c) s ^= a[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(s ^ (s >> 32));
}
__global__ void k_fma64(uint32_t* out, uint32_t seed) {
  double a[CHAINS];
  for (int c = 0; c < CHAINS; ++c) a[c] = (double)(seed + threadIdx.x * 7 + c);
  double b = 1.0000001, d = 1e-9;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) a[c] = fma(a[c], b, d);
  }
  double s = 0;
  for (int c = 0; c < CHAINS; ++c) s += a[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s;
}
__global__ void k_fma32(uint32_t* out, uint32_t seed) {
  float a[CHAINS];
  for (int c = 0; c < CHAINS; ++c) a[c] = (float)(seed + threadIdx.x * 7 + c);
  float b = 1.0000001f, d = 1e-9f;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) a[c] = fmaf(a[c], b, d);
  }
  float s = 0;
  for (int c = 0; c < CHAINS; ++c) s += a[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s;
}
// full Shoup: r = a*w - hi(a*w')*q  (lazy, r in [0,2q))
__global__ void k_shoup(uint32_t* out, uint64_t q, uint64_t w, uint64_t wp) {
  uint64_t a[CHAINS];
  for (int c = 0; c < CHAINS; ++c) a[c] = (threadIdx.x * 7919ull + c) % q;
  for (int i = 0; i < ITERS / 8; ++i) {
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) {
      uint64_t qh = __umul64hi(a[c], wp);
      uint64_t r = a[c] * w - qh * q;
      a[c] = r;
    }
  }
  uint64_t s = 0;
  for (int c = 0; c < CHAINS; ++c) s ^= a[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(s ^ (s >> 32));
}
// double-based Shoup-like modmul for q < 2^50
__global__ void k_dshoup(uint32_t* out, double q, double w, double qinv) {
  double a[CHAINS];
  for (int c = 0; c < CHAINS; ++c) a[c] = (double)((threadIdx.x * 7919ull + c) % 1000003ull);
  for (int i = 0; i < ITERS / 8; ++i) {
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) {
      double h = a[c] * w;
      double l = fma(a[c], w, -h);
      double qt = rint(h * qinv);
      double r = fma(-qt, q, h) + l;
      r = (r < 0) ? r + q : r;
      a[c] = r;
    }
  }
  double s = 0;
  for (int c = 0; c < CHAINS; ++c) s += a[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s;
}
__global__ void k_copy(const uint4* __restrict__ in, uint4* __restrict__ out, size_t n) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  size_t stride = (size_t)gridDim.x * blockDim.x;
  for (; i < n; i += stride) out[i] = in[i];
}

int main() {
  const int threads = 256, blocks = 256 * 8;
  uint32_t* out; hipMalloc(&out, sizeof(uint32_t) * threads * blocks);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  double lanes = (double)threads * blocks;
  auto run = [&](const char* name, auto launch, double ops_per_lane) {
    launch(); hipDeviceSynchronize();
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) launch();
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1); ms /= 5;
    double rate = lanes * ops_per_lane / (ms * 1e-3);
    printf("%-10s %8.3f ms  %8.2f G lane-ops/s  (full-rate VALU = 78.6 T/s at 2.4GHz -> ratio %.3f)\n",
           name, ms, rate / 1e9, rate / 78.6e12);
  };
  run("mul_lo32", [&]{ k_mullo<<<blocks, threads>>>(out, 12345); }, (double)ITERS * CHAINS);
  run("mul_hi32", [&]{ k_mulhi<<<blocks, threads>>>(out, 12345); }, (double)ITERS * CHAINS);
  run("mad_u64", [&]{ k_mad64<<<blocks, threads>>>(out, 12345); }, (double)ITERS * CHAINS);
  run("fma_f64", [&]{ k_fma64<<<blocks, threads>>>(out, 12345); }, (double)ITERS * CHAINS);
  run("fma_f32", [&]{ k_fma32<<<blocks, threads>>>(out, 12345); }, (double)ITERS * CHAINS);
  uint64_t q = 1152921504606830593ull; // 2^60 - 2^14 + 1 (prime-ish; only for timing)
  uint64_t w = 123456789012345ull % q;
  unsigned __int128 wp128 = ((unsigned __int128)w << 64) / q;
  run("shoup64", [&]{ k_shoup<<<blocks, threads>>>(out, q, w, (uint64_t)wp128); }, (double)(ITERS / 8) * CHAINS);
  double dq = 1125899906826241.0;
  run("dshoup", [&]{ k_dshoup<<<blocks, threads>>>(out, dq, 12345678901.0, 1.0 / dq); }, (double)(ITERS / 8) * CHAINS);
  size_t bytes = (size_t)1 << 30;
  uint4 *a, *b; hipMalloc(&a, bytes); hipMalloc(&b, bytes); hipMemset(a, 1, bytes);
  size_t n = bytes / 16;
  k_copy<<<256 * 16, 256>>>(a, b, n); hipDeviceSynchronize();
  hipEventRecord(e0);
  for (int r = 0; r < 10; ++r) k_copy<<<256 * 16, 256>>>(a, b, n);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1); ms /= 10;
  printf("copy 1GiB: %.3f ms  %.2f TB/s (r+w)\n", ms, 2.0 * bytes / (ms * 1e-3) / 1e12);
  return 0;
}
