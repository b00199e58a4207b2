// Butterfly throughput microbenchmark (register-only, no memory in the loop):
// the NTT's forward radix-2 butterfly (Harvey lazy + special-prime Montgomery
// from modarith.hpp / ntt.hip) on 16 words per thread, 8 independent
// butterflies per stage, 4 stages per round.  Reports butterflies/s for the
// whole GPU, to compare with the NTT kernels' butterfly rate.
//   hipcc --offload-arch=gfx950 -O3 -I../../include bfly.hip -o bfly && ./bfly
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../herdsman_amd/csrc/modarith.hpp"

__device__ __forceinline__ u64 harvey_csub(u64 x, u64 neg_m) {
  const u64 d = x + neg_m;
  const u32 m = (u32)((int32_t)(u32)(d >> 32) >> 31);
  const u64 mm = ((u64)m << 32) | m;
  return (x & mm) | (d & ~mm);
}

template <int ROUNDS>
__global__ void __launch_bounds__(256) bfly(u64 *out, u64 q, u32 q_hi, u64 w0) {
  u64 x[16], W[8];
  const u32 t = blockIdx.x * 256 + threadIdx.x;
  for (int i = 0; i < 16; ++i) x[i] = (t * 0x9E3779B97F4A7C15ull + i * 0x632BE59BD9B4E019ull) % q;
  for (int i = 0; i < 8; ++i) W[i] = (w0 + i * 0x1234567ull + t) % q;
  const u64 q2 = 2 * q;
  u64 nq2 = 0 - q2, q2p1 = q2 + 1;
  asm("" : "+s"(nq2));
  asm("" : "+s"(q2p1));
  for (int rd = 0; rd < ROUNDS; ++rd) {
#pragma unroll
    for (int st = 0; st < 4; ++st) {
      const int half = 8 >> st;
      u64 A[8], U[8], V[8], Wt[8];
      int n = 0;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        if (r & half) continue;
        U[n] = harvey_csub(x[r], nq2);
        A[n] = x[r + half];
        Wt[n] = W[(n + st) & 7];
        ++n;
      }
      mont_mul_sp_vec<8>(V, A, Wt, q_hi);
      n = 0;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        if (r & half) continue;
        x[r] = U[n] + V[n];
        x[r + half] = (U[n] + q2p1) + ~V[n];
        ++n;
      }
    }
  }
  u64 acc = 0;
  for (int i = 0; i < 16; ++i) acc ^= x[i];
  out[t] = acc;
}

int main() {
  const u64 q = 1152921504606584833ull;  // 2^60 - 2^32*k + 1 style special prime is not needed for timing
  const u32 q_hi = (u32)(q >> 32);
  const int blocks = 256 * 16, threads = 256;
  u64 *out;
  hipMalloc(&out, sizeof(u64) * blocks * threads);
  constexpr int ROUNDS = 64;
  hipLaunchKernelGGL(bfly<ROUNDS>, dim3(blocks), dim3(threads), 0, 0, out, q, q_hi, 12345);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  const int reps = 10;
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(bfly<ROUNDS>, dim3(blocks), dim3(threads), 0, 0, out, q, q_hi, 12345 + i);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double bf = (double)blocks * threads * ROUNDS * 4 * 8 * reps;
  printf("butterflies/s: %.3e  (%.2f ms per launch)\n", bf / (ms * 1e-3), ms / reps);
  printf("equivalent N=2^16 limb-NTT/s (524288 butterflies each): %.3e\n", bf / (ms * 1e-3) / 524288.0);
  return 0;
}
