// Base-conversion dot product throughput (register-only): y = sum_{i<4} v_i h_i mod q
// (a) 128-bit accumulation + one Montgomery reduction (dot_mont, modarith.hpp)
// (b) one special-prime Montgomery product per term, lazy sum, final csub chain
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../herdsman_amd/csrc/modarith.hpp"

template <int MODE, int ROUNDS>
__global__ void __launch_bounds__(256) kdot(u64 *out, u64 q, u32 q_hi, u64 seed) {
  const u32 t = blockIdx.x * 256 + threadIdx.x;
  u64 v[4], h[4];
  for (int i = 0; i < 4; ++i) {
    v[i] = (t * 0x9E3779B97F4A7C15ull + i * 0x632BE59BD9B4E019ull + seed) % q;
    h[i] = (seed * 7 + i * 0x1234567ull) % q;
  }
  ModInfo m{q, 0, 0, q_hi, 1};
  u64 acc = 0;
  for (int rd = 0; rd < ROUNDS; ++rd) {
    u64 y[4];
#pragma unroll
    for (int tt = 0; tt < 4; ++tt) {  // 4 independent targets per round (ILP)
      u64 hh[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) hh[i] = h[i] + tt;
      if (MODE == 0) {
        y[tt] = dot_mont<4, true>(v, hh, 1, 4, m);
      } else {
        u64 s = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) s += mont_mul_sp(v[i], hh[i], q_hi);
        s = csub(s, 4 * q);
        s = csub(s, 2 * q);
        y[tt] = csub(s, q);
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = y[i];
    acc ^= y[0];
  }
  out[t] = acc;
}

template <int MODE>
void run(u64 *out, u64 q, u32 qh) {
  constexpr int ROUNDS = 256;
  const int blocks = 256 * 16;
  hipLaunchKernelGGL((kdot<MODE, ROUNDS>), dim3(blocks), dim3(256), 0, 0, out, q, qh, 1);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  for (int i = 0; i < 5; ++i) hipLaunchKernelGGL((kdot<MODE, ROUNDS>), dim3(blocks), dim3(256), 0, 0, out, q, qh, i + 2);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double dots = (double)blocks * 256 * ROUNDS * 4 * 5;
  printf("mode %d: %.3e 4-term dots/s\n", MODE, dots / (ms * 1e-3));
}

int main() {
  const u64 q = 1152921504606584833ull;
  u64 *out;
  (void)hipMalloc(&out, sizeof(u64) * 256 * 16 * 256);
  run<0>(out, q, (u32)(q >> 32));
  run<1>(out, q, (u32)(q >> 32));
  return 0;
}
