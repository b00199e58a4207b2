// Exchange microbenchmark: the NTT's inter-group data exchange (ntt.hip
// group_loop) -- a 16 x 16 transpose of u64 words among the 16 threads of one
// sub-transform, each thread holding 16 words in VGPRs -- done two ways:
//   lds : 16 ds_write_b64 + barrier + 16 ds_read_b64 (the padded slot map of
//         ntt.hip lds_idx), as the NTT does it;
//   bperm: cross-lane ds_bpermute_b32 inside the 16-lane group: a lane-dependent
//         register rotation (4 conditional-rotate stages, selects), 16 rounds of
//         2 ds_bpermute_b32 (lo / hi word), and the inverse rotation.
// Both kernels apply an even number of transposes, so the output must equal
// the input (checked).  Reports the launch time and the
// words exchanged per second over the whole GPU.
//   hipcc --offload-arch=gfx950 -O3 xchg.hip -o xchg && ./xchg
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>
#include <vector>

typedef uint64_t u64;
typedef uint32_t u32;

constexpr int PAD = 256 + 16 + 1;  // ntt.hip lds_idx<8>: one pad word per 16 and per sub-transform

template <int REPS>
__global__ void __launch_bounds__(256) x_lds(u64 *io) {
  __shared__ u64 lds[16 * PAD];
  const u32 tid = threadIdx.x, w = tid / 16, l = tid % 16;
  u64 *p = io + ((size_t)blockIdx.x * 256 + tid) * 16;
  u64 x[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) x[r] = p[r];
  for (int rep = 0; rep < REPS; ++rep) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const u32 k = l * 16 + r;
      lds[w * PAD + k + (k >> 4)] = x[r];
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const u32 k = r * 16 + l;
      x[r] = lds[w * PAD + k + (k >> 4)];
    }
    __syncthreads();
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) p[r] = x[r];
}

// z[k] <- z[(k + s*dir) & 15] where the lane's bit decides (lane-dependent rotation)
// (the lane bit is made opaque, so each stage stays 32 selects on one mask
// instead of being merged into a dynamically indexed select tree)
__device__ __forceinline__ void rot_stage(u64 (&z)[16], u32 bit, int s) {
  u32 m = 0u - bit;
  asm volatile("" : "+v"(m));
  const u64 mm = ((u64)m << 32) | m;
  u64 t[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) t[k] = (z[(k + s) & 15] & mm) | (z[k] & ~mm);
#pragma unroll
  for (int k = 0; k < 16; ++k) z[k] = t[k];
}

template <int REPS>
__global__ void __launch_bounds__(256) x_bperm(u64 *io) {
  const u32 tid = threadIdx.x, lane = tid & 63, l = lane & 15, gbase = lane & ~15u;
  u64 *p = io + ((size_t)blockIdx.x * 256 + tid) * 16;
  u64 x[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) x[r] = p[r];
  for (int rep = 0; rep < REPS; ++rep) {
    // z[k] = x[(l + k) & 15]
#pragma unroll
    for (int b = 0; b < 4; ++b) rot_stage(x, (l >> b) & 1, 1 << b);
    // round j: receive from lane (l - j) its z[j] = element (row l - j, col l)
    u64 w[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int addr = (int)((gbase + ((l - j) & 15)) << 2);
      const u32 lo = (u32)__builtin_amdgcn_ds_bpermute(addr, (int)(u32)x[j]);
      const u32 hi = (u32)__builtin_amdgcn_ds_bpermute(addr, (int)(u32)(x[j] >> 32));
      w[j] = ((u64)hi << 32) | lo;
    }
    // y[k] = w[(l - k) & 15]: u[k] = w[(-k) & 15] (static), then y[k] = u[(k - l) & 15]
#pragma unroll
    for (int k = 0; k < 16; ++k) x[k] = w[(16 - k) & 15];
#pragma unroll
    for (int b = 0; b < 4; ++b) rot_stage(x, (l >> b) & 1, 16 - (1 << b));
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) p[r] = x[r];
}

template <typename F>
static float time_it(F launch, int reps) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  launch();
  hipDeviceSynchronize();
  hipEventRecord(e0);
  for (int i = 0; i < reps; ++i) launch();
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return ms / reps;
}

int main() {
  constexpr int REPS = 64;  // exchanges per kernel (even: the output equals the input)
  const int blocks = 256 * 16;
  const size_t words = (size_t)blocks * 256 * 16;
  std::vector<u64> h(words), back(words);
  for (size_t i = 0; i < words; ++i) h[i] = i * 0x9E3779B97F4A7C15ull;
  u64 *d;
  hipMalloc(&d, words * 8);
  const char *names[2] = {"lds  ", "bperm"};
  for (int v = 0; v < 2; ++v) {
    hipMemcpy(d, h.data(), words * 8, hipMemcpyHostToDevice);
    auto launch = [&] {
      if (v == 0) hipLaunchKernelGGL(x_lds<REPS>, dim3(blocks), dim3(256), 0, 0, d);
      else hipLaunchKernelGGL(x_bperm<REPS>, dim3(blocks), dim3(256), 0, 0, d);
    };
    const float ms = time_it(launch, 5);
    hipMemcpy(back.data(), d, words * 8, hipMemcpyDeviceToHost);
    bool ok = back == h;
    // one transpose applied twice is the identity; check one transpose too
    if (ok) {
      hipMemcpy(d, h.data(), words * 8, hipMemcpyHostToDevice);
      if (v == 0) hipLaunchKernelGGL(x_lds<1>, dim3(blocks), dim3(256), 0, 0, d);
      else hipLaunchKernelGGL(x_bperm<1>, dim3(blocks), dim3(256), 0, 0, d);
      hipMemcpy(back.data(), d, words * 8, hipMemcpyDeviceToHost);
      for (size_t g = 0; g < (size_t)blocks * 16 && ok; ++g)  // 16 threads x 16 words per group
        for (int r = 0; r < 16 && ok; ++r)
          for (int c = 0; c < 16 && ok; ++c) ok = back[g * 256 + r * 16 + c] == h[g * 256 + c * 16 + r];
    }
    printf("%s: %.3f ms per launch (%d workgroups x %d exchanges), transpose %s\n", names[v], ms, blocks, REPS,
           ok ? "ok" : "WRONG");
    printf("%s: %.1f G word-exchanges/s\n", names[v], (double)words * REPS / (ms * 1e-3) / 1e9);
  }
  hipFree(d);
  return 0;
}
