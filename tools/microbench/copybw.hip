// HBM streaming microbenchmark for the NTT passes' access patterns.
// Every kernel moves 32 KiB tiles: a 256-thread workgroup loads 16 u64 per
// thread (all loads in flight, as the NTT passes do), then stores them back to
// the same positions (in place, like the passes) or to a second buffer.
// Patterns (one tile = 4096 words; a "limb" is a 256 x 256 word matrix):
//   col8   : 16 adjacent columns x 256 rows, 8 B per lane (the column pass:
//            each wave instruction = 4 rows x 128 B)
//   row8   : 16 contiguous rows of 256 words, lane-contiguous 16-word runs
//            per row (the row pass's group-0 layout: 4 rows x 128 B)
//   flat8  : the tile as one contiguous run, 512 B per wave instruction
//   flat16 : the same with 16-B accesses (8 per thread)
//   col16  : 16 columns x 256 rows, 16-B accesses (8 rows x 128 B per wave)
// Reports algorithmic GB/s = (bytes read + bytes written) / time.
//   hipcc --offload-arch=gfx950 -O3 copybw.hip -o copybw && ./copybw
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

typedef uint64_t u64;
typedef uint32_t u32;
struct u64x2 {
  u64 a, b;
};

template <int PAT, bool NT>
__global__ void __launch_bounds__(256) copy_tile(const u64 *in, u64 *out) {
  const u32 tid = threadIdx.x;
  const size_t tile = blockIdx.x;
  if constexpr (PAT == 0 || PAT == 1 || PAT == 2) {
    u32 off[16];
    const size_t limb = tile / 16, blk = tile % 16;
    const size_t base = limb * 65536;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      if (PAT == 0) {  // col8: column blk*16 + tid%16, rows tid/16 + 16 r
        off[r] = (u32)((tid / 16 + 16 * r) * 256 + blk * 16 + tid % 16);
      } else if (PAT == 1) {  // row8: row blk*16 + tid/16, words tid%16 + 16 r
        off[r] = (u32)((blk * 16 + tid / 16) * 256 + tid % 16 + 16 * r);
      } else {  // flat8
        off[r] = (u32)(blk * 4096 + tid + 256 * r);
      }
    }
    u64 x[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) x[r] = NT ? __builtin_nontemporal_load(in + base + off[r]) : in[base + off[r]];
#pragma unroll
    for (int r = 0; r < 16; ++r) out[base + off[r]] = x[r] + 1;
  } else {
    const u64x2 *in2 = (const u64x2 *)in;
    u64x2 *out2 = (u64x2 *)out;
    u32 off[8];
    const size_t limb = tile / 16, blk = tile % 16;
    const size_t base = limb * 32768;  // in u64x2
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      if (PAT == 3) {  // flat16
        off[r] = (u32)(blk * 2048 + tid + 256 * r);
      } else {  // col16: columns blk*16 + 2 (tid%8) .. +1, rows tid/8 + 32 r
        off[r] = (u32)((tid / 8 + 32 * r) * 128 + blk * 8 + tid % 8);
      }
    }
    u64x2 x[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) x[r] = in2[base + off[r]];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      x[r].a += 1;
      out2[base + off[r]] = x[r];
    }
  }
}

template <int PAT, bool NT>
double run(const char *name, u64 *a, u64 *b, size_t words, bool inplace) {
  const u32 tiles = (u32)(words / 4096);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((copy_tile<PAT, NT>), dim3(tiles), dim3(256), 0, 0, a, inplace ? a : b);
  const int reps = 10;
  hipEventRecord(e0, 0);
  for (int i = 0; i < reps; ++i)
    hipLaunchKernelGGL((copy_tile<PAT, NT>), dim3(tiles), dim3(256), 0, 0, a, inplace ? a : b);
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  ms /= reps;
  const double gbs = 2.0 * words * 8 / (ms * 1e-3) / 1e9;
  printf("%-8s %-3s %-10s %8.3f ms  %7.0f GB/s\n", name, NT ? "nt" : "", inplace ? "in-place" : "out", ms, gbs);
  return gbs;
}

int main() {
  const size_t words = (size_t)4608 * 65536;  // 2.25 GiB, the roofline loop's 4608 limbs
  u64 *a, *b;
  if (hipMalloc(&a, words * 8) != hipSuccess || hipMalloc(&b, words * 8) != hipSuccess) {
    printf("alloc failed\n");
    return 1;
  }
  hipMemset(a, 0, words * 8);
  hipMemset(b, 0, words * 8);
  for (int ip = 1; ip >= 0; --ip) {
    run<0, false>("col8", a, b, words, ip);
    run<0, true>("col8", a, b, words, ip);
    run<1, false>("row8", a, b, words, ip);
    run<1, true>("row8", a, b, words, ip);
    run<2, false>("flat8", a, b, words, ip);
    run<3, false>("flat16", a, b, words, ip);
    run<4, false>("col16", a, b, words, ip);
  }
  hipFree(a);
  hipFree(b);
  return 0;
}
