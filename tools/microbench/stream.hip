// HBM streaming ceiling on MI355X for the NTT passes' tile shapes.
// copybw.hip moved one 32 KiB tile per workgroup (load 16 words per thread, then
// store them) and reached 5.0-5.4 TB/s; this one varies what that left fixed:
//   - read-only and write-only sweeps (the two halves of a copy),
//   - persistent grids (k workgroups per CU) looping over tiles, with the next
//     tile's loads issued before the current tile's stores (software pipelined),
//   - non-temporal loads / stores, in place against out of place,
//   - 8-byte (the NTT's u64 words) and 16-byte accesses.
// Tiles are the NTT pass shapes: col8 (16 adjacent columns x 256 rows of a
// 256 x 256 limb, four 128 B row segments per wave instruction), row8 (16 rows,
// lane-contiguous 16-word runs), flat8 / flat16 (one contiguous 32 KiB run).
// Prints GB/s = (bytes read + bytes written) / time over 4608 limbs (2.25 GiB).
//   hipcc --offload-arch=gfx950 -O3 stream.hip -o stream && ./stream
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

typedef uint64_t u64;
typedef uint32_t u32;

enum { COL8 = 0, ROW8 = 1, FLAT8 = 2, FLAT16 = 3, LINE16 = 4, COL32 = 5, COL64 = 6, COL128 = 7 };
// COLc (round 6): the column pass's pattern with wider row
// segments: a tile is c adjacent columns x 4096/c rows of a 256 x 256 limb, a
// wave instruction reads 64/c rows x c words (c = 32: two 256 B segments,
// 64: one 512 B segment, 128: half of a 1 KiB segment pair) at the 2 KiB row
// stride.  COL8 is c = 16 (four 128 B segments).
template <int PAT>
constexpr u32 col_width() { return PAT == COL32 ? 32 : PAT == COL64 ? 64 : PAT == COL128 ? 128 : 16; }
enum { COPY = 0, READ = 1, WRITE = 2, READL2 = 3 };  // READL2: the reads cycle over 64 tiles (2 MiB, L2-resident)

template <int PAT>
__device__ __forceinline__ u32 off_of(u32 tid, u32 blk, int r) {
  if (PAT == COL8) return (tid / 16 + 16 * r) * 256 + blk * 16 + tid % 16;
  if (PAT == COL32 || PAT == COL64 || PAT == COL128) {
    constexpr u32 C = col_width<PAT>(), G = 256 / C;  // column groups per limb
    const u32 row0 = (blk / G) * (4096 / C);
    return (row0 + tid / C + (256 / C) * r) * 256 + (blk % G) * C + tid % C;
  }
  if (PAT == ROW8) return (blk * 16 + tid / 16) * 256 + tid % 16 + 16 * r;
  if (PAT == FLAT8) return blk * 4096 + tid + 256 * r;
  if (PAT == FLAT16) return blk * 4096 + 2 * (tid + 256 * r);  // word index of a 16-B pair (r < 8)
  return blk * 4096 + 16 * tid + 2 * r;  // LINE16: each lane owns one 128-B line, 8 pairs (a row pass's last-group layout)
}

struct w2 {
  u64 a, b;
};

// one tile = 4096 words; NR words (or pairs) per thread
template <int PAT>
struct Tile {
  static constexpr bool PAIR = PAT == FLAT16 || PAT == LINE16;
  static constexpr int NR = PAIR ? 8 : 16;
  typedef typename std::conditional<PAIR, w2, u64>::type T;
};

template <int PAT, bool NTL>
__device__ __forceinline__ void tload(typename Tile<PAT>::T (&x)[Tile<PAT>::NR], const u64 *in, u32 tile, u32 tid) {
  const u64 *base = in + (size_t)(tile / 16) * 65536;
  const u32 blk = tile % 16;
#pragma unroll
  for (int r = 0; r < Tile<PAT>::NR; ++r) {
    const u32 o = off_of<PAT>(tid, blk, r);
    if constexpr (Tile<PAT>::PAIR) {
      const w2 *p = (const w2 *)(base + o);
      if (NTL) {
        x[r].a = __builtin_nontemporal_load(&p->a);
        x[r].b = __builtin_nontemporal_load(&p->b);
      } else {
        x[r] = *p;
      }
    } else {
      x[r] = NTL ? __builtin_nontemporal_load(base + o) : base[o];
    }
  }
}

template <int PAT, bool NTS>
__device__ __forceinline__ void tstore(const typename Tile<PAT>::T (&x)[Tile<PAT>::NR], u64 *out, u32 tile, u32 tid) {
  u64 *base = out + (size_t)(tile / 16) * 65536;
  const u32 blk = tile % 16;
#pragma unroll
  for (int r = 0; r < Tile<PAT>::NR; ++r) {
    const u32 o = off_of<PAT>(tid, blk, r);
    if constexpr (Tile<PAT>::PAIR) {
      w2 *p = (w2 *)(base + o);
      if (NTS) {
        __builtin_nontemporal_store(x[r].a, &p->a);
        __builtin_nontemporal_store(x[r].b, &p->b);
      } else {
        *p = x[r];
      }
    } else {
      if (NTS) __builtin_nontemporal_store(x[r], base + o);
      else base[o] = x[r];
    }
  }
}

template <int PAT>
__device__ __forceinline__ void bump(typename Tile<PAT>::T &v) {
  if constexpr (Tile<PAT>::PAIR) v.a += 1;
  else v += 1;
}

// MODE COPY: every tile loaded and stored (+1); PIPE: the next tile's loads are
// issued before this tile's stores.  READ: XOR of every word, one word out per
// thread.  WRITE: a constant stored.  Grid-stride over the tiles.
template <int PAT, int MODE, bool PIPE, bool NTL, bool NTS>
__global__ void __launch_bounds__(256) stream_k(const u64 *in, u64 *out, u32 tiles, u64 *sink) {
  using T = typename Tile<PAT>::T;
  constexpr int NR = Tile<PAT>::NR;
  const u32 tid = threadIdx.x;
  u32 t = blockIdx.x;
  if (t >= tiles) return;
  if constexpr (MODE == READ || MODE == READL2) {
    u64 acc = 0;
    for (; t < tiles; t += gridDim.x) {
      T x[NR];
      tload<PAT, NTL>(x, in, MODE == READL2 ? (t & 63) : t, tid);
#pragma unroll
      for (int r = 0; r < NR; ++r) {
        if constexpr (Tile<PAT>::PAIR) acc ^= x[r].a ^ x[r].b;
        else acc ^= x[r];
      }
    }
    sink[blockIdx.x * 256 + tid] = acc;
  } else if constexpr (MODE == WRITE) {
    T x[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      if constexpr (Tile<PAT>::PAIR) x[r] = w2{tid + (u64)r, (u64)r};
      else x[r] = tid + (u64)r;
    }
    for (; t < tiles; t += gridDim.x) tstore<PAT, NTS>(x, out, t, tid);
  } else if constexpr (!PIPE) {
    for (; t < tiles; t += gridDim.x) {
      T x[NR];
      tload<PAT, NTL>(x, in, t, tid);
#pragma unroll
      for (int r = 0; r < NR; ++r) bump<PAT>(x[r]);
      tstore<PAT, NTS>(x, out, t, tid);
    }
  } else {
    T x[NR];
    tload<PAT, NTL>(x, in, t, tid);
    for (;;) {
      const u32 tn = t + gridDim.x;
      T y[NR];
      if (tn < tiles) tload<PAT, NTL>(y, in, tn, tid);
#pragma unroll
      for (int r = 0; r < NR; ++r) bump<PAT>(x[r]);
      tstore<PAT, NTS>(x, out, t, tid);
      if (tn >= tiles) break;
#pragma unroll
      for (int r = 0; r < NR; ++r) x[r] = y[r];
      t = tn;
    }
  }
}

static const char *pname[] = {"col8", "row8", "flat8", "flat16", "line16", "col32", "col64", "col128"};
static const char *mname[] = {"copy", "read", "write", "readL2"};

template <int PAT, int MODE, bool PIPE, bool NTL, bool NTS>
void run(u64 *a, u64 *b, u64 *sink, size_t words, bool inplace, u32 wg_per_cu) {
  const u32 tiles = (u32)(words / 4096);
  const u32 grid = wg_per_cu ? 256 * wg_per_cu : tiles;
  u64 *dst = inplace ? a : b;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int i = 0; i < 3; ++i)
    hipLaunchKernelGGL((stream_k<PAT, MODE, PIPE, NTL, NTS>), dim3(grid), dim3(256), 0, 0, a, dst, tiles, sink);
  const int reps = 10;
  hipEventRecord(e0, 0);
  for (int i = 0; i < reps; ++i)
    hipLaunchKernelGGL((stream_k<PAT, MODE, PIPE, NTL, NTS>), dim3(grid), dim3(256), 0, 0, a, dst, tiles, sink);
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  ms /= reps;
  const double bytes = (MODE == COPY ? 2.0 : 1.0) * words * 8;
  char grid_s[32];
  if (wg_per_cu) snprintf(grid_s, sizeof grid_s, "%u/CU", wg_per_cu);
  else snprintf(grid_s, sizeof grid_s, "1 tile/WG");
  printf("%-6s %-5s %-4s ntl=%d nts=%d %-8s %-9s %8.3f ms %7.0f GB/s\n", pname[PAT], mname[MODE], PIPE ? "pipe" : "",
         NTL, NTS, MODE == COPY ? (inplace ? "in-place" : "out") : "", grid_s, ms, bytes / (ms * 1e-3) / 1e9);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
}

template <int PAT>
void sweep(u64 *a, u64 *b, u64 *sink, size_t words) {
  run<PAT, READ, false, false, false>(a, b, sink, words, false, 0);
  run<PAT, READ, false, true, false>(a, b, sink, words, false, 0);
  run<PAT, READ, false, false, false>(a, b, sink, words, false, 4);
  run<PAT, READ, false, false, false>(a, b, sink, words, false, 8);
  run<PAT, WRITE, false, false, false>(a, b, sink, words, false, 0);
  run<PAT, WRITE, false, false, true>(a, b, sink, words, false, 0);
  run<PAT, WRITE, false, false, false>(a, b, sink, words, false, 8);
  for (int ip = 1; ip >= 0; --ip) {
    run<PAT, COPY, false, false, false>(a, b, sink, words, ip, 0);
    run<PAT, COPY, false, true, false>(a, b, sink, words, ip, 0);
    run<PAT, COPY, false, true, true>(a, b, sink, words, ip, 0);
    run<PAT, COPY, false, false, true>(a, b, sink, words, ip, 0);
    run<PAT, COPY, false, false, false>(a, b, sink, words, ip, 4);
    run<PAT, COPY, false, false, false>(a, b, sink, words, ip, 8);
    run<PAT, COPY, true, false, false>(a, b, sink, words, ip, 2);
    run<PAT, COPY, true, false, false>(a, b, sink, words, ip, 4);
    run<PAT, COPY, true, true, false>(a, b, sink, words, ip, 4);
    run<PAT, COPY, true, true, true>(a, b, sink, words, ip, 4);
  }
}

// L2-served reads (every workgroup re-reads 64 tiles = 2 MiB): 8-byte against
// 16-byte accesses per lane, the question for the fused passes' operand loads
void l2_sweep(u64 *a, u64 *b, u64 *sink, size_t words) {
  run<FLAT8, READL2, false, false, false>(a, b, sink, words, false, 0);
  run<FLAT16, READL2, false, false, false>(a, b, sink, words, false, 0);
  run<ROW8, READL2, false, false, false>(a, b, sink, words, false, 0);
  run<FLAT8, READL2, false, false, false>(a, b, sink, words, false, 4);
  run<FLAT16, READL2, false, false, false>(a, b, sink, words, false, 4);
}

// a row pass storing straight from its last butterfly group (each lane one
// 128-B line, 8 x 16-B accesses) against the re-laid-out pair layout
void line_sweep(u64 *a, u64 *b, u64 *sink, size_t words) {
  run<LINE16, READ, false, true, false>(a, b, sink, words, false, 0);
  run<FLAT16, READ, false, true, false>(a, b, sink, words, false, 0);
  run<LINE16, WRITE, false, false, true>(a, b, sink, words, false, 0);
  run<FLAT16, WRITE, false, false, true>(a, b, sink, words, false, 0);
  run<LINE16, WRITE, false, false, false>(a, b, sink, words, false, 0);
  run<LINE16, COPY, false, true, true>(a, b, sink, words, true, 0);
  run<FLAT16, COPY, false, true, true>(a, b, sink, words, true, 0);
  run<LINE16, COPY, false, false, false>(a, b, sink, words, true, 0);
  run<LINE16, READL2, false, false, false>(a, b, sink, words, false, 0);
  run<FLAT16, READL2, false, false, false>(a, b, sink, words, false, 0);
}

// column segment width: 128 B (col8) .. 1 KiB (col128)
template <int PAT>
void col_width_sweep(u64 *a, u64 *b, u64 *sink, size_t words) {
  run<PAT, READ, false, true, false>(a, b, sink, words, false, 0);
  run<PAT, WRITE, false, false, true>(a, b, sink, words, false, 0);
  run<PAT, COPY, false, true, true>(a, b, sink, words, true, 0);
  run<PAT, COPY, false, true, true>(a, b, sink, words, false, 0);
  run<PAT, COPY, true, true, true>(a, b, sink, words, true, 2);
  run<PAT, COPY, true, true, true>(a, b, sink, words, true, 4);
}

int main(int argc, char **argv) {
  const size_t words = (size_t)4608 * 65536;  // 2.25 GiB: the roofline loop's 4608 limbs
  u64 *a, *b, *sink;
  if (hipMalloc(&a, words * 8) != hipSuccess || hipMalloc(&b, words * 8) != hipSuccess ||
      hipMalloc(&sink, (size_t)(words / 4096) * 256 * 8) != hipSuccess) {
    printf("alloc failed\n");
    return 1;
  }
  hipMemset(a, 1, words * 8);
  hipMemset(b, 2, words * 8);
  if (argc > 1 && argv[1][0] == 'r') {  // ./stream row: lane-line against lane-contiguous pairs
    line_sweep(a, b, sink, words);
    return 0;
  }
  if (argc > 1 && argv[1][0] == 'c') {  // ./stream col: column segment width
    col_width_sweep<COL8>(a, b, sink, words);
    col_width_sweep<COL32>(a, b, sink, words);
    col_width_sweep<COL64>(a, b, sink, words);
    col_width_sweep<COL128>(a, b, sink, words);
    col_width_sweep<ROW8>(a, b, sink, words);
    return 0;
  }
  if (argc > 1 && argv[1][0] == 'l') {  // ./stream l2
    l2_sweep(a, b, sink, words);
    return 0;
  }
  sweep<FLAT16>(a, b, sink, words);
  sweep<FLAT8>(a, b, sink, words);
  sweep<ROW8>(a, b, sink, words);
  sweep<COL8>(a, b, sink, words);
  hipFree(a);
  hipFree(b);
  hipFree(sink);
  return 0;
}
