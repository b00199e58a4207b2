// Fast base conversion on the matrix cores: a feasibility measurement for
// the conversions fused into the NTT column passes (ntt.hip PRO_CONV).
//
// The conversion y_m = sum_i v_i h[i][m] mod p_m (4 sources, 12 targets: one
// ModUp digit of the metric parameters) is done two ways over NC coefficients:
//   valu : dot_mont (modarith.hpp) -- 4 special-prime Montgomery products per
//          target, as the backend does it today;
//   mfma : v_mfma_i32_32x32x32_i8.  Each source is written in 8 balanced
//          signed base-256 digits, d_a = byte_a(v + 0x80..80) - 128, which is
//          one 64-bit add and one xor: (v + 0x80..80) ^ 0x80..80 holds the
//          digits as int8.  The constants C[i][a][m] = h[i][m] R 256^a mod p_m
//          are written the same way, digit b.  Then
//             S[m][b] = sum_{i,a} d_{i,a} digit_b(C[i][a][m])   (|S| < 2^19)
//          is a 32 x 32 x 32 int8 matrix product per 32 coefficients and 4
//          targets (K = 4 sources x 8 digits, rows = 4 targets x 8 digits b),
//          and y_m = mont_reduce(sum_b S[m][b] 256^b + k_m p_m), k_m p_m an
//          offset that makes the sum non-negative.
//          Row map: a lane's 16 accumulators are rows (q&3) + 8(q>>2) + 4h
//          (h = lane >> 5), so rows are assigned so that lane half h owns all
//          8 digits of targets 2h and 2h+1: no cross-lane exchange.
// Both kernels repeat the 12-target conversion REPS times with REPS constant
// sets and store the XOR of the canonical results, so REPS > 1 measures the
// arithmetic rather than HBM.  Every result is checked against a host
// __int128 computation.
//   hipcc --offload-arch=gfx950 -O3 bconv_mfma.hip -o bconv_mfma && ./bconv_mfma
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>

#include "../../herdsman_amd/csrc/modarith.hpp"

typedef int64_t i64;
typedef unsigned __int128 u128;
typedef __attribute__((ext_vector_type(4))) int v4i;
typedef __attribute__((ext_vector_type(16))) int v16i;

constexpr int NS = 4, NT = 12, NSET = 8;
constexpr u64 K80 = 0x8080808080808080ull;

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

struct Tgt {
  ModInfo m;
  u64 offset;  // A of conv_mfma's offset A + B 2^32 = k p
};

// ---------------------------------------------------------------- valu
template <int REPS>
__global__ void __launch_bounds__(256) conv_valu(const u64 *__restrict__ v, u64 *__restrict__ y,
                                                 const u64 *__restrict__ hR, const Tgt *__restrict__ tg, u32 nc) {
  const u32 k = blockIdx.x * 256 + threadIdx.x;
  if (k >= nc) return;
  u64 x[NS];
#pragma unroll
  for (int i = 0; i < NS; ++i) x[i] = v[(size_t)i * nc + k];
  u64 out[NT] = {};
  for (int r = 0; r < REPS; ++r) {
    const u64 *h = hR + (size_t)(r % NSET) * NS * NT;  // [set][i][m]
#pragma unroll
    for (int m = 0; m < NT; ++m) out[m] ^= dot_mont<NS, true>(x, h + m, NT, NS, tg[m].m);
  }
#pragma unroll
  for (int m = 0; m < NT; ++m) y[(size_t)m * nc + k] = out[m];
}

// ---------------------------------------------------------------- mfma
// afrag: [set][t (3)][lane (64)] v4i -- the A operand of MFMA t
template <int REPS>
__global__ void __launch_bounds__(256) conv_mfma(const u64 *__restrict__ v, u64 *__restrict__ y,
                                                 const v4i *__restrict__ afrag, const Tgt *__restrict__ tg, u32 nc) {
  const u32 lane = threadIdx.x & 63, h = lane >> 5, c = lane & 31;
  const u32 tile = blockIdx.x * 4 + (threadIdx.x >> 6);
  const u32 k = tile * 32 + c;
  if (tile * 32 >= nc) return;
  // B operand: digits of sources 2h, 2h+1 of coefficient k (k = 16h + j)
  const u64 w0 = (v[(size_t)(2 * h) * nc + k] + K80) ^ K80;
  const u64 w1 = (v[(size_t)(2 * h + 1) * nc + k] + K80) ^ K80;
  const v4i b = {(int)(u32)w0, (int)(u32)(w0 >> 32), (int)(u32)w1, (int)(u32)(w1 >> 32)};
  // this lane's 6 targets (4t + 2h + u) in registers: the index depends on h
  u64 tq[6], tbl[6];
  u32 tqh[6];
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    const Tgt &T = tg[4 * (j >> 1) + 2 * h + (j & 1)];
    tq[j] = T.m.q, tqh[j] = T.m.q_hi, tbl[j] = T.offset;
  }
  u64 out[6] = {};
  for (int r = 0; r < REPS; ++r) {
    const v4i *af = afrag + (size_t)(r % NSET) * 3 * 64;
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      const v16i zero = {};
      const v16i s = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[t * 64 + lane], b, zero, 0, 0, 0);
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        // target 4t + 2h + u: digit b in accumulator 8u + b
        // digit pairs in 32 bits (|S| < 2^19, so S_b + 256 S_b+1 < 2^28), then 64
        const int x01 = s[8 * u] + s[8 * u + 1] * 256, x23 = s[8 * u + 2] + s[8 * u + 3] * 256;
        const int x45 = s[8 * u + 4] + s[8 * u + 5] * 256, x67 = s[8 * u + 6] + s[8 * u + 7] * 256;
        // T = lo + hi 2^32 (|lo|, |hi| < 2^45) made non-negative by offsets
        // A + B 2^32 = k p (B = 2^45, A in [2^45, 2^45 + p)): the residue is
        // unchanged and the 128-bit assembly needs no carry compare
        const int j = 2 * t + u;
        const u64 lo = (u64)((i64)x01 + (i64)x23 * 65536) + tbl[j];  // + A
        const u64 hi = (u64)((i64)x45 + (i64)x67 * 65536) + (1ull << 45);
        const u64 t1 = (lo >> 32) + (u32)hi;  // < 2^33
        ModInfo mi{};
        mi.q_hi = tqh[j];
        const U128 T{(u64)(u32)lo | (t1 << 32), (hi >> 32) + (t1 >> 32)};
        out[j] ^= csub(mont_reduce<true>(T, mi), tq[j]);
      }
    }
  }
#pragma unroll
  for (int t = 0; t < 3; ++t)
#pragma unroll
    for (int u = 0; u < 2; ++u) y[(size_t)(4 * t + 2 * h + u) * nc + k] = out[2 * t + u];
}

// ---------------------------------------------------------------- host
static u64 mulmod(u64 a, u64 b, u64 q) { return (u64)((u128)a * b % q); }
static u64 powmod(u64 a, u64 e, u64 q) {
  u64 r = 1;
  for (a %= q; e; e >>= 1, a = mulmod(a, a, q))
    if (e & 1) r = mulmod(r, a, q);
  return r;
}
static bool is_prime(u64 n) {
  if (n < 2) return false;
  for (u64 p : {2ull, 3ull, 5ull, 7ull, 11ull, 13ull, 17ull, 19ull, 23ull, 29ull, 31ull, 37ull})
    if (n % p == 0) return n == p;
  u64 d = n - 1;
  int s = 0;
  while (!(d & 1)) d >>= 1, ++s;
  for (u64 a : {2ull, 3ull, 5ull, 7ull, 11ull, 13ull, 17ull, 19ull, 23ull, 29ull, 31ull, 37ull}) {
    u64 x = powmod(a, d, n);
    if (x == 1 || x == n - 1) continue;
    bool ok = false;
    for (int i = 1; i < s && !ok; ++i) ok = (x = mulmod(x, x, n)) == n - 1;
    if (!ok) return false;
  }
  return true;
}
static u64 rng_state = 0x1234567887654321ull;
static u64 rnd() {
  rng_state += 0x9E3779B97F4A7C15ull;
  return splitmix64(rng_state);
}

int main() {
  // 16 special primes q = k 2^32 + 1 just below 2^60 (4 sources, 12 targets)
  std::vector<u64> pr;
  for (u64 kk = (1ull << 28) - 1; pr.size() < NS + NT; --kk)
    if (is_prime((kk << 32) | 1)) pr.push_back((kk << 32) | 1);
  const u64 *src = pr.data(), *dst = pr.data() + NS;
  std::vector<Tgt> tg(NT);
  for (int m = 0; m < NT; ++m) {
    const u64 p = dst[m];
    u64 inv = 1;  // p^-1 mod 2^64
    for (int i = 0; i < 6; ++i) inv *= 2 - p * inv;
    tg[m].m = ModInfo{p, 0 - inv, 0, (u32)(p >> 32), 1};
    const u128 B32 = (u128)1 << 77;  // B 2^32, B = 2^45
    const u128 kp = ((B32 + ((u128)1 << 45)) / p + 1) * p;
    tg[m].offset = (u64)(kp - B32);  // A
  }
  // constants h[set][i][m] < p_m
  std::vector<u64> h((size_t)NSET * NS * NT), hR(h.size());
  for (int s = 0; s < NSET; ++s)
    for (int i = 0; i < NS; ++i)
      for (int m = 0; m < NT; ++m) {
        const size_t o = ((size_t)s * NS + i) * NT + m;
        h[o] = rnd() % dst[m];
        hR[o] = (u64)(((u128)h[o] << 64) % dst[m]);  // h R mod p: mont_mul(v, hR) = v h
      }
  // A fragments: lane l, row r = l & 31, k = 16 (l >> 5) + j
  std::vector<v4i> af((size_t)NSET * 3 * 64);
  for (int s = 0; s < NSET; ++s)
    for (int t = 0; t < 3; ++t)
      for (int l = 0; l < 64; ++l) {
        const int r = l & 31, hk = l >> 5;
        const int hr = (r >> 2) & 1, g = r >> 3, bd = (r & 3) + 4 * (g & 1), ml = 2 * hr + (g >> 1);
        const int m = 4 * t + ml;
        uint8_t bytes[16];
        for (int j = 0; j < 16; ++j) {
          const int i = 2 * hk + (j >> 3), a = j & 7;
          const u64 p = dst[m];
          const u64 cst = mulmod(hR[((size_t)s * NS + i) * NT + m], powmod(256, a, p), p);  // h R 256^a
          bytes[j] = (uint8_t)(((cst + K80) ^ K80) >> (8 * bd));
        }
        v4i f;
        for (int w = 0; w < 4; ++w) f[w] = (int)(bytes[4 * w] | bytes[4 * w + 1] << 8 | bytes[4 * w + 2] << 16 | (u32)bytes[4 * w + 3] << 24);
        af[((size_t)s * 3 + t) * 64 + l] = f;
      }
  const u32 nc = 1u << 22;
  std::vector<u64> v((size_t)NS * nc);
  for (int i = 0; i < NS; ++i)
    for (u32 k = 0; k < nc; ++k) v[(size_t)i * nc + k] = rnd() % src[i];

  u64 *dv, *dy, *dh;
  v4i *daf;
  Tgt *dtg;
  CHECK(hipMalloc(&dv, v.size() * 8));
  CHECK(hipMalloc(&dy, (size_t)NT * nc * 8));
  CHECK(hipMalloc(&dh, hR.size() * 8));
  CHECK(hipMalloc(&daf, af.size() * sizeof(v4i)));
  CHECK(hipMalloc(&dtg, tg.size() * sizeof(Tgt)));
  CHECK(hipMemcpy(dv, v.data(), v.size() * 8, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(dh, hR.data(), hR.size() * 8, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(daf, af.data(), af.size() * sizeof(v4i), hipMemcpyHostToDevice));
  CHECK(hipMemcpy(dtg, tg.data(), tg.size() * sizeof(Tgt), hipMemcpyHostToDevice));

  // host reference of the XOR over `reps` sets, checked on every 997th coefficient
  auto check = [&](int reps, const char *what) {
    std::vector<u64> out((size_t)NT * nc);
    CHECK(hipMemcpy(out.data(), dy, out.size() * 8, hipMemcpyDeviceToHost));
    size_t bad = 0, tested = 0;
    for (u32 k = 0; k < nc; k += 997)
      for (int m = 0; m < NT; ++m) {
        u64 e = 0;
        for (int r = 0; r < reps; ++r) {
          u128 acc = 0;
          for (int i = 0; i < NS; ++i) acc += (u128)v[(size_t)i * nc + k] * h[((size_t)(r % NSET) * NS + i) * NT + m];
          e ^= (u64)(acc % dst[m]);
        }
        ++tested;
        if (out[(size_t)m * nc + k] != e && bad++ < 4)
          printf("  %s mismatch k=%u m=%d got %llx want %llx\n", what, k, m, (unsigned long long)out[(size_t)m * nc + k],
                 (unsigned long long)e);
      }
    printf("%s reps=%d check: %zu / %zu mismatches\n", what, reps, bad, tested);
    return bad == 0;
  };
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  auto timeit = [&](auto launch) {
    launch();
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0));
    for (int it = 0; it < 10; ++it) launch();
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    return ms / 10;
  };
  bool ok = true;
  const dim3 gv(nc / 256), gm(nc / 128);  // mfma: 4 waves x 32 coefficients per block
  hipLaunchKernelGGL(conv_valu<1>, gv, dim3(256), 0, 0, dv, dy, dh, dtg, nc);
  ok &= check(1, "valu");
  hipLaunchKernelGGL(conv_mfma<1>, gm, dim3(256), 0, 0, dv, dy, daf, dtg, nc);
  ok &= check(1, "mfma");
  if (!ok) return 1;
  hipLaunchKernelGGL(conv_valu<16>, gv, dim3(256), 0, 0, dv, dy, dh, dtg, nc);
  ok &= check(16, "valu");
  hipLaunchKernelGGL(conv_mfma<16>, gm, dim3(256), 0, 0, dv, dy, daf, dtg, nc);
  ok &= check(16, "mfma");
  if (!ok) return 1;
  const double conv1 = (double)nc * NT;  // target residues per rep
  const float tv1 = timeit([&] { hipLaunchKernelGGL(conv_valu<1>, gv, dim3(256), 0, 0, dv, dy, dh, dtg, nc); });
  const float tm1 = timeit([&] { hipLaunchKernelGGL(conv_mfma<1>, gm, dim3(256), 0, 0, dv, dy, daf, dtg, nc); });
  const float tv = timeit([&] { hipLaunchKernelGGL(conv_valu<16>, gv, dim3(256), 0, 0, dv, dy, dh, dtg, nc); });
  const float tm = timeit([&] { hipLaunchKernelGGL(conv_mfma<16>, gm, dim3(256), 0, 0, dv, dy, daf, dtg, nc); });
  const double bytes = (double)nc * (NS + NT) * 8;
  printf("NC=%u coefficients, %d sources -> %d targets\n", nc, NS, NT);
  printf("reps=1  (HBM: %.0f MB)  valu %.3f ms (%.2f TB/s)  mfma %.3f ms (%.2f TB/s)\n", bytes / 1e6, tv1,
         bytes / tv1 / 1e9, tm1, bytes / tm1 / 1e9);
  printf("reps=16 (arithmetic)    valu %.3f ms = %.1f G target-residues/s   mfma %.3f ms = %.1f G/s   ratio %.2fx\n", tv,
         conv1 * 16 / tv / 1e6, tm, conv1 * 16 / tm / 1e6, tv / tm);
  return 0;
}
