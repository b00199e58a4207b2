// ntt_ksf.hip -- the fused key-switch finish of CKKS mul+relin and rotation (KSF)
// (kernel templates: ntt_core.hpp)
//
// With the tensor product split (PRO_TENSOR2 + EPI_KSQT) one ciphertext's key
// switch still moves the Q limbs of the non-own ModUp digits through HBM twice
// more than it must: the ModUp row pass reads their column-pass intermediates
// and writes ext, and EPI_KSQT reads ext back, once per output poly b.  Here
// ONE workgroup per (limb, ciphertext, row block) does all of it for both b:
//   1. the own digit and the base, from the ciphertexts a, b (as EPI_KSQT):
//        acc_b = d2 ksk_own,b + base_b P      (base_0 = a0 b0, base_1 = a0 b1 + a1 b0)
//   2. every non-own digit j: the row transform of its ModUp intermediate
//      (the forward row pass, in registers), then acc_b += ext_j ksk_j,b
//   3. for b = 0, 1: the row transform of NTT(conv_b)'s intermediate and the
//      ModDown finish out_b = (acc_b - conv_b) P^-1 = base_b + (acc_b' - conv_b) P^-1
// so ext's Q limbs are never stored (the P limbs: ksp_fused_pass below; with
// both, ntt_fwd_modup_launch runs ModUp's column passes only).  The two
// accumulators (32 words per thread) stay in registers across the four row
// transforms: 3 waves per SIMD.
// A rotation (ROT) runs the same finish with the own digit's word sigma_g(c1) R
// and the base sigma_g(c0) (poly 0) gathered from the ciphertext, so
// PRO_AUTOMORPH stores neither.
// Bit-exact with the unfused path: the same butterflies (run_group) on the
// same lazy ranges; the sums differ only in their representatives mod q_i.
// Round 6: the accumulators run at the scale R^-2 (ModUp's Q targets arrive
// times R^-1, ModDown's conv times R^-2, the finish multiplies by P^-1 R^3:
// fhe_ctx::modup_tabs_ksf / moddown_ksf / d_pinv3), so the own digit is four
// plain Montgomery products (no 128-bit product, no reduction with carry
// compares, no R^3 product), and on moduli below 2^60 the digit sums stay lazy
// (below 8q) until the finish: -17% VALU instructions (tools/isa_count.py).
#include "ntt_core.hpp"

#ifndef KSF_FUSE
#define KSF_FUSE 1  // CKKS mul+relin: the fused key-switch finish where it applies (ks_fused_finish_ok)
#endif
#ifndef KSF_LSW
#define KSF_LSW 4  // butterflies per lock-step chunk (run_group LSW): 8 needs more temporaries than the accumulators leave
#endif
#ifndef KSP_LSW
#define KSP_LSW 2  // the same for the P side (6-9 VGPRs spill, outside the loops: addresses for the INTT phase)
#endif
#ifndef KSF_MINW
// minimum waves per SIMD (the accumulators take 64 VGPRs).  2, not 3: the
// metric instantiation still allocates 168 VGPRs (3 waves) but without the
// 5 spills the 3-wave bound produced: ksf_pass 1.90 -> 1.83 ms per wave,
// ct-mult +0.8%, headline +0.4% (profiles/r06/ab_ksf_minw.txt)
#define KSF_MINW 2
#endif
#ifndef KSP_MINW
#define KSP_MINW 3  // the P side (2: 187 VGPRs, 2 waves, 0.61 -> 0.68 ms)
#endif
#ifndef KSP_MINW15
#define KSP_MINW15 KSP_MINW  // the same at N = 2^15 (BFV C3's all-limb pass)
#endif

namespace {

// a loop unrolled by construction: f(integral_constant<int, i>) for i < N (the
// unroll pragma gives up on these bodies for size, and a rolled loop over the
// accumulators would put them in scratch)
template <class F, int... I>
__device__ __forceinline__ void sfor_impl(F &&f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void sfor(F &&f) {
  sfor_impl(f, std::make_integer_sequence<int, N>{});
}

struct KspArgs {
  u64 *acc;             // [2n][QP][N]: the P rows receive INTT(acc_P)'s row pass
  const u64 *ext;       // [n][ndig][QP][N] ModUp's column-pass outputs (P limbs)
  const u64 *ksk;       // [ndig][2][kQP][N]
  const ModInfo *mods;
  const u64 *twf, *twi; // forward / inverse twiddles [nmod][N]
  u32 L, QP, kQP, kshift, ndig;
  u32 l0;               // the launch's first limb (L: the P limbs; 0: BFV's Q limbs)
};

struct KsfArgs {
  const u64 *conv;      // [2n][L][N] NTT(conv)'s column-pass output (ModDown)
  const u64 *ext;       // [n][ndig][QP][N] ModUp's column-pass outputs (Q limbs of the non-own digits)
  const u64 *ksk;       // [ndig][2][kQP][N]
  const u64 *ta, *tb;   // [n][2][L][N] the ciphertexts
  u64 *out;             // [n][2][L][N]
  const ModInfo *mods;  // the Q limbs first
  const u64 *tw;        // forward twiddles [nmod][N]
  const u64 *pinv;      // [L] P^-1 R^3 (the accumulator scale R^-2)
  const u64 *pplain;    // [L] P mod q_i
  const u64 *pm1;       // [L] P R^-1 mod q_i
  u32 L, QP, kQP, ndig, alpha;
  u32 g;                // ROT: the Galois element (ta = the ciphertexts, read through sigma_g)
};

// ROT: a CKKS rotation's finish instead: the own digit's word is sigma_g(c1) R
// and the base sigma_g(c0) (poly 0 only), both gathered from the ciphertext.
// SP: the special-modulus Montgomery product (q = 1 mod 2^32), else the generic one.
template <int LOG_N, int KD, bool WIDE, bool ROT, bool SP>
__global__ void __launch_bounds__(256, KSF_MINW) ksf_pass(KsfArgs a) {
  constexpr int S = 8, LOGR = 4, W = 16, R = 16, S0 = LOG_N - S;
  using G0 = Grp<S, LOGR, 0>;
  using G1 = Grp<S, LOGR, 1>;
  using IO = IoL<S, LOGR>;
  static_assert(IO::STEP == 2 && (S + LOGR - 1) / LOGR == 2, "two 16-word groups, pair IO");
  extern __shared__ u64 lds[];
  constexpr size_t N = (size_t)1 << LOG_N;

  // (row block, ciphertext, limb); as EPI_KSQ, every ciphertext of one (limb,
  // row block) on consecutive workgroup ids of ONE XCD, so the limb's key rows
  // stay in that XCD's L2 for the whole batch
  const u32 tid = threadIdx.x;
  u32 bx = blockIdx.x, ct = blockIdx.y, limb = blockIdx.z;
  if (((gridDim.x * gridDim.z) & 7) == 0) {
    const u32 np = gridDim.y, lin = blockIdx.x + gridDim.x * (blockIdx.y + np * blockIdx.z);
    const u32 r = lin >> 3, g = (r / np) * 8 + (lin & 7);
    ct = r % np;
    bx = g % gridDim.x;
    limb = g / gridDim.x;
  }
  const ModInfo mi = a.mods[limb];
  const u64 q = mi.q, q2 = 2 * q;
  const u64 *tw = a.tw + ((size_t)limb << LOG_N);
  const u32 ts = tid % (1u << (S - LOGR)), w = tid / (1u << (S - LOGR));
  const u32 row = bx * W + w, gb = row << S;
  const u32 vin = (gb + G0::k_thr(ts)) << 3;  // the row pass's load layout (group 0)
  const u32 vio = (gb + IO::k_thr(ts)) << 3;  // the re-laid-out store layout (pairs)
  const u32 jown = limb / a.alpha;
  const u64 *kb = a.ksk + (size_t)limb * N;  // key row of digit j, poly b: + j kj + b kbs
  const size_t kj = (size_t)2 * a.kQP * N, kbs = (size_t)a.kQP * N;
  const u64 *eb = a.ext + ((size_t)ct * a.ndig * a.QP + limb) * N;  // digit j: + j QP N
  const size_t LN = (size_t)a.L * N;
  const size_t co = ((size_t)2 * ct * a.L + limb) * N;  // (ct, poly 0, limb) of [n][2][L][N]
  const u64 *a0 = a.ta + co, *a1 = a0 + LN, *b0 = a.tb + co, *b1 = b0 + LN;

  u64 nq1 = 0 - q, nq2 = 0 - q2, nq4 = 0 - 2 * q2;
  asm("" : "+s"(nq1));
  asm("" : "+s"(nq2));
  asm("" : "+s"(nq4));

  // the forward row pass of one 16-row block in registers: x in the group-0
  // layout in, NTT outputs (lazy, as the row pass leaves them) in the IO layout
  // out.  Each sub-transform's 16 threads sit in one wave, so consecutive
  // transforms may reuse its LDS slots without a barrier in between.
  // (scheduling fences around it: left free, the compiler hoists the next
  // phase's key and operand loads above the transform and spills)
  const auto row_io = [&](u64 (&x)[R]) {
    __builtin_amdgcn_sched_barrier(0);
    u64 t[16];
    G0::template load_tw<S0>(t, tw, row, ts);
    run_group<S, LOGR, 0, S0, false, SP, WIDE, KSF_LSW>(x, t, q2, mi);
    G1::template load_tw<S0>(t, tw, row, ts);
    const u32 l0 = lds_idx<S>(w, G0::k_thr(ts));
#pragma unroll
    for (int r = 0; r < R; ++r) lds[l0 + G0::k_reg(r) + lds_pad(G0::k_reg(r))] = x[r];
    __syncthreads();
    const u32 l1 = lds_idx<S>(w, G1::k_thr(ts));
#pragma unroll
    for (int r = 0; r < R; ++r) x[r] = lds[l1 + G1::k_reg(r) + lds_pad(G1::k_reg(r))];
    run_group<S, LOGR, 1, S0, false, SP, WIDE, KSF_LSW>(x, t, q2, mi);
#pragma unroll
    for (int r = 0; r < R; ++r) lds[l1 + G1::k_reg(r) + lds_pad(G1::k_reg(r))] = x[r];
    __syncthreads();
    const u32 l2 = lds_idx<S>(w, IO::k_thr(ts));
#pragma unroll
    for (int r = 0; r < R; ++r) x[r] = lds[l2 + IO::k_reg(r) + lds_pad(IO::k_reg(r))];
    __builtin_amdgcn_sched_barrier(0);
  };

  // 1. the own digit and the base, every term at the accumulator scale R^-2
  //    (the finish's constant P^-1 R^3 cancels it): no 128-bit products
  u64 acc0[R], acc1[R];
  if constexpr (ROT) {
    const u64 *k0 = kb + jown * kj, *k1 = k0 + kbs;
    const u64 one = 1, pm = a.pm1[limb];  // P R^-1
    sfor<R / 2>([&](auto I) {
      constexpr int r = 2 * decltype(I)::value;
      const u32 kr = IO::k_reg(r);
      const u64x2 K0 = ld2_b(k0 + kr, vio), K1 = ld2_b(k1 + kr, vio);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const u32 src = aut_src<LOG_N>((vio >> 3) + kr + h, a.g);
        const u64 y0 = ld_b(a0, src), y1 = ld_b(a1, src);  // sigma_g(c0), sigma_g(c1)
        const u64 e = mont_mul<SP>(y1, one, mi);           // sigma_g(c1) R^-1
        acc0[r + h] = mont_mul<SP>(e, K0[h], mi) + mont_mul<SP>(y0, pm, mi);
        acc1[r + h] = mont_mul<SP>(e, K1[h], mi);
        if constexpr (!WIDE) acc0[r + h] = harvey_csub(acc0[r + h], nq2);
      }
    });
  } else {
    const u64 pp = a.pplain[limb];  // P mod q
    const u64 *k0 = kb + jown * kj, *k1 = k0 + kbs;
    sfor<R / 2>([&](auto I) {
      constexpr int r = 2 * decltype(I)::value;
      const u32 kr = IO::k_reg(r);
      const u64x2 A0 = ld2_b(a0 + kr, vio), A1 = ld2_b(a1 + kr, vio);
      const u64x2 B0 = ld2_b(b0 + kr, vio), B1 = ld2_b(b1 + kr, vio);
      const u64x2 K0 = ld2_b(k0 + kr, vio), K1 = ld2_b(k1 + kr, vio);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const u64 x0 = A0[h], x1 = A1[h], y0 = B0[h], y1 = B1[h];
        const u64 t = mont_mul<SP>(x1, y1, mi);                                  // d2 R^-1
        const u64 d0 = mont_mul<SP>(x0, y0, mi);                                 // base_0 R^-1
        const u64 d1 = mont_mul<SP>(x0, y1, mi) + mont_mul<SP>(x1, y0, mi);      // base_1 R^-1, < 4q
        acc0[r + h] = mont_mul<SP>(t, K0[h], mi) + mont_mul<SP>(d0, pp, mi);    // < 4q
        acc1[r + h] = mont_mul<SP>(t, K1[h], mi) + mont_mul<SP>(d1, pp, mi);
        if constexpr (!WIDE) {
          acc0[r + h] = harvey_csub(acc0[r + h], nq2);
          acc1[r + h] = harvey_csub(acc1[r + h], nq2);
        }
      }
    });
  }
  // 2. the non-own digits: their ModUp row transform here, then the products
  for (int j = 0; j < KD; ++j) {
    if (j == (int)jown) continue;  // uniform
    u64 x[R];
#pragma unroll
    for (int r = 0; r < R; ++r) x[r] = ld_d(eb + (size_t)j * a.QP * N + G0::k_reg(r), vin);
    row_io(x);  // ext_j R, lazy (< 8q WIDE, < 4q)
    const u64 *k0 = kb + j * kj, *k1 = k0 + kbs;
    sfor<R / 2>([&](auto I) {
      constexpr int r = 2 * decltype(I)::value;
      const u32 kr = IO::k_reg(r);
      const u64x2 K0 = ld2_b(k0 + kr, vio), K1 = ld2_b(k1 + kr, vio);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        // WIDE (q < 2^60): lazy sums, below 4q + 2 x 2q = 8q < 2^63 after two non-own digits
        acc0[r + h] = acc0[r + h] + mont_mul<SP>(x[r + h], K0[h], mi);
        acc1[r + h] = acc1[r + h] + mont_mul<SP>(x[r + h], K1[h], mi);
        if constexpr (!WIDE) {
          acc0[r + h] = harvey_csub(acc0[r + h], nq2);
          acc1[r + h] = harvey_csub(acc1[r + h], nq2);
        }
      }
    });
  }
  // 3. NTT(conv_b)'s row transform and the ModDown finish, b = 0, 1
  u64 cb1 = (WIDE ? 2 * q2 : q2) + 1;  // B q + 1: (acc + cb1) + ~v = acc + B q - v (< 8q WIDE)
  asm("" : "+s"(cb1));
  const u64 pinv = a.pinv[limb];
  const auto finish = [&](const u64(&acc)[R], int b) {
    u64 x[R];
    const u64 *cv = a.conv + co + b * LN;
#pragma unroll
    for (int r = 0; r < R; ++r) x[r] = ld_d(cv + G0::k_reg(r), vin);
    row_io(x);
    u64 *ob = a.out + co + b * LN;
    sfor<R / 2>([&](auto I) {
      constexpr int r = 2 * decltype(I)::value;
      u64 o[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const u64 v = harvey_csub(x[r + h], WIDE ? nq4 : nq2);  // below 4q (WIDE) / 2q
        const u64 s = WIDE ? harvey_csub(acc[r + h], nq4) : harvey_csub(acc[r + h], nq1);  // < 4q / < q
        o[h] = harvey_csub(mont_mul<SP>((s + cb1) + ~v, pinv, mi), nq1);
      }
      st2_e(ob + IO::k_reg(r), vio, u64x2{o[0], o[1]});
    });
  };
  finish(acc0, 0);
  finish(acc1, 1);
}


template <int LOG_N, int KD, bool WIDE, bool ROT>
int ksf_launch(fhe_ctx *c, const KsfArgs &a, u32 n) {
  constexpr size_t lds = lds_bytes<8, 16>();
  const dim3 grid((1u << (LOG_N - 8)) / 16, n, a.L);
  if (c->special) hipLaunchKernelGGL((ksf_pass<LOG_N, KD, WIDE, ROT, true>), grid, dim3(256), lds, c->stream, a);
  else hipLaunchKernelGGL((ksf_pass<LOG_N, KD, WIDE, ROT, false>), grid, dim3(256), lds, c->stream, a);
  return fhe_check(c, hipGetLastError(), "ksf_pass launch");
}

template <int LOG_N, int KD>
int ksf_dispatch(fhe_ctx *c, const KsfArgs &a, u32 n) {
  const bool wide = c->moduli[0] < (1ull << 60);
  if (a.g) return wide ? ksf_launch<LOG_N, KD, true, true>(c, a, n) : ksf_launch<LOG_N, KD, false, true>(c, a, n);
  return wide ? ksf_launch<LOG_N, KD, true, false>(c, a, n) : ksf_launch<LOG_N, KD, false, false>(c, a, n);
}

// The P side of the same key switch (KSP fused): one workgroup per (P limb,
// ct, row block) row-transforms every digit's ModUp intermediate of the limb
// (they are all non-own), forms acc_P,b = sum_j ext_j ksk_j,b R^-1 for b = 0, 1
// and runs the first (row) pass of INTT(acc_P,b) on it, so the ModUp row pass
// and PRO_KSP's ext reads go away; the INTT's column pass follows as before.
// BFV (round 6, all limbs): the same over every limb of Q u P -- on a Q limb
// the own digit's slot holds the column-pass intermediate of the limb's own
// d R -- so BFV's ext is never written by a row pass and never read back.
template <int LOG_N, int KD, bool WIDE, bool SP>
__global__ void __launch_bounds__(256, LOG_N == 15 ? KSP_MINW15 : KSP_MINW) ksp_fused_pass(KspArgs a) {
  constexpr int S = 8, LOGR = 4, W = 16, R = 16, S0 = LOG_N - S;
  using G0 = Grp<S, LOGR, 0>;
  using G1 = Grp<S, LOGR, 1>;
  using IO = IoL<S, LOGR>;
  extern __shared__ u64 lds[];
  constexpr size_t N = (size_t)1 << LOG_N;
  const u32 tid = threadIdx.x;
  u32 bx = blockIdx.x, ct = blockIdx.y, pl = blockIdx.z;  // pl: the launch's limb (0..gridDim.z-1)
  if (((gridDim.x * gridDim.z) & 7) == 0) {
    const u32 np = gridDim.y, lin = blockIdx.x + gridDim.x * (blockIdx.y + np * blockIdx.z);
    const u32 r = lin >> 3, g = (r / np) * 8 + (lin & 7);
    ct = r % np;
    bx = g % gridDim.x;
    pl = g / gridDim.x;
  }
  const u32 limb = a.l0 + pl;  // index in Q u P
  const ModInfo mi = a.mods[limb];
  const u64 q = mi.q, q2 = 2 * q;
  const u64 *twf = a.twf + ((size_t)limb << LOG_N), *twi = a.twi + ((size_t)limb << LOG_N);
  const u32 ts = tid % (1u << (S - LOGR)), w = tid / (1u << (S - LOGR));
  const u32 row = bx * W + w, gb = row << S;
  const u32 vin = (gb + G0::k_thr(ts)) << 3;
  const u32 vio = (gb + IO::k_thr(ts)) << 3;
  const u64 *kb = a.ksk + (size_t)(limb + a.kshift) * N;  // key row i + kshift (a view's P limbs)
  const size_t kj = (size_t)2 * a.kQP * N, kbs = (size_t)a.kQP * N;
  const u64 *eb = a.ext + ((size_t)ct * a.ndig * a.QP + limb) * N;
  u64 nq1 = 0 - q, nq2 = 0 - q2;
  asm("" : "+s"(nq1));
  asm("" : "+s"(nq2));
  const auto row_io = [&](u64 (&x)[R]) {
    __builtin_amdgcn_sched_barrier(0);
    u64 t[16];
    G0::template load_tw<S0>(t, twf, row, ts);
    run_group<S, LOGR, 0, S0, false, SP, WIDE, KSP_LSW>(x, t, q2, mi);
    G1::template load_tw<S0>(t, twf, row, ts);
    const u32 l0 = lds_idx<S>(w, G0::k_thr(ts));
#pragma unroll
    for (int r = 0; r < R; ++r) lds[l0 + G0::k_reg(r) + lds_pad(G0::k_reg(r))] = x[r];
    __syncthreads();
    const u32 l1 = lds_idx<S>(w, G1::k_thr(ts));
#pragma unroll
    for (int r = 0; r < R; ++r) x[r] = lds[l1 + G1::k_reg(r) + lds_pad(G1::k_reg(r))];
    run_group<S, LOGR, 1, S0, false, SP, WIDE, KSP_LSW>(x, t, q2, mi);
#pragma unroll
    for (int r = 0; r < R; ++r) lds[l1 + G1::k_reg(r) + lds_pad(G1::k_reg(r))] = x[r];
    __syncthreads();
    const u32 l2 = lds_idx<S>(w, IO::k_thr(ts));
#pragma unroll
    for (int r = 0; r < R; ++r) x[r] = lds[l2 + IO::k_reg(r) + lds_pad(IO::k_reg(r))];
    __builtin_amdgcn_sched_barrier(0);
  };
  // acc_P,b over every digit (the products are below 1.5q): reduced by 2q
  // after every second digit only, so below 3.5q < 2^63 at the end (q < 2^61)
  u64 acc0[R], acc1[R];
#pragma unroll
  for (int r = 0; r < R; ++r) acc0[r] = acc1[r] = 0;
#pragma unroll
  for (int j = 0; j < KD; ++j) {
    __builtin_amdgcn_sched_barrier(0);  // the next digit's loads stay below this digit's products
    u64 x[R];
#pragma unroll
    for (int r = 0; r < R; ++r) x[r] = ld_d(eb + (size_t)j * a.QP * N + G0::k_reg(r), vin);
    row_io(x);
    const u64 *k0 = kb + j * kj, *k1 = k0 + kbs;
    sfor<R / 2>([&](auto I) {
      constexpr int r = 2 * decltype(I)::value;
      const u32 kr = IO::k_reg(r);
      const u64x2 K0 = ld2_b(k0 + kr, vio), K1 = ld2_b(k1 + kr, vio);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        acc0[r + h] = acc0[r + h] + mont_mul<SP>(x[r + h], K0[h], mi);
        acc1[r + h] = acc1[r + h] + mont_mul<SP>(x[r + h], K1[h], mi);
        if (j & 1) {  // compile-time (the digit loop is unrolled)
          acc0[r + h] = harvey_csub(acc0[r + h], nq2);
          acc1[r + h] = harvey_csub(acc1[r + h], nq2);
        }
      }
    });
  }
  // the first (row) pass of INTT(acc_P,b): canonical acc in the IO layout ->
  // group 1 -> group 0, stored in the group-0 layout (as PRO_KSP's pass does)
  const u32 vst = (gb + G0::k_thr(ts)) << 3;
  const auto inv_row = [&](const u64(&acc)[R], int b) {
    __builtin_amdgcn_sched_barrier(0);
    u64 x[R], t[16];
    G1::template load_tw<S0>(t, twi, row, ts);
    const u32 l2 = lds_idx<S>(w, IO::k_thr(ts));
#pragma unroll
    for (int r = 0; r < R; ++r) {
      // canonical: below 3.5q (odd KD) or 2q (even KD) before the reductions
      const u64 v = KD & 1 ? harvey_csub(acc[r], nq2) : acc[r];
      lds[l2 + IO::k_reg(r) + lds_pad(IO::k_reg(r))] = harvey_csub(v, nq1);
    }
    __syncthreads();
    const u32 l1 = lds_idx<S>(w, G1::k_thr(ts));
#pragma unroll
    for (int r = 0; r < R; ++r) x[r] = lds[l1 + G1::k_reg(r) + lds_pad(G1::k_reg(r))];
    run_group<S, LOGR, 1, S0, true, SP, false, KSP_LSW>(x, t, q2, mi);
    G0::template load_tw<S0>(t, twi, row, ts);
#pragma unroll
    for (int r = 0; r < R; ++r) lds[l1 + G1::k_reg(r) + lds_pad(G1::k_reg(r))] = x[r];
    __syncthreads();
    const u32 l0 = lds_idx<S>(w, G0::k_thr(ts));
#pragma unroll
    for (int r = 0; r < R; ++r) x[r] = lds[l0 + G0::k_reg(r) + lds_pad(G0::k_reg(r))];
    run_group<S, LOGR, 0, S0, true, SP, false, KSP_LSW>(x, t, q2, mi);
    u64 *dst = a.acc + ((size_t)(2 * ct + b) * a.QP + limb) * N;
#pragma unroll
    for (int r = 0; r < R; ++r) st_d(dst + G0::k_reg(r), vst, x[r]);
  };
  inv_row(acc0, 0);
  inv_row(acc1, 1);
}

}  // namespace

template <int LOG_N, int KD, bool WIDE>
int ksp_launch(fhe_ctx *c, const KspArgs &a, u32 n, u32 nl) {
  constexpr size_t lds = lds_bytes<8, 16>();
  const dim3 grid((1u << (LOG_N - 8)) / 16, n, nl);
  if (c->special) hipLaunchKernelGGL((ksp_fused_pass<LOG_N, KD, WIDE, true>), grid, dim3(256), lds, c->stream, a);
  else hipLaunchKernelGGL((ksp_fused_pass<LOG_N, KD, WIDE, false>), grid, dim3(256), lds, c->stream, a);
  return fhe_check(c, hipGetLastError(), "ksp_fused_pass launch");
}
template <int LOG_N, int KD>
int ksp_dispatch(fhe_ctx *c, const KspArgs &a, u32 n, u32 nl) {
  return c->moduli[a.l0] < (1ull << 60) ? ksp_launch<LOG_N, KD, true>(c, a, n, nl)
                                        : ksp_launch<LOG_N, KD, false>(c, a, n, nl);
}
// every modulus of [l0, l0 + nl) in one lazy-schedule class
static bool one_class(const fhe_ctx *c, u32 l0, u32 nl) {
  const bool wide = c->moduli[l0] < (1ull << 60);
  for (u32 i = l0 + 1; i < l0 + nl; ++i)
    if ((c->moduli[i] < (1ull << 60)) != wide) return false;
  return true;
}

// The fused finish applies: N = 2^15 or 2^16 (a 256-point row pass), at most 3
// digits, the Q limbs in one lazy-schedule class and the P limbs in one.
bool ks_fused_finish_ok(const fhe_ctx *c, u32 ndig) {
  if (!KSF_FUSE || (c->log_n != 15 && c->log_n != 16) || ndig < 1 || ndig > 3 || !c->L || c->K < 1) return false;
  // the P side (ntt_ksp_fused_launch): one lazy-schedule class over the P limbs too
  return one_class(c, 0, c->L) && one_class(c, c->L, c->K);
}

#ifndef BFV_KS_EXTFREE
#define BFV_KS_EXTFREE 1  // BFV: ModUp's row transforms inside the all-limb inner-product pass (ksp_fused_pass)
#endif
int ntt_fwd_col_launch(fhe_ctx *c, const LimbMap &m, const u64 *src) {
  if (c->log_n < 15) return fhe_fail(c, FHE_ERR_UNSUPPORTED, "column pass alone: log_n");
  const u32 per = 65535u;  // polys per launch (gridDim.y)
  for (u32 p0 = 0; p0 < m.n_polys; p0 += per) {
    const size_t off = (size_t)p0 * m.poly_stride * c->n;
    NttArgs a{};
    a.map = m;
    a.map.base = m.base + off;
    a.map.n_polys = std::min(per, m.n_polys - p0);
    a.src = src ? src + off : nullptr;  // out of place: the column pass reads src, writes map
    a.tw = c->d_tw_fwd;
    a.mods = c->d_mods;
    a.ninv = c->d_ninv;
    a.log_n = c->log_n;
    if (a.map.cnt) {
      const int rc = ntt_col_plain(c, a, false, a.map.n_polys * a.map.cnt);
      if (rc) return rc;
    }
  }
  return FHE_OK;
}

bool bfv_ks_extfree_ok(const fhe_ctx *c, u32 ndig) {
  return BFV_KS_EXTFREE && c->bfv_ks_fuse && c->d_bfv_kscale && !c->key_pshift && ks_fused_finish_ok(c, ndig);
}

// INTT(acc_P) with the P limbs' ModUp row transforms and inner product fused
// into its first pass (ksp_fused_pass), then its column pass (d_iscale), as
// ntt_inv_ksp_launch leaves acc's P rows
// skip_col (CONVF): the column pass runs inside ModDown's CONVF launch instead
int ntt_ksp_fused_launch(fhe_ctx *c, u64 *acc, const u64 *ext, const u64 *ksk, u32 n, u32 ndig, bool all_limbs,
                         bool skip_col) {
  if (!ks_fused_finish_ok(c, ndig)) return fhe_fail(c, FHE_ERR_UNSUPPORTED, "fused P-limb key switch: shape");
  if (all_limbs && !bfv_ks_extfree_ok(c, ndig))
    return fhe_fail(c, FHE_ERR_UNSUPPORTED, "fused all-limb key switch: BFV tables");
  const u32 L = c->L, K = c->K, QP = L + K;
  const size_t N = c->n;
  const u32 per = 32767u;  // ciphertexts per launch (the column pass takes 2 polys per ct on gridDim.y)
  for (u32 c0 = 0; c0 < n; c0 += per) {
    const u32 nc = std::min(per, n - c0);
    KspArgs k{};
    k.acc = acc + (size_t)c0 * 2 * QP * N;
    k.ext = ext + (size_t)c0 * ndig * QP * N;
    k.ksk = ksk;
    k.mods = c->d_mods;
    k.twf = c->d_tw_fwd;
    k.twi = c->d_tw_inv;
    k.L = L;
    k.QP = QP;
    k.kQP = ctx_key_qp(c);
    k.ndig = ndig;
    int rc = FHE_OK;
    // one launch per modulus class: BFV's Q limbs (key rows = limb), then the P limbs
    for (int part = all_limbs ? 0 : 1; part < 2 && !rc; ++part) {
      k.l0 = part ? L : 0;
      k.kshift = part ? c->key_pshift : 0;
      const u32 nl = part ? K : L;
      if (c->log_n == 15) {
        rc = ndig == 1 ? ksp_dispatch<15, 1>(c, k, nc, nl) : ndig == 2 ? ksp_dispatch<15, 2>(c, k, nc, nl)
                                                                        : ksp_dispatch<15, 3>(c, k, nc, nl);
      } else {
        rc = ndig == 1 ? ksp_dispatch<16, 1>(c, k, nc, nl) : ndig == 2 ? ksp_dispatch<16, 2>(c, k, nc, nl)
                                                                        : ksp_dispatch<16, 3>(c, k, nc, nl);
      }
    }
    if (rc) return rc;
    if (skip_col && !all_limbs) continue;
    NttArgs a{};
    a.map = all_limbs ? LimbMap{k.acc, QP, QP, 0, QP, 0, 0, 2 * nc} : LimbMap{k.acc, QP, K, L, QP, 0, 0, 2 * nc};
    a.tw = c->d_tw_inv;
    a.mods = c->d_mods;
    a.ninv = c->d_ninv;
    a.log_n = c->log_n;
    a.scale = all_limbs ? c->d_bfv_kscale : c->d_iscale;
    if ((rc = ntt_col_plain(c, a, true, 2 * nc * a.map.cnt))) return rc;
  }
  return FHE_OK;
}

int ntt_ks_fused_finish_launch(fhe_ctx *c, const u64 *conv, const u64 *ext, const u64 *ksk, u32 ndig,
                               const u64 *ta, const u64 *tb, u64 *out, u32 n, u32 g) {
  if (!ks_fused_finish_ok(c, ndig)) return fhe_fail(c, FHE_ERR_UNSUPPORTED, "fused key-switch finish: shape");
  if (!c->d_pinv3) return fhe_fail(c, FHE_ERR_UNSUPPORTED, "fused key-switch finish: tables");
  const size_t N = c->n, L = c->L, QP = c->L + c->K;
  const u32 per = 65535u;  // gridDim.y
  for (u32 c0 = 0; c0 < n; c0 += per) {
    const u32 nc = std::min(per, n - c0);
    KsfArgs a{};
    a.conv = conv + (size_t)c0 * 2 * L * N;
    a.ext = ext + (size_t)c0 * ndig * QP * N;
    a.ksk = ksk;
    a.ta = ta + (size_t)c0 * 2 * L * N;
    a.tb = g ? nullptr : tb + (size_t)c0 * 2 * L * N;
    a.g = g;
    a.out = out + (size_t)c0 * 2 * L * N;
    a.mods = c->d_mods;
    a.tw = c->d_tw_fwd;
    a.pinv = c->d_pinv3;
    a.pplain = c->d_pplain;
    a.pm1 = c->d_pm1;
    a.L = c->L;
    a.QP = (u32)QP;
    a.kQP = ctx_key_qp(c);
    a.ndig = ndig;
    a.alpha = c->alpha;
    int rc;
    if (c->log_n == 15) {
      rc = ndig == 1 ? ksf_dispatch<15, 1>(c, a, nc) : ndig == 2 ? ksf_dispatch<15, 2>(c, a, nc)
                                                                  : ksf_dispatch<15, 3>(c, a, nc);
    } else {
      rc = ndig == 1 ? ksf_dispatch<16, 1>(c, a, nc) : ndig == 2 ? ksf_dispatch<16, 2>(c, a, nc)
                                                                  : ksf_dispatch<16, 3>(c, a, nc);
    }
    if (rc) return rc;
  }
  return FHE_OK;
}
