// ntt.hip -- negacyclic NTT / INTT for gfx950.
//
// Algorithm (same transform as the oracle's orc_ntt_fwd, oracle/fhe_oracle.c):
// Harvey's lazy Cooley-Tukey forward (natural in, bit-reversed out, values in
// [0,4q) between stages, or [0,8q) with fewer reductions for q < 2^60 -- see
// wide_csub) and Gentleman-Sande inverse ([0,2q)).  The twiddle of
// butterfly (j, j+t) at global stage s is psi^brv(2^s + (j >> (logN - s))),
// stored in Montgomery form (psi^e * 2^64 mod q) so one mont_mul = 6
// quarter-rate multiplies gives the exact product (modarith.hpp).
//
// MI355X mapping.  One limb-polynomial of N u64 words is split into passes;
// a pass owns global stages [s0, s0+S) and works on independent
// sub-transforms of 2^S elements at stride N >> (s0+S):
//   N <= 2^13 : ONE pass, one residue per workgroup (up to 64 KiB of LDS) --
//               the north-star "one-residue-per-WG"; at N = 2^14 (128 KiB, one
//               1024-thread workgroup per CU) the fused prologue/epilogue
//               passes keep it, while plain NTTs run two 7-stage passes with 4
//               workgroups per CU, which measured 2% faster (C2) despite the
//               intermediate's round trip;
//   N  = 2^15..2^17 : two passes (column pass of stride N/2^S1, then row pass
//               of contiguous 2^S2 blocks), because a 512 KiB N=2^16 residue
//               exceeds the 160 KiB LDS of a CU.
// Pass geometry (N, stages, stride, last) is compile-time, so every element
// address is one per-thread 32-bit offset plus a constant on a scalar base.
// Inside a pass each thread keeps R = 16 elements in VGPRs and runs LOGR = 4
// butterfly stages in registers per "group"; groups are separated by ONE LDS
// exchange (write, barrier, read).  The first group loads straight from HBM
// and the last group stores straight to HBM (128 B row segments for column
// passes, 16 contiguous words per lane for row passes), and each group's
// twiddles are fetched while the previous group computes, so neither the
// data nor the twiddle latency sits on the VALU critical path.
#include <algorithm>

#include "context.hpp"

#ifndef KSQ_PD
#define KSQ_PD 2  // EPI_KSQ operand prefetch depth (elements; 3 measured no faster, profiles/r03/ab_ksq_pd_aut.txt)
#endif
#ifndef TENSOR_CHUNK
#define TENSOR_CHUNK 65535u  // ciphertexts per INTT(d2) pass pair (MALL-sized chunks: see DESIGN §4)
#endif
#ifndef COMBINE_CHUNK
#define COMBINE_CHUNK 65534u  // polys per NTT(conv) pass pair (even)
#endif
#ifndef KSQ_GI
#define KSQ_GI 1  // EPI_KSQ: (limb, row block) groups interleaved per XCD (4: kernel -1.6% but headline -0.2%, profiles/r03/ab_group_interleave.txt)
#endif
#ifndef KSP_GI
#define KSP_GI 1  // PRO_KSP: the same
#endif
#ifndef KSP_PD
#define KSP_PD 2  // PRO_KSP operand prefetch depth (elements)
#endif
#ifndef GEN_VEC
#define GEN_VEC 0  // 1: generic moduli's butterfly and KS products in lock-step (mont_mul_gen_vec): -0.6% on OpenFHE-style primes, profiles/r03/ab_gen_vec.txt
#endif
#ifndef CONV_SP60
#define CONV_SP60 1  // PRO_CONV on special targets below 2^60: the column sums reduced in place (dot_cols_sp60); headline +0.8%, profiles/r03/ab_conv_sp60.txt
#endif
#ifndef CONV_COLS
#define CONV_COLS 1  // PRO_CONV: 31-bit column sums (dot_cols); 0: dot_mont_lazy
#endif
#ifndef AUT_PD
#define AUT_PD 2  // PRO_AUTOMORPH gather prefetch depth (elements)
#endif
#ifndef MODUP_COL_SPLIT
#define MODUP_COL_SPLIT 1
#endif

namespace {

struct NttArgs {
  LimbMap map;
  const u64 *tw;         // [nmod][N], Montgomery form
  const ModInfo *mods;   // [nmod]
  const u64 *ninv;       // [nmod], N^-1 in Montgomery form
  u32 log_n;
  // inverse only: leave out the N^-1 scaling (the consumer's conversion
  // constants carry it, fhe_ctx::fold_ninv); outputs stay canonical
  u32 noscale;
  // inverse only: if set, the last pass multiplies by scale[mod] (Montgomery
  // form) instead of N^-1: the per-source constant of a following base
  // conversion rides on the transform (fhe_ctx::d_iscale), so its outputs are
  // already the conversion's canonical v_i = [x (S/s_i)^-1]_{s_i}
  const u64 *scale;
  // forward only: the first pass reads its limbs from src (the same layout as
  // map.base: poly stride and limb positions) instead of transforming in
  // place -- an out-of-place NTT, so a caller's input is never copied first
  const u64 *src;
  // forward only: leave the outputs in the lazy range (below 8q < 2^63), for a
  // consumer whose Montgomery products accept any input below 2^63 (the KS
  // inner product on special moduli)
  u32 lazy_out;
  // EPI_COMBINE (forward last pass over the ModDown conversion conv [p][L][N],
  // p = 2 ct + b): out[p][i] = (add_mask bit b ? base[p][i] : 0) + (acc[p][i] - conv) P^-1
  const u64 *e_acc;      // [p][e_acc_stride][N]
  const u64 *e_base;     // [p][L][N], may alias e_out
  u64 *e_out;            // [p][L][N]
  const u64 *e_pinv;     // [L] P^-1 R mod q_i
  u32 e_acc_stride;
  u32 e_add_mask;
  u32 e_g;  // combine: 0, or the base is read as sigma_g(base) (rotation: sigma_g(c0) never stored)
  // EPI_KSQ (EPI_COMBINE whose acc_Q is the key-switching inner product, formed
  // here instead of being read): acc[p][i] = sum_j ext[ct][j][i] ksk[j][b][i] R^-1,
  // p = 2 ct + b, with ext [ct][e_ndig][e_QP][N] and ksk [e_ndig][2][e_QP][N]
  const u64 *e_ext, *e_ksk;
  u32 e_ndig, e_QP;
  // PRO_TENSOR (first pass of the inverse NTT of d2 in CKKS mul+relin, poly =
  // ciphertext): the pass reads the operands a, b [ct][2][L][N] instead of d2,
  // writes the relinearisation base out[ct][0] = a0 b0, out[ct][1] = a0 b1 + a1 b0
  // and the own-digit ext slot d2 R, and transforms d2 = a1 b1 (the tensor
  // product fused here: d2 never makes an HBM round trip before the INTT)
  const u64 *t_a, *t_b;
  u64 *t_out;            // may alias t_a / t_b (element-wise)
  u64 *t_ext;            // [ct][ndig][QP][N]
  u32 t_L, t_QP, t_alpha, t_ndig;
  // PRO_AUTOMORPH (first pass of the inverse NTT of sigma_g(c1) in CKKS
  // rotation): reads the input ciphertext t_a [ct][2][L][N] (NTT form) at the
  // permuted slots, writes the key-switch base t_out[ct][0] = sigma_g(c0) and
  // the own-digit ext slot sigma_g(c1) R, and transforms sigma_g(c1)
  u32 t_g;
  // PRO_CONV (first (column) pass of a forward NTT): the pass's input limb is
  // the fast base conversion y_m = sum_i v_i h[i][m] of c_ns canonical source
  // limbs v_i at c_src[poly][c_src_first + i] (poly stride c_src_stride limbs),
  // m = the active-limb index of the map; conv never makes an HBM round trip
  const u64 *c_src;
  const u64 *c_h;        // [ns][nd] ConvTab.h
  u32 c_src_stride, c_src_first, c_ns, c_nd;
};

// EPI_COMBINE: epilogue of a forward last pass; PRO_TENSOR: prologue of an
// inverse first (row) pass
// PRO_BFVT: prologue of the inverse first (row) pass of the BFV tensor
// product e = (a0 b0, a0 b1 + a1 b0, a1 b1) in one RNS base
// PRO_CONV: prologue of a forward first (column) pass, the base conversion
// that produces its input
// EPI_KSQ + d - 1: EPI_COMBINE with the Q limbs' key-switching inner product
// over d = 1..4 digits fused in (the digit count is compile-time)
// PRO_CONV + ns - 1: the conversion prologue over ns = 1..4 source limbs (compile-time)
// PRO_KSP + d - 1: prologue of the inverse first (row) pass of INTT(acc_P):
// the P limbs' key-switching inner product over d = 1..4 digits (acc_P is
// formed at the load positions and never stored)
enum { EPI_NONE = 0, EPI_COMBINE = 1, PRO_TENSOR = 2, PRO_AUTOMORPH = 3, PRO_BFVT = 4, EPI_KSQ = 6, PRO_CONV = 11,
       PRO_KSP = 16 };
__host__ __device__ constexpr bool is_conv(int e) { return e >= PRO_CONV && e < PRO_CONV + 4; }
__host__ __device__ constexpr int conv_ns(int e) { return e - PRO_CONV + 1; }
__host__ __device__ constexpr bool is_ksq(int e) { return e >= EPI_KSQ && e < EPI_KSQ + 4; }
__host__ __device__ constexpr int ksq_digits(int e) { return e - EPI_KSQ + 1; }
__host__ __device__ constexpr bool is_combine(int e) { return e == EPI_COMBINE || is_ksq(e); }
__host__ __device__ constexpr bool is_ksp(int e) { return e >= PRO_KSP && e < PRO_KSP + 4; }
__host__ __device__ constexpr int ksp_digits(int e) { return e - PRO_KSP + 1; }

// NTT-domain automorphism: slot k holds a(psi^e), e = 2 brv(k) + 1, and
// sigma_g(a)(psi^e) = a(psi^(e g)); the byte offset of the source slot of k.
// The 64 lanes of a coalesced load read one aligned 64-slot block of the
// source (g only permutes inside it).
template <int LOG_N>
__device__ __forceinline__ u32 aut_src(u32 k, u32 g) {
  constexpr u32 MASK = (2u << LOG_N) - 1;
  const u32 e = (((__brev(k) >> (32 - LOG_N)) << 1) | 1) * g & MASK;
  return (__brev(e >> 1) >> (32 - LOG_N)) << 3;
}

// per-workgroup epilogue / prologue operands (resolved once per limb)
struct EpiRow {
  const u64 *acc;
  const u64 *kext, *kksk;  // EPI_KSQ, PRO_KSP: digit 0's ext / key row of this limb (digit j at + j stride)
  size_t ext_j, ksk_j;     // digit strides (words)
  const u64 *base;
  u64 *out;
  u64 pinv;
  bool add;
  const u64 *a0, *a1, *b0, *b1;  // PRO_TENSOR
  u64 *o0, *o1, *ext;
  u32 g;  // PRO_AUTOMORPH (a0, a1 = c0, c1 of the limb; o0 = base or null; ext); combine: e_g
  u32 e;  // PRO_BFVT: which tensor output (0, 1, 2) this poly is
  const u64 *src;  // PRO_CONV: source limb 0 of this poly (limb i at src + i N)
  u64 h[4];        // PRO_CONV: h[i][m] of this workgroup's target limb
};

// LDS slot of element k of sub-transform w: one pad word per 16 words and per
// sub-transform keeps every exchange pattern free of bank conflicts
// (SQ_LDS_BANK_CONFLICT = 0), and the slot stays affine in the register index
// r, so the 16 accesses of a thread share one address register.
// Element access at a 32-bit word index from a scalar (per-workgroup) base:
// the byte offset is formed in 32 bits so the load/store uses the
// `global_load v, v_off, s[base:base+1]` form (one VALU op per address).
__device__ __forceinline__ u64 ld_at(const u64 *base, u32 idx) {
  return *(const u64 *)((const char *)base + (idx << 3));
}
// the same at a byte offset (per-thread offsets computed once per pass)
__device__ __forceinline__ u64 ld_b(const u64 *base, u32 off) { return *(const u64 *)((const char *)base + off); }
// a pass's own data words are read once: non-temporal (A/B on one box: the
// forward NTT -1%; the fused prologue/epilogue operand streams lose with nt,
// so they keep ld_b; nt stores measured neutral)
__device__ __forceinline__ u64 ld_d(const u64 *base, u32 off) {
  return __builtin_nontemporal_load((const u64 *)((const char *)base + off));
}
__device__ __forceinline__ void st_b(u64 *base, u32 off, u64 v) { *(u64 *)((char *)base + off) = v; }

template <int S>
__device__ __forceinline__ u32 lds_idx(u32 w, u32 k) {
  constexpr u32 SUB = 1u << S;
  constexpr u32 PAD = SUB + (SUB >> 4) + 1;
  return w * PAD + k + (k >> 4);
}
template <int S, int W>
constexpr size_t lds_bytes() {
  return (size_t)W * ((1u << S) + (1u << S >> 4) + 1) * sizeof(u64);
}


// Group geometry (compile time): group g covers local stages
// [g*LOGR, g*LOGR + nb); its butterfly bits are k bits [p, p+nb).  A thread
// holds R = 2^LOGR elements k(r) = hh<<(p+nb+ex) | rx<<(p+nb) | rb<<p | lo_t;
// k_thr(ts) is the per-thread part, k_reg(r) the compile-time part.
template <int S, int LOGR, int G>
struct Grp {
  static constexpr int nb = (S - G * LOGR) < LOGR ? (S - G * LOGR) : LOGR;
  static constexpr int ex = LOGR - nb;
  static constexpr int p = S - G * LOGR - nb;
  static constexpr int NTW = (1 << ex) * ((1 << nb) - 1);  // distinct twiddles per thread
  __device__ static __forceinline__ u32 k_thr(u32 ts) {
    return ((ts >> p) << (p + nb + ex)) | (ts & ((1u << p) - 1));
  }
  static constexpr u32 k_reg(int r) {
    return ((u32)(r >> nb) << (p + nb)) | ((u32)(r & ((1 << nb) - 1)) << p);
  }
  __device__ static __forceinline__ u32 k_of(int r, u32 ts) { return k_thr(ts) | k_reg(r); }
  // slot of (tau, rx, d) in the per-thread twiddle array, d < 2^tau
  __device__ static constexpr int slot(int tau, int rx, int d) { return rx * ((1 << nb) - 1) + (1 << tau) - 1 + d; }
  // twiddle of local stage sigma = G*LOGR + tau: index 2^(s0+sigma) + hi 2^sigma + kk,
  // kk = (hh 2^ex + rx) 2^tau + d.  The thread-dependent part (hi, hh) is one
  // 32-bit offset per tau; the rest is a compile-time offset on a scalar base.
  template <int S0>
  __device__ static __forceinline__ void load_tw(u64 (&t)[16], const u64 *tw, u32 hi, u32 ts) {
    const u32 hh = ts >> p;
#pragma unroll
    for (int tau = 0; tau < nb; ++tau) {
      const int sigma = G * LOGR + tau;
      const u32 thr = (hi << sigma) + (hh << (ex + tau));
#pragma unroll
      for (int rx = 0; rx < (1 << ex); ++rx)
#pragma unroll
        for (int d = 0; d < (1 << tau); ++d)
          t[slot(tau, rx, d)] = ld_at(tw + ((1u << (S0 + sigma)) + ((u32)rx << tau) + (u32)d), thr);
    }
  }
};

// x - m if that is non-negative, else x (x, m < 2^63; neg_m = -m), selected
// by the sign word with two v_bfi_b32: no VCC compare/select, so no hazard nops
__device__ __forceinline__ u64 harvey_csub(u64 x, u64 neg_m) {
  const u64 d = x + neg_m;
  const u32 m = (u32)((int32_t)(u32)(d >> 32) >> 31);  // all ones iff d < 0
  const u64 mm = ((u64)m << 32) | m;
  return (x & mm) | (d & ~mm);
}

// Forward lazy-range schedule.  NARROW (every modulus): values in [0,4q)
// between stages, U = csub(X, 2q) at every stage (Harvey).  WIDE (moduli
// q < 2^60, i.e. 8q < 2^63, the Montgomery input bound; the special product
// is below 1.5q, the generic one below 2q): a stage with
// input bound B q gives outputs below (B+2) q without any reduction
// (X' = X + V < (B+1.5) q, Y' = X + 2q - V < (B+2) q), so from an input in
// [0,4q) the stages run 4 -> 6 -> 8 and then alternate csub(X, 4q) (8 -> 6)
// with none (6 -> 8): global stages 2, 4, 6, ... reduce, the others do not,
// and 7 of the 16 stages of N = 2^16 reduce instead of 16.  Pass outputs stay
// below 8q < 2^63; the last stage canonicalises from [0,8q).
__host__ __device__ constexpr bool wide_csub(int gs) { return gs >= 2 && (gs & 1) == 0; }

template <int S, int LOGR, int G, int S0, bool INV, bool SP, bool WIDE>
__device__ __forceinline__ void run_group(u64 (&x)[16], const u64 (&t)[16], u64 q2, const ModInfo &mi) {
  using GP = Grp<S, LOGR, G>;
  constexpr int R = 1 << LOGR;
#pragma unroll
  for (int ti = 0; ti < GP::nb; ++ti) {
    const int tau = INV ? GP::nb - 1 - ti : ti;
    const int half = 1 << (GP::nb - 1 - tau);
    if constexpr (SP || GEN_VEC) {
      // the R/2 butterflies of this stage in lock-step (see mont_mul_sp_vec)
      constexpr int H = R / 2;
      u64 A[H], Wt[H], V[H], U[H];
      int lo_idx[H];
      {
        int n = 0;
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const int rb = r & ((1 << GP::nb) - 1), rx = r >> GP::nb;
          if (rb & half) continue;
          lo_idx[n] = r;
          Wt[n] = t[GP::slot(tau, rx, rb >> (GP::nb - tau))];
          ++n;
        }
      }
      // 64-bit adds of SGPR constants as single v_lshl_add_u64 (no carry
      // chain through VCC, which costs s_nop wait states): a - b = a + (2q+1) + ~b - 2q
      u64 nq2 = 0 - q2, q2p1 = q2 + 1, nq4 = 0 - 2 * q2;
      asm("" : "+s"(nq2));
      asm("" : "+s"(q2p1));
      asm("" : "+s"(nq4));
      const int gs = S0 + G * LOGR + tau;  // global stage
      const bool red = !WIDE || wide_csub(gs);
#pragma unroll
      for (int i = 0; i < H; ++i) {
        const u64 X = x[lo_idx[i]], Y = x[lo_idx[i] + half];
        if (!INV) {
          U[i] = !red ? X : harvey_csub(X, WIDE ? nq4 : nq2);
          A[i] = Y;
        } else {
          U[i] = harvey_csub(X + Y, nq2);
          A[i] = (X + q2p1) + ~Y;
        }
      }
      if constexpr (SP) mont_mul_sp_vec<H>(V, A, Wt, mi.q_hi);
      else mont_mul_gen_vec<H>(V, A, Wt, mi);
#pragma unroll
      for (int i = 0; i < H; ++i) {
        if (!INV) {
          x[lo_idx[i]] = U[i] + V[i];
          x[lo_idx[i] + half] = (U[i] + q2p1) + ~V[i];
        } else {
          x[lo_idx[i]] = U[i];
          x[lo_idx[i] + half] = V[i];
        }
      }
      continue;
    }
    // generic moduli: the same lazy schedules (the generic Montgomery product
    // is below 2q and accepts any input below 8q, since 8q^2 < q 2^64)
    u64 nq2 = 0 - q2, q2p1 = q2 + 1, nq4 = 0 - 2 * q2;
    asm("" : "+s"(nq2));
    asm("" : "+s"(q2p1));
    asm("" : "+s"(nq4));
    const bool red = !WIDE || wide_csub(S0 + G * LOGR + tau);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int rb = r & ((1 << GP::nb) - 1), rx = r >> GP::nb;
      if (rb & half) continue;
      const u64 w = t[GP::slot(tau, rx, rb >> (GP::nb - tau))];
      u64 &X = x[r];
      u64 &Y = x[r + half];
      if (!INV) {
        const u64 uu = !red ? X : harvey_csub(X, WIDE ? nq4 : nq2);
        const u64 v = mont_mul<SP>(Y, w, mi);
        X = uu + v;
        Y = (uu + q2p1) + ~v;
      } else {
        const u64 uu = X, vv = Y;
        X = harvey_csub(uu + vv, nq2);
        Y = mont_mul<SP>((uu + q2p1) + ~vv, w, mi);
      }
    }
  }
}

// Compile-time pass geometry.  A pass owns global stages [S0, S0+S) of an
// N = 2^LOG_N transform; column passes work at element stride 2^LS, row passes
// on contiguous blocks.  The last pass canonicalises (and scales by N^-1).
template <int LOG_N, int S, bool COLS, bool INV>
struct PassGeo {
  static constexpr bool single = S == LOG_N;
  static constexpr int S0 = COLS ? 0 : LOG_N - S;
  static constexpr int LS = COLS ? LOG_N - S : 0;
  static constexpr bool LAST = single || (COLS == INV);
};

template <int LOG_N, int S, int LOGR, int W, bool INV, bool COLS, bool SP, bool WIDE, int EPI, int GI>
__device__ __forceinline__ void group_loop(u64 (&x)[16], u64 (&tc)[16], u64 *lds, const u64 *tw, u64 *data,
                                           u32 voff, u32 w, u32 ts, u32 hi, const NttArgs &a,
                                           const ModInfo &mi, u32 mod, const EpiRow &ep) {
  using PG = PassGeo<LOG_N, S, COLS, INV>;
  constexpr int NG = (S + LOGR - 1) / LOGR;
  constexpr int R = 1 << LOGR;
  constexpr int G = INV ? NG - 1 - GI : GI;
  using GP = Grp<S, LOGR, G>;
  const u64 q = mi.q, q2 = 2 * q;
  if constexpr (GI + 1 < NG) {
    constexpr int GN = INV ? NG - 2 - GI : GI + 1;
    u64 tn[16];
    Grp<S, LOGR, GN>::template load_tw<PG::S0>(tn, tw, hi, ts);  // in flight while this group computes
    run_group<S, LOGR, G, PG::S0, INV, SP, WIDE>(x, tc, q2, mi);
    const u32 lw = lds_idx<S>(w, GP::k_thr(ts));
#pragma unroll
    for (int r = 0; r < R; ++r) lds[lw + GP::k_reg(r) + (GP::k_reg(r) >> 4)] = x[r];
    __syncthreads();
    const u32 lr = lds_idx<S>(w, Grp<S, LOGR, GN>::k_thr(ts));
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const u32 kr = Grp<S, LOGR, GN>::k_reg(r);
      x[r] = lds[lr + kr + (kr >> 4)];
    }
    group_loop<LOG_N, S, LOGR, W, INV, COLS, SP, WIDE, EPI, GI + 1>(x, tn, lds, tw, data, voff, w, ts, hi, a, mi,
                                                                     mod, ep);
  } else {
    // EPI_COMBINE: the epilogue's acc and base words are in flight while the
    // last group computes (the LDS footprint caps occupancy at 4 waves per
    // SIMD, so the 128-VGPR budget has room for them)
    constexpr int RE = is_combine(EPI) ? R : 1;
    u64 pa[RE], pb[RE];
    if constexpr (is_combine(EPI)) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if constexpr (EPI == EPI_COMBINE) pa[r] = ld_b(ep.acc + Grp<S, LOGR, 0>::k_reg(r), voff);
        const u32 kr = Grp<S, LOGR, 0>::k_reg(r);
        if (!ep.add) pb[r] = 0;
        else if (ep.g) pb[r] = ld_b(ep.base, aut_src<LOG_N>((voff >> 3) + kr, ep.g));  // sigma_g(base)
        else pb[r] = ld_b(ep.base + kr, voff);
      }
    }
    run_group<S, LOGR, G, PG::S0, INV, SP, WIDE>(x, tc, q2, mi);
    // negated reduction constants pinned in SGPRs, so each conditional
    // subtraction is one v_lshl_add_u64 with a scalar operand (left to itself
    // the compiler forms x - m as a v_subrev_co/v_subb_co borrow chain with
    // s_nop hazard padding)
    u64 nq1 = 0 - q, nq2 = 0 - q2, nq4 = 0 - 2 * q2;
    asm("" : "+s"(nq1));
    asm("" : "+s"(nq2));
    asm("" : "+s"(nq4));
    // EPI_COMBINE: B q + 1, so (acc + cb1) + ~v = acc + B q - v
    u64 cb1 = (WIDE ? 2 * q2 : q2) + 1;
    asm("" : "+s"(cb1));
    if constexpr (PG::LAST) {
      if constexpr (is_combine(EPI)) {
        // the ModDown finish takes NTT(conv) below 4q (WIDE) / 2q: one
        // conditional subtraction instead of canonicalising (see the epilogue)
#pragma unroll
        for (int r = 0; r < R; ++r) x[r] = harvey_csub(x[r], WIDE ? nq4 : nq2);
      } else if constexpr (!INV) {
        if (!a.lazy_out) {
#pragma unroll
          for (int r = 0; r < R; ++r) {
            u64 v = x[r];
            if (WIDE) v = harvey_csub(v, nq4);
            x[r] = harvey_csub(harvey_csub(v, nq2), nq1);
          }
        }
      } else {
        if (a.noscale && !a.scale) {
#pragma unroll
          for (int r = 0; r < R; ++r) x[r] = harvey_csub(x[r], nq1);  // GS outputs are below 2q
        } else {
          const u64 sc = a.scale ? a.scale[mod] : a.ninv[mod];
#pragma unroll
          for (int r = 0; r < R; ++r) x[r] = harvey_csub(mont_mul<SP>(x[r], sc, mi), nq1);
        }
      }
    }
    if constexpr (!COLS && G != 0) {
      // EPI_KSQ: the key-switching operands (ext and key words, KD of each per
      // element) are software-pipelined PD elements deep, and the first PD
      // elements' loads are in flight across the re-layout barrier
      constexpr int KD = is_ksq(EPI) ? ksq_digits(EPI) : 1;
      constexpr int PD = is_ksq(EPI) && SP ? KSQ_PD : 1;
      u64 ek[PD + 1][2 * KD];
      if constexpr (is_ksq(EPI)) {
#pragma unroll
        for (int r = 0; r < PD; ++r) {
          const u32 kr = Grp<S, LOGR, 0>::k_reg(r);
#pragma unroll
          for (int j = 0; j < KD; ++j) {
            ek[r][j] = ld_b(ep.kext + j * ep.ext_j + kr, voff);
            ek[r][KD + j] = ld_b(ep.kksk + j * ep.ksk_j + kr, voff);
          }
        }
      }
      // row pass ending in a group whose lanes each own contiguous words:
      // re-layout through LDS so the HBM store is coalesced (group-0 layout)
      const u32 lw = lds_idx<S>(w, GP::k_thr(ts));
#pragma unroll
      for (int r = 0; r < R; ++r) lds[lw + GP::k_reg(r) + (GP::k_reg(r) >> 4)] = x[r];
      __syncthreads();
      using G0 = Grp<S, LOGR, 0>;
      const u32 lr = lds_idx<S>(w, G0::k_thr(ts));
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const u32 kr = G0::k_reg(r);
        const u64 v = lds[lr + kr + (kr >> 4)];
        if constexpr (is_combine(EPI)) {
          // ModDown finish fused into the last pass of NTT(conv): conv never reaches HBM.
          // acc - conv is formed as acc + Bq - v (v < Bq, B = 4 WIDE / 2): below
          // 5q < 2^63 for q < 2^60 and 3q < 2^63 for q < 2^61, inside the
          // Montgomery input bound, whose product below 1.5q (2q generic)
          // is canonicalised by one conditional subtraction
          u64 acc;
          if constexpr (is_ksq(EPI)) {
            // acc_Q = sum_j ext_j ksk_j R^-1 (ext carries R), at the store
            // position: acc_Q never makes an HBM round trip.  Each product is
            // below 1.5q (2q generic), so one subtraction of 4q (WIDE) leaves
            // the lazy sum below 4q; otherwise it is made canonical.
            if (r + PD < R) {
              const u32 kn = G0::k_reg(r + PD);
#pragma unroll
              for (int j = 0; j < KD; ++j) {
                ek[(r + PD) % (PD + 1)][j] = ld_b(ep.kext + j * ep.ext_j + kn, voff);
                ek[(r + PD) % (PD + 1)][KD + j] = ld_b(ep.kksk + j * ep.ksk_j + kn, voff);
              }
            }
            u64 e[KD], k[KD], pr[KD];
#pragma unroll
            for (int j = 0; j < KD; ++j) {
              e[j] = ek[r % (PD + 1)][j];
              k[j] = ek[r % (PD + 1)][KD + j];
            }
            if constexpr (SP) {
              mont_mul_sp_vec<KD>(pr, e, k, mi.q_hi);
            } else if constexpr (GEN_VEC) {
              mont_mul_gen_vec<KD>(pr, e, k, mi);
            } else {
#pragma unroll
              for (int j = 0; j < KD; ++j) pr[j] = mont_mul<SP>(e[j], k[j], mi);
            }
            acc = pr[0];
            if constexpr (WIDE) {
              // q < 2^60: the whole sum stays below 6q < 2^63
#pragma unroll
              for (int j = 1; j < KD; ++j) acc += pr[j];
              if constexpr (KD > 2) acc = harvey_csub(acc, nq4);
            } else {
              // q < 2^61: keep the running sum below 2q, then canonical
#pragma unroll
              for (int j = 1; j < KD; ++j) acc = harvey_csub(acc + pr[j], nq2);
              acc = harvey_csub(acc, nq1);
            }
          } else {
            acc = pa[r];
          }
          u64 ks = harvey_csub(mont_mul<SP>((acc + cb1) + ~v, ep.pinv, mi), nq1);
          if (ep.add) ks = add_mod(ks, pb[r], q);
          st_b(ep.out + kr, voff, ks);
        } else {
          st_b(data + kr, voff, v);
        }
      }
    } else {
      static_assert(!is_combine(EPI), "epilogues run in the re-laid-out row store");
      // column pass (or single pass ending in group 0): element k of this
      // thread sits at voff + k_reg(r) << LS -- a compile-time offset on the
      // scalar base, so the address costs no VALU
#pragma unroll
      for (int r = 0; r < R; ++r) st_b(data + ((size_t)GP::k_reg(r) << PG::LS), voff, x[r]);
    }
  }
}

template <int LOG_N, int S, int LOGR, int W, bool INV, bool COLS, bool SP, bool WIDE, int EPI>
__device__ __forceinline__ void pass_body(const NttArgs &a, u64 *lds, u64 *data, const u64 *tw, const ModInfo &mi,
                                          u32 mod, u32 w, u32 ts, u32 hi, u32 gb, const EpiRow &ep) {
  using PG = PassGeo<LOG_N, S, COLS, INV>;
  constexpr int R = 1 << LOGR;
  constexpr int NG = (S + LOGR - 1) / LOGR;
  constexpr int G0 = INV ? NG - 1 : 0;
  u64 tc[16];
  Grp<S, LOGR, G0>::template load_tw<PG::S0>(tc, tw, hi, ts);
  u64 x[R];
  u32 voff;  // byte offset of this thread's element k_thr of the first (HBM) group layout
  if constexpr (!COLS && G0 != 0) {
    // row pass starting in a per-lane-contiguous group: coalesced load in the
    // group-0 layout, then one LDS re-layout
    using GZ = Grp<S, LOGR, 0>;
    voff = (gb + GZ::k_thr(ts)) << 3;
    if constexpr (EPI == PRO_TENSOR) {
      // the CKKS tensor formulas, element-wise at the coalesced positions.
      // Software-pipelined PD elements deep: the operand loads of element
      // r + PD are issued before element r's stores (the outputs may alias the
      // operands element-wise only, so the compiler would otherwise wait for
      // each element's loads right after the previous element's stores)
      constexpr int PD = SP ? 2 : 0;  // the generic products need the registers
      u64 op[PD + 1][4];
#pragma unroll
      for (int r = 0; r < PD; ++r) {
        const u32 kr = GZ::k_reg(r);
        op[r][0] = ld_b(ep.a0 + kr, voff), op[r][1] = ld_b(ep.a1 + kr, voff);
        op[r][2] = ld_b(ep.b0 + kr, voff), op[r][3] = ld_b(ep.b1 + kr, voff);
      }
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const u32 kr = GZ::k_reg(r);
        if (r + PD < R) {
          const u32 kn = GZ::k_reg(r + PD);
          u64(&o)[4] = op[(r + PD) % (PD + 1)];
          o[0] = ld_b(ep.a0 + kn, voff), o[1] = ld_b(ep.a1 + kn, voff);
          o[2] = ld_b(ep.b0 + kn, voff), o[3] = ld_b(ep.b1 + kn, voff);
        }
        const u64 a0 = op[r % (PD + 1)][0], a1 = op[r % (PD + 1)][1];
        const u64 b0 = op[r % (PD + 1)][2], b1 = op[r % (PD + 1)][3];
        st_b(ep.o0 + kr, voff, mul_mod<SP>(a0, b0, mi));
        U128 s = mul128(a0, b1);
        mac128(s, a1, b0);
        st_b(ep.o1 + kr, voff, reduce128<SP>(s, mi));
        const u64 t = mont_mul<SP>(mont_reduce<SP>(mul128(a1, b1), mi), mi.r2, mi);  // d2 in [0, 2q)
        x[r] = csub(t, mi.q);
        st_b(ep.ext + kr, voff, csub(mont_mul<SP>(t, mi.r2, mi), mi.q));  // d2 R
      }
    } else if constexpr (EPI == PRO_BFVT) {
      // the BFV tensor formulas at the coalesced positions; e is per workgroup
      if (ep.e == 1) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const u32 kr = GZ::k_reg(r);
          U128 s = mul128(ld_b(ep.a0 + kr, voff), ld_b(ep.b1 + kr, voff));
          mac128(s, ld_b(ep.a1 + kr, voff), ld_b(ep.b0 + kr, voff));
          x[r] = reduce128<SP>(s, mi);
        }
      } else {
        // e = 0: (a0, b0), e = 2: (a1, b1) -- the pair is resolved in ntt_pass
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const u32 kr = GZ::k_reg(r);
          x[r] = mul_mod<SP>(ld_b(ep.a0 + kr, voff), ld_b(ep.b0 + kr, voff), mi);
        }
      }
    } else if constexpr (EPI == PRO_AUTOMORPH) {
      // NTT-domain automorphism (aut_src), software-pipelined like PRO_TENSOR:
      // element r + PD's gathers are issued before element r's stores.  With
      // o0 null, sigma(c0) is not stored (the combine reads it as sigma_g(c0))
      constexpr int PD = AUT_PD;
      const auto src_of = [&](int r) { return aut_src<LOG_N>((voff >> 3) + GZ::k_reg(r), ep.g); };
      u64 y[PD + 1][2];
#pragma unroll
      for (int r = 0; r < PD; ++r) {
        const u32 sr = src_of(r);
        y[r][0] = ep.o0 ? ld_b(ep.a0, sr) : 0, y[r][1] = ld_b(ep.a1, sr);
      }
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const u32 kr = GZ::k_reg(r);
        if (r + PD < R) {
          const u32 sn = src_of(r + PD);
          y[(r + PD) % (PD + 1)][0] = ep.o0 ? ld_b(ep.a0, sn) : 0, y[(r + PD) % (PD + 1)][1] = ld_b(ep.a1, sn);
        }
        const u64 y0 = y[r % (PD + 1)][0], y1 = y[r % (PD + 1)][1];
        if (ep.o0) st_b(ep.o0 + kr, voff, y0);
        x[r] = y1;
        st_b(ep.ext + kr, voff, csub63(mont_mul<SP>(y1, mi.r2, mi), mi.q));  // sigma(c1) R
      }
    } else if constexpr (is_ksp(EPI)) {
      // acc_P = sum_j ext_j ksk_j R^-1 (ks_inner_kernel; ext carries R) at the
      // coalesced positions, canonical: the products are below 1.5q (2q
      // generic), the running sum is kept below 2q.  Operands software-
      // pipelined PD elements deep (as EPI_KSQ)
      constexpr int KD = ksp_digits(EPI);
      constexpr int PD = SP ? KSP_PD : 1;
      u64 nq1 = 0 - mi.q, nq2 = 0 - 2 * mi.q;
      asm("" : "+s"(nq1));
      asm("" : "+s"(nq2));
      u64 ek[PD + 1][2 * KD];
#pragma unroll
      for (int r = 0; r < PD; ++r) {
        const u32 kr = GZ::k_reg(r);
#pragma unroll
        for (int j = 0; j < KD; ++j) {
          ek[r][j] = ld_b(ep.kext + j * ep.ext_j + kr, voff);
          ek[r][KD + j] = ld_b(ep.kksk + j * ep.ksk_j + kr, voff);
        }
      }
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if (r + PD < R) {
          const u32 kn = GZ::k_reg(r + PD);
#pragma unroll
          for (int j = 0; j < KD; ++j) {
            ek[(r + PD) % (PD + 1)][j] = ld_b(ep.kext + j * ep.ext_j + kn, voff);
            ek[(r + PD) % (PD + 1)][KD + j] = ld_b(ep.kksk + j * ep.ksk_j + kn, voff);
          }
        }
        u64 e[KD], k[KD], pr[KD];
#pragma unroll
        for (int j = 0; j < KD; ++j) {
          e[j] = ek[r % (PD + 1)][j];
          k[j] = ek[r % (PD + 1)][KD + j];
        }
        if constexpr (SP) {
          mont_mul_sp_vec<KD>(pr, e, k, mi.q_hi);
        } else if constexpr (GEN_VEC) {
          mont_mul_gen_vec<KD>(pr, e, k, mi);
        } else {
#pragma unroll
          for (int j = 0; j < KD; ++j) pr[j] = mont_mul<SP>(e[j], k[j], mi);
        }
        u64 acc = pr[0];
#pragma unroll
        for (int j = 1; j < KD; ++j) acc = harvey_csub(acc + pr[j], nq2);
        x[r] = harvey_csub(acc, nq1);
      }
    } else {
#pragma unroll
      for (int r = 0; r < R; ++r) x[r] = ld_d(data + GZ::k_reg(r), voff);
    }
    const u32 lw = lds_idx<S>(w, GZ::k_thr(ts));
#pragma unroll
    for (int r = 0; r < R; ++r) lds[lw + GZ::k_reg(r) + (GZ::k_reg(r) >> 4)] = x[r];
    __syncthreads();
    using GF = Grp<S, LOGR, G0>;
    const u32 lr = lds_idx<S>(w, GF::k_thr(ts));
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const u32 kr = GF::k_reg(r);
      x[r] = lds[lr + kr + (kr >> 4)];
    }
  } else {
    using GF = Grp<S, LOGR, G0>;
    voff = (gb + (GF::k_thr(ts) << PG::LS)) << 3;
    if constexpr (is_conv(EPI)) {
      // the base conversion (conv_apply, oracle) of this element from the NS
      // source limbs at the same position, 4 elements at a time (NS is a
      // template parameter: no per-term predication)
      constexpr int NS = conv_ns(EPI);
      constexpr size_t NW = (size_t)1 << LOG_N;
      u32 hc0[NS], hc1[NS];  // the constants' 31-bit digits (uniform, SGPRs)
#pragma unroll
      for (int i = 0; i < NS; ++i) split31(ep.h[i], hc0[i], hc1[i]);
#pragma unroll
      for (int c0 = 0; c0 < R; c0 += 4) {
        u64 sv[4][NS];
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int i = 0; i < NS; ++i)
            sv[j][i] = ld_b(ep.src + i * NW + ((size_t)GF::k_reg(c0 + j) << PG::LS), voff);
#pragma unroll
        for (int j = 0; j < 4; ++j)
          x[c0 + j] = CONV_COLS && SP && WIDE && CONV_SP60 ? dot_cols_sp60<NS>(sv[j], hc0, hc1, mi.q_hi)  // < 2q
                      : CONV_COLS ? dot_cols<NS, SP>(sv[j], hc0, hc1, mi)                                  // < 2q
                                  : dot_mont_lazy<NS, SP, WIDE>(sv[j], ep.h, 1, NS, mi);                   // < 4q
      }
    } else {
      // the first forward pass may read out of place (NttArgs::src)
      const u64 *din = data;
      if constexpr (!INV && PG::S0 == 0)
        if (a.src) din = a.src + (data - a.map.base);
#pragma unroll
      for (int r = 0; r < R; ++r) x[r] = ld_d(din + ((size_t)GF::k_reg(r) << PG::LS), voff);
    }
  }
  // the final store uses the group-0 layout for row passes and the last
  // group's layout for column passes; recompute the offset for the latter
  if constexpr (COLS) {
    constexpr int GL = INV ? 0 : NG - 1;
    voff = (gb + (Grp<S, LOGR, GL>::k_thr(ts) << PG::LS)) << 3;
  } else {
    voff = (gb + Grp<S, LOGR, 0>::k_thr(ts)) << 3;
  }
  group_loop<LOG_N, S, LOGR, W, INV, COLS, SP, WIDE, EPI, 0>(x, tc, lds, tw, data, voff, w, ts, hi, a, mi, mod, ep);
}

#ifndef NTT_MINW
#define NTT_MINW 1
#endif
// WM (forward passes): the lazy schedule of the launch's moduli, chosen on the
// host (wide_mode): 1 all WIDE (q < 2^60), 0 all narrow, 2 mixed (a per-
// workgroup branch between both; the kernel then carries both code paths and
// needs ~150 VGPRs instead of ~90, i.e. 3 waves per SIMD instead of the 4 the
// LDS allows: a launch over one modulus class avoids it)
template <int LOG_N, int S, int LOGR, int W, bool INV, bool COLS, bool SP, int EPI, int WM>
__global__ void __launch_bounds__(W << (S - LOGR), (W << (S - LOGR)) == 256 ? NTT_MINW : 1) ntt_pass(NttArgs a) {
  static_assert(is_combine(EPI) || EPI == EPI_NONE || EPI == PRO_TENSOR || EPI == PRO_AUTOMORPH ||
                    EPI == PRO_BFVT || is_conv(EPI) || is_ksp(EPI),
                "ntt_pass epilogues");
  static_assert(!is_conv(EPI) || (!INV && COLS), "the conversion prologue feeds a forward column pass");
  static_assert(!is_combine(EPI) || (!INV && !COLS), "epilogues follow a forward row pass");
  static_assert((EPI != PRO_TENSOR && EPI != PRO_AUTOMORPH && EPI != PRO_BFVT && !is_ksp(EPI)) || (INV && !COLS),
                "prologues feed an inverse row pass");
  using PG = PassGeo<LOG_N, S, COLS, INV>;
  static_assert(!is_combine(EPI) || PG::LAST, "epilogues run in the last pass");
  constexpr int T = 1 << (S - LOGR);
  static_assert(LOGR == 4, "register tile is 16 words");
  extern __shared__ u64 lds[];

  // (poly, limb) come from gridDim.y / gridDim.z, so every per-workgroup
  // quantity is scalar (SGPR) and element addresses are 32-bit offsets from a
  // scalar base (global_load ... saddr): no 64-bit VALU address arithmetic
  const u32 tid = threadIdx.x;
  u32 bx = blockIdx.x, poly = blockIdx.y, act = blockIdx.z;
  if constexpr (EPI == EPI_NONE) {
    // every block of one job (poly, limb) on ONE XCD (ids are dealt
    // round-robin over the 8 XCDs), jobs still in dispatch order: the blocks'
    // row segments of one residue meet in one L2 (forward launch 2.07 ->
    // 2.01 ms, profiles/r03/ab_xcd_job.txt)
    const u32 nj = gridDim.y * gridDim.z;
    if ((nj & 7) == 0) {
      const u32 lin = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
      const u32 r = lin >> 3;
      bx = r % gridDim.x;
      const u32 j = (r / gridDim.x) * 8 + (lin & 7);
      poly = j % gridDim.y;
      act = j / gridDim.y;
    }
  }
  if constexpr (is_ksq(EPI) || is_ksp(EPI)) {
    // the 2 n polys (ct, b) of one (limb, row block) on consecutive workgroup
    // ids of ONE XCD: the limb's key rows (2 dnum of them) stay in that XCD's
    // L2 for the whole batch, and the b = 1 item re-reads the ext rows the
    // b = 0 item just fetched
    // GI groups are interleaved per XCD (their key rows all L2-resident)
    constexpr u32 GIW = is_ksq(EPI) ? KSQ_GI : KSP_GI;
    const u32 np = gridDim.y, lin = blockIdx.x + gridDim.x * (blockIdx.y + np * blockIdx.z);
    const u32 r = lin >> 3, gpx = gridDim.x * gridDim.z / 8;  // groups per XCD
    const u32 GI = gpx % GIW == 0 ? GIW : 1;
    const u32 within = r % (GI * np);
    const u32 g = ((r / (GI * np)) * GI + within % GI) * 8 + (lin & 7);  // g = (limb, row block)
    poly = within / GI;
    bx = g % gridDim.x;
    act = g / gridDim.x;
  }
  if constexpr (is_conv(EPI)) {
    // the T target limbs of one source block (poly, column block) run on
    // consecutive workgroup ids of ONE XCD (ids are dealt round-robin over the
    // 8 XCDs), so the ns source limbs come from that XCD's L2 after the first
    // read instead of being re-fetched from HBM once per target
    const u32 cbs = gridDim.x, T = gridDim.z, nsb = gridDim.x * gridDim.y;
    const u32 lin = blockIdx.x + cbs * (blockIdx.y + gridDim.y * blockIdx.z);
    u32 sb;
    if ((nsb & 7) == 0) {
      const u32 rest = lin >> 3;
      act = rest % T;
      sb = (rest / T) * 8 + (lin & 7);
    } else {
      act = lin % T;
      sb = lin / T;
    }
    bx = sb % cbs;
    poly = sb / cbs;
  }
  const u32 limb = limbmap_limb(a.map, act);
  const u32 mod = a.map.mod_offset + limb;
  u64 *data = a.map.base + (((size_t)poly * a.map.poly_stride + limb) << LOG_N);
  const ModInfo mi = a.mods[mod];
  const u64 *tw = a.tw + ((size_t)mod << LOG_N);
  constexpr u32 stride = 1u << PG::LS;

  // column passes put the W sub-transforms (adjacent columns) on adjacent
  // lanes: every wave access is four 128 B row segments
  u32 w, ts;
  if (COLS) { w = tid % W; ts = tid / W; } else { ts = tid % T; w = tid / T; }
  const u32 u = bx * W + w;
  const u32 hi = u >> PG::LS;
  const u32 gb = (hi << (S + PG::LS)) + (u & (stride - 1));

  EpiRow ep{};
  if constexpr (is_ksp(EPI)) {
    const size_t N = (size_t)1 << LOG_N;
    ep.ext_j = (size_t)a.e_QP * N;
    ep.ksk_j = 2 * ep.ext_j;
    ep.kext = a.e_ext + ((size_t)(poly >> 1) * a.e_ndig * a.e_QP + limb) * N;
    ep.kksk = a.e_ksk + ((size_t)(poly & 1) * a.e_QP + limb) * N;
  }
  if constexpr (is_combine(EPI)) {
    if constexpr (is_ksq(EPI)) {
      const size_t N = (size_t)1 << LOG_N;
      ep.ext_j = (size_t)a.e_QP * N;
      ep.ksk_j = 2 * ep.ext_j;
      ep.kext = a.e_ext + ((size_t)(poly >> 1) * a.e_ndig * a.e_QP + limb) * N;
      ep.kksk = a.e_ksk + ((size_t)(poly & 1) * a.e_QP + limb) * N;
    }
    ep.acc = a.e_acc + (((size_t)poly * a.e_acc_stride + limb) << LOG_N);
    ep.base = a.e_base + (((size_t)poly * a.map.poly_stride + limb) << LOG_N);
    ep.out = a.e_out + (((size_t)poly * a.map.poly_stride + limb) << LOG_N);
    ep.pinv = a.e_pinv[limb];
    ep.add = (a.e_add_mask >> (poly & 1)) & 1;
    ep.g = a.e_g;
  }
  if constexpr (EPI == PRO_TENSOR) {
    const size_t LN = (size_t)a.t_L << LOG_N;
    const size_t o = ((size_t)poly * 2 * a.t_L + limb) << LOG_N;
    ep.a0 = a.t_a + o;
    ep.a1 = ep.a0 + LN;
    ep.b0 = a.t_b + o;
    ep.b1 = ep.b0 + LN;
    ep.o0 = a.t_out + o;
    ep.o1 = ep.o0 + LN;
    ep.ext = a.t_ext + (((size_t)(poly * a.t_ndig + limb / a.t_alpha) * a.t_QP + limb) << LOG_N);
  }
  if constexpr (EPI == PRO_BFVT) {
    // poly = 3 ct + e; the inputs are t_a, t_b [ct][2][nl][N] = (a0, a1), (b0, b1)
    const size_t LN = (size_t)a.t_L << LOG_N;
    const size_t o = ((size_t)(poly / 3) * 2 * a.t_L + limb) << LOG_N;
    const u64 *xa = a.t_a + o, *xb = a.t_b + o;
    ep.e = poly % 3;
    ep.a0 = ep.e == 2 ? xa + LN : xa;
    ep.a1 = xa + LN;
    ep.b0 = ep.e == 2 ? xb + LN : xb;
    ep.b1 = xb + LN;
  }
  if constexpr (EPI == PRO_AUTOMORPH) {
    const size_t LN = (size_t)a.t_L << LOG_N;
    const size_t o = ((size_t)poly * 2 * a.t_L + limb) << LOG_N;
    ep.a0 = a.t_a + o;
    ep.a1 = ep.a0 + LN;
    ep.o0 = a.t_out ? a.t_out + o : nullptr;
    ep.ext = a.t_ext + (((size_t)(poly * a.t_ndig + limb / a.t_alpha) * a.t_QP + limb) << LOG_N);
    ep.g = a.t_g;
  }
  if constexpr (is_conv(EPI)) {
    ep.src = a.c_src + (((size_t)poly * a.c_src_stride + a.c_src_first) << LOG_N);
#pragma unroll
    for (int i = 0; i < conv_ns(EPI); ++i) ep.h[i] = a.c_h[(size_t)i * a.c_nd + act];
  }
  if constexpr (!INV && WM == 2) {
    // WIDE lazy schedule for moduli below 2^60 (per-workgroup uniform branch)
    if (mi.q < (1ull << 60)) {
      pass_body<LOG_N, S, LOGR, W, INV, COLS, SP, true, EPI>(a, lds, data, tw, mi, mod, w, ts, hi, gb, ep);
      return;
    }
  }
  pass_body<LOG_N, S, LOGR, W, INV, COLS, SP, !INV && WM == 1, EPI>(a, lds, data, tw, mi, mod, w, ts, hi, gb, ep);
}

// lazy-schedule class of the moduli a launch over map m touches (ntt_pass WM)
int wide_mode(const fhe_ctx *c, const LimbMap &m) {
  bool wide = false, narrow = false;
  for (u32 act = 0; act < m.cnt; ++act) {
    const u64 q = c->moduli[m.mod_offset + limbmap_limb(m, act)];
    (q < (1ull << 60) ? wide : narrow) = true;
  }
  return wide && narrow ? 2 : wide ? 1 : 0;
}

template <int LOG_N, int S, int W, bool COLS, bool INV, bool SP, int EPI, int WM = 0>
int launch_one(fhe_ctx *c, const NttArgs &a, u32 n_jobs) {
  constexpr int LOGR = 4;
  constexpr int NT = W << (S - LOGR);
  constexpr size_t lds = lds_bytes<S, W>();
  constexpr u32 subs = 1u << (LOG_N - S);
  // dispatch order: row blocks, then polys, then limbs -- the resident
  // workgroups share one modulus, so its twiddle table stays in L2
  dim3 grid(subs / W, n_jobs / a.map.cnt, a.map.cnt);
  auto k = ntt_pass<LOG_N, S, LOGR, W, INV, COLS, SP, EPI, WM>;
  if (lds > 64 * 1024) (void)hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(k, grid, dim3(NT), lds, c->stream, a);
  return fhe_check(c, hipGetLastError(), "ntt_pass launch");
}

// a forward pass, with the lazy schedule class of its moduli
template <int LOG_N, int S, int W, bool COLS, int EPI, bool SP>
int launch_fwd(fhe_ctx *c, const NttArgs &a, u32 n_jobs) {
  switch (wide_mode(c, a.map)) {
    case 1: return launch_one<LOG_N, S, W, COLS, false, SP, EPI, 1>(c, a, n_jobs);
    case 0: return launch_one<LOG_N, S, W, COLS, false, SP, EPI, 0>(c, a, n_jobs);
  }
  return launch_one<LOG_N, S, W, COLS, false, SP, EPI, 2>(c, a, n_jobs);
}

template <int LOG_N, int S, int W, bool COLS, int EPI = EPI_NONE>
int launch_pass(fhe_ctx *c, const NttArgs &a, bool inv, u32 n_jobs) {
  if constexpr (is_combine(EPI) || is_conv(EPI)) {
    if (inv) return fhe_fail(c, FHE_ERR_INVALID, "ntt epilogue on an inverse pass");
    return c->special ? launch_fwd<LOG_N, S, W, COLS, EPI, true>(c, a, n_jobs)
                      : launch_fwd<LOG_N, S, W, COLS, EPI, false>(c, a, n_jobs);
  } else if constexpr (EPI == PRO_TENSOR || EPI == PRO_AUTOMORPH || EPI == PRO_BFVT || is_ksp(EPI)) {
    if (!inv) return fhe_fail(c, FHE_ERR_INVALID, "prologue on a forward pass");
    return c->special ? launch_one<LOG_N, S, W, COLS, true, true, EPI>(c, a, n_jobs)
                      : launch_one<LOG_N, S, W, COLS, true, false, EPI>(c, a, n_jobs);
  } else {
    if (c->special)
      return inv ? launch_one<LOG_N, S, W, COLS, true, true, EPI>(c, a, n_jobs)
                 : launch_fwd<LOG_N, S, W, COLS, EPI, true>(c, a, n_jobs);
    return inv ? launch_one<LOG_N, S, W, COLS, true, false, EPI>(c, a, n_jobs)
               : launch_fwd<LOG_N, S, W, COLS, EPI, false>(c, a, n_jobs);
  }
}

// one pass over a whole residue (N <= 2^14)
template <int EPI = EPI_NONE>
int single_pass(fhe_ctx *c, const NttArgs &a, bool inv, u32 n_jobs) {
  switch (a.log_n) {
    case 10: return launch_pass<10, 10, 1, false, EPI>(c, a, inv, n_jobs);
    case 11: return launch_pass<11, 11, 1, false, EPI>(c, a, inv, n_jobs);
    case 12: return launch_pass<12, 12, 1, false, EPI>(c, a, inv, n_jobs);
    case 13: return launch_pass<13, 13, 1, false, EPI>(c, a, inv, n_jobs);
    case 14: return launch_pass<14, 14, 1, false, EPI>(c, a, inv, n_jobs);
  }
  return fhe_fail(c, FHE_ERR_UNSUPPORTED, "single_pass: log_n");
}

// column pass: stages [0, S1), stride N >> S1
template <int EPI = EPI_NONE>
int col_pass(fhe_ctx *c, const NttArgs &a, bool inv, u32 n_jobs) {
  if constexpr (EPI == EPI_NONE)
    if (a.log_n == 14) return launch_pass<14, 7, 32, true, EPI>(c, a, inv, n_jobs);
  switch (a.log_n) {
    case 15: return launch_pass<15, 7, 32, true, EPI>(c, a, inv, n_jobs);
    case 16: return launch_pass<16, 8, 16, true, EPI>(c, a, inv, n_jobs);
    case 17: return launch_pass<17, 8, 16, true, EPI>(c, a, inv, n_jobs);
  }
  return fhe_fail(c, FHE_ERR_UNSUPPORTED, "col_pass: log_n");
}

// row pass: stages [S1, logN), contiguous blocks
template <int EPI = EPI_NONE>
int row_pass(fhe_ctx *c, const NttArgs &a, bool inv, u32 n_jobs) {
  if constexpr (EPI == EPI_NONE)
    if (a.log_n == 14) return launch_pass<14, 7, 32, false, EPI>(c, a, inv, n_jobs);
  switch (a.log_n) {
    case 15: return launch_pass<15, 8, 16, false, EPI>(c, a, inv, n_jobs);
    case 16: return launch_pass<16, 8, 16, false, EPI>(c, a, inv, n_jobs);
    case 17: return launch_pass<17, 9, 8, false, EPI>(c, a, inv, n_jobs);
  }
  return fhe_fail(c, FHE_ERR_UNSUPPORTED, "row_pass: log_n");
}

// the forward column pass with the conversion prologue over a.c_ns sources
int conv_col_pass(fhe_ctx *c, const NttArgs &a, u32 n_jobs) {
  switch (a.c_ns) {
    case 1: return col_pass<PRO_CONV>(c, a, false, n_jobs);
    case 2: return col_pass<PRO_CONV + 1>(c, a, false, n_jobs);
    case 3: return col_pass<PRO_CONV + 2>(c, a, false, n_jobs);
    case 4: return col_pass<PRO_CONV + 3>(c, a, false, n_jobs);
  }
  return fhe_fail(c, FHE_ERR_UNSUPPORTED, "conversion prologue: 1..4 source limbs");
}

}  // namespace

int ntt_launch(fhe_ctx *c, const LimbMap &m, bool inverse, bool noscale, bool lazy_out, const u64 *scale,
               const u64 *src) {
  const u32 n_jobs = m.n_polys * m.cnt;
  if (n_jobs == 0) return FHE_OK;
  if (inverse && src) return fhe_fail(c, FHE_ERR_INVALID, "out-of-place inverse NTT");
  if (m.n_polys > 65535u) {
    // split along polys to respect gridDim.y
    const u32 per = 65535u;
    for (u32 p0 = 0; p0 < m.n_polys; p0 += per) {
      LimbMap sub = m;
      const size_t off = (size_t)p0 * m.poly_stride * c->n;
      sub.base = m.base + off;
      sub.n_polys = (m.n_polys - p0) < per ? (m.n_polys - p0) : per;
      int rc = ntt_launch(c, sub, inverse, noscale, lazy_out, scale, src ? src + off : nullptr);
      if (rc) return rc;
    }
    return FHE_OK;
  }
  NttArgs a{};
  a.map = m;
  a.tw = inverse ? c->d_tw_inv : c->d_tw_fwd;
  a.mods = c->d_mods;
  a.ninv = c->d_ninv;
  a.log_n = c->log_n;
  a.noscale = inverse && noscale;
  a.scale = inverse ? scale : nullptr;
  a.lazy_out = !inverse && lazy_out;
  a.src = src;
  // N = 2^14: two passes of 7 stages with 32 sub-transforms per workgroup (35 KiB
  // of LDS, 4 workgroups per CU) instead of one pass per residue (128 KiB,
  // one workgroup of 16 waves per CU)
  if (c->log_n <= 13) return single_pass(c, a, inverse, n_jobs);
  int rc;
  if (!inverse) {
    rc = col_pass(c, a, false, n_jobs);
    if (rc) return rc;
    a.src = nullptr;  // the row pass works in place on the column pass's output
    return row_pass(c, a, false, n_jobs);
  }
  rc = row_pass(c, a, true, n_jobs);
  if (rc) return rc;
  return col_pass(c, a, true, n_jobs);
}

// Forward NTT of the ModDown conversion conv (all L limbs of 2n polys) with
// the ModDown finish fused into its last pass (EPI_COMBINE):
//   out[p][i] = (add_mask bit (p & 1) ? base[p][i] : 0) + (acc[p][i] - NTT(conv)[p][i]) P^-1  mod q_i
// conv is transformed in place by the first pass only; acc rows have stride acc_stride limbs.
// With ext (EPI_KSQ, two-pass sizes) acc's Q limbs are not read: the last pass
// forms acc[2 ct + b][i] = sum_j ext[ct][j][i] ksk[j][b][i] R^-1 itself.
int ntt_fwd_combine_launch(fhe_ctx *c, u64 *conv, u32 n_polys, const u64 *acc, u32 acc_stride, const u64 *base,
                           u64 *out, u32 add_mask, const ConvTab *pro, const u64 *ext, const u64 *ksk, u32 ndig,
                           u32 base_g) {
  const u32 L = c->L, QP = c->L + c->K;
  const size_t N = c->n;
  if (ext && (c->log_n <= 14 || ndig > 4 || (n_polys & 1)))
    return fhe_fail(c, FHE_ERR_UNSUPPORTED, "fused key-switch inner product: log_n / digits");
  if (base_g && c->log_n <= 14) return fhe_fail(c, FHE_ERR_UNSUPPORTED, "rotated combine base: log_n");
  const u32 per = COMBINE_CHUNK;  // polys per pass pair: gridDim.y, even (the polys of a ciphertext stay together)
  for (u32 p0 = 0; p0 < n_polys; p0 += per) {
    const u32 np = std::min(per, n_polys - p0);
    NttArgs a{};
    a.map = LimbMap{conv + (size_t)p0 * L * N, L, L, 0, L, 0, 0, np};
    a.tw = c->d_tw_fwd;
    a.mods = c->d_mods;
    a.ninv = c->d_ninv;
    a.log_n = c->log_n;
    a.e_acc = acc + (size_t)p0 * acc_stride * N;
    a.e_base = base + (size_t)p0 * L * N;
    a.e_out = out + (size_t)p0 * L * N;
    a.e_pinv = c->d_pinv;
    a.e_acc_stride = acc_stride;
    a.e_add_mask = add_mask;
    a.e_g = base_g & ((2u << c->log_n) - 1);
    if (ext) {
      a.e_ext = ext + (size_t)(p0 / 2) * ndig * QP * N;
      a.e_ksk = ksk;
      a.e_ndig = ndig;
      a.e_QP = QP;
    }
    const u32 n_jobs = np * L;
    int rc;
    if (c->log_n <= 14) {
      rc = single_pass<EPI_COMBINE>(c, a, false, n_jobs);
    } else {
      if (pro) {
        // the ModDown conversion P -> Q as the column pass's prologue: the
        // sources are acc's P limbs, already scaled by the INTT (d_iscale)
        a.c_src = acc + (size_t)p0 * acc_stride * N;
        a.c_src_stride = acc_stride;
        a.c_src_first = L;
        a.c_ns = pro->ns;
        a.c_nd = pro->nd;
        a.c_h = pro->h;
        rc = conv_col_pass(c, a, n_jobs);
      } else {
        rc = col_pass(c, a, false, n_jobs);
      }
      if (rc) return rc;
      switch (ext ? ndig : 0) {
        case 1: rc = row_pass<EPI_KSQ>(c, a, false, n_jobs); break;
        case 2: rc = row_pass<EPI_KSQ + 1>(c, a, false, n_jobs); break;
        case 3: rc = row_pass<EPI_KSQ + 2>(c, a, false, n_jobs); break;
        case 4: rc = row_pass<EPI_KSQ + 3>(c, a, false, n_jobs); break;
        default: rc = row_pass<EPI_COMBINE>(c, a, false, n_jobs);
      }
    }
    if (rc) return rc;
  }
  return FHE_OK;
}

// ModUp of digit j fused into the forward NTT of its converted limbs: the
// column pass computes each target limb's conversion y_m = sum_i v_i h[i][m]
// from the digit's source limbs v_i of dc (canonical, already scaled by the
// INTT through d_iscale) as its prologue (PRO_CONV), so the converted limbs
// never make an HBM round trip; the row pass leaves lazy outputs (< 8q) for
// the inner product on special moduli, as keyswitch_run's separate NTT does.
int ntt_fwd_modup_launch(fhe_ctx *c, const u64 *dc, u64 *ext, u32 n, u32 ndig, u32 j) {
  const u32 L = c->L, QP = c->L + c->K, N = c->n;
  const u32 lo = j * c->alpha, hi = std::min(lo + c->alpha, L);
  const ConvTab &tab = c->modup_tabs[j];
  if (c->log_n <= 14 || tab.ns > 4) return fhe_fail(c, FHE_ERR_UNSUPPORTED, "fused ModUp: log_n / digit size");
  const u32 per = 65535u;  // gridDim.y
  for (u32 p0 = 0; p0 < n; p0 += per) {
    const u32 np = std::min(per, n - p0);
    NttArgs a{};
    a.map = LimbMap{ext + ((size_t)p0 * ndig + j) * QP * N, ndig * QP, QP - (hi - lo), 0, lo, hi - lo, 0, np};
    a.tw = c->d_tw_fwd;
    a.mods = c->d_mods;
    a.ninv = c->d_ninv;
    a.log_n = c->log_n;
    a.lazy_out = c->special;
    a.c_src = dc + (size_t)p0 * L * N;
    a.c_src_stride = L;
    a.c_src_first = lo;
    a.c_ns = tab.ns;
    a.c_nd = tab.nd;
    a.c_h = tab.h;
    const u32 n_jobs = np * a.map.cnt;
    // one launch per modulus class where that splits the targets into a Q part
    // and a P part of one class each (ntt_pass WM: a kernel carrying both lazy
    // schedules needs 150-160 VGPRs, 3 waves per SIMD); the P part's targets
    // start at column L - alpha of the conversion table
    NttArgs aq = a, ap = a;
    aq.map = LimbMap{a.map.base, a.map.poly_stride, L - (hi - lo), 0, lo, hi - lo, 0, np};
    ap.map = LimbMap{a.map.base, a.map.poly_stride, c->K, L, c->K, 0, 0, np};
    ap.c_h = tab.h + (L - (hi - lo));
    const int wq = wide_mode(c, aq.map), wp = wide_mode(c, ap.map);
    int rc;
    if (wq != 2 && wp != 2 && wq != wp && aq.map.cnt && ap.map.cnt) {
#if MODUP_COL_SPLIT
      if ((rc = conv_col_pass(c, aq, np * aq.map.cnt))) return rc;
      if ((rc = conv_col_pass(c, ap, np * ap.map.cnt))) return rc;
#else
      if ((rc = conv_col_pass(c, a, n_jobs))) return rc;
#endif
      if ((rc = row_pass(c, aq, false, np * aq.map.cnt))) return rc;
      rc = row_pass(c, ap, false, np * ap.map.cnt);
    } else {
      if ((rc = conv_col_pass(c, a, n_jobs))) return rc;
      rc = row_pass(c, a, false, n_jobs);
    }
    if (rc) return rc;
  }
  return FHE_OK;
}

// CKKS mul+relin front end: the tensor product fused into the first pass of
// the inverse NTT of d2 (PRO_TENSOR).  a, b, out: [n][2][L][N] (out may alias
// a or b); dc [n][L][N] receives INTT(d2); ext's own-digit slots receive d2 R.
int ntt_inv_tensor_launch(fhe_ctx *c, const u64 *a, const u64 *b, u64 *out, u64 *dc, u64 *ext, u32 n, u32 ndig) {
  const u32 L = c->L, QP = c->L + c->K;
  const size_t N = c->n;
  const u32 per = TENSOR_CHUNK;  // ciphertexts per pass pair (gridDim.y <= 65535)
  for (u32 p0 = 0; p0 < n; p0 += per) {
    const u32 np = std::min(per, n - p0);
    NttArgs t{};
    t.map = LimbMap{dc + (size_t)p0 * L * N, L, L, 0, L, 0, 0, np};
    t.tw = c->d_tw_inv;
    t.mods = c->d_mods;
    t.ninv = c->d_ninv;
    t.log_n = c->log_n;
    t.t_a = a + (size_t)p0 * 2 * L * N;
    t.t_b = b + (size_t)p0 * 2 * L * N;
    t.t_out = out + (size_t)p0 * 2 * L * N;
    t.t_ext = ext + (size_t)p0 * ndig * QP * N;
    t.t_L = L;
    t.t_QP = QP;
    t.t_alpha = c->alpha;
    t.t_ndig = ndig;
    // dc feeds ModUp only: its per-source constants (N^-1 folded in) ride on
    // this INTT when ModUp is fused into the next NTT, else N^-1 is skipped
    if (c->fuse_modup) t.scale = c->d_iscale;
    else t.noscale = c->fold_ninv;
    const u32 n_jobs = np * L;
    int rc;
    if (c->log_n <= 14) {
      rc = single_pass<PRO_TENSOR>(c, t, true, n_jobs);
    } else {
      if ((rc = row_pass<PRO_TENSOR>(c, t, true, n_jobs))) return rc;
      rc = col_pass(c, t, true, n_jobs);
    }
    if (rc) return rc;
  }
  return FHE_OK;
}

// CKKS rotation front end: the NTT-domain automorphism sigma_g (and the KS
// preparation of sigma_g(c1)) fused into the first pass of its inverse NTT
// (PRO_AUTOMORPH).  ct [n][2][L][N] must not alias base; base[ct][0] receives
// sigma_g(c0), dc INTT(sigma_g(c1)), ext's own-digit slots sigma_g(c1) R.
int ntt_inv_automorph_launch(fhe_ctx *c, const u64 *ct, u32 g, u64 *base, u64 *dc, u64 *ext, u32 n, u32 ndig) {
  const u32 L = c->L, QP = c->L + c->K;
  const size_t N = c->n;
  if (c->log_n <= 14) return fhe_fail(c, FHE_ERR_UNSUPPORTED, "automorphism prologue: log_n");
  const u32 per = 65535u;  // gridDim.y
  for (u32 p0 = 0; p0 < n; p0 += per) {
    const u32 np = std::min(per, n - p0);
    NttArgs t{};
    t.map = LimbMap{dc + (size_t)p0 * L * N, L, L, 0, L, 0, 0, np};
    t.tw = c->d_tw_inv;
    t.mods = c->d_mods;
    t.ninv = c->d_ninv;
    t.log_n = c->log_n;
    t.t_a = ct + (size_t)p0 * 2 * L * N;
    t.t_out = base ? base + (size_t)p0 * 2 * L * N : nullptr;
    t.t_ext = ext + (size_t)p0 * ndig * QP * N;
    t.t_L = L;
    t.t_QP = QP;
    t.t_alpha = c->alpha;
    t.t_ndig = ndig;
    t.t_g = g & ((2u << c->log_n) - 1);
    if (c->fuse_modup) t.scale = c->d_iscale;  // dc feeds ModUp only (as in ntt_inv_tensor_launch)
    else t.noscale = c->fold_ninv;
    int rc;
    if ((rc = row_pass<PRO_AUTOMORPH>(c, t, true, np * L))) return rc;
    if ((rc = col_pass(c, t, true, np * L))) return rc;
  }
  return FHE_OK;
}

// INTT of the P limbs of the key-switching accumulator acc [2n][QP][N], with
// their inner product acc_P[2 ct + b][k] = sum_j ext[ct][j][k] ksk[j][b][k] R^-1
// (ks_inner_kernel) formed in the first (row) pass (PRO_KSP): acc_P is never
// stored, the P rows of acc receive INTT(acc_P) times d_iscale (ModDown's
// source constants, as ntt_launch(..., d_iscale) gives them)
int ntt_inv_ksp_launch(fhe_ctx *c, u64 *acc, const u64 *ext, const u64 *ksk, u32 n, u32 ndig) {
  const u32 L = c->L, K = c->K, QP = L + K;
  const size_t N = c->n;
  if (c->log_n <= 14 || ndig < 1 || ndig > 4)
    return fhe_fail(c, FHE_ERR_UNSUPPORTED, "fused P-limb inner product: log_n / digits");
  const u32 per = 65534u;  // gridDim.y, even (the polys of a ciphertext stay together)
  for (u32 p0 = 0; p0 < 2 * n; p0 += per) {
    const u32 np = std::min(per, 2 * n - p0);
    NttArgs a{};
    a.map = LimbMap{acc + (size_t)p0 * QP * N, QP, K, L, QP, 0, 0, np};
    a.tw = c->d_tw_inv;
    a.mods = c->d_mods;
    a.ninv = c->d_ninv;
    a.log_n = c->log_n;
    a.scale = c->d_iscale;
    a.e_ext = ext + (size_t)(p0 / 2) * ndig * QP * N;
    a.e_ksk = ksk;
    a.e_ndig = ndig;
    a.e_QP = QP;
    const u32 n_jobs = np * K;
    int rc;
    switch (ndig) {
      case 1: rc = row_pass<PRO_KSP>(c, a, true, n_jobs); break;
      case 2: rc = row_pass<PRO_KSP + 1>(c, a, true, n_jobs); break;
      case 3: rc = row_pass<PRO_KSP + 2>(c, a, true, n_jobs); break;
      default: rc = row_pass<PRO_KSP + 3>(c, a, true, n_jobs); break;
    }
    if (rc) return rc;
    if ((rc = col_pass(c, a, true, n_jobs))) return rc;
  }
  return FHE_OK;
}

// BFV mul+relin: the tensor product of xa = (a0, a1) and xb = (b0, b1), each
// [n][2][nl][N] in NTT form, in the nl-limb base starting at modulus mod_offset, fused into the
// first pass of its inverse NTT (PRO_BFVT); e [n][3][nl][N] receives the
// coefficient-form products WITHOUT the N^-1 factor (behz_floor's constants
// carry it).
int ntt_inv_bfv_tensor_launch(fhe_ctx *c, const u64 *xa, const u64 *xb, u64 *e, u32 nl, u32 mod_offset, u32 n) {
  const size_t N = c->n;
  const u32 per = 65535u;  // gridDim.y, a multiple of 3
  for (u32 p0 = 0; p0 < 3 * n; p0 += per) {
    const u32 np = std::min(per, 3 * n - p0);
    NttArgs t{};
    t.map = LimbMap{e + (size_t)p0 * nl * N, nl, nl, 0, nl, 0, mod_offset, np};
    t.tw = c->d_tw_inv;
    t.mods = c->d_mods;
    t.ninv = c->d_ninv;
    t.log_n = c->log_n;
    t.noscale = 1;
    t.t_a = xa + (size_t)(p0 / 3) * 2 * nl * N;
    t.t_b = xb + (size_t)(p0 / 3) * 2 * nl * N;
    t.t_L = nl;
    const u32 n_jobs = np * nl;
    int rc;
    if (c->log_n <= 14) {
      rc = single_pass<PRO_BFVT>(c, t, true, n_jobs);
    } else {
      if ((rc = row_pass<PRO_BFVT>(c, t, true, n_jobs))) return rc;
      rc = col_pass(c, t, true, n_jobs);
    }
    if (rc) return rc;
  }
  return FHE_OK;
}
