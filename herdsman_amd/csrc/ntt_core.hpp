// ntt_core.hpp -- negacyclic NTT / INTT pass kernels for gfx950 (templates; host entry points in ntt*.hip).
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
#pragma once
#include <algorithm>
#include <type_traits>

#include "context.hpp"

#ifndef KSQT_MINW
#define KSQT_MINW 3  // EPI_KSQT (special moduli) minimum waves per SIMD (4: 128 VGPRs, spills, -1.5%)
#endif
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
  const u64 *e_ta, *e_tb;  // EPI_KSQT: the operands a, b [ct][2][L][N] of the tensor product (the base)
  u32 e_ndig, e_QP;
  u32 e_kQP, e_kshift;  // key rows per digit half; key row of limb i >= L is i + e_kshift (level views)
  u32 e_ext_g;          // EPI_KSQG / PRO_KSPG: ext is read as sigma_g(ext) (hoisted rotation)
  // EPI_KSQG / PRO_KSPG over several Galois elements in one launch (hoisted
  // rotations of few ciphertexts): poly p belongs to rotation r = p / e_rp and
  // ciphertext poly p % e_rp; rotation r's key, element and output replace
  // e_ksk, e_ext_g / e_g and e_out.  e_rp = 0: one rotation.
  u32 e_rp;
  const u64 *e_ksk_r[FHE_ROT_BATCH];
  u64 *e_out_r[FHE_ROT_BATCH];
  u32 e_g_r[FHE_ROT_BATCH];
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
  // one source only (rescale): the central lift of the dropped limb, y - [q_l]_{q_m}
  // where the source word exceeds c_lift_half (0: plain conversion)
  u64 c_lift_half;
  const u64 *c_lift_sub;  // [nd] q_l mod q_m
  // every source modulus is below 2^60: the column sums reduce in place
  // (dot_cols_sp60) for special targets below 2^61 too, not only below 2^60
  u32 c_src60;
};

// The passes shared by several entry points, compiled once (ntt.hip, ntt_conv*.hip):
// plain forward / inverse passes (single = N <= 2^14 one-pass, col, row) and
// the forward column pass with the conversion prologue over a.c_ns sources.
int ntt_single_plain(fhe_ctx *c, const NttArgs &a, bool inv, u32 n_jobs);
int ntt_col_plain(fhe_ctx *c, const NttArgs &a, bool inv, u32 n_jobs);
int ntt_row_plain(fhe_ctx *c, const NttArgs &a, bool inv, u32 n_jobs);
int ntt_conv_col(fhe_ctx *c, const NttArgs &a, u32 n_jobs);
int ntt_conv_col12(fhe_ctx *c, const NttArgs &a, u32 n_jobs);

namespace {



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
// EPI_KSQG / PRO_KSPG + d - 1: the same with the ext words gathered through
// sigma_g (NttArgs::e_ext_g): the inner product of a hoisted rotation, whose
// one ModUp of c1 serves every Galois element
// PRO_TENSOR2 / EPI_KSQT + d - 1: CKKS mul+relin with the tensor product split
// between the two ends of the key switch: the INTT(d2) prologue forms d2 = a1 b1
// only, and the ModDown finish forms its base d0 = a0 b0 (b = 0) or
// d1 = a0 b1 + a1 b0 (b = 1) from a and b itself, and the own digit's ext word
// d2 R as well, so d0, d1 and d2 R never reach HBM
enum { EPI_NONE = 0, EPI_COMBINE = 1, PRO_TENSOR = 2, PRO_AUTOMORPH = 3, PRO_BFVT = 4, PRO_TENSOR2 = 5, EPI_KSQ = 6,
       PRO_CONV = 11, PRO_KSP = 16, EPI_KSQG = 21, PRO_KSPG = 26, EPI_KSQT = 31 };
__host__ __device__ constexpr bool is_tensor(int e) { return e == PRO_TENSOR || e == PRO_TENSOR2; }
__host__ __device__ constexpr bool ksq_tensor(int e) { return e >= EPI_KSQT && e < EPI_KSQT + 4; }
__host__ __device__ constexpr bool is_conv(int e) { return e >= PRO_CONV && e < PRO_CONV + 4; }
__host__ __device__ constexpr int conv_ns(int e) { return e - PRO_CONV + 1; }
__host__ __device__ constexpr bool ksq_gather(int e) { return e >= EPI_KSQG && e < EPI_KSQG + 4; }
__host__ __device__ constexpr bool is_ksq(int e) {
  return (e >= EPI_KSQ && e < EPI_KSQ + 4) || ksq_gather(e) || ksq_tensor(e);
}
__host__ __device__ constexpr int ksq_digits(int e) {
  return e - (ksq_gather(e) ? EPI_KSQG : ksq_tensor(e) ? EPI_KSQT : EPI_KSQ) + 1;
}
__host__ __device__ constexpr bool is_combine(int e) { return e == EPI_COMBINE || is_ksq(e); }
__host__ __device__ constexpr bool ksp_gather(int e) { return e >= PRO_KSPG && e < PRO_KSPG + 4; }
__host__ __device__ constexpr bool is_ksp(int e) { return (e >= PRO_KSP && e < PRO_KSP + 4) || ksp_gather(e); }
__host__ __device__ constexpr int ksp_digits(int e) { return e - (ksp_gather(e) ? PRO_KSPG : PRO_KSP) + 1; }

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
  u32 xg;  // EPI_KSQG / PRO_KSPG: the Galois element ext is gathered through
  u32 e;  // PRO_BFVT: which tensor output (0, 1, 2) this poly is; EPI_KSQT: b
  u32 jown;  // EPI_KSQT: the digit this limb belongs to (its ext word is d2 R, formed here)
  const u64 *src;  // PRO_CONV: source limb 0 of this poly (limb i at src + i N)
  u64 h[4];        // PRO_CONV: h[i][m] of this workgroup's target limb
  u64 lift_sub;    // PRO_CONV, one source, rescale lift: q_l mod q_m
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
#ifndef NTT_NTST
#define NTT_NTST 3  // bit 0: the passes' own data stores non-temporal; bit 1: the fused epilogue/prologue outputs too
#endif
// a pass's own data words (bit 0) and its fused outputs (bit 1) are written once
__device__ __forceinline__ void st_d(u64 *base, u32 off, u64 v) {
  if constexpr (NTT_NTST & 1) __builtin_nontemporal_store(v, (u64 *)((char *)base + off));
  else st_b(base, off, v);
}
__device__ __forceinline__ void st_e(u64 *base, u32 off, u64 v) {
  if constexpr (NTT_NTST & 2) __builtin_nontemporal_store(v, (u64 *)((char *)base + off));
  else st_b(base, off, v);
}
// 16-byte accesses of two adjacent words (PAIR_IO): an L2-served 16-B load per
// lane moves 1.8x the bytes per second of an 8-B one (30-36 against 17-19 TB/s,
// profiles/r05/microbench_stream_l2.txt)
typedef u64 u64x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u64x2 ld2_b(const u64 *base, u32 off) { return *(const u64x2 *)((const char *)base + off); }
__device__ __forceinline__ u64x2 ld2_d(const u64 *base, u32 off) {
  return __builtin_nontemporal_load((const u64x2 *)((const char *)base + off));
}
__device__ __forceinline__ void st2_d(u64 *base, u32 off, u64x2 v) {
  if constexpr (NTT_NTST & 1) __builtin_nontemporal_store(v, (u64x2 *)((char *)base + off));
  else *(u64x2 *)((char *)base + off) = v;
}
__device__ __forceinline__ void st2_e(u64 *base, u32 off, u64x2 v) {
  if constexpr (NTT_NTST & 2) __builtin_nontemporal_store(v, (u64x2 *)((char *)base + off));
  else *(u64x2 *)((char *)base + off) = v;
}

#ifndef LDS_PAD
#define LDS_PAD 1  // 0: unpadded exchange tile (32 KiB at S = 8, W = 16: 5 workgroups per CU, bank conflicts)
#endif
__host__ __device__ constexpr u32 lds_pad(u32 k) { return LDS_PAD ? (k >> 4) : 0; }
template <int S>
__device__ __forceinline__ u32 lds_idx(u32 w, u32 k) {
  constexpr u32 SUB = 1u << S;
  constexpr u32 PAD = SUB + (LDS_PAD ? (SUB >> 4) + 1 : 0);
  return w * PAD + k + lds_pad(k);
}
template <int S, int W>
constexpr size_t lds_bytes() {
  return (size_t)W * ((1u << S) + (LDS_PAD ? (1u << S >> 4) + 1 : 0)) * sizeof(u64);
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

#ifndef PAIR_IO
#define PAIR_IO 1  // 16-byte HBM/L2 accesses on the re-laid-out side of row passes (0: 8-byte, group-0 layout)
#endif
// The HBM-facing layout of the side of a row (or single) pass that goes
// through an LDS re-layout anyway: the forward pass's store and its epilogue
// operands, the inverse pass's load and its prologue operands.  With PAIR_IO,
// thread ts of a T-thread sub-transform owns words 2ts and 2ts + 1 of every
// 2T-word run, so each pair (registers 2j, 2j + 1) is one 16-byte access
// and a wave instruction moves four 256 B segments; else the group-0
// layout (words ts + T r, 8-byte accesses).  Thread and register bits are
// disjoint either way, so the LDS pad splits between them (lds_pad).
template <int S, int LOGR, bool P = PAIR_IO>
struct IoL {
  static constexpr u32 T = 1u << (S - LOGR);
  static constexpr int STEP = P ? 2 : 1;  // words per access
  __device__ static __forceinline__ u32 k_thr(u32 ts) { return P ? ts << 1 : Grp<S, LOGR, 0>::k_thr(ts); }
  static constexpr u32 k_reg(int r) {
    return P ? ((u32)(r & 1) | ((u32)(r >> 1) * 2 * T)) : Grp<S, LOGR, 0>::k_reg(r);
  }
};

// a wave-uniform 64-bit value made visibly uniform (two v_readfirstlane_b32, or
// s_movs when it already lives in SGPRs), so an asm "+s" constraint can pin it
// in SGPRs: without it ROCm 7.2 fails the generic-moduli persistent pass, whose
// unrolled residue loop carries the modulus through a VGPR phi ("illegal VGPR
// to SGPR copy")
__device__ __forceinline__ u64 uniform64(u64 x) {
  const u32 lo = __builtin_amdgcn_readfirstlane((u32)x), hi = __builtin_amdgcn_readfirstlane((u32)(x >> 32));
  return ((u64)hi << 32) | lo;
}

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

// LSW: butterflies per lock-step chunk (all R/2 of a stage by default; the
// persistent single pass, which also holds the next residue, takes 4 so the
// products' temporaries fit beside its second register tile)
template <int S, int LOGR, int G, int S0, bool INV, bool SP, bool WIDE, int LSW = 8>
__device__ __forceinline__ void run_group(u64 (&x)[16], const u64 (&t)[16], u64 q2, const ModInfo &mi) {
  using GP = Grp<S, LOGR, G>;
  constexpr int R = 1 << LOGR;
#pragma unroll
  for (int ti = 0; ti < GP::nb; ++ti) {
    const int tau = INV ? GP::nb - 1 - ti : ti;
    const int half = 1 << (GP::nb - 1 - tau);
    if constexpr (SP || GEN_VEC) {
      // the R/2 butterflies of this stage in lock-step (see mont_mul_sp_vec),
      // CH at a time
      constexpr int H = R / 2, CH = LSW < H ? LSW : H;
      int lo_idx[H], w_idx[H];
      {
        int n = 0;
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const int rb = r & ((1 << GP::nb) - 1), rx = r >> GP::nb;
          if (rb & half) continue;
          lo_idx[n] = r;
          w_idx[n] = GP::slot(tau, rx, rb >> (GP::nb - tau));
          ++n;
        }
      }
      // 64-bit adds of SGPR constants as single v_lshl_add_u64; the butterfly's
      // difference U + 2q - V as v_lshl_add_u64 + v_sub_co_u32 + v_subb_co_u32
      // (round 6: 4 issue slots against 6 for (U + 2q + 1) + ~V; the borrow's
      // VCC hazard costs s_nop wait states, which other waves fill: headline
      // +1.4..2.0%, NTT INV -2.2% on a paired A/B, profiles/r06/ab_bfly_sub.txt)
      const u64 q2u = uniform64(q2);
      u64 nq2 = 0 - q2u, q2c = q2u, nq4 = 0 - 2 * q2u;
      asm("" : "+s"(nq2));
      asm("" : "+s"(q2c));
      asm("" : "+s"(nq4));
      const int gs = S0 + G * LOGR + tau;  // global stage
      const bool red = !WIDE || wide_csub(gs);
#pragma unroll
      for (int c0 = 0; c0 < H; c0 += CH) {
        u64 A[CH], Wt[CH], V[CH], U[CH];
#pragma unroll
        for (int i = 0; i < CH; ++i) {
          const u64 X = x[lo_idx[c0 + i]], Y = x[lo_idx[c0 + i] + half];
          Wt[i] = t[w_idx[c0 + i]];
          if (!INV) {
            U[i] = !red ? X : harvey_csub(X, WIDE ? nq4 : nq2);
            A[i] = Y;
          } else {
            U[i] = harvey_csub(X + Y, nq2);
            A[i] = (X + q2c) - Y;
          }
        }
        if constexpr (SP) mont_mul_sp_vec<CH>(V, A, Wt, mi.q_hi);
        else mont_mul_gen_vec<CH>(V, A, Wt, mi);
#pragma unroll
        for (int i = 0; i < CH; ++i) {
          if (!INV) {
            x[lo_idx[c0 + i]] = U[i] + V[i];
            x[lo_idx[c0 + i] + half] = (U[i] + q2c) - V[i];
          } else {
            x[lo_idx[c0 + i]] = U[i];
            x[lo_idx[c0 + i] + half] = V[i];
          }
        }
      }
      continue;
    }
    // generic moduli: the same lazy schedules (the generic Montgomery product
    // is below 2q and accepts any input below 8q, since 8q^2 < q 2^64)
    const u64 q2u = uniform64(q2);
    u64 nq2 = 0 - q2u, q2c = q2u, nq4 = 0 - 2 * q2u;
    asm("" : "+s"(nq2));
    asm("" : "+s"(q2c));
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
        Y = (uu + q2c) - v;
      } else {
        const u64 uu = X, vv = Y;
        X = harvey_csub(uu + vv, nq2);
        Y = mont_mul<SP>((uu + q2c) - vv, w, mi);
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

#ifndef PERSIST_LSW
#define PERSIST_LSW 2  // lock-step butterflies per chunk in the persistent single pass (run_group LSW)
#endif
// group_loop's hook between a group's twiddle prefetch and its butterflies
// (the persistent single pass loads the next residue there, ResidueFetch)
struct NoFetch {
  template <int GI, int NG>
  __device__ __forceinline__ void issue() {}
};

template <int LOG_N, int S, int LOGR, int W, bool INV, bool COLS, bool SP, bool WIDE, int EPI, int GI,
          class PF = NoFetch>
__device__ __forceinline__ void group_loop(u64 (&x)[16], u64 (&tc)[16], u64 *lds, const u64 *tw, u64 *data,
                                           u32 voff, u32 w, u32 ts, u32 hi, const NttArgs &a,
                                           const ModInfo &mi, u32 mod, const EpiRow &ep, PF &pf) {
  using PG = PassGeo<LOG_N, S, COLS, INV>;
  constexpr int NG = (S + LOGR - 1) / LOGR;
  constexpr int R = 1 << LOGR;
  constexpr int G = INV ? NG - 1 - GI : GI;
  using GP = Grp<S, LOGR, G>;
  const u64 q = mi.q, q2 = 2 * q;
  if constexpr (GI + 1 < NG) {
    constexpr int GN = INV ? NG - 2 - GI : GI + 1;
    // the next group's twiddles are in flight while this group computes; with
    // a residue fetch riding along (ntt_persist) they are loaded after it
    // instead, under the exchange (the second register tile leaves no room)
    constexpr bool TW_AHEAD = std::is_same<PF, NoFetch>::value;
    u64 tn[16];
    if constexpr (TW_AHEAD) Grp<S, LOGR, GN>::template load_tw<PG::S0>(tn, tw, hi, ts);
    pf.template issue<GI, NG>();
    run_group<S, LOGR, G, PG::S0, INV, SP, WIDE, TW_AHEAD ? 8 : PERSIST_LSW>(x, tc, q2, mi);
    if constexpr (!TW_AHEAD) Grp<S, LOGR, GN>::template load_tw<PG::S0>(tn, tw, hi, ts);
    const u32 lw = lds_idx<S>(w, GP::k_thr(ts));
#pragma unroll
    for (int r = 0; r < R; ++r) lds[lw + GP::k_reg(r) + lds_pad(GP::k_reg(r))] = x[r];
    __syncthreads();
    const u32 lr = lds_idx<S>(w, Grp<S, LOGR, GN>::k_thr(ts));
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const u32 kr = Grp<S, LOGR, GN>::k_reg(r);
      x[r] = lds[lr + kr + lds_pad(kr)];
    }
    group_loop<LOG_N, S, LOGR, W, INV, COLS, SP, WIDE, EPI, GI + 1>(x, tn, lds, tw, data, voff, w, ts, hi, a, mi,
                                                                     mod, ep, pf);
  } else {
    // EPI_COMBINE: the epilogue's acc and base words are in flight while the
    // last group computes (the LDS footprint caps occupancy at 4 waves per
    // SIMD, so the 128-VGPR budget has room for them)
    constexpr int RE = is_combine(EPI) ? R : 1;
    constexpr int RB = is_combine(EPI) && !ksq_tensor(EPI) ? R : 1;  // EPI_KSQT forms its base in the store loop
    using IO = IoL<S, LOGR>;
    u64 pa[RE], pb[RB];
    if constexpr (is_combine(EPI)) {
#pragma unroll
      for (int r = 0; r < R; r += IO::STEP) {
        const u32 kr = IO::k_reg(r);
        if constexpr (IO::STEP == 2) {
          if constexpr (EPI == EPI_COMBINE) {
            const u64x2 v = ld2_b(ep.acc + kr, voff);
            pa[r] = v.x, pa[r + 1] = v.y;
          }
          if constexpr (ksq_tensor(EPI)) {
          } else if (!ep.add) {
            pb[r] = pb[r + 1] = 0;
          } else if (ep.g) {  // sigma_g(base): a gather, word by word
            pb[r] = ld_b(ep.base, aut_src<LOG_N>((voff >> 3) + kr, ep.g));
            pb[r + 1] = ld_b(ep.base, aut_src<LOG_N>((voff >> 3) + kr + 1, ep.g));
          } else {
            const u64x2 v = ld2_b(ep.base + kr, voff);
            pb[r] = v.x, pb[r + 1] = v.y;
          }
        } else {
          if constexpr (EPI == EPI_COMBINE) pa[r] = ld_b(ep.acc + kr, voff);
          if constexpr (ksq_tensor(EPI)) {
          } else if (!ep.add) pb[r] = 0;
          else if (ep.g) pb[r] = ld_b(ep.base, aut_src<LOG_N>((voff >> 3) + kr, ep.g));  // sigma_g(base)
          else pb[r] = ld_b(ep.base + kr, voff);
        }
      }
    }
    run_group<S, LOGR, G, PG::S0, INV, SP, WIDE, std::is_same<PF, NoFetch>::value ? 8 : PERSIST_LSW>(x, tc, q2, mi);
    // negated reduction constants pinned in SGPRs, so each conditional
    // subtraction is one v_lshl_add_u64 with a scalar operand (left to itself
    // the compiler forms x - m as a v_subrev_co/v_subb_co borrow chain with
    // s_nop hazard padding)
    const u64 qu = uniform64(q);
    u64 nq1 = 0 - qu, nq2 = 0 - 2 * qu, nq4 = 0 - 4 * qu;
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
      // element) are software-pipelined PD elements (PAIR_IO: PD / 2 pairs)
      // deep, and the first ones' loads are in flight across the re-layout barrier
      constexpr int KD = is_ksq(EPI) ? ksq_digits(EPI) : 1;
      constexpr int PD = is_ksq(EPI) && SP ? KSQ_PD : 1;
      constexpr int ST = IO::STEP, NST = R / ST, PDS = (PD + ST - 1) / ST;
      u64 ek[PDS + 1][2 * KD][ST];
      const auto fetch = [&](int st, u64 (&slot)[2 * KD][ST]) {
        const u32 kr = IO::k_reg(st * ST);
#pragma unroll
        for (int j = 0; j < KD; ++j) {
          if (ksq_tensor(EPI) && j == (int)ep.jown) {
            // EPI_KSQT: the own digit's ext word is formed from a1 b1 (not stored)
          } else if constexpr (ksq_gather(EPI)) {
#pragma unroll
            for (int h = 0; h < ST; ++h)
              slot[j][h] = ld_b(ep.kext + j * ep.ext_j, aut_src<LOG_N>((voff >> 3) + kr + h, ep.xg));
          } else if constexpr (ST == 2) {
            const u64x2 e2 = ld2_b(ep.kext + kr + j * ep.ext_j, voff);
            slot[j][0] = e2.x, slot[j][1] = e2.y;
          } else {
            slot[j][0] = ld_b(ep.kext + kr + j * ep.ext_j, voff);
          }
          if constexpr (ST == 2) {
            const u64x2 k2 = ld2_b(ep.kksk + j * ep.ksk_j + kr, voff);
            slot[KD + j][0] = k2.x, slot[KD + j][1] = k2.y;
          } else {
            slot[KD + j][0] = ld_b(ep.kksk + j * ep.ksk_j + kr, voff);
          }
        }
      };
      // EPI_KSQT: the tensor operands (a0, a1, b0, b1) of the base (d0 for b = 0,
      // d1 for b = 1: TM = 1, 2) and of the own digit's ext word d2 R, loaded in
      // the step that uses them.
      // A ring of them beside the key-switching one took the pass past 128 VGPRs
      // (one step ahead: no faster, profiles/r05/ab_tensor_split.txt).  The b = 1
      // workgroup follows the b = 0 one on the same XCD (the remap in ntt_pass),
      // so its a0, b0 come mostly from L2.
      constexpr int NTO = ksq_tensor(EPI) ? 4 : 1;
      const auto tfetch = [&](auto tm, int st, u64 (&slot)[NTO][ST]) {
        constexpr int TM = decltype(tm)::value;
        if constexpr (TM != 0) {
          const u32 kr = IO::k_reg(st * ST);
          const u64 *src[4] = {ep.a0, ep.a1, ep.b0, ep.b1};
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            if constexpr (ST == 2) {
              const u64x2 v2 = ld2_b(src[i] + kr, voff);
              slot[i][0] = v2.x, slot[i][1] = v2.y;
            } else {
              slot[i][0] = ld_b(src[i] + kr, voff);
            }
          }
        }
      };
      // EPI_KSQT: R^3 mod q (canonical), the own digit's scale
      u64 r3 = 0;
      if constexpr (ksq_tensor(EPI)) r3 = csub(mont_mul<SP>(mi.r2, mi.r2, mi), q);
      const auto store_rows = [&](auto tm) {
        constexpr int TM = decltype(tm)::value;
        if constexpr (is_ksq(EPI)) {
#pragma unroll
          for (int st = 0; st < PDS; ++st) fetch(st, ek[st]);
        }
        // row pass ending in a group whose lanes each own contiguous words:
        // re-layout through LDS so the HBM store is coalesced (the IO layout)
        const u32 lw = lds_idx<S>(w, GP::k_thr(ts));
#pragma unroll
        for (int r = 0; r < R; ++r) lds[lw + GP::k_reg(r) + lds_pad(GP::k_reg(r))] = x[r];
        __syncthreads();
        const u32 lr = lds_idx<S>(w, IO::k_thr(ts));
#pragma unroll
        for (int st = 0; st < NST; ++st) {
          if constexpr (is_ksq(EPI)) {
            if (st + PDS < NST) fetch(st + PDS, ek[(st + PDS) % (PDS + 1)]);
          }
          u64 t[NTO][ST];
          tfetch(tm, st, t);
          u64 o[ST];
#pragma unroll
          for (int h = 0; h < ST; ++h) {
            const int r = st * ST + h;
            const u32 kr = IO::k_reg(r);
            const u64 v = lds[lr + kr + lds_pad(kr)];
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
                u64 e[KD], k[KD], pr[KD];
                u64 eown = 0;
                if constexpr (TM != 0) {
                  // d2 R = (a1 b1 R^-1) R^3 R^-1, below 1.5q (the product takes it lazy)
                  eown = mont_mul<SP>(mont_reduce<SP>(mul128(t[1][h], t[3][h]), mi), r3, mi);
                }
#pragma unroll
                for (int j = 0; j < KD; ++j) {
                  e[j] = TM != 0 && j == (int)ep.jown ? eown : ek[st % (PDS + 1)][j][h];
                  k[j] = ek[st % (PDS + 1)][KD + j][h];
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
              if constexpr (TM != 0) {
                // the base of this poly from the ciphertexts: d0 = a0 b0, d1 = a0 b1 + a1 b0
                u64 bv;
                if constexpr (TM == 1) {
                  bv = mul_mod<SP>(t[0][h], t[2][h], mi);
                } else {
                  U128 sm = mul128(t[0][h], t[3][h]);
                  mac128(sm, t[1][h], t[2][h]);
                  bv = reduce128<SP>(sm, mi);
                }
                ks = add_mod(ks, bv, q);
              } else if (ep.add) {
                ks = add_mod(ks, pb[r], q);
              }
              o[h] = ks;
            } else {
              o[h] = v;
            }
          }
          const u32 ko = IO::k_reg(st * ST);
          if constexpr (ST == 2) {
            if constexpr (is_combine(EPI)) st2_e(ep.out + ko, voff, u64x2{o[0], o[1]});
            else st2_d(data + ko, voff, u64x2{o[0], o[1]});
          } else {
            if constexpr (is_combine(EPI)) st_e(ep.out + ko, voff, o[0]);
            else st_d(data + ko, voff, o[0]);
          }
        }
      };
      using T0 = std::integral_constant<int, 0>;
      if constexpr (ksq_tensor(EPI)) {
        if (ep.e == 0) store_rows(std::integral_constant<int, 1>{});
        else store_rows(std::integral_constant<int, 2>{});
      } else {
        store_rows(T0{});
      }
    } else {
      static_assert(!is_combine(EPI), "epilogues run in the re-laid-out row store");
      // column pass (or single pass ending in group 0): element k of this
      // thread sits at voff + k_reg(r) << LS -- a compile-time offset on the
      // scalar base, so the address costs no VALU
#pragma unroll
      for (int r = 0; r < R; ++r) st_d(data + ((size_t)GP::k_reg(r) << PG::LS), voff, x[r]);
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
  // the first group's twiddles: a row pass with an operand prologue loads them
  // after it (they are not needed before the re-layout, and held through the
  // prologue they pushed the operand ring into spills)
  constexpr bool TW_LATE = !COLS && G0 != 0 && EPI != EPI_NONE;
  if constexpr (!TW_LATE) Grp<S, LOGR, G0>::template load_tw<PG::S0>(tc, tw, hi, ts);
  u64 x[R];
  u32 voff;  // byte offset of this thread's element k_thr of the first (HBM) group layout
  if constexpr (!COLS && G0 != 0) {
    // row pass starting in a per-lane-contiguous group: coalesced load in the
    // IO layout (16-byte pairs with PAIR_IO), then one LDS re-layout.  The
    // key-switch prologue keeps 8-byte loads: with pairs of its 2 KD operand
    // streams the compiler holds 12 KD words across steps and spills (61-139
    // VGPRs at KD = 3-4 under the 4-wave bound)
    using GZ = IoL<S, LOGR, PAIR_IO && !is_ksp(EPI)>;
    constexpr int ST = GZ::STEP;
    voff = (gb + GZ::k_thr(ts)) << 3;
    if constexpr (is_tensor(EPI)) {
      // the CKKS tensor formulas, element-wise at the coalesced positions
      // (PRO_TENSOR2: d2 only; EPI_KSQT forms d0 and d1).
      // Software-pipelined PD steps deep: the operand loads of step s + PD
      // are issued before step s's stores (the outputs may alias the
      // operands element-wise only, so the compiler would otherwise wait for
      // each step's loads right after the previous step's stores)
      constexpr int PD = SP ? (ST == 2 ? 1 : 2) : 0;  // the generic products need the registers
      constexpr int NST = R / ST;
      constexpr bool ALL = EPI == PRO_TENSOR;
      constexpr int NO = ALL ? 4 : 2;  // operand streams: (a0, a1, b0, b1) or (a1, b1)
      u64 op[PD + 1][NO][ST];
      const auto fetch = [&](int st, u64 (&o)[NO][ST]) {
        const u32 kn = GZ::k_reg(st * ST);
        const u64 *src[4] = {ALL ? ep.a0 : ep.a1, ALL ? ep.a1 : ep.b1, ep.b0, ep.b1};
#pragma unroll
        for (int i = 0; i < NO; ++i) {
          if constexpr (ST == 2) {
            const u64x2 v = ld2_b(src[i] + kn, voff);
            o[i][0] = v.x, o[i][1] = v.y;
          } else {
            o[i][0] = ld_b(src[i] + kn, voff);
          }
        }
      };
#pragma unroll
      for (int st = 0; st < PD; ++st) fetch(st, op[st]);
#pragma unroll
      for (int st = 0; st < NST; ++st) {
        if (st + PD < NST) fetch(st + PD, op[(st + PD) % (PD + 1)]);
        u64 o0[ST], o1[ST], oe[ST];
#pragma unroll
        for (int h = 0; h < ST; ++h) {
          const u64 a1 = op[st % (PD + 1)][ALL ? 1 : 0][h], b1 = op[st % (PD + 1)][ALL ? 3 : 1][h];
          if constexpr (ALL) {
            const u64 a0 = op[st % (PD + 1)][0][h], b0 = op[st % (PD + 1)][2][h];
            o0[h] = mul_mod<SP>(a0, b0, mi);
            U128 sm = mul128(a0, b1);
            mac128(sm, a1, b0);
            o1[h] = reduce128<SP>(sm, mi);
          }
          // PRO_TENSOR2: d2 R^-1 (< 1.5q; the INTT's output scale carries the R,
          // ntt_inv_tensor_launch); PRO_TENSOR: d2 in [0, 2q)
          const u64 t = ALL ? mont_mul<SP>(mont_reduce<SP>(mul128(a1, b1), mi), mi.r2, mi) : mont_mul<SP>(a1, b1, mi);
          x[st * ST + h] = csub(t, mi.q);
          if constexpr (ALL) oe[h] = csub(mont_mul<SP>(t, mi.r2, mi), mi.q);  // d2 R
        }
        const u32 kr = GZ::k_reg(st * ST);
        if constexpr (ST == 2) {
          if constexpr (ALL) {
            st2_e(ep.o0 + kr, voff, u64x2{o0[0], o0[1]});
            st2_e(ep.o1 + kr, voff, u64x2{o1[0], o1[1]});
            st2_e(ep.ext + kr, voff, u64x2{oe[0], oe[1]});
          }
        } else {
          if constexpr (ALL) {
            st_e(ep.o0 + kr, voff, o0[0]);
            st_e(ep.o1 + kr, voff, o1[0]);
            st_e(ep.ext + kr, voff, oe[0]);
          }
        }
      }
    } else if constexpr (EPI == PRO_BFVT) {
      // the BFV tensor formulas at the coalesced positions; e is per workgroup
      const auto ld = [&](const u64 *base, int r0, u64 (&v)[ST]) {
        if constexpr (ST == 2) {
          const u64x2 t = ld2_b(base + GZ::k_reg(r0), voff);
          v[0] = t.x, v[1] = t.y;
        } else {
          v[0] = ld_b(base + GZ::k_reg(r0), voff);
        }
      };
      if (ep.e == 1) {
#pragma unroll
        for (int r = 0; r < R; r += ST) {
          u64 a0[ST], a1[ST], b0[ST], b1[ST];
          ld(ep.a0, r, a0), ld(ep.b1, r, b1), ld(ep.a1, r, a1), ld(ep.b0, r, b0);
#pragma unroll
          for (int h = 0; h < ST; ++h) {
            U128 sm = mul128(a0[h], b1[h]);
            mac128(sm, a1[h], b0[h]);
            x[r + h] = reduce128<SP>(sm, mi);
          }
        }
      } else {
        // e = 0: (a0, b0), e = 2: (a1, b1) -- the pair is resolved in ntt_pass
#pragma unroll
        for (int r = 0; r < R; r += ST) {
          u64 a0[ST], b0[ST];
          ld(ep.a0, r, a0), ld(ep.b0, r, b0);
#pragma unroll
          for (int h = 0; h < ST; ++h) x[r + h] = mul_mod<SP>(a0[h], b0[h], mi);
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
        if (ep.o0) st_e(ep.o0 + kr, voff, y0);
        x[r] = y1;
        if (ep.ext) st_e(ep.ext + kr, voff, csub63(mont_mul<SP>(y1, mi.r2, mi), mi.q));  // sigma(c1) R
      }
    } else if constexpr (is_ksp(EPI)) {
      // acc_P = sum_j ext_j ksk_j R^-1 (ks_inner_kernel; ext carries R) at the
      // coalesced positions, canonical: the products are below 1.5q (2q
      // generic), the running sum is kept below 2q.  Operands software-
      // pipelined PD elements (PD / 2 pairs) deep (as EPI_KSQ)
      constexpr int KD = ksp_digits(EPI);
      constexpr int PD = SP || ksp_gather(EPI) ? KSP_PD : 1;
      constexpr int NST = R / ST, PDS = (PD + ST - 1) / ST;
      u64 nq1 = 0 - mi.q, nq2 = 0 - 2 * mi.q;
      asm("" : "+s"(nq1));
      asm("" : "+s"(nq2));
      u64 ek[PDS + 1][2 * KD][ST];
      const auto fetch = [&](int st, u64 (&slot)[2 * KD][ST]) {
        const u32 kn = GZ::k_reg(st * ST);
#pragma unroll
        for (int j = 0; j < KD; ++j) {
          if constexpr (ksp_gather(EPI)) {
#pragma unroll
            for (int h = 0; h < ST; ++h)
              slot[j][h] = ld_b(ep.kext + j * ep.ext_j, aut_src<LOG_N>((voff >> 3) + kn + h, ep.xg));
          } else if constexpr (ST == 2) {
            const u64x2 e2 = ld2_b(ep.kext + kn + j * ep.ext_j, voff);
            slot[j][0] = e2.x, slot[j][1] = e2.y;
          } else {
            slot[j][0] = ld_b(ep.kext + kn + j * ep.ext_j, voff);
          }
          if constexpr (ST == 2) {
            const u64x2 k2 = ld2_b(ep.kksk + j * ep.ksk_j + kn, voff);
            slot[KD + j][0] = k2.x, slot[KD + j][1] = k2.y;
          } else {
            slot[KD + j][0] = ld_b(ep.kksk + j * ep.ksk_j + kn, voff);
          }
        }
      };
#pragma unroll
      for (int st = 0; st < PDS; ++st) fetch(st, ek[st]);
#pragma unroll
      for (int st = 0; st < NST; ++st) {
        if (st + PDS < NST) fetch(st + PDS, ek[(st + PDS) % (PDS + 1)]);
#pragma unroll
        for (int h = 0; h < ST; ++h) {
          u64 e[KD], k[KD], pr[KD];
#pragma unroll
          for (int j = 0; j < KD; ++j) {
            e[j] = ek[st % (PDS + 1)][j][h];
            k[j] = ek[st % (PDS + 1)][KD + j][h];
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
          x[st * ST + h] = harvey_csub(acc, nq1);
        }
      }
    } else {
#pragma unroll
      for (int r = 0; r < R; r += ST) {
        if constexpr (ST == 2) {
          const u64x2 v = ld2_d(data + GZ::k_reg(r), voff);
          x[r] = v.x, x[r + 1] = v.y;
        } else {
          x[r] = ld_d(data + GZ::k_reg(r), voff);
        }
      }
    }
    if constexpr (TW_LATE) Grp<S, LOGR, G0>::template load_tw<PG::S0>(tc, tw, hi, ts);
    const u32 lw = lds_idx<S>(w, GZ::k_thr(ts));
#pragma unroll
    for (int r = 0; r < R; ++r) lds[lw + GZ::k_reg(r) + lds_pad(GZ::k_reg(r))] = x[r];
    __syncthreads();
    using GF = Grp<S, LOGR, G0>;
    const u32 lr = lds_idx<S>(w, GF::k_thr(ts));
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const u32 kr = GF::k_reg(r);
      x[r] = lds[lr + kr + lds_pad(kr)];
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
      // special targets: the in-place column reduction where one side of every
      // product is below 2^60 (WIDE targets, or sources below 2^60: ModUp's P
      // targets; result < 1.25q), else the 128-bit combine (a uniform branch)
      const bool sp60 = CONV_COLS && SP && CONV_SP60 && (WIDE || a.c_src60);
#pragma unroll
      for (int c0 = 0; c0 < R; c0 += 4) {
        u64 sv[4][NS];
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int i = 0; i < NS; ++i)
            sv[j][i] = ld_b(ep.src + i * NW + ((size_t)GF::k_reg(c0 + j) << PG::LS), voff);
        if (sp60) {
#pragma unroll
          for (int j = 0; j < 4; ++j) x[c0 + j] = dot_cols_sp60<NS>(sv[j], hc0, hc1, mi.q_hi);  // < 1.25q
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            x[c0 + j] = CONV_COLS ? dot_cols<NS, SP>(sv[j], hc0, hc1, mi)                  // < 2q
                                  : dot_mont_lazy<NS, SP, WIDE>(sv[j], ep.h, 1, NS, mi);   // < 4q
        }
        if constexpr (NS == 1 && CONV_COLS) {
          // rescale: the central lift (x - q_l for x > q_l / 2) of the single
          // source, as y + q - [q_l]_{q_m} < 3q (a uniform branch per launch)
          if (a.c_lift_half) {
            const u64 add = mi.q - ep.lift_sub;
#pragma unroll
            for (int j = 0; j < 4; ++j) x[c0 + j] += sv[j][0] > a.c_lift_half ? add : 0;
          }
        }
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
    // forward: the re-laid-out IO layout (group_loop's store); inverse: the
    // last group is group 0 and stores straight from registers
    voff = (gb + (INV ? Grp<S, LOGR, 0>::k_thr(ts) : IoL<S, LOGR>::k_thr(ts))) << 3;
  }
  NoFetch nf;
  group_loop<LOG_N, S, LOGR, W, INV, COLS, SP, WIDE, EPI, 0>(x, tc, lds, tw, data, voff, w, ts, hi, a, mi, mod, ep,
                                                             nf);
}

// ---- persistent one-residue-per-workgroup pass (N = 2^13, 2^14; plain NTT/INTT)
// A one-shot single pass at N = 2^14 holds a 128 KiB residue in one 1024-thread
// workgroup per CU, so its HBM loads, butterflies, barrier-separated exchanges
// and stores run one after the other with nothing to overlap them (it lost to
// two 7-stage passes).  Here each workgroup loops over residues and loads the
// NEXT residue's 16 words per thread into a second register tile while the
// current one is transformed: the loads are issued in pieces behind each
// group's twiddle prefetch (vmcnt counts in issue order, so a piece issued
// there does not delay the waits of the group it rides on), and the stores of
// residue j drain under the transform of residue j + 1.
#ifndef PERSIST_FETCH
#define PERSIST_FETCH 8  // words of the next residue prefetched per thread (the rest load when it starts)
#endif
template <class LAYOUT>
struct ResidueFetch {
  u64 (&nx)[16];
  const u64 *src;  // the next residue (null: none)
  u32 voff;        // this thread's element of the load layout
  // piece GI of NG - 1: the PERSIST_FETCH loads spread over the groups that load twiddles
  template <int GI, int NG>
  __device__ __forceinline__ void issue() {
    constexpr int F = PERSIST_FETCH, P = NG - 1, lo = F * GI / P, hi = F * (GI + 1) / P;
    if (!src) return;
#pragma unroll
    for (int r = lo; r < hi; ++r) nx[r] = ld_d(src + LAYOUT::k_reg(r), voff);
  }
};


template <int LOG_N, bool INV, bool SP, int WM, int K>
__global__ void __launch_bounds__(1 << (LOG_N - 4)) ntt_persist(NttArgs a, u32 n_jobs) {
  constexpr int S = LOG_N, LOGR = 4, W = 1, R = 16;
  constexpr bool WIDE = !INV && WM == 1;
  static_assert(WM != 2 || INV, "one lazy schedule class per persistent launch");
  using PG = PassGeo<LOG_N, S, false, INV>;
  static_assert(PG::single && PG::LAST, "one pass per residue");
  constexpr int NG = (S + LOGR - 1) / LOGR;
  constexpr int G0 = INV ? NG - 1 : 0;
  // loads: forward in the first group's own (group-0) layout, inverse in the
  // IO layout followed by an LDS re-layout; stores: forward through the
  // re-layout into the IO layout, inverse straight from group 0
  using GZ = typename std::conditional<INV, IoL<S, LOGR>, Grp<S, LOGR, 0>>::type;
  using GS = typename std::conditional<INV, Grp<S, LOGR, 0>, IoL<S, LOGR>>::type;
  using GF = Grp<S, LOGR, G0>;
  extern __shared__ u64 lds[];
  const u32 ts = threadIdx.x, w = 0, hi = 0;
  const u32 voff = GZ::k_thr(ts) << 3, voff_st = GS::k_thr(ts) << 3;
  const u32 np = a.map.n_polys;
  // residue j of this workgroup: job blockIdx.x + j gridDim.x (K residues per
  // workgroup, the loop fully unrolled: no loop-carried modulus or address)
  const auto residue = [&](int j, u32 &mod) -> u64 * {
    const u32 job = blockIdx.x + (u32)j * gridDim.x;
    if (job >= n_jobs) return nullptr;
    const u32 poly = job % np, limb = limbmap_limb(a.map, job / np);
    mod = __builtin_amdgcn_readfirstlane(a.map.mod_offset + limb);
    const size_t off = ((size_t)poly * a.map.poly_stride + limb) << LOG_N;
    // uniform: SGPRs (readfirstlane) -- without it the compiler left the second
    // residue's offset in VGPRs and failed ("illegal VGPR to SGPR copy")
    const u32 lo = __builtin_amdgcn_readfirstlane((u32)off), hi32 = __builtin_amdgcn_readfirstlane((u32)(off >> 32));
    return a.map.base + (((size_t)hi32 << 32) | lo);
  };
  const auto source = [&](u64 *d) -> const u64 * {  // the first forward pass may read out of place
    return d && !INV && a.src ? a.src + (d - a.map.base) : d;
  };
  u64 x[R], nx[R];
  u32 mod = 0;
  u64 *data = residue(0, mod);
  if (!data) return;
  {
    const u64 *din = source(data);
#pragma unroll
    for (int r = 0; r < R; ++r) x[r] = ld_d(din + GZ::k_reg(r), voff);
  }
#pragma unroll
  for (int j = 0; j < K; ++j) {
    u32 nmod = 0;
    u64 *ndata = j + 1 < K ? residue(j + 1, nmod) : nullptr;
    ResidueFetch<GZ> pf{nx, source(ndata), voff};
    const ModInfo mi = a.mods[mod];
    const u64 *tw = a.tw + ((size_t)mod << LOG_N);
    u64 tc[16];
    GF::template load_tw<PG::S0>(tc, tw, hi, ts);
    if constexpr (G0 != 0) {
      // inverse: from the coalesced layout into the first (per-lane-contiguous) group's
#pragma unroll
      for (int r = 0; r < R; ++r) lds[lds_idx<S>(w, GZ::k_thr(ts)) + GZ::k_reg(r) + lds_pad(GZ::k_reg(r))] = x[r];
      __syncthreads();
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const u32 kr = GF::k_reg(r);
        x[r] = lds[lds_idx<S>(w, GF::k_thr(ts)) + kr + lds_pad(kr)];
      }
    }
    EpiRow ep{};
    group_loop<LOG_N, S, LOGR, W, INV, false, SP, WIDE, EPI_NONE, 0>(x, tc, lds, tw, data, voff_st, w, ts, hi, a,
                                                                     mi, mod, ep, pf);
    if (!ndata) return;
    __syncthreads();  // this residue's last LDS reads before the next one's first writes
#pragma unroll
    for (int r = 0; r < R; ++r) x[r] = r < PERSIST_FETCH ? nx[r] : ld_d(pf.src + GZ::k_reg(r), voff);
    mod = nmod;
    data = ndata;
  }
}

#ifndef PERSIST_K
#define PERSIST_K 4  // residues per workgroup of the one-pass kernel (its register double buffer runs across them)
#endif
// one-pass launch: ceil(n_jobs / K) workgroups of K residues each
template <int LOG_N, bool INV, bool SP, int WM>
int launch_persist(fhe_ctx *c, const NttArgs &a, u32 n_jobs) {
  constexpr size_t lds = lds_bytes<LOG_N, 1>();
  auto k = ntt_persist<LOG_N, INV, SP, WM, PERSIST_K>;
  if (lds > 64 * 1024) (void)hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  const u32 grid = (n_jobs + PERSIST_K - 1) / PERSIST_K;
  hipLaunchKernelGGL(k, dim3(grid), dim3(1u << (LOG_N - 4)), lds, c->stream, a, n_jobs);
  return fhe_check(c, hipGetLastError(), "ntt_persist launch");
}


#ifndef NTT_MINW
#define NTT_MINW 1
#endif
// WM (forward passes): the lazy schedule of the launch's moduli, chosen on the
// host (wide_mode): 1 all WIDE (q < 2^60), 0 all narrow, 2 mixed (a per-
// workgroup branch between both; the kernel then carries both code paths and
// needs ~150 VGPRs instead of ~90, i.e. 3 waves per SIMD instead of the 4 the
// LDS allows: a launch over one modulus class avoids it)
// The tensor prologue asks for 4 waves per SIMD (the LDS allows 4 workgroups
// per CU anyway), so its 16-byte operand pairs stay within 128 VGPRs
__host__ __device__ constexpr int pass_min_waves(int EPI, bool SP, int threads) {
  return threads != 256 ? 1 : (PAIR_IO && is_tensor(EPI) && SP) ? 4 : (ksq_tensor(EPI) && SP) ? KSQT_MINW : NTT_MINW;
}
template <int LOG_N, int S, int LOGR, int W, bool INV, bool COLS, bool SP, int EPI, int WM>
__global__ void __launch_bounds__(W << (S - LOGR), pass_min_waves(EPI, SP, W << (S - LOGR)))
    ntt_pass(NttArgs a) {
  static_assert(is_combine(EPI) || EPI == EPI_NONE || is_tensor(EPI) || EPI == PRO_AUTOMORPH ||
                    EPI == PRO_BFVT || is_conv(EPI) || is_ksp(EPI),
                "ntt_pass epilogues");
  static_assert(!is_conv(EPI) || (!INV && COLS), "the conversion prologue feeds a forward column pass");
  static_assert(!is_combine(EPI) || (!INV && !COLS), "epilogues follow a forward row pass");
  static_assert((!is_tensor(EPI) && EPI != PRO_AUTOMORPH && EPI != PRO_BFVT && !is_ksp(EPI)) || (INV && !COLS),
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
    // The remap is one-to-one only when the (limb, row block) groups fill the 8
    // XCDs evenly; other shapes keep the plain blockIdx mapping
    constexpr u32 GIW = is_ksq(EPI) ? KSQ_GI : KSP_GI;
    if (((gridDim.x * gridDim.z) & 7) == 0) {
      const u32 np = gridDim.y, lin = blockIdx.x + gridDim.x * (blockIdx.y + np * blockIdx.z);
      const u32 r = lin >> 3, gpx = gridDim.x * gridDim.z / 8;  // groups per XCD
      const u32 GI = gpx % GIW == 0 ? GIW : 1;
      const u32 within = r % (GI * np);
      const u32 g = ((r / (GI * np)) * GI + within % GI) * 8 + (lin & 7);  // g = (limb, row block)
      poly = within / GI;
      bx = g % gridDim.x;
      act = g / gridDim.x;
    }
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
  // rotation-batched gather passes: this poly's rotation and ciphertext poly
  u32 rot = 0, cpoly = poly;
  const u64 *ksk = a.e_ksk;
  if constexpr (ksq_gather(EPI) || ksp_gather(EPI)) {
    ep.xg = a.e_ext_g;
    if (a.e_rp) {
      rot = poly / a.e_rp;
      cpoly = poly - rot * a.e_rp;
      ksk = a.e_ksk_r[rot];
      ep.xg = a.e_g_r[rot];
    }
  }
  if constexpr (is_ksp(EPI)) {
    // P limbs: key row limb + e_kshift (a level view reads the full-level key)
    const size_t N = (size_t)1 << LOG_N;
    ep.ext_j = (size_t)a.e_QP * N;
    ep.ksk_j = (size_t)2 * a.e_kQP * N;
    ep.kext = a.e_ext + ((size_t)(cpoly >> 1) * a.e_ndig * a.e_QP + limb) * N;
    ep.kksk = ksk + ((size_t)(cpoly & 1) * a.e_kQP + limb + a.e_kshift) * N;
  }
  if constexpr (is_combine(EPI)) {
    if constexpr (is_ksq(EPI)) {
      const size_t N = (size_t)1 << LOG_N;
      ep.ext_j = (size_t)a.e_QP * N;
      ep.ksk_j = (size_t)2 * a.e_kQP * N;
      ep.kext = a.e_ext + ((size_t)(cpoly >> 1) * a.e_ndig * a.e_QP + limb) * N;
      ep.kksk = ksk + ((size_t)(cpoly & 1) * a.e_kQP + limb) * N;  // Q limbs: key row = limb
    }
    ep.acc = a.e_acc + (((size_t)poly * a.e_acc_stride + limb) << LOG_N);
    ep.base = a.e_base + (((size_t)cpoly * a.map.poly_stride + limb) << LOG_N);
    ep.out = (ksq_gather(EPI) && a.e_rp ? a.e_out_r[rot] : a.e_out) +
             (((size_t)cpoly * a.map.poly_stride + limb) << LOG_N);
    ep.pinv = a.e_pinv[limb];
    ep.add = (a.e_add_mask >> (poly & 1)) & 1;
    ep.g = ksq_gather(EPI) && a.e_rp ? a.e_g_r[rot] : a.e_g;
    if constexpr (ksq_tensor(EPI)) {
      // this poly's ciphertext (ct, b) = (cpoly / 2, cpoly % 2): a_j, b_j at (2 ct + j, limb)
      const size_t LN = (size_t)a.map.poly_stride << LOG_N;
      const size_t o = (((size_t)(cpoly & ~1u) * a.map.poly_stride + limb) << LOG_N);
      ep.a0 = a.e_ta + o;
      ep.a1 = ep.a0 + LN;
      ep.b0 = a.e_tb + o;
      ep.b1 = ep.b0 + LN;
      ep.e = cpoly & 1;
      ep.jown = limb / a.t_alpha;
    }
  }
  if constexpr (is_tensor(EPI)) {
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
    ep.ext = a.t_ext ? a.t_ext + (((size_t)(poly * a.t_ndig + limb / a.t_alpha) * a.t_QP + limb) << LOG_N) : nullptr;
    ep.g = a.t_g;
  }
  if constexpr (is_conv(EPI)) {
    ep.src = a.c_src + (((size_t)poly * a.c_src_stride + a.c_src_first) << LOG_N);
#pragma unroll
    for (int i = 0; i < conv_ns(EPI); ++i) ep.h[i] = a.c_h[(size_t)i * a.c_nd + act];
    if (conv_ns(EPI) == 1 && a.c_lift_sub) ep.lift_sub = a.c_lift_sub[act];
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
[[maybe_unused]] int wide_mode(const fhe_ctx *c, const LimbMap &m) {
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
  } else if constexpr (is_tensor(EPI) || EPI == PRO_AUTOMORPH || EPI == PRO_BFVT || is_ksp(EPI)) {
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

}  // namespace
