// rns.hip -- element-wise RNS kernels, fast base conversion, hybrid key
// switching, automorphisms and BFV (BEHZ) scaling for gfx950.
//
// Every kernel here is a per-coefficient map over HBM-resident limb-polys:
// one thread per coefficient, consecutive lanes on consecutive coefficients
// (512 B per wave-instruction of u64), (item, limb) on gridDim.y.  Constants
// (CRT tables) are tiny, pre-scaled into Montgomery form on the host and stay
// in L2.  Each kernel restates the oracle function named in its comment
// (oracle/fhe_oracle.c); every step is exact modular arithmetic with the same
// formula, only the reduction strategy differs (Montgomery, modarith.hpp), so
// results are bit-identical.
//
// Template parameter SP selects the q = 1 (mod 2^32) Montgomery reduction
// (2 multiplies) or the generic one (7 multiplies); see modarith.hpp.
#include <algorithm>
#include <cstring>

#include "context.hpp"

#define EW_BLOCK 256

namespace {

// sum_{i < ns} v[i] * h[i * hs] mod m, exact, given canonical v[i] and
// R-pre-scaled constants h.  Chunks of 4 keep each 128-bit sum < q * 2^64.
template <int NS, bool SP>
__device__ __forceinline__ u64 dot_mont(const u64 (&v)[NS], const u64 *h, size_t hs, u32 ns, const ModInfo &m) {
  u64 res = 0;
#pragma unroll
  for (int c0 = 0; c0 < NS; c0 += 4) {
    if (c0 < (int)ns) {
      U128 acc{0, 0};
#pragma unroll
      for (int i = c0; i < c0 + 4 && i < NS; ++i)
        if (i < (int)ns) mac128(acc, v[i], h[(size_t)i * hs]);
      const u64 part = csub(mont_reduce<SP>(acc, m), m.q);
      res = c0 == 0 ? part : add_mod(res, part, m.q);
    }
  }
  return res;
}

// ------------------------------------------------------------ element-wise
template <EwOp OP, bool SP>
__global__ void __launch_bounds__(EW_BLOCK) ew_kernel(const u64 *__restrict__ a, const u64 *__restrict__ b,
                                                      u64 *__restrict__ out, const ModInfo *mods, u32 mod_begin,
                                                      u32 n_limbs, u32 log_n) {
  const u32 k = blockIdx.x * EW_BLOCK + threadIdx.x;
  const u32 job = blockIdx.y;
  const ModInfo m = mods[mod_begin + job % n_limbs];
  const size_t o = ((size_t)job << log_n) + k;
  const u64 x = a[o], y = b[o];
  u64 r;
  if (OP == EwOp::Add) r = add_mod(x, y, m.q);
  else if (OP == EwOp::Sub) r = sub_mod(x, y, m.q);
  else r = mul_mod<SP>(x, y, m);
  out[o] = r;
}

// orc_fill_uniform
__global__ void __launch_bounds__(EW_BLOCK) fill_kernel(u64 *out, const ModInfo *mods, u32 mod_begin, u32 n_limbs,
                                                        u32 log_n, u64 seed) {
  const u32 k = blockIdx.x * EW_BLOCK + threadIdx.x;
  const u32 job = blockIdx.y;
  const u64 q = mods[mod_begin + job % n_limbs].q;
  const size_t w = ((size_t)job << log_n) + k;
  out[w] = mulhi64(stream_word(seed, w), q);
}

// --------------------------------------------------------- base conversion
// conv_apply (oracle): v_i = [x_i (S/s_i)^-1]_{s_i};  y_m = sum_i v_i [S/s_i]_{d_m} mod d_m.
template <int NS, bool SP>
__global__ void __launch_bounds__(EW_BLOCK) conv_kernel(const u64 *__restrict__ src, u32 src_stride,
                                                        u64 *__restrict__ dst, u32 dst_stride, ConvTab t,
                                                        const ModInfo *mods, u32 log_n) {
  const u32 k = blockIdx.x * EW_BLOCK + threadIdx.x;
  const u32 p = blockIdx.y;
  const size_t N = (size_t)1 << log_n;
  const u64 *s = src + (size_t)p * src_stride * N + k;
  u64 *d = dst + (size_t)p * dst_stride * N + k;
  u64 v[NS];
#pragma unroll
  for (int i = 0; i < NS; ++i) {
    v[i] = 0;
    if (i < (int)t.ns) {
      const ModInfo ms = mods[t.src_mod[i]];
      v[i] = csub(mont_mul<SP>(s[i * N], t.hinv[i], ms), ms.q);
    }
  }
  for (u32 m = 0; m < t.nd; ++m) d[m * N] = dot_mont<NS, SP>(v, t.h + m, t.nd, t.ns, mods[t.dst_mod[m]]);
}

// ModUp (keyswitch_one, oracle).  For digit j the digit's own limbs are
// copied from `own` (NTT form for CKKS, coefficient form for BFV), every other
// limb of Q u P is the fast base conversion of the digit's coefficient-form
// limbs.  All outputs are written times R (Montgomery form) so the KS inner
// product needs a single reduction.
template <int NS, bool SP>
__global__ void __launch_bounds__(EW_BLOCK) modup_kernel(const u64 *__restrict__ dc, u32 dc_stride,
                                                         const u64 *__restrict__ own, u32 own_stride,
                                                         u64 *__restrict__ ext, const ConvTab *tabs,
                                                         const ModInfo *mods, u32 QP, u32 alpha, u32 ndig,
                                                         u32 log_n) {
  const u32 k = blockIdx.x * EW_BLOCK + threadIdx.x;
  const u32 ct = blockIdx.y / ndig, j = blockIdx.y % ndig;
  const size_t N = (size_t)1 << log_n;
  const u32 lo = j * alpha;
  const ConvTab t = tabs[j];
  u64 *e = ext + ((size_t)(ct * ndig + j) * QP) * N + k;
  const u64 *s = dc + ((size_t)ct * dc_stride + lo) * N + k;
  const u64 *o = own + ((size_t)ct * own_stride + lo) * N + k;
  u64 v[NS];
#pragma unroll
  for (int i = 0; i < NS; ++i) {
    v[i] = 0;
    if (i < (int)t.ns) {
      const ModInfo ms = mods[lo + i];
      v[i] = csub(mont_mul<SP>(s[i * N], t.hinv[i], ms), ms.q);
      e[(lo + i) * N] = csub(mont_mul<SP>(o[i * N], ms.r2, ms), ms.q);  // own limb * R
    }
  }
  // destinations are limbs of Q u P: dst_mod[m] is also the limb index
  for (u32 m = 0; m < t.nd; ++m) {
    const u32 dm = t.dst_mod[m];
    e[dm * N] = dot_mont<NS, SP>(v, t.h + m, t.nd, t.ns, mods[dm]);
  }
}

// KS inner product (keyswitch_one, oracle):
//   acc_b[i] = sum_j ext_j[i] * ksk[j][b][i]  mod m_i,  b in {0,1}
// ext carries a factor R, removed by the one Montgomery reduction per chunk.
template <bool SP>
__global__ void __launch_bounds__(EW_BLOCK) ks_inner_kernel(const u64 *__restrict__ ext, const u64 *__restrict__ ksk,
                                                            u64 *__restrict__ acc, const ModInfo *mods, u32 QP,
                                                            u32 ndig, u32 log_n) {
  const u32 k = blockIdx.x * EW_BLOCK + threadIdx.x;
  const u32 ct = blockIdx.y / QP, i = blockIdx.y % QP;
  const size_t N = (size_t)1 << log_n;
  const ModInfo m = mods[i];
  u64 r0 = 0, r1 = 0;
  for (u32 j0 = 0; j0 < ndig; j0 += 4) {
    U128 a0{0, 0}, a1{0, 0};
    for (u32 j = j0; j < j0 + 4 && j < ndig; ++j) {
      const u64 x = ext[((size_t)(ct * ndig + j) * QP + i) * N + k];
      mac128(a0, x, ksk[((size_t)(2 * j) * QP + i) * N + k]);
      mac128(a1, x, ksk[((size_t)(2 * j + 1) * QP + i) * N + k]);
    }
    r0 = add_mod(r0, csub(mont_reduce<SP>(a0, m), m.q), m.q);
    r1 = add_mod(r1, csub(mont_reduce<SP>(a1, m), m.q), m.q);
  }
  acc[((size_t)(2 * ct) * QP + i) * N + k] = r0;
  acc[((size_t)(2 * ct + 1) * QP + i) * N + k] = r1;
}

// ModDown finish: out_b[i] = base_b[i] + (acc_b[i] - conv_b[i]) * P^-1 mod q_i
template <bool SP>
__global__ void __launch_bounds__(EW_BLOCK) ks_combine_kernel(const u64 *__restrict__ acc,
                                                              const u64 *__restrict__ conv, const u64 *base,
                                                              u64 *out, const u64 *pinv, const ModInfo *mods, u32 L,
                                                              u32 QP, u32 log_n, u32 add_mask) {
  const u32 k = blockIdx.x * EW_BLOCK + threadIdx.x;
  const u32 ct = blockIdx.y / (2 * L), r = blockIdx.y % (2 * L), b = r / L, i = r % L;
  const size_t N = (size_t)1 << log_n;
  const ModInfo m = mods[i];
  const u64 a = acc[((size_t)(2 * ct + b) * QP + i) * N + k];
  const u64 cv = conv[((size_t)(2 * ct + b) * L + i) * N + k];
  u64 ks = csub(mont_mul<SP>(sub_mod(a, cv, m.q), pinv[i], m), m.q);
  const size_t o = ((size_t)(2 * ct + b) * L + i) * N + k;
  if (add_mask & (1u << b)) ks = add_mod(ks, base[o], m.q);
  out[o] = ks;
}

// CKKS tensor (orc_mul_relin): d0 = a0 b0, d1 = a0 b1 + a1 b0, d2 = a1 b1.
// Generic strides so BFV reuses it on Q and on Bsk.
struct TensorArgs {
  const u64 *a;
  const u64 *b;
  u64 *e01;
  u64 *e2;
  size_t a_ct, a_poly;   // strides in words
  size_t b_ct, b_poly;
  size_t e_ct, e_poly;
  size_t e2_ct;
  u32 nl, mod_offset, log_n;
};
template <bool SP>
__global__ void __launch_bounds__(EW_BLOCK) tensor_kernel(TensorArgs t, const ModInfo *mods) {
  const u32 k = blockIdx.x * EW_BLOCK + threadIdx.x;
  const u32 ct = blockIdx.y / t.nl, l = blockIdx.y % t.nl;
  const size_t off = ((size_t)l << t.log_n) + k;
  const ModInfo m = mods[t.mod_offset + l];
  const u64 *A = t.a + ct * t.a_ct + off, *B = t.b + ct * t.b_ct + off;
  const u64 a0 = A[0], a1 = A[t.a_poly], b0 = B[0], b1 = B[t.b_poly];
  u64 *E = t.e01 + ct * t.e_ct + off;
  E[0] = mul_mod<SP>(a0, b0, m);
  U128 s = mul128(a0, b1);
  mac128(s, a1, b0);
  E[t.e_poly] = reduce128<SP>(s, m);
  t.e2[ct * t.e2_ct + off] = mul_mod<SP>(a1, b1, m);
}

// NTT-domain automorphism (orc_automorph_ntt): slot k holds a(psi^(2brv(k)+1))
__global__ void __launch_bounds__(EW_BLOCK) automorph_ntt_kernel(const u64 *__restrict__ in, u64 *__restrict__ out,
                                                                 u32 g, u32 log_n) {
  const u32 k = blockIdx.x * EW_BLOCK + threadIdx.x;
  const size_t base = (size_t)blockIdx.y << log_n;
  const u32 mask = (2u << log_n) - 1;
  const u32 e = 2 * (__brev(k) >> (32 - log_n)) + 1;
  const u32 e2 = (u32)(((u64)e * g) & mask);
  const u32 src = __brev((e2 - 1) >> 1) >> (32 - log_n);
  out[base + k] = in[base + src];
}

// coefficient-domain automorphism (orc_automorph_coef) as a gather:
// out[d] = a[j0] if j0 < N else -a[j0 - N], j0 = d * g^-1 mod 2N
__global__ void __launch_bounds__(EW_BLOCK) automorph_coef_kernel(const u64 *__restrict__ in, u64 *__restrict__ out,
                                                                  u32 ginv, const ModInfo *mods, u32 n_limbs,
                                                                  u32 log_n) {
  const u32 d = blockIdx.x * EW_BLOCK + threadIdx.x;
  const size_t base = (size_t)blockIdx.y << log_n;
  const u32 n = 1u << log_n, mask = 2 * n - 1;
  const u32 j0 = (u32)(((u64)d * ginv) & mask);
  u64 v;
  if (j0 < n) {
    v = in[base + j0];
  } else {
    const u64 q = mods[blockIdx.y % n_limbs].q;
    const u64 x = in[base + j0 - n];
    v = x ? q - x : 0;
  }
  out[base + d] = v;
}

// ----------------------------------------------------------------- BEHZ
// Constants for SEAL-style BEHZ (behz_init in the oracle), Montgomery
// pre-scaled ("_R" = times 2^64 mod the modulus it is used with).
#define BEHZ_MAXL 24
struct BehzDev {
  u32 L, nB, bsk0;                 // bsk0 = first Bsk modulus id
  u32 neg_inv_q_mod_mt;            // -Q^-1 mod 2^32
  u32 h_mod_mt[BEHZ_MAXL];         // (Q/q_i) mod 2^32
  u64 mt_hinv_R[BEHZ_MAXL];        // 2^32 (Q/q_i)^-1 mod q_i
  u64 t_hinv_R[BEHZ_MAXL];         // t (Q/q_i)^-1 mod q_i
  u64 h_q_bsk_R[BEHZ_MAXL][BEHZ_MAXL + 1];  // (Q/q_i) mod b_j
  u64 q_mod_bsk_R[BEHZ_MAXL + 1];  // Q mod b_j
  u64 inv_mt_bsk_R[BEHZ_MAXL + 1]; // 2^-32 mod b_j
  u64 inv_q_bsk_R[BEHZ_MAXL + 1];  // Q^-1 mod b_j
  u64 t_bsk_R[BEHZ_MAXL + 1];      // t mod b_j
  u64 b_hinv_R[BEHZ_MAXL];         // (B/b_j)^-1 mod b_j
  u64 h_b_msk_R[BEHZ_MAXL];        // (B/b_j) mod m_sk
  u64 inv_b_msk_R;                 // B^-1 mod m_sk
  u64 b_mod_q_R[BEHZ_MAXL];        // B mod q_i
  u64 h_b_q_R[BEHZ_MAXL][BEHZ_MAXL];  // (B/b_j) mod q_i
};

// behz_extend (oracle): fastbconv_m_tilde then sm_mrq.  x [L] coef -> [nB] coef
template <int NL, bool SP>
__global__ void __launch_bounds__(EW_BLOCK) behz_extend_kernel(const u64 *__restrict__ xq, u64 *__restrict__ xb,
                                                               const BehzDev *bz, const ModInfo *mods, u32 log_n) {
  const u32 k = blockIdx.x * EW_BLOCK + threadIdx.x;
  const u32 p = blockIdx.y;
  const size_t N = (size_t)1 << log_n;
  const u32 L = bz->L, nB = bz->nB;
  const u64 *s = xq + (size_t)p * L * N + k;
  u64 v[NL];
  u32 xmt = 0;
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    v[i] = 0;
    if (i < (int)L) {
      const ModInfo m = mods[i];
      v[i] = csub(mont_mul<SP>(s[i * N], bz->mt_hinv_R[i], m), m.q);
      xmt += (u32)v[i] * bz->h_mod_mt[i];
    }
  }
  const u32 r = xmt * bz->neg_inv_q_mod_mt;
  u64 *d = xb + (size_t)p * nB * N + k;
  for (u32 j = 0; j < nB; ++j) {
    const ModInfo m = mods[bz->bsk0 + j];
    const u64 xbj = dot_mont<NL, SP>(v, &bz->h_q_bsk_R[0][j], BEHZ_MAXL + 1, L, m);
    const u64 rr = r >= 0x80000000u ? (u64)r + m.q - (1ull << 32) : (u64)r;   // centered r mod b
    const u64 sum = add_mod(xbj, csub(mont_mul<SP>(rr, bz->q_mod_bsk_R[j], m), m.q), m.q);
    d[j * N] = csub(mont_mul<SP>(sum, bz->inv_mt_bsk_R[j], m), m.q);
  }
}

// behz_floor_to_q (oracle): fast_floor in Bsk then fastbconv_sk back to Q.
template <int NL, bool SP>
__global__ void __launch_bounds__(EW_BLOCK) behz_floor_kernel(const u64 *__restrict__ eq, const u64 *__restrict__ eb,
                                                              u64 *__restrict__ out01, u64 *__restrict__ out2,
                                                              const BehzDev *bz, const ModInfo *mods, u32 log_n) {
  const u32 k = blockIdx.x * EW_BLOCK + threadIdx.x;
  const u32 ct = blockIdx.y / 3, p = blockIdx.y % 3;
  const size_t N = (size_t)1 << log_n;
  const u32 L = bz->L, nB = bz->nB;
  const u64 *xq = eq + ((size_t)(ct * 3 + p) * L) * N + k;
  const u64 *xb = eb + ((size_t)(ct * 3 + p) * nB) * N + k;
  u64 v[NL];
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    v[i] = 0;
    if (i < (int)L) {
      const ModInfo m = mods[i];
      v[i] = csub(mont_mul<SP>(xq[i * N], bz->t_hinv_R[i], m), m.q);  // [t x (Q/q_i)^-1]_{q_i}
    }
  }
  // fast_floor: ((t x)_b - conv_Q->b(t x)) * Q^-1, then fastbconv_sk weights
  u64 w[NL];
  u64 flsk = 0;
#pragma unroll
  for (int j = 0; j < NL + 1; ++j) {
    if (j < (int)nB) {
      const ModInfo m = mods[bz->bsk0 + j];
      const u64 cv = dot_mont<NL, SP>(v, &bz->h_q_bsk_R[0][j], BEHZ_MAXL + 1, L, m);
      const u64 tx = csub(mont_mul<SP>(xb[j * N], bz->t_bsk_R[j], m), m.q);
      const u64 fl = csub(mont_mul<SP>(sub_mod(tx, cv, m.q), bz->inv_q_bsk_R[j], m), m.q);
      if (j == (int)nB - 1) flsk = fl;
      else if (j < NL) w[j] = csub(mont_mul<SP>(fl, bz->b_hinv_R[j], m), m.q);
    } else if (j < NL) {
      w[j] = 0;
    }
  }
  const ModInfo msk = mods[bz->bsk0 + nB - 1];
  const u64 cmsk = dot_mont<NL, SP>(w, bz->h_b_msk_R, 1, nB - 1, msk);
  const u64 alpha = csub(mont_mul<SP>(sub_mod(cmsk, flsk, msk.q), bz->inv_b_msk_R, msk), msk.q);
  const bool neg = alpha > msk.q / 2;
  const u64 amag = neg ? msk.q - alpha : alpha;
  u64 *o = (p < 2) ? out01 + ((size_t)(ct * 2 + p) * L) * N + k : out2 + ((size_t)ct * L) * N + k;
  for (u32 i = 0; i < L; ++i) {
    const ModInfo m = mods[i];
    const u64 cq = dot_mont<NL, SP>(w, &bz->h_b_q_R[0][i], BEHZ_MAXL, nB - 1, m);
    const u64 ab = csub(mont_mul<SP>(amag, bz->b_mod_q_R[i], m), m.q);
    o[i * N] = neg ? add_mod(cq, ab, m.q) : sub_mod(cq, ab, m.q);
  }
}

// ------------------------------------------------------- host launchers
template <bool SP>
int ew_impl(fhe_ctx *c, EwOp op, const u64 *a, const u64 *b, u64 *out, u32 jobs, u32 mod_begin, u32 n_limbs) {
  dim3 grid(c->n / EW_BLOCK, jobs);
  switch (op) {
    case EwOp::Add: hipLaunchKernelGGL((ew_kernel<EwOp::Add, SP>), grid, dim3(EW_BLOCK), 0, c->stream, a, b, out, c->d_mods, mod_begin, n_limbs, c->log_n); break;
    case EwOp::Sub: hipLaunchKernelGGL((ew_kernel<EwOp::Sub, SP>), grid, dim3(EW_BLOCK), 0, c->stream, a, b, out, c->d_mods, mod_begin, n_limbs, c->log_n); break;
    case EwOp::Mul: hipLaunchKernelGGL((ew_kernel<EwOp::Mul, SP>), grid, dim3(EW_BLOCK), 0, c->stream, a, b, out, c->d_mods, mod_begin, n_limbs, c->log_n); break;
  }
  return fhe_check(c, hipGetLastError(), "ew_kernel");
}

template <bool SP>
int conv_impl(fhe_ctx *c, const ConvTab &t, const u64 *src, u32 ss, u64 *dst, u32 ds, u32 n) {
  dim3 grid(c->n / EW_BLOCK, n);
  if (t.ns <= 4) hipLaunchKernelGGL((conv_kernel<4, SP>), grid, dim3(EW_BLOCK), 0, c->stream, src, ss, dst, ds, t, c->d_mods, c->log_n);
  else if (t.ns <= 8) hipLaunchKernelGGL((conv_kernel<8, SP>), grid, dim3(EW_BLOCK), 0, c->stream, src, ss, dst, ds, t, c->d_mods, c->log_n);
  else if (t.ns <= 16) hipLaunchKernelGGL((conv_kernel<16, SP>), grid, dim3(EW_BLOCK), 0, c->stream, src, ss, dst, ds, t, c->d_mods, c->log_n);
  else return fhe_fail(c, FHE_ERR_UNSUPPORTED, "base conversion with more than 16 source moduli");
  return fhe_check(c, hipGetLastError(), "conv_kernel");
}

template <bool SP>
int modup_impl(fhe_ctx *c, const u64 *dc, u32 dcs, const u64 *own, u32 owns, u64 *ext, u32 n, u32 ndig) {
  dim3 grid(c->n / EW_BLOCK, n * ndig);
  const u32 QP = c->L + c->K;
  if (c->alpha <= 4)
    hipLaunchKernelGGL((modup_kernel<4, SP>), grid, dim3(EW_BLOCK), 0, c->stream, dc, dcs, own, owns, ext, c->d_modup, c->d_mods, QP, c->alpha, ndig, c->log_n);
  else if (c->alpha <= 8)
    hipLaunchKernelGGL((modup_kernel<8, SP>), grid, dim3(EW_BLOCK), 0, c->stream, dc, dcs, own, owns, ext, c->d_modup, c->d_mods, QP, c->alpha, ndig, c->log_n);
  else
    hipLaunchKernelGGL((modup_kernel<16, SP>), grid, dim3(EW_BLOCK), 0, c->stream, dc, dcs, own, owns, ext, c->d_modup, c->d_mods, QP, c->alpha, ndig, c->log_n);
  return fhe_check(c, hipGetLastError(), "modup_kernel");
}

template <bool SP>
int inner_impl(fhe_ctx *c, const u64 *ext, const u64 *ksk, u64 *acc, u32 n, u32 ndig) {
  const u32 QP = c->L + c->K;
  hipLaunchKernelGGL((ks_inner_kernel<SP>), dim3(c->n / EW_BLOCK, n * QP), dim3(EW_BLOCK), 0, c->stream, ext, ksk, acc,
                     c->d_mods, QP, ndig, c->log_n);
  return fhe_check(c, hipGetLastError(), "ks_inner_kernel");
}

template <bool SP>
int combine_impl(fhe_ctx *c, const u64 *acc, const u64 *conv, const u64 *base, u64 *out, u32 n, u32 add_mask) {
  const u32 L = c->L, QP = c->L + c->K;
  hipLaunchKernelGGL((ks_combine_kernel<SP>), dim3(c->n / EW_BLOCK, n * 2 * L), dim3(EW_BLOCK), 0, c->stream, acc,
                     conv, base, out, c->d_pinv, c->d_mods, L, QP, c->log_n, add_mask);
  return fhe_check(c, hipGetLastError(), "ks_combine_kernel");
}

template <bool SP>
int tensor_impl(fhe_ctx *c, const TensorArgs &t, u32 jobs) {
  hipLaunchKernelGGL((tensor_kernel<SP>), dim3(c->n / EW_BLOCK, jobs), dim3(EW_BLOCK), 0, c->stream, t, c->d_mods);
  return fhe_check(c, hipGetLastError(), "tensor_kernel");
}

template <bool SP>
int behz_extend_impl(fhe_ctx *c, const u64 *xq, u64 *xb, u32 polys) {
  dim3 grid(c->n / EW_BLOCK, polys);
  const BehzDev *bz = (const BehzDev *)c->behz;
  if (c->L <= 8) hipLaunchKernelGGL((behz_extend_kernel<8, SP>), grid, dim3(EW_BLOCK), 0, c->stream, xq, xb, bz, c->d_mods, c->log_n);
  else if (c->L <= 16) hipLaunchKernelGGL((behz_extend_kernel<16, SP>), grid, dim3(EW_BLOCK), 0, c->stream, xq, xb, bz, c->d_mods, c->log_n);
  else hipLaunchKernelGGL((behz_extend_kernel<24, SP>), grid, dim3(EW_BLOCK), 0, c->stream, xq, xb, bz, c->d_mods, c->log_n);
  return fhe_check(c, hipGetLastError(), "behz_extend");
}

template <bool SP>
int behz_floor_impl(fhe_ctx *c, const u64 *eq, const u64 *eb, u64 *out01, u64 *out2, u32 n) {
  dim3 grid(c->n / EW_BLOCK, n * 3);
  const BehzDev *bz = (const BehzDev *)c->behz;
  if (c->L <= 8) hipLaunchKernelGGL((behz_floor_kernel<8, SP>), grid, dim3(EW_BLOCK), 0, c->stream, eq, eb, out01, out2, bz, c->d_mods, c->log_n);
  else if (c->L <= 16) hipLaunchKernelGGL((behz_floor_kernel<16, SP>), grid, dim3(EW_BLOCK), 0, c->stream, eq, eb, out01, out2, bz, c->d_mods, c->log_n);
  else hipLaunchKernelGGL((behz_floor_kernel<24, SP>), grid, dim3(EW_BLOCK), 0, c->stream, eq, eb, out01, out2, bz, c->d_mods, c->log_n);
  return fhe_check(c, hipGetLastError(), "behz_floor");
}

#define SP_DISPATCH(c, fn, ...) ((c)->special ? fn<true>(__VA_ARGS__) : fn<false>(__VA_ARGS__))

}  // namespace

// =================================================================== host

int ew_launch(fhe_ctx *c, EwOp op, const u64 *a, const u64 *b, u64 *out, u32 n_polys, u32 mod_begin, u32 n_limbs) {
  const u32 jobs = n_polys * n_limbs;
  if (!jobs) return FHE_OK;
  return SP_DISPATCH(c, ew_impl, c, op, a, b, out, jobs, mod_begin, n_limbs);
}

int fill_uniform_launch(fhe_ctx *c, u64 *data, u32 n_polys, u32 mod_begin, u32 n_limbs, u64 seed) {
  const u32 jobs = n_polys * n_limbs;
  if (!jobs) return FHE_OK;
  hipLaunchKernelGGL(fill_kernel, dim3(c->n / EW_BLOCK, jobs), dim3(EW_BLOCK), 0, c->stream, data, c->d_mods,
                     mod_begin, n_limbs, c->log_n, seed);
  return fhe_check(c, hipGetLastError(), "fill_kernel");
}

int conv_launch(fhe_ctx *c, const ConvTab &t, const u64 *src, u32 src_poly_stride, u64 *dst, u32 dst_poly_stride,
                u32 n) {
  if (!n) return FHE_OK;
  return SP_DISPATCH(c, conv_impl, c, t, src, src_poly_stride, dst, dst_poly_stride, n);
}

size_t keyswitch_ws_bytes(const fhe_ctx *c, u32 n) {
  const size_t N = c->n, L = c->L, QP = c->L + c->K;
  return sizeof(u64) * N * n * (L + c->dnum * QP + 2 * QP + 2 * L);
}

// Hybrid key switching, batched over n inputs (keyswitch_one, oracle).
//   d   : [n][d_stride limbs], the L limbs of item i at d + i*d_stride*N
//         (NTT form iff ntt_form, i.e. CKKS)
//   out : [n][2][L][N], out_b = (add_mask bit b ? base_b : 0) + KS(d)_b;
//         base may alias out (element-wise), d must not alias out.
int keyswitch_ex(fhe_ctx *c, const u64 *d, u32 d_stride, const u64 *ksk, const u64 *base, u64 *out, u32 n,
                 u32 add_mask, bool ntt_form, u64 *ws) {
  const u32 L = c->L, K = c->K, QP = L + K, N = c->n;
  const u32 ndig = (L + c->alpha - 1) / c->alpha;
  u64 *dc = ws;                                   // [n][L][N]
  u64 *ext = dc + (size_t)n * L * N;              // [n][ndig][QP][N]
  u64 *acc = ext + (size_t)n * ndig * QP * N;     // [n][2][QP][N]
  u64 *conv = acc + (size_t)n * 2 * QP * N;       // [n][2][L][N]
  int rc;
  // 1. coefficient-form copy of d
  rc = fhe_check(c, hipMemcpy2DAsync(dc, (size_t)L * N * 8, d, (size_t)d_stride * N * 8, (size_t)L * N * 8, n,
                                     hipMemcpyDeviceToDevice, c->stream), "ks copy");
  if (rc) return rc;
  if (ntt_form) {
    if ((rc = ntt_launch(c, LimbMap{dc, L, L, 0, L, 0, 0, n}, true))) return rc;
  }
  // 2. ModUp all digits.  Own limbs: NTT-form d for CKKS; coefficient-form dc for BFV (NTT'd below)
  if ((rc = SP_DISPATCH(c, modup_impl, c, dc, L, ntt_form ? d : dc, ntt_form ? d_stride : L, ext, n, ndig)))
    return rc;
  // 3. NTT the converted limbs (all limbs for BFV, whose own limbs are coefficient form)
  for (u32 j = 0; j < ndig; ++j) {
    const u32 lo = j * c->alpha, hi = std::min(lo + c->alpha, L);
    LimbMap m{ext + (size_t)j * QP * N, ndig * QP, ntt_form ? QP - (hi - lo) : QP, 0,
              ntt_form ? lo : QP, ntt_form ? hi - lo : 0, 0, n};
    if ((rc = ntt_launch(c, m, false))) return rc;
  }
  // 4. inner product with the key
  if ((rc = SP_DISPATCH(c, inner_impl, c, ext, ksk, acc, n, ndig))) return rc;
  // 5. ModDown: INTT the P part (all of Q u P for BFV), convert P -> Q
  if ((rc = ntt_launch(c, LimbMap{acc, QP, ntt_form ? K : QP, ntt_form ? L : 0, QP, 0, 0, 2 * n}, true))) return rc;
  if ((rc = conv_launch(c, c->moddown, acc + (size_t)L * N, QP, conv, L, 2 * n))) return rc;
  if (ntt_form) {
    if ((rc = ntt_launch(c, LimbMap{conv, L, L, 0, L, 0, 0, 2 * n}, false))) return rc;
  }
  // 6. combine
  return SP_DISPATCH(c, combine_impl, c, acc, conv, base, out, n, add_mask);
}

int tensor_launch(fhe_ctx *c, const u64 *a, size_t a_ct, size_t a_poly, const u64 *b, size_t b_ct, size_t b_poly,
                  u64 *e01, size_t e_ct, size_t e_poly, u64 *e2, size_t e2_ct, u32 n_ct, u32 nl, u32 mod_offset) {
  TensorArgs t{a, b, e01, e2, a_ct, a_poly, b_ct, b_poly, e_ct, e_poly, e2_ct, nl, mod_offset, c->log_n};
  return SP_DISPATCH(c, tensor_impl, c, t, n_ct * nl);
}

int automorph_launch(fhe_ctx *c, const u64 *in, u64 *out, u32 g, u32 n_polys, bool ntt_form) {
  const u32 jobs = n_polys * c->L;
  if (ntt_form) {
    hipLaunchKernelGGL(automorph_ntt_kernel, dim3(c->n / EW_BLOCK, jobs), dim3(EW_BLOCK), 0, c->stream, in, out, g,
                       c->log_n);
  } else {
    // g^-1 mod 2N (g odd): Newton iteration on the 2-adic inverse
    u32 inv = g;
    for (int i = 0; i < 5; ++i) inv *= 2u - g * inv;
    inv &= (2u * c->n) - 1;
    hipLaunchKernelGGL(automorph_coef_kernel, dim3(c->n / EW_BLOCK, jobs), dim3(EW_BLOCK), 0, c->stream, in, out,
                       inv, c->d_mods, c->L, c->log_n);
  }
  return fhe_check(c, hipGetLastError(), "automorph_kernel");
}

// ------------------------------------------------------------ BEHZ setup
int behz_setup(fhe_ctx *c) {
  const u32 L = c->L, nB = c->nB, bsk0 = c->L + c->K;
  if (L > BEHZ_MAXL) return fhe_fail(c, FHE_ERR_UNSUPPORTED, "BFV with L > 24");
  BehzDev *B = new BehzDev();
  std::memset(B, 0, sizeof(BehzDev));
  B->L = L; B->nB = nB; B->bsk0 = bsk0;
  const u64 *qq = c->moduli.data(), *bsk = c->moduli.data() + bsk0;
  const u64 msk = bsk[nB - 1];
  const u64 mt = 1ull << 32;
  auto M = host_mulmod;
  auto R = host_to_mont;
  for (u32 i = 0; i < L; ++i) {
    u64 qh = 1, hm = 1;
    for (u32 k = 0; k < L; ++k)
      if (k != i) { qh = M(qh, qq[k] % qq[i], qq[i]); hm = (hm * (qq[k] & 0xffffffffull)) & 0xffffffffull; }
    const u64 hinv = host_inv(qh, qq[i]);
    B->mt_hinv_R[i] = R(M(hinv, mt % qq[i], qq[i]), qq[i]);
    B->t_hinv_R[i] = R(M(hinv, c->t % qq[i], qq[i]), qq[i]);
    B->h_mod_mt[i] = (u32)hm;
    for (u32 j = 0; j < nB; ++j) {
      u64 p2 = 1;
      for (u32 k = 0; k < L; ++k) if (k != i) p2 = M(p2, qq[k] % bsk[j], bsk[j]);
      B->h_q_bsk_R[i][j] = R(p2, bsk[j]);
    }
    u64 bm = 1;
    for (u32 k = 0; k + 1 < nB; ++k) bm = M(bm, bsk[k] % qq[i], qq[i]);
    B->b_mod_q_R[i] = R(bm, qq[i]);
  }
  u64 qm = 1;
  for (u32 k = 0; k < L; ++k) qm = (qm * (qq[k] & 0xffffffffull)) & 0xffffffffull;
  u32 inv = (u32)qm;
  for (int it = 0; it < 5; ++it) inv *= 2u - (u32)qm * inv;
  B->neg_inv_q_mod_mt = 0u - inv;
  for (u32 j = 0; j < nB; ++j) {
    const u64 b = bsk[j];
    u64 qmb = 1;
    for (u32 k = 0; k < L; ++k) qmb = M(qmb, qq[k] % b, b);
    B->q_mod_bsk_R[j] = R(qmb, b);
    B->inv_q_bsk_R[j] = R(host_inv(qmb, b), b);
    B->inv_mt_bsk_R[j] = R(host_inv(mt % b, b), b);
    B->t_bsk_R[j] = R(c->t % b, b);
  }
  for (u32 j = 0; j + 1 < nB; ++j) {
    u64 bh = 1, bhm = 1;
    for (u32 k = 0; k + 1 < nB; ++k)
      if (k != j) { bh = M(bh, bsk[k] % bsk[j], bsk[j]); bhm = M(bhm, bsk[k] % msk, msk); }
    B->b_hinv_R[j] = R(host_inv(bh, bsk[j]), bsk[j]);
    B->h_b_msk_R[j] = R(bhm, msk);
    for (u32 i = 0; i < L; ++i) {
      u64 p2 = 1;
      for (u32 k = 0; k + 1 < nB; ++k) if (k != j) p2 = M(p2, bsk[k] % qq[i], qq[i]);
      B->h_b_q_R[j][i] = R(p2, qq[i]);
    }
  }
  u64 bmsk = 1;
  for (u32 k = 0; k + 1 < nB; ++k) bmsk = M(bmsk, bsk[k] % msk, msk);
  B->inv_b_msk_R = R(host_inv(bmsk, msk), msk);
  c->behz = ctx_upload(c, B, sizeof(BehzDev));
  delete B;
  return c->behz ? FHE_OK : FHE_ERR_OOM;
}

size_t bfv_mul_ws_bytes(const fhe_ctx *c, u32 n) {
  const size_t N = c->n, L = c->L, nB = c->nB;
  return sizeof(u64) * N * n * (4 * L + 4 * nB + 3 * L + 3 * nB + L) + keyswitch_ws_bytes(c, n);
}

int bfv_mul_relin_impl(fhe_ctx *c, const u64 *a, const u64 *b, const u64 *rlk, u64 *out, u32 n) {
  const u32 L = c->L, nB = c->nB, N = c->n, bsk0 = c->L + c->K;
  void *wsv;
  int rc = ctx_workspace(c, bfv_mul_ws_bytes(c, n), &wsv);
  if (rc) return rc;
  u64 *xq = (u64 *)wsv;                       // [n][4][L][N]
  u64 *xb = xq + (size_t)n * 4 * L * N;       // [n][4][nB][N]
  u64 *eq = xb + (size_t)n * 4 * nB * N;      // [n][3][L][N]
  u64 *eb = eq + (size_t)n * 3 * L * N;       // [n][3][nB][N]
  u64 *r2 = eb + (size_t)n * 3 * nB * N;      // [n][L][N]
  u64 *ksws = r2 + (size_t)n * L * N;
  const size_t ct_words = (size_t)2 * L * N, LN = (size_t)L * N, BN = (size_t)nB * N;
  // 1. gather a0,a1,b0,b1 per item
  if ((rc = fhe_check(c, hipMemcpy2DAsync(xq, 4 * LN * 8, a, ct_words * 8, ct_words * 8, n,
                                          hipMemcpyDeviceToDevice, c->stream), "bfv copy a")))
    return rc;
  if ((rc = fhe_check(c, hipMemcpy2DAsync(xq + ct_words, 4 * LN * 8, b, ct_words * 8, ct_words * 8, n,
                                          hipMemcpyDeviceToDevice, c->stream), "bfv copy b")))
    return rc;
  // 2. extend to Bsk (coefficient form)
  if ((rc = SP_DISPATCH(c, behz_extend_impl, c, xq, xb, n * 4))) return rc;
  // 3. NTT in Q and Bsk
  if ((rc = ntt_launch(c, LimbMap{xq, L, L, 0, L, 0, 0, 4 * n}, false))) return rc;
  if ((rc = ntt_launch(c, LimbMap{xb, nB, nB, 0, nB, 0, bsk0, 4 * n}, false))) return rc;
  // 4. tensor in both bases
  if ((rc = tensor_launch(c, xq, 4 * LN, LN, xq + 2 * LN, 4 * LN, LN, eq, 3 * LN, LN, eq + 2 * LN, 3 * LN, n, L, 0)))
    return rc;
  if ((rc = tensor_launch(c, xb, 4 * BN, BN, xb + 2 * BN, 4 * BN, BN, eb, 3 * BN, BN, eb + 2 * BN, 3 * BN, n, nB,
                          bsk0)))
    return rc;
  if ((rc = ntt_launch(c, LimbMap{eq, L, L, 0, L, 0, 0, 3 * n}, true))) return rc;
  if ((rc = ntt_launch(c, LimbMap{eb, nB, nB, 0, nB, 0, bsk0, 3 * n}, true))) return rc;
  // 5. scale and round: r0, r1 -> out, r2 -> workspace
  if ((rc = SP_DISPATCH(c, behz_floor_impl, c, eq, eb, out, r2, n))) return rc;
  // 6. relinearize r2 and add to (r0, r1)
  return keyswitch_ex(c, r2, L, rlk, out, out, n, 3u, false, ksws);
}
