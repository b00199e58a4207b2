// rns.hip -- element-wise RNS kernels, fast base conversion, hybrid key
// switching, automorphisms and BFV (BEHZ) scaling for gfx950.
//
// Every kernel here is a per-coefficient map over HBM-resident limb-polys:
// one thread per coefficient, consecutive lanes on consecutive coefficients
// (512 B per wave-instruction of u64), (item, limb) on gridDim.y.  They are
// HBM-bound apart from the 128-bit Barrett reductions; the CRT / Shoup
// constants are tiny and stay in L2.  Each kernel restates the oracle
// function named in its comment (oracle/fhe_oracle.c), which is how results
// are bit-identical: every step is exact modular arithmetic with the same
// formula, only the reduction strategy (lazy Shoup / Barrett) differs.
#include <algorithm>
#include <cstring>

#include "context.hpp"

#define EW_BLOCK 256

namespace {

// ------------------------------------------------------------ element-wise
template <EwOp OP>
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
  else r = mul_mod(x, y, m);
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
// The dot product is accumulated exactly in 128 bits (ns <= 16 terms of
// < 2^124 each) and reduced once with Barrett.
template <int NS>
__device__ __forceinline__ void conv_coef(const ConvTab &t, const ModInfo *mods, const u64 *s, size_t s_step,
                                          u64 *d, size_t d_step) {
  u64 v[NS];
#pragma unroll
  for (int i = 0; i < NS; ++i) {
    if (i < (int)t.ns) {
      const Tw h = t.hinv[i];
      v[i] = shoup(s[i * s_step], h.w, h.ws, mods[t.src_mod[i]].q);
    }
  }
  for (u32 m = 0; m < t.nd; ++m) {
    U128 acc{0, 0};
    const u64 *hm = t.h + m;
#pragma unroll
    for (int i = 0; i < NS; ++i)
      if (i < (int)t.ns) mac128(acc, v[i], hm[(size_t)i * t.nd]);
    d[m * d_step] = reduce128(acc, mods[t.dst_mod[m]]);
  }
}

template <int NS>
__global__ void __launch_bounds__(EW_BLOCK) conv_kernel(const u64 *__restrict__ src, u32 src_stride,
                                                        u64 *__restrict__ dst, u32 dst_stride, ConvTab t,
                                                        const ModInfo *mods, u32 log_n) {
  const u32 k = blockIdx.x * EW_BLOCK + threadIdx.x;
  const u32 p = blockIdx.y;
  const size_t N = (size_t)1 << log_n;
  conv_coef<NS>(t, mods, src + p * src_stride * N + k, N, dst + p * dst_stride * N + k, N);
}

// ModUp of one digit (keyswitch_one, oracle): the digit's own limbs are copied
// from `own` (NTT form for CKKS, coefficient form for BFV), every other limb
// of Q u P is the fast base conversion of the digit's coefficient-form limbs.
template <int NS>
__global__ void __launch_bounds__(EW_BLOCK) modup_kernel(const u64 *__restrict__ dc, u32 dc_stride,
                                                         const u64 *__restrict__ own, u32 own_stride,
                                                         u64 *__restrict__ ext, const ConvTab *tabs,
                                                         const ModInfo *mods, u32 L, u32 QP, u32 alpha, u32 dnum,
                                                         u32 log_n) {
  const u32 k = blockIdx.x * EW_BLOCK + threadIdx.x;
  const u32 ct = blockIdx.y / dnum, j = blockIdx.y % dnum;
  const size_t N = (size_t)1 << log_n;
  const u32 lo = j * alpha;
  const ConvTab t = tabs[j];
  u64 *e = ext + ((size_t)(ct * dnum + j) * QP) * N + k;
  for (u32 i = 0; i < t.ns; ++i) e[(lo + i) * N] = own[((size_t)ct * own_stride + lo + i) * N + k];
  const u64 *s = dc + ((size_t)ct * dc_stride + lo) * N + k;
  // destinations are limbs of Q u P: dst_mod[m] is also the limb index
  u64 v[NS];
#pragma unroll
  for (int i = 0; i < NS; ++i) {
    if (i < (int)t.ns) {
      const Tw h = t.hinv[i];
      v[i] = shoup(s[i * N], h.w, h.ws, mods[lo + i].q);
    }
  }
  for (u32 m = 0; m < t.nd; ++m) {
    U128 acc{0, 0};
#pragma unroll
    for (int i = 0; i < NS; ++i)
      if (i < (int)t.ns) mac128(acc, v[i], t.h[(size_t)i * t.nd + m]);
    const u32 dm = t.dst_mod[m];
    e[dm * N] = reduce128(acc, mods[dm]);
  }
}

// KS inner product (keyswitch_one, oracle):
//   acc_b[i] = sum_j ext_j[i] * ksk[j][b][i]  mod m_i,  b in {0,1}
__global__ void __launch_bounds__(EW_BLOCK) ks_inner_kernel(const u64 *__restrict__ ext, const u64 *__restrict__ ksk,
                                                            u64 *__restrict__ acc, const ModInfo *mods, u32 QP,
                                                            u32 dnum, u32 ndig, u32 log_n) {
  const u32 k = blockIdx.x * EW_BLOCK + threadIdx.x;
  const u32 ct = blockIdx.y / QP, i = blockIdx.y % QP;
  const size_t N = (size_t)1 << log_n;
  const ModInfo m = mods[i];
  U128 a0{0, 0}, a1{0, 0};
  for (u32 j = 0; j < ndig; ++j) {
    const u64 x = ext[((size_t)(ct * dnum + j) * QP + i) * N + k];
    const u64 k0 = ksk[((size_t)(2 * j) * QP + i) * N + k];
    const u64 k1 = ksk[((size_t)(2 * j + 1) * QP + i) * N + k];
    mac128(a0, x, k0);
    mac128(a1, x, k1);
    if ((j & 3) == 3 && j + 1 < ndig) {  // keep the 128-bit sums below q * 2^64
      a0 = U128{reduce128(a0, m), 0};
      a1 = U128{reduce128(a1, m), 0};
    }
  }
  acc[((size_t)(2 * ct) * QP + i) * N + k] = reduce128(a0, m);
  acc[((size_t)(2 * ct + 1) * QP + i) * N + k] = reduce128(a1, m);
}

// ModDown finish: out_b[i] = base_b[i] + (acc_b[i] - conv_b[i]) * P^-1 mod q_i
__global__ void __launch_bounds__(EW_BLOCK) ks_combine_kernel(const u64 *__restrict__ acc,
                                                              const u64 *__restrict__ conv, const u64 *base,
                                                              u64 *out, const Tw *pinv, const ModInfo *mods, u32 L,
                                                              u32 QP, u32 log_n, u32 add_mask) {
  const u32 k = blockIdx.x * EW_BLOCK + threadIdx.x;
  const u32 ct = blockIdx.y / (2 * L), r = blockIdx.y % (2 * L), b = r / L, i = r % L;
  const size_t N = (size_t)1 << log_n;
  const u64 q = mods[i].q;
  const u64 a = acc[((size_t)(2 * ct + b) * QP + i) * N + k];
  const u64 cv = conv[((size_t)(2 * ct + b) * L + i) * N + k];
  const Tw pi = pinv[i];
  u64 ks = shoup(sub_mod(a, cv, q), pi.w, pi.ws, q);
  const size_t o = ((size_t)(2 * ct + b) * L + i) * N + k;
  if (add_mask & (1u << b)) ks = add_mod(ks, base[o], q);
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
__global__ void __launch_bounds__(EW_BLOCK) tensor_kernel(TensorArgs t, const ModInfo *mods) {
  const u32 k = blockIdx.x * EW_BLOCK + threadIdx.x;
  const u32 ct = blockIdx.y / t.nl, l = blockIdx.y % t.nl;
  const size_t off = ((size_t)l << t.log_n) + k;
  const ModInfo m = mods[t.mod_offset + l];
  const u64 *A = t.a + ct * t.a_ct + off, *B = t.b + ct * t.b_ct + off;
  const u64 a0 = A[0], a1 = A[t.a_poly], b0 = B[0], b1 = B[t.b_poly];
  u64 *E = t.e01 + ct * t.e_ct + off;
  E[0] = mul_mod(a0, b0, m);
  U128 s = mul128(a0, b1);
  mac128(s, a1, b0);
  E[t.e_poly] = reduce128(s, m);
  t.e2[ct * t.e2_ct + off] = mul_mod(a1, b1, m);
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
#define BEHZ_MAXL 24
struct BehzDev {
  u32 L, nB, bsk0;                 // bsk0 = first Bsk modulus id
  u32 neg_inv_q_mod_mt;
  u32 h_mod_mt[BEHZ_MAXL];         // (Q/q_i) mod 2^32
  Tw mt_hinv[BEHZ_MAXL];           // 2^32 (Q/q_i)^-1 mod q_i
  Tw q_hinv[BEHZ_MAXL];            // (Q/q_i)^-1 mod q_i
  Tw t_q[BEHZ_MAXL];               // t mod q_i
  u64 q_mod_bsk[BEHZ_MAXL + 1];    // Q mod b
  Tw inv_mt_bsk[BEHZ_MAXL + 1];    // 2^-32 mod b
  Tw inv_q_bsk[BEHZ_MAXL + 1];     // Q^-1 mod b
  Tw t_bsk[BEHZ_MAXL + 1];         // t mod b
  Tw b_hinv[BEHZ_MAXL];            // (B/b_j)^-1 mod b_j
  u64 h_b_msk[BEHZ_MAXL];          // (B/b_j) mod m_sk
  Tw inv_b_msk;                    // B^-1 mod m_sk
  u64 b_mod_q[BEHZ_MAXL];          // B mod q_i
  u64 h_q_bsk[BEHZ_MAXL][BEHZ_MAXL + 1];  // (Q/q_i) mod b
  u64 h_b_q[BEHZ_MAXL][BEHZ_MAXL];        // (B/b_j) mod q_i
};

// behz_extend (oracle): fastbconv_m_tilde then sm_mrq.  x [L] coef -> [nB] coef
template <int NL>
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
    if (i < (int)L) {
      const Tw h = bz->mt_hinv[i];
      v[i] = shoup(s[i * N], h.w, h.ws, mods[i].q);
      xmt += (u32)v[i] * bz->h_mod_mt[i];
    }
  }
  const u32 r = xmt * bz->neg_inv_q_mod_mt;
  u64 *d = xb + (size_t)p * nB * N + k;
  for (u32 j = 0; j < nB; ++j) {
    const ModInfo m = mods[bz->bsk0 + j];
    U128 acc{0, 0};
#pragma unroll
    for (int i = 0; i < NL; ++i)
      if (i < (int)L) mac128(acc, v[i], bz->h_q_bsk[i][j]);
    const u64 xbj = reduce128(acc, m);
    const u64 rr = r >= 0x80000000u ? (u64)r + m.q - (1ull << 32) : (u64)r;
    const u64 sum = add_mod(xbj, mul_mod(bz->q_mod_bsk[j], rr, m), m.q);
    const Tw im = bz->inv_mt_bsk[j];
    d[j * N] = shoup(sum, im.w, im.ws, m.q);
  }
}

// behz_floor_to_q (oracle): fast_floor in Bsk then fastbconv_sk back to Q.
template <int NL>
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
    if (i < (int)L) {
      const u64 q = mods[i].q;
      const Tw tq = bz->t_q[i], h = bz->q_hinv[i];
      v[i] = shoup(shoup(xq[i * N], tq.w, tq.ws, q), h.w, h.ws, q);
    }
  }
  u64 fl[NL + 1];
#pragma unroll
  for (int j = 0; j < NL + 1; ++j) {
    if (j < (int)nB) {
      const ModInfo m = mods[bz->bsk0 + j];
      U128 acc{0, 0};
#pragma unroll
      for (int i = 0; i < NL; ++i)
        if (i < (int)L) mac128(acc, v[i], bz->h_q_bsk[i][j]);
      const u64 cv = reduce128(acc, m);
      const Tw tb = bz->t_bsk[j], iq = bz->inv_q_bsk[j];
      const u64 tx = shoup(xb[j * N], tb.w, tb.ws, m.q);
      fl[j] = shoup(sub_mod(tx, cv, m.q), iq.w, iq.ws, m.q);
    }
  }
  // fastbconv_sk
  u64 w[NL];
  U128 am{0, 0};
#pragma unroll
  for (int j = 0; j < NL; ++j) {
    if (j < (int)nB - 1) {
      const Tw h = bz->b_hinv[j];
      w[j] = shoup(fl[j], h.w, h.ws, mods[bz->bsk0 + j].q);
      mac128(am, w[j], bz->h_b_msk[j]);
    }
  }
  const ModInfo msk = mods[bz->bsk0 + nB - 1];
  u64 flsk = 0;
#pragma unroll
  for (int j = 0; j < NL + 1; ++j)
    if (j == (int)nB - 1) flsk = fl[j];
  const u64 cmsk = reduce128(am, msk);
  const Tw ib = bz->inv_b_msk;
  const u64 alpha = shoup(sub_mod(cmsk, flsk, msk.q), ib.w, ib.ws, msk.q);
  const bool neg = alpha > msk.q / 2;
  u64 *o = (p < 2) ? out01 + ((size_t)(ct * 2 + p) * L) * N + k : out2 + ((size_t)ct * L) * N + k;
  for (u32 i = 0; i < L; ++i) {
    const ModInfo m = mods[i];
    U128 acc{0, 0};
#pragma unroll
    for (int j = 0; j < NL; ++j)
      if (j < (int)nB - 1) mac128(acc, w[j], bz->h_b_q[j][i]);
    u64 cq = reduce128(acc, m);
    if (neg) {
      const u64 a = msk.q - alpha;  // < 2^61, fine as a mul_mod operand
      cq = add_mod(cq, mul_mod(bz->b_mod_q[i], a, m), m.q);
    } else {
      cq = sub_mod(cq, mul_mod(bz->b_mod_q[i], alpha, m), m.q);
    }
    o[i * N] = cq;
  }
}

}  // namespace

// =================================================================== host

int ew_launch(fhe_ctx *c, EwOp op, const u64 *a, const u64 *b, u64 *out, u32 n_polys, u32 mod_begin, u32 n_limbs) {
  const u32 jobs = n_polys * n_limbs;
  if (!jobs) return FHE_OK;
  dim3 grid(c->n / EW_BLOCK, jobs);
  switch (op) {
    case EwOp::Add: hipLaunchKernelGGL(ew_kernel<EwOp::Add>, grid, dim3(EW_BLOCK), 0, c->stream, a, b, out, c->d_mods, mod_begin, n_limbs, c->log_n); break;
    case EwOp::Sub: hipLaunchKernelGGL(ew_kernel<EwOp::Sub>, grid, dim3(EW_BLOCK), 0, c->stream, a, b, out, c->d_mods, mod_begin, n_limbs, c->log_n); break;
    case EwOp::Mul: hipLaunchKernelGGL(ew_kernel<EwOp::Mul>, grid, dim3(EW_BLOCK), 0, c->stream, a, b, out, c->d_mods, mod_begin, n_limbs, c->log_n); break;
  }
  return fhe_check(c, hipGetLastError(), "ew_kernel");
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
  dim3 grid(c->n / EW_BLOCK, n);
  if (t.ns <= 4) hipLaunchKernelGGL(conv_kernel<4>, grid, dim3(EW_BLOCK), 0, c->stream, src, src_poly_stride, dst, dst_poly_stride, t, c->d_mods, c->log_n);
  else if (t.ns <= 8) hipLaunchKernelGGL(conv_kernel<8>, grid, dim3(EW_BLOCK), 0, c->stream, src, src_poly_stride, dst, dst_poly_stride, t, c->d_mods, c->log_n);
  else if (t.ns <= 16) hipLaunchKernelGGL(conv_kernel<16>, grid, dim3(EW_BLOCK), 0, c->stream, src, src_poly_stride, dst, dst_poly_stride, t, c->d_mods, c->log_n);
  else return fhe_fail(c, FHE_ERR_UNSUPPORTED, "base conversion with more than 16 source moduli");
  return fhe_check(c, hipGetLastError(), "conv_kernel");
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
  u64 *dc = ws;                                   // [n][L][N]
  u64 *ext = dc + (size_t)n * L * N;              // [n][dnum][QP][N]
  u64 *acc = ext + (size_t)n * c->dnum * QP * N;  // [n][2][QP][N]
  u64 *conv = acc + (size_t)n * 2 * QP * N;       // [n][2][L][N]
  int rc;
  // 1. coefficient-form copy of d
  rc = fhe_check(c, hipMemcpy2DAsync(dc, (size_t)L * N * 8, d, (size_t)d_stride * N * 8, (size_t)L * N * 8, n,
                                     hipMemcpyDeviceToDevice, c->stream), "ks copy");
  if (rc) return rc;
  if (ntt_form) {
    LimbMap m{dc, L, L, 0, L, 0, 0, n};
    if ((rc = ntt_launch(c, m, true))) return rc;
  }
  // 2. ModUp all digits
  const u32 ndig = (L + c->alpha - 1) / c->alpha;
  {
    dim3 grid(N / EW_BLOCK, n * ndig);
    // own limbs: NTT-form d for CKKS; coefficient-form dc for BFV (NTT'd below)
    const u64 *own = ntt_form ? d : dc;
    const u32 own_stride = ntt_form ? d_stride : L;
    const ConvTab *tabs = c->d_modup;
    if (c->alpha <= 4)
      hipLaunchKernelGGL(modup_kernel<4>, grid, dim3(EW_BLOCK), 0, c->stream, dc, L, own, own_stride, ext, tabs, c->d_mods, L, QP, c->alpha, ndig, c->log_n);
    else if (c->alpha <= 8)
      hipLaunchKernelGGL(modup_kernel<8>, grid, dim3(EW_BLOCK), 0, c->stream, dc, L, own, own_stride, ext, tabs, c->d_mods, L, QP, c->alpha, ndig, c->log_n);
    else if (c->alpha <= 16)
      hipLaunchKernelGGL(modup_kernel<16>, grid, dim3(EW_BLOCK), 0, c->stream, dc, L, own, own_stride, ext, tabs, c->d_mods, L, QP, c->alpha, ndig, c->log_n);
    else
      return fhe_fail(c, FHE_ERR_UNSUPPORTED, "alpha > 16");
    if ((rc = fhe_check(c, hipGetLastError(), "modup_kernel"))) return rc;
  }
  // 3. NTT the converted limbs (all limbs for BFV, whose own limbs are coefficient form)
  for (u32 j = 0; j < ndig; ++j) {
    const u32 lo = j * c->alpha, hi = std::min(lo + c->alpha, L);
    LimbMap m{ext + (size_t)j * QP * N, ndig * QP, ntt_form ? QP - (hi - lo) : QP, 0,
              ntt_form ? lo : QP, ntt_form ? hi - lo : 0, 0, n};
    if ((rc = ntt_launch(c, m, false))) return rc;
  }
  // 4. inner product with the key
  hipLaunchKernelGGL(ks_inner_kernel, dim3(N / EW_BLOCK, n * QP), dim3(EW_BLOCK), 0, c->stream, ext, ksk, acc,
                     c->d_mods, QP, ndig, ndig, c->log_n);
  if ((rc = fhe_check(c, hipGetLastError(), "ks_inner_kernel"))) return rc;
  // 5. ModDown: INTT the P part (all of Q u P for BFV), convert P -> Q
  {
    LimbMap m{acc, QP, ntt_form ? K : QP, ntt_form ? L : 0, QP, 0, 0, 2 * n};
    if ((rc = ntt_launch(c, m, true))) return rc;
  }
  if ((rc = conv_launch(c, c->moddown, acc + (size_t)L * N, QP, conv, L, 2 * n))) return rc;
  if (ntt_form) {
    LimbMap m{conv, L, L, 0, L, 0, 0, 2 * n};
    if ((rc = ntt_launch(c, m, false))) return rc;
  }
  // 6. combine
  hipLaunchKernelGGL(ks_combine_kernel, dim3(N / EW_BLOCK, n * 2 * L), dim3(EW_BLOCK), 0, c->stream, acc, conv, base,
                     out, c->d_pinv, c->d_mods, L, QP, c->log_n, add_mask);
  return fhe_check(c, hipGetLastError(), "ks_combine_kernel");
}

int tensor_launch(fhe_ctx *c, const u64 *a, size_t a_ct, size_t a_poly, const u64 *b, size_t b_ct, size_t b_poly,
                  u64 *e01, size_t e_ct, size_t e_poly, u64 *e2, size_t e2_ct, u32 n_ct, u32 nl, u32 mod_offset) {
  TensorArgs t{a, b, e01, e2, a_ct, a_poly, b_ct, b_poly, e_ct, e_poly, e2_ct, nl, mod_offset, c->log_n};
  hipLaunchKernelGGL(tensor_kernel, dim3(c->n / EW_BLOCK, n_ct * nl), dim3(EW_BLOCK), 0, c->stream, t, c->d_mods);
  return fhe_check(c, hipGetLastError(), "tensor_kernel");
}

int automorph_launch(fhe_ctx *c, const u64 *in, u64 *out, u32 g, u32 n_polys, bool ntt_form) {
  const u32 jobs = n_polys * c->L;
  if (ntt_form) {
    hipLaunchKernelGGL(automorph_ntt_kernel, dim3(c->n / EW_BLOCK, jobs), dim3(EW_BLOCK), 0, c->stream, in, out, g,
                       c->log_n);
  } else {
    // g^-1 mod 2N (g odd): Newton iteration on 2-adic inverse
    u32 inv = g;
    for (int i = 0; i < 5; ++i) inv *= 2u - g * inv;
    inv &= (2u * c->n) - 1;
    hipLaunchKernelGGL(automorph_coef_kernel, dim3(c->n / EW_BLOCK, jobs), dim3(EW_BLOCK), 0, c->stream, in, out,
                       inv, c->d_mods, c->L, c->log_n);
  }
  return fhe_check(c, hipGetLastError(), "automorph_kernel");
}

// ------------------------------------------------------------ BEHZ setup
static u64 h_mulmod(u64 a, u64 b, u64 q) { return (u64)(((unsigned __int128)a * b) % q); }
static u64 h_pow(u64 b, u64 e, u64 q) {
  u64 r = 1 % q;
  b %= q;
  while (e) {
    if (e & 1) r = h_mulmod(r, b, q);
    b = h_mulmod(b, b, q);
    e >>= 1;
  }
  return r;
}
static u64 h_inv(u64 a, u64 q) { return h_pow(a % q, q - 2, q); }
static Tw h_tw(u64 w, u64 q) { return Tw{w, (u64)(((unsigned __int128)w << 64) / q)}; }

int behz_setup(fhe_ctx *c) {
  const u32 L = c->L, nB = c->nB, bsk0 = c->L + c->K;
  if (L > BEHZ_MAXL) return fhe_fail(c, FHE_ERR_UNSUPPORTED, "BFV with L > 24");
  BehzDev *B = new BehzDev();
  std::memset(B, 0, sizeof(BehzDev));
  B->L = L; B->nB = nB; B->bsk0 = bsk0;
  const u64 *qq = c->moduli.data(), *bsk = c->moduli.data() + bsk0;
  const u64 msk = bsk[nB - 1];
  const u64 mt = 1ull << 32;
  for (u32 i = 0; i < L; ++i) {
    u64 qh = 1, hm = 1;
    for (u32 k = 0; k < L; ++k)
      if (k != i) { qh = h_mulmod(qh, qq[k] % qq[i], qq[i]); hm = (hm * (qq[k] & 0xffffffffull)) & 0xffffffffull; }
    const u64 hinv = h_inv(qh, qq[i]);
    B->q_hinv[i] = h_tw(hinv, qq[i]);
    B->mt_hinv[i] = h_tw(h_mulmod(hinv, mt % qq[i], qq[i]), qq[i]);
    B->h_mod_mt[i] = (u32)hm;
    B->t_q[i] = h_tw(c->t % qq[i], qq[i]);
    for (u32 j = 0; j < nB; ++j) {
      u64 p2 = 1;
      for (u32 k = 0; k < L; ++k) if (k != i) p2 = h_mulmod(p2, qq[k] % bsk[j], bsk[j]);
      B->h_q_bsk[i][j] = p2;
    }
    u64 bm = 1;
    for (u32 k = 0; k + 1 < nB; ++k) bm = h_mulmod(bm, bsk[k] % qq[i], qq[i]);
    B->b_mod_q[i] = bm;
  }
  u64 qm = 1;
  for (u32 k = 0; k < L; ++k) qm = (qm * (qq[k] & 0xffffffffull)) & 0xffffffffull;
  u32 inv = (u32)qm;
  for (int it = 0; it < 5; ++it) inv *= 2u - (u32)qm * inv;
  B->neg_inv_q_mod_mt = 0u - inv;
  for (u32 j = 0; j < nB; ++j) {
    const u64 b = bsk[j];
    u64 qmb = 1;
    for (u32 k = 0; k < L; ++k) qmb = h_mulmod(qmb, qq[k] % b, b);
    B->q_mod_bsk[j] = qmb;
    B->inv_q_bsk[j] = h_tw(h_inv(qmb, b), b);
    B->inv_mt_bsk[j] = h_tw(h_inv(mt % b, b), b);
    B->t_bsk[j] = h_tw(c->t % b, b);
  }
  for (u32 j = 0; j + 1 < nB; ++j) {
    u64 bh = 1, bhm = 1;
    for (u32 k = 0; k + 1 < nB; ++k)
      if (k != j) { bh = h_mulmod(bh, bsk[k] % bsk[j], bsk[j]); bhm = h_mulmod(bhm, bsk[k] % msk, msk); }
    B->b_hinv[j] = h_tw(h_inv(bh, bsk[j]), bsk[j]);
    B->h_b_msk[j] = bhm;
    for (u32 i = 0; i < L; ++i) {
      u64 p2 = 1;
      for (u32 k = 0; k + 1 < nB; ++k) if (k != j) p2 = h_mulmod(p2, bsk[k] % qq[i], qq[i]);
      B->h_b_q[j][i] = p2;
    }
  }
  u64 bmsk = 1;
  for (u32 k = 0; k + 1 < nB; ++k) bmsk = h_mulmod(bmsk, bsk[k] % msk, msk);
  B->inv_b_msk = h_tw(h_inv(bmsk, msk), msk);
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
  const size_t ct_words = (size_t)2 * L * N;
  // 1. gather a0,a1,b0,b1 per item
  if ((rc = fhe_check(c, hipMemcpy2DAsync(xq, 4 * (size_t)L * N * 8, a, ct_words * 8, ct_words * 8, n,
                                          hipMemcpyDeviceToDevice, c->stream), "bfv copy a")))
    return rc;
  if ((rc = fhe_check(c, hipMemcpy2DAsync(xq + ct_words, 4 * (size_t)L * N * 8, b, ct_words * 8, ct_words * 8, n,
                                          hipMemcpyDeviceToDevice, c->stream), "bfv copy b")))
    return rc;
  // 2. extend to Bsk (coefficient form)
  {
    dim3 grid(N / EW_BLOCK, n * 4);
    const BehzDev *bz = (const BehzDev *)c->behz;
    if (L <= 8) hipLaunchKernelGGL(behz_extend_kernel<8>, grid, dim3(EW_BLOCK), 0, c->stream, xq, xb, bz, c->d_mods, c->log_n);
    else if (L <= 16) hipLaunchKernelGGL(behz_extend_kernel<16>, grid, dim3(EW_BLOCK), 0, c->stream, xq, xb, bz, c->d_mods, c->log_n);
    else hipLaunchKernelGGL(behz_extend_kernel<24>, grid, dim3(EW_BLOCK), 0, c->stream, xq, xb, bz, c->d_mods, c->log_n);
    if ((rc = fhe_check(c, hipGetLastError(), "behz_extend"))) return rc;
  }
  // 3. NTT in Q and Bsk
  if ((rc = ntt_launch(c, LimbMap{xq, L, L, 0, L, 0, 0, 4 * n}, false))) return rc;
  if ((rc = ntt_launch(c, LimbMap{xb, nB, nB, 0, nB, 0, bsk0, 4 * n}, false))) return rc;
  // 4. tensor in both bases
  if ((rc = tensor_launch(c, xq, 4 * (size_t)L * N, (size_t)L * N, xq + 2 * (size_t)L * N, 4 * (size_t)L * N,
                          (size_t)L * N, eq, 3 * (size_t)L * N, (size_t)L * N, eq + 2 * (size_t)L * N,
                          3 * (size_t)L * N, n, L, 0)))
    return rc;
  if ((rc = tensor_launch(c, xb, 4 * (size_t)nB * N, (size_t)nB * N, xb + 2 * (size_t)nB * N, 4 * (size_t)nB * N,
                          (size_t)nB * N, eb, 3 * (size_t)nB * N, (size_t)nB * N, eb + 2 * (size_t)nB * N,
                          3 * (size_t)nB * N, n, nB, bsk0)))
    return rc;
  if ((rc = ntt_launch(c, LimbMap{eq, L, L, 0, L, 0, 0, 3 * n}, true))) return rc;
  if ((rc = ntt_launch(c, LimbMap{eb, nB, nB, 0, nB, 0, bsk0, 3 * n}, true))) return rc;
  // 5. scale and round: r0, r1 -> out, r2 -> workspace
  {
    dim3 grid(N / EW_BLOCK, n * 3);
    const BehzDev *bz = (const BehzDev *)c->behz;
    if (L <= 8) hipLaunchKernelGGL(behz_floor_kernel<8>, grid, dim3(EW_BLOCK), 0, c->stream, eq, eb, out, r2, bz, c->d_mods, c->log_n);
    else if (L <= 16) hipLaunchKernelGGL(behz_floor_kernel<16>, grid, dim3(EW_BLOCK), 0, c->stream, eq, eb, out, r2, bz, c->d_mods, c->log_n);
    else hipLaunchKernelGGL(behz_floor_kernel<24>, grid, dim3(EW_BLOCK), 0, c->stream, eq, eb, out, r2, bz, c->d_mods, c->log_n);
    if ((rc = fhe_check(c, hipGetLastError(), "behz_floor"))) return rc;
  }
  // 6. relinearize r2 and add to (r0, r1)
  return keyswitch_ex(c, r2, L, rlk, out, out, n, 3u, false, ksws);
}
