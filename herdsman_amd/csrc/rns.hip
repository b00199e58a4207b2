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
#include <vector>

#include "context.hpp"

#define EW_BLOCK 256

namespace {

// Streaming stores/loads for data that is written or read exactly once per
// kernel and consumed by a later kernel (far larger than L2/MALL).
template <typename T>
__device__ __forceinline__ void st_nt(T *p, T v) { __builtin_nontemporal_store(v, p); }
template <typename T>
__device__ __forceinline__ T ld_nt(const T *p) { return __builtin_nontemporal_load(p); }

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
                                                        u32 log_n, u64 seed, u32 job0) {
  const u32 k = blockIdx.x * EW_BLOCK + threadIdx.x;
  const u32 job = job0 + blockIdx.y;  // the stream index is global over chunked launches
  const u64 q = mods[mod_begin + job % n_limbs].q;
  const size_t w = ((size_t)job << log_n) + k;
  out[w] = mulhi64(stream_word(seed, w), q);
}

// --------------------------------------------------------- base conversion
#define CONV_MAX_ND 48
// Conversion tables of one workgroup's ConvTab staged in LDS once, so the
// per-target loop of conv_store issues no dependent global/scalar loads.
template <int NS>
struct ConvLds {
  u64 h[NS * CONV_MAX_ND];
  u64 q[CONV_MAX_ND];
  u64 aux[CONV_MAX_ND];  // q_hi (special) or -q^-1 (generic)
  u32 dm[CONV_MAX_ND];
};
template <int NS, bool SP>
__device__ __forceinline__ void conv_stage(ConvLds<NS> &sh, const ConvTab &t, const ModInfo *mods) {
  for (u32 x = threadIdx.x; x < t.ns * t.nd; x += EW_BLOCK) sh.h[x] = t.h[x];
  for (u32 x = threadIdx.x; x < t.nd; x += EW_BLOCK) {
    const u32 dm = t.dst_mod[x];
    const ModInfo mi = mods[dm];
    sh.dm[x] = dm;
    sh.q[x] = mi.q;
    sh.aux[x] = SP ? mi.q_hi : mi.qinv_neg;
  }
}
// y_m = sum_i v_i h[i][m] for every target m, streamed to out[slot(m) * N]
// (slot = the target's modulus id when by_mod, else m), for the CPT
// coefficients of this thread (at stride EW_BLOCK)
// LAZY: outputs in the forward NTT's input range (dot_mont_lazy), for a
// conversion transformed next (ModUp)
template <int NS, bool SP, int CPT, bool LAZY = false>
__device__ __forceinline__ void conv_store(const ConvLds<NS> &sh, const u64 (&v)[CPT][NS], u32 ns, u32 nd, u64 *out,
                                           size_t N, bool by_mod, u32 mod_base) {
#pragma unroll 1
  for (u32 m = 0; m < nd; ++m) {
    ModInfo mi;
    mi.q = sh.q[m];
    mi.q_hi = (u32)sh.aux[m];
    mi.qinv_neg = sh.aux[m];
    u64 *o = out + (by_mod ? sh.dm[m] - mod_base : m) * N;
#pragma unroll
    for (int c = 0; c < CPT; ++c)
      st_nt(o + c * EW_BLOCK, LAZY ? dot_mont_lazy<NS, SP>(v[c], sh.h + m, nd, ns, mi)
                                   : dot_mont<NS, SP>(v[c], sh.h + m, nd, ns, mi));
  }
}

// Coefficients per thread of the conversion kernels: the per-workgroup table
// staging (a chain of dependent loads and a barrier) is amortised over
// CPT * EW_BLOCK coefficients, each thread has CPT * ns source loads in
// flight, and they are issued before the staging so their latency overlaps it.
constexpr int CONV_CPT = 2;

// v_i = [x_i (S/s_i)^-1]_{s_i} for the CPT coefficients (source i uses
// modulus src_mod[i], or mod0 + i when src_mod is null)
template <int NS, bool SP>
__device__ __forceinline__ void conv_scale(u64 (&v)[CONV_CPT][NS], const u64 (&x)[CONV_CPT][NS], const ConvTab &t,
                                           const ModInfo *mods, const u32 *src_mod, u32 mod0) {
#pragma unroll
  for (int i = 0; i < NS; ++i) {
    const bool on = i < (int)t.ns;
    const ModInfo ms = mods[src_mod ? src_mod[on ? i : 0] : mod0 + (on ? i : 0)];
    const u64 hv = t.hinv[on ? i : 0];
#pragma unroll
    for (int c = 0; c < CONV_CPT; ++c) v[c][i] = on ? csub63(mont_mul<SP>(x[c][i], hv, ms), ms.q) : 0;
  }
}

// conv_apply (oracle): v_i = [x_i (S/s_i)^-1]_{s_i};  y_m = sum_i v_i [S/s_i]_{d_m} mod d_m.
template <int NS, bool SP>
__global__ void __launch_bounds__(EW_BLOCK) conv_kernel(const u64 *__restrict__ src, u32 src_stride,
                                                        u64 *__restrict__ dst, u32 dst_stride, ConvTab t,
                                                        const ModInfo *mods, u32 log_n) {
  __shared__ ConvLds<NS> sh;
  const u32 k = blockIdx.x * (EW_BLOCK * CONV_CPT) + threadIdx.x;
  const u32 p = blockIdx.y;
  const size_t N = (size_t)1 << log_n;
  const u64 *s = src + (size_t)p * src_stride * N + k;
  u64 x[CONV_CPT][NS];
#pragma unroll
  for (int i = 0; i < NS; ++i)
#pragma unroll
    for (int c = 0; c < CONV_CPT; ++c) x[c][i] = i < (int)t.ns ? ld_nt(s + i * N + c * EW_BLOCK) : 0;
  conv_stage<NS, SP>(sh, t, mods);
  u64 v[CONV_CPT][NS];
  conv_scale<NS, SP>(v, x, t, mods, t.src_mod, 0);
  __syncthreads();
  conv_store<NS, SP, CONV_CPT>(sh, v, t.ns, t.nd, dst + (size_t)p * dst_stride * N + k, N, false, 0);
}

// ModUp (keyswitch_one, oracle): every limb of Q u P outside digit j is the
// fast base conversion of the digit's coefficient-form limbs (the digit's own
// limbs were already placed in ext by the producing kernel, ks_prep / tensor /
// automorph).  Outputs are written times R (Montgomery form) so the KS inner
// product needs a single reduction.  The conversion table of the digit and the
// destination moduli are staged in LDS once per workgroup, so the per-target
// loop issues no dependent global/scalar loads (CONV_CPT coefficients per thread).
template <int NS, bool SP>
__global__ void __launch_bounds__(EW_BLOCK) modup_kernel(const u64 *__restrict__ dc, u32 dc_stride,
                                                         u64 *__restrict__ ext, const ConvTab *tabs,
                                                         const ModInfo *mods, u32 QP, u32 alpha, u32 ndig,
                                                         u32 log_n) {
  __shared__ ConvLds<NS> sh;
  const u32 k = blockIdx.x * (EW_BLOCK * CONV_CPT) + threadIdx.x;
  const u32 ct = blockIdx.y / ndig, j = blockIdx.y % ndig;
  const size_t N = (size_t)1 << log_n;
  const u32 lo = j * alpha;
  const ConvTab t = tabs[j];
  const u64 *s = dc + ((size_t)ct * dc_stride + lo) * N + k;
  u64 x[CONV_CPT][NS];
#pragma unroll
  for (int i = 0; i < NS; ++i)
#pragma unroll
    for (int c = 0; c < CONV_CPT; ++c) x[c][i] = i < (int)t.ns ? ld_nt(s + i * N + c * EW_BLOCK) : 0;
  conv_stage<NS, SP>(sh, t, mods);
  u64 v[CONV_CPT][NS];
  conv_scale<NS, SP>(v, x, t, mods, nullptr, lo);
  __syncthreads();
  // the converted limbs go straight into the forward NTT: lazy range suffices
  conv_store<NS, SP, CONV_CPT, true>(sh, v, t.ns, t.nd, ext + ((size_t)(ct * ndig + j) * QP) * N + k, N, true, 0);
}

// KS preparation for an input d (fhe_keyswitch): dc = d and the own-digit
// slot of ext = d * R.  (mul_relin / rotate fuse this into the tensor INTT /
// automorphism prologues, BFV mul_relin into the BEHZ floor.)
template <bool SP>
__global__ void __launch_bounds__(EW_BLOCK) ks_prep_kernel(const u64 *__restrict__ d, u32 d_stride,
                                                           u64 *__restrict__ dc, u64 *__restrict__ ext,
                                                           const ModInfo *mods, u32 L, u32 QP, u32 alpha, u32 ndig,
                                                           u32 log_n, const u64 *dsc) {
  const u32 k = blockIdx.x * EW_BLOCK + threadIdx.x;
  const u32 ct = blockIdx.y / L, i = blockIdx.y % L, j = i / alpha;
  const size_t N = (size_t)1 << log_n;
  const ModInfo m = mods[i];
  const u64 x = d[((size_t)ct * d_stride + i) * N + k];
  // dsc (fused BFV key switch): dc holds ModUp's scaled sources x (Q_j/q_i)^-1
  dc[((size_t)ct * L + i) * N + k] = dsc ? csub63(mont_mul<SP>(x, dsc[i], m), m.q) : x;
  ext[((size_t)(ct * ndig + j) * QP + i) * N + k] = csub63(mont_mul<SP>(x, m.r2, m), m.q);
}

// KS inner product (keyswitch_one, oracle):
//   acc_b[i] = sum_j ext_j[i] * ksk[j][b][i]  mod m_i,  b in {0,1}
// One thread owns (limb i, coefficient k) for the WHOLE batch: the 2*dnum
// key words are loaded once and reused by every ciphertext, so the 48 MiB key
// is read once per call instead of once per ciphertext (up to 16 digits; more
// digits stream the key words with the digits).  ext carries a factor R, which
// the Montgomery products of dot_mont remove.
template <bool SP, int MAXD>
__global__ void __launch_bounds__(EW_BLOCK) ks_inner_kernel(const u64 *__restrict__ ext, const u64 *__restrict__ ksk,
                                                            u64 *__restrict__ acc, const ModInfo *mods, u32 QP,
                                                            u32 ndig, u32 n_ct, u32 log_n, u32 limb0, u32 kQP,
                                                            u32 L, u32 kshift) {
  const u32 k = blockIdx.x * EW_BLOCK + threadIdx.x;
  const u32 i = limb0 + blockIdx.y;
  const size_t N = (size_t)1 << log_n;
  const ModInfo m = mods[i];
  const size_t ext_ct = (size_t)ndig * QP * N, acc_ct = (size_t)2 * QP * N;
  const u64 *e = ext + (size_t)i * N + k;
  u64 *o = acc + (size_t)i * N + k;
  // key word (j, b) at kp[(2 j + b) kQP N]; the key row of a P limb of a level
  // view is i + kshift (the full-level key layout)
  const u64 *kp = ksk + (size_t)(i + (i >= L ? kshift : 0)) * N + k;
  if constexpr (MAXD > 0) {
    // the 2 ndig key words of this coefficient stay in registers for the whole batch
    u64 k0[MAXD], k1[MAXD];
#pragma unroll
    for (int j = 0; j < MAXD; ++j) {
      k0[j] = j < (int)ndig ? kp[(size_t)(2 * j) * kQP * N] : 0;
      k1[j] = j < (int)ndig ? kp[(size_t)(2 * j + 1) * kQP * N] : 0;
    }
    // software pipeline over the batch: the next ciphertext's digit words are
    // in flight while this one's products are formed
    u64 x[MAXD];
#pragma unroll
    for (int j = 0; j < MAXD; ++j) x[j] = (j < (int)ndig && n_ct) ? ld_nt(e + (size_t)j * QP * N) : 0;
#pragma unroll 1
    for (u32 ct = 0; ct < n_ct; ++ct) {
      u64 xn[MAXD];
      const bool more = ct + 1 < n_ct;
#pragma unroll
      for (int j = 0; j < MAXD; ++j)
        xn[j] = (j < (int)ndig && more) ? ld_nt(e + (ct + 1) * ext_ct + (size_t)j * QP * N) : 0;
      st_nt(o + ct * acc_ct, dot_mont<MAXD, SP>(x, k0, 1, ndig, m));
      st_nt(o + ct * acc_ct + (size_t)QP * N, dot_mont<MAXD, SP>(x, k1, 1, ndig, m));
#pragma unroll
      for (int j = 0; j < MAXD; ++j) x[j] = xn[j];
    }
  } else {
    // many digits (> 16): stream the key words with the digits, 4 at a time
    for (u32 ct = 0; ct < n_ct; ++ct) {
      u64 r0 = 0, r1 = 0;
      for (u32 j0 = 0; j0 < ndig; j0 += 4) {
        u64 x[4], h0[4], h1[4];
        const u32 nj = ndig - j0 < 4 ? ndig - j0 : 4;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const bool on = j < (int)nj;
          x[j] = on ? ld_nt(e + ct * ext_ct + (size_t)(j0 + j) * QP * N) : 0;
          h0[j] = on ? kp[(size_t)(2 * (j0 + j)) * kQP * N] : 0;
          h1[j] = on ? kp[(size_t)(2 * (j0 + j) + 1) * kQP * N] : 0;
        }
        r0 = add_mod(r0, dot_mont<4, SP>(x, h0, 1, nj, m), m.q);
        r1 = add_mod(r1, dot_mont<4, SP>(x, h1, 1, nj, m), m.q);
      }
      st_nt(o + ct * acc_ct, r0);
      st_nt(o + ct * acc_ct + (size_t)QP * N, r1);
    }
  }
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
  u64 ks = csub63(mont_mul<SP>(sub_mod(a, cv, m.q), pinv[i], m), m.q);
  const size_t o = ((size_t)(2 * ct + b) * L + i) * N + k;
  if (add_mask & (1u << b)) ks = add_mod(ks, base[o], m.q);
  out[o] = ks;
}

// Fused BFV ModDown finish (coefficient domain, bfv_ks_fused): the P -> Q
// conversion of acc's P limbs (already scaled by INTT(acc)'s output constants
// d_bfv_kscale, so they are the conversion's v_k) as 31-bit column sums, and the
// combine, per element:  out_b[i] = base_b[i] + (acc_b[i] - sum_k v_k [P/p_k]_{q_i}) P^-1.
// h = the ModDown table [K][L] ((P/p_k) R mod q_i), K <= 4.
// several rotations' ModDown in one launch (hoisted BFV rotations of few
// ciphertexts): poly p of acc is rotation p / rp, ciphertext poly p % rp
struct BfvRotOut {
  u32 rp;  // 0: one rotation (the out / base_ginv arguments)
  u64 *out[FHE_ROT_BATCH];
  u32 ginv[FHE_ROT_BATCH];
};
template <bool SP>
__global__ void __launch_bounds__(EW_BLOCK) bfv_moddown_kernel(const u64 *__restrict__ acc, const u64 *base, u64 *out,
                                                               const u64 *__restrict__ h, const u64 *pinv,
                                                               const ModInfo *mods, u32 L, u32 K, u32 QP,
                                                               u32 log_n, u32 add_mask, u32 base_ginv, BfvRotOut ro) {
  const u32 k = blockIdx.x * EW_BLOCK + threadIdx.x;
  const u32 p = blockIdx.y / L, i = blockIdx.y % L;  // p = 2 ct + b (of the rotation batch)
  u32 cp = p;
  if (ro.rp) {
    const u32 r = p / ro.rp;
    cp = p - r * ro.rp;
    out = ro.out[r];
    base_ginv = ro.ginv[r];
  }
  const size_t N = (size_t)1 << log_n;
  const ModInfo m = mods[i];
  const u64 *ap = acc + (size_t)p * QP * N + k;
  u64 v[4];
  u32 h0[4], h1[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const bool on = j < (int)K;
    v[j] = on ? ap[(size_t)(L + j) * N] : 0;
    if (on) split31(h[(size_t)j * L + i], h0[j], h1[j]);
    else h0[j] = h1[j] = 0;
  }
  const u64 cv = csub63(dot_cols<4, SP>(v, h0, h1, m), m.q);
  u64 ks = csub63(mont_mul<SP>(sub_mod(ap[(size_t)i * N], cv, m.q), pinv[i], m), m.q);
  const size_t o = ((size_t)cp * L + i) * N + k;
  if (add_mask & (1u << (p & 1))) {
    u64 bv;
    if (base_ginv) {
      // the base read through the coefficient automorphism (rotation: sigma_g(c0)
      // is never stored; the map of aut_rows_coef_kernel)
      const u32 n = 1u << log_n, j0 = (u32)(((u64)k * base_ginv) & (2 * n - 1));
      const u64 *bp = base + ((size_t)cp * L + i) * N;
      bv = j0 < n ? bp[j0] : (bp[j0 - n] ? m.q - bp[j0 - n] : 0);
    } else {
      bv = base[o];
    }
    ks = add_mod(ks, bv, m.q);
  }
  out[o] = ks;
}

// Double-hoisted rotation sum (orc_rotate_sum_hoisted_at): the key-switch
// inner products of up to ROT_SUM_MAX Galois elements over every limb of Q u P,
//   acc_b[i][k] (+)= sum_r sum_j ext_j[i][sigma_{g_r}(k)] ksk_r[j][b][row(i)][k] R^-1,
// ext in the NTT domain (times R, lazy below 8q on special moduli).  One thread
// per (coefficient, limb, ciphertext); acc canonical.
#define ROT_SUM_MAX 16
struct RotSumArgs {
  u32 nr;
  const u64 *ksk[ROT_SUM_MAX];
  const u64 *pt[ROT_SUM_MAX];  // hoisted linear transform: element r's plaintext ([L+K][N] NTT), or null
  u32 g[ROT_SUM_MAX];  // Galois elements (NTT gathers); the coefficient map takes g^-1 (aut_sum_kernel)
};
__device__ __forceinline__ u32 ntt_aut_src(u32 k, u32 g, u32 log_n) {
  const u32 mask = (2u << log_n) - 1;
  const u32 e = 2 * (__brev(k) >> (32 - log_n)) + 1;
  const u32 e2 = (u32)(((u64)e * g) & mask);
  return __brev((e2 - 1) >> 1) >> (32 - log_n);
}
template <bool SP>
__global__ void __launch_bounds__(EW_BLOCK) rot_sum_inner_kernel(const u64 *__restrict__ ext, u64 *__restrict__ acc,
                                                                 RotSumArgs ra, const ModInfo *mods, u32 L, u32 QP,
                                                                 u32 ndig, u32 kQP, u32 kshift, u32 log_n,
                                                                 u32 accumulate) {
  const u32 k = blockIdx.x * EW_BLOCK + threadIdx.x, i = blockIdx.y, ct = blockIdx.z;
  const size_t N = (size_t)1 << log_n;
  const ModInfo m = mods[i];  // the context's own index space (a level view: Q_m then P)
  const u64 *e = ext + ((size_t)ct * ndig * QP + i) * N;
  const size_t row = i < L ? i : i + kshift;  // the full-level key row
  const u64 q2 = 2 * m.q;
  u64 s0 = 0, s1 = 0;
  for (u32 r = 0; r < ra.nr; ++r) {
    const u32 src = ntt_aut_src(k, ra.g[r], log_n);
    const u64 *kp = ra.ksk[r] + row * N + k;
    u64 t0 = 0, t1 = 0;
    for (u32 j = 0; j < ndig; ++j) {
      const u64 x = e[(size_t)j * QP * N + src];
      t0 = csub(t0 + mont_mul<SP>(x, kp[(size_t)(2 * j) * kQP * N], m), q2);  // < 2q
      t1 = csub(t1 + mont_mul<SP>(x, kp[(size_t)(2 * j + 1) * kQP * N], m), q2);
    }
    if (ra.pt[r]) {  // times the plaintext: w = pt R, so mont_mul(t, w) = t pt
      const u64 w = csub(mont_mul<SP>(ra.pt[r][row * N + k], m.r2, m), m.q);
      t0 = mont_mul<SP>(t0, w, m);
      t1 = mont_mul<SP>(t1, w, m);
    }
    s0 = csub(s0 + t0, q2);
    s1 = csub(s1 + t1, q2);
  }
  s0 = csub(s0, m.q);
  s1 = csub(s1, m.q);
  u64 *o0 = acc + ((size_t)ct * 2 * QP + i) * N + k, *o1 = o0 + (size_t)QP * N;
  if (accumulate) {
    s0 = add_mod(s0, *o0, m.q);
    s1 = add_mod(s1, *o1, m.q);
  }
  *o0 = s0;
  *o1 = s1;
}
// base[ct][0][i] (+)= sum_r sigma_{g_r}(c0[ct][i]): NTT-domain gathers (CKKS) or
// the signed coefficient map with g^-1 (BFV)
template <bool SP>
__global__ void __launch_bounds__(EW_BLOCK) rot_sum_base_kernel(const u64 *__restrict__ ct, u64 *__restrict__ base,
                                                                RotSumArgs ra, const ModInfo *mods, u32 L, u32 log_n,
                                                                u32 coef, u32 accumulate) {
  const u32 k = blockIdx.x * EW_BLOCK + threadIdx.x, i = blockIdx.y, c = blockIdx.z;
  const size_t N = (size_t)1 << log_n;
  const ModInfo m = mods[i];
  const u64 q = m.q;
  const u64 *c0 = ct + ((size_t)c * 2 * L + i) * N;
  u64 s = 0;
  for (u32 r = 0; r < ra.nr; ++r) {
    u64 v;
    if (coef) {
      const u32 n = 1u << log_n, j0 = (u32)(((u64)k * ra.g[r]) & (2 * n - 1));
      v = j0 < n ? c0[j0] : (c0[j0 - n] ? q - c0[j0 - n] : 0);
    } else {
      v = c0[ntt_aut_src(k, ra.g[r], log_n)];
    }
    if (ra.pt[r]) {  // NTT domain (CKKS): times the plaintext's Q row i
      const u64 w = csub(mont_mul<SP>(ra.pt[r][(size_t)i * N + k], m.r2, m), q);
      v = csub(mont_mul<SP>(v, w, m), q);
    }
    s = add_mod(s, v, q);
  }
  u64 *o = base + ((size_t)c * 2 * L + i) * N + k;
  *o = accumulate ? add_mod(s, *o, q) : s;
}

// Rotation input: (c0, c1) -> sigma_g, fused with the key-switch preparation:
//   base[ct][0] = sigma(c0); dc[ct] = sigma(c1); ext[ct][own] = sigma(c1) * R.
// NTT domain (CKKS): slot permutation; coefficient domain (BFV): signed gather.
template <bool SP, bool NTT>
__global__ void __launch_bounds__(EW_BLOCK) automorph_ks_kernel(const u64 *__restrict__ ct_in, u64 *__restrict__ base,
                                                                u64 *__restrict__ dc, u64 *__restrict__ ext, u32 g,
                                                                const ModInfo *mods, u32 L, u32 QP, u32 alpha,
                                                                u32 ndig, u32 log_n, const u64 *dsc) {
  const u32 k = blockIdx.x * EW_BLOCK + threadIdx.x;
  const u32 ct = blockIdx.y / L, i = blockIdx.y % L, j = i / alpha;
  const size_t N = (size_t)1 << log_n, LN = (size_t)L * N;
  const ModInfo m = mods[i];
  const u64 *c0 = ct_in + (size_t)ct * 2 * LN + (size_t)i * N, *c1 = c0 + LN;
  u64 y0, y1;
  if (NTT) {
    const u32 mask = (2u << log_n) - 1;
    const u32 e = 2 * (__brev(k) >> (32 - log_n)) + 1;
    const u32 e2 = (u32)(((u64)e * g) & mask);
    const u32 src = __brev((e2 - 1) >> 1) >> (32 - log_n);
    y0 = c0[src];
    y1 = c1[src];
  } else {
    // here g carries g^-1 mod 2N
    const u32 n = 1u << log_n, mask = 2 * n - 1;
    const u32 j0 = (u32)(((u64)k * g) & mask);
    if (j0 < n) {
      y0 = c0[j0];
      y1 = c1[j0];
    } else {
      const u64 x0 = c0[j0 - n], x1 = c1[j0 - n];
      y0 = x0 ? m.q - x0 : 0;
      y1 = x1 ? m.q - x1 : 0;
    }
  }
  if (base) base[(size_t)ct * 2 * LN + (size_t)i * N + k] = y0;
  dc[(size_t)ct * LN + (size_t)i * N + k] = dsc ? csub63(mont_mul<SP>(y1, dsc[i], m), m.q) : y1;
  ext[((size_t)(ct * ndig + j) * QP + i) * N + k] = csub63(mont_mul<SP>(y1, m.r2, m), m.q);
}

// ------------------------------------------------- base conversions on MFMA
// BEHZ_MFMA = 1 builds the BEHZ extension and floor on the matrix cores
// (below).  Built, bit-exact, and rejected on measurement: C3 -4.6% (floor
// 1331 us and extension 834 us per 128-ct call against 1055 and 654 for the
// VALU kernels).  With the sp60 column sums the VALU form costs 36 issue slots
// per coefficient; the MFMA form spends 57 (32 coefficients per wave, half the
// targets of each block per lane half, the combine and the per-half constant
// selects), and both kernels are VALU-issue bound (busy 1.04 / 0.98,
// profiles/r06/stall_c3.txt), so the extra slots cost time directly
// (profiles/r06/ab_bfv_behz_mfma.txt).
#ifndef BEHZ_MFMA
#define BEHZ_MFMA 0
#endif
#if BEHZ_MFMA
// A fast base conversion y_t = sum_i v_i h[i][t] mod m_t over 8 sources is a
// dense contraction, so at the BEHZ kernels' C3 shape it runs on the matrix
// cores (v_mfma_i32_32x32x32_i8).  Sources and constants are written in 8
// balanced signed base-256 digits (d_a = byte_a(v + 0x80..80) - 128: one 64-bit
// add and one xor); the constant operand holds, per target t and result digit
// b, the digits of C[i][a][t] = h[i][t] 256^a mod m_t, so that
//   S[t][b] = sum_{i,a} d_{i,a} digit_b(C[i][a][t])     (|S| <= 64 2^14 = 2^20)
// and y_t = mont_reduce(sum_b S[t][b] 256^b + k m_t) (constants pre-scaled by R,
// k m_t an offset that makes the 128-bit sum non-negative).  One wave handles
// 32 coefficients: lane (h, c) = (lane >> 5, lane & 31) supplies sources
// {2h, 2h+1} (MFMA 0) and {4+2h, 5+2h} (MFMA 1) of coefficient c, and the
// rows of the constant operand are ordered so that lane half h receives all 8
// digits of targets 2h and 2h+1 of each 4-target block -- the layout of the
// sources of the next contraction (no cross-lane exchange).  Prototype and
// bit-check: tools/microbench/bconv_mfma.hip (round 2).
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
struct MfmaConv {
  v4i af[3][2][64];  // [4-target block][k step (4 sources)][lane] constant operand
  u64 off[12];       // per target: A of the offset A + 2^45 2^32 = k m_t
};
// this lane's source s (0..3) of an 8-source contraction
__device__ __forceinline__ int mfma_src(int h, int s) { return (s >> 1) * 4 + 2 * h + (s & 1); }
// the data operand of k step m from this lane's 4 source words
__device__ __forceinline__ v4i mfma_digits(u64 x, u64 y) {
  constexpr u64 K80 = 0x8080808080808080ull;
  const u64 a = (x + K80) ^ K80, b = (y + K80) ^ K80;
  return v4i{(int)(u32)a, (int)(u32)(a >> 32), (int)(u32)b, (int)(u32)(b >> 32)};
}
// target 2h + u of 4-target block s: its 8 result digits recombined and
// reduced, canonical (the constants carry R: mont_reduce's R^-1 cancels it)
__device__ __forceinline__ u64 mfma_combine(const v16i &s, int u, u64 offA, const ModInfo &m) {
  typedef int64_t i64;
  const int x01 = s[8 * u] + s[8 * u + 1] * 256, x23 = s[8 * u + 2] + s[8 * u + 3] * 256;
  const int x45 = s[8 * u + 4] + s[8 * u + 5] * 256, x67 = s[8 * u + 6] + s[8 * u + 7] * 256;
  const u64 lo = (u64)((i64)x01 + (i64)x23 * 65536) + offA;          // |.| < 2^45 before the offset
  const u64 hi = (u64)((i64)x45 + (i64)x67 * 65536) + (1ull << 45);
  const u64 t1 = (lo >> 32) + (u32)hi;
  const U128 T{(u64)(u32)lo | (t1 << 32), (hi >> 32) + (t1 >> 32)};
  return csub63(mont_reduce<true>(T, m), m.q);
}
// lane half h's value of a pair indexed uniformly: both loaded as scalars,
// one select (a lane-dependent index would turn every constant and modulus
// load of the MFMA kernels into a vector load)
// (i0 < 0: block 2 of a 9-target contraction, target 8 only, lane half 0)
template <class T>
__device__ __forceinline__ T half_pick(u32 h, const T *x, int i0) {
  if (i0 < 0) return x[8];
  const T a = x[i0], b = x[i0 + 2];
  return h ? b : a;
}
__device__ __forceinline__ ModInfo half_mod(u32 h, const ModInfo *mods, int i0) {
  if (i0 < 0) return mods[8];
  const ModInfo a = mods[i0], b = mods[i0 + 2];
  ModInfo m;
  m.q = h ? b.q : a.q;
  m.qinv_neg = h ? b.qinv_neg : a.qinv_neg;
  m.r2 = h ? b.r2 : a.r2;
  m.q_hi = h ? b.q_hi : a.q_hi;
  m.special = 1;
  return m;
}
// 4-target block blk of a contraction, over both k steps
__device__ __forceinline__ v16i mfma_conv1(const MfmaConv &f, int blk, const v4i &d0, const v4i &d1, u32 lane) {
  const v16i z = {};
  const v16i a = __builtin_amdgcn_mfma_i32_32x32x32_i8(f.af[blk][0][lane], d0, z, 0, 0, 0);
  return __builtin_amdgcn_mfma_i32_32x32x32_i8(f.af[blk][1][lane], d1, a, 0, 0, 0);
}
#endif  // BEHZ_MFMA

// ----------------------------------------------------------------- BEHZ
// Constants for SEAL-style BEHZ (behz_init in the oracle), Montgomery
// pre-scaled ("_R" = times 2^64 mod the modulus it is used with).
#define BEHZ_MAXL 24
// The constant factors that follow a conversion are folded into its weights
// (a product of canonical residues by c, then by c', is the canonical residue
// of one product by c c'), so each output costs one Montgomery product fewer
// than the formula as written (extend: sm_mrq's 2^-32; floor: Q^-1 and the
// fastbconv_sk weight (B/b_j)^-1, or B^-1 for m_sk).  The outputs are the same
// residues, bit for bit.
struct BehzDev {
  u32 L, nB, bsk0;                 // bsk0 = first Bsk modulus id
  u32 neg_inv_q_mod_mt;            // -Q^-1 mod 2^32
  u32 h_mod_mt[BEHZ_MAXL];         // (Q/q_i) mod 2^32
  u64 mt_hinv_R[BEHZ_MAXL];        // 2^32 (Q/q_i)^-1 mod q_i
  u64 t_hinv_R[BEHZ_MAXL];         // t (Q/q_i)^-1 mod q_i
  u64 hx_R[BEHZ_MAXL][BEHZ_MAXL + 1];  // extend: (Q/q_i) 2^-32 mod b_j
  u64 qx_R[BEHZ_MAXL + 1];             // extend: Q 2^-32 mod b_j
  u64 hf_R[BEHZ_MAXL][BEHZ_MAXL + 1];  // floor: -(Q/q_i) Q^-1 c_j mod b_j
  u64 tf_R[BEHZ_MAXL + 1];             // floor: t Q^-1 c_j mod b_j
                                       //   (c_j = (B/b_j)^-1, for m_sk: B^-1)
  u64 hbm_R[BEHZ_MAXL];                // floor: (B/b_j) B^-1 mod m_sk
  u64 b_mod_q_R[BEHZ_MAXL];        // B mod q_i
  u64 h_b_q_R[BEHZ_MAXL][BEHZ_MAXL];  // (B/b_j) mod q_i
#if BEHZ_MFMA
  // (L = 8, special moduli): the three dense contractions on the matrix cores
  // (behz_*_mfma_kernel): extension Q -> Bsk (hx), floor Q -> Bsk (hf), floor
  // B -> Q (h_b_q), each 8 sources -> up to 12 targets
  MfmaConv mx, mf, mq;
#endif
};

// BEHZ_WPE: waves per SIMD forced on both kernels (8: -1.5% C3 against the
// compiler's 7, profiles/r06/ab_bfv_behz_mfma.txt)
#ifdef BEHZ_WPE
#define BEHZ_OCC __attribute__((amdgpu_waves_per_eu(BEHZ_WPE)))
#else
#define BEHZ_OCC
#endif
#ifndef HPS_S60
#define HPS_S60 1  // HPS's conversions on the in-place 31-bit column sums (hps_sp60)
#endif
#ifndef BEHZ_FENCES
#define BEHZ_FENCES 9
#endif
// a scheduling fence per target of the BEHZ kernels: left free, the scheduler
// hoists every target's uniform constants (hx / hf, h_b_q: up to 136 words,
// split into 31-bit digits) to the top, past the 102 SGPRs, and spills them to
// VGPR lanes (v_writelane / v_readlane).  Fenced, the extension drops 13% of its
// VALU instructions and runs at 36 VGPRs (8 waves): 650 -> 555 us per C3 call.
// The floor's fences (bits 2, 4) remove its 104 SGPR spills too but cost 2% of
// C3 (its Bsk loads can no longer run ahead of the previous target's products,
// also with a one-ahead prefetch): profiles/r06/ab_behz_fences.txt.  The HPS
// extension on column sums (bit 8): 86 -> 36 VGPRs, +0.4..0.9% on HPS C3
// (profiles/r06/ab_hps_sp60.txt)
// BEHZ_FENCES bits: 1 the extension's targets, 2 the floor's Bsk targets, 4 the floor's Q targets,
// 8 the HPS extension's targets
#define BEHZ_FENCE(bit)                                          \
  do {                                                           \
    if constexpr (BEHZ_FENCES & (bit)) __builtin_amdgcn_sched_barrier(0); \
  } while (0)
#ifndef BEHZ_NT
#define BEHZ_NT 0  // BEHZ floor: 1 = non-temporal loads, 2 = stores (1, 2, 3 all within +-0.5% of 0 on C3: ab_bfv_behz_nt.txt)
#endif
template <class T>
__device__ __forceinline__ T behz_ld(const T *p) {
  if constexpr (BEHZ_NT & 1) return __builtin_nontemporal_load(p);
  else return *p;
}
template <class T>
__device__ __forceinline__ void behz_st(T *p, T v) {
  if constexpr (BEHZ_NT & 2) __builtin_nontemporal_store(v, p);
  else *p = v;
}
#ifndef BEHZ_COLS
#define BEHZ_COLS 0  // 1: BEHZ dot products as 31-bit column sums (dot_cols_canon): extend +8%, floor -0.7%, C3 -0.9% (profiles/r03/ab_conv_cols.txt)
#endif
// S60 (round 6): special moduli where one side of every product is below 2^60
// (Q sources below 2^60 into Bsk targets, or Bsk sources into Q targets below
// 2^60): 31-bit column sums reduced in place (dot_cols_sp60, < 1.25m per 4
// terms), one reduction per 4 terms instead of a Montgomery product per term
template <int NL>
__device__ __forceinline__ u64 dot_sp60_canon(const u64 (&v)[NL], const u64 *h, size_t hs, u32 ns, const ModInfo &m) {
  u64 res = 0;
  const u64 m2 = 2 * m.q;
#pragma unroll
  for (int c0 = 0; c0 < NL; c0 += 4) {
    if (c0 < (int)ns) {
      u64 vv[4];
      u32 h0[4], h1[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bool on = c0 + i < NL && c0 + i < (int)ns;
        vv[i] = on ? v[c0 + i < NL ? c0 + i : 0] : 0;
        if (on) split31(h[(size_t)(c0 + i) * hs], h0[i], h1[i]);
        else h0[i] = h1[i] = 0;
      }
      const u64 part = dot_cols_sp60<4>(vv, h0, h1, m.q_hi);  // < 1.25m
      res = c0 == 0 ? part : csub63(res + part, m2);            // < 2m
    }
  }
  return csub63(res, m.q);
}
template <int NL, bool SP, bool S60 = false>
__device__ __forceinline__ u64 behz_dot(const u64 (&v)[NL], const u64 *h, size_t hs, u32 ns, const ModInfo &m) {
  if constexpr (SP && S60) return dot_sp60_canon<NL>(v, h, hs, ns, m);
  else if constexpr (BEHZ_COLS) return dot_cols_canon<NL, SP>(v, h, hs, ns, m);
  else return dot_mont<NL, SP>(v, h, hs, ns, m);
}

// behz_extend (oracle): fastbconv_m_tilde then sm_mrq.  x [L] coef -> [nB] coef
// EX: L == NL exactly (nB = L + 1 always), so every loop is unrolled with no
// per-limb guards (the C3 parameters); otherwise NL bounds L.
template <int NL, bool SP, bool EX, bool S60>
// Poly p = 4 item + w of the BFV product's operands (w: a0, a1, b0, b1) is
// read straight from the ciphertexts and extended to Bsk in xb [2][n][2][nB][N]
// (the a and b parts, each in the ciphertexts' own layout).  The Q part is not
// copied: its forward NTT reads a and b out of place (bfv_mul_relin_impl).
__global__ void __launch_bounds__(EW_BLOCK) BEHZ_OCC behz_extend_kernel(const u64 *__restrict__ a, const u64 *__restrict__ b,
                                                               u64 *__restrict__ xb, const BehzDev *bz,
                                                               const ModInfo *mods, u32 log_n, u32 n_items) {
  const u32 k = blockIdx.x * EW_BLOCK + threadIdx.x;
  const u32 p = blockIdx.y, item = p >> 2, w = p & 3;
  const size_t N = (size_t)1 << log_n;
  const u32 L = EX ? NL : bz->L, nB = L + 1;
  const u64 *s = (w < 2 ? a : b) + ((size_t)(2 * item + (w & 1)) * L) * N + k;
  u64 v[NL];
  u32 xmt = 0;
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    v[i] = 0;
    if (EX || i < (int)L) {
      const ModInfo m = mods[i];
      const u64 x = ld_nt(s + i * N);
      v[i] = csub63(mont_mul<SP>(x, bz->mt_hinv_R[i], m), m.q);
      xmt += (u32)v[i] * bz->h_mod_mt[i];
    }
  }
  const u32 r = xmt * bz->neg_inv_q_mod_mt;
  u64 *d = xb + ((size_t)((w >> 1) * n_items + item) * 2 + (w & 1)) * nB * N + k;
  constexpr int UJ = EX ? NL + 1 : 1;  // unrolled only with compile-time bounds
#pragma unroll UJ
  for (int j = 0; j < NL + 1; ++j) {
    BEHZ_FENCE(1);
    if (EX || j < (int)nB) {
      const ModInfo m = mods[bz->bsk0 + j];
      // (sum_i v_i (Q/q_i) + r Q) 2^-32, the 2^-32 folded into the weights
      const u64 xbj = behz_dot<NL, SP, S60>(v, &bz->hx_R[0][j], BEHZ_MAXL + 1, L, m);
      const u64 rr = r >= 0x80000000u ? (u64)r + m.q - (1ull << 32) : (u64)r;   // centered r mod b
      d[j * N] = csub63(xbj + csub63(mont_mul<SP>(rr, bz->qx_R[j], m), m.q), m.q);
    }
  }
}

// behz_floor_to_q (oracle): fast_floor in Bsk then fastbconv_sk back to Q.
// The third output r2 goes straight into the key-switch scratch (the KS
// preparation of ks_prep_kernel fused here): dc = r2 and the own-digit ext
// slot = r2 R, so r2 is not written and read back by a separate kernel.
template <int NL, bool SP, bool EX, bool S60>
__global__ void __launch_bounds__(EW_BLOCK) BEHZ_OCC behz_floor_kernel(const u64 *__restrict__ eq, const u64 *__restrict__ eb,
                                                              u64 *__restrict__ out01, u64 *__restrict__ dc,
                                                              u64 *__restrict__ ext, const BehzDev *bz,
                                                              const ModInfo *mods, u32 log_n, u32 QP, u32 dig_len,
                                                              u32 ndig, const u64 *dsc) {
  const u32 k = blockIdx.x * EW_BLOCK + threadIdx.x;
  const u32 ct = blockIdx.y / 3, p = blockIdx.y % 3;
  const size_t N = (size_t)1 << log_n;
  const u32 L = EX ? NL : bz->L, nB = L + 1;
  const u64 *xq = eq + ((size_t)(ct * 3 + p) * L) * N + k;
  const u64 *xb = eb + ((size_t)(ct * 3 + p) * nB) * N + k;
  u64 v[NL];
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    v[i] = 0;
    if (EX || i < (int)L) {
      const ModInfo m = mods[i];
      v[i] = csub63(mont_mul<SP>(behz_ld(xq + i * N), bz->t_hinv_R[i], m), m.q);  // [t x (Q/q_i)^-1]_{q_i}
    }
  }
  // fast_floor: ((t x)_b - conv_Q->b(t x)) * Q^-1, then the fastbconv_sk
  // weight: w_j = (x_b t Q^-1 c_j) + sum_i v_i (-(Q/q_i) Q^-1 c_j), one dot
  // product and one product (the constants carry Q^-1 and c_j)
  u64 w[NL];
  u64 flsk = 0;
#pragma unroll
  for (int j = 0; j < NL + 1; ++j) {
    BEHZ_FENCE(2);
    if (EX || j < (int)nB) {
      const ModInfo m = mods[bz->bsk0 + j];
      const u64 cv = behz_dot<NL, SP, S60>(v, &bz->hf_R[0][j], BEHZ_MAXL + 1, L, m);
      const u64 tx = csub63(mont_mul<SP>(behz_ld(xb + j * N), bz->tf_R[j], m), m.q);
      const u64 wj = csub63(tx + cv, m.q);
      if (j == (int)nB - 1) flsk = wj;
      else if (j < NL) w[j] = wj;
    } else if (j < NL) {
      w[j] = 0;
    }
  }
  const ModInfo msk = mods[bz->bsk0 + nB - 1];
  const u64 alpha = sub_mod(behz_dot<NL, SP>(w, bz->hbm_R, 1, nB - 1, msk), flsk, msk.q);  // B^-1 folded in
  const bool neg = alpha > msk.q / 2;
  const u64 amag = neg ? msk.q - alpha : alpha;
  u64 *o = (p < 2) ? out01 + ((size_t)(ct * 2 + p) * L) * N + k : dc + ((size_t)ct * L) * N + k;
  for (int i = 0; i < (EX ? NL : (int)L); ++i) {
    BEHZ_FENCE(4);
    const ModInfo m = mods[i];
    const u64 cq = behz_dot<NL, SP, S60>(w, &bz->h_b_q_R[0][i], BEHZ_MAXL, nB - 1, m);
    const u64 ab = csub63(mont_mul<SP>(amag, bz->b_mod_q_R[i], m), m.q);
    const u64 r = csub63(cq + (neg ? ab : m.q - ab), m.q);  // cq -/+ ab (ab = 0 gives cq + q -> cq)
    // dsc (fused BFV relinearisation): dc holds ModUp's scaled sources r (Q_j/q_i)^-1
    behz_st(o + i * N, p == 2 && dsc ? csub63(mont_mul<SP>(r, dsc[i], m), m.q) : r);
    if (p == 2) behz_st(ext + ((size_t)(ct * ndig + i / dig_len) * QP + i) * N + k, csub63(mont_mul<SP>(r, m.r2, m), m.q));
  }
}

#if BEHZ_MFMA
// The same two kernels at L = 8 on special moduli with their dense
// contractions on the matrix cores (MfmaConv above); bit-identical outputs
// (every conversion is the same residue, canonical).  One wave = 32
// coefficients, lane half h owns sources / targets {2h, 2h+1, 4+2h, 5+2h}.
__global__ void __launch_bounds__(EW_BLOCK) behz_extend_mfma_kernel(const u64 *__restrict__ a,
                                                                    const u64 *__restrict__ b, u64 *__restrict__ xb,
                                                                    const BehzDev *bz, const ModInfo *mods, u32 log_n,
                                                                    u32 n_items) {
  constexpr int L = 8, nB = 9;
  const u32 lane = threadIdx.x & 63, h = lane >> 5, c = lane & 31;
  const u32 k = (blockIdx.x * (EW_BLOCK / 64) + (threadIdx.x >> 6)) * 32 + c;
  const u32 p = blockIdx.y, item = p >> 2, w = p & 3;
  const size_t N = (size_t)1 << log_n;
  const u64 *src = (w < 2 ? a : b) + ((size_t)(2 * item + (w & 1)) * L) * N + k;
  u64 v[4];
  u32 xmt = 0;
#pragma unroll
  for (int s_ = 0; s_ < 4; ++s_) {
    const int i = mfma_src(h, s_), i0 = mfma_src(0, s_);
    const ModInfo m = half_mod(h, mods, i0);
    v[s_] = csub63(mont_mul<true>(ld_nt(src + i * N), half_pick(h, bz->mt_hinv_R, i0), m), m.q);
    xmt += (u32)v[s_] * half_pick(h, bz->h_mod_mt, i0);
  }
  xmt += __shfl_xor(xmt, 32);  // the other lane half's four sources
  const u32 r = xmt * bz->neg_inv_q_mod_mt;
  const v4i d0 = mfma_digits(v[0], v[1]), d1 = mfma_digits(v[2], v[3]);
  u64 *d = xb + ((size_t)((w >> 1) * n_items + item) * 2 + (w & 1)) * nB * N + k;
#pragma unroll
  for (int blk = 0; blk < 3; ++blk) {
    const v16i acc = mfma_conv1(bz->mx, blk, d0, d1, lane);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int j = 4 * blk + 2 * h + u;
      if (j < nB) {
        const int j0 = 4 * blk + u, jp = blk == 2 ? -1 : j0;  // block 2: j = 8 only (lane half 0)
        const ModInfo m = half_mod(h, mods + bz->bsk0, jp);
        const u64 xbj = mfma_combine(acc, u, half_pick(h, bz->mx.off, jp), m);
        const u64 rr = r >= 0x80000000u ? (u64)r + m.q - (1ull << 32) : (u64)r;  // centered r mod b
        d[j * N] = csub63(xbj + csub63(mont_mul<true>(rr, half_pick(h, bz->qx_R, jp), m), m.q), m.q);
      }
    }
  }
}

__global__ void __launch_bounds__(EW_BLOCK) behz_floor_mfma_kernel(const u64 *__restrict__ eq,
                                                                   const u64 *__restrict__ eb, u64 *__restrict__ out01,
                                                                   u64 *__restrict__ dc, u64 *__restrict__ ext,
                                                                   const BehzDev *bz, const ModInfo *mods, u32 log_n,
                                                                   u32 QP, u32 dig_len, u32 ndig, const u64 *dsc) {
  constexpr int L = 8, nB = 9;
  const u32 lane = threadIdx.x & 63, h = lane >> 5, c = lane & 31;
  const u32 k = (blockIdx.x * (EW_BLOCK / 64) + (threadIdx.x >> 6)) * 32 + c;
  const u32 ct = blockIdx.y / 3, p = blockIdx.y % 3;
  const size_t N = (size_t)1 << log_n;
  const u64 *xq = eq + ((size_t)(ct * 3 + p) * L) * N + k;
  const u64 *xb = eb + ((size_t)(ct * 3 + p) * nB) * N + k;
  u64 v[4];
#pragma unroll
  for (int s_ = 0; s_ < 4; ++s_) {
    const int i = mfma_src(h, s_), i0 = mfma_src(0, s_);
    const ModInfo m = half_mod(h, mods, i0);
    v[s_] = csub63(mont_mul<true>(xq[i * N], half_pick(h, bz->t_hinv_R, i0), m), m.q);  // [t x (Q/q_i)^-1]_{q_i}
  }
  // fast_floor's conversion Q -> Bsk; w_j = x_b t Q^-1 c_j + conv_j (the constants carry Q^-1 c_j)
  u64 xbv[6];
#pragma unroll
  for (int q = 0; q < 6; ++q) {
    const int j = 4 * (q >> 1) + 2 * h + (q & 1);
    xbv[q] = j < nB ? xb[j * N] : 0;
  }
#pragma unroll
  for (int q = 0; q < 6; ++q) asm volatile("" : "+v"(xbv[q]));
  const v4i d0 = mfma_digits(v[0], v[1]), d1 = mfma_digits(v[2], v[3]);
  u64 wv[6];  // w_j of this lane's targets j = 4 blk + 2 h + u (j = 8: m_sk, lane half 0)
#pragma unroll
  for (int blk = 0; blk < 3; ++blk) {
    const v16i acc = mfma_conv1(bz->mf, blk, d0, d1, lane);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int j = 4 * blk + 2 * h + u;
      wv[2 * blk + u] = 0;
      if (j < nB) {
        const int j0 = 4 * blk + u, jp = blk == 2 ? -1 : j0;  // block 2: j = 8 only (lane half 0)
        const ModInfo m = half_mod(h, mods + bz->bsk0, jp);
        const u64 cv = mfma_combine(acc, u, half_pick(h, bz->mf.off, jp), m);
        const u64 tx = csub63(mont_mul<true>(xbv[2 * blk + u], half_pick(h, bz->tf_R, jp), m), m.q);
        wv[2 * blk + u] = csub63(tx + cv, m.q);
      }
    }
  }
  // alpha = sum_{j < 8} w_j (B/b_j) B^-1 - w_msk  (mod m_sk): each lane half its 4 terms
  const ModInfo msk = mods[bz->bsk0 + nB - 1];
  u64 part = 0;
#pragma unroll
  for (int s_ = 0; s_ < 4; ++s_) part += mont_mul<true>(wv[s_], half_pick(h, bz->hbm_R, mfma_src(0, s_)), msk);  // < 6 m_sk
  part = csub63(csub63(csub(part, 4 * msk.q), 2 * msk.q), msk.q);
  const u64 other = __shfl_xor(part, 32);
  const u64 flsk = __shfl(wv[4], c);  // w_8 lives in lane half 0
  const u64 alpha = sub_mod(add_mod(part, other, msk.q), flsk, msk.q);
  const bool neg = alpha > msk.q / 2;
  const u64 amag = neg ? msk.q - alpha : alpha;
  // fastbconv_sk's conversion B -> Q: this lane's w_j are exactly the sources it supplies
  const v4i e0 = mfma_digits(wv[0], wv[1]), e1 = mfma_digits(wv[2], wv[3]);
  u64 *o = (p < 2) ? out01 + ((size_t)(ct * 2 + p) * L) * N + k : dc + ((size_t)ct * L) * N + k;
#pragma unroll
  for (int blk = 0; blk < 2; ++blk) {
    const v16i acc = mfma_conv1(bz->mq, blk, e0, e1, lane);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int i = 4 * blk + 2 * h + u, i0 = 4 * blk + u;
      const ModInfo m = half_mod(h, mods, i0);
      const u64 cq = mfma_combine(acc, u, half_pick(h, bz->mq.off, i0), m);
      const u64 ab = csub63(mont_mul<true>(amag, half_pick(h, bz->b_mod_q_R, i0), m), m.q);
      const u64 rr = csub63(cq + (neg ? ab : m.q - ab), m.q);
      o[i * N] = p == 2 && dsc ? csub63(mont_mul<true>(rr, half_pick(h, dsc, i0), m), m.q) : rr;
      if (p == 2) ext[((size_t)(ct * ndig + i / dig_len) * QP + i) * N + k] = csub63(mont_mul<true>(rr, m.r2, m), m.q);
    }
  }
}
#endif  // BEHZ_MFMA

// ------------------------------------------------------------------ HPS
// BFV multiplication by Halevi-Polyakov-Shoup (oracle hps_*; OpenFHE BFVrns
// "HPS"), auxiliary base P = the Bsk primes.  Same pipeline as BEHZ (the two
// kernels below replace behz_extend / behz_floor; NTT, tensor and relinearise
// are shared).  The doubles are single rounded IEEE operations in the oracle's
// order: fp contraction is off in these kernels (no v_fma_f64), u64 -> f64 is
// round-to-nearest as in C, and the truncations are floor of positive values.
struct HpsDev {
  u32 L, nB, bsk0;
  u64 qt_R[BEHZ_MAXL];                   // (Q/q_i)^-1 R mod q_i
  double invq[BEHZ_MAXL];                // 1 / q_i
  u64 qstar_R[BEHZ_MAXL][BEHZ_MAXL + 1];  // [Q/q_i]_{p_j} R
  u64 Q_R[BEHZ_MAXL + 1];                // Q R mod p_j
  u64 ninv_R[BEHZ_MAXL];                 // N^-1 R mod q_i (the tensor's INTT skips N^-1)
  double frac[BEHZ_MAXL];                // num_i / q_i, num_i = [t (Q/q_i)^-1]_{q_i}
  u64 I_R[BEHZ_MAXL][BEHZ_MAXL + 1];     // [-num_i q_i^-1]_{p_j} R
  u64 lam_R[BEHZ_MAXL + 1];              // t Q^-1 N^-1 R mod p_j (applied to the unscaled e_{p_j})
  u64 pt_R[BEHZ_MAXL + 1];               // (P/p_j)^-1 R mod p_j
  double invp[BEHZ_MAXL + 1];            // 1 / p_j
  u64 pstar_R[BEHZ_MAXL + 1][BEHZ_MAXL];  // [P/p_j]_{q_i} R
  u64 P_R[BEHZ_MAXL];                    // P R mod q_i
};

// floor(s + 0.5) and floor(s) of a non-negative double, as the oracle's (u64) casts
__device__ __forceinline__ u64 hps_round(double s) {
#pragma clang fp contract(off)
  return (u64)(s + 0.5);
}
__device__ __forceinline__ u64 hps_round_down(double s) { return (u64)s; }

// init + sum_i y_i * w_i, left to right, each product and each sum rounded
template <int NL, bool EX>
__device__ __forceinline__ double hps_fsum(const u64 (&y)[NL], const double *w, u32 n, double init) {
#pragma clang fp contract(off)
  double s = init;
#pragma unroll
  for (int i = 0; i < NL; ++i)
    if (EX || i < (int)n) s = s + (double)y[i] * w[i];
  return s;
}

// Q -> P, the exact extension of the centred lift: y_i = [x_i (Q/q_i)^-1],
// v = floor(0.5 + sum y_i / q_i), x mod p_j = sum_i y_i [Q/q_i]_{p_j} - v [Q]_{p_j}.
// Layout as behz_extend_kernel (xb [2][n][2][nB][N]).
template <int NL, bool SP, bool EX, bool S60 = false>
__global__ void __launch_bounds__(EW_BLOCK) hps_extend_kernel(const u64 *__restrict__ a, const u64 *__restrict__ b,
                                                              u64 *__restrict__ xb, const HpsDev *hp,
                                                              const ModInfo *mods, u32 log_n, u32 n_items) {
  const u32 k = blockIdx.x * EW_BLOCK + threadIdx.x;
  const u32 p = blockIdx.y, item = p >> 2, w = p & 3;
  const size_t N = (size_t)1 << log_n;
  const u32 L = EX ? NL : hp->L, nB = L + 1;
  const u64 *s = (w < 2 ? a : b) + ((size_t)(2 * item + (w & 1)) * L) * N + k;
  u64 y[NL];
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    y[i] = 0;
    if (EX || i < (int)L) {
      const ModInfo m = mods[i];
      y[i] = csub63(mont_mul<SP>(ld_nt(s + i * N), hp->qt_R[i], m), m.q);
    }
  }
  const u64 v = hps_round(hps_fsum<NL, EX>(y, hp->invq, L, 0.0));
  u64 *d = xb + ((size_t)((w >> 1) * n_items + item) * 2 + (w & 1)) * nB * N + k;
  constexpr int UJ = EX ? NL + 1 : 1;
#pragma unroll UJ
  for (int j = 0; j < NL + 1; ++j) {
    BEHZ_FENCE(8);
    if (EX || j < (int)nB) {
      const ModInfo m = mods[hp->bsk0 + j];
      const u64 x = behz_dot<NL, SP, S60>(y, &hp->qstar_R[0][j], BEHZ_MAXL + 1, L, m);
      const u64 vq = csub63(mont_mul<SP>(v, hp->Q_R[j], m), m.q);
      d[j * N] = sub_mod(x, vq, m.q);
    }
  }
}

// d in Q u P (coefficient form, INTT without N^-1) -> round(t d / Q) in P ->
// Q.  In P: z_j = sum_i x_i I_ij + e_{p_j} t Q^-1 N^-1 + [r]_{p_j}, r =
// floor(0.5 + sum x_i f_i) (x_i = d mod q_i, the INTT's N^-1 applied first);
// then y_j = [z_j (P/p_j)^-1], v = floor(0.5 + sum y_j / p_j) and
// out_i = sum_j y_j [P/p_j]_{q_i} - v [P]_{q_i}.  Outputs as behz_floor_kernel
// (r0, r1 -> out01; r2 -> dc and its own-digit ext slot times R).
template <int NL, bool SP, bool EX, bool S60 = false>
__global__ void __launch_bounds__(EW_BLOCK) hps_scale_kernel(const u64 *__restrict__ eq, const u64 *__restrict__ eb,
                                                             u64 *__restrict__ out01, u64 *__restrict__ dc,
                                                             u64 *__restrict__ ext, const HpsDev *hp,
                                                             const ModInfo *mods, u32 log_n, u32 QP, u32 dig_len,
                                                             u32 ndig, const u64 *dsc) {
  const u32 k = blockIdx.x * EW_BLOCK + threadIdx.x;
  const u32 ct = blockIdx.y / 3, p = blockIdx.y % 3;
  const size_t N = (size_t)1 << log_n;
  const u32 L = EX ? NL : hp->L, nB = L + 1;
  const u64 *xq = eq + ((size_t)(ct * 3 + p) * L) * N + k;
  const u64 *xb = eb + ((size_t)(ct * 3 + p) * nB) * N + k;
  u64 x[NL];  // d mod q_i, canonical
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    x[i] = 0;
    if (EX || i < (int)L) {
      const ModInfo m = mods[i];
      x[i] = csub63(mont_mul<SP>(ld_nt(xq + i * N), hp->ninv_R[i], m), m.q);
    }
  }
  const u64 r = hps_round_down(hps_fsum<NL, EX>(x, hp->frac, L, 0.5));  // < L 2^61
  u64 y[NL + 1];
  constexpr int UJ = EX ? NL + 1 : 1;
#pragma unroll UJ
  for (int j = 0; j < NL + 1; ++j) {
    y[j] = 0;
    if (EX || j < (int)nB) {
      const ModInfo m = mods[hp->bsk0 + j];
      const u64 zi = behz_dot<NL, SP, S60>(x, &hp->I_R[0][j], BEHZ_MAXL + 1, L, m);
      const u64 zp = csub63(mont_mul<SP>(ld_nt(xb + j * N), hp->lam_R[j], m), m.q);
      const u64 zj = add_mod(add_mod(zi, zp, m.q), reduce128<SP>(U128{r, 0}, m), m.q);
      y[j] = csub63(mont_mul<SP>(zj, hp->pt_R[j], m), m.q);
    }
  }
  const u64 v = hps_round(hps_fsum<NL + 1, EX>(y, hp->invp, nB, 0.0));
  u64 *o = (p < 2) ? out01 + ((size_t)(ct * 2 + p) * L) * N + k : dc + ((size_t)ct * L) * N + k;
  for (int i = 0; i < (EX ? NL : (int)L); ++i) {
    const ModInfo m = mods[i];
    const u64 cq = behz_dot<NL + 1, SP, S60>(y, &hp->pstar_R[0][i], BEHZ_MAXL, nB, m);
    const u64 vp = csub63(mont_mul<SP>(v, hp->P_R[i], m), m.q);
    const u64 res = sub_mod(cq, vp, m.q);
    o[i * N] = p == 2 && dsc ? csub63(mont_mul<SP>(res, dsc[i], m), m.q) : res;
    if (p == 2) ext[((size_t)(ct * ndig + i / dig_len) * QP + i) * N + k] = csub63(mont_mul<SP>(res, m.r2, m), m.q);
  }
}

// CKKS rescale, the lift of the dropped limb (orc_rescale): x = INTT(c_{m})
// in [0, q_m) becomes, for each remaining modulus q_i, [x]_{q_i} if
// x <= q_m / 2, else [x - q_m]_{q_i} (the central lift OpenFHE's SwitchModulus
// and SEAL's divide_and_round_q_last use).  x [2n][N] -> conv [2n][m][N],
// canonical; the NTT of conv and the finish (c_i - NTT(conv)) q_m^-1 run in
// ntt_fwd_combine_launch.
template <bool SP>
__global__ void __launch_bounds__(EW_BLOCK) rescale_lift_kernel(const u64 *__restrict__ x, u64 *__restrict__ conv,
                                                                const ModInfo *mods, const u64 *qm_mod, u32 m,
                                                                u64 half, u32 log_n) {
  const u32 k = blockIdx.x * EW_BLOCK + threadIdx.x;
  const u32 p = blockIdx.y / m, i = blockIdx.y % m;
  const size_t N = (size_t)1 << log_n;
  const ModInfo mi = mods[i];
  const u64 v = x[(size_t)p * N + k];
  u64 r = reduce128<SP>(U128{v, 0}, mi);  // exact v mod q_i
  if (v > half) r = sub_mod(r, qm_mod[i], mi.q);
  conv[((size_t)p * m + i) * N + k] = r;
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
  dim3 grid(c->n / (EW_BLOCK * CONV_CPT), n);
  if (t.ns <= 4) hipLaunchKernelGGL((conv_kernel<4, SP>), grid, dim3(EW_BLOCK), 0, c->stream, src, ss, dst, ds, t, c->d_mods, c->log_n);
  else if (t.ns <= 8) hipLaunchKernelGGL((conv_kernel<8, SP>), grid, dim3(EW_BLOCK), 0, c->stream, src, ss, dst, ds, t, c->d_mods, c->log_n);
  else if (t.ns <= 16) hipLaunchKernelGGL((conv_kernel<16, SP>), grid, dim3(EW_BLOCK), 0, c->stream, src, ss, dst, ds, t, c->d_mods, c->log_n);
  else return fhe_fail(c, FHE_ERR_UNSUPPORTED, "base conversion with more than 16 source moduli");
  return fhe_check(c, hipGetLastError(), "conv_kernel");
}

template <bool SP>
int modup_impl(fhe_ctx *c, const u64 *dc, u32 dcs, u64 *ext, u32 n, u32 ndig) {
  dim3 grid(c->n / (EW_BLOCK * CONV_CPT), n * ndig);
  const u32 QP = c->L + c->K;
  if (c->alpha <= 4)
    hipLaunchKernelGGL((modup_kernel<4, SP>), grid, dim3(EW_BLOCK), 0, c->stream, dc, dcs, ext, c->d_modup, c->d_mods, QP, c->alpha, ndig, c->log_n);
  else if (c->alpha <= 8)
    hipLaunchKernelGGL((modup_kernel<8, SP>), grid, dim3(EW_BLOCK), 0, c->stream, dc, dcs, ext, c->d_modup, c->d_mods, QP, c->alpha, ndig, c->log_n);
  else
    hipLaunchKernelGGL((modup_kernel<16, SP>), grid, dim3(EW_BLOCK), 0, c->stream, dc, dcs, ext, c->d_modup, c->d_mods, QP, c->alpha, ndig, c->log_n);
  return fhe_check(c, hipGetLastError(), "modup_kernel");
}

// limbs [limb0, limb0 + nl) of Q u P
template <bool SP>
int inner_impl(fhe_ctx *c, const u64 *ext, const u64 *ksk, u64 *acc, u32 n, u32 ndig, u32 limb0, u32 nl) {
  const u32 QP = c->L + c->K, kQP = ctx_key_qp(c), L = c->L, ks = c->key_pshift;
  dim3 grid(c->n / EW_BLOCK, nl);
  if (ndig <= 4)
    hipLaunchKernelGGL((ks_inner_kernel<SP, 4>), grid, dim3(EW_BLOCK), 0, c->stream, ext, ksk, acc, c->d_mods, QP, ndig, n, c->log_n, limb0, kQP, L, ks);
  else if (ndig <= 8)
    hipLaunchKernelGGL((ks_inner_kernel<SP, 8>), grid, dim3(EW_BLOCK), 0, c->stream, ext, ksk, acc, c->d_mods, QP, ndig, n, c->log_n, limb0, kQP, L, ks);
  else if (ndig <= 16)
    hipLaunchKernelGGL((ks_inner_kernel<SP, 16>), grid, dim3(EW_BLOCK), 0, c->stream, ext, ksk, acc, c->d_mods, QP, ndig, n, c->log_n, limb0, kQP, L, ks);
  else
    hipLaunchKernelGGL((ks_inner_kernel<SP, 0>), grid, dim3(EW_BLOCK), 0, c->stream, ext, ksk, acc, c->d_mods, QP, ndig, n, c->log_n, limb0, kQP, L, ks);
  return fhe_check(c, hipGetLastError(), "ks_inner_kernel");
}

template <bool SP>
int ks_prep_impl(fhe_ctx *c, const u64 *d, u32 d_stride, u64 *dc, u64 *ext, u32 n, u32 ndig,
                 const u64 *dsc = nullptr) {
  hipLaunchKernelGGL((ks_prep_kernel<SP>), dim3(c->n / EW_BLOCK, n * c->L), dim3(EW_BLOCK), 0, c->stream, d, d_stride,
                     dc, ext, c->d_mods, c->L, c->L + c->K, c->alpha, ndig, c->log_n, dsc);
  return fhe_check(c, hipGetLastError(), "ks_prep_kernel");
}

// g^-1 mod 2N (g odd) by Newton iteration on the 2-adic inverse
static u32 galois_inv(u32 g, u32 log_n) {
  u32 inv = g;
  for (int i = 0; i < 5; ++i) inv *= 2u - g * inv;
  return inv & ((2u << log_n) - 1);
}

template <bool SP>
int automorph_ks_impl(fhe_ctx *c, const u64 *ct, u64 *base, u64 *dc, u64 *ext, u32 g, u32 n, u32 ndig, bool ntt,
                      const u64 *dsc = nullptr) {
  dim3 grid(c->n / EW_BLOCK, n * c->L);
  const u32 QP = c->L + c->K;
  if (ntt) {
    hipLaunchKernelGGL((automorph_ks_kernel<SP, true>), grid, dim3(EW_BLOCK), 0, c->stream, ct, base, dc, ext, g,
                       c->d_mods, c->L, QP, c->alpha, ndig, c->log_n, dsc);
  } else {
    const u32 inv = galois_inv(g, c->log_n);
    hipLaunchKernelGGL((automorph_ks_kernel<SP, false>), grid, dim3(EW_BLOCK), 0, c->stream, ct, base, dc, ext, inv,
                       c->d_mods, c->L, QP, c->alpha, ndig, c->log_n, dsc);
  }
  return fhe_check(c, hipGetLastError(), "automorph_ks_kernel");
}

template <bool SP>
int combine_impl(fhe_ctx *c, const u64 *acc, const u64 *conv, const u64 *base, u64 *out, u32 n, u32 add_mask) {
  const u32 L = c->L, QP = c->L + c->K;
  hipLaunchKernelGGL((ks_combine_kernel<SP>), dim3(c->n / EW_BLOCK, n * 2 * L), dim3(EW_BLOCK), 0, c->stream, acc,
                     conv, base, out, c->d_pinv, c->d_mods, L, QP, c->log_n, add_mask);
  return fhe_check(c, hipGetLastError(), "ks_combine_kernel");
}

// the S60 BEHZ kernels: every Q modulus below 2^60 (the other side of each of
// their dot products is then below 2^60: dot_cols_sp60's bound)
static bool behz_q60(const fhe_ctx *c) {
  for (u32 i = 0; i < c->L; ++i)
    if (c->moduli[i] >= (1ull << 60)) return false;
  return true;
}
// HPS's conversions on the in-place column sums (dot_sp60_canon): Q below 2^60
// (Q -> Bsk: the sources; Bsk -> Q: the targets and their constants) and every
// Bsk modulus below 2^61 (the sp60 reduction's bound on the modulus)
static bool hps_sp60(const fhe_ctx *c) {
  if (!HPS_S60 || !behz_q60(c)) return false;
  for (u32 j = 0; j < c->nB; ++j)
    if (c->moduli[c->L + c->K + j] >= (1ull << 61)) return false;
  return true;
}

template <bool SP>
int behz_extend_impl(fhe_ctx *c, const u64 *a, const u64 *b, u64 *xb, u32 n) {
  dim3 grid(c->n / EW_BLOCK, 4 * n);
  const BehzDev *bz = (const BehzDev *)c->behz;
#if BEHZ_MFMA
  if (SP && c->L == 8 && c->n >= 128)
    hipLaunchKernelGGL(behz_extend_mfma_kernel, dim3(c->n / 128, 4 * n), dim3(EW_BLOCK), 0, c->stream, a, b, xb, bz,
                       c->d_mods, c->log_n, n);
  else
#endif
  if (c->L == 8 && behz_q60(c)) hipLaunchKernelGGL((behz_extend_kernel<8, SP, true, true>), grid, dim3(EW_BLOCK), 0, c->stream, a, b, xb, bz, c->d_mods, c->log_n, n);
  else if (c->L <= 8) hipLaunchKernelGGL((behz_extend_kernel<8, SP, false, false>), grid, dim3(EW_BLOCK), 0, c->stream, a, b, xb, bz, c->d_mods, c->log_n, n);
  else if (c->L <= 16) hipLaunchKernelGGL((behz_extend_kernel<16, SP, false, false>), grid, dim3(EW_BLOCK), 0, c->stream, a, b, xb, bz, c->d_mods, c->log_n, n);
  else hipLaunchKernelGGL((behz_extend_kernel<24, SP, false, false>), grid, dim3(EW_BLOCK), 0, c->stream, a, b, xb, bz, c->d_mods, c->log_n, n);
  return fhe_check(c, hipGetLastError(), "behz_extend");
}

template <bool SP>
int behz_floor_impl(fhe_ctx *c, const u64 *eq, const u64 *eb, u64 *out01, u64 *dc, u64 *ext, u32 n, u32 ndig,
                    const u64 *dsc) {
  dim3 grid(c->n / EW_BLOCK, n * 3);
  const BehzDev *bz = (const BehzDev *)c->behz;
  const u32 QP = c->L + c->K;
#if BEHZ_MFMA
  if (SP && c->L == 8 && c->n >= 128)
    hipLaunchKernelGGL(behz_floor_mfma_kernel, dim3(c->n / 128, n * 3), dim3(EW_BLOCK), 0, c->stream, eq, eb, out01,
                       dc, ext, bz, c->d_mods, c->log_n, QP, c->alpha, ndig, dsc);
  else
#endif
  if (c->L == 8 && behz_q60(c)) hipLaunchKernelGGL((behz_floor_kernel<8, SP, true, true>), grid, dim3(EW_BLOCK), 0, c->stream, eq, eb, out01, dc, ext, bz, c->d_mods, c->log_n, QP, c->alpha, ndig, dsc);
  else if (c->L <= 8) hipLaunchKernelGGL((behz_floor_kernel<8, SP, false, false>), grid, dim3(EW_BLOCK), 0, c->stream, eq, eb, out01, dc, ext, bz, c->d_mods, c->log_n, QP, c->alpha, ndig, dsc);
  else if (c->L <= 16) hipLaunchKernelGGL((behz_floor_kernel<16, SP, false, false>), grid, dim3(EW_BLOCK), 0, c->stream, eq, eb, out01, dc, ext, bz, c->d_mods, c->log_n, QP, c->alpha, ndig, dsc);
  else hipLaunchKernelGGL((behz_floor_kernel<24, SP, false, false>), grid, dim3(EW_BLOCK), 0, c->stream, eq, eb, out01, dc, ext, bz, c->d_mods, c->log_n, QP, c->alpha, ndig, dsc);
  return fhe_check(c, hipGetLastError(), "behz_floor");
}

template <bool SP>
int hps_extend_impl(fhe_ctx *c, const u64 *a, const u64 *b, u64 *xb, u32 n) {
  dim3 grid(c->n / EW_BLOCK, 4 * n);
  const HpsDev *hp = (const HpsDev *)c->hps;
  if (c->L == 8 && hps_sp60(c)) hipLaunchKernelGGL((hps_extend_kernel<8, SP, true, true>), grid, dim3(EW_BLOCK), 0, c->stream, a, b, xb, hp, c->d_mods, c->log_n, n);
  else if (c->L == 8) hipLaunchKernelGGL((hps_extend_kernel<8, SP, true>), grid, dim3(EW_BLOCK), 0, c->stream, a, b, xb, hp, c->d_mods, c->log_n, n);
  else if (c->L <= 8) hipLaunchKernelGGL((hps_extend_kernel<8, SP, false>), grid, dim3(EW_BLOCK), 0, c->stream, a, b, xb, hp, c->d_mods, c->log_n, n);
  else if (c->L <= 16) hipLaunchKernelGGL((hps_extend_kernel<16, SP, false>), grid, dim3(EW_BLOCK), 0, c->stream, a, b, xb, hp, c->d_mods, c->log_n, n);
  else hipLaunchKernelGGL((hps_extend_kernel<24, SP, false>), grid, dim3(EW_BLOCK), 0, c->stream, a, b, xb, hp, c->d_mods, c->log_n, n);
  return fhe_check(c, hipGetLastError(), "hps_extend");
}

template <bool SP>
int hps_scale_impl(fhe_ctx *c, const u64 *eq, const u64 *eb, u64 *out01, u64 *dc, u64 *ext, u32 n, u32 ndig,
                   const u64 *dsc) {
  dim3 grid(c->n / EW_BLOCK, n * 3);
  const HpsDev *hp = (const HpsDev *)c->hps;
  const u32 QP = c->L + c->K;
  if (c->L == 8 && hps_sp60(c)) hipLaunchKernelGGL((hps_scale_kernel<8, SP, true, true>), grid, dim3(EW_BLOCK), 0, c->stream, eq, eb, out01, dc, ext, hp, c->d_mods, c->log_n, QP, c->alpha, ndig, dsc);
  else if (c->L == 8) hipLaunchKernelGGL((hps_scale_kernel<8, SP, true>), grid, dim3(EW_BLOCK), 0, c->stream, eq, eb, out01, dc, ext, hp, c->d_mods, c->log_n, QP, c->alpha, ndig, dsc);
  else if (c->L <= 8) hipLaunchKernelGGL((hps_scale_kernel<8, SP, false>), grid, dim3(EW_BLOCK), 0, c->stream, eq, eb, out01, dc, ext, hp, c->d_mods, c->log_n, QP, c->alpha, ndig, dsc);
  else if (c->L <= 16) hipLaunchKernelGGL((hps_scale_kernel<16, SP, false>), grid, dim3(EW_BLOCK), 0, c->stream, eq, eb, out01, dc, ext, hp, c->d_mods, c->log_n, QP, c->alpha, ndig, dsc);
  else hipLaunchKernelGGL((hps_scale_kernel<24, SP, false>), grid, dim3(EW_BLOCK), 0, c->stream, eq, eb, out01, dc, ext, hp, c->d_mods, c->log_n, QP, c->alpha, ndig, dsc);
  return fhe_check(c, hipGetLastError(), "hps_scale");
}

#define SP_DISPATCH(c, fn, ...) ((c)->special ? fn<true>(__VA_ARGS__) : fn<false>(__VA_ARGS__))

}  // namespace

// =================================================================== host

// The per-coefficient kernels put (item, limb) on gridDim.y (< 2^16): larger
// batches are issued as several launches over whole polys.
static u32 polys_per_launch(u32 n_limbs) { return std::max<u32>(1, kMaxGridY / std::max<u32>(1, n_limbs)); }

int ew_launch(fhe_ctx *c, EwOp op, const u64 *a, const u64 *b, u64 *out, u32 n_polys, u32 mod_begin, u32 n_limbs) {
  const u32 per = polys_per_launch(n_limbs);
  for (u32 p0 = 0; p0 < n_polys; p0 += per) {
    const u32 np = std::min(per, n_polys - p0);
    const size_t off = (size_t)p0 * n_limbs * c->n;
    const int rc = SP_DISPATCH(c, ew_impl, c, op, a + off, b + off, out + off, np * n_limbs, mod_begin, n_limbs);
    if (rc) return rc;
  }
  return FHE_OK;
}

int fill_uniform_launch(fhe_ctx *c, u64 *data, u32 n_polys, u32 mod_begin, u32 n_limbs, u64 seed) {
  const u32 per = polys_per_launch(n_limbs);
  for (u32 p0 = 0; p0 < n_polys; p0 += per) {
    const u32 np = std::min(per, n_polys - p0);
    hipLaunchKernelGGL(fill_kernel, dim3(c->n / EW_BLOCK, np * n_limbs), dim3(EW_BLOCK), 0, c->stream, data,
                       c->d_mods, mod_begin, n_limbs, c->log_n, seed, p0 * n_limbs);
    const int rc = fhe_check(c, hipGetLastError(), "fill_kernel");
    if (rc) return rc;
  }
  return FHE_OK;
}

int conv_launch(fhe_ctx *c, const ConvTab &t, const u64 *src, u32 src_poly_stride, u64 *dst, u32 dst_poly_stride,
                u32 n) {
  for (u32 p0 = 0; p0 < n; p0 += kMaxGridY) {
    const u32 np = std::min(kMaxGridY, n - p0);
    const int rc = SP_DISPATCH(c, conv_impl, c, t, src + (size_t)p0 * src_poly_stride * c->n, src_poly_stride,
                               dst + (size_t)p0 * dst_poly_stride * c->n, dst_poly_stride, np);
    if (rc) return rc;
  }
  return FHE_OK;
}

size_t keyswitch_ws_bytes(const fhe_ctx *c, u32 n) {
  const size_t N = c->n, L = c->L, QP = c->L + c->K;
  return sizeof(u64) * N * n * (L + c->dnum * QP + 2 * QP + 2 * L);
}

// Key-switch scratch layout (keyswitch_ws_bytes):
//   dc   [n][L][N]        the input d; INTT'd in place for CKKS
//   ext  [n][ndig][QP][N] ModUp output times R (own-digit limbs written by the producer)
//   acc  [n][2][QP][N]    inner product
//   conv [n][2][L][N]     ModDown conversion
struct KsWs {
  u64 *dc, *ext, *acc, *conv;
  u32 ndig;
};
#ifndef BFV_KS_FUSE
#define BFV_KS_FUSE 1  // BFV mul+relin: the fused relinearisation (bfv_ks_fused) where the context allows it
#endif
#ifndef KSP_FUSE
#define KSP_FUSE 1  // the P limbs' inner product inside INTT(acc_P)'s first pass (0: ks_inner_kernel)
#endif
#ifndef ROT_FUSE
#define ROT_FUSE 1  // CKKS rotation: the fused key-switch finish (ntt_ksf.hip) where it applies
#endif
#ifndef TENSOR_SPLIT
#define TENSOR_SPLIT 1  // CKKS mul+relin: d0, d1 formed in the ModDown finish (ckks_mul_relin_impl)
#endif
static bool ranges_overlap(const u64 *x, const u64 *y, size_t bytes) {
  const char *p = (const char *)x, *q = (const char *)y;
  return p < q + bytes && q < p + bytes;
}
static KsWs ks_layout(const fhe_ctx *c, u32 n, u64 *ws) {
  const size_t L = c->L, QP = c->L + c->K, N = c->n;
  KsWs w;
  w.ndig = (c->L + c->alpha - 1) / c->alpha;
  w.dc = ws;
  w.ext = w.dc + n * L * N;
  w.acc = w.ext + n * w.ndig * QP * N;
  w.conv = w.acc + n * 2 * QP * N;
  return w;
}

// Hybrid key switching on a PREPARED scratch (dc and the own-digit limbs of
// ext filled by ks_prep / the tensor INTT prologue / automorph_ks / the BEHZ floor).
//   out : [n][2][L][N], out_b = (add_mask bit b ? base_b : 0) + KS(d)_b;
//         base may alias out (element-wise).
//   base_g (NTT form with the fused ModDown only): base_b is read as
//         sigma_g(base_b); base must not overlap out.
// Split in two for hoisted rotations: ks_extend (steps 1-3: INTT, ModUp, NTT of
// the converted limbs, into w.ext) runs once per input, ks_finish (steps 4-6:
// inner product, ModDown) once per key.
// rows_scale (CONVF): dc holds INTT(d)'s row-pass output, whose column pass
// (output scale rows_scale) runs inside ModUp's CONVF launches
static int ks_extend(fhe_ctx *c, const KsWs &w, u32 n, bool ntt_form, bool dc_is_coef, bool q_rows = true,
                     const u64 *rows_scale = nullptr) {
  const u32 L = c->L, QP = L + c->K, N = c->n, ndig = w.ndig;
  u64 *dc = w.dc, *ext = w.ext;
  int rc;
  // CKKS at two-pass sizes: ModUp runs inside the column pass of the NTT of
  // its outputs (ntt_fwd_modup_launch); dc then holds ModUp's scaled sources
  const bool fused_modup = ntt_form && c->fuse_modup;
  // 1. INTT d (CKKS), unless the producer already did (ntt_inv_tensor_launch)
  if (ntt_form && !dc_is_coef &&
      (rc = ntt_launch(c, LimbMap{dc, L, L, 0, L, 0, 0, n}, true, !fused_modup && c->fold_ninv, false,
                       fused_modup ? c->d_iscale : nullptr)))
    return rc;
  if (fused_modup) {
    // 2-3. ModUp + NTT of the converted limbs, one digit at a time
    for (u32 j = 0; j < ndig; ++j)
      if ((rc = ntt_fwd_modup_launch(c, dc, ext, n, ndig, j, q_rows, true, rows_scale))) return rc;
  }
  if (!q_rows && !fused_modup) return fhe_fail(c, FHE_ERR_INVALID, "ModUp without Q rows: fused ModUp only");
  // 2. ModUp: every non-own limb of every digit
  if (!fused_modup && (rc = SP_DISPATCH(c, modup_impl, c, dc, L, ext, n, ndig))) return rc;
  // 3. NTT the converted limbs (all limbs for BFV, whose own limbs are coefficient form)
  for (u32 j = 0; j < ndig && !fused_modup; ++j) {
    const u32 lo = j * c->alpha, hi = std::min(lo + c->alpha, L);
    LimbMap m{ext + (size_t)j * QP * N, ndig * QP, ntt_form ? QP - (hi - lo) : QP, 0,
              ntt_form ? lo : QP, ntt_form ? hi - lo : 0, 0, n};
    // special moduli: the inner product's Montgomery products take the lazy
    // (< 8q) NTT outputs as they are, so the last pass skips canonicalising
    if ((rc = ntt_launch(c, m, false, false, c->special))) return rc;
  }
  return FHE_OK;
}

// ext_g (NTT form, fused ModDown, at most 4 digits only): the inner product
// reads ext as sigma_g(ext) (EPI_KSQG / PRO_KSPG)
static bool ks_fused_inner(const fhe_ctx *c, u32 ndig, bool ntt_form) {
  return ntt_form && c->fuse_moddown && ndig <= 4 && KSP_FUSE;
}
static int ks_finish(fhe_ctx *c, const KsWs &w, const u64 *ext, const u64 *ksk, const u64 *base, u64 *out, u32 n,
                     u32 add_mask, bool ntt_form, u32 base_g, u32 ext_g, const TensorSrc *tsrc = nullptr) {
  const u32 L = c->L, K = c->K, QP = L + K, N = c->n, ndig = w.ndig;
  u64 *acc = w.acc, *conv = w.conv;
  int rc;
  if (ext_g && !ks_fused_inner(c, ndig, ntt_form))
    return fhe_fail(c, FHE_ERR_UNSUPPORTED, "gathered key-switch input without the fused inner product");
  // 4. inner product with the key.  With the fused ModDown and at most 4
  //    digits, the Q limbs' inner product runs inside the last pass of
  //    NTT(conv) (EPI_KSQ), so only the P limbs (ModDown's sources) are formed
  //    here: acc_Q is never written and read back
  //    The P limbs' inner product runs likewise inside the first pass of
  //    INTT(acc_P) (PRO_KSP): no ks_inner_kernel at all
  const bool ksq = ntt_form && c->fuse_moddown && ndig <= 4;
  if (!(ksq && KSP_FUSE) && (rc = SP_DISPATCH(c, inner_impl, c, ext, ksk, acc, n, ndig, ksq ? L : 0, ksq ? K : QP)))
    return rc;
  // 5-6. ModDown for NTT-form results: INTT the P part with the conversion's
  //      source constants as its output scale, then NTT(conv) with the P -> Q
  //      conversion in its first pass and the combine in its last
  //      (out = base + (acc_Q - conv) P^-1): conv never makes an HBM round trip
  if (ntt_form && c->fuse_moddown) {
    if (tsrc && tsrc->fused) rc = ntt_ksp_fused_launch(c, acc, ext, ksk, n, ndig, false, tsrc->convf);
    else if (ksq && KSP_FUSE) rc = ntt_inv_ksp_launch(c, acc, ext, ksk, n, ndig, ext_g);
    else rc = ntt_launch(c, LimbMap{acc, QP, K, L, QP, 0, 0, 2 * n}, true, false, false, c->d_iscale);
    if (rc) return rc;
    if (tsrc && !(ksq && KSP_FUSE)) return fhe_fail(c, FHE_ERR_INVALID, "split tensor product without EPI_KSQ");
    const ConvTab *md = tsrc && tsrc->fused ? &c->moddown_ksf : &c->moddown;  // the fused finish's scale
    return ntt_fwd_combine_launch(c, conv, 2 * n, acc, QP, base, out, add_mask, md, ksq ? ext : nullptr,
                                  ksk, ndig, base_g, nullptr, nullptr, ext_g, nullptr, tsrc);
  }
  if (base_g) return fhe_fail(c, FHE_ERR_UNSUPPORTED, "rotated key-switch base without the fused ModDown");
  // 5. ModDown: INTT the P part (all of Q u P for BFV), convert P -> Q
  if ((rc = ntt_launch(c, LimbMap{acc, QP, ntt_form ? K : QP, ntt_form ? L : 0, QP, 0, 0, 2 * n}, true,
                       ntt_form && c->fold_ninv)))
    return rc;
  if ((rc = conv_launch(c, c->moddown, acc + (size_t)L * N, QP, conv, L, 2 * n))) return rc;
  // 6. combine: fused into the last pass of NTT(conv) for NTT-form results
  if (ntt_form) return ntt_fwd_combine_launch(c, conv, 2 * n, acc, QP, base, out, add_mask);
  return SP_DISPATCH(c, combine_impl, c, acc, conv, base, out, n, add_mask);
}

static int keyswitch_run(fhe_ctx *c, const KsWs &w, const u64 *ksk, const u64 *base, u64 *out, u32 n, u32 add_mask,
                         bool ntt_form, bool dc_is_coef = false, u32 base_g = 0, const TensorSrc *tsrc = nullptr) {
  const u64 *rows_scale = tsrc && tsrc->convf ? c->d_iscale_t : nullptr;  // INTT(d2)'s scale (ntt_inv_tensor_launch)
  int rc = ks_extend(c, w, n, ntt_form, dc_is_coef, !(tsrc && tsrc->fused), rows_scale);
  return rc ? rc : ks_finish(c, w, w.ext, ksk, base, out, n, add_mask, ntt_form, base_g, 0, tsrc);
}

// BFV_MD_COEF: one thread per coefficient of a poly forms all L outputs (the
// K P-limb sources read once into registers instead of once per output limb
// through L2)
#ifndef BFV_MD_COEF
#define BFV_MD_COEF 1
#endif
namespace {
template <bool SP>
__global__ void __launch_bounds__(EW_BLOCK) bfv_moddown_coef_kernel(const u64 *__restrict__ acc, const u64 *base,
                                                                    u64 *out, const u64 *__restrict__ h,
                                                                    const u64 *pinv, const ModInfo *mods, u32 L,
                                                                    u32 K, u32 QP, u32 log_n, u32 add_mask,
                                                                    u32 base_ginv, BfvRotOut ro) {
  const u32 k = blockIdx.x * EW_BLOCK + threadIdx.x;
  const u32 p = blockIdx.y;  // 2 ct + b (of the rotation batch)
  u32 cp = p;
  if (ro.rp) {
    const u32 r = p / ro.rp;
    cp = p - r * ro.rp;
    out = ro.out[r];
    base_ginv = ro.ginv[r];
  }
  const size_t N = (size_t)1 << log_n;
  const u64 *ap = acc + (size_t)p * QP * N + k;
  u64 v[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) v[j] = j < (int)K ? ap[(size_t)(L + j) * N] : 0;
  const bool add = add_mask & (1u << (p & 1));
  const u32 n = 1u << log_n, j0 = (u32)(((u64)k * base_ginv) & (2 * n - 1));
  for (u32 i = 0; i < L; ++i) {
    const ModInfo m = mods[i];
    u32 h0[4], h1[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (j < (int)K) split31(h[(size_t)j * L + i], h0[j], h1[j]);
      else h0[j] = h1[j] = 0;
    }
    const u64 cv = csub63(dot_cols<4, SP>(v, h0, h1, m), m.q);
    u64 ks = csub63(mont_mul<SP>(sub_mod(ap[(size_t)i * N], cv, m.q), pinv[i], m), m.q);
    const size_t o = ((size_t)cp * L + i) * N + k;
    if (add) {
      u64 bv;
      if (base_ginv) {
        const u64 *bp = base + ((size_t)cp * L + i) * N;
        bv = j0 < n ? bp[j0] : (bp[j0 - n] ? m.q - bp[j0 - n] : 0);
      } else {
        bv = base[o];
      }
      ks = add_mod(ks, bv, m.q);
    }
    out[o] = ks;
  }
}
}  // namespace

template <bool SP>
static int bfv_moddown_impl(fhe_ctx *c, const u64 *acc, const u64 *base, u64 *out, u32 n, u32 add_mask,
                            u32 base_ginv, const RotBatch *rb = nullptr) {
  const u32 L = c->L, per = std::max<u32>(1, kMaxGridY / L);
  const size_t N = c->n, QP = c->L + c->K;
  BfvRotOut ro{};
  const u32 nr = rb ? rb->nr : 1;
  if (rb) {
    // one launch over the batch: acc holds nr rotations of the n ciphertexts
    if (nr < 1 || nr > FHE_ROT_BATCH || 2 * n * nr > per) return fhe_fail(c, FHE_ERR_INVALID, "rotation batch");
    ro.rp = 2 * n;
    for (u32 r = 0; r < nr; ++r) {
      ro.out[r] = rb->out[r];
      ro.ginv[r] = galois_inv(rb->g[r], c->log_n);
    }
  }
  if (BFV_MD_COEF && c->K <= 4 && 2 * n * nr <= kMaxGridY) {
    hipLaunchKernelGGL((bfv_moddown_coef_kernel<SP>), dim3(c->n / EW_BLOCK, 2 * n * nr), dim3(EW_BLOCK), 0,
                       c->stream, acc, base, rb ? nullptr : out, c->moddown.h, c->d_pinv, c->d_mods, L, c->K,
                       (u32)QP, c->log_n, add_mask, base_ginv, ro);
    return fhe_check(c, hipGetLastError(), "bfv_moddown_coef_kernel");
  }
  for (u32 p0 = 0; p0 < 2 * n * nr; p0 += per) {
    const u32 np = std::min(per, 2 * n * nr - p0);
    hipLaunchKernelGGL((bfv_moddown_kernel<SP>), dim3(c->n / EW_BLOCK, np * L), dim3(EW_BLOCK), 0, c->stream,
                       acc + (size_t)p0 * QP * N, base + (rb ? 0 : (size_t)p0 * L * N),
                       rb ? nullptr : out + (size_t)p0 * L * N, c->moddown.h, c->d_pinv, c->d_mods, L, c->K,
                       (u32)QP, c->log_n, add_mask, base_ginv, ro);
    int rc = fhe_check(c, hipGetLastError(), "bfv_moddown_kernel");
    if (rc) return rc;
  }
  return FHE_OK;
}

// BFV relinearisation at two-pass sizes (c->bfv_ks_fuse), the coefficient-
// domain counterpart of keyswitch_run's fused CKKS path, on a prepared scratch
// whose dc holds ModUp's SCALED sources (the floor's dsc) and whose ext holds
// the own-digit limbs d R (coefficient form):
//   ModUp of digit j inside the column pass of the NTT of its converted limbs
//   (ntt_fwd_modup_launch), the own limbs' NTT, then INTT(acc) over every limb
//   of Q u P with the inner product in its first pass (PRO_KSP over all
//   limbs; the P limbs come out as ModDown's v_k, the Q limbs as plain
//   coefficients), and ModDown + combine in one kernel (bfv_moddown_kernel):
//   no ModUp, inner-product or conversion intermediate reaches HBM.
// Split for hoisted rotations: bfv_ks_extend once per input, bfv_ks_finish per
// key (ext_g: the inner product reads sigma_g(ext), PRO_KSPG; base_ginv: the
// base is read as sigma_g(base) by the coefficient map, base apart from out).
// extfree (round 6, bfv_ks_extfree_ok): ext keeps every digit's COLUMN-pass
// intermediates (ModUp's targets and the own limbs' column pass), and the
// all-limb fused pass (ksp_fused_pass) row-transforms them itself: ext is never
// written by a row pass and never read back.  Hoisted rotations gather ext
// through sigma_g and keep the stored, row-transformed ext.
static bool bfv_fused(const fhe_ctx *c) { return c->bfv_ks_fuse && BFV_KS_FUSE; }
static int bfv_ks_extend(fhe_ctx *c, const KsWs &w, u32 n, bool extfree = false) {
  const u32 L = c->L, QP = L + c->K, N = c->n, ndig = w.ndig;
  int rc;
  for (u32 j = 0; j < ndig; ++j)
    if ((rc = ntt_fwd_modup_launch(c, w.dc, w.ext, n, ndig, j, !extfree, false))) return rc;
  for (u32 j = 0; j < ndig; ++j) {
    const u32 lo = j * c->alpha, hi = std::min(lo + c->alpha, L);
    const LimbMap own{w.ext + (size_t)j * QP * N, ndig * QP, hi - lo, lo, hi - lo, 0, 0, n};
    if (extfree) {
      if ((rc = ntt_fwd_col_launch(c, own))) return rc;
    } else if ((rc = ntt_launch(c, own, false, false, c->special))) {
      return rc;
    }
  }
  return FHE_OK;
}
static int bfv_ks_finish(fhe_ctx *c, const KsWs &w, const u64 *ksk, const u64 *base, u64 *out, u32 n, u32 add_mask,
                         u32 ext_g = 0, u32 base_ginv = 0, bool extfree = false) {
  int rc = extfree ? ntt_ksp_fused_launch(c, w.acc, w.ext, ksk, n, w.ndig, true)
                   : ntt_inv_ksp_launch(c, w.acc, w.ext, ksk, n, w.ndig, ext_g, true);
  return rc ? rc : SP_DISPATCH(c, bfv_moddown_impl, c, w.acc, base, out, n, add_mask, base_ginv);
}
static int bfv_ks_fused(fhe_ctx *c, const KsWs &w, const u64 *ksk, const u64 *base, u64 *out, u32 n, u32 add_mask,
                        u32 base_ginv = 0) {
  const bool ef = bfv_ks_extfree_ok(c, w.ndig);
  int rc = bfv_ks_extend(c, w, n, ef);
  return rc ? rc : bfv_ks_finish(c, w, ksk, base, out, n, add_mask, 0, base_ginv, ef);
}

// Hybrid key switching of an arbitrary input d ([n][d_stride limbs], the L
// limbs first; NTT form iff ntt_form).  d must not alias out.
int keyswitch_ex(fhe_ctx *c, const u64 *d, u32 d_stride, const u64 *ksk, const u64 *base, u64 *out, u32 n,
                 u32 add_mask, bool ntt_form, u64 *ws) {
  const KsWs w = ks_layout(c, n, ws);
  const bool fused = !ntt_form && bfv_fused(c);
  int rc = SP_DISPATCH(c, ks_prep_impl, c, d, d_stride, w.dc, w.ext, n, w.ndig, fused ? c->d_bfv_dscale : nullptr);
  if (rc) return rc;
  if (fused) return bfv_ks_fused(c, w, ksk, base, out, n, add_mask);
  return keyswitch_run(c, w, ksk, base, out, n, add_mask, ntt_form);
}

// CKKS ct x ct: the tensor product (and the KS preparation of d2) runs inside
// the first pass of INTT(d2) (ntt.hip PRO_TENSOR), then relinearise.
// At two-pass sizes with the fused inner product the tensor product is split
// (TENSOR_SPLIT): d2 = a1 b1 in INTT(d2)'s first pass (PRO_TENSOR2) and the
// base d0, d1 in the ModDown finish (EPI_KSQT), so d0 and d1 never make an HBM
// round trip.  The finish reads a and b after other workgroups have written
// out, so out must not overlap them; an aliased call takes the unsplit path.
int ckks_mul_relin_impl(fhe_ctx *c, const u64 *a, const u64 *b, const u64 *rlk, u64 *out, u32 n) {
  void *ws;
  int rc = ctx_workspace(c, keyswitch_ws_bytes(c, n), &ws);
  if (rc) return rc;
  const KsWs w = ks_layout(c, n, (u64 *)ws);
  const size_t bytes = sizeof(u64) * 2 * c->L * c->n * (size_t)n;
  // the fused key switch (ntt_ksf.hip) where it applies; else the split finish
  // EPI_KSQT on special moduli only (the generic-product EPI_KSQT keeps its
  // operand ring in scratch, -18%)
  const bool apart = !ranges_overlap(out, a, bytes) && !ranges_overlap(out, b, bytes);
  const bool pre = TENSOR_SPLIT && c->log_n > 14 && c->fuse_moddown && w.ndig <= 3 && KSP_FUSE && apart;
  const bool fused = pre && c->fuse_modup && ks_fused_finish_ok(c, w.ndig);
  const bool split = fused || (pre && c->special);
  // CONVF: INTT(d2)'s and INTT(acc_P)'s column passes run inside the ModUp and
  // ModDown conversion kernels (ntt_convf.hip): 4-limb digits and 4 P limbs
  const bool cf = fused && c->d_iscale_t && c->L % c->alpha == 0 && convf_ok(c, c->alpha) && convf_ok(c, c->K);
  if ((rc = ntt_inv_tensor_launch(c, a, b, out, w.dc, w.ext, n, w.ndig, split, cf))) return rc;
  const TensorSrc ts{a, b, fused, 0, cf};
  return keyswitch_run(c, w, rlk, out, out, n, 3u, true, true, 0, split ? &ts : nullptr);
}

// Rotation: automorphism (fused with the KS preparation of sigma(c1)) + KS.
int rotate_impl(fhe_ctx *c, const u64 *ct, u32 g, const u64 *gk, u64 *out, u32 n, bool ntt_form) {
  const size_t LN = (size_t)c->L * c->n;
  void *ws;
  int rc = ctx_workspace(c, sizeof(u64) * n * 2 * LN + keyswitch_ws_bytes(c, n), &ws);
  if (rc) return rc;
  u64 *base = (u64 *)ws;  // [n][2][L][N], poly 0 = sigma(c0)
  const KsWs w = ks_layout(c, n, base + n * 2 * LN);
  if (ntt_form && c->log_n > 14) {
    // CKKS at two-pass sizes: the automorphism runs inside the first pass of
    // INTT(sigma(c1)).  With the fused ModDown and out apart from ct, sigma(c0)
    // is never stored: the combine reads c0 through sigma_g itself
    const u64 *ce = ct + (size_t)n * 2 * LN;
    const bool apart = out + (size_t)n * 2 * LN <= ct || ce <= out;
    const bool read_sigma = c->fuse_moddown && apart;
    // the fused finish (ntt_ksf.hip) forms the own digit's sigma_g(c1) R itself
    const bool fused = read_sigma && ROT_FUSE && c->fuse_modup && KSP_FUSE && ks_fused_finish_ok(c, w.ndig);
    if ((rc = ntt_inv_automorph_launch(c, ct, g, read_sigma ? nullptr : base, w.dc, fused ? nullptr : w.ext, n,
                                       w.ndig)))
      return rc;
    const TensorSrc ts{ct, nullptr, true, g & ((2u << c->log_n) - 1)};
    return keyswitch_run(c, w, gk, read_sigma ? ct : base, out, n, 1u, true, true, read_sigma ? g : 0u,
                         fused ? &ts : nullptr);
  }
  if (!ntt_form && bfv_fused(c)) {
    // BFV at two-pass sizes: the fused key switch; with out apart from ct,
    // sigma(c0) is never stored (the ModDown kernel reads c0 through the
    // coefficient map)
    const u64 *ce = ct + (size_t)n * 2 * LN;
    const bool apart = out + (size_t)n * 2 * LN <= ct || ce <= out;
    if ((rc = SP_DISPATCH(c, automorph_ks_impl, c, ct, apart ? nullptr : base, w.dc, w.ext, g, n, w.ndig, false,
                          c->d_bfv_dscale)))
      return rc;
    return bfv_ks_fused(c, w, gk, apart ? ct : base, out, n, 1u, apart ? galois_inv(g, c->log_n) : 0);
  }
  if ((rc = SP_DISPATCH(c, automorph_ks_impl, c, ct, base, w.dc, w.ext, g, n, w.ndig, ntt_form, nullptr))) return rc;
  return keyswitch_run(c, w, gk, base, out, n, 1u, ntt_form);
}


// NTT-domain automorphism of whole rows: dst row r = sigma_g(src row r), rows
// taken rpg at a time from groups src_gs / dst_gs rows apart (the hoisted
// rotation's generic path: sigma_g on the ModUp output and on c0)
__global__ void __launch_bounds__(EW_BLOCK) aut_rows_kernel(const u64 *__restrict__ src, u32 src_gs,
                                                            u64 *__restrict__ dst, u32 dst_gs, u32 rpg, u32 g,
                                                            u32 log_n) {
  const u32 k = blockIdx.x * EW_BLOCK + threadIdx.x, r = blockIdx.y;
  const size_t N = (size_t)1 << log_n, grp = r / rpg, i = r % rpg;
  const u32 mask = (2u << log_n) - 1;
  const u32 e = 2 * (__brev(k) >> (32 - log_n)) + 1;
  const u32 e2 = (u32)(((u64)e * g) & mask);
  const u32 sk = __brev((e2 - 1) >> 1) >> (32 - log_n);
  dst[(grp * dst_gs + i) * N + k] = src[(grp * src_gs + i) * N + sk];
}
// the coefficient-domain automorphism of whole rows (BFV): dst[k g mod 2N] =
// +-src[k], i.e. dst[j] = +-src[j g^-1 mod 2N] (automorph_ks_kernel's map);
// row r of a group is limb r % rpg (its modulus for the sign flip)
__global__ void __launch_bounds__(EW_BLOCK) aut_rows_coef_kernel(const u64 *__restrict__ src, u32 src_gs,
                                                                 u64 *__restrict__ dst, u32 dst_gs, u32 rpg,
                                                                 u32 ginv, const ModInfo *mods, u32 log_n) {
  const u32 k = blockIdx.x * EW_BLOCK + threadIdx.x, r = blockIdx.y;
  const size_t N = (size_t)1 << log_n, grp = r / rpg, i = r % rpg;
  const u32 n = 1u << log_n, j0 = (u32)(((u64)k * ginv) & (2 * n - 1));
  const u64 *s = src + (grp * src_gs + i) * N;
  u64 v;
  if (j0 < n) {
    v = s[j0];
  } else {
    const u64 x = s[j0 - n];
    v = x ? mods[i].q - x : 0;
  }
  dst[(grp * dst_gs + i) * N + k] = v;
}

static int aut_rows(fhe_ctx *c, const u64 *src, u32 src_gs, u64 *dst, u32 dst_gs, u32 rpg, u32 n_rows, u32 g,
                    bool coef = false) {
  const u32 per = kMaxGridY / rpg * rpg;
  if (!per) return fhe_fail(c, FHE_ERR_UNSUPPORTED, "aut_rows: rows per group exceed the grid");
  const size_t N = c->n;
  for (u32 r0 = 0; r0 < n_rows; r0 += per) {
    const u32 nr = std::min(per, n_rows - r0), g0 = r0 / rpg;
    if (coef)
      hipLaunchKernelGGL(aut_rows_coef_kernel, dim3(c->n / EW_BLOCK, nr), dim3(EW_BLOCK), 0, c->stream,
                         src + (size_t)g0 * src_gs * N, src_gs, dst + (size_t)g0 * dst_gs * N, dst_gs, rpg, g,
                         c->d_mods, c->log_n);
    else
      hipLaunchKernelGGL(aut_rows_kernel, dim3(c->n / EW_BLOCK, nr), dim3(EW_BLOCK), 0, c->stream,
                         src + (size_t)g0 * src_gs * N, src_gs, dst + (size_t)g0 * dst_gs * N, dst_gs, rpg, g,
                         c->log_n);
    int rc = fhe_check(c, hipGetLastError(), "aut_rows_kernel");
    if (rc) return rc;
  }
  return FHE_OK;
}

// the gather path (sigma_g inside the fused inner-product passes) needs only
// the key-switch scratch; the generic one also sigma_g(ext) and sigma_g(c0)
static bool hoisted_gather(const fhe_ctx *c) {
  if (c->params.scheme != FHE_SCHEME_CKKS) return bfv_fused(c);  // BFV: PRO_KSPG over all limbs
  return c->log_n > 14 && ks_fused_inner(c, (c->L + c->alpha - 1) / c->alpha, true);
}
// CKKS gather path with few ciphertexts: up to FHE_ROT_BATCH Galois elements
// per launch of the gather passes, while the batch stays within ROT_BATCH_CTS
// ciphertexts' accumulators (a launch over one ciphertext fills 1.5 workgroups
// per CU; hoisting's common case is one ciphertext and many rotations)
constexpr u32 ROT_BATCH_CTS = 32;
static u32 hoisted_rot_batch(const fhe_ctx *c, u32 n) {
  if (!hoisted_gather(c)) return 1;
  return std::max<u32>(1, std::min<u32>(FHE_ROT_BATCH, ROT_BATCH_CTS / std::max<u32>(n, 1)));
}
size_t rotate_hoisted_ws_bytes(const fhe_ctx *c, u32 n) {
  const size_t N = c->n, L = c->L, QP = c->L + c->K, ndig = (c->L + c->alpha - 1) / c->alpha;
  const size_t nrb = hoisted_rot_batch(c, n);
  if (nrb > 1) return keyswitch_ws_bytes(c, n) + sizeof(u64) * N * n * nrb * (2 * QP + 2 * L);
  return keyswitch_ws_bytes(c, n) + (hoisted_gather(c) ? 0 : sizeof(u64) * N * n * (ndig * QP + 2 * L));
}

// Hoisted rotations (oracle orc_rotate_hoisted, OpenFHE EvalFastRotation):
// c1 is extended ONCE (INTT, ModUp, NTT of the converted limbs), then every
// Galois element g_r key-switches sigma_g(ext) -- not ModUp(sigma_g(c1)), so the
// bits differ from rotate_impl's by the ModUp error term -- and adds sigma_g(c0).
// Two-pass sizes with the fused inner product: sigma_g is a gather inside the
// inner-product passes (EPI_KSQG / PRO_KSPG) and the combine reads c0 through
// sigma_g, so a rotation costs its key switch's inner product and ModDown only.
// Otherwise sigma_g(ext) and sigma_g(c0) are materialised (aut_rows_kernel).
// BFV (coefficient form) takes that path too: ext is permuted in the NTT
// domain the inner product runs in, c0 by the signed coefficient map, and the
// finish is the coefficient-domain ModDown.  outs[r] must not overlap ct.
int rotate_hoisted_impl(fhe_ctx *c, const u64 *ct, u32 n_rot, const u32 *galois, const u64 *const *gks,
                        u64 *const *outs, u32 n) {
  const size_t LN = (size_t)c->L * c->n, QP = c->L + c->K;
  void *ws;
  int rc = ctx_workspace(c, rotate_hoisted_ws_bytes(c, n), &ws);
  if (rc) return rc;
  const KsWs w = ks_layout(c, n, (u64 *)ws);
  u64 *ext_g = w.conv + n * 2 * LN;      // [n][ndig][QP][N] (generic path)
  u64 *base = ext_g + n * w.ndig * QP * c->n;  // [n][2][L][N], poly 0 = sigma(c0) (generic path)
  const bool gather = hoisted_gather(c), ckks = c->params.scheme == FHE_SCHEME_CKKS;
  if (!ckks && gather) {
    // BFV on the fused passes: scaled ModUp sources, one extension, then per
    // element the gathered all-limb inner product and the coefficient-domain
    // ModDown reading c0 through the coefficient map
    if ((rc = SP_DISPATCH(c, ks_prep_impl, c, ct + LN, 2 * c->L, w.dc, w.ext, n, w.ndig, c->d_bfv_dscale))) return rc;
    if ((rc = bfv_ks_extend(c, w, n))) return rc;
    const u32 nrb = hoisted_rot_batch(c, n);
    if (nrb > 1) {
      // few ciphertexts: several Galois elements per launch (as CKKS below)
      u64 *accb = w.conv + (size_t)n * 2 * LN;
      for (u32 r0 = 0; r0 < n_rot; r0 += nrb) {
        RotBatch rb{};
        rb.nr = std::min(nrb, n_rot - r0);
        for (u32 r = 0; r < rb.nr; ++r) {
          rb.ksk[r] = gks[r0 + r];
          rb.out[r] = outs[r0 + r];
          rb.g[r] = galois[r0 + r];
        }
        if ((rc = ntt_inv_ksp_launch(c, accb, w.ext, nullptr, n, w.ndig, 0, true, &rb))) return rc;
        if ((rc = SP_DISPATCH(c, bfv_moddown_impl, c, accb, ct, nullptr, n, 1u, 0u, &rb))) return rc;
      }
      return FHE_OK;
    }
    for (u32 r = 0; r < n_rot; ++r)
      if ((rc = bfv_ks_finish(c, w, gks[r], ct, outs[r], n, 1u, galois[r], galois_inv(galois[r], c->log_n))))
        return rc;
    return FHE_OK;
  }
  if (ckks && c->log_n > 14) {
    // the identity automorphism: INTT(c1) with the ModUp source scaling and
    // the own-digit slots c1 R, as rotate_impl's fused prologue
    if ((rc = ntt_inv_automorph_launch(c, ct, 1u, nullptr, w.dc, w.ext, n, w.ndig))) return rc;
  } else if ((rc = SP_DISPATCH(c, ks_prep_impl, c, ct + LN, 2 * c->L, w.dc, w.ext, n, w.ndig, nullptr))) {
    return rc;
  }
  if ((rc = ks_extend(c, w, n, ckks, ckks && c->log_n > 14))) return rc;
  const u32 nrb = hoisted_rot_batch(c, n);
  if (nrb > 1) {
    // several Galois elements per launch: accumulators and conversions of the
    // batch after the key-switch scratch
    const u32 ndig = w.ndig;
    u64 *accb = w.conv + (size_t)n * 2 * LN, *convb = accb + (size_t)nrb * n * 2 * QP * c->n;
    for (u32 r0 = 0; r0 < n_rot; r0 += nrb) {
      RotBatch rb{};
      rb.nr = std::min(nrb, n_rot - r0);
      for (u32 r = 0; r < rb.nr; ++r) {
        rb.ksk[r] = gks[r0 + r];
        rb.out[r] = outs[r0 + r];
        rb.g[r] = galois[r0 + r];
      }
      if ((rc = ntt_inv_ksp_launch(c, accb, w.ext, nullptr, n, ndig, 0, false, &rb))) return rc;
      if ((rc = ntt_fwd_combine_launch(c, convb, 2 * n * rb.nr, accb, (u32)QP, ct, nullptr, 1u, &c->moddown, w.ext,
                                       nullptr, ndig, 0, nullptr, nullptr, 0, &rb)))
        return rc;
    }
    return FHE_OK;
  }
  for (u32 r = 0; r < n_rot; ++r) {
    const u32 g = galois[r];
    if (gather) {
      rc = ks_finish(c, w, w.ext, gks[r], ct, outs[r], n, 1u, true, g, g);
    } else {
      if ((rc = aut_rows(c, w.ext, w.ndig * QP, ext_g, w.ndig * QP, w.ndig * QP, n * w.ndig * QP, g))) return rc;
      const u32 gb = ckks ? g : galois_inv(g, c->log_n);
      if ((rc = aut_rows(c, ct, 2 * c->L, base, 2 * c->L, c->L, n * c->L, gb, !ckks))) return rc;
      rc = ks_finish(c, w, ext_g, gks[r], base, outs[r], n, 1u, ckks, 0, 0);
    }
    if (rc) return rc;
  }
  return FHE_OK;
}

size_t rotate_sum_ws_bytes(const fhe_ctx *c, u32 n) {
  return keyswitch_ws_bytes(c, n) + sizeof(u64) * c->n * (size_t)n * 2 * c->L;
}

// Double-hoisted rotation sum (orc_rotate_sum_hoisted_at; Bossuat et al.'s
// hoisted ModDown): c1 extended once, the inner products of every Galois
// element summed over Q u P (rot_sum_inner_kernel, sigma_g as a gather), ONE
// ModDown, plus sum_r sigma_{g_r}(c0).  out may alias ct (ct is read before the
// ModDown writes out).
int rotate_sum_hoisted_impl(fhe_ctx *c, const u64 *ct, u32 n_rot, const u32 *galois, const u64 *const *gks, u64 *out,
                            u32 n, const u64 *const *pts) {
  const size_t LN = (size_t)c->L * c->n;
  const u32 L = c->L, K = c->K, QP = L + K;
  const bool ckks = c->params.scheme == FHE_SCHEME_CKKS;
  void *ws;
  int rc = ctx_workspace(c, rotate_sum_ws_bytes(c, n), &ws);
  if (rc) return rc;
  const KsWs w = ks_layout(c, n, (u64 *)ws);
  u64 *base = w.conv + (size_t)n * 2 * LN;  // [n][2][L][N], poly 0 = sum_r sigma_r(c0)
  if (ckks && c->log_n > 14) {
    if ((rc = ntt_inv_automorph_launch(c, ct, 1u, nullptr, w.dc, w.ext, n, w.ndig))) return rc;
  } else if ((rc = SP_DISPATCH(c, ks_prep_impl, c, ct + LN, 2 * L, w.dc, w.ext, n, w.ndig, nullptr))) {
    return rc;
  }
  if ((rc = ks_extend(c, w, n, ckks, ckks && c->log_n > 14))) return rc;
  for (u32 r0 = 0; r0 < n_rot; r0 += ROT_SUM_MAX) {
    RotSumArgs ra{}, rb{};
    ra.nr = rb.nr = std::min<u32>(ROT_SUM_MAX, n_rot - r0);
    for (u32 r = 0; r < ra.nr; ++r) {
      ra.ksk[r] = gks[r0 + r];
      ra.pt[r] = rb.pt[r] = pts ? pts[r0 + r] : nullptr;
      ra.g[r] = galois[r0 + r] & ((2u << c->log_n) - 1);
      rb.g[r] = ckks ? ra.g[r] : galois_inv(galois[r0 + r], c->log_n);
    }
    for (u32 c0 = 0; c0 < n; c0 += kMaxGridY) {
      const u32 nc = std::min<u32>(kMaxGridY, n - c0);
      if (c->special)
        hipLaunchKernelGGL((rot_sum_inner_kernel<true>), dim3(c->n / EW_BLOCK, QP, nc), dim3(EW_BLOCK), 0, c->stream,
                           w.ext + (size_t)c0 * w.ndig * QP * c->n, w.acc + (size_t)c0 * 2 * QP * c->n, ra, c->d_mods,
                           L, QP, w.ndig, ctx_key_qp(c), c->key_pshift, c->log_n, r0 > 0 ? 1u : 0u);
      else
        hipLaunchKernelGGL((rot_sum_inner_kernel<false>), dim3(c->n / EW_BLOCK, QP, nc), dim3(EW_BLOCK), 0, c->stream,
                           w.ext + (size_t)c0 * w.ndig * QP * c->n, w.acc + (size_t)c0 * 2 * QP * c->n, ra, c->d_mods,
                           L, QP, w.ndig, ctx_key_qp(c), c->key_pshift, c->log_n, r0 > 0 ? 1u : 0u);
      if ((rc = fhe_check(c, hipGetLastError(), "rot_sum_inner_kernel"))) return rc;
      if (c->special)
        hipLaunchKernelGGL((rot_sum_base_kernel<true>), dim3(c->n / EW_BLOCK, L, nc), dim3(EW_BLOCK), 0, c->stream,
                           ct + (size_t)c0 * 2 * LN, base + (size_t)c0 * 2 * LN, rb, c->d_mods, L, c->log_n,
                           ckks ? 0u : 1u, r0 > 0 ? 1u : 0u);
      else
        hipLaunchKernelGGL((rot_sum_base_kernel<false>), dim3(c->n / EW_BLOCK, L, nc), dim3(EW_BLOCK), 0, c->stream,
                           ct + (size_t)c0 * 2 * LN, base + (size_t)c0 * 2 * LN, rb, c->d_mods, L, c->log_n,
                           ckks ? 0u : 1u, r0 > 0 ? 1u : 0u);
      if ((rc = fhe_check(c, hipGetLastError(), "rot_sum_base_kernel"))) return rc;
    }
  }
  // ONE ModDown of the summed accumulator (keyswitch_run's finish without the
  // fused inner products): out = base + (acc_Q - Conv(acc_P)) P^-1
  u64 *acc = w.acc, *conv = w.conv;
  const size_t N = c->n;
  if (ckks && c->fuse_moddown) {
    if ((rc = ntt_launch(c, LimbMap{acc, QP, K, L, QP, 0, 0, 2 * n}, true, false, false, c->d_iscale))) return rc;
    return ntt_fwd_combine_launch(c, conv, 2 * n, acc, QP, base, out, 1u, &c->moddown);
  }
  if ((rc = ntt_launch(c, LimbMap{acc, QP, ckks ? K : QP, ckks ? L : 0, QP, 0, 0, 2 * n}, true,
                       ckks && c->fold_ninv)))
    return rc;
  if ((rc = conv_launch(c, c->moddown, acc + (size_t)L * N, QP, conv, L, 2 * n))) return rc;
  if (ckks) return ntt_fwd_combine_launch(c, conv, 2 * n, acc, QP, base, out, 1u);
  return SP_DISPATCH(c, combine_impl, c, acc, conv, base, out, n, 1u);
}

// ------------------------------------------------------------ CKKS rescale
size_t rescale_ws_bytes(const fhe_ctx *lo, u32 n) { return sizeof(u64) * lo->n * 2 * (size_t)n * (1 + lo->L); }

template <bool SP>
static int rescale_lift(fhe_ctx *lo, const u64 *x, u64 *conv, const u64 *qm_mod, u64 half, u32 n_polys) {
  const u32 m = lo->L, per = std::max<u32>(1, kMaxGridY / m);
  for (u32 p0 = 0; p0 < n_polys; p0 += per) {
    const u32 np = std::min(per, n_polys - p0);
    hipLaunchKernelGGL((rescale_lift_kernel<SP>), dim3(lo->n / EW_BLOCK, np * m), dim3(EW_BLOCK), 0, lo->stream,
                       x + (size_t)p0 * lo->n, conv + (size_t)p0 * m * lo->n, lo->d_mods, qm_mod, m, half,
                       lo->log_n);
    int rc = fhe_check(lo, hipGetLastError(), "rescale_lift_kernel");
    if (rc) return rc;
  }
  return FHE_OK;
}

// Rescale n ciphertexts of level m + 1 (context `up`) to level m (context
// `lo`): the dropped limb c_m of each of the 2n polys is copied out and
// inverse-transformed over q_m on `up`, lifted to the m remaining moduli,
// and ntt_fwd_combine_launch transforms the lift and forms
// out_i = (c_i - NTT(lift)_i) q_m^-1 in its last pass (acc = ct with stride
// m + 1 limbs, the epilogue constant d_qdrop = q_m^-1 R).
int rescale_impl(fhe_ctx *up, fhe_ctx *lo, const u64 *ct, u64 *out, u32 n) {
  const u32 m = lo->L;
  const size_t N = lo->n;
  void *ws;
  int rc = ctx_workspace(lo, rescale_ws_bytes(lo, n), &ws);
  if (rc) return rc;
  u64 *x = (u64 *)ws, *conv = x + (size_t)2 * n * N;
  if ((rc = fhe_check(lo, hipMemcpy2DAsync(x, N * 8, ct + (size_t)m * N, (size_t)(m + 1) * N * 8, N * 8, 2 * n,
                                           hipMemcpyDeviceToDevice, lo->stream), "rescale copy")))
    return rc;
  if ((rc = ntt_launch(up, LimbMap{x, 1, 1, 0, 1, 0, m, 2 * n}, true))) return rc;
  const u64 qm = up->moduli[m];
  if (lo->log_n >= 15) {
    // two-pass sizes: the lift runs as the 1-source conversion prologue of the
    // NTT's column pass (PRO_CONV with the central-lift step), so the lifted
    // limbs never make an HBM round trip
    const ConvSrc src{x, 1, 0, qm >> 1, lo->d_qdrop + m};
    return ntt_fwd_combine_launch(lo, conv, 2 * n, ct, m + 1, out, out, 0u, &lo->lift, nullptr, nullptr, 0, 0,
                                  lo->d_qdrop, &src);
  }
  if ((rc = SP_DISPATCH(lo, rescale_lift, lo, x, conv, lo->d_qdrop + m, qm >> 1, 2 * n))) return rc;
  return ntt_fwd_combine_launch(lo, conv, 2 * n, ct, m + 1, out, out, 0u, nullptr, nullptr, nullptr, 0, 0,
                                lo->d_qdrop);
}

// ------------------------------------------------------------ BEHZ setup
// MfmaConv constant operands for 8 sources -> targets tm (at most 12) with
// constants cst(i, t) (Montgomery pre-scaled, < tm[t]): lane l of the operand of
// block blk, k step m supplies row r = l & 31 -- target 4 blk + 2 ((r >> 2) & 1)
// + (r >> 4), result digit (r & 3) + 4 ((r >> 3) & 1) -- and k = 16 (l >> 5) + jj
// -- source 4 m + 2 (l >> 5) + (jj >> 3), digit a = jj & 7 -- (bconv_mfma.hip);
// the offsets make recombined sums non-negative (mfma_combine)
#if BEHZ_MFMA
template <class F>
static void mfma_conv_tables(MfmaConv &f, const std::vector<u64> &tm, F cst) {
  constexpr u64 K80 = 0x8080808080808080ull;
  typedef unsigned __int128 u128;
  const u32 nt = (u32)tm.size();
  for (int blk = 0; blk < 3; ++blk)
    for (int m = 0; m < 2; ++m)
      for (int l = 0; l < 64; ++l) {
        const int r = l & 31, hk = l >> 5;
        const int hr = (r >> 2) & 1, g = r >> 3, bd = (r & 3) + 4 * (g & 1), ml = 2 * hr + (g >> 1);
        const u32 t = 4 * blk + ml;
        uint8_t by[16];
        for (int jj = 0; jj < 16; ++jj) {
          const u32 i = 4 * m + 2 * hk + (jj >> 3), a = jj & 7;
          by[jj] = 0;
          if (t < nt) {
            u64 s256 = 1;
            for (u32 e = 0; e < a; ++e) s256 = host_mulmod(s256, 256, tm[t]);
            const u64 cv = host_mulmod(cst(i, t), s256, tm[t]);  // h R 256^a mod m_t
            by[jj] = (uint8_t)(((cv + K80) ^ K80) >> (8 * bd));
          }
        }
        v4i w;
        for (int q = 0; q < 4; ++q)
          w[q] = (int)((u32)by[4 * q] | (u32)by[4 * q + 1] << 8 | (u32)by[4 * q + 2] << 16 | (u32)by[4 * q + 3] << 24);
        f.af[blk][m][l] = w;
      }
  const u128 B32 = (u128)1 << 77;  // 2^45 2^32
  for (u32 t = 0; t < nt; ++t) {
    const u128 kp = ((B32 + ((u128)1 << 45)) / tm[t] + 1) * tm[t];
    f.off[t] = (u64)(kp - B32);
  }
}
#endif

int behz_setup(fhe_ctx *c) {
  const u32 L = c->L, nB = c->nB, bsk0 = c->L + c->K;
  if (L > BEHZ_MAXL) return fhe_fail(c, FHE_ERR_UNSUPPORTED, "BFV with L > 24");
  BehzDev *B = new BehzDev();
  std::memset(B, 0, sizeof(BehzDev));
  B->L = L; B->nB = nB; B->bsk0 = bsk0;
  const u64 *qq = c->moduli.data(), *bsk = c->moduli.data() + bsk0;
  const u64 msk = bsk[nB - 1];
  const u64 mt = 1ull << 32;
  std::vector<std::vector<u64>> h_q_bsk(L, std::vector<u64>(nB));  // (Q/q_i) mod b_j
  std::vector<u64> cj(nB);                                          // the floor's c_j
  auto M = host_mulmod;
  auto R = host_to_mont;
  for (u32 i = 0; i < L; ++i) {
    u64 qh = 1, hm = 1;
    for (u32 k = 0; k < L; ++k)
      if (k != i) { qh = M(qh, qq[k] % qq[i], qq[i]); hm = (hm * (qq[k] & 0xffffffffull)) & 0xffffffffull; }
    const u64 hinv = host_inv(qh, qq[i]);
    B->mt_hinv_R[i] = R(M(hinv, mt % qq[i], qq[i]), qq[i]);
    // the floor's inputs come from an inverse NTT without its N^-1 (bfv_mul_relin_impl): fold it here
    B->t_hinv_R[i] = R(M(M(hinv, c->t % qq[i], qq[i]), host_inv(c->n % qq[i], qq[i]), qq[i]), qq[i]);
    B->h_mod_mt[i] = (u32)hm;
    for (u32 j = 0; j < nB; ++j) h_q_bsk[i][j] = 1;
    for (u32 j = 0; j < nB; ++j)
      for (u32 k = 0; k < L; ++k) if (k != i) h_q_bsk[i][j] = M(h_q_bsk[i][j], qq[k] % bsk[j], bsk[j]);
    u64 bm = 1;
    for (u32 k = 0; k + 1 < nB; ++k) bm = M(bm, bsk[k] % qq[i], qq[i]);
    B->b_mod_q_R[i] = R(bm, qq[i]);
  }
  u64 qm = 1;
  for (u32 k = 0; k < L; ++k) qm = (qm * (qq[k] & 0xffffffffull)) & 0xffffffffull;
  u32 inv = (u32)qm;
  for (int it = 0; it < 5; ++it) inv *= 2u - (u32)qm * inv;
  B->neg_inv_q_mod_mt = 0u - inv;
  u64 bmsk = 1;
  for (u32 k = 0; k + 1 < nB; ++k) bmsk = M(bmsk, bsk[k] % msk, msk);
  const u64 inv_b_msk = host_inv(bmsk, msk);
  for (u32 j = 0; j + 1 < nB; ++j) {
    u64 bh = 1, bhm = 1;
    for (u32 k = 0; k + 1 < nB; ++k)
      if (k != j) { bh = M(bh, bsk[k] % bsk[j], bsk[j]); bhm = M(bhm, bsk[k] % msk, msk); }
    cj[j] = host_inv(bh, bsk[j]);
    B->hbm_R[j] = R(M(bhm, inv_b_msk, msk), msk);
    for (u32 i = 0; i < L; ++i) {
      u64 p2 = 1;
      for (u32 k = 0; k + 1 < nB; ++k) if (k != j) p2 = M(p2, bsk[k] % qq[i], qq[i]);
      B->h_b_q_R[j][i] = R(p2, qq[i]);
    }
  }
  cj[nB - 1] = inv_b_msk;
  for (u32 j = 0; j < nB; ++j) {
    const u64 b = bsk[j];
    u64 qmb = 1;
    for (u32 k = 0; k < L; ++k) qmb = M(qmb, qq[k] % b, b);
    const u64 inv_mt = host_inv(mt % b, b), qf = M(host_inv(qmb, b), cj[j], b);  // Q^-1 c_j
    B->qx_R[j] = R(M(qmb, inv_mt, b), b);
    B->tf_R[j] = R(M(M(c->t % b, host_inv(c->n % b, b), b), qf, b), b);
    for (u32 i = 0; i < L; ++i) {
      B->hx_R[i][j] = R(M(h_q_bsk[i][j], inv_mt, b), b);
      B->hf_R[i][j] = R((b - M(h_q_bsk[i][j], qf, b)) % b, b);
    }
  }
#if BEHZ_MFMA
  if (L == 8 && c->special) {
    // the MFMA contractions' constant operands (behz_*_mfma_kernel)
    std::vector<u64> bq(qq, qq + L), bb(bsk, bsk + nB);
    mfma_conv_tables(B->mx, bb, [&](u32 i, u32 j) { return B->hx_R[i][j]; });
    mfma_conv_tables(B->mf, bb, [&](u32 i, u32 j) { return B->hf_R[i][j]; });
    mfma_conv_tables(B->mq, bq, [&](u32 j, u32 i) { return B->h_b_q_R[j][i]; });
  }
#endif
  c->behz = ctx_upload(c, B, sizeof(BehzDev));
  delete B;
  return c->behz ? FHE_OK : FHE_ERR_OOM;
}

// HPS constants (oracle hps_init; the doubles by the same two C operations)
int hps_setup(fhe_ctx *c) {
  const u32 L = c->L, nB = c->nB, bsk0 = c->L + c->K;
  if (L > BEHZ_MAXL) return fhe_fail(c, FHE_ERR_UNSUPPORTED, "BFV with L > 24");
  HpsDev *H = new HpsDev();
  std::memset(H, 0, sizeof(HpsDev));
  H->L = L; H->nB = nB; H->bsk0 = bsk0;
  const u64 *qq = c->moduli.data(), *pp = c->moduli.data() + bsk0;
  auto M = host_mulmod;
  auto R = host_to_mont;
  for (u32 i = 0; i < L; ++i) {
    const u64 q = qq[i];
    u64 h = 1;
    for (u32 k = 0; k < L; ++k) if (k != i) h = M(h, qq[k] % q, q);
    const u64 qt = host_inv(h, q), num = M(c->t % q, qt, q);
    H->qt_R[i] = R(qt, q);
    H->invq[i] = 1.0 / (double)q;
    H->frac[i] = (double)num / (double)q;
    H->ninv_R[i] = R(host_inv(c->n % q, q), q);
    u64 Pm = 1;
    for (u32 k = 0; k < nB; ++k) Pm = M(Pm, pp[k] % q, q);
    H->P_R[i] = R(Pm, q);
    for (u32 j = 0; j < nB; ++j) {
      const u64 pj = pp[j];
      u64 qs = 1, ps = 1;
      for (u32 k = 0; k < L; ++k) if (k != i) qs = M(qs, qq[k] % pj, pj);
      H->qstar_R[i][j] = R(qs, pj);
      H->I_R[i][j] = R(M((pj - num % pj) % pj, host_inv(q % pj, pj), pj), pj);
      for (u32 k = 0; k < nB; ++k) if (k != j) ps = M(ps, pp[k] % q, q);
      H->pstar_R[j][i] = R(ps, q);
    }
  }
  for (u32 j = 0; j < nB; ++j) {
    const u64 pj = pp[j];
    u64 Qm = 1, h = 1;
    for (u32 k = 0; k < L; ++k) Qm = M(Qm, qq[k] % pj, pj);
    H->Q_R[j] = R(Qm, pj);
    H->lam_R[j] = R(M(M(c->t % pj, host_inv(Qm, pj), pj), host_inv(c->n % pj, pj), pj), pj);
    for (u32 k = 0; k < nB; ++k) if (k != j) h = M(h, pp[k] % pj, pj);
    H->pt_R[j] = R(host_inv(h, pj), pj);
    H->invp[j] = 1.0 / (double)pj;
  }
  c->hps = ctx_upload(c, H, sizeof(HpsDev));
  delete H;
  return c->hps ? FHE_OK : FHE_ERR_OOM;
}


size_t bfv_mul_ws_bytes(const fhe_ctx *c, u32 n) {
  const size_t N = c->n, L = c->L, nB = c->nB;
  return sizeof(u64) * N * n * (4 * L + 4 * nB + 3 * L + 3 * nB) + keyswitch_ws_bytes(c, n);
}

int bfv_mul_relin_impl(fhe_ctx *c, const u64 *a, const u64 *b, const u64 *rlk, u64 *out, u32 n) {
  const u32 L = c->L, nB = c->nB, N = c->n, bsk0 = c->L + c->K;
  void *wsv;
  int rc = ctx_workspace(c, bfv_mul_ws_bytes(c, n), &wsv);
  if (rc) return rc;
  u64 *xq = (u64 *)wsv;                       // [2][n][2][L][N]: NTT(a), NTT(b)
  u64 *xb = xq + (size_t)n * 4 * L * N;       // [2][n][2][nB][N]: the Bsk extensions
  u64 *eq = xb + (size_t)n * 4 * nB * N;      // [n][3][L][N]
  u64 *eb = eq + (size_t)n * 3 * L * N;       // [n][3][nB][N]
  const KsWs w = ks_layout(c, n, eb + (size_t)n * 3 * nB * N);
  // 1-2. extend a0,a1,b0,b1 to Bsk (coefficient form): BEHZ (m~ + sm_mrq) or
  //      HPS (the exact centred lift, fhe_params.flags FHE_FLAG_BFV_HPS)
  if ((rc = c->hps ? SP_DISPATCH(c, hps_extend_impl, c, a, b, xb, n) : SP_DISPATCH(c, behz_extend_impl, c, a, b, xb, n)))
    return rc;
  // 3-4 fused (BFVT): the forward column passes here (the Q part out of place,
  //    straight from the ciphertexts); the forward row passes, the tensor and
  //    the inverse row passes in one kernel per base, then the inverse column passes
  if (bfvt_fused_ok(c)) {
    if ((rc = ntt_fwd_col_launch(c, LimbMap{xq, L, L, 0, L, 0, 0, 2 * n}, a))) return rc;
    if ((rc = ntt_fwd_col_launch(c, LimbMap{xq + (size_t)n * 2 * L * N, L, L, 0, L, 0, 0, 2 * n}, b))) return rc;
    if ((rc = ntt_fwd_col_launch(c, LimbMap{xb, nB, nB, 0, nB, 0, bsk0, 4 * n}))) return rc;
    if ((rc = ntt_bfv_tensor_fused_launch(c, xq, xq + (size_t)n * 2 * L * N, eq, L, 0, n))) return rc;
    if ((rc = ntt_bfv_tensor_fused_launch(c, xb, xb + (size_t)n * 2 * nB * N, eb, nB, bsk0, n))) return rc;
  } else {
  // 3. NTT in Q and Bsk
  //    (the Q part out of place, straight from the ciphertexts)
  if ((rc = ntt_launch(c, LimbMap{xq, L, L, 0, L, 0, 0, 2 * n}, false, false, false, nullptr, a))) return rc;
  if ((rc = ntt_launch(c, LimbMap{xq + (size_t)n * 2 * L * N, L, L, 0, L, 0, 0, 2 * n}, false, false, false, nullptr,
                       b)))
    return rc;
  if ((rc = ntt_launch(c, LimbMap{xb, nB, nB, 0, nB, 0, bsk0, 4 * n}, false))) return rc;
  // 4. tensor in both bases, fused into the first pass of its inverse NTT
  //    (unscaled: behz_floor's t constants carry N^-1)
  if ((rc = ntt_inv_bfv_tensor_launch(c, xq, xq + (size_t)n * 2 * L * N, eq, L, 0, n))) return rc;
  if ((rc = ntt_inv_bfv_tensor_launch(c, xb, xb + (size_t)n * 2 * nB * N, eb, nB, bsk0, n))) return rc;
  }
  // 5. scale and round: r0, r1 -> out; r2 -> the key-switch scratch, prepared
  //    (BEHZ floor, or HPS simple scaling + exact P -> Q)
  const u64 *dsc = bfv_fused(c) ? c->d_bfv_dscale : nullptr;
  if ((rc = c->hps ? SP_DISPATCH(c, hps_scale_impl, c, eq, eb, out, w.dc, w.ext, n, w.ndig, dsc)
                   : SP_DISPATCH(c, behz_floor_impl, c, eq, eb, out, w.dc, w.ext, n, w.ndig, dsc)))
    return rc;
  // 6. relinearize r2 and add to (r0, r1)
  if (dsc) return bfv_ks_fused(c, w, rlk, out, out, n, 3u);
  return keyswitch_run(c, w, rlk, out, out, n, 3u, false);
}
