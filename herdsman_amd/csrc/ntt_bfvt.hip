// ntt_bfvt.hip -- BFV's tensor product between its forward and inverse NTTs,
// with both row passes fused around it (BFVT fused)
// (kernel templates: ntt_core.hpp; the row transforms as in ntt_ksf.hip)
//
// BFV mul+relin (bfv_mul_relin_impl) transforms a0, a1, b0, b1 to NTT form in
// Q and in Bsk, forms d0 = a0 b0, d1 = a0 b1 + a1 b0, d2 = a1 b1 and
// transforms the three back.  Unfused, the forward row pass stores the four
// NTTs and the tensor's inverse row pass (PRO_BFVT) reads them back: eight
// limb-polys of HBM traffic per (ciphertext, limb) between two transforms that
// could share registers.  Here ONE workgroup per (limb, ciphertext, 16-row
// block) runs the forward row transform of each of the four column-pass
// intermediates in registers, forms the products element-wise in the IO
// layout, and runs the inverse row transform of each product, storing the
// three inverse row-pass outputs the inverse column pass reads.  Per
// (ciphertext, limb) it reads 4 and writes 3 limb-polys instead of 4 + 4 + 4 +
// 3 (the forward row pass's read and write, the tensor pass's read and write).
// Bit-exact with the unfused path: the products are the canonical residues
// the PRO_BFVT prologue forms (mul_mod, reduce128), the inverse transform runs
// the same butterflies on them.
// Order (the four operands never live at once): A0, B0 -> d0 out; B1 -> P =
// A0 B1 (A0 dies); A1 -> d1 = P + A1 B0, d2 = A1 B1.  Peak: B0, B1, P and A1
// under its transform, 3 waves per SIMD as the key-switch finish.
#include "ntt_core.hpp"

#ifndef BFVT_FUSE
#define BFVT_FUSE 1  // BFV mul: the fused row passes around the tensor product (bfvt_fused_ok)
#endif
#ifndef BFVT_LSW
#define BFVT_LSW 2  // butterflies per lock-step chunk (run_group LSW)
#endif
#ifndef BFVT_MINW
#define BFVT_MINW 2  // minimum waves per SIMD (3: ~48 VGPRs spill, C3 -2.2%, profiles/r06/ab_bfvt.txt)
#endif
#ifndef BFVT_PF
#define BFVT_PF 0  // 1: each operand's loads issued during the previous operand's transform
#endif
#ifndef BFVT_STASH
#define BFVT_STASH 0  // 1: a0 b1 parked in d1's output rows (L2) while a1 is transformed, instead of in registers
#endif

namespace {

struct BfvtArgs {
  const u64 *xa, *xb;   // [n][2][nl][N] the forward column-pass outputs of (a0, a1) and (b0, b1)
  u64 *e;               // [n][3][nl][N] the inverse row-pass outputs of d0, d1, d2
  const ModInfo *mods;  // indexed l0 + limb
  const u64 *twf, *twi; // forward / inverse twiddles [nmod][N]
  u32 nl, l0;
};

template <int LOG_N, bool WIDE, bool SP>
__global__ void __launch_bounds__(256, BFVT_MINW) bfvt_fused_pass(BfvtArgs a) {
  constexpr int S = 8, LOGR = 4, W = 16, R = 16, S0 = LOG_N - S;
  using G0 = Grp<S, LOGR, 0>;
  using G1 = Grp<S, LOGR, 1>;
  using IO = IoL<S, LOGR>;
  extern __shared__ u64 lds[];
  constexpr size_t N = (size_t)1 << LOG_N;
  // dispatch order: row blocks, then ciphertexts, then limbs -- the resident
  // workgroups share one modulus, so its twiddle rows stay in L2
  const u32 tid = threadIdx.x, bx = blockIdx.x, ct = blockIdx.y, pl = blockIdx.z;
  const u32 mod = a.l0 + pl;
  const ModInfo mi = a.mods[mod];
  const u64 q = mi.q, q2 = 2 * q;
  const u64 *twf = a.twf + ((size_t)mod << LOG_N), *twi = a.twi + ((size_t)mod << LOG_N);
  const u32 ts = tid % (1u << (S - LOGR)), w = tid / (1u << (S - LOGR));
  const u32 row = bx * W + w, gb = row << S;
  const u32 vg0 = (gb + G0::k_thr(ts)) << 3;  // the group-0 layout (forward loads, inverse stores)
  const size_t LN = (size_t)a.nl * N;
  const size_t io = ((size_t)2 * ct * a.nl + pl) * N;
  const u64 *pa0 = a.xa + io, *pa1 = pa0 + LN, *pb0 = a.xb + io, *pb1 = pb0 + LN;
  u64 *pe = a.e + ((size_t)3 * ct * a.nl + pl) * N;
  u64 nq1 = 0 - q, nq2 = 0 - q2, nq4 = 0 - 2 * q2;
  asm("" : "+s"(nq1));
  asm("" : "+s"(nq2));
  asm("" : "+s"(nq4));
  const u64 r2 = mi.r2;

  // the forward row pass of one 16-row block in registers (the column pass's
  // output in the group-0 layout in, canonical NTT outputs in the IO layout
  // out).  Each sub-transform's 16 threads sit in one wave, so consecutive
  // transforms reuse its LDS slots without a barrier in between.
  const auto load = [&](const u64 *src, u64 (&x)[R]) {
#pragma unroll
    for (int r = 0; r < R; ++r) x[r] = ld_d(src + G0::k_reg(r), vg0);
  };
  // BFVT_PF: x is already loaded; the next operand's loads (nsrc -> nx) are
  // issued behind this transform's first twiddle loads, so the transform's
  // first wait does not include them
  const auto fwd_pf = [&](u64 (&x)[R], const u64 *nsrc, u64 (&nx)[R]) {
    __builtin_amdgcn_sched_barrier(0);
    u64 t[16];
    G0::template load_tw<S0>(t, twf, row, ts);
    if (nsrc) load(nsrc, nx);
    run_group<S, LOGR, 0, S0, false, SP, WIDE, BFVT_LSW>(x, t, q2, mi);
    G1::template load_tw<S0>(t, twf, row, ts);
    const u32 l0 = lds_idx<S>(w, G0::k_thr(ts));
#pragma unroll
    for (int r = 0; r < R; ++r) lds[l0 + G0::k_reg(r) + lds_pad(G0::k_reg(r))] = x[r];
    __syncthreads();
    const u32 l1 = lds_idx<S>(w, G1::k_thr(ts));
#pragma unroll
    for (int r = 0; r < R; ++r) x[r] = lds[l1 + G1::k_reg(r) + lds_pad(G1::k_reg(r))];
    run_group<S, LOGR, 1, S0, false, SP, WIDE, BFVT_LSW>(x, t, q2, mi);
#pragma unroll
    for (int r = 0; r < R; ++r) lds[l1 + G1::k_reg(r) + lds_pad(G1::k_reg(r))] = x[r];
    __syncthreads();
    const u32 l2 = lds_idx<S>(w, IO::k_thr(ts));
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const u64 v = lds[l2 + IO::k_reg(r) + lds_pad(IO::k_reg(r))];  // lazy: < 8q WIDE, < 4q
      x[r] = harvey_csub(harvey_csub(WIDE ? harvey_csub(v, nq4) : v, nq2), nq1);
    }
    __builtin_amdgcn_sched_barrier(0);
  };
  const auto fwd = [&](const u64 *src, u64 (&x)[R]) {
    __builtin_amdgcn_sched_barrier(0);
    load(src, x);
    fwd_pf(x, nullptr, x);
  };
  // the first (row) pass of the inverse NTT of canonical x in the IO layout:
  // group 1, group 0, stored in the group-0 layout (PRO_BFVT's row pass; no
  // scaling, the inverse column pass follows)
  const auto inv = [&](u64 (&x)[R], u64 *dst) {
    __builtin_amdgcn_sched_barrier(0);
    u64 t[16];
    G1::template load_tw<S0>(t, twi, row, ts);
    const u32 l2 = lds_idx<S>(w, IO::k_thr(ts));
#pragma unroll
    for (int r = 0; r < R; ++r) lds[l2 + IO::k_reg(r) + lds_pad(IO::k_reg(r))] = x[r];
    __syncthreads();
    const u32 l1 = lds_idx<S>(w, G1::k_thr(ts));
#pragma unroll
    for (int r = 0; r < R; ++r) x[r] = lds[l1 + G1::k_reg(r) + lds_pad(G1::k_reg(r))];
    run_group<S, LOGR, 1, S0, true, SP, false, BFVT_LSW>(x, t, q2, mi);
    G0::template load_tw<S0>(t, twi, row, ts);
#pragma unroll
    for (int r = 0; r < R; ++r) lds[l1 + G1::k_reg(r) + lds_pad(G1::k_reg(r))] = x[r];
    __syncthreads();
    const u32 l0 = lds_idx<S>(w, G0::k_thr(ts));
#pragma unroll
    for (int r = 0; r < R; ++r) x[r] = lds[l0 + G0::k_reg(r) + lds_pad(G0::k_reg(r))];
    run_group<S, LOGR, 0, S0, true, SP, false, BFVT_LSW>(x, t, q2, mi);
#pragma unroll
    for (int r = 0; r < R; ++r) st_d(dst + G0::k_reg(r), vg0, x[r]);
  };
  // canonical x y mod q: (x y R^-1) R
  const auto prod = [&](u64 x, u64 y) { return harvey_csub(mont_mul<SP>(mont_mul<SP>(x, y, mi), r2, mi), nq1); };

  u64 A0[R], B0[R], B1[R], P[R], A1[R];
  if constexpr (BFVT_PF) {
    load(pa0, A0);
    fwd_pf(A0, pb0, B0);
    fwd_pf(B0, pb1, B1);
  } else {
    fwd(pa0, A0);
    fwd(pb0, B0);
  }
  {
    u64 d0[R];
#pragma unroll
    for (int r = 0; r < R; ++r) d0[r] = prod(A0[r], B0[r]);
    inv(d0, pe);
  }
  if constexpr (BFVT_PF) fwd_pf(B1, pa1, A1);
  else fwd(pb1, B1);
#pragma unroll
  for (int r = 0; r < R; ++r) P[r] = mont_mul<SP>(A0[r], B1[r], mi);  // a0 b1 R^-1, < 2q
  const u32 vio = (gb + IO::k_thr(ts)) << 3;
  if constexpr (BFVT_STASH) {
    // parked in this thread's own IO-layout words of d1's output rows: read
    // back by the same thread before the inverse transform's barriers, so no
    // other thread's store of d1 can overtake it
#pragma unroll
    for (int r = 0; r < R; r += 2) *(u64x2 *)((char *)(pe + LN + IO::k_reg(r)) + vio) = u64x2{P[r], P[r + 1]};
    asm volatile("" ::: "memory");
  }
  if constexpr (BFVT_PF) fwd_pf(A1, nullptr, A1);
  else fwd(pa1, A1);
  if constexpr (BFVT_STASH) {
    asm volatile("" ::: "memory");
#pragma unroll
    for (int r = 0; r < R; r += 2) {
      const u64x2 v = ld2_b(pe + LN + IO::k_reg(r), vio);
      P[r] = v.x, P[r + 1] = v.y;
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const u64 s = harvey_csub(P[r] + mont_mul<SP>(A1[r], B0[r], mi), nq2);  // (a0 b1 + a1 b0) R^-1, < 2q
    P[r] = harvey_csub(mont_mul<SP>(s, r2, mi), nq1);
    A1[r] = prod(A1[r], B1[r]);
  }
  inv(P, pe + LN);
  inv(A1, pe + 2 * LN);
}

template <int LOG_N, bool WIDE>
int bfvt_launch(fhe_ctx *c, const BfvtArgs &a, u32 n) {
  constexpr size_t lds = lds_bytes<8, 16>();
  const dim3 grid((1u << (LOG_N - 8)) / 16, n, a.nl);
  if (c->special) hipLaunchKernelGGL((bfvt_fused_pass<LOG_N, WIDE, true>), grid, dim3(256), lds, c->stream, a);
  else hipLaunchKernelGGL((bfvt_fused_pass<LOG_N, WIDE, false>), grid, dim3(256), lds, c->stream, a);
  return fhe_check(c, hipGetLastError(), "bfvt_fused_pass launch");
}

// the limbs [l0, l0 + nl) in one lazy-schedule class (the forward row
// transform's WIDE schedule is per launch)
bool bfvt_one_class(const fhe_ctx *c, u32 l0, u32 nl) {
  const bool wide = c->moduli[l0] < (1ull << 60);
  for (u32 i = l0 + 1; i < l0 + nl; ++i)
    if ((c->moduli[i] < (1ull << 60)) != wide) return false;
  return true;
}

}  // namespace

// The fused row passes apply: N = 2^15 or 2^16 (a 256-point row pass), each
// base (Q, Bsk) in one lazy-schedule class.
bool bfvt_fused_ok(const fhe_ctx *c) {
  return BFVT_FUSE && (c->log_n == 15 || c->log_n == 16) && c->nB && bfvt_one_class(c, 0, c->L) &&
         bfvt_one_class(c, c->L + c->K, c->nB);
}

// BFV mul+relin: xa = (a0, a1), xb = (b0, b1), each [n][2][nl][N] after the
// forward COLUMN pass in the nl-limb base starting at modulus mod_offset; e
// [n][3][nl][N] receives the coefficient-form tensor products WITHOUT the N^-1
// factor (behz_floor's / hps_scale's constants carry it), as
// ntt_inv_bfv_tensor_launch leaves them after the full forward NTT.
int ntt_bfv_tensor_fused_launch(fhe_ctx *c, const u64 *xa, const u64 *xb, u64 *e, u32 nl, u32 mod_offset, u32 n) {
  if (!bfvt_fused_ok(c)) return fhe_fail(c, FHE_ERR_UNSUPPORTED, "fused BFV tensor: shape");
  const size_t N = c->n;
  const bool wide = c->moduli[mod_offset] < (1ull << 60);
  const u32 per = 21845u;  // ciphertexts per launch: the inverse column pass takes 3 polys per ct on gridDim.y
  for (u32 c0 = 0; c0 < n; c0 += per) {
    const u32 nc = std::min(per, n - c0);
    BfvtArgs b{};
    b.xa = xa + (size_t)c0 * 2 * nl * N;
    b.xb = xb + (size_t)c0 * 2 * nl * N;
    b.e = e + (size_t)c0 * 3 * nl * N;
    b.mods = c->d_mods;
    b.twf = c->d_tw_fwd;
    b.twi = c->d_tw_inv;
    b.nl = nl;
    b.l0 = mod_offset;
    int rc = c->log_n == 15 ? (wide ? bfvt_launch<15, true>(c, b, nc) : bfvt_launch<15, false>(c, b, nc))
                            : (wide ? bfvt_launch<16, true>(c, b, nc) : bfvt_launch<16, false>(c, b, nc));
    if (rc) return rc;
    NttArgs t{};
    t.map = LimbMap{b.e, nl, nl, 0, nl, 0, mod_offset, 3 * nc};
    t.tw = c->d_tw_inv;
    t.mods = c->d_mods;
    t.ninv = c->d_ninv;
    t.log_n = c->log_n;
    t.noscale = 1;
    if ((rc = ntt_col_plain(c, t, true, 3 * nc * nl))) return rc;
  }
  return FHE_OK;
}
