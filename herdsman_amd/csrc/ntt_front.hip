// ntt_front.hip -- inverse-NTT front ends: CKKS tensor (PRO_TENSOR), rotation (PRO_AUTOMORPH), BFV tensor (PRO_BFVT)
// (kernel templates: ntt_core.hpp; one translation unit per entry-point family so
// the ~360 pass kernels compile in parallel)
#include "ntt_core.hpp"

// CKKS mul+relin front end: the tensor product fused into the first pass of
// the inverse NTT of d2 (PRO_TENSOR).  a, b, out: [n][2][L][N] (out may alias
// a or b); dc [n][L][N] receives INTT(d2); ext's own-digit slots receive d2 R.
// d2_only: out and ext are left alone (PRO_TENSOR2: only a1 and b1 are read;
// EPI_KSQT forms d0, d1 and the own digit's ext word d2 R).
int ntt_inv_tensor_launch(fhe_ctx *c, const u64 *a, const u64 *b, u64 *out, u64 *dc, u64 *ext, u32 n, u32 ndig,
                          bool d2_only, bool rows_only) {
  const u32 L = c->L, QP = c->L + c->K;
  const size_t N = c->n;
  if (d2_only && c->log_n <= 14) return fhe_fail(c, FHE_ERR_UNSUPPORTED, "split tensor product: log_n");
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
    // PRO_TENSOR2 forms d2 R^-1 (one Montgomery product): its scale carries R
    // (d_iscale_t; without the fused ModUp, R in place of the skipped N^-1)
    if (d2_only && !c->fold_ninv) return fhe_fail(c, FHE_ERR_UNSUPPORTED, "split tensor product: scaling");
    if (c->fuse_modup) t.scale = d2_only ? c->d_iscale_t : c->d_iscale;
    else if (d2_only) t.scale = c->d_r2;
    else t.noscale = c->fold_ninv;
    const u32 n_jobs = np * L;
    int rc;
    if (c->log_n <= 14) {
      rc = single_pass<PRO_TENSOR>(c, t, true, n_jobs);
    } else {
      if ((rc = d2_only ? row_pass<PRO_TENSOR2>(c, t, true, n_jobs) : row_pass<PRO_TENSOR>(c, t, true, n_jobs)))
        return rc;
      // rows_only: the column pass runs inside ModUp's CONVF launches (ntt_convf.hip)
      rc = rows_only ? FHE_OK : ntt_col_plain(c, t, true, n_jobs);
    }
    if (rc) return rc;
  }
  return FHE_OK;
}

// CKKS rotation front end: the NTT-domain automorphism sigma_g (and the KS
// preparation of sigma_g(c1)) fused into the first pass of its inverse NTT
// (PRO_AUTOMORPH).  ct [n][2][L][N] must not alias base; base[ct][0] receives
// sigma_g(c0), dc INTT(sigma_g(c1)), ext's own-digit slots sigma_g(c1) R (ext
// null: not stored, the fused key-switch finish forms them).
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
    t.t_ext = ext ? ext + (size_t)p0 * ndig * QP * N : nullptr;
    t.t_L = L;
    t.t_QP = QP;
    t.t_alpha = c->alpha;
    t.t_ndig = ndig;
    t.t_g = g & ((2u << c->log_n) - 1);
    if (c->fuse_modup) t.scale = c->d_iscale;  // dc feeds ModUp only (as in ntt_inv_tensor_launch)
    else t.noscale = c->fold_ninv;
    int rc;
    if ((rc = row_pass<PRO_AUTOMORPH>(c, t, true, np * L))) return rc;
    if ((rc = ntt_col_plain(c, t, true, np * L))) return rc;
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
      rc = ntt_col_plain(c, t, true, n_jobs);
    }
    if (rc) return rc;
  }
  return FHE_OK;
}

