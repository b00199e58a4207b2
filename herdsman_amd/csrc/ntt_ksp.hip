// ntt_ksp.hip -- ModUp fused into the NTT of its outputs, INTT(acc_P) with the P-limb inner product (PRO_KSP)
// (kernel templates: ntt_core.hpp; one translation unit per entry-point family so
// the ~360 pass kernels compile in parallel)
#include "ntt_core.hpp"

// ModUp of digit j fused into the forward NTT of its converted limbs: the
// column pass computes each target limb's conversion y_m = sum_i v_i h[i][m]
// from the digit's source limbs v_i of dc (canonical, already scaled by the
// INTT through d_iscale) as its prologue (PRO_CONV), so the converted limbs
// never make an HBM round trip; the row pass leaves lazy outputs (< 8q) for
// the inner product on special moduli, as keyswitch_run's separate NTT does.
// src_rows_scale (CONVF, the fused key switch): dc holds INTT(d2)'s ROW-pass
// output; its column pass (output scale src_rows_scale) runs in the same
// kernel as the conversion and the targets' column passes (ntt_convf.hip).
int ntt_fwd_modup_launch(fhe_ctx *c, const u64 *dc, u64 *ext, u32 n, u32 ndig, u32 j, bool q_rows, bool ksf_scale,
                         const u64 *src_rows_scale) {
  const u32 L = c->L, QP = c->L + c->K, N = c->n;
  const u32 lo = j * c->alpha, hi = std::min(lo + c->alpha, L);
  // q_rows false (the fused key switch): Q targets at its accumulator scale
  const bool ksf = !q_rows && ksf_scale;
  if (ksf && c->modup_tabs_ksf.size() <= j) return fhe_fail(c, FHE_ERR_UNSUPPORTED, "fused ModUp: ksf tables");
  const ConvTab &tab = ksf ? c->modup_tabs_ksf[j] : c->modup_tabs[j];
  if (c->log_n <= 14 || tab.ns > 4) return fhe_fail(c, FHE_ERR_UNSUPPORTED, "fused ModUp: log_n / digit size");
  if (src_rows_scale && (q_rows || !convf_ok(c, tab.ns)))
    return fhe_fail(c, FHE_ERR_UNSUPPORTED, "fused ModUp from row-pass sources: shape");
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
    a.c_src60 = 1;
    for (u32 i = lo; i < hi; ++i) a.c_src60 &= c->moduli[i] < (1ull << 60);
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
    if (!q_rows && src_rows_scale) {
      ConvfArgs f{};
      f.src = a.c_src;
      f.src_stride = L;
      f.src_first = lo;
      f.src_mod0 = lo;
      f.scale = src_rows_scale;
      f.tmap = a.map;
      f.h = tab.h;
      f.nd = tab.nd;
      f.src60 = a.c_src60;
      f.mods = c->d_mods;
      f.twi = c->d_tw_inv;
      f.twf = c->d_tw_fwd;
      rc = ntt_convf_launch(c, f, tab.ns);
    } else if (!q_rows) {
      // the fused key switch transforms every target's rows itself (ntt_ksf.hip)
      rc = ntt_conv_col(c, a, n_jobs);
    } else if (wq != 2 && wp != 2 && wq != wp && aq.map.cnt && ap.map.cnt) {
#if MODUP_COL_SPLIT
      if ((rc = ntt_conv_col(c, aq, np * aq.map.cnt))) return rc;
      if ((rc = ntt_conv_col(c, ap, np * ap.map.cnt))) return rc;
#else
      if ((rc = ntt_conv_col(c, a, n_jobs))) return rc;
#endif
      if ((rc = ntt_row_plain(c, aq, false, np * aq.map.cnt))) return rc;
      rc = ntt_row_plain(c, ap, false, np * ap.map.cnt);
    } else {
      if ((rc = ntt_conv_col(c, a, n_jobs))) return rc;
      rc = ntt_row_plain(c, a, false, n_jobs);
    }
    if (rc) return rc;
  }
  return FHE_OK;
}

// INTT of the P limbs of the key-switching accumulator acc [2n][QP][N], with
// their inner product acc_P[2 ct + b][k] = sum_j ext[ct][j][k] ksk[j][b][k] R^-1
// (ks_inner_kernel) formed in the first (row) pass (PRO_KSP): acc_P is never
// stored, the P rows of acc receive INTT(acc_P) times d_iscale (ModDown's
// source constants, as ntt_launch(..., d_iscale) gives them)
int ntt_inv_ksp_launch(fhe_ctx *c, u64 *acc, const u64 *ext, const u64 *ksk, u32 n, u32 ndig, u32 ext_g,
                       bool all_limbs, const RotBatch *rb) {
  const u32 L = c->L, K = c->K, QP = L + K;
  const size_t N = c->n;
  if (c->log_n <= 14 || ndig < 1 || ndig > 4)
    return fhe_fail(c, FHE_ERR_UNSUPPORTED, "fused P-limb inner product: log_n / digits");
  if (all_limbs && (!c->d_bfv_kscale || c->key_pshift))
    return fhe_fail(c, FHE_ERR_UNSUPPORTED, "fused all-limb inner product: BFV tables");
  const u32 l0 = all_limbs ? 0 : L, nl = all_limbs ? QP : K;
  // rb: acc holds rb->nr rotations' accumulators of the n ciphertexts, one chunk
  const u32 nr = rb ? rb->nr : 1;
  if (rb && (nr < 1 || nr > FHE_ROT_BATCH || 2 * n * nr > 65534u))
    return fhe_fail(c, FHE_ERR_INVALID, "rotation batch: count / size");
  const u32 per = 65534u;  // gridDim.y, even (the polys of a ciphertext stay together)
  for (u32 p0 = 0; p0 < 2 * n * nr; p0 += per) {
    const u32 np = std::min(per, 2 * n * nr - p0);
    NttArgs a{};
    a.map = LimbMap{acc + (size_t)p0 * QP * N, QP, nl, l0, QP, 0, 0, np};
    a.tw = c->d_tw_inv;
    a.mods = c->d_mods;
    a.ninv = c->d_ninv;
    a.log_n = c->log_n;
    a.scale = all_limbs ? c->d_bfv_kscale : c->d_iscale;
    a.e_ext = ext + (size_t)(p0 / 2) * ndig * QP * N;
    a.e_ksk = ksk;
    a.e_ndig = ndig;
    a.e_QP = QP;
    a.e_kQP = ctx_key_qp(c);
    a.e_kshift = c->key_pshift;
    a.e_ext_g = ext_g & ((2u << c->log_n) - 1);
    if (rb) {
      a.e_rp = 2 * n;
      for (u32 r = 0; r < nr; ++r) {
        a.e_ksk_r[r] = rb->ksk[r];
        a.e_g_r[r] = rb->g[r] & ((2u << c->log_n) - 1);
      }
    }
    const u32 n_jobs = np * nl;
    int rc;
    switch (ndig + (ext_g || rb ? 4 : 0)) {
      case 1: rc = row_pass<PRO_KSP>(c, a, true, n_jobs); break;
      case 2: rc = row_pass<PRO_KSP + 1>(c, a, true, n_jobs); break;
      case 3: rc = row_pass<PRO_KSP + 2>(c, a, true, n_jobs); break;
      case 4: rc = row_pass<PRO_KSP + 3>(c, a, true, n_jobs); break;
      case 5: rc = row_pass<PRO_KSPG>(c, a, true, n_jobs); break;
      case 6: rc = row_pass<PRO_KSPG + 1>(c, a, true, n_jobs); break;
      case 7: rc = row_pass<PRO_KSPG + 2>(c, a, true, n_jobs); break;
      default: rc = row_pass<PRO_KSPG + 3>(c, a, true, n_jobs); break;
    }
    if (rc) return rc;
    if ((rc = ntt_col_plain(c, a, true, n_jobs))) return rc;
  }
  return FHE_OK;
}

