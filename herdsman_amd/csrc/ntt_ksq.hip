// ntt_ksq.hip -- NTT(conv) with the ModDown finish (EPI_COMBINE) and the Q-limb inner product (EPI_KSQ)
// (kernel templates: ntt_core.hpp; one translation unit per entry-point family so
// the ~360 pass kernels compile in parallel)
#include "ntt_core.hpp"

// Forward NTT of the ModDown conversion conv (all L limbs of 2n polys) with
// the ModDown finish fused into its last pass (EPI_COMBINE):
//   out[p][i] = (add_mask bit (p & 1) ? base[p][i] : 0) + (acc[p][i] - NTT(conv)[p][i]) P^-1  mod q_i
// conv is transformed in place by the first pass only; acc rows have stride acc_stride limbs.
// With ext (EPI_KSQ, two-pass sizes) acc's Q limbs are not read: the last pass
// forms acc[2 ct + b][i] = sum_j ext[ct][j][i] ksk[j][b][i] R^-1 itself.
int ntt_fwd_combine_launch(fhe_ctx *c, u64 *conv, u32 n_polys, const u64 *acc, u32 acc_stride, const u64 *base,
                           u64 *out, u32 add_mask, const ConvTab *pro, const u64 *ext, const u64 *ksk, u32 ndig,
                           u32 base_g, const u64 *pinv, const ConvSrc *pro_src, u32 ext_g, const RotBatch *rb,
                           const TensorSrc *tsrc) {
  const u32 L = c->L, QP = c->L + c->K;
  const size_t N = c->n;
  if (ext && (c->log_n <= 14 || ndig > 4 || (n_polys & 1)))
    return fhe_fail(c, FHE_ERR_UNSUPPORTED, "fused key-switch inner product: log_n / digits");
  if (base_g && c->log_n <= 14) return fhe_fail(c, FHE_ERR_UNSUPPORTED, "rotated combine base: log_n");
  if ((ext_g || rb) && !ext) return fhe_fail(c, FHE_ERR_INVALID, "gathered ext without the fused inner product");
  // tsrc: the base is formed from the ciphertexts (EPI_KSQT), added to both polys;
  // tsrc->g: a rotation's fused finish (base sigma_g(c0) on poly 0)
  if (tsrc && (!ext || ext_g || rb ||
               (tsrc->g ? !tsrc->fused || (base_g & ((2u << c->log_n) - 1)) != tsrc->g || add_mask != 1u
                                                : base_g || add_mask != 3u)))
    return fhe_fail(c, FHE_ERR_INVALID, "fused finish: plain fused inner product only");
  // rb: the n_polys = 2 n nr polys of rb->nr rotations in one chunk; base (the
  // ciphertexts, read through each rotation's sigma_g) has 2 n polys
  if (rb && (rb->nr < 1 || rb->nr > FHE_ROT_BATCH || n_polys > COMBINE_CHUNK || n_polys % (2 * rb->nr)))
    return fhe_fail(c, FHE_ERR_INVALID, "rotation batch: count / size");
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
    a.e_pinv = pinv ? pinv : c->d_pinv;
    a.e_acc_stride = acc_stride;
    a.e_add_mask = add_mask;
    a.e_g = base_g & ((2u << c->log_n) - 1);
    if (ext) {
      a.e_ext = ext + (size_t)(p0 / 2) * ndig * QP * N;
      a.e_ksk = ksk;
      a.e_ndig = ndig;
      a.e_QP = QP;
      a.e_kQP = ctx_key_qp(c);
      if (tsrc) {
        a.e_ta = tsrc->a + (size_t)p0 * L * N;  // poly p0 = 2 ct: ciphertext ct's a_0
        a.e_tb = tsrc->b ? tsrc->b + (size_t)p0 * L * N : nullptr;
        a.t_alpha = c->alpha;  // the own digit of limb i: i / alpha (its ext word is formed, not read)
      }
      a.e_ext_g = ext_g & ((2u << c->log_n) - 1);
      if (rb) {
        a.e_rp = n_polys / rb->nr;
        for (u32 r = 0; r < rb->nr; ++r) {
          a.e_ksk_r[r] = rb->ksk[r];
          a.e_out_r[r] = rb->out[r];
          a.e_g_r[r] = rb->g[r] & ((2u << c->log_n) - 1);
        }
      }
    }
    const u32 n_jobs = np * L;
    int rc;
    if (c->log_n <= 14) {
      rc = single_pass<EPI_COMBINE>(c, a, false, n_jobs);
    } else {
      if (pro) {
        // the ModDown conversion P -> Q as the column pass's prologue: the
        // sources are acc's P limbs, already scaled by the INTT (d_iscale)
        if (pro_src) {
          a.c_src = pro_src->src + (size_t)p0 * pro_src->stride * N;
          a.c_src_stride = pro_src->stride;
          a.c_src_first = pro_src->first;
          a.c_lift_half = pro_src->lift_half;
          a.c_lift_sub = pro_src->lift_sub;
        } else {
          a.c_src = acc + (size_t)p0 * acc_stride * N;
          a.c_src_stride = acc_stride;
          a.c_src_first = L;
        }
        a.c_ns = pro->ns;
        a.c_nd = pro->nd;
        a.c_h = pro->h;
        if (tsrc && tsrc->convf && !pro_src) {
          // CONVF: acc's P rows hold INTT(acc_P)'s row-pass output; its column
          // pass (d_iscale) runs in the conversion's kernel (ntt_convf.hip)
          ConvfArgs f{};
          f.src = a.c_src;
          f.src_stride = acc_stride;
          f.src_first = L;
          f.src_mod0 = L;
          f.scale = c->d_iscale;
          f.tmap = a.map;
          f.h = pro->h;
          f.nd = pro->nd;
          f.src60 = 0;
          f.mods = c->d_mods;
          f.twi = c->d_tw_inv;
          f.twf = c->d_tw_fwd;
          rc = ntt_convf_launch(c, f, pro->ns);
        } else {
          rc = ntt_conv_col(c, a, n_jobs);
        }
      } else {
        rc = ntt_col_plain(c, a, false, n_jobs);
      }
      if (rc) return rc;
      if (tsrc && tsrc->fused) {
        // the row transforms of ext's Q limbs and of NTT(conv), the inner
        // product and the finish in one kernel (ntt_ksf.hip)
        rc = ntt_ks_fused_finish_launch(c, a.map.base, a.e_ext, ksk, ndig, a.e_ta, a.e_tb, a.e_out, np / 2,
                                        tsrc->g);
        if (rc) return rc;
        continue;
      }
      switch (ext ? ndig + (ext_g || rb ? 4 : 0) + (tsrc ? 8 : 0) : 0) {
        case 9: rc = row_pass<EPI_KSQT>(c, a, false, n_jobs); break;
        case 10: rc = row_pass<EPI_KSQT + 1>(c, a, false, n_jobs); break;
        case 11: rc = row_pass<EPI_KSQT + 2>(c, a, false, n_jobs); break;
        case 12: rc = fhe_fail(c, FHE_ERR_UNSUPPORTED, "split tensor product: 4 digits"); break;  // spills
        case 5: rc = row_pass<EPI_KSQG>(c, a, false, n_jobs); break;
        case 6: rc = row_pass<EPI_KSQG + 1>(c, a, false, n_jobs); break;
        case 7: rc = row_pass<EPI_KSQG + 2>(c, a, false, n_jobs); break;
        case 8: rc = row_pass<EPI_KSQG + 3>(c, a, false, n_jobs); break;
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

