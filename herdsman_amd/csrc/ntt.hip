// ntt.hip -- negacyclic NTT / INTT for gfx950: the plain passes and ntt_launch.
// The algorithm and the MI355X mapping are described at the top of ntt_core.hpp;
// the fused entry points live in ntt_ksq.hip, ntt_ksp.hip, ntt_front.hip and the
// conversion column passes in ntt_conv12.hip / ntt_conv34.hip.
#include "ntt_core.hpp"

int ntt_single_plain(fhe_ctx *c, const NttArgs &a, bool inv, u32 n_jobs) { return single_pass(c, a, inv, n_jobs); }
int ntt_col_plain(fhe_ctx *c, const NttArgs &a, bool inv, u32 n_jobs) { return col_pass(c, a, inv, n_jobs); }
int ntt_row_plain(fhe_ctx *c, const NttArgs &a, bool inv, u32 n_jobs) { return row_pass(c, a, inv, n_jobs); }


#ifndef NTT_PERSIST
#define NTT_PERSIST 14  // plain NTTs at log_n in [NTT_PERSIST, 14] run the persistent one-pass kernel (15: none)
#endif

// the persistent one-residue-per-workgroup pass (ntt_persist), or 1 if the
// launch's moduli mix both lazy-schedule classes (the two-pass path takes it).
// Generic moduli too (round 6): the modulus constants the butterflies pin in
// SGPRs are made visibly uniform (uniform64), which clears ROCm 7.2's
// "illegal VGPR to SGPR copy" on the generic multi-residue instantiations.
template <int LOG_N, bool SP>
static int persist_sp(fhe_ctx *c, const NttArgs &a, bool inv, u32 n_jobs) {
  if (inv) return launch_persist<LOG_N, true, SP, 0>(c, a, n_jobs);
  switch (wide_mode(c, a.map)) {
    case 1: return launch_persist<LOG_N, false, SP, 1>(c, a, n_jobs);
    case 0: return launch_persist<LOG_N, false, SP, 0>(c, a, n_jobs);
  }
  return 1;
}
template <int LOG_N>
static int persist(fhe_ctx *c, const NttArgs &a, bool inv, u32 n_jobs) {
  return c->special ? persist_sp<LOG_N, true>(c, a, inv, n_jobs) : persist_sp<LOG_N, false>(c, a, inv, n_jobs);
}

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
  // N = 2^14: the persistent one-pass kernel (ntt_persist: one 1024-thread
  // workgroup per CU with 128 KiB of LDS, PERSIST_K residues per workgroup, the
  // next residue prefetched into registers).  Launches mixing both lazy-schedule
  // classes take two passes of 7 stages with 32 sub-transforms per workgroup
  // (35 KiB of LDS, 4 workgroups per CU).
  int rc;
  if (c->log_n >= NTT_PERSIST && c->log_n <= 14) {
    rc = c->log_n == 14 ? persist<14>(c, a, inverse, n_jobs)
                        : NTT_PERSIST <= 13 ? persist<NTT_PERSIST <= 13 ? 13 : 14>(c, a, inverse, n_jobs) : 1;
    if (rc != 1) return rc;
  }
  if (c->log_n <= 13) return single_pass(c, a, inverse, n_jobs);
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

