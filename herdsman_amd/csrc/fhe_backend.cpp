// fhe_backend.cpp -- C ABI (include/plugins/fhe_backend.h): context setup,
// parameter precomputation and op orchestration.  Host code only; kernels
// live in ntt.hip / rns.hip.  Nothing here computes on the CPU what the ABI
// promises to compute on the GPU: host work is limited to one-off table
// generation at context creation (primes, roots, CRT constants).
#include <cstdlib>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <map>
#include <memory>
#include <new>
#include <string>
#include <vector>

#include "context.hpp"

typedef unsigned __int128 u128;

// ------------------------------------------------------------ host math
static u64 hmul(u64 a, u64 b, u64 q) { return (u64)(((u128)a * b) % q); }
static u64 hpow(u64 b, u64 e, u64 q) {
  u64 r = 1 % q;
  b %= q;
  while (e) {
    if (e & 1) r = hmul(r, b, q);
    b = hmul(b, b, q);
    e >>= 1;
  }
  return r;
}
static u64 hinv(u64 a, u64 q) { return hpow(a % q, q - 2, q); }
static u64 tomont(u64 x, u64 q) { return (u64)(((u128)(x % q) << 64) % q); }
u64 host_mulmod(u64 a, u64 b, u64 q) { return hmul(a, b, q); }
u64 host_inv(u64 a, u64 q) { return hinv(a, q); }
u64 host_to_mont(u64 x, u64 q) { return tomont(x, q); }
static u32 hbrv(u32 x, u32 bits) {
  u32 r = 0;
  for (u32 i = 0; i < bits; ++i) { r = (r << 1) | (x & 1); x >>= 1; }
  return r;
}
static bool is_prime(u64 n) {
  static const u64 bases[] = {2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37};
  if (n < 2) return false;
  for (u64 b : bases) {
    if (n == b) return true;
    if (n % b == 0) return false;
  }
  u64 d = n - 1;
  int s = 0;
  while (!(d & 1)) { d >>= 1; ++s; }
  for (u64 a : bases) {
    u64 x = hpow(a, d, n);
    if (x == 1 || x == n - 1) continue;
    bool comp = true;
    for (int r = 1; r < s; ++r) {
      x = hmul(x, x, n);
      if (x == n - 1) { comp = false; break; }
    }
    if (comp) return false;
  }
  return true;
}
// Prime family of the backend: the largest primes q < 2^bits with
// q = 1 (mod 2^32), descending, not in `used`.  q = 1 mod 2^32 implies
// q = 1 mod 2N for every N <= 2^31 (NTT-friendly) and makes the Montgomery
// quotient digit free on 32-bit multipliers (modarith.hpp).
static bool gen_primes(u32 bits, u32 count, std::vector<u64> &used, std::vector<u64> &out) {
  const u64 step = 1ull << 32;
  for (u64 k = ((1ull << bits) - 2) / step; k > 0 && count; --k) {
    const u64 q = k * step + 1;
    if (std::find(used.begin(), used.end(), q) != used.end()) continue;
    if (is_prime(q)) { out.push_back(q); used.push_back(q); --count; }
  }
  return count == 0;
}
// smallest primitive 2N-th root of unity mod q
static u64 min_psi(u64 q, u32 log_n) {
  const u64 n = 1ull << log_n;
  u64 g = 0;
  for (u64 x = 2; x < q; ++x) {
    g = hpow(x, (q - 1) / (2 * n), q);
    if (hpow(g, n, q) == q - 1) break;
  }
  const u64 g2 = hmul(g, g, q);
  u64 best = g, cur = g;
  for (u64 k = 1; k < n; ++k) {
    cur = hmul(cur, g2, q);
    if (cur < best) best = cur;
  }
  return best;
}

// ------------------------------------------------------------ helpers
int fhe_fail(fhe_ctx *c, int code, const std::string &msg) {
  if (c) c->err = msg;
  return code;
}
int fhe_check(fhe_ctx *c, hipError_t e, const char *what) {
  if (e == hipSuccess) return FHE_OK;
  return fhe_fail(c, e == hipErrorOutOfMemory ? FHE_ERR_OOM : FHE_ERR_DEVICE,
                  std::string(what) + ": " + hipGetErrorString(e));
}
void *ctx_upload(fhe_ctx *c, const void *host, size_t bytes) {
  void *p = nullptr;
  if (hipMalloc(&p, bytes) != hipSuccess) return nullptr;
  if (hipMemcpy(p, host, bytes, hipMemcpyHostToDevice) != hipSuccess) {
    (void)hipFree(p);
    return nullptr;
  }
  c->blobs.push_back(p);
  return p;
}
// level views use their parent's workspace (they run on its stream)
int ctx_workspace(fhe_ctx *c, size_t bytes, void **out) {
  fhe_ctx *o = c->parent ? c->parent : c;
  if (bytes > o->ws_bytes) {
    if (o->ws) {
      int rc = fhe_check(c, hipStreamSynchronize(c->stream), "workspace sync");
      if (rc) return rc;
      (void)hipFree(o->ws);
      o->ws = nullptr;
      o->ws_bytes = 0;
    }
    int rc = fhe_check(c, hipMalloc(&o->ws, bytes), "workspace alloc");
    if (rc) return rc;
    o->ws_bytes = bytes;
  }
  *out = o->ws;
  return FHE_OK;
}

// fold_ninv: the sources arrive as N * x (an inverse NTT without its N^-1), so
// the per-source constant also carries N^-1
ConvTab make_conv_tab(fhe_ctx *c, const std::vector<u32> &src, const std::vector<u32> &dst, int r_exp,
                      bool fold_ninv, int r_exp_q) {
  ConvTab t{};
  t.ns = (u32)src.size();
  t.nd = (u32)dst.size();
  std::vector<u64> hi(t.ns);
  std::vector<u64> h((size_t)t.ns * t.nd);
  for (u32 i = 0; i < t.ns; ++i) {
    const u64 si = c->moduli[src[i]];
    u64 prod = 1;
    for (u32 k = 0; k < t.ns; ++k)
      if (k != i) prod = hmul(prod, c->moduli[src[k]] % si, si);
    hi[i] = tomont(fold_ninv ? hmul(hinv(prod, si), hinv((u64)c->n % si, si), si) : hinv(prod, si), si);
    for (u32 m = 0; m < t.nd; ++m) {
      const u64 dm = c->moduli[dst[m]];
      u64 p2 = 1;
      for (u32 k = 0; k < t.ns; ++k)
        if (k != i) p2 = hmul(p2, c->moduli[src[k]] % dm, dm);
      const int ex = r_exp_q != kNoExp && dst[m] < c->L ? r_exp_q : r_exp;
      for (int e = 0; e < ex; ++e) p2 = tomont(p2, dm);
      for (int e = ex; e < 0; ++e) p2 = hmul(p2, hinv(tomont(1, dm), dm), dm);  // times R^-1
      h[(size_t)i * t.nd + m] = p2;
    }
  }
  t.src_mod = (const u32 *)ctx_upload(c, src.data(), sizeof(u32) * t.ns);
  t.dst_mod = (const u32 *)ctx_upload(c, dst.data(), sizeof(u32) * std::max<u32>(t.nd, 1));
  t.hinv = (const u64 *)ctx_upload(c, hi.data(), sizeof(u64) * t.ns);
  t.h = (const u64 *)ctx_upload(c, h.data(), sizeof(u64) * std::max<size_t>(h.size(), 1));
  return t;
}

static void ctx_release(fhe_ctx *c) {
  if (!c) return;
  for (fhe_ctx *v : c->views)
    if (v) {
      ctx_release(v);
      delete v;
    }
  c->views.clear();
  for (void *p : c->blobs) (void)hipFree(p);
  c->blobs.clear();
  c->conv_cache.clear();
  if (c->ws) (void)hipFree(c->ws);
  c->ws = nullptr;
  if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
  c->own_stream = nullptr;
  for (hipEvent_t &e : c->marks) {
    if (e) (void)hipEventDestroy(e);
    e = nullptr;
  }
}

// ------------------------------------------------------------ context
// alpha: digit size override (level views keep their parent's alpha, which
// ceil(m / dnum_m) need not reproduce)
static int ctx_build(fhe_ctx *c, const fhe_params *p, u32 alpha = 0) {
  c->params = *p;
  c->params.moduli = nullptr;
  c->log_n = p->log_n;
  c->n = 1u << p->log_n;
  c->L = p->num_q;
  c->K = p->num_p;
  c->dnum = p->dnum;
  c->alpha = alpha ? alpha : (c->L + c->dnum - 1) / c->dnum;
  c->t = p->plain_modulus;
  c->nB = p->scheme == FHE_SCHEME_BFV ? c->L + 1 : 0;
  c->nmod = c->L + c->K + c->nB;
  if (p->scheme > FHE_SCHEME_BFV) return fhe_fail(c, FHE_ERR_INVALID, "unknown scheme");
  if (p->flags & ~FHE_FLAG_BFV_HPS) return fhe_fail(c, FHE_ERR_INVALID, "unknown fhe_params.flags bits");
  if ((p->flags & FHE_FLAG_BFV_HPS) && p->scheme != FHE_SCHEME_BFV)
    return fhe_fail(c, FHE_ERR_INVALID, "FHE_FLAG_BFV_HPS on a CKKS context");
  if (p->log_n < 10 || p->log_n > 17) return fhe_fail(c, FHE_ERR_UNSUPPORTED, "log_n must be in [10, 17]");
  if (c->L == 0 || c->dnum == 0 || c->dnum > c->L) return fhe_fail(c, FHE_ERR_INVALID, "need 1 <= dnum <= L");
  if (c->alpha > 16) return fhe_fail(c, FHE_ERR_UNSUPPORTED, "alpha = ceil(L/dnum) must be <= 16");
  if (c->K > 16) return fhe_fail(c, FHE_ERR_UNSUPPORTED, "K must be <= 16");
  if (c->nmod > FHE_MAX_MODS) return fhe_fail(c, FHE_ERR_UNSUPPORTED, "too many moduli");
  if (p->scheme == FHE_SCHEME_BFV && (c->t < 2 || c->K == 0))
    return fhe_fail(c, FHE_ERR_INVALID, "BFV needs a plain modulus t >= 2 and K >= 1");
  // moduli
  if (p->moduli) {
    c->moduli.assign(p->moduli, p->moduli + c->nmod);
    const u64 two_n = 2ull << p->log_n;
    for (u64 q : c->moduli)
      if (q >= (1ull << 61) || q % two_n != 1 || !is_prime(q))
        return fhe_fail(c, FHE_ERR_INVALID, "explicit modulus is not an NTT-friendly prime < 2^61");
    for (size_t i = 0; i < c->moduli.size(); ++i)
      for (size_t j = 0; j < i; ++j)
        if (c->moduli[i] == c->moduli[j]) return fhe_fail(c, FHE_ERR_INVALID, "duplicate modulus");
  } else {
    if (p->q_bits < 36 || p->q_bits > 61 || p->p_bits < 36 || p->p_bits > 61)
      return fhe_fail(c, FHE_ERR_INVALID, "q_bits / p_bits must be in [36, 61]");
    std::vector<u64> used;
    if (!gen_primes(p->q_bits, c->L, used, c->moduli) || !gen_primes(p->p_bits, c->K, used, c->moduli) ||
        !gen_primes(p->p_bits, c->nB, used, c->moduli))
      return fhe_fail(c, FHE_ERR_INVALID, "not enough primes q = 1 mod 2^32 below the bit bound");
  }
  c->special = true;
  for (u64 q : c->moduli) c->special = c->special && ((q & 0xffffffffull) == 1);
  c->fold_ninv = p->scheme == FHE_SCHEME_CKKS;
  const u32 n = c->n, nm = c->nmod;
  // per-modulus tables, constants in Montgomery form (x * 2^64 mod q)
  std::vector<ModInfo> mods(nm);
  std::vector<u64> twf((size_t)nm * n), twi((size_t)nm * n), ninv(nm), r2(nm);
  std::vector<u64> pw(n), ipw(n);
  for (u32 m = 0; m < nm; ++m) {
    const u64 q = c->moduli[m];
    u64 inv = q;  // q^-1 mod 2^64 by Newton iteration
    for (int it = 0; it < 6; ++it) inv *= 2 - q * inv;
    r2[m] = tomont(tomont(1, q), q);
    mods[m] = ModInfo{q, 0 - inv, r2[m], (u32)(q >> 32), (u32)((q & 0xffffffffull) == 1)};
    const u64 psi = min_psi(q, c->log_n), ipsi = hinv(psi, q);
    u64 a = 1, b = 1;
    for (u32 i = 0; i < n; ++i) { pw[i] = a; ipw[i] = b; a = hmul(a, psi, q); b = hmul(b, ipsi, q); }
    for (u32 i = 0; i < n; ++i) {
      const u32 r = hbrv(i, c->log_n);
      twf[(size_t)m * n + i] = tomont(pw[r], q);
      twi[(size_t)m * n + i] = tomont(ipw[r], q);
    }
    ninv[m] = tomont(hinv(n, q), q);
  }
  c->d_mods = (ModInfo *)ctx_upload(c, mods.data(), sizeof(ModInfo) * nm);
  c->d_tw_fwd = (u64 *)ctx_upload(c, twf.data(), sizeof(u64) * twf.size());
  c->d_tw_inv = (u64 *)ctx_upload(c, twi.data(), sizeof(u64) * twi.size());
  c->d_ninv = (u64 *)ctx_upload(c, ninv.data(), sizeof(u64) * nm);
  c->d_r2 = (u64 *)ctx_upload(c, r2.data(), sizeof(u64) * nm);
  if (!c->d_mods || !c->d_tw_fwd || !c->d_tw_inv || !c->d_ninv || !c->d_r2)
    return fhe_fail(c, FHE_ERR_OOM, "table upload");
  // key-switching tables
  if (c->K) {
    const u32 L = c->L, QP = c->L + c->K;
    std::vector<u64> pinv(L), pr2(L);
    for (u32 i = 0; i < L; ++i) {
      const u64 q = c->moduli[i];
      u64 P = 1;
      for (u32 k = 0; k < c->K; ++k) P = hmul(P, c->moduli[L + k] % q, q);
      pinv[i] = tomont(hinv(P, q), q);
      pr2[i] = tomont(tomont(P, q), q);
    }
    c->d_pinv = (u64 *)ctx_upload(c, pinv.data(), sizeof(u64) * L);
    c->d_pr2 = (u64 *)ctx_upload(c, pr2.data(), sizeof(u64) * L);
    std::vector<ConvTab> tabs;
    for (u32 j = 0; j * c->alpha < L; ++j) {
      const u32 lo = j * c->alpha, hi = std::min(lo + c->alpha, L);
      std::vector<u32> src, dst;
      for (u32 i = lo; i < hi; ++i) src.push_back(i);
      for (u32 i = 0; i < QP; ++i)
        if (i < lo || i >= hi) dst.push_back(i);
      tabs.push_back(make_conv_tab(c, src, dst, 2, c->fold_ninv));  // ModUp output carries a factor R
    }
    c->d_modup = (ConvTab *)ctx_upload(c, tabs.data(), sizeof(ConvTab) * tabs.size());
    c->modup_tabs = tabs;
    std::vector<u32> src, dst;
    for (u32 k = 0; k < c->K; ++k) src.push_back(L + k);
    for (u32 i = 0; i < L; ++i) dst.push_back(i);
    c->moddown = make_conv_tab(c, src, dst, 1, c->fold_ninv);
    if (!c->d_pinv || !c->d_pr2 || !c->d_modup || !c->moddown.h) return fhe_fail(c, FHE_ERR_OOM, "ks table upload");
    // ModDown fused into NTT(conv): INTT(acc_P)'s output constants carry the
    // conversion's (P/p_k)^-1 and N^-1 (two-pass sizes, at most 4 sources)
    c->fuse_moddown = c->fold_ninv && c->log_n >= 15 && c->K <= 4;
    // ModUp fused into the column pass of the NTT of its outputs likewise
    // (at most 4 sources per digit: the PRO_CONV prologue)
    c->fuse_modup = c->fuse_moddown && c->alpha <= 4;
    if (c->fuse_moddown) {
      std::vector<u64> isc(c->nmod, 0);
      for (u32 k = 0; k < c->K; ++k) {
        const u64 pk = c->moduli[L + k];
        u64 prod = 1;
        for (u32 m = 0; m < c->K; ++m)
          if (m != k) prod = hmul(prod, c->moduli[L + m] % pk, pk);
        isc[L + k] = tomont(hmul(hinv(prod, pk), hinv((u64)c->n % pk, pk), pk), pk);
      }
      // Q limbs: ModUp's per-source constant N^-1 (Q_j/q_i)^-1 (make_conv_tab, fold_ninv)
      for (u32 i = 0; c->fuse_modup && i < L; ++i) {
        const u32 lo = i / c->alpha * c->alpha, hi = std::min(lo + c->alpha, L);
        const u64 qi = c->moduli[i];
        u64 prod = 1;
        for (u32 m = lo; m < hi; ++m)
          if (m != i) prod = hmul(prod, c->moduli[m] % qi, qi);
        isc[i] = tomont(hmul(hinv(prod, qi), hinv((u64)c->n % qi, qi), qi), qi);
      }
      c->d_iscale = (u64 *)ctx_upload(c, isc.data(), sizeof(u64) * isc.size());
      std::vector<u64> isct(isc.size());
      for (u32 m = 0; m < c->nmod; ++m) isct[m] = tomont(isc[m], c->moduli[m]);
      c->d_iscale_t = (u64 *)ctx_upload(c, isct.data(), sizeof(u64) * isct.size());
      if (!c->d_iscale || !c->d_iscale_t) return fhe_fail(c, FHE_ERR_OOM, "ks table upload");
    }
    // the fused key switch's tables (ntt_ksf.hip: accumulator scale R^-2)
    if (c->fuse_modup) {
      for (u32 j = 0; j * c->alpha < L; ++j) {
        const u32 lo = j * c->alpha, hi = std::min(lo + c->alpha, L);
        std::vector<u32> src, dst;
        for (u32 i = lo; i < hi; ++i) src.push_back(i);
        for (u32 i = 0; i < QP; ++i)
          if (i < lo || i >= hi) dst.push_back(i);
        c->modup_tabs_ksf.push_back(make_conv_tab(c, src, dst, 2, c->fold_ninv, 0));  // Q targets times R^-1
        if (!c->modup_tabs_ksf.back().h) return fhe_fail(c, FHE_ERR_OOM, "ks table upload");
      }
      std::vector<u32> src, dst;
      for (u32 k = 0; k < c->K; ++k) src.push_back(L + k);
      for (u32 i = 0; i < L; ++i) dst.push_back(i);
      c->moddown_ksf = make_conv_tab(c, src, dst, -1, c->fold_ninv);  // conv times R^-2
      std::vector<u64> pinv3(L), pplain(L), pm1(L);
      for (u32 i = 0; i < L; ++i) {
        const u64 q = c->moduli[i];
        u64 P = 1;
        for (u32 k = 0; k < c->K; ++k) P = hmul(P, c->moduli[L + k] % q, q);
        pinv3[i] = tomont(tomont(tomont(hinv(P, q), q), q), q);
        pplain[i] = P;
        pm1[i] = hmul(P, hinv(tomont(1, q), q), q);
      }
      c->d_pinv3 = (u64 *)ctx_upload(c, pinv3.data(), sizeof(u64) * L);
      c->d_pplain = (u64 *)ctx_upload(c, pplain.data(), sizeof(u64) * L);
      c->d_pm1 = (u64 *)ctx_upload(c, pm1.data(), sizeof(u64) * L);
      if (!c->moddown_ksf.h || !c->d_pinv3 || !c->d_pplain || !c->d_pm1)
        return fhe_fail(c, FHE_ERR_OOM, "ks table upload");
    }
    // BFV relinearisation with the fused passes (bfv_ks_fused, rns.hip)
    const u32 ndig = (L + c->alpha - 1) / c->alpha;
    c->bfv_ks_fuse = p->scheme == FHE_SCHEME_BFV && c->log_n >= 15 && c->alpha <= 4 && c->K <= 4 && ndig <= 4;
    if (c->bfv_ks_fuse) {
      std::vector<u64> dsc(L), ksc(c->nmod, 0);
      for (u32 i = 0; i < L; ++i) {
        const u32 lo = i / c->alpha * c->alpha, hi = std::min(lo + c->alpha, L);
        const u64 qi = c->moduli[i];
        u64 prod = 1;
        for (u32 m = lo; m < hi; ++m)
          if (m != i) prod = hmul(prod, c->moduli[m] % qi, qi);
        dsc[i] = tomont(hinv(prod, qi), qi);
        ksc[i] = tomont(hinv((u64)c->n % qi, qi), qi);
      }
      for (u32 k = 0; k < c->K; ++k) {
        const u64 pk = c->moduli[L + k];
        u64 prod = 1;
        for (u32 m = 0; m < c->K; ++m)
          if (m != k) prod = hmul(prod, c->moduli[L + m] % pk, pk);
        ksc[L + k] = tomont(hmul(hinv(prod, pk), hinv((u64)c->n % pk, pk), pk), pk);
      }
      c->d_bfv_dscale = (u64 *)ctx_upload(c, dsc.data(), sizeof(u64) * L);
      c->d_bfv_kscale = (u64 *)ctx_upload(c, ksc.data(), sizeof(u64) * ksc.size());
      if (!c->d_bfv_dscale || !c->d_bfv_kscale) return fhe_fail(c, FHE_ERR_OOM, "ks table upload");
    }
  }
  if (p->scheme == FHE_SCHEME_BFV) {
    int rc = (p->flags & FHE_FLAG_BFV_HPS) ? hps_setup(c) : behz_setup(c);
    if (rc) return rc;
  }
  return FHE_OK;
}

// ------------------------------------------------------------ level views
int ctx_level(fhe_ctx *c, u32 m, fhe_ctx **out) {
  fhe_ctx *r = c->parent ? c->parent : c;
  *out = nullptr;
  if (m == r->L) {
    *out = r;
    return FHE_OK;
  }
  if (r->params.scheme != FHE_SCHEME_CKKS) return fhe_fail(c, FHE_ERR_UNSUPPORTED, "reduced levels are CKKS only");
  if (m < 1 || m > r->L) return fhe_fail(c, FHE_ERR_INVALID, "level must be in [1, L]");
  if (r->views.size() < r->L) r->views.resize(r->L, nullptr);
  fhe_ctx *v = r->views[m];
  if (!v) {
    v = new (std::nothrow) fhe_ctx();
    if (!v) return fhe_fail(c, FHE_ERR_OOM, "level view");
    v->parent = r;
    v->device = r->device;
    v->stream = r->stream;
    fhe_params p = r->params;
    std::vector<u64> mods(r->moduli.begin(), r->moduli.begin() + m);
    mods.insert(mods.end(), r->moduli.begin() + r->L, r->moduli.begin() + r->L + r->K);
    p.num_q = m;
    p.dnum = (m + r->alpha - 1) / r->alpha;
    p.moduli = mods.data();
    int rc = ctx_build(v, &p, r->alpha);
    if (!rc) {
      v->key_qp = r->L + r->K;
      v->key_pshift = r->L - m;
      // rescale m+1 -> m: q_m^-1 R mod q_i, then q_m mod q_i (i < m)
      const u64 qm = r->moduli[m];
      std::vector<u64> qd(2 * (size_t)m);
      for (u32 i = 0; i < m; ++i) {
        const u64 qi = r->moduli[i];
        qd[i] = tomont(hinv(qm % qi, qi), qi);
        qd[m + i] = qm % qi;
      }
      v->d_qdrop = (u64 *)ctx_upload(v, qd.data(), sizeof(u64) * qd.size());
      // the rescale lift as a 1-source conversion prologue: h = R mod q_i (y = x mod q_i)
      std::vector<u64> h1(m);
      for (u32 i = 0; i < m; ++i) h1[i] = tomont(1, r->moduli[i]);
      v->lift.ns = 1;
      v->lift.nd = m;
      v->lift.h = (const u64 *)ctx_upload(v, h1.data(), sizeof(u64) * m);
      if (!v->d_qdrop || !v->lift.h) rc = fhe_fail(v, FHE_ERR_OOM, "level view tables");
    }
    if (rc) {
      fhe_fail(c, rc, "level view: " + v->err);
      ctx_release(v);
      delete v;
      return rc;
    }
    r->views[m] = v;
  }
  v->stream = r->stream;
  v->err.clear();
  *out = v;
  return FHE_OK;
}

static thread_local std::string g_create_error;

extern "C" {

int fhe_ctx_create(const fhe_params *params, int device, fhe_ctx **out) {
  if (!params || !out) return FHE_ERR_INVALID;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    g_create_error = "no HIP device";
    return FHE_ERR_DEVICE;
  }
  if (device < 0 || device >= ndev) return FHE_ERR_INVALID;
  DeviceIdBind bind(device);  // the caller's current device is restored on return
  if (!bind.ok) {
    g_create_error = "hipSetDevice failed";
    return FHE_ERR_DEVICE;
  }
  fhe_ctx *c = new (std::nothrow) fhe_ctx();
  if (!c) return FHE_ERR_OOM;
  c->device = device;
  int rc = ctx_build(c, params);
  if (rc) {
    g_create_error = c->err;
    ctx_release(c);
    delete c;
    return rc;
  }
  *out = c;
  return FHE_OK;
}

void fhe_ctx_destroy(fhe_ctx *c) {
  if (!c) return;
  DeviceIdBind bind(c->device);
  (void)hipStreamSynchronize(c->stream);
  ctx_release(c);
  delete c;
}

const char *fhe_last_error(const fhe_ctx *c) { return c ? c->err.c_str() : g_create_error.c_str(); }

int fhe_ctx_moduli(const fhe_ctx *c, uint64_t *out, uint32_t cap, uint32_t *count) {
  if (!c) return FHE_ERR_INVALID;
  if (count) *count = c->nmod;
  if (out) std::memcpy(out, c->moduli.data(), sizeof(u64) * std::min(cap, c->nmod));
  return FHE_OK;
}

int fhe_set_stream(fhe_ctx *c, void *stream) {
  if (!c) return FHE_ERR_INVALID;
  c->stream = (hipStream_t)stream;
  return FHE_OK;
}

int fhe_synchronize(fhe_ctx *c) {
  if (!c) return FHE_ERR_INVALID;
  DeviceBind bind(c);
  return fhe_check(c, hipStreamSynchronize(c->stream), "synchronize");
}

int fhe_mark(fhe_ctx *c, uint32_t slot) {
  if (!c) return FHE_ERR_INVALID;
  if (slot >= FHE_MAX_MARKS) return fhe_fail(c, FHE_ERR_INVALID, "mark slot out of range");
  DeviceBind bind(c);
  if (!c->marks[slot]) {
    // blocking sync: a lane thread waiting on a batch sleeps instead of spinning
    // against the lanes' IO threads (HERD_FHE_SPIN_WAIT=1 keeps the spin wait)
    static const bool spin = [] {
      const char *e = getenv("HERD_FHE_SPIN_WAIT");
      return e && e[0] == '1';
    }();
    const unsigned flags = hipEventDisableTiming | (spin ? 0u : hipEventBlockingSync);
    int rc = fhe_check(c, hipEventCreateWithFlags(&c->marks[slot], flags), "mark create");
    if (rc) return rc;
  }
  return fhe_check(c, hipEventRecord(c->marks[slot], c->stream), "mark record");
}

int fhe_wait_mark(fhe_ctx *c, uint32_t slot) {
  if (!c) return FHE_ERR_INVALID;
  if (slot >= FHE_MAX_MARKS || !c->marks[slot]) return fhe_fail(c, FHE_ERR_INVALID, "wait on an unrecorded mark");
  DeviceBind bind(c);
  return fhe_check(c, hipEventSynchronize(c->marks[slot]), "mark wait");
}

int fhe_reserve(fhe_ctx *c, uint32_t max_batch) {
  if (!c) return FHE_ERR_INVALID;
  DeviceBind bind(c);
  max_batch = std::min(max_batch, kCtChunk);  // ops run in passes of at most kCtChunk ciphertexts
  size_t need = (size_t)sizeof(u64) * c->n * max_batch * 2 * c->L;  // rotate / mul scratch
  if (c->K) need += keyswitch_ws_bytes(c, max_batch);
  if (c->K) need = std::max({need, rotate_hoisted_ws_bytes(c, max_batch), rotate_sum_ws_bytes(c, max_batch)});
  if (c->nB) need = std::max(need, bfv_mul_ws_bytes(c, max_batch));
  void *p;
  return ctx_workspace(c, need, &p);
}

int fhe_dev_alloc(fhe_ctx *c, size_t bytes, void **out) {
  if (!c || !out) return FHE_ERR_INVALID;
  DeviceBind bind(c);
  return fhe_check(c, hipMalloc(out, bytes), "hipMalloc");
}
int fhe_dev_free(fhe_ctx *c, void *ptr) {
  if (!c) return FHE_ERR_INVALID;
  DeviceBind bind(c);
  return fhe_check(c, hipFree(ptr), "hipFree");
}
int fhe_memcpy_h2d(fhe_ctx *c, void *dst, const void *src, size_t bytes) {
  if (!c) return FHE_ERR_INVALID;
  DeviceBind bind(c);
  int rc = fhe_check(c, hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->stream), "h2d");
  if (rc) return rc;
  // the host buffer may be reused as soon as this returns (callers stage
  // successive inputs through one pageable buffer)
  return fhe_check(c, hipStreamSynchronize(c->stream), "h2d sync");
}
int fhe_memcpy_d2h(fhe_ctx *c, void *dst, const void *src, size_t bytes) {
  if (!c) return FHE_ERR_INVALID;
  DeviceBind bind(c);
  int rc = fhe_check(c, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c->stream), "d2h");
  if (rc) return rc;
  return fhe_check(c, hipStreamSynchronize(c->stream), "d2h sync");
}

int fhe_host_alloc(fhe_ctx *c, size_t bytes, void **out) {
  if (!c || !out) return FHE_ERR_INVALID;
  DeviceBind bind(c);
  return fhe_check(c, hipHostMalloc(out, bytes, hipHostMallocDefault), "hipHostMalloc");
}
int fhe_host_free(fhe_ctx *c, void *ptr) {
  if (!c) return FHE_ERR_INVALID;
  return fhe_check(c, hipHostFree(ptr), "hipHostFree");
}
int fhe_memcpy_h2d_async(fhe_ctx *c, void *dst, const void *src, size_t bytes) {
  if (!c) return FHE_ERR_INVALID;
  DeviceBind bind(c);
  return fhe_check(c, hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->stream), "h2d async");
}
int fhe_memcpy_d2h_async(fhe_ctx *c, void *dst, const void *src, size_t bytes) {
  if (!c) return FHE_ERR_INVALID;
  DeviceBind bind(c);
  return fhe_check(c, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c->stream), "d2h async");
}
int fhe_memcpy_d2d_async(fhe_ctx *c, void *dst, const void *src, size_t bytes) {
  if (!c) return FHE_ERR_INVALID;
  DeviceBind bind(c);
  return fhe_check(c, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, c->stream), "d2d async");
}
int fhe_use_own_stream(fhe_ctx *c) {
  if (!c) return FHE_ERR_INVALID;
  DeviceBind bind(c);
  if (!c->own_stream) {
    int rc = fhe_check(c, hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking), "stream create");
    if (rc) return rc;
  }
  c->stream = c->own_stream;
  return FHE_OK;
}

// an empty batch (count == 0) is a no-op that accepts null buffers
static int check_range(fhe_ctx *c, const void *p, uint32_t mod_begin, uint32_t n_limbs, uint32_t count) {
  if (!c) return FHE_ERR_INVALID;
  if (n_limbs == 0 || mod_begin + n_limbs > c->nmod) return fhe_fail(c, FHE_ERR_INVALID, "modulus range");
  if (!p && count) return fhe_fail(c, FHE_ERR_INVALID, "null buffer");
  return FHE_OK;
}

int fhe_ntt_fwd(fhe_ctx *c, uint64_t *data, uint32_t n_polys, uint32_t mod_begin, uint32_t n_limbs) {
  int rc = check_range(c, data, mod_begin, n_limbs, n_polys);
  if (rc) return rc;
  DeviceBind bind(c);
  return ntt_launch(c, LimbMap{data, n_limbs, n_limbs, 0, n_limbs, 0, mod_begin, n_polys}, false);
}
int fhe_ntt_inv(fhe_ctx *c, uint64_t *data, uint32_t n_polys, uint32_t mod_begin, uint32_t n_limbs) {
  int rc = check_range(c, data, mod_begin, n_limbs, n_polys);
  if (rc) return rc;
  DeviceBind bind(c);
  return ntt_launch(c, LimbMap{data, n_limbs, n_limbs, 0, n_limbs, 0, mod_begin, n_polys}, true);
}

static int ew(fhe_ctx *c, EwOp op, const uint64_t *a, const uint64_t *b, uint64_t *out, uint32_t n_polys,
              uint32_t mod_begin, uint32_t n_limbs) {
  int rc = check_range(c, a, mod_begin, n_limbs, n_polys);
  if (rc) return rc;
  DeviceBind bind(c);
  if (!n_polys) return FHE_OK;
  if (!b || !out) return fhe_fail(c, FHE_ERR_INVALID, "null buffer");
  return ew_launch(c, op, a, b, out, n_polys, mod_begin, n_limbs);
}
int fhe_poly_add(fhe_ctx *c, const uint64_t *a, const uint64_t *b, uint64_t *out, uint32_t n, uint32_t mb, uint32_t nl) {
  return ew(c, EwOp::Add, a, b, out, n, mb, nl);
}
int fhe_poly_sub(fhe_ctx *c, const uint64_t *a, const uint64_t *b, uint64_t *out, uint32_t n, uint32_t mb, uint32_t nl) {
  return ew(c, EwOp::Sub, a, b, out, n, mb, nl);
}
int fhe_poly_mul(fhe_ctx *c, const uint64_t *a, const uint64_t *b, uint64_t *out, uint32_t n, uint32_t mb, uint32_t nl) {
  return ew(c, EwOp::Mul, a, b, out, n, mb, nl);
}

int fhe_base_conv(fhe_ctx *c, const uint64_t *src, const uint32_t *src_mods, uint32_t n_src, uint64_t *dst,
                  const uint32_t *dst_mods, uint32_t n_dst, uint32_t n) {
  if (!c || !src || !dst || !src_mods || !dst_mods) return fhe_fail(c, FHE_ERR_INVALID, "null argument");
  if (n_src == 0 || n_src > 16 || n_dst == 0 || n_dst > FHE_MAX_MODS)
    return fhe_fail(c, FHE_ERR_INVALID, "conversion sizes");
  std::vector<u32> s(src_mods, src_mods + n_src), d(dst_mods, dst_mods + n_dst);
  for (u32 x : s)
    if (x >= c->nmod) return fhe_fail(c, FHE_ERR_INVALID, "modulus id");
  for (u32 x : d)
    if (x >= c->nmod) return fhe_fail(c, FHE_ERR_INVALID, "modulus id");
  DeviceBind bind(c);
  std::vector<u32> key(s);
  key.push_back(~0u);
  key.insert(key.end(), d.begin(), d.end());
  auto it = c->conv_cache.find(key);
  ConvTab t;
  if (it == c->conv_cache.end()) {
    t = make_conv_tab(c, s, d, 1);
    if (!t.h) return fhe_fail(c, FHE_ERR_OOM, "conv table");
    c->conv_cache.emplace(std::move(key), t);
  } else {
    t = it->second;
  }
  return conv_launch(c, t, src, n_src, dst, n_dst, n);
}

int fhe_fill_uniform(fhe_ctx *c, uint64_t *data, uint32_t n_polys, uint32_t mod_begin, uint32_t n_limbs,
                     uint64_t seed) {
  int rc = check_range(c, data, mod_begin, n_limbs, n_polys);
  if (rc) return rc;
  DeviceBind bind(c);
  return fill_uniform_launch(c, data, n_polys, mod_begin, n_limbs, seed);
}

int fhe_add(fhe_ctx *c, const uint64_t *a, const uint64_t *b, uint64_t *out, uint32_t n_ct) {
  return ew(c, EwOp::Add, a, b, out, 2 * n_ct, 0, c ? c->L : 1);
}
int fhe_sub(fhe_ctx *c, const uint64_t *a, const uint64_t *b, uint64_t *out, uint32_t n_ct) {
  return ew(c, EwOp::Sub, a, b, out, 2 * n_ct, 0, c ? c->L : 1);
}

static int need_ks(fhe_ctx *c, const void *a, const void *k, const void *out, uint32_t n) {
  if (!c) return FHE_ERR_INVALID;
  if (c->K == 0) return fhe_fail(c, FHE_ERR_UNSUPPORTED, "context has no special primes (K = 0)");
  if (n && (!a || !k || !out)) return fhe_fail(c, FHE_ERR_INVALID, "null buffer");
  return FHE_OK;
}

int fhe_mul_relin(fhe_ctx *c, const uint64_t *a, const uint64_t *b, const uint64_t *rlk, uint64_t *out,
                  uint32_t n_ct) {
  int rc = need_ks(c, a, rlk, out, n_ct);
  if (rc) return rc;
  DeviceBind bind(c);
  if (!n_ct) return FHE_OK;
  if (!b) return fhe_fail(c, FHE_ERR_INVALID, "null buffer");
  const size_t cw = (size_t)2 * c->L * c->n;
  for (uint32_t c0 = 0; c0 < n_ct; c0 += kCtChunk) {
    const uint32_t m = std::min(kCtChunk, n_ct - c0);
    const size_t o = c0 * cw;
    rc = c->params.scheme == FHE_SCHEME_BFV ? bfv_mul_relin_impl(c, a + o, b + o, rlk, out + o, m)
                                            : ckks_mul_relin_impl(c, a + o, b + o, rlk, out + o, m);
    if (rc) return rc;
  }
  return FHE_OK;
}

int fhe_keyswitch(fhe_ctx *c, const uint64_t *d, const uint64_t *ksk, uint64_t *out, uint32_t n) {
  int rc = need_ks(c, d, ksk, out, n);
  if (rc) return rc;
  DeviceBind bind(c);
  if (!n) return FHE_OK;
  void *ws;
  if ((rc = ctx_workspace(c, keyswitch_ws_bytes(c, std::min(n, kCtChunk)), &ws))) return rc;
  const size_t LN = (size_t)c->L * c->n;
  for (uint32_t c0 = 0; c0 < n; c0 += kCtChunk) {
    const uint32_t m = std::min(kCtChunk, n - c0);
    rc = keyswitch_ex(c, d + c0 * LN, c->L, ksk, out + c0 * 2 * LN, out + c0 * 2 * LN, m, 0u,
                      c->params.scheme == FHE_SCHEME_CKKS, (u64 *)ws);
    if (rc) return rc;
  }
  return FHE_OK;
}

int fhe_rotate(fhe_ctx *c, const uint64_t *ct, uint32_t g, const uint64_t *gk, uint64_t *out, uint32_t n_ct) {
  int rc = need_ks(c, ct, gk, out, n_ct);
  if (rc) return rc;
  DeviceBind bind(c);
  if ((g & 1) == 0 || g >= 2 * c->n) return fhe_fail(c, FHE_ERR_INVALID, "galois element must be odd and < 2N");
  if (!n_ct) return FHE_OK;
  const size_t cw = (size_t)2 * c->L * c->n;
  for (uint32_t c0 = 0; c0 < n_ct; c0 += kCtChunk) {
    const uint32_t m = std::min(kCtChunk, n_ct - c0);
    if ((rc = rotate_impl(c, ct + c0 * cw, g, gk, out + c0 * cw, m, c->params.scheme == FHE_SCHEME_CKKS))) return rc;
  }
  return FHE_OK;
}

int fhe_rotate_hoisted(fhe_ctx *c, const uint64_t *ct, uint32_t n_rot, const uint32_t *galois,
                       const uint64_t *const *gks, uint64_t *const *outs, uint32_t n_ct) {
  if (!c) return FHE_ERR_INVALID;
  if (c->K == 0) return fhe_fail(c, FHE_ERR_UNSUPPORTED, "context has no special primes (K = 0)");
  if (n_rot && (!galois || !gks || !outs)) return fhe_fail(c, FHE_ERR_INVALID, "null array");
  DeviceBind bind(c);
  const size_t cw = (size_t)2 * c->L * c->n;
  for (uint32_t r = 0; r < n_rot; ++r) {
    const uint32_t g = galois[r];
    if ((g & 1) == 0 || g >= 2 * c->n) return fhe_fail(c, FHE_ERR_INVALID, "galois element must be odd and < 2N");
    if (n_ct && (!gks[r] || !outs[r] || !ct)) return fhe_fail(c, FHE_ERR_INVALID, "null buffer");
    // the combine reads c0 through sigma_g: outs must not overlap ct
    if (n_ct && outs[r] < ct + n_ct * cw && ct < outs[r] + n_ct * cw)
      return fhe_fail(c, FHE_ERR_INVALID, "hoisted rotation output overlaps its input");
    for (uint32_t q = 0; q < r && n_ct; ++q)
      if (outs[r] < outs[q] + n_ct * cw && outs[q] < outs[r] + n_ct * cw)
        return fhe_fail(c, FHE_ERR_INVALID, "hoisted rotation outputs overlap each other");
  }
  if (!n_ct || !n_rot) return FHE_OK;
  std::vector<u64 *> o(n_rot);
  for (uint32_t c0 = 0; c0 < n_ct; c0 += kCtChunk) {
    const uint32_t m = std::min(kCtChunk, n_ct - c0);
    for (uint32_t r = 0; r < n_rot; ++r) o[r] = outs[r] + c0 * cw;
    int rc = rotate_hoisted_impl(c, ct + c0 * cw, n_rot, galois, gks, o.data(), m);
    if (rc) return rc;
  }
  return FHE_OK;
}

static int rot_sum(fhe_ctx *c, const uint64_t *ct, uint32_t n_rot, const uint32_t *galois, const uint64_t *const *gks,
                   const uint64_t *const *pts, uint64_t *out, uint32_t n_ct);
int fhe_rotate_sum_hoisted(fhe_ctx *c, const uint64_t *ct, uint32_t n_rot, const uint32_t *galois,
                           const uint64_t *const *gks, uint64_t *out, uint32_t n_ct) {
  return rot_sum(c, ct, n_rot, galois, gks, nullptr, out, n_ct);
}
int fhe_linear_hoisted(fhe_ctx *c, const uint64_t *ct, uint32_t n_rot, const uint32_t *galois,
                       const uint64_t *const *gks, const uint64_t *const *pts, uint64_t *out, uint32_t n_ct) {
  if (!c) return FHE_ERR_INVALID;
  if (c->params.scheme != FHE_SCHEME_CKKS) return fhe_fail(c, FHE_ERR_UNSUPPORTED, "hoisted linear transforms are CKKS only");
  if (n_ct && n_rot && !pts) return fhe_fail(c, FHE_ERR_INVALID, "null plaintext array");
  for (uint32_t r = 0; n_ct && r < n_rot; ++r)
    if (!pts[r]) return fhe_fail(c, FHE_ERR_INVALID, "null plaintext");
  return rot_sum(c, ct, n_rot, galois, gks, pts, out, n_ct);
}
static int rot_sum(fhe_ctx *c, const uint64_t *ct, uint32_t n_rot, const uint32_t *galois, const uint64_t *const *gks,
                   const uint64_t *const *pts, uint64_t *out, uint32_t n_ct) {
  if (!c) return FHE_ERR_INVALID;
  if (c->K == 0) return fhe_fail(c, FHE_ERR_UNSUPPORTED, "context has no special primes (K = 0)");
  if (!n_ct) return FHE_OK;
  if (!n_rot || !galois || !gks || !ct || !out) return fhe_fail(c, FHE_ERR_INVALID, "null array or no rotations");
  DeviceBind bind(c);
  for (uint32_t r = 0; r < n_rot; ++r) {
    const uint32_t g = galois[r];
    if ((g & 1) == 0 || g >= 2 * c->n) return fhe_fail(c, FHE_ERR_INVALID, "galois element must be odd and < 2N");
    if (!gks[r]) return fhe_fail(c, FHE_ERR_INVALID, "null key");
  }
  const size_t cw = (size_t)2 * c->L * c->n;
  // in place (out == ct) or apart: the work runs in chunks of kCtChunk
  // ciphertexts, and a partly overlapping out would overwrite rows of ct that
  // a later chunk still reads
  if (out != ct && !(out + n_ct * cw <= ct || ct + n_ct * cw <= out))
    return fhe_fail(c, FHE_ERR_INVALID, "rotation sum output partly overlaps its input (use out == ct or apart)");
  for (uint32_t c0 = 0; c0 < n_ct; c0 += kCtChunk) {
    const uint32_t m = std::min(kCtChunk, n_ct - c0);
    int rc = rotate_sum_hoisted_impl(c, ct + c0 * cw, n_rot, galois, gks, out + c0 * cw, m, pts);
    if (rc) return rc;
  }
  return FHE_OK;
}

// ---- CKKS levels: the op of the level-m view, its error reported on c
static int at_level(fhe_ctx *c, uint32_t level, fhe_ctx **v) {
  if (!c) return FHE_ERR_INVALID;
  return ctx_level(c, level, v);
}
static int from_view(fhe_ctx *c, fhe_ctx *v, int rc) {
  if (rc && v != c) c->err = v->err;
  return rc;
}

// BFV ciphertexts live at level L only (ctx_level): the element-wise ops say so too
static int ew_level_ok(fhe_ctx *c, uint32_t level) {
  if (level == 0 || level > c->L) return fhe_fail(c, FHE_ERR_INVALID, "level must be in [1, L]");
  if (c->params.scheme == FHE_SCHEME_BFV && level != c->L)
    return fhe_fail(c, FHE_ERR_UNSUPPORTED, "BFV ciphertexts have no reduced levels (level must be L)");
  return FHE_OK;
}
int fhe_add_at(fhe_ctx *c, const uint64_t *a, const uint64_t *b, uint64_t *out, uint32_t n_ct, uint32_t level) {
  if (!c) return FHE_ERR_INVALID;
  if (int rc = ew_level_ok(c, level)) return rc;
  return ew(c, EwOp::Add, a, b, out, 2 * n_ct, 0, level);
}
int fhe_sub_at(fhe_ctx *c, const uint64_t *a, const uint64_t *b, uint64_t *out, uint32_t n_ct, uint32_t level) {
  if (!c) return FHE_ERR_INVALID;
  if (int rc = ew_level_ok(c, level)) return rc;
  return ew(c, EwOp::Sub, a, b, out, 2 * n_ct, 0, level);
}
int fhe_mul_relin_at(fhe_ctx *c, const uint64_t *a, const uint64_t *b, const uint64_t *rlk, uint64_t *out,
                     uint32_t n_ct, uint32_t level) {
  fhe_ctx *v;
  DeviceBind bind(c);
  int rc = at_level(c, level, &v);
  return rc ? rc : from_view(c, v, fhe_mul_relin(v, a, b, rlk, out, n_ct));
}
int fhe_rotate_at(fhe_ctx *c, const uint64_t *ct, uint32_t g, const uint64_t *gk, uint64_t *out, uint32_t n_ct,
                  uint32_t level) {
  fhe_ctx *v;
  DeviceBind bind(c);
  int rc = at_level(c, level, &v);
  return rc ? rc : from_view(c, v, fhe_rotate(v, ct, g, gk, out, n_ct));
}
int fhe_keyswitch_at(fhe_ctx *c, const uint64_t *d, const uint64_t *ksk, uint64_t *out, uint32_t n,
                     uint32_t level) {
  fhe_ctx *v;
  DeviceBind bind(c);
  int rc = at_level(c, level, &v);
  return rc ? rc : from_view(c, v, fhe_keyswitch(v, d, ksk, out, n));
}

int fhe_rotate_hoisted_at(fhe_ctx *c, const uint64_t *ct, uint32_t n_rot, const uint32_t *galois,
                          const uint64_t *const *gks, uint64_t *const *outs, uint32_t n_ct, uint32_t level) {
  fhe_ctx *v;
  DeviceBind bind(c);
  int rc = at_level(c, level, &v);
  return rc ? rc : from_view(c, v, fhe_rotate_hoisted(v, ct, n_rot, galois, gks, outs, n_ct));
}

int fhe_rotate_sum_hoisted_at(fhe_ctx *c, const uint64_t *ct, uint32_t n_rot, const uint32_t *galois,
                              const uint64_t *const *gks, uint64_t *out, uint32_t n_ct, uint32_t level) {
  fhe_ctx *v;
  DeviceBind bind(c);
  int rc = at_level(c, level, &v);
  return rc ? rc : from_view(c, v, fhe_rotate_sum_hoisted(v, ct, n_rot, galois, gks, out, n_ct));
}

int fhe_linear_hoisted_at(fhe_ctx *c, const uint64_t *ct, uint32_t n_rot, const uint32_t *galois,
                          const uint64_t *const *gks, const uint64_t *const *pts, uint64_t *out, uint32_t n_ct,
                          uint32_t level) {
  fhe_ctx *v;
  DeviceBind bind(c);
  int rc = at_level(c, level, &v);
  return rc ? rc : from_view(c, v, fhe_linear_hoisted(v, ct, n_rot, galois, gks, pts, out, n_ct));
}

int fhe_rescale(fhe_ctx *c, const uint64_t *ct, uint64_t *out, uint32_t n_ct, uint32_t level) {
  if (!c) return FHE_ERR_INVALID;
  if (c->params.scheme != FHE_SCHEME_CKKS) return fhe_fail(c, FHE_ERR_UNSUPPORTED, "rescale is CKKS only");
  if (level < 2 || level > c->L) return fhe_fail(c, FHE_ERR_INVALID, "rescale needs 2 <= level <= L");
  if (!n_ct) return FHE_OK;
  if (!ct || !out) return fhe_fail(c, FHE_ERR_INVALID, "null buffer");
  const size_t N = c->n, in_w = (size_t)2 * level * N, out_w = (size_t)2 * (level - 1) * N;
  const uint64_t *ce = ct + n_ct * in_w, *oe = out + n_ct * out_w;
  if (!(oe <= ct || ce <= out)) return fhe_fail(c, FHE_ERR_INVALID, "rescale output overlaps its input");
  DeviceBind bind(c);
  fhe_ctx *up, *lo;
  int rc = ctx_level(c, level, &up);
  if (!rc) rc = ctx_level(c, level - 1, &lo);
  if (rc) return rc;
  for (uint32_t c0 = 0; c0 < n_ct; c0 += kCtChunk) {
    const uint32_t m = std::min(kCtChunk, n_ct - c0);
    if ((rc = rescale_impl(up, lo, ct + c0 * in_w, out + c0 * out_w, m))) return from_view(c, lo, rc);
  }
  return FHE_OK;
}

int fhe_level_reduce(fhe_ctx *c, const uint64_t *ct, uint64_t *out, uint32_t n_ct, uint32_t level_in,
                     uint32_t level_out) {
  if (!c) return FHE_ERR_INVALID;
  if (c->params.scheme != FHE_SCHEME_CKKS) return fhe_fail(c, FHE_ERR_UNSUPPORTED, "level reduce is CKKS only");
  if (level_in > c->L || level_out == 0 || level_out >= level_in)
    return fhe_fail(c, FHE_ERR_INVALID, "level reduce needs 1 <= level_out < level_in <= L");
  if (!n_ct) return FHE_OK;
  if (!ct || !out) return fhe_fail(c, FHE_ERR_INVALID, "null buffer");
  const size_t N = c->n, in_w = (size_t)2 * level_in * N, out_w = (size_t)2 * level_out * N;
  if (!(out + n_ct * out_w <= ct || ct + n_ct * in_w <= out))
    return fhe_fail(c, FHE_ERR_INVALID, "level reduce output overlaps its input");
  DeviceBind bind(c);
  // one strided copy: 2 n_ct rows of level_out limbs, source pitch level_in limbs
  return fhe_check(c, hipMemcpy2DAsync(out, level_out * N * 8, ct, level_in * N * 8, level_out * N * 8,
                                       (size_t)2 * n_ct, hipMemcpyDeviceToDevice, c->stream),
                   "level reduce");
}

int fhe_galois_elt(const fhe_ctx *c, int32_t steps, uint32_t *out) {
  if (!c || !out) return FHE_ERR_INVALID;
  const int64_t ord = c->n / 2;
  int64_t s = steps % ord;
  if (s < 0) s += ord;
  *out = (u32)hpow(5, (u64)s, 2ull * c->n);
  return FHE_OK;
}

static int combine(fhe_ctx *c, int op, uint64_t *a, const uint64_t *b, const uint64_t *rlk, uint32_t n) {
  return op == FHE_REDUCE_ADD ? fhe_add(c, a, b, a, n) : fhe_mul_relin(c, a, b, rlk, a, n);
}

int fhe_reduce(fhe_ctx *c, uint64_t *cts, uint32_t n_ct, int op, const uint64_t *rlk, uint64_t *out) {
  if (!c) return FHE_ERR_INVALID;
  DeviceBind bind(c);
  if (!cts || !out) return fhe_fail(c, FHE_ERR_INVALID, "null buffer");
  if (op != FHE_REDUCE_ADD && op != FHE_REDUCE_MUL_RELIN) return fhe_fail(c, FHE_ERR_INVALID, "reduce op");
  if (op == FHE_REDUCE_MUL_RELIN && !rlk) return fhe_fail(c, FHE_ERR_INVALID, "reduce MUL_RELIN needs rlk");
  if (n_ct == 0) return fhe_fail(c, FHE_ERR_INVALID, "reduce over no ciphertexts");
  const size_t cw = (size_t)2 * c->L * c->n;
  for (uint32_t live = n_ct; live > 1;) {
    const uint32_t half = live / 2;
    int rc = combine(c, op, cts, cts + (size_t)(live - half) * cw, rlk, half);
    if (rc) return rc;
    live -= half;
  }
  if (out != cts) return fhe_check(c, hipMemcpyAsync(out, cts, cw * 8, hipMemcpyDeviceToDevice, c->stream), "copy");
  return FHE_OK;
}

int fhe_reduce_at(fhe_ctx *c, uint64_t *cts, uint32_t n_ct, int op, const uint64_t *rlk, uint64_t *out,
                  uint32_t level) {
  fhe_ctx *v;
  DeviceBind bind(c);
  int rc = at_level(c, level, &v);
  return rc ? rc : from_view(c, v, fhe_reduce(v, cts, n_ct, op, rlk, out));
}

int fhe_reduce_schedule(int rank, int world, int root, int32_t *steps, int cap) {
  if (world < 1 || rank < 0 || rank >= world || root < 0 || root >= world || (!steps && cap > 0)) return FHE_ERR_INVALID;
  const int rel = (rank - root + world) % world;
  int n = 0;
  for (int s = 1; s < world; s <<= 1) {
    if (rel % (2 * s) == s) {  // send the partial result one level up, then stop
      if (n >= cap) return FHE_ERR_INVALID;
      steps[n++] = -(((rel - s + root) % world) + 1);
      break;
    }
    if (rel % (2 * s) == 0 && rel + s < world) {
      if (n >= cap) return FHE_ERR_INVALID;
      steps[n++] = ((rel + s + root) % world) + 1;
    }
  }
  return n;
}

int fhe_reduce_ranks_at(fhe_ctx *c, uint64_t *ct, int op, const uint64_t *rlk, void *comm, int root, uint64_t *tmp,
                        uint32_t level) {
  fhe_ctx *v;
  DeviceBind bind(c);
  int rc = at_level(c, level, &v);
  return rc ? rc : from_view(c, v, fhe_reduce_ranks(v, ct, op, rlk, comm, root, tmp));
}

int fhe_reduce_ranks(fhe_ctx *c, uint64_t *ct, int op, const uint64_t *rlk, void *comm, int root, uint64_t *tmp) {
  if (!c) return FHE_ERR_INVALID;
  DeviceBind bind(c);
  if (!ct || !comm || !tmp) return fhe_fail(c, FHE_ERR_INVALID, "null argument");
  if (op != FHE_REDUCE_ADD && op != FHE_REDUCE_MUL_RELIN) return fhe_fail(c, FHE_ERR_INVALID, "reduce op");
  if (op == FHE_REDUCE_MUL_RELIN && !rlk) return fhe_fail(c, FHE_ERR_INVALID, "reduce MUL_RELIN needs rlk");
  int rank = 0, world = 1;
  if (ncclCommUserRank((ncclComm_t)comm, &rank) != ncclSuccess || ncclCommCount((ncclComm_t)comm, &world) != ncclSuccess)
    return fhe_fail(c, FHE_ERR_DEVICE, "RCCL communicator query");
  int32_t steps[32];
  const int n = fhe_reduce_schedule(rank, world, root, steps, 32);
  if (n < 0) return fhe_fail(c, FHE_ERR_INVALID, "reduce schedule (root / world)");
  const size_t cw = (size_t)2 * c->L * c->n;
  for (int i = 0; i < n; ++i) {
    ncclResult_t r;
    if (steps[i] > 0) {
      r = ncclRecv(tmp, cw, ncclUint64, steps[i] - 1, (ncclComm_t)comm, c->stream);
      if (r != ncclSuccess) return fhe_fail(c, FHE_ERR_DEVICE, std::string("ncclRecv: ") + ncclGetErrorString(r));
      const int rc = combine(c, op, ct, tmp, rlk, 1);
      if (rc) return rc;
    } else {
      r = ncclSend(ct, cw, ncclUint64, -steps[i] - 1, (ncclComm_t)comm, c->stream);
      if (r != ncclSuccess) return fhe_fail(c, FHE_ERR_DEVICE, std::string("ncclSend: ") + ncclGetErrorString(r));
    }
  }
  return FHE_OK;
}

int fhe_bcast_key(fhe_ctx *c, uint64_t *key, size_t words, void *comm, int root) {
  if (!c || !key || !comm) return fhe_fail(c, FHE_ERR_INVALID, "null argument");
  DeviceBind bind(c);
  ncclResult_t r = ncclBroadcast(key, key, words, ncclUint64, root, (ncclComm_t)comm, c->stream);
  if (r != ncclSuccess) return fhe_fail(c, FHE_ERR_DEVICE, std::string("ncclBroadcast: ") + ncclGetErrorString(r));
  return FHE_OK;
}

}  // extern "C"
