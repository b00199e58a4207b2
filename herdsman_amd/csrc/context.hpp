// context.hpp -- internal state behind the fhe_ctx handle of fhe_backend.h.
#pragma once
#include <hip/hip_runtime.h>

#include <map>
#include <string>
#include <vector>

#include "../../include/plugins/fhe_backend.h"
#include "modarith.hpp"

#define FHE_MAX_MODS 48
#define FHE_MAX_CONV_SRC 16
#define FHE_ROT_BATCH 8  // Galois elements per launch of the rotation-batched gather passes

// gridDim.y of the per-coefficient kernels holds (item, limb); every launch
// keeps it below this bound
constexpr u32 kMaxGridY = 65535;
// ciphertext ops run over batches of at most this many ciphertexts per internal
// pass: every grid's y-dimension stays below kMaxGridY (2 L <= 94 rows per
// ciphertext) and the key-switch scratch stays bounded (29 GiB at N=2^16, L=12)
constexpr u32 kCtChunk = 512;

// A batch of limb-polynomials inside a [poly][poly_stride][N] buffer: active
// limb a of poly p is limb `first + (a < skip_lo ? a : a + skip_len)` and uses
// modulus `mod_offset + limb`.  Covers whole polys, Q- or P-parts and the
// "all limbs except this digit" sets of ModUp.
struct LimbMap {
  u64 *base;
  u32 poly_stride;
  u32 cnt;
  u32 first;
  u32 skip_lo;
  u32 skip_len;
  u32 mod_offset;
  u32 n_polys;
};

__host__ __device__ __forceinline__ u32 limbmap_limb(const LimbMap &m, u32 act) {
  return m.first + (act < m.skip_lo ? act : act + m.skip_len);
}

// Fast base conversion table (device): src moduli -> dst moduli, Montgomery
// pre-scaled:  v_i = mont_mul(x_i, hinv[i]) = [x_i (S/s_i)^-1]_{s_i} exactly,
// y_m = mont_reduce(sum_i v_i h[i][m]) = (sum_i v_i (S/s_i)) * R^(e-1) mod d_m
// where h = (S/s_i) * R^e (e = 1: plain result, e = 2: result times R).
struct ConvTab {
  u32 ns, nd;
  const u32 *src_mod; // [ns] modulus ids of the sources
  const u32 *dst_mod; // [nd] modulus ids of the destinations
  const u64 *hinv;    // [ns] (S/s_i)^-1 * R mod s_i
  const u64 *h;       // [ns][nd] (S/s_i) * R^e mod d_m
};

struct fhe_ctx {
  fhe_params params{};
  int device = 0;
  hipStream_t stream = nullptr;
  hipStream_t own_stream = nullptr;  // fhe_use_own_stream
  std::string err;
  u32 log_n = 0, n = 0, L = 0, K = 0, dnum = 0, alpha = 0, nB = 0, nmod = 0;
  u64 t = 0;
  bool special = false;        // every modulus = 1 mod 2^32 (fast Montgomery)
  // CKKS: the ModUp / ModDown conversion constants carry N^-1, so the inverse
  // NTTs that feed them (INTT(d), INTT(acc_P)) skip their scaling
  bool fold_ninv = false;
  std::vector<u64> moduli;
  // device-resident tables (constants in Montgomery form, x * 2^64 mod q)
  ModInfo *d_mods = nullptr;   // [nmod]
  u64 *d_tw_fwd = nullptr;     // [nmod][N]  psi^brv(i) R
  u64 *d_tw_inv = nullptr;     // [nmod][N]  psi^-brv(i) R
  u64 *d_ninv = nullptr;       // [nmod]     N^-1 R
  u64 *d_pinv = nullptr;       // [L]        P^-1 R mod q_i
  u64 *d_pr2 = nullptr;        // [L]        P R^2 mod q_i (the fused finish folds its base into acc as base P)
  u64 *d_r2 = nullptr;         // [nmod]     R^2 mod q (x -> x R)
  ConvTab *d_modup = nullptr;  // device array [ceil(L/alpha)], h scaled by R^2
  ConvTab moddown{};           // P -> Q, h scaled by R
  // per-modulus INTT output constants for conversions fused into the next
  // NTT (CKKS, 2^15 <= N, K <= 4): P limbs N^-1 (P/p_k)^-1 R, so INTT(acc_P)
  // emits ModDown's canonical v_k directly (ntt_fwd_combine_launch PRO_CONV);
  // with fuse_modup also Q limbs N^-1 (Q_j/q_i)^-1 R (q_i in digit j), so the
  // INTT of the key-switch input emits ModUp's v_i (ntt_fwd_modup_launch)
  u64 *d_iscale = nullptr;     // [nmod]
  u64 *d_iscale_t = nullptr;   // [nmod] d_iscale times R: INTT(d2) of the split tensor product (PRO_TENSOR2 forms d2 R^-1)
  bool fuse_moddown = false;
  bool fuse_modup = false;     // also alpha <= 4
  // BFV relinearisation at two-pass sizes (alpha, K, digits <= 4): ModUp in the
  // NTT column pass, the inner product in INTT(acc)'s first pass, ModDown and
  // the combine in one coefficient-domain kernel (bfv_ks_fused)
  bool bfv_ks_fuse = false;
  u64 *d_bfv_dscale = nullptr;  // [L] (Q_j/q_i)^-1 R: the floor writes ModUp's scaled sources
  u64 *d_bfv_kscale = nullptr;  // [nmod] INTT(acc) output constants: N^-1 (Q), N^-1 (P/p_k)^-1 (P), Montgomery
  std::vector<ConvTab> modup_tabs;  // host copies of d_modup (device pointers inside)
  // the fused key switch (ntt_ksf.hip) accumulates at the scale R^-2, which
  // saves the own digit's R^3 product: ModUp's Q targets come out times R^-1
  // (its P targets times R, as modup_tabs), ModDown's times R^-2, and the
  // finish multiplies by P^-1 R^3; the own digit's base takes P and P R^-1
  std::vector<ConvTab> modup_tabs_ksf;
  ConvTab moddown_ksf{};
  u64 *d_pinv3 = nullptr;  // [L] P^-1 R^3 mod q_i
  u64 *d_pplain = nullptr; // [L] P mod q_i
  u64 *d_pm1 = nullptr;    // [L] P R^-1 mod q_i
  std::vector<void *> blobs;   // device allocations owned by the context
  void *behz = nullptr;        // BEHZ device constants (BFV)
  void *hps = nullptr;         // HPS device constants (BFV with FHE_FLAG_BFV_HPS): BFV mul uses HPS
  // fhe_base_conv tables by (src ids, ~0, dst ids); their device arrays are
  // blobs of this context, so they are freed with it
  std::map<std::vector<u32>, ConvTab> conv_cache;
  // scratch
  void *ws = nullptr;
  size_t ws_bytes = 0;
  // fhe_mark / fhe_wait_mark events, created on first use
  hipEvent_t marks[FHE_MAX_MARKS] = {};
  // ---- CKKS levels (fhe_*_at, fhe_rescale).  A ciphertext at level m < L has
  // the first m Q limbs; its ops run on a LEVEL VIEW: a context over the moduli
  // Q_m u P (index space [0,m) = Q_m, [m,m+K) = P) with the parent's alpha, so
  // the digits partition the m active limbs (the last one possibly partial).
  // Views are built on first use, share the parent's stream and workspace and
  // are destroyed with it.  Switching keys stay in the full-level layout
  // [dnum][2][L+K][N]: view limb i reads key row i (Q) or i + key_pshift (P).
  fhe_ctx *parent = nullptr;
  std::vector<fhe_ctx *> views;  // [m] = view at level m (1 <= m < L), null until used
  u32 key_qp = 0;                // key rows per digit half (0: L + K)
  u32 key_pshift = 0;            // L_parent - m for a view
  u64 *d_qdrop = nullptr;        // view at level m: [2m] = q_m^-1 R mod q_i, then q_m mod q_i (rescale m+1 -> m)
  ConvTab lift{};                // view at level m: the 1-source "conversion" of the rescale lift, h = R mod q_i
};

// key layout of a context (level views read the parent's full-level keys)
inline u32 ctx_key_qp(const fhe_ctx *c) { return c->key_qp ? c->key_qp : c->L + c->K; }
// *out = the context of level m (1 <= m <= L): c's root itself for m = L, else
// its view (built on first use); an FHE_ERR_* code with c->err set on failure
int ctx_level(fhe_ctx *c, u32 m, fhe_ctx **out);

// Binds the context's device for the duration of an ABI call and restores the
// caller's current device: a host thread may drive contexts on several GPUs,
// and workspace allocations / null-stream launches follow the current device.
struct DeviceBind {
  int prev = -1;
  explicit DeviceBind(const fhe_ctx *c) {
    if (c && hipGetDevice(&prev) == hipSuccess && prev != c->device) (void)hipSetDevice(c->device);
    else prev = -1;
  }
  ~DeviceBind() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
  DeviceBind(const DeviceBind &) = delete;
  DeviceBind &operator=(const DeviceBind &) = delete;
};

// The same for a bare device id (context creation and destruction).
struct DeviceIdBind {
  int prev = -1;
  bool ok = true;  // dev is the current device (fhe_ctx_create fails with FHE_ERR_DEVICE otherwise)
  explicit DeviceIdBind(int dev) {
    int cur = -1;
    if (hipGetDevice(&cur) != hipSuccess) {
      ok = hipSetDevice(dev) == hipSuccess;  // nothing to restore
      return;
    }
    if (cur == dev) return;
    ok = hipSetDevice(dev) == hipSuccess;
    if (ok) prev = cur;
  }
  ~DeviceIdBind() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
  DeviceIdBind(const DeviceIdBind &) = delete;
  DeviceIdBind &operator=(const DeviceIdBind &) = delete;
};

// helpers shared by the translation units (fhe_backend.cpp)
int fhe_fail(fhe_ctx *c, int code, const std::string &msg);
int fhe_check(fhe_ctx *c, hipError_t e, const char *what);
void *ctx_upload(fhe_ctx *c, const void *host, size_t bytes);  // owned blob
int ctx_workspace(fhe_ctx *c, size_t bytes, void **out);
// r_exp_q: the exponent for targets among the Q limbs (index < L) instead
// (kNoExp: r_exp for every target); negative exponents scale by R^-1
constexpr int kNoExp = 1000;
ConvTab make_conv_tab(fhe_ctx *c, const std::vector<u32> &src, const std::vector<u32> &dst, int r_exp,
                      bool fold_ninv = false, int r_exp_q = kNoExp);
// host modular helpers
u64 host_mulmod(u64 a, u64 b, u64 q);
u64 host_inv(u64 a, u64 q);
u64 host_to_mont(u64 x, u64 q);  // x * 2^64 mod q

// NTT (ntt.hip)
// noscale (inverse): no N^-1 multiply; lazy_out (forward): outputs below 8q, not canonical
// scale (inverse): per-modulus output constants replacing N^-1 (d_iscale)
// src (forward): read the input from src (same layout as m.base) instead of in place
int ntt_launch(fhe_ctx *c, const LimbMap &m, bool inverse, bool noscale = false, bool lazy_out = false,
               const u64 *scale = nullptr, const u64 *src = nullptr);
// pro: the ModDown conversion of acc's P limbs (scaled by d_iscale) fused into
// the column pass (PRO_CONV); null = conv already holds the converted limbs
// ext / ksk: acc's Q limbs are the key-switching inner product of ext [n][ndig][QP][N]
// with ksk [ndig][2][QP][N], formed in the last pass instead of read (EPI_KSQ)
// pinv: the epilogue's per-limb constant (null: P^-1, d_pinv; rescale: q_last^-1, d_qdrop)
// pro_src: the prologue's sources (null: acc's P limbs, ModDown); rescale passes
// the dropped limb with its central-lift constants
struct ConvSrc {
  const u64 *src;      // [n_polys][stride][N]
  u32 stride, first;
  u64 lift_half;       // 0: plain conversion
  const u64 *lift_sub;  // [nd] device
};
// CKKS mul+relin with the tensor product split (EPI_KSQT): the base of the
// ModDown finish is formed from the ciphertexts a, b [n][2][L][N] themselves
struct TensorSrc {
  const u64 *a, *b;
  bool fused;  // the whole finish in one kernel (ntt_ks_fused_finish_launch); ModUp skips its Q row passes
  u32 g = 0;   // fused only: a CKKS rotation by g instead (a = the ciphertexts, read through sigma_g; b unused)
  bool convf = false;  // fused only: ModUp and ModDown as CONVF launches (dc holds INTT(d2)'s row-pass output)
};
// Hoisted rotations of few ciphertexts: nr Galois elements' gather passes in
// one launch (poly p of the batch = rotation p / (2 n), ciphertext poly p % (2 n))
struct RotBatch {
  u32 nr;
  const u64 *ksk[FHE_ROT_BATCH];
  u64 *out[FHE_ROT_BATCH];
  u32 g[FHE_ROT_BATCH];
};
int ntt_fwd_combine_launch(fhe_ctx *c, u64 *conv, u32 n_polys, const u64 *acc, u32 acc_stride, const u64 *base,
                           u64 *out, u32 add_mask, const ConvTab *pro = nullptr, const u64 *ext = nullptr,
                           const u64 *ksk = nullptr, u32 ndig = 0, u32 base_g = 0, const u64 *pinv = nullptr,
                           const ConvSrc *pro_src = nullptr, u32 ext_g = 0, const RotBatch *rb = nullptr,
                           const TensorSrc *tsrc = nullptr);
// ModUp of digit j fused into the column pass of the forward NTT of its
// converted limbs (PRO_CONV; sources = dc's digit limbs, scaled by the INTT
// through d_iscale); ext_j [n][ndig*QP][N] slots outside the digit receive
// the lazy (< 8q) NTT outputs times R
// (q_rows false: every target keeps its column-pass output, for the fused key switch)
// ksf_scale (q_rows false only): the Q targets at the fused CKKS finish's
// scale (modup_tabs_ksf); else every target times R (modup_tabs; BFV)
int ntt_fwd_modup_launch(fhe_ctx *c, const u64 *dc, u64 *ext, u32 n, u32 ndig, u32 j, bool q_rows = true,
                         bool ksf_scale = true, const u64 *src_rows_scale = nullptr);
int ntt_inv_bfv_tensor_launch(fhe_ctx *c, const u64 *xa, const u64 *xb, u64 *e, u32 nl, u32 mod_offset, u32 n);
// INTT(acc_P) with the P limbs' key-switching inner product in its first pass
// (ext_g != 0: ext is read as sigma_g(ext), the hoisted rotation's inner product)
// (all_limbs: every Q u P limb with the output constants d_bfv_kscale, BFV)
int ntt_inv_ksp_launch(fhe_ctx *c, u64 *acc, const u64 *ext, const u64 *ksk, u32 n, u32 ndig, u32 ext_g = 0,
                       bool all_limbs = false, const RotBatch *rb = nullptr);
// (base null: sigma(c0) is not stored; the combine then reads it with base_g)
int ntt_inv_automorph_launch(fhe_ctx *c, const u64 *ct, u32 g, u64 *base, u64 *dc, u64 *ext, u32 n, u32 ndig);
// the fused key-switch finish of CKKS mul+relin (ntt_ksf.hip): the row
// transforms of the non-own ModUp digits' Q limbs and of NTT(conv), the inner
// product and the ModDown finish in one workgroup per (limb, ct, row block)
bool ks_fused_finish_ok(const fhe_ctx *c, u32 ndig);
// (g != 0: the rotation's finish, ta = the ciphertexts read through sigma_g, tb unused)
// ntt_ksp_fused_launch: the P side -- the P limbs' ModUp row transforms, their
// inner product and INTT(acc_P) (acc's P rows as ntt_inv_ksp_launch leaves them)
// (all_limbs: BFV -- every Q u P limb, each digit's column-pass intermediates
// own limbs included, INTT output constants d_bfv_kscale)
int ntt_ksp_fused_launch(fhe_ctx *c, u64 *acc, const u64 *ext, const u64 *ksk, u32 n, u32 ndig,
                         bool all_limbs = false, bool skip_col = false);
// CONVF (ntt_convf.hip): an inverse NTT's column pass (sources: its row pass's
// output, scaled on the way out), a base conversion and the forward column
// pass of every target, in one kernel per (column block, poly)
struct ConvfArgs {
  const u64 *src;                        // [n_polys][src_stride][N] the inverse's row-pass output
  u32 src_stride, src_first, src_mod0;   // source limb i: src_first + i, modulus src_mod0 + i
  const u64 *scale;                      // per modulus: the inverse's output scale
  LimbMap tmap;                          // the targets (their forward column-pass outputs)
  const u64 *h;                          // the conversion table (ConvTab::h, nd targets)
  u32 nd, src60;
  const ModInfo *mods;
  const u64 *twi, *twf;
};
bool convf_ok(const fhe_ctx *c, u32 ns);
int ntt_convf_launch(fhe_ctx *c, const ConvfArgs &a, u32 ns);
// the BFV key switch without a stored ext applies (ntt_ksf.hip)
bool bfv_ks_extfree_ok(const fhe_ctx *c, u32 ndig);
// the first (column) pass of a forward NTT alone (two-pass sizes): its
// intermediate for a fused consumer that runs the row transforms itself
int ntt_fwd_col_launch(fhe_ctx *c, const LimbMap &m, const u64 *src = nullptr);
// BFV mul: the forward row passes, the tensor product and the inverse row
// passes of Q or Bsk in one kernel, then the inverse column pass (ntt_bfvt.hip)
bool bfvt_fused_ok(const fhe_ctx *c);
int ntt_bfv_tensor_fused_launch(fhe_ctx *c, const u64 *xa, const u64 *xb, u64 *e, u32 nl, u32 mod_offset, u32 n);
int ntt_ks_fused_finish_launch(fhe_ctx *c, const u64 *conv, const u64 *ext, const u64 *ksk, u32 ndig,
                               const u64 *ta, const u64 *tb, u64 *out, u32 n, u32 g = 0);
// d2_only (PRO_TENSOR2, two-pass sizes): out is not written; the ModDown
// finish forms d0 and d1 (ntt_fwd_combine_launch with a TensorSrc)
int ntt_inv_tensor_launch(fhe_ctx *c, const u64 *a, const u64 *b, u64 *out, u64 *dc, u64 *ext, u32 n, u32 ndig,
                          bool d2_only = false, bool rows_only = false);
// RNS kernels (rns.hip)
enum class EwOp { Add, Sub, Mul };
int ew_launch(fhe_ctx *c, EwOp op, const u64 *a, const u64 *b, u64 *out, u32 n_polys, u32 mod_begin, u32 n_limbs);
int conv_launch(fhe_ctx *c, const ConvTab &t, const u64 *src, u32 src_poly_stride, u64 *dst,
                u32 dst_poly_stride, u32 n);
int fill_uniform_launch(fhe_ctx *c, u64 *data, u32 n_polys, u32 mod_begin, u32 n_limbs, u64 seed);
int keyswitch_ex(fhe_ctx *c, const u64 *d, u32 d_stride, const u64 *ksk, const u64 *base, u64 *out, u32 n,
                 u32 add_mask, bool ntt_form, u64 *ws);
int ckks_mul_relin_impl(fhe_ctx *c, const u64 *a, const u64 *b, const u64 *rlk, u64 *out, u32 n);
int rotate_impl(fhe_ctx *c, const u64 *ct, u32 g, const u64 *gk, u64 *out, u32 n, bool ntt_form);
// CKKS hoisted rotations: one ModUp of c1 serves n_rot Galois elements
// (outs[r] [n][2][L][N], apart from ct; gks[r] device keys)
int rotate_hoisted_impl(fhe_ctx *c, const u64 *ct, u32 n_rot, const u32 *galois, const u64 *const *gks,
                        u64 *const *outs, u32 n);
size_t rotate_hoisted_ws_bytes(const fhe_ctx *c, u32 n);
// double-hoisted rotation sum: out [n][2][L][N] = sum_r rot_{g_r}(ct), one ModDown
// (pts: the hoisted linear transform sum_r pts[r] (.) rot_r(ct), CKKS; null: plain sum)
int rotate_sum_hoisted_impl(fhe_ctx *c, const u64 *ct, u32 n_rot, const u32 *galois, const u64 *const *gks, u64 *out,
                            u32 n, const u64 *const *pts = nullptr);
size_t rotate_sum_ws_bytes(const fhe_ctx *c, u32 n);
// CKKS rescale of n ciphertexts of level m + 1 (on `up`, the context of level
// m + 1) to level m (on `lo`, the context of level m); ct must not overlap out
int rescale_impl(fhe_ctx *up, fhe_ctx *lo, const u64 *ct, u64 *out, u32 n);
size_t rescale_ws_bytes(const fhe_ctx *lo, u32 n);
int bfv_mul_relin_impl(fhe_ctx *c, const u64 *a, const u64 *b, const u64 *rlk, u64 *out, u32 n_ct);
int behz_setup(fhe_ctx *c);
int hps_setup(fhe_ctx *c);
size_t keyswitch_ws_bytes(const fhe_ctx *c, u32 n);
size_t bfv_mul_ws_bytes(const fhe_ctx *c, u32 n);
