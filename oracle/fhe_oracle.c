/*
 * fhe_oracle.c -- CPU ORACLE (test infrastructure only; see fhe_oracle.h).
 *
 * Plain-C restatement of the RNS arithmetic the herdsman FHE backend must
 * reproduce bit-for-bit.  herdsman itself holds no such code (SURVEY.md §0,
 * §8c: /root/reference has no NTT/RNS/keyswitch; OpenFHE is linked at
 * /root/reference/CMakeLists.txt:73,210-211 but never called), so every
 * function below cites the published algorithm it restates instead of a
 * reference file:line:
 *   - NTT: Harvey, "Faster arithmetic for number-theoretic transforms"
 *     (2014), negacyclic Cooley-Tukey forward / Gentleman-Sande inverse with
 *     psi^brv twiddles and Shoup multiplication (the SEAL/OpenFHE layout);
 *   - fast base conversion / hybrid key switching: Han-Ki (CT-RSA 2020),
 *     Bossuat et al. (Eurocrypt 2021) "ModUp / ModDown";
 *   - BFV multiplication: Bajard-Eynard-Hasan-Zucca (SAC 2016), in the form
 *     of SEAL's RNSTool (fastbconv_m_tilde, sm_mrq, fast_floor,
 *     fastbconv_sk).
 * Pinned by tests/golden/ (generated from oracle/bigint_model.py).
 */
#include "fhe_oracle.h"

#include <stdlib.h>
#include <string.h>
#include <stdio.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef unsigned __int128 u128;
#define MAXM 48

typedef struct {
  uint64_t q;
  uint64_t psi;
  uint64_t *w;      /* psi^brv(i), i in [0,N) */
  uint64_t *ws;     /* Shoup companions */
  uint64_t *iw;     /* psi^-brv(i) */
  uint64_t *iws;
  uint64_t ninv, ninvs;
} orc_mod;

struct orc_ctx {
  uint32_t scheme, log_n, n, L, K, dnum, alpha, nB; /* nB = |Bsk| (BFV) */
  uint32_t bfv_mult;                                /* ORC_BFV_BEHZ or ORC_BFV_HPS */
  uint64_t t;
  uint32_t nmod;
  orc_mod m[MAXM];
};

/* ------------------------------------------------------------ arithmetic */
static inline uint64_t mulmod(uint64_t a, uint64_t b, uint64_t q) {
  return (uint64_t)(((u128)a * b) % q);
}
static inline uint64_t addmod(uint64_t a, uint64_t b, uint64_t q) {
  uint64_t s = a + b;
  return s >= q ? s - q : s;
}
static inline uint64_t submod(uint64_t a, uint64_t b, uint64_t q) {
  return a >= b ? a - b : a + q - b;
}
static uint64_t powmod(uint64_t b, uint64_t e, uint64_t q) {
  uint64_t r = 1 % q;
  b %= q;
  while (e) {
    if (e & 1) r = mulmod(r, b, q);
    b = mulmod(b, b, q);
    e >>= 1;
  }
  return r;
}
/* q prime -> inverse via Fermat */
static uint64_t invmod(uint64_t a, uint64_t q) { return powmod(a % q, q - 2, q); }
static inline uint64_t shoup_pre(uint64_t w, uint64_t q) {
  return (uint64_t)(((u128)w << 64) / q);
}
/* Shoup: w*a mod q for any a < 2^64, result canonical */
static inline uint64_t shoup_mul(uint64_t a, uint64_t w, uint64_t ws, uint64_t q) {
  uint64_t qh = (uint64_t)(((u128)a * ws) >> 64);
  uint64_t r = a * w - qh * q;
  return r >= q ? r - q : r;
}
static inline uint32_t brv(uint32_t x, uint32_t bits) {
  uint32_t r = 0;
  for (uint32_t i = 0; i < bits; ++i) { r = (r << 1) | (x & 1); x >>= 1; }
  return r;
}

static int is_prime_u64(uint64_t n) {
  static const uint64_t bases[] = {2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37};
  if (n < 2) return 0;
  for (int i = 0; i < 12; ++i) {
    if (n == bases[i]) return 1;
    if (n % bases[i] == 0) return 0;
  }
  uint64_t d = n - 1; int s = 0;
  while (!(d & 1)) { d >>= 1; ++s; }
  for (int i = 0; i < 12; ++i) {
    uint64_t x = powmod(bases[i], d, n);
    if (x == 1 || x == n - 1) continue;
    int comp = 1;
    for (int r = 1; r < s; ++r) {
      x = mulmod(x, x, n);
      if (x == n - 1) { comp = 0; break; }
    }
    if (comp) return 0;
  }
  return 1;
}

uint32_t orc_gen_primes(uint32_t bits, uint32_t log_n, uint32_t count, const uint64_t *excl,
                        uint32_t n_excl, uint64_t *out) {
  /* The backend's prime family: q = k * 2^32 + 1 < 2^bits, descending.
   * q = 1 mod 2^32 implies q = 1 mod 2N for every N <= 2^31. */
  (void)log_n;
  const uint64_t step = 1ull << 32;
  uint64_t k = ((bits >= 64 ? ~0ull : (1ull << bits)) - 2) / step;
  uint32_t got = 0;
  for (; k > 0 && got < count; --k) {
    uint64_t q = k * step + 1;
    int skip = 0;
    for (uint32_t e = 0; e < n_excl; ++e) if (excl[e] == q) skip = 1;
    for (uint32_t e = 0; e < got; ++e) if (out[e] == q) skip = 1;
    if (!skip && is_prime_u64(q)) out[got++] = q;
  }
  return got;
}

/* smallest primitive 2N-th root of unity mod q */
static uint64_t min_psi(uint64_t q, uint32_t log_n) {
  uint64_t n = 1ull << log_n, two_n = 2 * n;
  uint64_t g = 0;
  for (uint64_t x = 2; x < q; ++x) {
    g = powmod(x, (q - 1) / two_n, q);
    if (powmod(g, n, q) == q - 1) break;
  }
  uint64_t g2 = mulmod(g, g, q), best = g, cur = g;
  for (uint64_t k = 1; k < n; ++k) {
    cur = mulmod(cur, g2, q);
    if (cur < best) best = cur;
  }
  return best;
}

static void mod_init(orc_mod *m, uint64_t q, uint32_t log_n) {
  uint32_t n = 1u << log_n;
  m->q = q;
  m->psi = min_psi(q, log_n);
  uint64_t ipsi = invmod(m->psi, q);
  m->w = malloc(sizeof(uint64_t) * n); m->ws = malloc(sizeof(uint64_t) * n);
  m->iw = malloc(sizeof(uint64_t) * n); m->iws = malloc(sizeof(uint64_t) * n);
  uint64_t p = 1, ip = 1;
  uint64_t *pw = malloc(sizeof(uint64_t) * n), *ipw = malloc(sizeof(uint64_t) * n);
  for (uint32_t i = 0; i < n; ++i) { pw[i] = p; ipw[i] = ip; p = mulmod(p, m->psi, q); ip = mulmod(ip, ipsi, q); }
  for (uint32_t i = 0; i < n; ++i) {
    uint32_t r = brv(i, log_n);
    m->w[i] = pw[r]; m->ws[i] = shoup_pre(pw[r], q);
    m->iw[i] = ipw[r]; m->iws[i] = shoup_pre(ipw[r], q);
  }
  free(pw); free(ipw);
  m->ninv = invmod(n, q); m->ninvs = shoup_pre(m->ninv, q);
}

void orc_set_threads(int n) {
#ifdef _OPENMP
  omp_set_num_threads(n);
#else
  (void)n;
#endif
}

orc_ctx *orc_ctx_create(uint32_t scheme, uint32_t log_n, uint32_t L, uint32_t K, uint32_t dnum,
                        uint32_t q_bits, uint32_t p_bits, uint64_t t, const uint64_t *moduli) {
  if (log_n < 2 || log_n > 17 || L == 0 || dnum == 0 || dnum > L) return NULL;
  orc_ctx *c = calloc(1, sizeof(orc_ctx));
  c->scheme = scheme; c->log_n = log_n; c->n = 1u << log_n;
  c->L = L; c->K = K; c->dnum = dnum; c->alpha = (L + dnum - 1) / dnum;
  c->t = t;
  c->nB = scheme == ORC_SCHEME_BFV ? L + 1 : 0;
  c->nmod = L + K + c->nB;
  if (c->nmod > MAXM) { free(c); return NULL; }
  uint64_t qs[MAXM];
  if (moduli) {
    memcpy(qs, moduli, sizeof(uint64_t) * c->nmod);
  } else {
    if (orc_gen_primes(q_bits, log_n, L, NULL, 0, qs) != L) { free(c); return NULL; }
    if (K && orc_gen_primes(p_bits, log_n, K, qs, L, qs + L) != K) { free(c); return NULL; }
    if (c->nB && orc_gen_primes(p_bits, log_n, c->nB, qs, L + K, qs + L + K) != c->nB) { free(c); return NULL; }
  }
  for (uint32_t i = 0; i < c->nmod; ++i) mod_init(&c->m[i], qs[i], log_n);
  return c;
}

int orc_set_bfv_mult(orc_ctx *c, uint32_t method) {
  if (method > ORC_BFV_HPS) return -1;
  c->bfv_mult = method;
  return 0;
}

void orc_ctx_destroy(orc_ctx *c) {
  if (!c) return;
  for (uint32_t i = 0; i < c->nmod; ++i) { free(c->m[i].w); free(c->m[i].ws); free(c->m[i].iw); free(c->m[i].iws); }
  free(c);
}
uint32_t orc_num_moduli(const orc_ctx *c) { return c->nmod; }
void orc_moduli(const orc_ctx *c, uint64_t *out) { for (uint32_t i = 0; i < c->nmod; ++i) out[i] = c->m[i].q; }
uint64_t orc_psi(const orc_ctx *c, uint32_t i) { return c->m[i].psi; }

/* ------------------------------------------------------------------ NTT */
/* Harvey forward negacyclic NTT (CT, natural in, bit-reversed out), lazy [0,4q) */
static void ntt_fwd_limb(const orc_mod *m, uint64_t *a, uint32_t n) {
  const uint64_t q = m->q, q2 = 2 * q;
  for (uint32_t mm = 1, t = n >> 1; mm < n; mm <<= 1, t >>= 1) {
    for (uint32_t i = 0; i < mm; ++i) {
      const uint64_t w = m->w[mm + i], ws = m->ws[mm + i];
      uint64_t *x = a + 2 * i * t, *y = x + t;
      for (uint32_t j = 0; j < t; ++j) {
        uint64_t u = x[j];
        if (u >= q2) u -= q2;
        uint64_t qh = (uint64_t)(((u128)y[j] * ws) >> 64);
        uint64_t v = y[j] * w - qh * q; /* [0,2q) */
        x[j] = u + v;
        y[j] = u - v + q2;
      }
    }
  }
  for (uint32_t j = 0; j < n; ++j) {
    uint64_t v = a[j];
    if (v >= q2) v -= q2;
    if (v >= q) v -= q;
    a[j] = v;
  }
}

/* Gentleman-Sande inverse (bit-reversed in, natural out, times N^-1) */
static void ntt_inv_limb(const orc_mod *m, uint64_t *a, uint32_t n) {
  const uint64_t q = m->q, q2 = 2 * q;
  for (uint32_t mm = n >> 1, t = 1; mm >= 1; mm >>= 1, t <<= 1) {
    for (uint32_t i = 0; i < mm; ++i) {
      const uint64_t w = m->iw[mm + i], ws = m->iws[mm + i];
      uint64_t *x = a + 2 * i * t, *y = x + t;
      for (uint32_t j = 0; j < t; ++j) {
        uint64_t u = x[j], v = y[j]; /* [0,2q) */
        uint64_t s = u + v;
        if (s >= q2) s -= q2;
        uint64_t d = u - v + q2;
        uint64_t qh = (uint64_t)(((u128)d * ws) >> 64);
        x[j] = s;
        y[j] = d * w - qh * q; /* [0,2q) */
      }
    }
    if (mm == 1) break;
  }
  for (uint32_t j = 0; j < n; ++j) a[j] = shoup_mul(a[j], m->ninv, m->ninvs, q);
}

void orc_ntt_fwd(const orc_ctx *c, uint64_t *data, uint32_t n_polys, uint32_t mb, uint32_t nl) {
  long total = (long)n_polys * nl;
#pragma omp parallel for schedule(static)
  for (long e = 0; e < total; ++e)
    ntt_fwd_limb(&c->m[mb + (uint32_t)(e % nl)], data + (size_t)e * c->n, c->n);
}
void orc_ntt_inv(const orc_ctx *c, uint64_t *data, uint32_t n_polys, uint32_t mb, uint32_t nl) {
  long total = (long)n_polys * nl;
#pragma omp parallel for schedule(static)
  for (long e = 0; e < total; ++e)
    ntt_inv_limb(&c->m[mb + (uint32_t)(e % nl)], data + (size_t)e * c->n, c->n);
}

/* --------------------------------------------------------------- dyadic */
#define DYADIC(name, expr)                                                              \
  void name(const orc_ctx *c, const uint64_t *a, const uint64_t *b, uint64_t *out,     \
            uint32_t n_polys, uint32_t mb, uint32_t nl) {                               \
    long total = (long)n_polys * nl;                                                   \
    _Pragma("omp parallel for schedule(static)")                                        \
    for (long e = 0; e < total; ++e) {                                                  \
      const uint64_t q = c->m[mb + (uint32_t)(e % nl)].q;                               \
      const size_t off = (size_t)e * c->n;                                              \
      for (uint32_t k = 0; k < c->n; ++k) {                                             \
        uint64_t x = a[off + k], y = b[off + k];                                        \
        out[off + k] = (expr);                                                          \
      }                                                                                 \
    }                                                                                   \
  }
DYADIC(orc_add, addmod(x, y, q))
DYADIC(orc_sub, submod(x, y, q))
DYADIC(orc_mul, mulmod(x, y, q))

/* ------------------------------------------------------------ automorph */
/* slot k holds a(psi^(2 brv(k) + 1)); sigma_g(a)(psi^e) = a(psi^(e g)) */
void orc_automorph_ntt(const orc_ctx *c, const uint64_t *in, uint64_t *out, uint32_t g,
                       uint32_t n_polys, uint32_t nl) {
  const uint32_t n = c->n, lg = c->log_n, mask = 2 * n - 1;
  uint32_t *perm = malloc(sizeof(uint32_t) * n);
  for (uint32_t k = 0; k < n; ++k) {
    uint32_t e = 2 * brv(k, lg) + 1;
    uint32_t e2 = (uint32_t)(((uint64_t)e * g) & mask);
    perm[k] = brv((e2 - 1) >> 1, lg);
  }
  long total = (long)n_polys * nl;
#pragma omp parallel for schedule(static)
  for (long e = 0; e < total; ++e) {
    const size_t off = (size_t)e * n;
    for (uint32_t k = 0; k < n; ++k) out[off + k] = in[off + perm[k]];
  }
  free(perm);
}

void orc_automorph_coef(const orc_ctx *c, const uint64_t *in, uint64_t *out, uint32_t g,
                        uint32_t n_polys, uint32_t mb, uint32_t nl) {
  const uint32_t n = c->n, mask = 2 * n - 1;
  long total = (long)n_polys * nl;
#pragma omp parallel for schedule(static)
  for (long e = 0; e < total; ++e) {
    const uint64_t q = c->m[mb + (uint32_t)(e % nl)].q;
    const size_t off = (size_t)e * n;
    for (uint32_t j = 0; j < n; ++j) {
      uint32_t d = (uint32_t)(((uint64_t)j * g) & mask);
      uint64_t v = in[off + j];
      if (d >= n) { d -= n; v = v ? q - v : 0; }
      out[off + d] = v;
    }
  }
}

uint32_t orc_galois_elt(const orc_ctx *c, int32_t steps) {
  uint64_t two_n = 2ull * c->n;
  uint64_t ord = c->n / 2; /* 5 has order N/2 mod 2N */
  int64_t s = steps % (int64_t)ord;
  if (s < 0) s += ord;
  uint64_t g = 1;
  for (int64_t i = 0; i < s; ++i) g = (g * 5) % two_n;
  return (uint32_t)g;
}

/* ------------------------------------------------------ base conversion */
/* Fast base conversion (Han-Ki / Bajard et al.):
 *   v_i = [x_i * (S/s_i)^-1]_{s_i};   y_m = sum_i v_i * [S/s_i]_m  mod m.
 * Approximate: y = x + u*S, 0 <= u < |S|. */
typedef struct {
  uint32_t ns, nd;
  uint64_t sq[MAXM], dq[MAXM];
  uint64_t hinv[MAXM], hinvs[MAXM];     /* (S/s_i)^-1 mod s_i + Shoup */
  uint64_t h[MAXM][MAXM];               /* [S/s_i] mod d_m : h[i][m] */
} conv_tab;

static void conv_tab_init(conv_tab *T, const uint64_t *sq, uint32_t ns, const uint64_t *dq, uint32_t nd) {
  T->ns = ns; T->nd = nd;
  for (uint32_t i = 0; i < ns; ++i) {
    T->sq[i] = sq[i];
    uint64_t prod = 1;
    for (uint32_t k = 0; k < ns; ++k) if (k != i) prod = mulmod(prod, sq[k] % sq[i], sq[i]);
    T->hinv[i] = invmod(prod, sq[i]);
    T->hinvs[i] = shoup_pre(T->hinv[i], sq[i]);
    for (uint32_t m = 0; m < nd; ++m) {
      uint64_t p2 = 1;
      for (uint32_t k = 0; k < ns; ++k) if (k != i) p2 = mulmod(p2, sq[k] % dq[m], dq[m]);
      T->h[i][m] = p2;
    }
  }
  for (uint32_t m = 0; m < nd; ++m) T->dq[m] = dq[m];
}

/* src: ns pointers to limbs (each N), dst: nd pointers */
static void conv_apply(const conv_tab *T, const uint64_t *const *src, uint64_t *const *dst, uint32_t n) {
  uint64_t v[MAXM];
  for (uint32_t k = 0; k < n; ++k) {
    for (uint32_t i = 0; i < T->ns; ++i) v[i] = shoup_mul(src[i][k], T->hinv[i], T->hinvs[i], T->sq[i]);
    for (uint32_t m = 0; m < T->nd; ++m) {
      u128 acc = 0;
      for (uint32_t i = 0; i < T->ns; ++i) acc += (u128)v[i] * T->h[i][m];
      dst[m][k] = (uint64_t)(acc % T->dq[m]);
    }
  }
}

void orc_base_conv(const orc_ctx *c, const uint64_t *src, const uint32_t *src_mods, uint32_t n_src,
                   uint64_t *dst, const uint32_t *dst_mods, uint32_t n_dst, uint32_t n) {
  conv_tab *T = malloc(sizeof(conv_tab));
  uint64_t sq[MAXM], dq[MAXM];
  for (uint32_t i = 0; i < n_src; ++i) sq[i] = c->m[src_mods[i]].q;
  for (uint32_t i = 0; i < n_dst; ++i) dq[i] = c->m[dst_mods[i]].q;
  conv_tab_init(T, sq, n_src, dq, n_dst);
#pragma omp parallel for schedule(static)
  for (long p = 0; p < (long)n; ++p) {
    const uint64_t *s[MAXM]; uint64_t *d[MAXM];
    for (uint32_t i = 0; i < n_src; ++i) s[i] = src + ((size_t)p * n_src + i) * c->n;
    for (uint32_t i = 0; i < n_dst; ++i) d[i] = dst + ((size_t)p * n_dst + i) * c->n;
    conv_apply(T, s, d, c->n);
  }
  free(T);
}

/* --------------------------------------------------------- key switching */
/* Hybrid key switching (dnum digits of alpha limbs, K special primes) at level
 * lvl <= L: d has the lvl active Q limbs, the digits partition them by alpha
 * (the last digit may be partial, digits past lvl are empty), ModUp extends
 * each digit to Q_lvl u P and the inner product uses the key rows of those
 * moduli: Q rows 0..lvl-1 and P rows L..L+K-1 of the full-level key (the
 * gadget g_j is P on digit j's limbs and 0 elsewhere, so dropping limbs keeps
 * sum_j [d]_{Q_j} g_j = P d mod q_i; OpenFHE's KeySwitchHYBRID at a reduced
 * level).  Level space: index i < lvl is q_i, lvl + k is p_k (modulus L + k).
 * in_ntt: 1 if d (and the result) is in NTT form (CKKS), 0 for coef form (BFV). */
/* ext_g != 0 (hoisted rotation, CKKS): the digits' extensions are computed for d
 * and then permuted by the NTT-domain automorphism sigma_g before the inner
 * product, i.e. sigma_g(ModUp(d)) stands in for ModUp(sigma_g(d)) -- the same
 * key-switching input up to its ModUp error term, so the bits differ from the
 * plain rotation's (OpenFHE EvalFastRotation on precomputed digits). */
static void keyswitch_lvl_g(const orc_ctx *c, const uint64_t *d, const uint64_t *ksk, uint64_t *out, int in_ntt,
                            uint32_t lvl, uint32_t ext_g);
static void keyswitch_lvl(const orc_ctx *c, const uint64_t *d, const uint64_t *ksk, uint64_t *out, int in_ntt,
                          uint32_t lvl) {
  keyswitch_lvl_g(c, d, ksk, out, in_ntt, lvl, 0);
}
/* n_keys > 1 (double-hoisted rotation sum): the inner products of every key
 * ksks[r] with sigma_{ext_gs[r]}(ModUp(d)) are summed before ONE ModDown. */
/* pts (optional, hoisted linear transform): key r's inner product is weighted by
 * the plaintext pts[r] ([L+K][N] NTT form, the rows of Q_lvl u P used like the
 * key's) before the sum. */
static void keyswitch_lvl_multi(const orc_ctx *c, const uint64_t *d, uint32_t n_keys, const uint64_t *const *ksks,
                                const uint32_t *ext_gs, const uint64_t *const *pts, uint64_t *out, int in_ntt,
                                uint32_t lvl);
static void keyswitch_lvl_g(const orc_ctx *c, const uint64_t *d, const uint64_t *ksk, uint64_t *out, int in_ntt,
                            uint32_t lvl, uint32_t ext_g) {
  keyswitch_lvl_multi(c, d, 1, &ksk, &ext_g, NULL, out, in_ntt, lvl);
}
static void keyswitch_lvl_multi(const orc_ctx *c, const uint64_t *d, uint32_t n_keys, const uint64_t *const *ksks,
                                const uint32_t *ext_gs, const uint64_t *const *pts, uint64_t *out, int in_ntt,
                                uint32_t lvl) {
  const uint32_t n = c->n, L = lvl, K = c->K, QP = L + K, QPk = c->L + K, A = c->alpha;
#define MI(i) ((i) < L ? (i) : c->L + ((i) - L))
  uint64_t *dc = malloc(sizeof(uint64_t) * L * n);        /* d in coef form */
  uint64_t *dn = malloc(sizeof(uint64_t) * L * n);        /* d in NTT form */
  uint64_t *ext = malloc(sizeof(uint64_t) * QP * n);
  uint64_t *acc = calloc((size_t)2 * QP * n, sizeof(uint64_t));
  memcpy(dc, d, sizeof(uint64_t) * L * n);
  memcpy(dn, d, sizeof(uint64_t) * L * n);
  if (in_ntt) orc_ntt_inv(c, dc, 1, 0, L); else orc_ntt_fwd(c, dn, 1, 0, L);
  conv_tab *T = malloc(sizeof(conv_tab));
  for (uint32_t j = 0; j < c->dnum; ++j) {
    uint32_t lo = j * A, hi = lo + A < L ? lo + A : L;
    if (lo >= L) break;
    /* ModUp: own limbs copied, the rest converted from the digit's limbs */
    uint64_t sq[MAXM], dq[MAXM]; uint32_t didx[MAXM], nd = 0;
    const uint64_t *sp[MAXM]; uint64_t *dp[MAXM];
    for (uint32_t i = lo; i < hi; ++i) { sq[i - lo] = c->m[i].q; sp[i - lo] = dc + (size_t)i * n; }
    for (uint32_t i = 0; i < QP; ++i) {
      if (i >= lo && i < hi) { memcpy(ext + (size_t)i * n, dn + (size_t)i * n, sizeof(uint64_t) * n); continue; }
      dq[nd] = c->m[MI(i)].q; didx[nd] = i; dp[nd] = ext + (size_t)i * n; ++nd;
    }
    conv_tab_init(T, sq, hi - lo, dq, nd);
    conv_apply(T, sp, dp, n);
    for (uint32_t k = 0; k < nd; ++k) ntt_fwd_limb(&c->m[MI(didx[k])], ext + (size_t)didx[k] * n, n);
    uint64_t *tmp = malloc(sizeof(uint64_t) * QP * n);
    for (uint32_t r = 0; r < n_keys; ++r) {
      const uint64_t *e = ext;
      if (ext_gs[r]) {  /* hoisted rotation: sigma_g on the digit's extension (a slot permutation per limb) */
        orc_automorph_ntt(c, ext, tmp, ext_gs[r], 1, QP);
        e = tmp;
      }
      /* inner product with key digit j (its rows of Q_lvl u P) */
      for (uint32_t b = 0; b < 2; ++b) {
        const uint64_t *kj = ksks[r] + ((size_t)(j * 2 + b) * QPk) * n;
        uint64_t *ab = acc + (size_t)b * QP * n;
        for (uint32_t i = 0; i < QP; ++i) {
          const uint64_t q = c->m[MI(i)].q;
          const uint64_t *kr = kj + (size_t)MI(i) * n;
          const uint64_t *pr = pts ? pts[r] + (size_t)MI(i) * n : NULL;
          for (uint32_t k = 0; k < n; ++k) {
            size_t o = (size_t)i * n + k;
            uint64_t v = mulmod(e[o], kr[k], q);
            if (pr) v = mulmod(v, pr[k] % q, q);
            ab[o] = addmod(ab[o], v, q);
          }
        }
      }
    }
    free(tmp);
  }
  /* ModDown: (acc_Q - Conv_{P->Q}(acc_P)) * P^-1 */
  uint64_t pq[MAXM], qq[MAXM];
  for (uint32_t k = 0; k < K; ++k) pq[k] = c->m[c->L + k].q;
  for (uint32_t i = 0; i < L; ++i) qq[i] = c->m[i].q;
  conv_tab_init(T, pq, K, qq, L);
  uint64_t *conv = malloc(sizeof(uint64_t) * L * n);
  for (uint32_t b = 0; b < 2; ++b) {
    uint64_t *ab = acc + (size_t)b * QP * n;
    if (!in_ntt) orc_ntt_inv(c, ab, 1, 0, L);
    orc_ntt_inv(c, ab + (size_t)L * n, 1, c->L, K);
    const uint64_t *sp[MAXM]; uint64_t *dp[MAXM];
    for (uint32_t k = 0; k < K; ++k) sp[k] = ab + (size_t)(L + k) * n;
    for (uint32_t i = 0; i < L; ++i) dp[i] = conv + (size_t)i * n;
    conv_apply(T, sp, dp, n);
    if (in_ntt) orc_ntt_fwd(c, conv, 1, 0, L);
    uint64_t *ob = out + (size_t)b * L * n;
    for (uint32_t i = 0; i < L; ++i) {
      const uint64_t q = c->m[i].q;
      uint64_t P = 1;
      for (uint32_t k = 0; k < K; ++k) P = mulmod(P, pq[k] % q, q);
      const uint64_t pinv = invmod(P, q);
      for (uint32_t k = 0; k < n; ++k) {
        size_t o = (size_t)i * n + k;
        ob[o] = mulmod(submod(ab[o], conv[o], q), pinv, q);
      }
    }
  }
#undef MI
  free(conv); free(T); free(dc); free(dn); free(ext); free(acc);
}

static void keyswitch_one(const orc_ctx *c, const uint64_t *d, const uint64_t *ksk, uint64_t *out, int in_ntt) {
  keyswitch_lvl(c, d, ksk, out, in_ntt, c->L);
}

void orc_keyswitch(const orc_ctx *c, const uint64_t *d, const uint64_t *ksk, uint64_t *out, uint32_t n) {
  const size_t L = c->L, N = c->n;
  for (uint32_t i = 0; i < n; ++i)
    keyswitch_one(c, d + i * L * N, ksk, out + i * 2 * L * N, c->scheme == ORC_SCHEME_CKKS);
}

void orc_ct_add(const orc_ctx *c, const uint64_t *a, const uint64_t *b, uint64_t *out, uint32_t n_ct) {
  orc_add(c, a, b, out, 2 * n_ct, 0, c->L);
}

/* ------------------------------------------------------------- BFV BEHZ */
/* Base layout for BEHZ: Bsk = moduli [L+K, L+K+L] (B = first L, m_sk last);
 * m_tilde = 2^32.  Restates SEAL RNSTool. */
typedef struct {
  conv_tab q_to_bskmt;  /* Q -> Bsk u {m_tilde}; m_tilde handled separately */
  conv_tab q_to_bsk;
  conv_tab b_to_q;
  conv_tab b_to_msk;
  uint64_t mt_hinv[MAXM], mt_hinvs[MAXM]; /* m_tilde * (Q/q_i)^-1 mod q_i */
  uint32_t h_mod_mt[MAXM];                /* (Q/q_i) mod 2^32 */
  uint32_t neg_inv_q_mod_mt;              /* -Q^-1 mod 2^32 */
  uint64_t q_mod_bsk[MAXM];               /* Q mod b */
  uint64_t inv_mt_mod_bsk[MAXM];          /* 2^-32 mod b */
  uint64_t inv_q_mod_bsk[MAXM];           /* Q^-1 mod b */
  uint64_t t_mod_q[MAXM], t_mod_bsk[MAXM];
  uint64_t inv_b_mod_msk;                 /* B^-1 mod m_sk */
  uint64_t b_mod_q[MAXM];                 /* B mod q_i */
} behz_tab;

static void behz_init(const orc_ctx *c, behz_tab *B) {
  const uint32_t L = c->L, nb = c->nB, bb = c->L + c->K;
  uint64_t qq[MAXM] = {0}, bsk[MAXM] = {0};
  for (uint32_t i = 0; i < L; ++i) qq[i] = c->m[i].q;
  for (uint32_t i = 0; i < nb; ++i) bsk[i] = c->m[bb + i].q;
  const uint64_t msk = bsk[nb - 1];
  conv_tab_init(&B->q_to_bsk, qq, L, bsk, nb);
  conv_tab_init(&B->b_to_q, bsk, nb - 1, qq, L);
  conv_tab_init(&B->b_to_msk, bsk, nb - 1, &msk, 1);
  const uint64_t mt = 1ull << 32;
  for (uint32_t i = 0; i < L; ++i) {
    uint64_t h = B->q_to_bsk.hinv[i];
    B->mt_hinv[i] = mulmod(h, mt % qq[i], qq[i]);
    B->mt_hinvs[i] = shoup_pre(B->mt_hinv[i], qq[i]);
    uint64_t hm = 1;
    for (uint32_t k = 0; k < L; ++k) if (k != i) hm = (hm * (qq[k] & 0xffffffffull)) & 0xffffffffull;
    B->h_mod_mt[i] = (uint32_t)hm;
  }
  uint64_t qm = 1;
  for (uint32_t k = 0; k < L; ++k) qm = (qm * (qq[k] & 0xffffffffull)) & 0xffffffffull;
  /* inverse of odd qm mod 2^32 by Newton */
  uint32_t inv = (uint32_t)qm;
  for (int it = 0; it < 5; ++it) inv *= 2u - (uint32_t)qm * inv;
  B->neg_inv_q_mod_mt = (uint32_t)(0u - inv);
  for (uint32_t j = 0; j < nb; ++j) {
    uint64_t b = bsk[j], qmb = 1;
    for (uint32_t k = 0; k < L; ++k) qmb = mulmod(qmb, qq[k] % b, b);
    B->q_mod_bsk[j] = qmb;
    B->inv_q_mod_bsk[j] = invmod(qmb, b);
    B->inv_mt_mod_bsk[j] = invmod(mt % b, b);
    B->t_mod_bsk[j] = c->t % b;
  }
  for (uint32_t i = 0; i < L; ++i) {
    B->t_mod_q[i] = c->t % qq[i];
    uint64_t bm = 1;
    for (uint32_t k = 0; k + 1 < nb; ++k) bm = mulmod(bm, bsk[k] % qq[i], qq[i]);
    B->b_mod_q[i] = bm;
  }
  uint64_t bmsk = 1;
  for (uint32_t k = 0; k + 1 < nb; ++k) bmsk = mulmod(bmsk, bsk[k] % msk, msk);
  B->inv_b_mod_msk = invmod(bmsk, msk);
}

/* x_q [L][N] coef -> x_bsk [nB][N] coef (fastbconv_m_tilde + sm_mrq) */
static void behz_extend(const orc_ctx *c, const behz_tab *B, const uint64_t *xq, uint64_t *xb) {
  const uint32_t L = c->L, n = c->n, nb = c->nB, bb = c->L + c->K;
  for (uint32_t k = 0; k < n; ++k) {
    uint64_t v[MAXM];
    for (uint32_t i = 0; i < L; ++i)
      v[i] = shoup_mul(xq[(size_t)i * n + k], B->mt_hinv[i], B->mt_hinvs[i], c->m[i].q);
    uint32_t xmt = 0;
    for (uint32_t i = 0; i < L; ++i) xmt += (uint32_t)v[i] * B->h_mod_mt[i];
    uint32_t r = xmt * B->neg_inv_q_mod_mt;          /* [0, 2^32) */
    for (uint32_t j = 0; j < nb; ++j) {
      const uint64_t b = c->m[bb + j].q;
      u128 acc = 0;
      for (uint32_t i = 0; i < L; ++i) acc += (u128)v[i] * B->q_to_bsk.h[i][j];
      uint64_t xbj = (uint64_t)(acc % b);
      /* centered r: r >= 2^31 means r - 2^32 */
      uint64_t rr = r >= 0x80000000u ? (uint64_t)r + b - (1ull << 32) % b : (uint64_t)r;
      rr %= b;
      uint64_t s = addmod(xbj, mulmod(B->q_mod_bsk[j], rr, b), b);
      xb[(size_t)j * n + k] = mulmod(s, B->inv_mt_mod_bsk[j], b);
    }
  }
}

/* (t*x) in Q and Bsk, coef form -> floor(t x / Q) in Bsk -> Q (fastbconv_sk) */
static void behz_floor_to_q(const orc_ctx *c, const behz_tab *B, const uint64_t *xq, const uint64_t *xb,
                            uint64_t *out) {
  const uint32_t L = c->L, n = c->n, nb = c->nB, bb = c->L + c->K;
  const uint64_t msk = c->m[bb + nb - 1].q;
  for (uint32_t k = 0; k < n; ++k) {
    uint64_t v[MAXM], fl[MAXM];
    /* fast_floor: ((t x)_b - conv_Q->b((t x)_Q)) * Q^-1 */
    for (uint32_t i = 0; i < L; ++i) {
      uint64_t tx = mulmod(xq[(size_t)i * n + k], B->t_mod_q[i], c->m[i].q);
      v[i] = shoup_mul(tx, B->q_to_bsk.hinv[i], B->q_to_bsk.hinvs[i], c->m[i].q);
    }
    for (uint32_t j = 0; j < nb; ++j) {
      const uint64_t b = c->m[bb + j].q;
      u128 acc = 0;
      for (uint32_t i = 0; i < L; ++i) acc += (u128)v[i] * B->q_to_bsk.h[i][j];
      uint64_t cv = (uint64_t)(acc % b);
      uint64_t tx = mulmod(xb[(size_t)j * n + k], B->t_mod_bsk[j], b);
      fl[j] = mulmod(submod(tx, cv, b), B->inv_q_mod_bsk[j], b);
    }
    /* fastbconv_sk: Bsk -> Q with Shenoy-Kumaresan correction */
    uint64_t w[MAXM];
    for (uint32_t j = 0; j + 1 < nb; ++j)
      w[j] = shoup_mul(fl[j], B->b_to_q.hinv[j], B->b_to_q.hinvs[j], c->m[bb + j].q);
    u128 am = 0;
    for (uint32_t j = 0; j + 1 < nb; ++j) am += (u128)w[j] * B->b_to_msk.h[j][0];
    uint64_t cmsk = (uint64_t)(am % msk);
    uint64_t alpha = mulmod(submod(cmsk, fl[nb - 1], msk), B->inv_b_mod_msk, msk);
    for (uint32_t i = 0; i < L; ++i) {
      const uint64_t q = c->m[i].q;
      u128 acc = 0;
      for (uint32_t j = 0; j + 1 < nb; ++j) acc += (u128)w[j] * B->b_to_q.h[j][i];
      uint64_t cq = (uint64_t)(acc % q);
      if (alpha > msk / 2) cq = addmod(cq, mulmod(B->b_mod_q[i], (msk - alpha) % q, q), q);
      else cq = submod(cq, mulmod(B->b_mod_q[i], alpha % q, q), q);
      out[(size_t)i * n + k] = cq;
    }
  }
}

/* ------------------------------------------------------------- BFV HPS */
/* Halevi-Polyakov-Shoup (CT-RSA 2019, "An Improved RNS Variant of the BFV
 * Homomorphic Encryption Scheme"), the multiplication technique OpenFHE's
 * BFVrns offers as HPS, with the auxiliary base P = the Bsk primes:
 *   1. exact extension of the centred lift Q -> P (section 2.4): y_i =
 *      [x_i (Q/q_i)^-1]_{q_i}, v = floor(0.5 + sum_i y_i / q_i) in doubles,
 *      x mod p_j = sum_i y_i [Q/q_i]_{p_j} - v [Q]_{p_j};
 *   2. tensor in Q u P;
 *   3. simple scaling by t/Q into P (section 4): with num_i = [t (Q/q_i)^-1]_{q_i},
 *      round(t d / Q) mod p_j = sum_i x_i I_ij + floor(0.5 + sum_i x_i f_i)
 *      + x_{p_j} [t Q^-1]_{p_j}, I_ij = [-num_i q_i^-1]_{p_j}, f_i = num_i / q_i;
 *   4. P -> Q by the exact extension of step 1.
 * Floating point: every double is one correctly rounded IEEE operation in a
 * fixed order, no contraction (-ffp-contract=off), so the backend reproduces
 * the same bits (oracle/bigint_model.py hps_* restates the same and checks the
 * result against round(t d / Q) on integers). */
typedef struct {
  uint64_t qt[MAXM], qts[MAXM];        /* (Q/q_i)^-1 mod q_i + Shoup */
  double invq[MAXM], frac[MAXM];       /* 1/q_i; num_i / q_i */
  uint64_t qstar_p[MAXM][MAXM];        /* [Q/q_i]_{p_j} */
  uint64_t Q_p[MAXM];                  /* [Q]_{p_j} */
  uint64_t I[MAXM][MAXM];              /* [-num_i q_i^-1]_{p_j} */
  uint64_t lam[MAXM];                  /* [t Q^-1]_{p_j} */
  uint64_t pt[MAXM], pts[MAXM];        /* (P/p_j)^-1 mod p_j */
  double invp[MAXM];
  uint64_t pstar_q[MAXM][MAXM];        /* [P/p_j]_{q_i} */
  uint64_t P_q[MAXM];                  /* [P]_{q_i} */
} hps_tab;

static void hps_init(const orc_ctx *c, hps_tab *H) {
  const uint32_t L = c->L, nb = c->nB, bb = c->L + c->K;
  for (uint32_t i = 0; i < L; ++i) {
    const uint64_t q = c->m[i].q;
    uint64_t h = 1;
    for (uint32_t k = 0; k < L; ++k) if (k != i) h = mulmod(h, c->m[k].q % q, q);
    H->qt[i] = invmod(h, q);
    H->qts[i] = shoup_pre(H->qt[i], q);
    H->invq[i] = 1.0 / (double)q;
    const uint64_t num = mulmod(c->t % q, H->qt[i], q);
    H->frac[i] = (double)num / (double)q;
    for (uint32_t j = 0; j < nb; ++j) {
      const uint64_t pj = c->m[bb + j].q;
      uint64_t qs = 1;
      for (uint32_t k = 0; k < L; ++k) if (k != i) qs = mulmod(qs, c->m[k].q % pj, pj);
      H->qstar_p[i][j] = qs;
      H->I[i][j] = mulmod((pj - num % pj) % pj, invmod(q % pj, pj), pj);
    }
  }
  for (uint32_t j = 0; j < nb; ++j) {
    const uint64_t pj = c->m[bb + j].q;
    uint64_t Qm = 1, h = 1;
    for (uint32_t k = 0; k < L; ++k) Qm = mulmod(Qm, c->m[k].q % pj, pj);
    H->Q_p[j] = Qm;
    H->lam[j] = mulmod(c->t % pj, invmod(Qm, pj), pj);
    for (uint32_t k = 0; k < nb; ++k) if (k != j) h = mulmod(h, c->m[bb + k].q % pj, pj);
    H->pt[j] = invmod(h, pj);
    H->pts[j] = shoup_pre(H->pt[j], pj);
    H->invp[j] = 1.0 / (double)pj;
  }
  for (uint32_t i = 0; i < L; ++i) {
    const uint64_t q = c->m[i].q;
    uint64_t Pm = 1;
    for (uint32_t k = 0; k < nb; ++k) Pm = mulmod(Pm, c->m[bb + k].q % q, q);
    H->P_q[i] = Pm;
    for (uint32_t j = 0; j < nb; ++j) {
      uint64_t ps = 1;
      for (uint32_t k = 0; k < nb; ++k) if (k != j) ps = mulmod(ps, c->m[bb + k].q % q, q);
      H->pstar_q[j][i] = ps;
    }
  }
}

/* x_q [L][N] coef -> x_p [nb][N] coef (the centred lift, exactly) */
static void hps_extend(const orc_ctx *c, const hps_tab *H, const uint64_t *xq, uint64_t *xp) {
  const uint32_t L = c->L, n = c->n, nb = c->nB, bb = c->L + c->K;
  for (uint32_t k = 0; k < n; ++k) {
    uint64_t y[MAXM];
    double s = 0.0;
    for (uint32_t i = 0; i < L; ++i) {
      y[i] = shoup_mul(xq[(size_t)i * n + k], H->qt[i], H->qts[i], c->m[i].q);
      s = s + (double)y[i] * H->invq[i];
    }
    const uint64_t v = (uint64_t)(s + 0.5);
    for (uint32_t j = 0; j < nb; ++j) {
      const uint64_t pj = c->m[bb + j].q;
      u128 acc = 0;
      for (uint32_t i = 0; i < L; ++i) acc += (u128)y[i] * H->qstar_p[i][j];
      xp[(size_t)j * n + k] = submod((uint64_t)(acc % pj), mulmod(v % pj, H->Q_p[j], pj), pj);
    }
  }
}

/* d in Q u P (coef, canonical) -> round(t d / Q) in P -> Q */
static void hps_scale_to_q(const orc_ctx *c, const hps_tab *H, const uint64_t *xq, const uint64_t *xp,
                           uint64_t *out) {
  const uint32_t L = c->L, n = c->n, nb = c->nB, bb = c->L + c->K;
  for (uint32_t k = 0; k < n; ++k) {
    double nu = 0.5;
    for (uint32_t i = 0; i < L; ++i) nu = nu + (double)xq[(size_t)i * n + k] * H->frac[i];
    const uint64_t r = (uint64_t)nu;
    uint64_t y[MAXM];
    double s = 0.0;
    for (uint32_t j = 0; j < nb; ++j) {
      const uint64_t pj = c->m[bb + j].q;
      u128 acc = (u128)xp[(size_t)j * n + k] * H->lam[j] + r;
      for (uint32_t i = 0; i < L; ++i) acc += (u128)xq[(size_t)i * n + k] * H->I[i][j];
      y[j] = shoup_mul((uint64_t)(acc % pj), H->pt[j], H->pts[j], pj);
      s = s + (double)y[j] * H->invp[j];
    }
    const uint64_t v = (uint64_t)(s + 0.5);
    for (uint32_t i = 0; i < L; ++i) {
      const uint64_t q = c->m[i].q;
      u128 acc = 0;
      for (uint32_t j = 0; j < nb; ++j) acc += (u128)y[j] * H->pstar_q[j][i];
      out[(size_t)i * n + k] = submod((uint64_t)(acc % q), mulmod(v % q, H->P_q[i], q), q);
    }
  }
}

static void bfv_mul_relin_one(const orc_ctx *c, const behz_tab *B, const hps_tab *H, const uint64_t *a,
                              const uint64_t *b, const uint64_t *rlk, uint64_t *out) {
  const uint32_t L = c->L, n = c->n, nb = c->nB, bb = c->L + c->K;
  const size_t LN = (size_t)L * n, BN = (size_t)nb * n;
  uint64_t *xq = malloc(sizeof(uint64_t) * 4 * LN), *xb = malloc(sizeof(uint64_t) * 4 * BN);
  /* 1. extend each of the 4 input polys to Bsk, then NTT in Q and Bsk */
  const uint64_t *in[4] = {a, a + LN, b, b + LN};
  for (int p = 0; p < 4; ++p) {
    memcpy(xq + p * LN, in[p], sizeof(uint64_t) * LN);
    if (H) hps_extend(c, H, in[p], xb + p * BN);
    else behz_extend(c, B, in[p], xb + p * BN);
  }
  orc_ntt_fwd(c, xq, 4, 0, L);
  orc_ntt_fwd(c, xb, 4, bb, nb);
  /* 2. tensor in Q and Bsk */
  uint64_t *eq = malloc(sizeof(uint64_t) * 3 * LN), *eb = malloc(sizeof(uint64_t) * 3 * BN);
  for (int base = 0; base < 2; ++base) {
    const uint32_t nl = base ? nb : L, m0 = base ? bb : 0;
    const size_t S = (size_t)nl * n;
    const uint64_t *x = base ? xb : xq;
    uint64_t *e = base ? eb : eq;
    for (uint32_t l = 0; l < nl; ++l) {
      const uint64_t q = c->m[m0 + l].q;
      for (uint32_t k = 0; k < n; ++k) {
        size_t o = (size_t)l * n + k;
        uint64_t a0 = x[o], a1 = x[S + o], b0 = x[2 * S + o], b1 = x[3 * S + o];
        e[o] = mulmod(a0, b0, q);
        e[S + o] = addmod(mulmod(a0, b1, q), mulmod(a1, b0, q), q);
        e[2 * S + o] = mulmod(a1, b1, q);
      }
    }
  }
  orc_ntt_inv(c, eq, 3, 0, L);
  orc_ntt_inv(c, eb, 3, bb, nb);
  /* 3. scale by t/Q with flooring, back to Q */
  uint64_t *r = malloc(sizeof(uint64_t) * 3 * LN);
  for (int p = 0; p < 3; ++p) {
    if (H) hps_scale_to_q(c, H, eq + p * LN, eb + p * BN, r + p * LN);
    else behz_floor_to_q(c, B, eq + p * LN, eb + p * BN, r + p * LN);
  }
  /* 4. relinearize r2 */
  uint64_t *ks = malloc(sizeof(uint64_t) * 2 * LN);
  keyswitch_one(c, r + 2 * LN, rlk, ks, 0);
  orc_add(c, r, ks, out, 2, 0, L);
  free(xq); free(xb); free(eq); free(eb); free(r); free(ks);
}

static void ckks_mul_relin_one(const orc_ctx *c, const uint64_t *a, const uint64_t *b, const uint64_t *rlk,
                               uint64_t *out, uint32_t lvl) {
  const size_t L = lvl, N = c->n;
  uint64_t *d = malloc(sizeof(uint64_t) * 3 * L * N);
  uint64_t *ks = malloc(sizeof(uint64_t) * 2 * L * N);
  const uint64_t *a0 = a, *a1 = a0 + L * N, *b0 = b, *b1 = b0 + L * N;
  for (uint32_t l = 0; l < L; ++l) {
    const uint64_t q = c->m[l].q;
    for (uint32_t k = 0; k < N; ++k) {
      size_t o = (size_t)l * N + k;
      d[o] = mulmod(a0[o], b0[o], q);
      d[L * N + o] = addmod(mulmod(a0[o], b1[o], q), mulmod(a1[o], b0[o], q), q);
      d[2 * L * N + o] = mulmod(a1[o], b1[o], q);
    }
  }
  keyswitch_lvl(c, d + 2 * L * N, rlk, ks, 1, lvl);
  orc_add(c, d, ks, out, 2, 0, (uint32_t)L);
  free(d); free(ks);
}

/* items are independent: one OpenMP thread per ciphertext (the inner
 * per-limb loops then run serially, nested parallelism being off). */
void orc_mul_relin(const orc_ctx *c, const uint64_t *a, const uint64_t *b, const uint64_t *rlk,
                   uint64_t *out, uint32_t n_ct) {
  const size_t L = c->L, N = c->n, CT = 2 * L * N;
  behz_tab *B = NULL;
  hps_tab *H = NULL;
  if (c->scheme == ORC_SCHEME_BFV) {
    if (c->bfv_mult == ORC_BFV_HPS) {
      H = malloc(sizeof(hps_tab));
      hps_init(c, H);
    } else {
      B = malloc(sizeof(behz_tab));
      behz_init(c, B);
    }
  }
#pragma omp parallel for schedule(dynamic, 1) if (n_ct > 1)
  for (long i = 0; i < (long)n_ct; ++i) {
    if (c->scheme == ORC_SCHEME_BFV) bfv_mul_relin_one(c, B, H, a + i * CT, b + i * CT, rlk, out + i * CT);
    else ckks_mul_relin_one(c, a + i * CT, b + i * CT, rlk, out + i * CT, c->L);
  }
  free(B);
  free(H);
}

/* The checker refuses what it does not implement, as the GPU ABI does
 * (fhe_backend.cpp ctx_level / ew_level_ok): BFV ciphertexts live at level L
 * only, and the level-lvl entries below compute the CKKS product and rescale.
 * Returns 0, or ORC_ERR_UNSUPPORTED / ORC_ERR_INVALID without touching out. */
static int level_ok(const orc_ctx *c, uint32_t lvl, int ckks_only) {
  if (lvl < 1 || lvl > c->L) return ORC_ERR_INVALID;
  if (c->scheme == ORC_SCHEME_BFV && (ckks_only || lvl != c->L)) return ORC_ERR_UNSUPPORTED;
  return 0;
}

static void rotate_lvl(const orc_ctx *c, const uint64_t *ct, uint32_t g, const uint64_t *gk, uint64_t *out,
                       uint32_t n_ct, uint32_t lvl) {
  const size_t L = lvl, N = c->n, CT = 2 * L * N;
  /* one ciphertext per thread, as the other batched ops */
#pragma omp parallel for schedule(dynamic, 1) if (n_ct > 1)
  for (long i = 0; i < (long)n_ct; ++i) {
    uint64_t *tmp = malloc(sizeof(uint64_t) * CT), *ks = malloc(sizeof(uint64_t) * CT);
    if (c->scheme == ORC_SCHEME_CKKS) orc_automorph_ntt(c, ct + i * CT, tmp, g, 2, (uint32_t)L);
    else orc_automorph_coef(c, ct + i * CT, tmp, g, 2, 0, (uint32_t)L);
    keyswitch_lvl(c, tmp + L * N, gk, ks, c->scheme == ORC_SCHEME_CKKS, lvl);
    orc_add(c, tmp, ks, out + i * CT, 1, 0, (uint32_t)L);
    memcpy(out + i * CT + L * N, ks + L * N, sizeof(uint64_t) * L * N);
    free(tmp); free(ks);
  }
}

void orc_rotate(const orc_ctx *c, const uint64_t *ct, uint32_t g, const uint64_t *gk, uint64_t *out,
                uint32_t n_ct) {
  rotate_lvl(c, ct, g, gk, out, n_ct, c->L);
}

/* Hoisted rotations: for each Galois element g_r of galois[0..n_rot),
 * outs[r] = (sigma(c0) + KS0, KS1) with KS over sigma_g(ModUp(c1)) and key
 * gks[r] -- one ModUp of c1 serves every rotation.  gks [n_rot][key],
 * outs [n_rot][n_ct][2][L][N].  CKKS: NTT form; BFV: coefficient form (the
 * extension is permuted in the NTT domain the key-switch inner product runs
 * in, c0 by the signed coefficient map; OpenFHE EvalFastRotation serves both). */
static void rotate_hoisted_lvl(const orc_ctx *c, const uint64_t *ct, uint32_t n_rot, const uint32_t *galois,
                               const uint64_t *gks, uint64_t *outs, uint32_t n_ct, uint32_t lvl) {
  const size_t L = lvl, N = c->n, CT = 2 * L * N, KW = (size_t)c->dnum * 2 * (c->L + c->K) * N;
  for (uint32_t r = 0; r < n_rot; ++r) {
#pragma omp parallel for schedule(dynamic, 1) if (n_ct > 1)
    for (long i = 0; i < (long)n_ct; ++i) {
      uint64_t *o = outs + ((size_t)r * n_ct + i) * CT;
      uint64_t *ks = malloc(sizeof(uint64_t) * CT);
      const int ckks = c->scheme == ORC_SCHEME_CKKS;
      keyswitch_lvl_g(c, ct + i * CT + L * N, gks + r * KW, ks, ckks, (uint32_t)L, galois[r]);
      if (ckks) orc_automorph_ntt(c, ct + i * CT, o, galois[r], 1, (uint32_t)L);
      else orc_automorph_coef(c, ct + i * CT, o, galois[r], 1, 0, (uint32_t)L);
      orc_add(c, o, ks, o, 1, 0, (uint32_t)L);
      memcpy(o + L * N, ks + L * N, sizeof(uint64_t) * L * N);
      free(ks);
    }
  }
}

void orc_rotate_hoisted(const orc_ctx *c, const uint64_t *ct, uint32_t n_rot, const uint32_t *galois,
                        const uint64_t *gks, uint64_t *outs, uint32_t n_ct) {
  rotate_hoisted_lvl(c, ct, n_rot, galois, gks, outs, n_ct, c->L);
}

/* the same at level lvl: ct, outs [..][2][lvl][N], full-level keys */
int orc_rotate_hoisted_at(const orc_ctx *c, const uint64_t *ct, uint32_t n_rot, const uint32_t *galois,
                          const uint64_t *gks, uint64_t *outs, uint32_t n_ct, uint32_t lvl) {
  const int rc = level_ok(c, lvl, 0);
  if (rc) return rc;
  rotate_hoisted_lvl(c, ct, n_rot, galois, gks, outs, n_ct, lvl);
  return 0;
}

/* Double-hoisted rotation sum (Bossuat et al.'s hoisted ModDown): out = sum_r
 * rot_{g_r}(ct), the key-switch inner products of every element summed in
 * Q u P before ONE ModDown, plus sum_r sigma_{g_r}(c0).  Decrypts to the sum of
 * the rotated messages; the bits differ from summing hoisted rotations by the
 * ModDown rounding.  out [n_ct][2][lvl][N]. */
int orc_rotate_sum_hoisted_at(const orc_ctx *c, const uint64_t *ct, uint32_t n_rot, const uint32_t *galois,
                              const uint64_t *gks, uint64_t *out, uint32_t n_ct, uint32_t lvl) {
  const int rc = level_ok(c, lvl, 0);
  if (rc) return rc;
  const size_t L = lvl, N = c->n, CT = 2 * L * N, KW = (size_t)c->dnum * 2 * (c->L + c->K) * N;
  const int ckks = c->scheme == ORC_SCHEME_CKKS;
  const uint64_t **ks_r = malloc(sizeof(uint64_t *) * (n_rot ? n_rot : 1));
  for (uint32_t r = 0; r < n_rot; ++r) ks_r[r] = gks + r * KW;
#pragma omp parallel for schedule(dynamic, 1) if (n_ct > 1)
  for (long i = 0; i < (long)n_ct; ++i) {
    uint64_t *o = out + i * CT;
    uint64_t *ks = malloc(sizeof(uint64_t) * CT), *rot = malloc(sizeof(uint64_t) * L * N);
    keyswitch_lvl_multi(c, ct + i * CT + L * N, n_rot, ks_r, galois, NULL, ks, ckks, (uint32_t)L);
    memcpy(o, ks, sizeof(uint64_t) * CT);
    for (uint32_t r = 0; r < n_rot; ++r) {
      if (ckks) orc_automorph_ntt(c, ct + i * CT, rot, galois[r], 1, (uint32_t)L);
      else orc_automorph_coef(c, ct + i * CT, rot, galois[r], 1, 0, (uint32_t)L);
      orc_add(c, o, rot, o, 1, 0, (uint32_t)L);
    }
    free(ks); free(rot);
  }
  free(ks_r);
  return 0;
}

/* Hoisted linear transform (CKKS): out = sum_r pts[r] (.) rot_{g_r}(ct), the
 * plaintext-weighted inner products of every element summed in Q u P before
 * ONE ModDown, plus sum_r pts[r] (.) sigma_{g_r}(c0).  pts [n_rot][L+K][N] in
 * the NTT domain (full-level rows; a level uses rows 0..lvl-1 and L..L+K-1). */
int orc_linear_hoisted_at(const orc_ctx *c, const uint64_t *ct, uint32_t n_rot, const uint32_t *galois,
                          const uint64_t *gks, const uint64_t *pts, uint64_t *out, uint32_t n_ct, uint32_t lvl) {
  const int rc = level_ok(c, lvl, 1);
  if (rc) return rc;
  const size_t L = lvl, N = c->n, CT = 2 * L * N, KW = (size_t)c->dnum * 2 * (c->L + c->K) * N;
  const size_t PW = (size_t)(c->L + c->K) * N;
  const uint64_t **ks_r = malloc(sizeof(uint64_t *) * (n_rot ? n_rot : 1));
  const uint64_t **pt_r = malloc(sizeof(uint64_t *) * (n_rot ? n_rot : 1));
  for (uint32_t r = 0; r < n_rot; ++r) { ks_r[r] = gks + r * KW; pt_r[r] = pts + r * PW; }
#pragma omp parallel for schedule(dynamic, 1) if (n_ct > 1)
  for (long i = 0; i < (long)n_ct; ++i) {
    uint64_t *o = out + i * CT;
    uint64_t *ks = malloc(sizeof(uint64_t) * CT), *rot = malloc(sizeof(uint64_t) * L * N);
    keyswitch_lvl_multi(c, ct + i * CT + L * N, n_rot, ks_r, galois, pt_r, ks, 1, (uint32_t)L);
    memcpy(o, ks, sizeof(uint64_t) * CT);
    for (uint32_t r = 0; r < n_rot; ++r) {
      orc_automorph_ntt(c, ct + i * CT, rot, galois[r], 1, (uint32_t)L);
      for (uint32_t li = 0; li < L; ++li) {
        const uint64_t q = c->m[li].q;
        for (size_t k = 0; k < N; ++k) {
          const size_t x = li * N + k;
          o[x] = addmod(o[x], mulmod(rot[x], pt_r[r][li * N + k] % q, q), q);
        }
      }
    }
    free(ks); free(rot);
  }
  free(ks_r); free(pt_r);
  return 0;
}

/* ------------------------------------------------- CKKS levels (rescale) */
int orc_keyswitch_at(const orc_ctx *c, const uint64_t *d, const uint64_t *ksk, uint64_t *out, uint32_t n,
                     uint32_t lvl) {
  const int rc = level_ok(c, lvl, 0);
  if (rc) return rc;
  const size_t N = c->n;
  for (uint32_t i = 0; i < n; ++i)
    keyswitch_lvl(c, d + i * lvl * N, ksk, out + i * 2 * lvl * N, c->scheme == ORC_SCHEME_CKKS, lvl);
  return 0;
}

int orc_mul_relin_at(const orc_ctx *c, const uint64_t *a, const uint64_t *b, const uint64_t *rlk,
                     uint64_t *out, uint32_t n_ct, uint32_t lvl) {
  const int rc = level_ok(c, lvl, 0);
  if (rc) return rc;
  if (c->scheme == ORC_SCHEME_BFV) { /* level L: the BFV product, as fhe_mul_relin_at's full-level context */
    orc_mul_relin(c, a, b, rlk, out, n_ct);
    return 0;
  }
  const size_t CT = 2 * (size_t)lvl * c->n;
#pragma omp parallel for schedule(dynamic, 1) if (n_ct > 1)
  for (long i = 0; i < (long)n_ct; ++i) ckks_mul_relin_one(c, a + i * CT, b + i * CT, rlk, out + i * CT, lvl);
  return 0;
}

int orc_rotate_at(const orc_ctx *c, const uint64_t *ct, uint32_t g, const uint64_t *gk, uint64_t *out,
                  uint32_t n_ct, uint32_t lvl) {
  const int rc = level_ok(c, lvl, 0);
  if (rc) return rc;
  rotate_lvl(c, ct, g, gk, out, n_ct, lvl);
  return 0;
}

/* CKKS rescale (OpenFHE DCRTPoly::DropLastElementAndScale, SEAL
 * divide_and_round_q_last_ntt_inplace): for the last limb x = INTT(c_{l-1})
 * lifted centrally (x - q_{l-1} if x > q_{l-1}/2, the same value both
 * libraries use), out_i = (c_i - NTT_i([x]_{q_i})) * q_{l-1}^-1 mod q_i,
 * i < l - 1 -- round(c / q_{l-1}) in RNS. */
int orc_rescale(const orc_ctx *c, const uint64_t *ct, uint64_t *out, uint32_t n_ct, uint32_t lvl) {
  const int rc = level_ok(c, lvl, 1);
  if (rc) return rc;
  if (lvl < 2) return ORC_ERR_INVALID;
  const size_t N = c->n, Li = lvl, Lo = lvl - 1;
  const uint64_t ql = c->m[Lo].q, half = ql >> 1;
#pragma omp parallel for schedule(dynamic, 1) if (n_ct > 1)
  for (long e = 0; e < 2 * (long)n_ct; ++e) {
    const uint64_t *src = ct + (size_t)e * Li * N;
    uint64_t *dst = out + (size_t)e * Lo * N;
    uint64_t *x = malloc(sizeof(uint64_t) * N), *y = malloc(sizeof(uint64_t) * N);
    memcpy(x, src + Lo * N, sizeof(uint64_t) * N);
    ntt_inv_limb(&c->m[Lo], x, (uint32_t)N);
    for (uint32_t i = 0; i < Lo; ++i) {
      const uint64_t q = c->m[i].q, qlm = ql % q, qinv = invmod(qlm, q);
      for (size_t k = 0; k < N; ++k) y[k] = x[k] > half ? submod(x[k] % q, qlm, q) : x[k] % q;
      ntt_fwd_limb(&c->m[i], y, (uint32_t)N);
      for (size_t k = 0; k < N; ++k) dst[i * N + k] = mulmod(submod(src[i * N + k], y[k], q), qinv, q);
    }
    free(x); free(y);
  }
  return 0;
}

/* -------------------------------------------------------------- sampling */
static inline uint64_t splitmix64(uint64_t z) {
  z ^= z >> 30; z *= 0xBF58476D1CE4E5B9ull;
  z ^= z >> 27; z *= 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
/* word w of stream `seed`: splitmix64(seed + (w+1) * golden) -- identical on the GPU */
static inline uint64_t stream_word(uint64_t seed, uint64_t w) {
  return splitmix64(seed + (w + 1) * 0x9E3779B97F4A7C15ull);
}

void orc_fill_uniform(const orc_ctx *c, uint64_t *data, uint32_t n_polys, uint32_t mb, uint32_t nl,
                      uint64_t seed) {
  const size_t N = c->n;
  long total = (long)n_polys * nl;
#pragma omp parallel for schedule(static)
  for (long e = 0; e < total; ++e) {
    const uint64_t q = c->m[mb + (uint32_t)(e % nl)].q;
    for (size_t k = 0; k < N; ++k) {
      size_t w = (size_t)e * N + k;
      data[w] = (uint64_t)(((u128)stream_word(seed, w) * q) >> 64);
    }
  }
}

void orc_sample_ternary(const orc_ctx *c, uint64_t seed, int64_t *coef) {
  for (uint32_t k = 0; k < c->n; ++k) coef[k] = (int64_t)(stream_word(seed, k) % 3) - 1;
}

/* centered binomial, eta = 21 (sigma ~ 3.24) */
void orc_sample_cbd(const orc_ctx *c, uint64_t seed, int64_t *coef) {
  for (uint32_t k = 0; k < c->n; ++k) {
    uint64_t x = stream_word(seed, k);
    coef[k] = (int64_t)__builtin_popcountll(x & 0x1FFFFFull) - (int64_t)__builtin_popcountll((x >> 21) & 0x1FFFFFull);
  }
}

void orc_signed_to_rns(const orc_ctx *c, const int64_t *coef, uint64_t *out, uint32_t mb, uint32_t nl, int ntt) {
  for (uint32_t l = 0; l < nl; ++l) {
    const uint64_t q = c->m[mb + l].q;
    for (uint32_t k = 0; k < c->n; ++k) {
      int64_t v = coef[k];
      uint64_t r = v >= 0 ? (uint64_t)v % q : (q - ((uint64_t)(-v) % q)) % q;
      out[(size_t)l * c->n + k] = r;
    }
  }
  if (ntt) orc_ntt_fwd(c, out, 1, mb, nl);
}

void orc_gen_switch_key(const orc_ctx *c, const uint64_t *sfrom, const uint64_t *sto, uint64_t seed,
                        uint64_t *ksk) {
  const uint32_t n = c->n, L = c->L, K = c->K, QP = L + K, A = c->alpha;
  int64_t *e = malloc(sizeof(int64_t) * n);
  uint64_t *er = malloc(sizeof(uint64_t) * QP * n);
  for (uint32_t j = 0; j < c->dnum; ++j) {
    uint64_t *b = ksk + ((size_t)(2 * j) * QP) * n, *a = b + (size_t)QP * n;
    orc_fill_uniform(c, a, 1, 0, QP, seed * 1000003ull + 2 * j + 1);
    orc_sample_cbd(c, seed * 1000003ull + 2 * j + 2, e);
    orc_signed_to_rns(c, e, er, 0, QP, 1);
    uint32_t lo = j * A, hi = lo + A < L ? lo + A : L;
    for (uint32_t i = 0; i < QP; ++i) {
      const uint64_t q = c->m[i].q;
      uint64_t Pm = 1;
      for (uint32_t k = 0; k < K; ++k) Pm = mulmod(Pm, c->m[L + k].q % q, q);
      for (uint32_t k = 0; k < n; ++k) {
        size_t o = (size_t)i * n + k;
        uint64_t v = submod(er[o], mulmod(a[o], sto[o], q), q);
        if (i >= lo && i < hi) v = addmod(v, mulmod(Pm, sfrom[o], q), q);
        b[o] = v;
      }
    }
  }
  free(e); free(er);
}

void orc_encrypt(const orc_ctx *c, const uint64_t *m_coef, const uint64_t *s_ntt, uint64_t seed, uint64_t *ct) {
  const uint32_t n = c->n, L = c->L;
  uint64_t *c0 = ct, *c1 = ct + (size_t)L * n;
  int64_t *e = malloc(sizeof(int64_t) * n);
  uint64_t *er = malloc(sizeof(uint64_t) * L * n), *mm = malloc(sizeof(uint64_t) * L * n);
  orc_fill_uniform(c, c1, 1, 0, L, seed * 7919ull + 1);          /* a, NTT form */
  orc_sample_cbd(c, seed * 7919ull + 2, e);
  orc_signed_to_rns(c, e, er, 0, L, 1);
  memcpy(mm, m_coef, sizeof(uint64_t) * L * n);
  orc_ntt_fwd(c, mm, 1, 0, L);
  for (uint32_t i = 0; i < L; ++i) {
    const uint64_t q = c->m[i].q;
    for (uint32_t k = 0; k < n; ++k) {
      size_t o = (size_t)i * n + k;
      c0[o] = addmod(submod(er[o], mulmod(c1[o], s_ntt[o], q), q), mm[o], q);
    }
  }
  if (c->scheme == ORC_SCHEME_BFV) orc_ntt_inv(c, ct, 2, 0, L);
  free(e); free(er); free(mm);
}

void orc_decrypt(const orc_ctx *c, const uint64_t *ct, const uint64_t *s_ntt, uint64_t *m_coef) {
  const uint32_t n = c->n, L = c->L;
  uint64_t *t = malloc(sizeof(uint64_t) * 2 * L * n);
  memcpy(t, ct, sizeof(uint64_t) * 2 * L * n);
  if (c->scheme == ORC_SCHEME_BFV) orc_ntt_fwd(c, t, 2, 0, L);
  for (uint32_t i = 0; i < L; ++i) {
    const uint64_t q = c->m[i].q;
    for (uint32_t k = 0; k < n; ++k) {
      size_t o = (size_t)i * n + k;
      m_coef[o] = addmod(t[o], mulmod(t[(size_t)L * n + o], s_ntt[o], q), q);
    }
  }
  orc_ntt_inv(c, m_coef, 1, 0, L);
  free(t);
}
