/*
 * fhe_oracle.h -- CPU ORACLE for the herdsman MI355X FHE backend.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library.  The product path
 * (herdsman_amd/, libherdsman_fhe.so) never links or calls it.
 *
 * PARITY STATUS: "parity unpinned" against herdsman itself.  herdsman
 * (/root/reference) contains no FHE arithmetic: it links OpenFHE
 * (/root/reference/CMakeLists.txt:73,210-211) but never calls it, and the
 * remote worker that would run the ciphertext ops is not in the tree
 * (/root/reference/src/execution/worker/grpc/grpc_worker_group.cpp:85,94 only
 * forwards MapTask/ReduceTask over gRPC).  OpenFHE and its version pin (the
 * empty `common` submodule, /root/reference/default.nix:4) are absent from
 * this image.  This oracle is therefore a plain-C restatement of the published
 * RNS algorithms OpenFHE/SEAL implement (Harvey NTT, fast base conversion,
 * hybrid key switching, BEHZ BFV multiplication), PINNED to mathematical
 * ground truth by tests/golden/ fixtures generated with the independent
 * Python big-integer model oracle/bigint_model.py.
 *
 * Conventions (identical in the GPU backend, include/plugins/fhe_backend.h):
 *  - words are u64, polynomials are limb-major [poly][limb][N];
 *  - forward NTT: natural order in, bit-reversed out,
 *    out[k] = a(psi^(2*brv(k)+1)) mod q, psi = the smallest primitive
 *    2N-th root of unity mod q; outputs canonical in [0, q);
 *  - ciphertext (c0, c1) decrypts as c0 + c1*s;
 *  - switching key from s' to s: [dnum][2][L+K][N] NTT form,
 *    key[j][0] = -a_j*s + e_j + g_j*s', key[j][1] = a_j,
 *    g_j = P mod q_i for q_i in digit j, 0 elsewhere (and 0 mod P).
 */
#ifndef HERDSMAN_FHE_ORACLE_H
#define HERDSMAN_FHE_ORACLE_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORC_SCHEME_CKKS 0u
#define ORC_SCHEME_BFV 1u
/* refusals of the level entries (the checker does not compute what it does not
 * implement: BFV has no reduced levels, rescale and linear transforms are CKKS) */
#define ORC_ERR_INVALID (-1)
#define ORC_ERR_UNSUPPORTED (-4)

typedef struct orc_ctx orc_ctx;

/* moduli: NULL -> deterministic generation (see orc_gen_primes).  Layout of
 * the modulus index space: [0,L) = Q, [L,L+K) = P, then (BFV only) the BEHZ
 * base Bsk = B (L primes) + m_sk, all NTT-friendly. */
orc_ctx *orc_ctx_create(uint32_t scheme, uint32_t log_n, uint32_t L, uint32_t K,
                        uint32_t dnum, uint32_t q_bits, uint32_t p_bits,
                        uint64_t plain_modulus, const uint64_t *moduli);
void orc_ctx_destroy(orc_ctx *c);
uint32_t orc_num_moduli(const orc_ctx *c);
void orc_moduli(const orc_ctx *c, uint64_t *out);
uint64_t orc_psi(const orc_ctx *c, uint32_t mod_idx);
/* count primes q < 2^bits, q = 1 mod 2^32 (hence mod 2N), descending, skipping `excl` */
uint32_t orc_gen_primes(uint32_t bits, uint32_t log_n, uint32_t count,
                        const uint64_t *excl, uint32_t n_excl, uint64_t *out);
void orc_set_threads(int n);
/* BFV multiplication technique: BEHZ (SEAL RNSTool form, the default) or HPS
 * (Halevi-Polyakov-Shoup, OpenFHE BFVrns "HPS"); returns 0, or -1 if unknown */
#define ORC_BFV_BEHZ 0u
#define ORC_BFV_HPS 1u
int orc_set_bfv_mult(orc_ctx *c, uint32_t method);

/* ---- primitive RNS ops: data [n_polys][n_limbs][N], limb l uses modulus mod_begin+l */
void orc_ntt_fwd(const orc_ctx *c, uint64_t *data, uint32_t n_polys, uint32_t mod_begin, uint32_t n_limbs);
void orc_ntt_inv(const orc_ctx *c, uint64_t *data, uint32_t n_polys, uint32_t mod_begin, uint32_t n_limbs);
void orc_add(const orc_ctx *c, const uint64_t *a, const uint64_t *b, uint64_t *out,
             uint32_t n_polys, uint32_t mod_begin, uint32_t n_limbs);
void orc_sub(const orc_ctx *c, const uint64_t *a, const uint64_t *b, uint64_t *out,
             uint32_t n_polys, uint32_t mod_begin, uint32_t n_limbs);
void orc_mul(const orc_ctx *c, const uint64_t *a, const uint64_t *b, uint64_t *out,
             uint32_t n_polys, uint32_t mod_begin, uint32_t n_limbs);
/* NTT-domain automorphism X -> X^g (g odd): a permutation of slots */
void orc_automorph_ntt(const orc_ctx *c, const uint64_t *in, uint64_t *out, uint32_t galois,
                       uint32_t n_polys, uint32_t n_limbs);
/* coefficient-domain automorphism (negacyclic index map with sign flip) */
void orc_automorph_coef(const orc_ctx *c, const uint64_t *in, uint64_t *out, uint32_t galois,
                        uint32_t n_polys, uint32_t mod_begin, uint32_t n_limbs);
/* fast base conversion: src [n][n_src][N] over moduli src_mods -> dst [n][n_dst][N] */
void orc_base_conv(const orc_ctx *c, const uint64_t *src, const uint32_t *src_mods, uint32_t n_src,
                   uint64_t *dst, const uint32_t *dst_mods, uint32_t n_dst, uint32_t n);

/* ---- ciphertext ops.  ct = [n_ct][2][L][N]; CKKS: NTT form; BFV: coefficient form */
void orc_ct_add(const orc_ctx *c, const uint64_t *a, const uint64_t *b, uint64_t *out, uint32_t n_ct);
/* hybrid key switch of d [n][L][N] (NTT form for CKKS, coef form for BFV) -> out [n][2][L][N] */
void orc_keyswitch(const orc_ctx *c, const uint64_t *d, const uint64_t *ksk, uint64_t *out, uint32_t n);
void orc_mul_relin(const orc_ctx *c, const uint64_t *a, const uint64_t *b, const uint64_t *rlk,
                   uint64_t *out, uint32_t n_ct);
void orc_rotate(const orc_ctx *c, const uint64_t *ct, uint32_t galois, const uint64_t *gk,
                uint64_t *out, uint32_t n_ct);
uint32_t orc_galois_elt(const orc_ctx *c, int32_t steps);

/* hoisted rotations of ct [n_ct][2][L][N] (CKKS in NTT form, BFV in coefficient form): outs [n_rot][n_ct][2][L][N],
 * gks [n_rot][dnum][2][L+K][N]; KS over sigma_g(ModUp(c1)) (one ModUp for all) */
void orc_rotate_hoisted(const orc_ctx *c, const uint64_t *ct, uint32_t n_rot, const uint32_t *galois,
                        const uint64_t *gks, uint64_t *outs, uint32_t n_ct);
int orc_rotate_hoisted_at(const orc_ctx *c, const uint64_t *ct, uint32_t n_rot, const uint32_t *galois,
                           const uint64_t *gks, uint64_t *outs, uint32_t n_ct, uint32_t lvl);
/* double-hoisted rotation sum: out [n_ct][2][lvl][N] = sum_r rot_{g_r}(ct), one ModDown */
int orc_rotate_sum_hoisted_at(const orc_ctx *c, const uint64_t *ct, uint32_t n_rot, const uint32_t *galois,
                               const uint64_t *gks, uint64_t *out, uint32_t n_ct, uint32_t lvl);
/* hoisted linear transform (CKKS): out = sum_r pts[r] (.) rot_{g_r}(ct), one ModDown */
int orc_linear_hoisted_at(const orc_ctx *c, const uint64_t *ct, uint32_t n_rot, const uint32_t *galois,
                           const uint64_t *gks, const uint64_t *pts, uint64_t *out, uint32_t n_ct, uint32_t lvl);

/* ---- CKKS levels: ciphertexts [n_ct][2][lvl][N] with the first lvl Q primes
 * (1 <= lvl <= L).  The *_at entries and rescale return 0, or ORC_ERR_* for a
 * level outside [1, L] or a BFV context below L (rescale and the linear
 * transform: any BFV context); BFV at level L runs the BFV op.  Key switching at level lvl uses the full-level key's rows
 * of Q_lvl u P (digits partition the lvl limbs by alpha). */
int orc_keyswitch_at(const orc_ctx *c, const uint64_t *d, const uint64_t *ksk, uint64_t *out, uint32_t n,
                      uint32_t lvl);
int orc_mul_relin_at(const orc_ctx *c, const uint64_t *a, const uint64_t *b, const uint64_t *rlk,
                      uint64_t *out, uint32_t n_ct, uint32_t lvl);
int orc_rotate_at(const orc_ctx *c, const uint64_t *ct, uint32_t galois, const uint64_t *gk,
                   uint64_t *out, uint32_t n_ct, uint32_t lvl);
/* rescale level lvl -> lvl - 1 (lvl >= 2): out [n_ct][2][lvl-1][N] = round(ct / q_{lvl-1}) */
int orc_rescale(const orc_ctx *c, const uint64_t *ct, uint64_t *out, uint32_t n_ct, uint32_t lvl);

/* ---- test helpers: sampling, keys, encryption */
void orc_fill_uniform(const orc_ctx *c, uint64_t *data, uint32_t n_polys, uint32_t mod_begin,
                      uint32_t n_limbs, uint64_t seed);
void orc_sample_ternary(const orc_ctx *c, uint64_t seed, int64_t *coef);
void orc_sample_cbd(const orc_ctx *c, uint64_t seed, int64_t *coef);
/* small signed coefficients -> RNS over moduli [mod_begin, mod_begin+n_limbs), optional NTT */
void orc_signed_to_rns(const orc_ctx *c, const int64_t *coef, uint64_t *out, uint32_t mod_begin,
                       uint32_t n_limbs, int ntt);
/* switching key s_from -> s_to; both secrets given in NTT form over Q u P ([L+K][N]) */
void orc_gen_switch_key(const orc_ctx *c, const uint64_t *s_from_ntt, const uint64_t *s_to_ntt,
                        uint64_t seed, uint64_t *ksk);
/* symmetric encryption of m (coef form over Q, already scaled for BFV) -> ct [2][L][N] */
void orc_encrypt(const orc_ctx *c, const uint64_t *m_coef, const uint64_t *s_ntt, uint64_t seed,
                 uint64_t *ct);
/* c0 + c1*s over Q, returned in coefficient form [L][N] */
void orc_decrypt(const orc_ctx *c, const uint64_t *ct, const uint64_t *s_ntt, uint64_t *m_coef);

#ifdef __cplusplus
}
#endif
#endif
