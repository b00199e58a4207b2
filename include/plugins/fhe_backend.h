/*
 * fhe_backend.h -- C ABI of the MI355X-native FHE ciphertext-op backend.
 *
 * This is the build's `include/plugins` operator surface (BASELINE.json
 * north_star).  herdsman (/root/reference) has no FHE operator surface of its
 * own: its only plugin is the gRPC token processor
 * (/root/reference/include/plugins/token_auth_metadata_processor.hpp:9-31),
 * and the arithmetic runs in remote workers reached through
 * IWorkerGroup::schedule_task (/root/reference/include/execution/worker/
 * i_worker_group.hpp:46; GrpcWorkerGroup::schedule_task at
 * /root/reference/src/execution/worker/grpc/grpc_worker_group.cpp:70-105).
 * Each entry point below REPLACES the remote `Worker.map` evaluation of one
 * ciphertext operation (grpc_worker_group.cpp:85 `stub->Asyncmap`) with an
 * in-process HIP call; the host-side caller is the GPU worker group
 * (herdsman_amd/host/gpu_worker_group.hpp), which keeps the IWorkerGroup
 * contract, so src/execution's Executor and the proto/service layer are
 * unchanged.
 *
 * Conventions (also those of the CPU oracle, oracle/fhe_oracle.h):
 *  - all words are u64; a polynomial is limb-major [limb][N]; batches are
 *    [item][poly][limb][N]; every pointer is DEVICE memory unless noted;
 *  - modulus index space: [0,L) = Q (ciphertext primes), [L,L+K) = P
 *    (special primes), then for BFV the BEHZ base Bsk (L+1 primes);
 *  - forward NTT: natural in, bit-reversed out, out[k] = a(psi^(2brv(k)+1)),
 *    psi = smallest primitive 2N-th root; outputs canonical in [0,q);
 *  - CKKS ciphertexts are kept in NTT form, BFV ciphertexts in coefficient
 *    form; (c0, c1) decrypts as c0 + c1*s;
 *  - switching keys: [dnum][2][L+K][N] NTT form (see oracle/fhe_oracle.h).
 *  - every function returns FHE_OK (0) or a negative FHE_ERR_*; the message
 *    is available from fhe_last_error(ctx).  No C++ exception crosses the ABI
 *    (matching IWorkerGroup's "no exceptions cross the seam",
 *    /root/reference/src/execution/executor/executor.cpp:168-178).
 *  - calls on one context are serialised by the caller; work is enqueued on
 *    the context's stream (fhe_set_stream) and is asynchronous.
 *  - a call over an empty batch (count 0) is a no-op and accepts null buffers
 *    (the other arguments are still validated).
 */
#ifndef HERDSMAN_PLUGINS_FHE_BACKEND_H
#define HERDSMAN_PLUGINS_FHE_BACKEND_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FHE_OK 0
#define FHE_ERR_INVALID -1
#define FHE_ERR_DEVICE -2
#define FHE_ERR_OOM -3
#define FHE_ERR_UNSUPPORTED -4

#define FHE_SCHEME_CKKS 0u
#define FHE_SCHEME_BFV 1u

typedef struct fhe_ctx fhe_ctx;

/* fhe_params.flags.  FHE_FLAG_BFV_HPS: BFV ct x ct multiplication by the HPS
 * technique (Halevi-Polyakov-Shoup: exact centred base extension to the
 * auxiliary base and simple scaling by t/Q with floating-point fractional
 * parts; OpenFHE BFVrns multiplication technique HPS) instead of BEHZ (SEAL's
 * RNSTool form, the default).  The two round differently, so their outputs
 * differ bit for bit; both decrypt to m1*m2 mod t. */
#define FHE_FLAG_BFV_HPS 1u

typedef struct fhe_params {
  uint32_t scheme;         /* FHE_SCHEME_CKKS or FHE_SCHEME_BFV */
  uint32_t log_n;          /* ring degree N = 2^log_n, 10..17 */
  uint32_t num_q;          /* L: ciphertext primes */
  uint32_t num_p;          /* K: special primes for hybrid key switching */
  uint32_t dnum;           /* number of key-switching digits, alpha = ceil(L/dnum) */
  uint32_t q_bits;         /* bit size for generated Q primes (<= 61) */
  uint32_t p_bits;         /* bit size for generated P / Bsk primes (<= 61) */
  uint32_t flags;          /* FHE_FLAG_*; 0 = defaults */
  uint64_t plain_modulus;  /* t (BFV only) */
  const uint64_t *moduli;  /* HOST pointer, optional explicit moduli in index-space order; NULL = generate */
} fhe_params;

/* ---- context -------------------------------------------------------- */
int fhe_ctx_create(const fhe_params *params, int device, fhe_ctx **out);
void fhe_ctx_destroy(fhe_ctx *ctx);
const char *fhe_last_error(const fhe_ctx *ctx);
/* SHA-256 (hex) of the sources this library was built from (herdsman_amd/csrc/
 * and this header, herdsman_amd/Makefile), so a loader can refuse a library
 * that does not match the sources it was shipped with */
const char *fhe_build_id(void);
/* number of moduli in the index space, and the moduli themselves (HOST out) */
int fhe_ctx_moduli(const fhe_ctx *ctx, uint64_t *out, uint32_t cap, uint32_t *count);
int fhe_set_stream(fhe_ctx *ctx, void *hip_stream);
int fhe_synchronize(fhe_ctx *ctx);
/* pre-size the context's scratch so later ops never allocate (graph capture) */
int fhe_reserve(fhe_ctx *ctx, uint32_t max_batch);

/* ---- device memory helpers (for callers without their own allocator) -- */
int fhe_dev_alloc(fhe_ctx *ctx, size_t bytes, void **out);
int fhe_dev_free(fhe_ctx *ctx, void *ptr);
/* h2d returns once the host buffer may be reused; d2h returns once the data has arrived */
int fhe_memcpy_h2d(fhe_ctx *ctx, void *dst, const void *src, size_t bytes);
int fhe_memcpy_d2h(fhe_ctx *ctx, void *dst, const void *src, size_t bytes);
/* pinned (page-locked) HOST staging memory, and copies that only enqueue on the
 * context's stream: the host buffer must come from fhe_host_alloc and stay
 * untouched until the next fhe_synchronize (a worker stages the inputs of a
 * batch while earlier copies and kernels run) */
int fhe_host_alloc(fhe_ctx *ctx, size_t bytes, void **out);
int fhe_host_free(fhe_ctx *ctx, void *ptr);
int fhe_memcpy_h2d_async(fhe_ctx *ctx, void *dst, const void *src, size_t bytes);
int fhe_memcpy_d2h_async(fhe_ctx *ctx, void *dst, const void *src, size_t bytes);
/* device-to-device copy enqueued on the context's stream (the worker group
 * keeps a MapTask's output frame resident in HBM for the stage that reads it) */
int fhe_memcpy_d2d_async(fhe_ctx *ctx, void *dst, const void *src, size_t bytes);
/* give the context a HIP stream of its own (non-blocking, destroyed with the
 * context) for callers without a stream of their own: several contexts on one
 * device then run concurrently, e.g. the worker group's lanes */
int fhe_use_own_stream(fhe_ctx *ctx);
/* stream marks for pipelined callers: fhe_mark records the work enqueued so far
 * on the context's stream in `slot` (< FHE_MAX_MARKS, re-recording overwrites);
 * fhe_wait_mark blocks the calling thread until that work is done, so a worker
 * can recycle the staging buffers of batch k while batch k+1 runs */
#define FHE_MAX_MARKS 16u
int fhe_mark(fhe_ctx *ctx, uint32_t slot);
int fhe_wait_mark(fhe_ctx *ctx, uint32_t slot);

/* ---- RNS primitives: data [n_polys][n_limbs][N]; limb l uses modulus mod_begin+l */
int fhe_ntt_fwd(fhe_ctx *ctx, uint64_t *data, uint32_t n_polys, uint32_t mod_begin, uint32_t n_limbs);
int fhe_ntt_inv(fhe_ctx *ctx, uint64_t *data, uint32_t n_polys, uint32_t mod_begin, uint32_t n_limbs);
int fhe_poly_add(fhe_ctx *ctx, const uint64_t *a, const uint64_t *b, uint64_t *out, uint32_t n_polys,
                 uint32_t mod_begin, uint32_t n_limbs);
int fhe_poly_sub(fhe_ctx *ctx, const uint64_t *a, const uint64_t *b, uint64_t *out, uint32_t n_polys,
                 uint32_t mod_begin, uint32_t n_limbs);
int fhe_poly_mul(fhe_ctx *ctx, const uint64_t *a, const uint64_t *b, uint64_t *out, uint32_t n_polys,
                 uint32_t mod_begin, uint32_t n_limbs);
/* fast base conversion: src [n][n_src][N] over moduli src_mods -> dst [n][n_dst][N] (index lists on HOST) */
int fhe_base_conv(fhe_ctx *ctx, const uint64_t *src, const uint32_t *src_mods, uint32_t n_src, uint64_t *dst,
                  const uint32_t *dst_mods, uint32_t n_dst, uint32_t n);
/* deterministic uniform fill: word w of the buffer = hi64(splitmix64(seed+(w+1)*phi) * q) */
int fhe_fill_uniform(fhe_ctx *ctx, uint64_t *data, uint32_t n_polys, uint32_t mod_begin, uint32_t n_limbs,
                     uint64_t seed);

/* ---- ciphertext operations (the operator surface) ---------------------
 * ct buffers: [n_ct][2][L][N]; keys: [dnum][2][L+K][N] */
int fhe_add(fhe_ctx *ctx, const uint64_t *a, const uint64_t *b, uint64_t *out, uint32_t n_ct);
int fhe_sub(fhe_ctx *ctx, const uint64_t *a, const uint64_t *b, uint64_t *out, uint32_t n_ct);
/* ct x ct multiply + relinearize (CKKS: NTT-domain tensor; BFV: BEHZ) */
int fhe_mul_relin(fhe_ctx *ctx, const uint64_t *a, const uint64_t *b, const uint64_t *rlk, uint64_t *out,
                  uint32_t n_ct);
/* hybrid key switch: d [n][L][N] -> out [n][2][L][N] (same domain as the scheme's ciphertexts) */
int fhe_keyswitch(fhe_ctx *ctx, const uint64_t *d, const uint64_t *ksk, uint64_t *out, uint32_t n);
/* automorphism X -> X^galois_elt followed by key switching with the Galois key */
int fhe_rotate(fhe_ctx *ctx, const uint64_t *ct, uint32_t galois_elt, const uint64_t *gk, uint64_t *out,
               uint32_t n_ct);
/* hoisted rotations (CKKS and BFV): n_rot Galois elements applied to the same n_ct
 * ciphertexts, c1's ModUp computed once (OpenFHE EvalFastRotationPrecompute +
 * EvalFastRotation, which herdsman's linked library provides for rotation-heavy
 * circuits).  galois_elts, gks, outs: HOST arrays of n_rot entries; gks[r] is a
 * device Galois key for galois_elts[r], outs[r] a device [n_ct][2][L][N]
 * buffer that must not overlap ct or another outs[q].  outs[r] =
 * (sigma(c0) + KS_0, KS_1) with KS over sigma_g(ModUp(c1)): decrypts like
 * fhe_rotate's result, but the bits differ from it by the ModUp error term
 * (oracle orc_rotate_hoisted).  CKKS in the NTT domain, BFV in the
 * coefficient domain, as the other ciphertext ops. */
int fhe_rotate_hoisted(fhe_ctx *ctx, const uint64_t *ct, uint32_t n_rot, const uint32_t *galois_elts,
                       const uint64_t *const *gks, uint64_t *const *outs, uint32_t n_ct);
/* double-hoisted rotation sum: out [n_ct][2][L][N] = sum_r rot_{galois_elts[r]}(ct)
 * with the key-switch inner products of all n_rot >= 1 elements summed in
 * Q u P before ONE ModDown (the hoisted-ModDown baby-step sum of linear
 * transforms).  Decrypts to the sum of the rotated messages; the bits differ
 * from adding fhe_rotate_hoisted's outputs by the ModDown rounding (oracle
 * orc_rotate_sum_hoisted_at).  galois_elts, gks: HOST arrays; out may be ct itself (in place) or apart from it; a partial overlap is FHE_ERR_INVALID. */
int fhe_rotate_sum_hoisted(fhe_ctx *ctx, const uint64_t *ct, uint32_t n_rot, const uint32_t *galois_elts,
                           const uint64_t *const *gks, uint64_t *out, uint32_t n_ct);
/* hoisted linear transform (CKKS; the baby-step block of a matrix-vector
 * product): out = sum_r pts[r] (.) rot_{galois_elts[r]}(ct), the plaintext-
 * weighted inner products summed in Q u P before ONE ModDown.  pts: HOST array
 * of n_rot device plaintexts [L+K][N] in the NTT domain (full-level rows, used
 * like the keys' at a reduced level); oracle orc_linear_hoisted_at. */
int fhe_linear_hoisted(fhe_ctx *ctx, const uint64_t *ct, uint32_t n_rot, const uint32_t *galois_elts,
                       const uint64_t *const *gks, const uint64_t *const *pts, uint64_t *out, uint32_t n_ct);
/* 5^steps mod 2N (steps may be negative); conjugation is 2N-1 */
int fhe_galois_elt(const fhe_ctx *ctx, int32_t steps, uint32_t *out);

/* ---- CKKS levels ("+ optional rescale") ---------------
 * A CKKS ciphertext at level m (1 <= m <= L) holds the first m Q limbs:
 * [n_ct][2][m][N], NTT form.  The *_at calls take such ciphertexts; key
 * switching at level m uses the FULL-level keys ([dnum][2][L+K][N]), reading
 * their rows of Q_m u P, with the digits partitioning the m active limbs by
 * alpha = ceil(L/dnum) (the last digit possibly partial) -- OpenFHE's hybrid
 * key switching at a reduced level (KeySwitchHYBRID on a level-dropped
 * DCRTPoly), which herdsman's linked library performs per multiply
 * (/root/reference/CMakeLists.txt:73,210-211).  level = L is the plain call.
 * BFV contexts support only level = L (FHE_ERR_UNSUPPORTED otherwise). */
int fhe_add_at(fhe_ctx *ctx, const uint64_t *a, const uint64_t *b, uint64_t *out, uint32_t n_ct, uint32_t level);
int fhe_sub_at(fhe_ctx *ctx, const uint64_t *a, const uint64_t *b, uint64_t *out, uint32_t n_ct, uint32_t level);
int fhe_mul_relin_at(fhe_ctx *ctx, const uint64_t *a, const uint64_t *b, const uint64_t *rlk, uint64_t *out,
                     uint32_t n_ct, uint32_t level);
int fhe_rotate_at(fhe_ctx *ctx, const uint64_t *ct, uint32_t galois_elt, const uint64_t *gk, uint64_t *out,
                  uint32_t n_ct, uint32_t level);
int fhe_keyswitch_at(fhe_ctx *ctx, const uint64_t *d, const uint64_t *ksk, uint64_t *out, uint32_t n,
                     uint32_t level);
int fhe_rotate_hoisted_at(fhe_ctx *ctx, const uint64_t *ct, uint32_t n_rot, const uint32_t *galois_elts,
                          const uint64_t *const *gks, uint64_t *const *outs, uint32_t n_ct, uint32_t level);
int fhe_rotate_sum_hoisted_at(fhe_ctx *ctx, const uint64_t *ct, uint32_t n_rot, const uint32_t *galois_elts,
                              const uint64_t *const *gks, uint64_t *out, uint32_t n_ct, uint32_t level);
int fhe_linear_hoisted_at(fhe_ctx *ctx, const uint64_t *ct, uint32_t n_rot, const uint32_t *galois_elts,
                          const uint64_t *const *gks, const uint64_t *const *pts, uint64_t *out, uint32_t n_ct,
                          uint32_t level);
/* CKKS rescale, level -> level - 1 (2 <= level <= L): out [n_ct][2][level-1][N]
 * = round(ct / q_{level-1}) -- OpenFHE DCRTPoly::DropLastElementAndScale /
 * SEAL divide_and_round_q_last_ntt (the dropped limb lifted centrally).
 * out must not overlap ct. */
int fhe_rescale(fhe_ctx *ctx, const uint64_t *ct, uint64_t *out, uint32_t n_ct, uint32_t level);
/* level_out < level_in: drop the Q limbs past level_out without scaling (OpenFHE
 * LevelReduce): out [n_ct][2][level_out][N] = the first level_out limbs of each
 * poly of ct [n_ct][2][level_in][N].  out must not overlap ct. */
int fhe_level_reduce(fhe_ctx *ctx, const uint64_t *ct, uint64_t *out, uint32_t n_ct, uint32_t level_in,
                     uint32_t level_out);
/* fhe_reduce on ciphertexts of level `level` (cts, out [.][2][level][N]) */
int fhe_reduce_at(fhe_ctx *ctx, uint64_t *cts, uint32_t n_ct, int op, const uint64_t *rlk, uint64_t *out,
                  uint32_t level);

/* ---- reductions ---------------------------------------
 * Homomorphic reduction of n_ct ciphertexts to one, the evaluation of one
 * herdsman ReduceTask (the cross-partition tree itself is planned by
 * /root/reference/src/service/execution_service.cpp:590-688).  Balanced tree,
 * one batched fhe_add / fhe_mul_relin per level: at a level with `live`
 * survivors, item i < live/2 absorbs item i + live - live/2 (an odd middle
 * item waits a level).  cts is the scratch and is overwritten; the result is
 * written to out (which may alias cts).  op MUL_RELIN needs rlk. */
#define FHE_REDUCE_ADD 0
#define FHE_REDUCE_MUL_RELIN 1
int fhe_reduce(fhe_ctx *ctx, uint64_t *cts, uint32_t n_ct, int op, const uint64_t *rlk, uint64_t *out);

/* ---- multi-GPU ---------------------------------------------------------
 * Broadcast an evaluation key (words u64 in device memory) from `root` to all
 * ranks of an RCCL communicator (ncclComm_t passed as void*).  The only
 * collective the backend uses. */
int fhe_bcast_key(fhe_ctx *ctx, uint64_t *key, size_t words, void *nccl_comm, int root);
/* Join of per-rank partial results: every rank holds one ciphertext `ct`
 * ([2][L][N]); a binomial tree of RCCL point-to-point transfers
 * (ncclSend/ncclRecv over xGMI) moves them towards `root`, and the receiving
 * rank combines with the mod-q op of `op` (RCCL has no modular reduction).
 * The result is in `ct` on root; tmp is one ciphertext of device scratch. */
int fhe_reduce_ranks(fhe_ctx *ctx, uint64_t *ct, int op, const uint64_t *rlk, void *nccl_comm, int root,
                     uint64_t *tmp);
/* the same on ciphertexts of level `level` (ct, tmp: [2][level][N]; CKKS) */
int fhe_reduce_ranks_at(fhe_ctx *ctx, uint64_t *ct, int op, const uint64_t *rlk, void *nccl_comm, int root,
                        uint64_t *tmp, uint32_t level);
/* The tree of fhe_reduce_ranks, host only: writes the rank's steps in order,
 * peer + 1 for "receive from peer and combine", -(peer + 1) for "send to peer
 * (then stop)"; returns the number of steps (<= cap) or a negative error. */
int fhe_reduce_schedule(int rank, int world, int root, int32_t *steps, int cap);

#ifdef __cplusplus
}
#endif
#endif
