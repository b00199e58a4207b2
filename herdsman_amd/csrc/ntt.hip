// ntt.hip -- negacyclic NTT / INTT for gfx950.
//
// Algorithm (same transform as the oracle's orc_ntt_fwd, oracle/fhe_oracle.c):
// Harvey's lazy Cooley-Tukey forward (natural in, bit-reversed out, values in
// [0,4q) between stages) and Gentleman-Sande inverse ([0,2q)).  The twiddle of
// butterfly (j, j+t) at global stage s is psi^brv(2^s + (j >> (logN - s))),
// stored in Montgomery form (psi^e * 2^64 mod q) so one mont_mul = 6
// quarter-rate multiplies gives the exact product (modarith.hpp).
//
// MI355X mapping.  One limb-polynomial of N u64 words is split into passes;
// a pass owns global stages [s0, s0+S) and works on independent
// sub-transforms of 2^S elements at stride N >> (s0+S):
//   N <= 2^14 : ONE pass, one residue per workgroup (2^14 x 8 B = 128 KiB in
//               LDS, 1024 threads) -- the north-star "one-residue-per-WG";
//   N  = 2^15..2^17 : two passes (column pass of stride N/2^S1, then row pass
//               of contiguous 2^S2 blocks), because a 512 KiB N=2^16 residue
//               exceeds the 160 KiB LDS of a CU.
// Inside a pass a workgroup holds W sub-transforms in LDS (coalesced 128 B
// row segments in and out); each thread keeps R = 16 elements in VGPRs and
// runs LOGR = 4 butterfly stages in registers between LDS exchanges.
#include "context.hpp"

namespace {

struct NttArgs {
  LimbMap map;
  const u64 *tw;         // [nmod][N], Montgomery form
  const ModInfo *mods;   // [nmod]
  const u64 *ninv;       // [nmod], N^-1 in Montgomery form
  u32 log_n;
  u32 s0;                // first global stage of this pass
  u32 log_stride;        // sub-transform element stride = 2^log_stride
  u32 last;              // canonicalise output (and scale by N^-1 for INTT)
};

template <int S>
__device__ __forceinline__ u32 lds_idx(u32 w, u32 k) {
  constexpr u32 SUB = 1u << S;
  constexpr u32 PAD = SUB + (SUB >> 4) + 1;
  return w * PAD + k + (k >> 4);
}

template <int S, int LOGR, int W, bool INV, bool COLS, bool SP>
__global__ void __launch_bounds__(W << (S - LOGR)) ntt_pass(NttArgs a) {
  constexpr int R = 1 << LOGR;
  constexpr int T = 1 << (S - LOGR);
  constexpr int NT = W * T;
  constexpr int NG = (S + LOGR - 1) / LOGR;
  constexpr int SUB = 1 << S;
  extern __shared__ u64 lds[];

  const u32 tid = threadIdx.x;
  const u32 e = blockIdx.y;
  const u32 cnt = a.map.cnt;
  const u32 poly = e / cnt, act = e - poly * cnt;
  const u32 limb = limbmap_limb(a.map, act);
  const u32 mod = a.map.mod_offset + limb;
  u64 *data = a.map.base + (((size_t)poly * a.map.poly_stride + limb) << a.log_n);
  const ModInfo mi = a.mods[mod];
  const u64 q = mi.q, q2 = 2 * q;
  const u64 *tw = a.tw + ((size_t)mod << a.log_n);
  const u32 stride = 1u << a.log_stride;

  // ---- coalesced global -> LDS load of the W sub-transforms of this block
  // element (w, k) of the tile = data[hi * 2^(S+ls) + k * stride + lo] with
  // sub-transform u = blockIdx.x * W + w, hi = u >> ls, lo = u & (stride-1)
#pragma unroll 4
  for (u32 idx = tid; idx < (u32)(W * SUB); idx += NT) {
    u32 w, k;
    if (COLS) { w = idx % W; k = idx / W; } else { w = idx / SUB; k = idx % SUB; }
    const u32 u = blockIdx.x * W + w;
    const size_t j = ((size_t)(u >> a.log_stride) << (S + a.log_stride)) + (size_t)k * stride +
                     (u & (stride - 1));
    lds[lds_idx<S>(w, k)] = data[j];
  }
  __syncthreads();

  u32 w, ts;
  if (COLS) { w = tid % W; ts = tid / W; } else { ts = tid % T; w = tid / T; }
  const u32 u = blockIdx.x * W + w;
  const u32 hi = u >> a.log_stride;

  u64 x[R];
#pragma unroll
  for (int gi = 0; gi < NG; ++gi) {
    const int g = INV ? NG - 1 - gi : gi;
    const int nb = (S - g * LOGR) < LOGR ? (S - g * LOGR) : LOGR;   // butterfly bits
    const int ex = LOGR - nb;                                      // extra register bits
    const int p = S - g * LOGR - nb;                               // lowest butterfly bit
    const u32 lo_t = ts & ((1u << p) - 1);
    const u32 hh = ts >> p;
    // k(r) = (hh << (p+nb+ex)) | (r_x << (p+nb)) | (r_b << p) | lo_t, r = (r_x << nb) | r_b
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const u32 rb = r & ((1 << nb) - 1), rx = r >> nb;
      const u32 k = (hh << (p + nb + ex)) | (rx << (p + nb)) | (rb << p) | lo_t;
      x[r] = lds[lds_idx<S>(w, k)];
    }
#pragma unroll
    for (int ti = 0; ti < nb; ++ti) {
      const int tau = INV ? nb - 1 - ti : ti;
      const u32 sigma = g * LOGR + tau;
      const u32 s = a.s0 + sigma;
      const int half = 1 << (nb - 1 - tau);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const u32 rb = r & ((1 << nb) - 1), rx = r >> nb;
        if (rb & half) continue;
        // top sigma bits of k for element r
        const u32 kk = ((((hh << ex) | rx) << tau) | (rb >> (nb - tau)));
        const u64 t = tw[(1u << s) + (hi << sigma) + kk];
        u64 &X = x[r];
        u64 &Y = x[r + half];
        if (!INV) {
          const u64 uu = X >= q2 ? X - q2 : X;
          const u64 v = mont_mul<SP>(Y, t, mi);
          X = uu + v;
          Y = uu - v + q2;
        } else {
          const u64 uu = X, vv = Y;
          const u64 sm = uu + vv;
          X = sm >= q2 ? sm - q2 : sm;
          Y = mont_mul<SP>(uu - vv + q2, t, mi);
        }
      }
    }
    if (gi == NG - 1 && a.last) {
      if (!INV) {
#pragma unroll
        for (int r = 0; r < R; ++r) x[r] = csub(csub(x[r], q2), q);
      } else {
        const u64 sc = a.ninv[mod];
#pragma unroll
        for (int r = 0; r < R; ++r) x[r] = csub(mont_mul<SP>(x[r], sc, mi), q);
      }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const u32 rb = r & ((1 << nb) - 1), rx = r >> nb;
      const u32 k = (hh << (p + nb + ex)) | (rx << (p + nb)) | (rb << p) | lo_t;
      lds[lds_idx<S>(w, k)] = x[r];
    }
    __syncthreads();
  }

  // ---- LDS -> global, coalesced
#pragma unroll 4
  for (u32 idx = tid; idx < (u32)(W * SUB); idx += NT) {
    u32 w2, k;
    if (COLS) { w2 = idx % W; k = idx / W; } else { w2 = idx / SUB; k = idx % SUB; }
    const u32 u2 = blockIdx.x * W + w2;
    const size_t j = ((size_t)(u2 >> a.log_stride) << (S + a.log_stride)) + (size_t)k * stride +
                     (u2 & (stride - 1));
    data[j] = lds[lds_idx<S>(w2, k)];
  }
}

template <int S, int W, bool COLS, bool INV, bool SP>
int launch_one(fhe_ctx *c, const NttArgs &a, u32 n_jobs) {
  constexpr int LOGR = 4;
  constexpr int NT = W << (S - LOGR);
  constexpr size_t SUB = 1u << S;
  constexpr size_t lds = (size_t)W * (SUB + (SUB >> 4) + 1) * sizeof(u64);
  const u32 subs = 1u << (a.log_n - S);
  dim3 grid(subs / W, n_jobs);
  auto k = ntt_pass<S, LOGR, W, INV, COLS, SP>;
  if (lds > 64 * 1024) (void)hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(k, grid, dim3(NT), lds, c->stream, a);
  return fhe_check(c, hipGetLastError(), "ntt_pass launch");
}

template <int S, int W, bool COLS>
int launch_pass(fhe_ctx *c, const NttArgs &a, bool inv, u32 n_jobs) {
  if (c->special)
    return inv ? launch_one<S, W, COLS, true, true>(c, a, n_jobs) : launch_one<S, W, COLS, false, true>(c, a, n_jobs);
  return inv ? launch_one<S, W, COLS, true, false>(c, a, n_jobs) : launch_one<S, W, COLS, false, false>(c, a, n_jobs);
}

// one pass over a whole residue (N <= 2^14)
int single_pass(fhe_ctx *c, NttArgs a, bool inv, u32 n_jobs) {
  a.s0 = 0;
  a.log_stride = 0;
  a.last = 1;
  switch (a.log_n) {
    case 10: return launch_pass<10, 1, false>(c, a, inv, n_jobs);
    case 11: return launch_pass<11, 1, false>(c, a, inv, n_jobs);
    case 12: return launch_pass<12, 1, false>(c, a, inv, n_jobs);
    case 13: return launch_pass<13, 1, false>(c, a, inv, n_jobs);
    case 14: return launch_pass<14, 1, false>(c, a, inv, n_jobs);
  }
  return fhe_fail(c, FHE_ERR_UNSUPPORTED, "single_pass: log_n");
}

// column pass: stages [0, S1), stride N >> S1
int col_pass(fhe_ctx *c, NttArgs a, bool inv, u32 n_jobs, bool last) {
  a.s0 = 0;
  a.last = last;
  switch (a.log_n) {
    case 15: a.log_stride = 15 - 7; return launch_pass<7, 32, true>(c, a, inv, n_jobs);
    case 16: a.log_stride = 16 - 8; return launch_pass<8, 16, true>(c, a, inv, n_jobs);
    case 17: a.log_stride = 17 - 8; return launch_pass<8, 16, true>(c, a, inv, n_jobs);
  }
  return fhe_fail(c, FHE_ERR_UNSUPPORTED, "col_pass: log_n");
}

// row pass: stages [S1, logN), contiguous blocks
int row_pass(fhe_ctx *c, NttArgs a, bool inv, u32 n_jobs, bool last) {
  a.log_stride = 0;
  a.last = last;
  switch (a.log_n) {
    case 15: a.s0 = 7; return launch_pass<8, 16, false>(c, a, inv, n_jobs);
    case 16: a.s0 = 8; return launch_pass<8, 16, false>(c, a, inv, n_jobs);
    case 17: a.s0 = 8; return launch_pass<9, 8, false>(c, a, inv, n_jobs);
  }
  return fhe_fail(c, FHE_ERR_UNSUPPORTED, "row_pass: log_n");
}

}  // namespace

int ntt_launch(fhe_ctx *c, const LimbMap &m, bool inverse) {
  const u32 n_jobs = m.n_polys * m.cnt;
  if (n_jobs == 0) return FHE_OK;
  if (n_jobs > 65535u) {
    // split along polys to respect gridDim.y
    u32 per = 65535u / m.cnt;
    for (u32 p0 = 0; p0 < m.n_polys; p0 += per) {
      LimbMap sub = m;
      sub.base = m.base + (size_t)p0 * m.poly_stride * c->n;
      sub.n_polys = (m.n_polys - p0) < per ? (m.n_polys - p0) : per;
      int rc = ntt_launch(c, sub, inverse);
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
  if (c->log_n <= 14) return single_pass(c, a, inverse, n_jobs);
  int rc;
  if (!inverse) {
    rc = col_pass(c, a, false, n_jobs, false);
    if (rc) return rc;
    return row_pass(c, a, false, n_jobs, true);
  }
  rc = row_pass(c, a, true, n_jobs, false);
  if (rc) return rc;
  return col_pass(c, a, true, n_jobs, true);
}
