// ntt_convf.hip -- a base conversion between the column pass of an inverse NTT
// and the column pass of the forward NTT of its outputs, in one kernel (CONVF)
// (kernel templates: ntt_core.hpp)
//
// The fused key switch converts twice at the two-pass sizes: ModUp (the
// digit's 4 Q limbs of INTT(d2) -> the 12 other limbs of Q u P) and ModDown
// (the 4 P limbs of INTT(acc_P) -> the 12 Q limbs).  Unfused, the inverse
// NTT's column pass writes its scaled outputs (the conversion's sources) to
// HBM, and the conversion column pass (PRO_CONV) of every target workgroup
// reads the 4 source tiles back through L2, 4 loads per output word, each
// group of them one exposed L2 latency.  Here ONE workgroup per (column block,
// poly) runs the inverse column transform of each source limb's row-pass output
// into registers (the 4 sources, 64 words per thread), then for every target
// limb forms the conversion element-wise and runs the forward column transform,
// storing the column-pass intermediate the row-side kernels read (ksf_pass /
// ksp_fused_pass).  The sources never reach HBM; each is read once.
// Bit-exact with the unfused pair: the inverse column transform's butterflies
// and output scale, the conversion (dot_cols_sp60 / dot_cols) and the forward
// column transform are the same functions on the same values (the inverse
// pass's last group layout is the forward pass's first, so no exchange between
// them).  A column's 256 elements span the workgroup's 4 waves, so every LDS
// exchange is fenced by a barrier on both sides.
#include "ntt_core.hpp"

// Built, bit-exact (GPU suite parity green) and rejected on measurement
// (profiles/r06/ab_convf.txt): the 4 sources (64 words per thread) plus a
// transform do not fit 2 waves per SIMD (110-140 VGPRs spill: ct-mult -19%),
// and at 1 wave (365 VGPRs) the L2 and HBM latencies it was to save are
// exposed instead (-2.4%; the 4 launches take what the 4 passes they replace
// took).  Off: CONVF=1 enables it.
#ifndef CONVF
#define CONVF 0
#endif
#ifndef CONVF_MINW
#define CONVF_MINW 1  // minimum waves per SIMD (2: the 4 sources hold 128 VGPRs and ~120 more spill)
#endif
#ifndef CONVF_LSW
#define CONVF_LSW 8  // butterflies per lock-step chunk (run_group LSW)
#endif

#if CONVF
namespace {

// a loop unrolled by construction (as ntt_ksf.hip's sfor): the unroll pragma
// gives up on the source loop's body for size, and a rolled loop indexes the
// source registers dynamically, which puts them in scratch
template <class F, int... I>
__device__ __forceinline__ void cf_for_impl(F &&f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void cf_for(F &&f) {
  cf_for_impl(f, std::make_integer_sequence<int, N>{});
}

template <int LOG_N, int S, int W, int NS, bool SP>
__global__ void __launch_bounds__(W << (S - 4), CONVF_MINW) convf_pass(ConvfArgs a) {
  constexpr int LOGR = 4, R = 16, LS = LOG_N - S;
  static_assert((S + LOGR - 1) / LOGR == 2, "two groups per column transform");
  static_assert(CONV_COLS, "the column-sum conversion (PRO_CONV's)");
  using G0 = Grp<S, LOGR, 0>;
  using G1 = Grp<S, LOGR, 1>;
  extern __shared__ u64 lds[];
  // the column-pass geometry of ntt_pass (COLS): W adjacent columns per
  // workgroup on adjacent lanes, so every wave access is 128 B row segments
  const u32 tid = threadIdx.x, bx = blockIdx.x, poly = blockIdx.y;
  const u32 w = tid % W, ts = tid / W;
  const u32 u = bx * W + w, hi = u >> LS;
  const u32 gb = (hi << (S + LS)) + (u & ((1u << LS) - 1));
  const u32 v1 = (gb + (G1::k_thr(ts) << LS)) << 3;  // group-1 layout: the inverse's input, the forward's output

  // one exchange between the groups of a column transform
  const auto xchg = [&](u64 (&x)[R], auto from, auto to) __attribute__((always_inline)) {
    using GA = Grp<S, LOGR, decltype(from)::value>;
    using GB = Grp<S, LOGR, decltype(to)::value>;
    __syncthreads();  // the previous transform's readers of the tile are done
    const u32 lw = lds_idx<S>(w, GA::k_thr(ts));
#pragma unroll
    for (int r = 0; r < R; ++r) lds[lw + GA::k_reg(r) + lds_pad(GA::k_reg(r))] = x[r];
    __syncthreads();
    const u32 lr = lds_idx<S>(w, GB::k_thr(ts));
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const u32 kr = GB::k_reg(r);
      x[r] = lds[lr + kr + lds_pad(kr)];
    }
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;

  // 1. the sources: the inverse column pass of each source limb, with its
  //    output scale (the conversion's source constants), kept in registers
  u64 v[NS][R];
  cf_for<NS>([&](auto I) __attribute__((always_inline)) {
    constexpr int i = decltype(I)::value;
    // scheduling fences: left free, the compiler hoists the next source's
    // loads and twiddles above this transform and spills
    __builtin_amdgcn_sched_barrier(0);
    const u32 ms = a.src_mod0 + i;
    const ModInfo mi = a.mods[ms];
    const u64 *tw = a.twi + ((size_t)ms << LOG_N);
    const u64 *d = a.src + (((size_t)poly * a.src_stride + a.src_first + i) << LOG_N);
    u64 t[16];
    G1::template load_tw<0>(t, tw, hi, ts);
#pragma unroll
    for (int r = 0; r < R; ++r) v[i][r] = ld_d(d + ((size_t)G1::k_reg(r) << LS), v1);
    run_group<S, LOGR, 1, 0, true, SP, false, CONVF_LSW>(v[i], t, 2 * mi.q, mi);
    xchg(v[i], I1{}, I0{});
    G0::template load_tw<0>(t, tw, hi, ts);
    run_group<S, LOGR, 0, 0, true, SP, false, CONVF_LSW>(v[i], t, 2 * mi.q, mi);
    u64 nq1 = 0 - uniform64(mi.q);
    asm("" : "+s"(nq1));
    const u64 sc = a.scale[ms];
#pragma unroll
    for (int r = 0; r < R; ++r) v[i][r] = harvey_csub(mont_mul<SP>(v[i][r], sc, mi), nq1);
    __builtin_amdgcn_sched_barrier(0);
  });

  // 2. every target: the conversion (PRO_CONV's), then the forward column pass
  const auto target = [&](auto wide, u32 act, const ModInfo &mi, const u64 *tw, u64 *dst) __attribute__((always_inline)) {
    constexpr bool WIDE = decltype(wide)::value;
    __builtin_amdgcn_sched_barrier(0);
    u32 hc0[NS], hc1[NS];  // the constants' 31-bit digits (uniform)
#pragma unroll
    for (int i = 0; i < NS; ++i) split31(a.h[(size_t)i * a.nd + act], hc0[i], hc1[i]);
    const bool sp60 = SP && CONV_SP60 && (WIDE || a.src60);
    u64 t[16];
    G0::template load_tw<0>(t, tw, hi, ts);
    u64 x[R];
    cf_for<R>([&](auto Rr) __attribute__((always_inline)) {
      constexpr int r = decltype(Rr)::value;
      u64 sv[NS];
#pragma unroll
      for (int i = 0; i < NS; ++i) sv[i] = v[i][r];
      x[r] = sp60 ? dot_cols_sp60<NS>(sv, hc0, hc1, mi.q_hi) : dot_cols<NS, SP>(sv, hc0, hc1, mi);
      if constexpr ((r & 3) == 3) __builtin_amdgcn_sched_barrier(0);  // 4 conversions at a time
    });
    run_group<S, LOGR, 0, 0, false, SP, WIDE, CONVF_LSW>(x, t, 2 * mi.q, mi);
    xchg(x, I0{}, I1{});
    G1::template load_tw<0>(t, tw, hi, ts);
    run_group<S, LOGR, 1, 0, false, SP, WIDE, CONVF_LSW>(x, t, 2 * mi.q, mi);
#pragma unroll
    for (int r = 0; r < R; ++r) st_d(dst + ((size_t)G1::k_reg(r) << LS), v1, x[r]);
    __builtin_amdgcn_sched_barrier(0);
  };
#pragma nounroll
  for (u32 act = 0; act < a.tmap.cnt; ++act) {
    const u32 limb = limbmap_limb(a.tmap, act);
    const u32 mt = a.tmap.mod_offset + limb;
    const ModInfo mi = a.mods[mt];
    const u64 *tw = a.twf + ((size_t)mt << LOG_N);
    u64 *dst = a.tmap.base + (((size_t)poly * a.tmap.poly_stride + limb) << LOG_N);
    // the lazy schedule of the target's class (a uniform branch, as ntt_pass WM = 2)
    if (mi.q < (1ull << 60)) target(std::true_type{}, act, mi, tw, dst);
    else target(std::false_type{}, act, mi, tw, dst);
  }
}

template <int LOG_N, int S, int W, int NS>
int convf_launch(fhe_ctx *c, const ConvfArgs &a, u32 n_polys) {
  constexpr size_t lds = lds_bytes<S, W>();
  const dim3 grid((1u << (LOG_N - S)) / W, n_polys);
  auto k = c->special ? convf_pass<LOG_N, S, W, NS, true> : convf_pass<LOG_N, S, W, NS, false>;
  if (lds > 64 * 1024) (void)hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(k, grid, dim3(W << (S - 4)), lds, c->stream, a);
  return fhe_check(c, hipGetLastError(), "convf_pass launch");
}

}  // namespace
#endif  // CONVF

// CONVF applies: the fused key switch's sizes (N = 2^16: 256-point columns in
// two groups; 2^15's 128-point columns take the same kernel) and 4 sources
bool convf_ok(const fhe_ctx *c, u32 ns) { return CONVF && (c->log_n == 15 || c->log_n == 16) && ns == 4; }

int ntt_convf_launch(fhe_ctx *c, const ConvfArgs &a, u32 ns) {
  if (!convf_ok(c, ns)) return fhe_fail(c, FHE_ERR_UNSUPPORTED, "fused conversion: shape");
#if CONVF
  const u32 per = 65535u;  // gridDim.y
  for (u32 p0 = 0; p0 < a.tmap.n_polys; p0 += per) {
    ConvfArgs b = a;
    const u32 np = std::min(per, a.tmap.n_polys - p0);
    b.src = a.src + (size_t)p0 * a.src_stride * c->n;
    b.tmap.base = a.tmap.base + (size_t)p0 * a.tmap.poly_stride * c->n;
    b.tmap.n_polys = np;
    const int rc = c->log_n == 16 ? convf_launch<16, 8, 16, 4>(c, b, np) : convf_launch<15, 7, 32, 4>(c, b, np);
    if (rc) return rc;
  }
#endif
  return FHE_OK;
}
