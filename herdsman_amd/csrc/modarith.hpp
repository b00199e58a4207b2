// modarith.hpp -- 64-bit modular arithmetic for gfx950 (device) and host.
//
// gfx950 has no 64x64 multiplier: every u64 product is built from 32x32->64
// v_mad_u64_u32 (half the issue rate of a 32-bit add, tools/microbench/
// valu64.hip), so the multiply count per modular product is the figure of
// merit, and the backend is built on Montgomery arithmetic with R = 2^64:
//   * mul128(a, b): the 128-bit product from exactly 4 v_mad_u64_u32;
//   * mont_reduce(T) = T * 2^-64 mod q in [0, 2q) for T < q * 2^64:
//       - "special" moduli q = 1 (mod 2^32) (the backend's default prime
//         family, still NTT-friendly for every N <= 2^31): q' = -q^-1 = -1 mod
//         2^32, so each of the two 32-bit Montgomery rounds needs ONE
//         v_mad_u64_u32 (m * q_hi) -- 2 multiplies in total;
//       - generic odd moduli (explicit OpenFHE-style primes): two 32-bit
//         rounds with q' = -q^-1 mod 2^32, 4 v_mad_u64_u32 + 2 v_mul_lo_u32
//         (mont_reduce, used after the 128-bit sums of the dot products; the
//         host keeps one 64-bit round); a single product interleaves the same
//         rounds with the operand words (mont_mul_gen: 8 + 2 multiplies);
//   * every constant operand (twiddles, CRT constants, N^-1, P^-1) is stored
//     pre-multiplied by R, so mont_mul(x, cR) = x * c exactly: a twiddle
//     multiply costs 4 + 2 = 6 multiplies (Shoup needs 10);
//   * dot products sum 128-bit products and reduce once; their constants are
//     pre-scaled so the R^-1 of the single reduction cancels.
// All moduli are < 2^61, so lazy values in [0, 4q) and the sums below stay
// inside the Montgomery bound T < q * 2^64.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint64_t u64;
typedef uint32_t u32;

#define HD __host__ __device__ __forceinline__

#ifndef GEN_RED_CIOS
#define GEN_RED_CIOS 1  // generic mont_reduce on the device: two 32-bit rounds (0: one 64-bit round)
#endif

struct ModInfo {
  u64 q;
  u64 qinv_neg;  // -q^-1 mod 2^64 (generic Montgomery)
  u64 r2;        // R^2 mod q  (mont_mul(x, r2) = x * R)
  u32 q_hi;      // q >> 32 (special Montgomery, q = q_hi * 2^32 + 1)
  u32 special;   // q = 1 mod 2^32
};

struct U128 {
  u64 lo, hi;
};

HD u64 mulhi64(u64 a, u64 b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __umul64hi(a, b);
#else
  return (u64)(((unsigned __int128)a * b) >> 64);
#endif
}

// full 128-bit product from four 32x32->64 multiply-adds
HD U128 mul128(u64 a, u64 b) {
#if defined(__HIP_DEVICE_COMPILE__)
  const u32 a0 = (u32)a, a1 = (u32)(a >> 32), b0 = (u32)b, b1 = (u32)(b >> 32);
  const u64 p00 = (u64)a0 * b0;
  const u64 p01 = (u64)a0 * b1 + (p00 >> 32);
  const u64 p10 = (u64)a1 * b0 + (u32)p01;
  const u64 p11 = (u64)a1 * b1 + (p01 >> 32) + (p10 >> 32);
  return U128{(p10 << 32) | (u32)p00, p11};
#else
  unsigned __int128 p = (unsigned __int128)a * b;
  return U128{(u64)p, (u64)(p >> 64)};
#endif
}

HD void add128(U128 &acc, const U128 &x) {
  const u64 s = acc.lo + x.lo;
  acc.hi += x.hi + (s < x.lo);
  acc.lo = s;
}
HD void mac128(U128 &acc, u64 a, u64 b) { add128(acc, mul128(a, b)); }

// T * 2^-64 mod q, result in [0, 2q); requires T < q * 2^64.
template <bool SP>
HD u64 mont_reduce(U128 T, const ModInfo &m) {
  if (SP) {
    // round 1: t0 = T mod 2^32, mq = -t0, T1 = (T >> 32) + (t0 != 0) + mq * q_hi
    const u32 t0 = (u32)T.lo;
    const u64 M = (u64)(0u - t0) * m.q_hi + (t0 != 0);  // < 2^61
    const u64 s = (T.hi << 32) | (T.lo >> 32);          // bits 32..95 of T
    const u64 r = s + M;
    const u32 top = (u32)(T.hi >> 32) + (r < s);        // bits 96..127 of T1
    // round 2 on T1 = top:r
    const u32 t1 = (u32)r;
    const u64 M2 = (u64)(0u - t1) * m.q_hi + (t1 != 0);
    return (((u64)top << 32) | (r >> 32)) + M2;
  } else {
#if defined(__HIP_DEVICE_COMPILE__) && GEN_RED_CIOS
    // two 32-bit Montgomery rounds, quotient digit m_k = t_k q' mod 2^32:
    // 2 v_mul_lo_u32 + 4 v_mad_u64_u32 (the 64-bit round: 3 for the quotient
    // + 4 for its high product).  T1 = (T + m0 q) / 2^32 < q (2^32 + 1) is 96
    // bits wide; T2 = (T1 + m1 q) / 2^32 < 2q.
    const u32 q0 = (u32)m.q, q1 = (u32)(m.q >> 32), qi = (u32)m.qinv_neg;
    const u32 t0 = (u32)T.lo;
    const u32 m0 = t0 * qi;
    const u64 A = (u64)m0 * q0 + t0;  // low word 0
    const u64 B = (u64)m0 * q1 + ((T.lo >> 32) + (A >> 32));
    const u64 sh = T.hi << 32;
    const u64 L1 = B + sh;
    const u32 H1 = (u32)(T.hi >> 32) + (L1 < sh);
    const u32 t1 = (u32)L1;
    const u32 m1 = t1 * qi;
    const u64 A2 = (u64)m1 * q0 + t1;
    const u64 B2 = (u64)m1 * q1 + ((L1 >> 32) + (A2 >> 32));
    return B2 + ((u64)H1 << 32);
#else
    const u64 mm = T.lo * m.qinv_neg;
    return T.hi + mulhi64(mm, m.q) + (T.lo != 0);
#endif
  }
}

// Special-modulus Montgomery product by word-serial CIOS: a < 2^63, b < q < 2^61,
// q = q_hi * 2^32 + 1.  Six v_mad_u64_u32, two v_not and no 64-bit add: the
// bounds a_hi < 2^31 and b_hi < 2^29 keep every partial sum below 2^64.
// Returns a*b*2^-64 mod q in [0, 1.5q).
//  * round 1 uses m0 = -P.lo mod 2^32; its "+ (P.lo != 0)" carry is folded into
//    the multiply-add that produces the word: P' = a0 b0 + (2^32 - 1) has
//    P'.hi = P.hi + (P.lo != 0) and ~P'.lo = m0;
//  * round 2 uses the integer multiplier m1 = ~X.lo + 1 in [1, 2^32] (still
//    = -X.lo mod 2^32, so X + m1 q is divisible by 2^32 and the quotient is
//    X.hi + 1 + ~X.lo q_hi + q_hi): its constant 1 + q_hi rides in the HIGH
//    word of round 1's 64-bit addend pair {P'.hi, 1 + q_hi}, which otherwise
//    holds a zero register -- the carry costs no instruction at all.
// OPAQUE keeps the compiler from rewriting ~P'.lo back into a (slow)
// v_mul_lo_u32 of the operands and from re-associating the mad chains.
#if defined(__HIP_DEVICE_COMPILE__)
#define OPAQUE(x) asm("" : "+v"(x))
#else
#define OPAQUE(x) (void)0
#endif
HD u64 mont_mul_sp(u64 a, u64 b, u32 q_hi) {
  const u32 a0 = (u32)a, a1 = (u32)(a >> 32), b0 = (u32)b, b1 = (u32)(b >> 32);
  const u64 csh = (u64)(q_hi + 1) << 32;
  u64 P = (u64)a0 * b0 + 0xFFFFFFFFull;
  OPAQUE(P);
  u64 V = (u64)(~(u32)P) * q_hi + ((u64)a1 * b0 + ((P >> 32) | csh));  // (a b0 + m0 q) / 2^32 + (1 + q_hi) 2^32
  OPAQUE(V);
  u64 X0 = (u64)a0 * b1 + V;
  OPAQUE(X0);
  return (u64)(~(u32)X0) * q_hi + ((u64)a1 * b1 + (X0 >> 32));
}

// M independent mont_mul_sp products written phase by phase, so the
// multiply chains of different products interleave in the instruction stream.
template <int M>
HD void mont_mul_sp_vec(u64 (&r)[M], const u64 (&a)[M], const u64 (&b)[M], u32 q_hi) {
  const u64 csh = (u64)(q_hi + 1) << 32;
  u64 t[M];
#pragma unroll
  for (int i = 0; i < M; ++i) {
    t[i] = (u64)(u32)a[i] * (u32)b[i] + 0xFFFFFFFFull;  // P'
    OPAQUE(t[i]);
  }
#pragma unroll
  for (int i = 0; i < M; ++i) {
    t[i] = (u64)(~(u32)t[i]) * q_hi + ((u64)(u32)(a[i] >> 32) * (u32)b[i] + ((t[i] >> 32) | csh));  // V
    OPAQUE(t[i]);  // keep the mad chain as written (no re-association into extra adds)
  }
#pragma unroll
  for (int i = 0; i < M; ++i) {
    t[i] = (u64)(u32)a[i] * (u32)(b[i] >> 32) + t[i];  // X
    OPAQUE(t[i]);
  }
#pragma unroll
  for (int i = 0; i < M; ++i)
    r[i] = (u64)(~(u32)t[i]) * q_hi + ((u64)(u32)(a[i] >> 32) * (u32)(b[i] >> 32) + (t[i] >> 32));
}

// Generic odd modulus q = q1 2^32 + q0 < 2^61: the same word-serial CIOS with
// a 32-bit quotient digit m_k = t_k q' (q' = -q^-1 mod 2^32, the low word of
// ModInfo::qinv_neg).  Eight v_mad_u64_u32 and two v_mul_lo_u32 (the 64-bit
// round of mont_reduce needs 11 multiplies and a carry compare).  Each column's
// carry out of the zeroed low word is W.hi of m_k q0 + t_k; with a1 < 2^31 and
// b1, q1 < 2^29 every partial sum stays below 2^64.  Returns a*b*2^-64 mod q
// in [0, 1.5q) for a < 2^63, b < q.
HD u64 mont_mul_gen(u64 a, u64 b, const ModInfo &m) {
  const u32 a0 = (u32)a, a1 = (u32)(a >> 32), b0 = (u32)b, b1 = (u32)(b >> 32);
  const u32 q0 = (u32)m.q, q1 = (u32)(m.q >> 32), qi = (u32)m.qinv_neg;
  u64 P = (u64)a0 * b0;
  OPAQUE(P);
  const u32 m0 = (u32)P * qi;
  u64 V = (u64)m0 * q1 + ((u64)a1 * b0 + (P >> 32));
  OPAQUE(V);
  V += ((u64)m0 * q0 + (u32)P) >> 32;  // (a b0 + m0 q) / 2^32
  OPAQUE(V);
  u64 X = (u64)a0 * b1 + V;
  OPAQUE(X);
  const u32 m1 = (u32)X * qi;
  u64 Y = (u64)m1 * q1 + ((u64)a1 * b1 + (X >> 32));
  OPAQUE(Y);
  return Y + (((u64)m1 * q0 + (u32)X) >> 32);
}

// M independent mont_mul_gen products phase by phase (as mont_mul_sp_vec), so
// the dependent chains of different products interleave
template <int M>
HD void mont_mul_gen_vec(u64 (&r)[M], const u64 (&a)[M], const u64 (&b)[M], const ModInfo &m) {
  const u32 q0 = (u32)m.q, q1 = (u32)(m.q >> 32), qi = (u32)m.qinv_neg;
  u64 P[M], V[M];
  u32 mk[M];
#pragma unroll
  for (int i = 0; i < M; ++i) {
    P[i] = (u64)(u32)a[i] * (u32)b[i];
    OPAQUE(P[i]);
  }
#pragma unroll
  for (int i = 0; i < M; ++i) mk[i] = (u32)P[i] * qi;
#pragma unroll
  for (int i = 0; i < M; ++i) {
    V[i] = (u64)mk[i] * q1 + ((u64)(u32)(a[i] >> 32) * (u32)b[i] + (P[i] >> 32));
    OPAQUE(V[i]);
  }
#pragma unroll
  for (int i = 0; i < M; ++i) {
    V[i] += ((u64)mk[i] * q0 + (u32)P[i]) >> 32;
    OPAQUE(V[i]);
  }
#pragma unroll
  for (int i = 0; i < M; ++i) {
    P[i] = (u64)(u32)a[i] * (u32)(b[i] >> 32) + V[i];  // X
    OPAQUE(P[i]);
  }
#pragma unroll
  for (int i = 0; i < M; ++i) mk[i] = (u32)P[i] * qi;
#pragma unroll
  for (int i = 0; i < M; ++i) {
    V[i] = (u64)mk[i] * q1 + ((u64)(u32)(a[i] >> 32) * (u32)(b[i] >> 32) + (P[i] >> 32));
    OPAQUE(V[i]);
  }
#pragma unroll
  for (int i = 0; i < M; ++i) r[i] = V[i] + (((u64)mk[i] * q0 + (u32)P[i]) >> 32);
}

template <bool SP>
HD u64 mont_mul(u64 a, u64 b, const ModInfo &m) {  // a*b*2^-64, [0,2q); a < 2^63, b < q
#if defined(__HIP_DEVICE_COMPILE__)
  if (SP) return mont_mul_sp(a, b, m.q_hi);
  return mont_mul_gen(a, b, m);
#endif
  return mont_reduce<SP>(mul128(a, b), m);
}

HD u64 csub(u64 a, u64 q) { return a >= q ? a - q : a; }
// the same for a, q < 2^63: the sign of a - q selects (a 64-bit add, a shift
// and two bitfield selects instead of a quarter-rate 64-bit compare, a borrow
// chain and two selects behind an s_nop hazard)
HD u64 csub63(u64 a, u64 q) {
#if defined(__HIP_DEVICE_COMPILE__)
  const u64 d = a - q;
  const u32 m = (u32)((int32_t)(u32)(d >> 32) >> 31);  // all ones iff a < q
  const u64 mm = ((u64)m << 32) | m;
  return (a & mm) | (d & ~mm);
#else
  return a >= q ? a - q : a;
#endif
}
HD u64 add_mod(u64 a, u64 b, u64 q) { return csub(a + b, q); }
HD u64 sub_mod(u64 a, u64 b, u64 q) { return a >= b ? a - b : a + q - b; }

// exact a*b mod q (canonical) for variable operands: (a*b/R) * R^2 / R
template <bool SP>
HD u64 mul_mod(u64 a, u64 b, const ModInfo &m) {
  return csub(mont_mul<SP>(mont_reduce<SP>(mul128(a, b), m), m.r2, m), m.q);
}
// exact (T mod q) for a 128-bit T < q * 2^64
template <bool SP>
HD u64 reduce128(U128 T, const ModInfo &m) {
  return csub(mont_mul<SP>(mont_reduce<SP>(T, m), m.r2, m), m.q);
}

// sum_{i < ns} v[i] * h[i * hs] * R^-1 mod m, exact and canonical, given
// canonical v[i] and constants h[i] < m (pre-scaled by the caller's power of R).
// Chunks of 4 terms:
//  - special moduli: one Montgomery product per term (each < 2m, so a chunk
//    sums below 8m < 2^64) and a 3-step conditional subtraction -- no 128-bit
//    carry chains (tools/microbench/dot.hip: 1.35x the 128-bit form);
//  - generic moduli: 128-bit sum (< q 2^64) and one Montgomery reduction.
template <int NS, bool SP>
HD u64 dot_mont(const u64 (&v)[NS], const u64 *h, size_t hs, u32 ns, const ModInfo &m) {
  u64 res = 0;
#pragma unroll
  for (int c0 = 0; c0 < NS; c0 += 4) {
    if (c0 < (int)ns) {
      u64 part;
      if (SP) {
        u64 sum = 0;
#pragma unroll
        for (int i = c0; i < c0 + 4 && i < NS; ++i)
          if (i < (int)ns) sum += mont_mul<SP>(v[i], h[(size_t)i * hs], m);
        part = csub63(csub63(csub(sum, 4 * m.q), 2 * m.q), m.q);  // sum < 6q may exceed 2^63
      } else {
        U128 acc{0, 0};
#pragma unroll
        for (int i = c0; i < c0 + 4 && i < NS; ++i)
          if (i < (int)ns) mac128(acc, v[i], h[(size_t)i * hs]);
        part = csub(mont_reduce<SP>(acc, m), m.q);
      }
      res = c0 == 0 ? part : csub63(res + part, m.q);  // both canonical
    }
  }
  return res;
}

// The same sum, left in the lazy range [0, 4q) (special moduli) or [0, 2q)
// (generic) -- the input range of the forward NTT (ntt.hip), so a conversion
// whose outputs are transformed next skips the last two (one) conditional
// subtractions; the residue is the same, the NTT's outputs are bit-identical.
// Q60: m < 2^60, so the lazy sums (< 8q) stay below 2^63 and the conditional
// subtractions can use the sign of a - q (csub63)
template <int NS, bool SP, bool Q60 = false>
HD u64 dot_mont_lazy(const u64 (&v)[NS], const u64 *h, size_t hs, u32 ns, const ModInfo &m) {
  u64 res = 0;
#pragma unroll
  for (int c0 = 0; c0 < NS; c0 += 4) {
    if (c0 < (int)ns) {
      u64 part;
      if (SP) {
        u64 sum = 0;  // <= 4 products below 1.5q each
#pragma unroll
        for (int i = c0; i < c0 + 4 && i < NS; ++i)
          if (i < (int)ns) sum += mont_mul<SP>(v[i], h[(size_t)i * hs], m);
        part = Q60 ? csub63(sum, 4 * m.q) : csub(sum, 4 * m.q);  // < 4q
        res = c0 == 0 ? part : Q60 ? csub63(res + part, 4 * m.q) : csub(res + part, 4 * m.q);
      } else {
        U128 acc{0, 0};
#pragma unroll
        for (int i = c0; i < c0 + 4 && i < NS; ++i)
          if (i < (int)ns) mac128(acc, v[i], h[(size_t)i * hs]);
        part = mont_reduce<SP>(acc, m);  // < 2q
        res = c0 == 0 ? part : csub(res + part, 2 * m.q);
      }
    }
  }
  return res;
}

// NS <= 4 canonical terms v_i < 2^61 (constants h_i < m < 2^61): the same
// sum as dot_mont_lazy by 31-bit column sums.  With v = v0 + v1 2^31
// (v0 < 2^31, v1 < 2^30: an and and a funnel shift) and h = h0 + h1 2^31 (split
// once per workgroup, uniform), every 32x32 partial product is below 2^62, so
// the three columns  C0 = sum v0 h0,  C1 = sum v0 h1 + v1 h0,  C2 = sum v1 h1
// accumulate in the 64-bit addend of v_mad_u64_u32 with no carries: 4 multiply-
// adds per term instead of the Montgomery product's 6 plus its lazy-sum adds
// and conditional subtractions.  T = C0 + C1 2^31 + C2 2^62 < 2^63 m is then
// reduced once (mont_reduce: [0, 2q); generic moduli save the 128-bit
// accumulation's carry chains).
template <int NS, bool SP>
HD u64 dot_cols(const u64 (&v)[NS], const u32 (&h0)[NS], const u32 (&h1)[NS], const ModInfo &m) {
  static_assert(NS >= 1 && NS <= 4, "column sums stay below 2^64 for at most 4 terms");
  u64 c0 = 0, c1 = 0, c2 = 0;
#pragma unroll
  for (int i = 0; i < NS; ++i) {
    const u32 v0 = (u32)v[i] & 0x7FFFFFFFu, v1 = (u32)(v[i] >> 31);
    c0 += (u64)v0 * h0[i];
    c1 += (u64)v0 * h1[i];
    c1 += (u64)v1 * h0[i];
    c2 += (u64)v1 * h1[i];
  }
  const u64 lo1 = c0 + (c1 << 31);
  const u64 lo = lo1 + (c2 << 62);
  const u64 hi = (c1 >> 33) + (c2 >> 2) + (lo1 < c0) + (lo < lo1);
  return mont_reduce<SP>(U128{lo, hi}, m);
}
// The same sum for a special modulus m = mh 2^32 + 1 < 2^61 where one side of
// every product is below 2^60 (m < 2^60, or sources v < 2^60: then v1 < 2^29
// or h1 < 2^29, and C1 stays below 2^64; result < 1.25m): the
// reduction runs on the columns themselves, as Montgomery rounds of 31, 31
// and 2 bits (m = 1 mod 2^31, so each quotient digit is -t mod 2^k and its
// multiple of m is u (m >> k) 2^k + u): C0 is folded into C1's accumulator, C1
// into C2's, with no 128-bit combine.  Each accumulator starts at 2^k - 1, so
// its top (acc >> k) already carries the round's "+ [t != 0]" and the digit is
// ~acc mod 2^k.  Bounds: C1 < 7 2^61 < 2^64, C2 < 2^62; result < 1.25m.
template <int NS>
HD u64 dot_cols_sp60(const u64 (&v)[NS], const u32 (&h0)[NS], const u32 (&h1)[NS], u32 q_hi) {
  static_assert(NS >= 1 && NS <= 4, "column sums stay below 2^64 for at most 4 terms");
  u32 v0[NS], v1[NS];
#pragma unroll
  for (int i = 0; i < NS; ++i) v0[i] = (u32)v[i] & 0x7FFFFFFFu, v1[i] = (u32)(v[i] >> 31);
  const u32 mh2 = q_hi << 1;  // m >> 31
  u64 c = 0x7FFFFFFFull;
#pragma unroll
  for (int i = 0; i < NS; ++i) c += (u64)v0[i] * h0[i];
  u32 u = ~(u32)c & 0x7FFFFFFFu;
  c = (u64)u * mh2 + ((c >> 31) + 0x7FFFFFFFull);
#pragma unroll
  for (int i = 0; i < NS; ++i) {
    c += (u64)v0[i] * h1[i];
    c += (u64)v1[i] * h0[i];
  }
  u = ~(u32)c & 0x7FFFFFFFu;
  c = (u64)u * mh2 + ((c >> 31) + 3);
#pragma unroll
  for (int i = 0; i < NS; ++i) c += (u64)v1[i] * h1[i];
  const u32 u2 = ~(u32)c & 3u;
  return (u64)(u2 << 30) * q_hi + (c >> 2);  // m >> 2 = q_hi 2^30
}

HD void split31(u64 h, u32 &h0, u32 &h1) {
  h0 = (u32)h & 0x7FFFFFFFu;
  h1 = (u32)(h >> 31);
}

// dot_mont's canonical sum (same arguments) by column sums over chunks of 4
// terms, each reduced once; constants are split where they are read (uniform
// operands: scalar instructions).  Terms past ns contribute zero digits.
template <int NS, bool SP>
HD u64 dot_cols_canon(const u64 (&v)[NS], const u64 *h, size_t hs, u32 ns, const ModInfo &m) {
  u64 res = 0;
#pragma unroll
  for (int c0 = 0; c0 < NS; c0 += 4) {
    if (c0 < (int)ns) {
      u64 vv[4];
      u32 h0[4], h1[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bool on = c0 + i < NS && c0 + i < (int)ns;
        vv[i] = on ? v[c0 + i < NS ? c0 + i : 0] : 0;
        if (on) split31(h[(size_t)(c0 + i) * hs], h0[i], h1[i]);
        else h0[i] = h1[i] = 0;
      }
      const u64 part = csub63(dot_cols<4, SP>(vv, h0, h1, m), m.q);
      res = c0 == 0 ? part : csub63(res + part, m.q);
    }
  }
  return res;
}

// SplitMix64 stream shared with the oracle (orc_fill_uniform)
HD u64 splitmix64(u64 z) {
  z ^= z >> 30;
  z *= 0xBF58476D1CE4E5B9ull;
  z ^= z >> 27;
  z *= 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
HD u64 stream_word(u64 seed, u64 w) { return splitmix64(seed + (w + 1) * 0x9E3779B97F4A7C15ull); }
