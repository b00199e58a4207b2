// modarith.hpp -- 64-bit modular arithmetic for gfx950 (device) and host.
//
// gfx950 has no 64x64 multiplier: a u64 product is emulated with 32-bit
// v_mul_hi_u32 / v_mad_u64_u32, both quarter rate (measured:
// tools/microbench/intops.hip, ~20 T lane-ops/s each).  A Shoup constant
// multiply is ~10 such instructions; the backend therefore uses
//   - Shoup multiplication for every constant operand (twiddles, CRT
//     constants), lazy in [0, 2q);
//   - 128-bit Barrett (mu = floor(2^128/q)) only for variable x variable
//     products and for reducing lazily accumulated 128-bit dot products.
// All moduli satisfy q < 2^62 so [0, 4q) lazy values fit a u64.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint64_t u64;
typedef uint32_t u32;

#define HD __host__ __device__ __forceinline__

struct alignas(16) Tw {  // twiddle and its Shoup companion floor(w*2^64/q)
  u64 w, ws;
};

struct ModInfo {
  u64 q;
  u64 mu_hi, mu_lo;  // floor(2^128 / q)
  u64 pad;
};

HD u64 mulhi64(u64 a, u64 b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __umul64hi(a, b);
#else
  return (u64)(((unsigned __int128)a * b) >> 64);
#endif
}

// Shoup: a*w mod q for any a < 2^64; result in [0, 2q)
HD u64 shoup_lazy(u64 a, u64 w, u64 ws, u64 q) {
  u64 qh = mulhi64(a, ws);
  return a * w - qh * q;
}
HD u64 shoup(u64 a, u64 w, u64 ws, u64 q) {
  u64 r = shoup_lazy(a, w, ws, q);
  return r >= q ? r - q : r;
}
HD u64 add_mod(u64 a, u64 b, u64 q) {
  u64 s = a + b;
  return s >= q ? s - q : s;
}
HD u64 sub_mod(u64 a, u64 b, u64 q) { return a >= b ? a - b : a + q - b; }
HD u64 csub(u64 a, u64 q) { return a >= q ? a - q : a; }

// 128-bit accumulator
struct U128 {
  u64 lo, hi;
};
HD void mac128(U128 &acc, u64 a, u64 b) {
  u64 lo = a * b, hi = mulhi64(a, b);
  u64 s = acc.lo + lo;
  acc.hi += hi + (s < lo);
  acc.lo = s;
}
HD U128 mul128(u64 a, u64 b) {
  U128 r;
  r.lo = a * b;
  r.hi = mulhi64(a, b);
  return r;
}

// Barrett reduction of x = hi*2^64 + lo, x < q*2^64, to [0, q).
// qt = floor(x*mu / 2^128) with all carries kept, so qt in {Q*-1, Q*} and a
// single conditional subtraction finishes.
HD u64 barrett128(u64 hi, u64 lo, u64 q, u64 mu_hi, u64 mu_lo) {
  u64 c = mulhi64(lo, mu_lo);
  u64 t0 = lo * mu_hi, t1 = mulhi64(lo, mu_hi);
  u64 s = t0 + c;
  u64 s_hi = t1 + (s < t0);
  u64 u0 = hi * mu_lo, u1 = mulhi64(hi, mu_lo);
  u64 s2 = s + u0;
  u64 carry = u1 + (s2 < s);
  u64 qt = hi * mu_hi + s_hi + carry;
  u64 r = lo - qt * q;
  return r >= q ? r - q : r;
}
HD u64 reduce128(U128 x, const ModInfo &m) { return barrett128(x.hi, x.lo, m.q, m.mu_hi, m.mu_lo); }
HD u64 mul_mod(u64 a, u64 b, const ModInfo &m) {
  U128 p = mul128(a, b);
  return barrett128(p.hi, p.lo, m.q, m.mu_hi, m.mu_lo);
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
