// Field64 / Field128 arithmetic for gfx950 (CDNA4), Montgomery multiplication built from
// v_mad_u64_u32 chains.  Replaces prio 0.15.1 `src/fp.rs` / `src/field.rs` (ext crate, called from
// the Prio3 prepare path at aggregator/src/aggregator.rs:1777-1786).
//
// Values are stored CANONICALLY (the DAP little-endian encoding is the storage format).  Constants
// derived inside kernels (roots of unity, powers of t / r, Lagrange weights) are kept in Montgomery
// form (x*R), so   mul(mont_const, canonical) == canonical product   and no conversions are needed
// on the data path.
//
//   Field64 : p = 2^64 - 2^32 + 1,        R = 2^64,  -p^-1 mod 2^32 = 0xFFFFFFFF
//   Field128: p = 2^128 - 28*2^64 + 1,    R = 2^128, -p^-1 mod 2^32 = 0xFFFFFFFF
// Both primes are == 1 mod 2^32, so each CIOS reduction word is m = -t0 and the m*p[0] product
// vanishes; the zero limbs of p fold away at compile time.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "inv128.h"

#define DEVI __device__ __forceinline__

struct F128 {
  uint32_t w[4];
};
struct F64 {
  uint32_t w[2];
};
#include "modadd.h"  // f128_add_chain / f128_sub_chain / f128_mont_mul1 (generated)

#ifndef P3G_ADD_CPP
#define P3G_ADD_CPP 0  // A/B: 1 = Field128 add / sub / mul in plain C++ (64-bit temporaries)
#endif

// ----------------------------------------------------------------------------------------------
// Field128
// ----------------------------------------------------------------------------------------------
struct Field128Ops {
  using T = F128;
  static constexpr int ES = 16;      // encoded size
  static constexpr int NW = 4;       // 32-bit limbs
  static constexpr uint32_t P0 = 1u, P1 = 0u, P2 = 0xFFFFFFE4u, P3 = 0xFFFFFFFFu;

  static DEVI F128 zero() { return F128{{0u, 0u, 0u, 0u}}; }
  // R mod p = 2^128 - p = 28*2^64 - 1  (Montgomery form of 1)
  static DEVI F128 one_mont() { return F128{{0xFFFFFFFFu, 0xFFFFFFFFu, 0x1Bu, 0u}}; }
  // R^2 mod p = 0x5587fffffffffffffcf1
  static DEVI F128 r2() { return F128{{0xFFFFFCF1u, 0xFFFFFFFFu, 0x5587u, 0u}}; }
  static DEVI F128 one() { return F128{{1u, 0u, 0u, 0u}}; }
  // (p+1)/2, canonical  (1/2)
  static DEVI F128 half() { return F128{{1u, 0u, 0xFFFFFFF2u, 0x7FFFFFFFu}}; }

  static DEVI bool is_canonical(const F128& a) {
    // a >= p = [1, 0, P2, P3]  <=>  w3 = P3 and (w2 > P2 or (w2 = P2 and (w1, w0) != 0)); written
    // without short-circuits so it compiles to lane-mask arithmetic, not divergent branches
    const bool top = a.w[3] == P3, gt2 = a.w[2] > P2, eq2 = a.w[2] == P2;
    const bool nz = (a.w[1] | a.w[0]) != 0u;
    return !(top & (gt2 | (eq2 & nz)));
  }
  static DEVI bool eq(const F128& a, const F128& b) {
    return ((a.w[0] ^ b.w[0]) | (a.w[1] ^ b.w[1]) | (a.w[2] ^ b.w[2]) | (a.w[3] ^ b.w[3])) == 0u;
  }
  static DEVI bool is_zero(const F128& a) { return (a.w[0] | a.w[1] | a.w[2] | a.w[3]) == 0u; }

  // a + b mod p.  With c = 2^128 - p = [FFFFFFFF, FFFFFFFF, 1B, 0]:
  //   s = a + b (carry k1);  u = s + c (carry k2);  result = (k1|k2) ? u : s.
  static DEVI F128 add(const F128& a, const F128& b) {
    if constexpr (!P3G_ADD_CPP) {
      F128 r;
      f128_add_chain(a, b, r);
      return r;
    }
    uint64_t t;
    uint32_t s0, s1, s2, s3, k1;
    t = (uint64_t)a.w[0] + b.w[0];            s0 = (uint32_t)t;
    t = (uint64_t)a.w[1] + b.w[1] + (t >> 32); s1 = (uint32_t)t;
    t = (uint64_t)a.w[2] + b.w[2] + (t >> 32); s2 = (uint32_t)t;
    t = (uint64_t)a.w[3] + b.w[3] + (t >> 32); s3 = (uint32_t)t; k1 = (uint32_t)(t >> 32);
    uint32_t u0, u1, u2, u3, k2;
    t = (uint64_t)s0 + 0xFFFFFFFFu;            u0 = (uint32_t)t;
    t = (uint64_t)s1 + 0xFFFFFFFFu + (t >> 32); u1 = (uint32_t)t;
    t = (uint64_t)s2 + 0x1Bu + (t >> 32);       u2 = (uint32_t)t;
    t = (uint64_t)s3 + (t >> 32);               u3 = (uint32_t)t; k2 = (uint32_t)(t >> 32);
    bool sel = (k1 | k2) != 0u;
    return F128{{sel ? u0 : s0, sel ? u1 : s1, sel ? u2 : s2, sel ? u3 : s3}};
  }
  // a - b mod p: d = a - b (borrow) ; if borrow: d += p
  static DEVI F128 sub(const F128& a, const F128& b) {
    if constexpr (!P3G_ADD_CPP) {
      F128 r;
      f128_sub_chain(a, b, r);
      return r;
    }
    int64_t t;
    uint32_t d0, d1, d2, d3;
    uint64_t u;
    u = (uint64_t)a.w[0] - b.w[0];                        d0 = (uint32_t)u; t = (int64_t)u >> 32;
    u = (uint64_t)a.w[1] - b.w[1] + (uint64_t)t;          d1 = (uint32_t)u; t = (int64_t)u >> 32;
    u = (uint64_t)a.w[2] - b.w[2] + (uint64_t)t;          d2 = (uint32_t)u; t = (int64_t)u >> 32;
    u = (uint64_t)a.w[3] - b.w[3] + (uint64_t)t;          d3 = (uint32_t)u; t = (int64_t)u >> 32;
    uint32_t m = (uint32_t)t;  // 0 or 0xFFFFFFFF
    // add p & m
    uint64_t c;
    c = (uint64_t)d0 + (P0 & m);            d0 = (uint32_t)c;
    c = (uint64_t)d1 + (P1 & m) + (c >> 32); d1 = (uint32_t)c;
    c = (uint64_t)d2 + (P2 & m) + (c >> 32); d2 = (uint32_t)c;
    c = (uint64_t)d3 + (P3 & m) + (c >> 32); d3 = (uint32_t)c;
    return F128{{d0, d1, d2, d3}};
  }
  static DEVI F128 neg(const F128& a) { return sub(zero(), a); }
  static DEVI F128 dbl(const F128& a) { return add(a, a); }

  // Montgomery product a*b*2^-128 mod p.  Inputs < p, output < p.
  // 256-bit product from 16 v_mad_u64_u32 (four 64x64 products), then a 2-step, 64-bit-word REDC
  // that needs no multiplier: p = 1 + (2^64 - 28) 2^64, so -p^-1 = -1 mod 2^64 (m = -t0) and
  // m * p / 2^64 = [ -28m (low word), +m (next word) ] after the exact division.
  static DEVI F128 mul(const F128& a, const F128& b) {
    if constexpr (!P3G_ADD_CPP) {
      F128 r;
      f128_mont_mul1(a, b, r);
      return r;
    }
    typedef unsigned __int128 u128;
    const uint64_t alo = ((uint64_t)a.w[1] << 32) | a.w[0], ahi = ((uint64_t)a.w[3] << 32) | a.w[2];
    const uint64_t blo = ((uint64_t)b.w[1] << 32) | b.w[0], bhi = ((uint64_t)b.w[3] << 32) | b.w[2];
    const u128 p00 = (u128)alo * blo, p01 = (u128)alo * bhi, p10 = (u128)ahi * blo,
               p11 = (u128)ahi * bhi;
    const uint64_t t0 = (uint64_t)p00;
    const u128 mid = (p00 >> 64) + (uint64_t)p01 + (uint64_t)p10;
    const uint64_t t1 = (uint64_t)mid;
    const u128 hi = (mid >> 64) + (p01 >> 64) + (p10 >> 64) + p11;
    const uint64_t t2 = (uint64_t)hi, t3 = (uint64_t)(hi >> 64);
    // REDC step 1
    uint64_t m = 0 - t0;
    u128 m28 = (u128)m * 28u;
    u128 w0 = (u128)t1 + (uint64_t)(t0 != 0);
    u128 x = (u128)t2 + m + ((u128)t3 << 64) + (w0 >> 64);
    uint64_t w0lo = (uint64_t)w0;
    uint64_t r0 = w0lo - (uint64_t)m28;
    x = x - (m28 >> 64) - (uint64_t)(w0lo < (uint64_t)m28);
    const uint64_t s0 = r0, s1 = (uint64_t)x, s2 = (uint64_t)(x >> 64);
    // REDC step 2
    m = 0 - s0;
    m28 = (u128)m * 28u;
    w0 = (u128)s1 + (uint64_t)(s0 != 0);
    x = (u128)s2 + m + (w0 >> 64);
    w0lo = (uint64_t)w0;
    r0 = w0lo - (uint64_t)m28;
    x = x - (m28 >> 64) - (uint64_t)(w0lo < (uint64_t)m28);
    // result (x:r0) < 2p
    u128 r = ((u128)(uint64_t)x << 64) | r0;
    const u128 P = ((u128)0xFFFFFFFFFFFFFFE4ull << 64) | 1u;
    if ((uint64_t)(x >> 64) != 0 || r >= P) r -= P;
    const uint64_t lo = (uint64_t)r, hh = (uint64_t)(r >> 64);
    return F128{{(uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hh, (uint32_t)(hh >> 32)}};
  }
  static DEVI F128 to_mont(const F128& a) { return mul(a, r2()); }
  static DEVI F128 from_mont(const F128& a) { return mul(a, one()); }

  static DEVI F128 load(const uint8_t* p) {
    const uint4 v = *reinterpret_cast<const uint4*>(p);
    return F128{{v.x, v.y, v.z, v.w}};
  }
  static DEVI void store(uint8_t* p, const F128& a) {
    *reinterpret_cast<uint4*>(p) = make_uint4(a.w[0], a.w[1], a.w[2], a.w[3]);
  }
  static DEVI F128 from_u64x2(uint64_t lo, uint64_t hi) {
    return F128{{(uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32)}};
  }
  static DEVI F128 from_u32(uint32_t x) { return F128{{x, 0u, 0u, 0u}}; }
};

// ----------------------------------------------------------------------------------------------
// Field64 (Goldilocks).  Used by Prio3Count only.
// ----------------------------------------------------------------------------------------------
struct Field64Ops {
  using T = F64;
  static constexpr int ES = 8;
  static constexpr int NW = 2;
  static constexpr uint32_t P0 = 1u, P1 = 0xFFFFFFFFu;

  static DEVI F64 zero() { return F64{{0u, 0u}}; }
  static DEVI F64 one_mont() { return F64{{0xFFFFFFFFu, 0u}}; }          // 2^64 mod p
  static DEVI F64 r2() { return F64{{0x00000001u, 0xFFFFFFFEu}}; }       // 2^128 mod p
  static DEVI F64 one() { return F64{{1u, 0u}}; }
  static DEVI F64 half() { return F64{{0x80000001u, 0x7FFFFFFFu}}; }      // (p+1)/2

  static DEVI uint64_t u(const F64& a) { return ((uint64_t)a.w[1] << 32) | a.w[0]; }
  static DEVI F64 mk(uint64_t x) { return F64{{(uint32_t)x, (uint32_t)(x >> 32)}}; }
  static constexpr uint64_t P = 0xFFFFFFFF00000001ull;

  static DEVI bool is_canonical(const F64& a) { return u(a) < P; }
  static DEVI bool eq(const F64& a, const F64& b) { return u(a) == u(b); }
  static DEVI bool is_zero(const F64& a) { return u(a) == 0ull; }
  static DEVI F64 add(const F64& a, const F64& b) {
    uint64_t x = u(a), y = u(b);
    uint64_t s = x + y;
    bool carry = s < x;
    uint64_t t = s + 0xFFFFFFFFull;  // s - p mod 2^64
    bool carry2 = t < s;
    return mk((carry || carry2) ? t : s);
  }
  static DEVI F64 sub(const F64& a, const F64& b) {
    uint64_t x = u(a), y = u(b);
    uint64_t d = x - y;
    return mk(x < y ? d + P : d);
  }
  static DEVI F64 neg(const F64& a) { return sub(zero(), a); }
  static DEVI F64 dbl(const F64& a) { return add(a, a); }
  static DEVI F64 mul(const F64& a, const F64& b) {
    uint32_t t0 = 0, t1 = 0, t2 = 0;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const uint32_t bi = b.w[i];
      uint64_t c;
      c = (uint64_t)a.w[0] * bi + t0;             t0 = (uint32_t)c;
      c = (uint64_t)a.w[1] * bi + t1 + (c >> 32); t1 = (uint32_t)c;
      c = (uint64_t)t2 + (c >> 32);
      t2 = (uint32_t)c;
      uint32_t t3 = (uint32_t)(c >> 32);
      const uint32_t m = 0u - t0;
      c = (uint64_t)m * P1 + t1 + (t0 != 0u ? 1u : 0u); t0 = (uint32_t)c;
      c = (uint64_t)t2 + (c >> 32);                     t1 = (uint32_t)c;
      t2 = t3 + (uint32_t)(c >> 32);
    }
    uint64_t r = ((uint64_t)t1 << 32) | t0;
    if (t2 != 0u || r >= P) r = r + 0xFFFFFFFFull;  // r - p mod 2^64
    return mk(r);
  }
  static DEVI F64 to_mont(const F64& a) { return mul(a, r2()); }
  static DEVI F64 from_mont(const F64& a) { return mul(a, one()); }
  static DEVI F64 load(const uint8_t* p) {
    const uint2 v = *reinterpret_cast<const uint2*>(p);
    return F64{{v.x, v.y}};
  }
  static DEVI void store(uint8_t* p, const F64& a) {
    *reinterpret_cast<uint2*>(p) = make_uint2(a.w[0], a.w[1]);
  }
  static DEVI F64 from_u32(uint32_t x) { return F64{{x, 0u}}; }
};

// Field128 inverse, Montgomery form in and out (0 -> 0): the canonical inverse y = (xR)^-1 by
// batched divsteps (inv128.h, ~6K simple ops), then one Montgomery product with R^3 mod p:
// y R^3 R^-1 = x^-1 R.  P3G_INV_EXP=1 selects the exponentiation x^(p-2) (an addition chain over
// p - 2 = [0xFFFFFFFFFFFFFFE3 | 0xFFFFFFFFFFFFFFFF] = 56 ones, 111000 11, 64 ones: 143 squarings
// + 12 multiplications), the form prio computes (same value).
#ifndef P3G_INV_EXP
#define P3G_INV_EXP 0
#endif
DEVI F128 sqn128(F128 x, int n) {
  for (int i = 0; i < n; ++i) x = Field128Ops::mul(x, x);
  return x;
}
DEVI F128 inv_mont128(const F128& x) {
  using FO = Field128Ops;
  if (!P3G_INV_EXP) {
    F128 y;
    inv128::inverse(x.w, y.w);
    return FO::mul(y, F128{{0xFFF6A82Fu, 0xFFFFFFFFu, 0x01054553u, 0u}});  // R^3 mod p
  }
  const F128 x2 = FO::mul(FO::mul(x, x), x);    // x^(2^2 - 1)
  const F128 x3 = FO::mul(FO::mul(x2, x2), x);  // 2^3 - 1
  const F128 x6 = FO::mul(sqn128(x3, 3), x3);
  const F128 x8 = FO::mul(sqn128(x6, 2), x2);
  const F128 x16 = FO::mul(sqn128(x8, 8), x8);
  const F128 x24 = FO::mul(sqn128(x16, 8), x8);
  const F128 x32 = FO::mul(sqn128(x16, 16), x16);
  const F128 x56 = FO::mul(sqn128(x32, 24), x24);
  const F128 x64 = FO::mul(sqn128(x56, 8), x8);
  F128 a = FO::mul(sqn128(x56, 3), x3);  // 59 ones
  a = sqn128(a, 3);                       // 000
  a = FO::mul(sqn128(a, 2), x2);          // 11
  return FO::mul(sqn128(a, 64), x64);     // 64 ones
}

// Montgomery-form power x^e (x in Montgomery form, result Montgomery form).
// x^(p - 2) for Field64 (Montgomery in, Montgomery out): p - 2 = (2^31 - 1) 2^33 + (2^32 - 1),
// an addition chain of 64 squarings + 9 multiplications (square-and-multiply: 64 + 63).
DEVI F64 inv_mont64(const F64& x) {
  using FO = Field64Ops;
  auto sqn = [](F64 a, int n) {
    for (int i = 0; i < n; ++i) a = FO::mul(a, a);
    return a;
  };
  const F64 x2 = FO::mul(FO::mul(x, x), x);  // x^(2^2 - 1)
  const F64 x3 = FO::mul(FO::mul(x2, x2), x);
  const F64 x6 = FO::mul(sqn(x3, 3), x3);
  const F64 x12 = FO::mul(sqn(x6, 6), x6);
  const F64 x24 = FO::mul(sqn(x12, 12), x12);
  const F64 x30 = FO::mul(sqn(x24, 6), x6);
  const F64 x31 = FO::mul(FO::mul(x30, x30), x);
  const F64 x32 = FO::mul(FO::mul(x31, x31), x);
  return FO::mul(sqn(x31, 33), x32);
}

template <class FO>
DEVI typename FO::T mont_pow(typename FO::T x, uint64_t e) {
  typename FO::T r = FO::one_mont();
  while (e) {
    if (e & 1) r = FO::mul(r, x);
    x = FO::mul(x, x);
    e >>= 1;
  }
  return r;
}
