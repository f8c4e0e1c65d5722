// Field128 inversion by batched Bernstein-Yang divsteps ("safegcd", half-delta form): 10 batches
// of 30 divsteps on the low 32 bits of (f, g), each batch's 2x2 transition matrix then applied to
// the full-precision (f, g) and to the Bezout coefficients (d, e) mod p in signed 30-bit limbs.
//
// prio 0.15.1 inverts Field128 elements by exponentiation x^(p-2) (src/fp.rs, ext crate); the
// FLP query reaches it once per report (the Lagrange-weight batch inversion, k_flp_weights; the
// Sum query's two denominators, k_flp_query_lane).  The result is the same field element; only
// the cost differs: 143 serial Montgomery squarings + 12 products (~22.6K VALU + ~9K hazard
// s_nops per lane) against ~6K simple 32-bit ops here, and no carry flags (all selects are
// arithmetic masks), so no VALU-carry wait states.
//
// 300 divsteps suffice for 128-bit inputs: the half-delta bound floor((45907 d + 26313) / 19929)
// = 296 for d = 128 (Bernstein-Yang, "Fast constant-time gcd computation and modular
// inversion", 2019, with the refined bound used by libsecp256k1's modinv32).  Written for the
// device and, for tests/test_inv128.py, the host (same source, g++).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define P3G_HD __host__ __device__ __forceinline__
#else
#define P3G_HD inline
#endif

namespace inv128 {

constexpr int32_t kM30 = 0x3FFFFFFF;
// p = 2^128 - 28 2^64 + 1 in signed 30-bit limbs (p^-1 = 1 mod 2^30: p == 1 mod 2^64)
constexpr int32_t kP[5] = {1, 0, 0x3FFFFE40, 0x3FFFFFFF, 0xFF};

struct Trans {
  int32_t u, v, q, r;
};

// 30 divsteps on the low 32 bits of f (odd) and g; returns the new zeta, fills t (entries scaled
// so that [f', g'] = t [f, g] / 2^30).
P3G_HD int32_t divsteps_30(int32_t zeta, uint32_t f, uint32_t g, Trans& t) {
  uint32_t u = 1, v = 0, q = 0, r = 1;
#pragma unroll
  for (int i = 0; i < 30; ++i) {
    const uint32_t c1 = (uint32_t)(zeta >> 31);  // zeta < 0
    const uint32_t c2 = 0u - (g & 1u);          // g odd
    const uint32_t x = (f ^ c1) - c1, y = (u ^ c1) - c1, z = (v ^ c1) - c1;
    g += x & c2;
    q += y & c2;
    r += z & c2;
    const uint32_t c3 = c1 & c2;  // zeta < 0 and g odd: swap
    zeta = (int32_t)(((uint32_t)zeta ^ c3) - 1u);
    f += g & c3;
    u += q & c3;
    v += r & c3;
    g >>= 1;
    u <<= 1;
    v <<= 1;
  }
  t.u = (int32_t)u;
  t.v = (int32_t)v;
  t.q = (int32_t)q;
  t.r = (int32_t)r;
  return zeta;
}

// (d, e) <- t (d, e) / 2^30 mod p, kept in (-2p, p)
P3G_HD void update_de(int32_t d[5], int32_t e[5], const Trans& t) {
  const int32_t u = t.u, v = t.v, q = t.q, r = t.r;
  const int32_t sd = d[4] >> 31, se = e[4] >> 31;
  int32_t md = (u & sd) + (v & se), me = (q & sd) + (r & se);
  int64_t cd = (int64_t)u * d[0] + (int64_t)v * e[0];
  int64_t ce = (int64_t)q * d[0] + (int64_t)r * e[0];
  // add md p, me p so that the low 30 bits vanish (p^-1 = 1 mod 2^30)
  md -= (int32_t)(((uint32_t)cd + (uint32_t)md) & (uint32_t)kM30);
  me -= (int32_t)(((uint32_t)ce + (uint32_t)me) & (uint32_t)kM30);
  cd += (int64_t)kP[0] * md;
  ce += (int64_t)kP[0] * me;
  cd >>= 30;
  ce >>= 30;
#pragma unroll
  for (int i = 1; i < 5; ++i) {
    cd += (int64_t)u * d[i] + (int64_t)v * e[i] + (int64_t)kP[i] * md;
    ce += (int64_t)q * d[i] + (int64_t)r * e[i] + (int64_t)kP[i] * me;
    d[i - 1] = (int32_t)cd & kM30;
    e[i - 1] = (int32_t)ce & kM30;
    cd >>= 30;
    ce >>= 30;
  }
  d[4] = (int32_t)cd;
  e[4] = (int32_t)ce;
}

// (f, g) <- t (f, g) / 2^30 (exact)
P3G_HD void update_fg(int32_t f[5], int32_t g[5], const Trans& t) {
  const int32_t u = t.u, v = t.v, q = t.q, r = t.r;
  int64_t cf = (int64_t)u * f[0] + (int64_t)v * g[0];
  int64_t cg = (int64_t)q * f[0] + (int64_t)r * g[0];
  cf >>= 30;
  cg >>= 30;
#pragma unroll
  for (int i = 1; i < 5; ++i) {
    cf += (int64_t)u * f[i] + (int64_t)v * g[i];
    cg += (int64_t)q * f[i] + (int64_t)r * g[i];
    f[i - 1] = (int32_t)cf & kM30;
    g[i - 1] = (int32_t)cg & kM30;
    cf >>= 30;
    cg >>= 30;
  }
  f[4] = (int32_t)cf;
  g[4] = (int32_t)cg;
}

// out = x^-1 mod p (canonical in, canonical out, little-endian 32-bit words; 0 -> 0)
P3G_HD void inverse(const uint32_t x[4], uint32_t out[4]) {
  int32_t f[5], g[5], d[5] = {0, 0, 0, 0, 0}, e[5] = {1, 0, 0, 0, 0};
#pragma unroll
  for (int i = 0; i < 5; ++i) f[i] = kP[i];
  // x in signed 30-bit limbs
  g[0] = (int32_t)(x[0] & (uint32_t)kM30);
  g[1] = (int32_t)(((x[0] >> 30) | (x[1] << 2)) & (uint32_t)kM30);
  g[2] = (int32_t)(((x[1] >> 28) | (x[2] << 4)) & (uint32_t)kM30);
  g[3] = (int32_t)(((x[2] >> 26) | (x[3] << 6)) & (uint32_t)kM30);
  g[4] = (int32_t)(x[3] >> 24);
  int32_t zeta = -1;
  for (int it = 0; it < 10; ++it) {
    Trans t;
    zeta = divsteps_30(zeta, (uint32_t)f[0] | ((uint32_t)f[1] << 30),
                       (uint32_t)g[0] | ((uint32_t)g[1] << 30), t);
    update_de(d, e, t);
    update_fg(f, g, t);
  }
  // f = +-1 (x != 0; x = 0 leaves d = 0); d in (-2p, p): d * sign(f), then into [0, p).
  // Limbs -> 160-bit two's complement words (d[0..3] in [0, 2^30), d[4] signed).
  uint32_t w[5];
  w[0] = (uint32_t)d[0] | ((uint32_t)d[1] << 30);
  w[1] = ((uint32_t)d[1] >> 2) | ((uint32_t)d[2] << 28);
  w[2] = ((uint32_t)d[2] >> 4) | ((uint32_t)d[3] << 26);
  w[3] = ((uint32_t)d[3] >> 6) | ((uint32_t)d[4] << 24);
  w[4] = (uint32_t)(d[4] >> 8);
  // negate if f < 0
  const uint32_t neg = (uint32_t)(f[4] >> 31);
  {
    uint64_t t = 1;
    for (int i = 0; i < 5; ++i) {
      const uint64_t s = (uint64_t)(w[i] ^ neg) + (t & neg);
      w[i] = (uint32_t)s;
      t = s >> 32;
    }
  }
  // value in (-p, 2p): add p if negative, then subtract p if >= p
  constexpr uint32_t P32[4] = {1u, 0u, 0xFFFFFFE4u, 0xFFFFFFFFu};
  {
    const uint32_t m = (uint32_t)((int32_t)w[4] >> 31);
    uint64_t c = 0;
    for (int i = 0; i < 5; ++i) {
      const uint64_t s = (uint64_t)w[i] + (i < 4 ? (P32[i] & m) : 0u) + c;
      w[i] = (uint32_t)s;
      c = s >> 32;
    }
    // w[4] is now 0 (or 1 when value >= 2^128, i.e. >= p)
  }
  {
    // s = w - p; keep s when w >= p (no borrow out of the 160-bit value)
    uint32_t s[5];
    int64_t b = 0;
    for (int i = 0; i < 5; ++i) {
      const int64_t dd = (int64_t)w[i] - (i < 4 ? (int64_t)P32[i] : 0) + b;
      s[i] = (uint32_t)dd;
      b = dd >> 32;  // 0 or -1
    }
    const uint32_t keep = (uint32_t)b;  // all ones: borrow (w < p): keep w
    for (int i = 0; i < 4; ++i) out[i] = (w[i] & keep) | (s[i] & ~keep);
  }
}

}  // namespace inv128
