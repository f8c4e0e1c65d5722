/*
 * prio3_ref.c -- C restatement of prio 0.15.1's Prio3 (draft-irtf-cfrg-vdaf-07), structured like
 * prio's CPU code.  TEST INFRASTRUCTURE / CPU BASELINE ONLY: used by tests/ (cross-checked against
 * oracle/prio3.py) and by bench.py's `cpu_baseline` leg.  Never linked into janus_amd.
 *
 * PARITY UNPINNED: prio 0.15.1 (Cargo.lock:2939-2963) is not vendored/buildable here; this follows
 * the same restatement as oracle/prio3.py (see its header for what is pinned).
 *
 * Structure mirrors prio so that its cost is representative of the reference CPU path:
 *   - Field64/Field128 in Montgomery form over u64 limbs with u128 products (prio src/fp.rs),
 *     converted at encode/decode;
 *   - portable (non-SIMD) Keccak-f[1600] behind SHAKE128 (keccak 0.1.4 / sha3 0.10.8);
 *   - FLP query = per-wire inverse DFT + Horner evaluation at t; gadget outputs by a size-2m DFT of
 *     the gadget polynomial (prio src/flp.rs QueryShimGadget, src/fft.rs);
 *   - FLP prove = wire interpolation + gadget polynomial by FFT multiplication (prio call_poly);
 *   - one report prepared sequentially per thread (Janus: sequential within an aggregation job,
 *     aggregator.rs:1613-1848; concurrency across jobs, binary_utils/job_driver.rs:119-216).
 * Not modelled (conservative, makes the baseline FASTER than prio): prio's helper re-expands its
 * measurement share in prepare_next; Janus's per-report Vec clones and BatchAggregation merges.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;
typedef uint64_t u64;
typedef uint8_t u8;
typedef uint32_t u32;

/* ============================ Keccak / SHAKE128 =========================================== */
static const u64 RC[24] = {
    0x0000000000000001ull, 0x0000000000008082ull, 0x800000000000808aull, 0x8000000080008000ull,
    0x000000000000808bull, 0x0000000080000001ull, 0x8000000080008081ull, 0x8000000000008009ull,
    0x000000000000008aull, 0x0000000000000088ull, 0x0000000080008009ull, 0x000000008000000aull,
    0x000000008000808bull, 0x800000000000008bull, 0x8000000000008089ull, 0x8000000000008003ull,
    0x8000000000008002ull, 0x8000000000000080ull, 0x000000000000800aull, 0x800000008000000aull,
    0x8000000080008081ull, 0x8000000000008080ull, 0x0000000080000001ull, 0x8000000080008008ull};
#define ROTL(x, n) (((x) << (n)) | ((x) >> ((64 - (n)) & 63)))

static void keccak_f1600(u64 a[25]) {
  for (int r = 0; r < 24; ++r) {
    u64 c0 = a[0] ^ a[5] ^ a[10] ^ a[15] ^ a[20], c1 = a[1] ^ a[6] ^ a[11] ^ a[16] ^ a[21];
    u64 c2 = a[2] ^ a[7] ^ a[12] ^ a[17] ^ a[22], c3 = a[3] ^ a[8] ^ a[13] ^ a[18] ^ a[23];
    u64 c4 = a[4] ^ a[9] ^ a[14] ^ a[19] ^ a[24];
    u64 d0 = c4 ^ ROTL(c1, 1), d1 = c0 ^ ROTL(c2, 1), d2 = c1 ^ ROTL(c3, 1);
    u64 d3 = c2 ^ ROTL(c4, 1), d4 = c3 ^ ROTL(c0, 1);
    u64 b0 = a[0] ^ d0, b10 = ROTL(a[1] ^ d1, 1), b20 = ROTL(a[2] ^ d2, 62);
    u64 b5 = ROTL(a[3] ^ d3, 28), b15 = ROTL(a[4] ^ d4, 27), b16 = ROTL(a[5] ^ d0, 36);
    u64 b1 = ROTL(a[6] ^ d1, 44), b11 = ROTL(a[7] ^ d2, 6), b21 = ROTL(a[8] ^ d3, 55);
    u64 b6 = ROTL(a[9] ^ d4, 20), b7 = ROTL(a[10] ^ d0, 3), b17 = ROTL(a[11] ^ d1, 10);
    u64 b2 = ROTL(a[12] ^ d2, 43), b12 = ROTL(a[13] ^ d3, 25), b22 = ROTL(a[14] ^ d4, 39);
    u64 b23 = ROTL(a[15] ^ d0, 41), b8 = ROTL(a[16] ^ d1, 45), b18 = ROTL(a[17] ^ d2, 15);
    u64 b3 = ROTL(a[18] ^ d3, 21), b13 = ROTL(a[19] ^ d4, 8), b14 = ROTL(a[20] ^ d0, 18);
    u64 b24 = ROTL(a[21] ^ d1, 2), b9 = ROTL(a[22] ^ d2, 61), b19 = ROTL(a[23] ^ d3, 56);
    u64 b4 = ROTL(a[24] ^ d4, 14);
    a[0] = b0 ^ (~b1 & b2) ^ RC[r]; a[1] = b1 ^ (~b2 & b3); a[2] = b2 ^ (~b3 & b4);
    a[3] = b3 ^ (~b4 & b0); a[4] = b4 ^ (~b0 & b1);
    a[5] = b5 ^ (~b6 & b7); a[6] = b6 ^ (~b7 & b8); a[7] = b7 ^ (~b8 & b9);
    a[8] = b8 ^ (~b9 & b5); a[9] = b9 ^ (~b5 & b6);
    a[10] = b10 ^ (~b11 & b12); a[11] = b11 ^ (~b12 & b13); a[12] = b12 ^ (~b13 & b14);
    a[13] = b13 ^ (~b14 & b10); a[14] = b14 ^ (~b10 & b11);
    a[15] = b15 ^ (~b16 & b17); a[16] = b16 ^ (~b17 & b18); a[17] = b17 ^ (~b18 & b19);
    a[18] = b18 ^ (~b19 & b15); a[19] = b19 ^ (~b15 & b16);
    a[20] = b20 ^ (~b21 & b22); a[21] = b21 ^ (~b22 & b23); a[22] = b22 ^ (~b23 & b24);
    a[23] = b23 ^ (~b24 & b20); a[24] = b24 ^ (~b20 & b21);
  }
}

typedef struct {
  u64 s[25];
  unsigned pos; /* byte position in the rate */
  int squeezing;
} shake;

#define RATE 168
static void shake_init(shake* h) {
  memset(h, 0, sizeof *h);
}
static void shake_absorb(shake* h, const u8* p, size_t n) {
  while (n) {
    if (h->pos == 0 && n >= RATE) { /* whole block, word-wise (LE host) */
      for (int w = 0; w < RATE / 8; ++w) {
        u64 v;
        memcpy(&v, p + 8 * w, 8);
        h->s[w] ^= v;
      }
      keccak_f1600(h->s);
      p += RATE;
      n -= RATE;
      continue;
    }
    unsigned take = RATE - h->pos;
    if (take > n) take = (unsigned)n;
    for (unsigned i = 0; i < take; ++i) {
      unsigned q = h->pos + i;
      h->s[q >> 3] ^= (u64)p[i] << (8 * (q & 7));
    }
    h->pos += take;
    p += take;
    n -= take;
    if (h->pos == RATE) {
      keccak_f1600(h->s);
      h->pos = 0;
    }
  }
}
static void shake_finish(shake* h) {
  h->s[h->pos >> 3] ^= (u64)0x1F << (8 * (h->pos & 7));
  h->s[(RATE - 1) >> 3] ^= (u64)0x80 << 56;
  keccak_f1600(h->s);
  h->pos = 0;
  h->squeezing = 1;
}
static void shake_squeeze(shake* h, u8* out, size_t n) {
  while (n) {
    if (h->pos == RATE) {
      keccak_f1600(h->s);
      h->pos = 0;
    }
    unsigned take = RATE - h->pos;
    if (take > n) take = (unsigned)n;
    for (unsigned i = 0; i < take; ++i) {
      unsigned q = h->pos + i;
      out[i] = (u8)(h->s[q >> 3] >> (8 * (q & 7)));
    }
    h->pos += take;
    out += take;
    n -= take;
  }
}

/* ============================ Fields (Montgomery, like prio fp.rs) ========================== */
typedef struct {
  int es;       /* encoded size */
  u128 p;
  u64 p0, p1;   /* limbs */
  u64 n0;       /* -p^-1 mod 2^64 */
  u128 r2;      /* R^2 mod p */
  u128 one;     /* R mod p */
} field;

static const field F128 = {16,
                           ((u128)0xFFFFFFFFFFFFFFE4ull << 64) | 1u,
                           1u,
                           0xFFFFFFFFFFFFFFE4ull,
                           0xFFFFFFFFFFFFFFFFull,
                           ((u128)0x5587ull << 64) | 0xfffffffffffffcf1ull,
                           ((u128)0x1Bull << 64) | 0xFFFFFFFFFFFFFFFFull};
static const field F64 = {8,
                          (u128)0xFFFFFFFF00000001ull,
                          0xFFFFFFFF00000001ull,
                          0,
                          0xFFFFFFFEFFFFFFFFull,
                          (u128)0xFFFFFFFE00000001ull,
                          (u128)0xFFFFFFFFull};

/* constant-time (branchless) add/sub, as prio's FieldParameters::{add, sub} */
static inline u128 f_add(const field* F, u128 a, u128 b) {
  u128 s = a + b;
  u128 carry = (u128)(s < a);
  u128 d = s - F->p;
  u128 borrow = (u128)(s < F->p);
  /* keep s if (no carry and s < p) */
  u128 keep = (u128)0 - (borrow & (carry ^ 1));
  return (s & keep) | (d & ~keep);
}
static inline u128 f_sub(const field* F, u128 a, u128 b) {
  u128 d = a - b;
  u128 mask = (u128)0 - (u128)(a < b);
  return d + (F->p & mask);
}
static inline u128 f_mul(const field* F, u128 a, u128 b) {
  if (F->es == 8) {
    u64 x = (u64)a, y = (u64)b;
    u128 t = (u128)x * y;
    u64 m = (u64)t * F->n0;
    u128 mp = (u128)m * F->p0;
    u128 s = t + mp;
    int carry = s < t;
    u64 hi = (u64)(s >> 64);
    u128 r = ((u128)carry << 64) | hi;
    if (r >= F->p) r -= F->p;
    return r;
  }
  /* 2-limb CIOS */
  u64 a0 = (u64)a, a1 = (u64)(a >> 64);
  u64 bw[2] = {(u64)b, (u64)(b >> 64)};
  u64 t0 = 0, t1 = 0, t2 = 0;
  for (int i = 0; i < 2; ++i) {
    u128 c = (u128)a0 * bw[i] + t0;
    t0 = (u64)c;
    c = (u128)a1 * bw[i] + t1 + (c >> 64);
    t1 = (u64)c;
    u128 s = (u128)t2 + (u64)(c >> 64);
    t2 = (u64)s;
    u64 t3 = (u64)(s >> 64);
    u64 m = t0 * F->n0;
    c = (u128)m * F->p0 + t0;
    c = (u128)m * F->p1 + t1 + (c >> 64);
    t0 = (u64)c;
    s = (u128)t2 + (u64)(c >> 64);
    t1 = (u64)s;
    t2 = t3 + (u64)(s >> 64);
  }
  u128 r = ((u128)t1 << 64) | t0;
  if (t2 || r >= F->p) r -= F->p;
  return r;
}
static inline u128 f_to_mont(const field* F, u128 a) { return f_mul(F, a, F->r2); }
static inline u128 f_from_mont(const field* F, u128 a) { return f_mul(F, a, 1); }
static u128 f_pow(const field* F, u128 x, u128 e) { /* x Montgomery */
  u128 r = F->one;
  while (e) {
    if (e & 1) r = f_mul(F, r, x);
    x = f_mul(F, x, x);
    e >>= 1;
  }
  return r;
}
static u128 f_inv(const field* F, u128 x) { return f_pow(F, x, F->p - 2); }
static inline u128 f_from_int(const field* F, u128 v) { return f_to_mont(F, v % F->p); }

static void f_encode(const field* F, u128 xm, u8* out) {
  u128 x = f_from_mont(F, xm);
  for (int i = 0; i < F->es; ++i) out[i] = (u8)(x >> (8 * i));
}
/* decode with range check; returns 0 on error */
static int f_decode(const field* F, const u8* in, u128* out) {
  u128 x = 0;
  for (int i = 0; i < F->es; ++i) x |= (u128)in[i] << (8 * i);
  if (x >= F->p) return 0;
  *out = f_to_mont(F, x);
  return 1;
}

/* next_vec: ES-byte LE chunks with rejection */
static void xof_next_vec(const field* F, shake* h, u128* out, size_t n) {
  u8 buf[16];
  size_t cnt = 0;
  while (cnt < n) {
    shake_squeeze(h, buf, F->es);
    u128 x = 0;
    for (int i = 0; i < F->es; ++i) x |= (u128)buf[i] << (8 * i);
    if (x < F->p) out[cnt++] = f_to_mont(F, x);
  }
}

/* ============================ FFT (prio src/fft.rs) ======================================== */
static u128 root_of_unity(const field* F, unsigned logn) { /* Montgomery; setup only */
  u128 g = f_to_mont(F, 7);
  return f_pow(F, g, (F->p - 1) >> logn);
}
/* out[i] = sum_j in[j] w^(ij), in zero-padded to n (n power of two) */
static void dft(const field* F, const u128* roots, u128* out, const u128* in, size_t in_len,
                size_t n) {
  unsigned logn = 0;
  while (((size_t)1 << logn) < n) ++logn;
  for (size_t i = 0; i < n; ++i) {
    size_t r = 0;
    for (unsigned b = 0; b < logn; ++b)
      if (i >> b & 1) r |= (size_t)1 << (logn - 1 - b);
    out[r] = i < in_len ? in[i] : 0;
  }
  /* loop order as prio fft.rs: one twiddle update per butterfly column */
  for (unsigned l = 1; l <= logn; ++l) {
    const size_t y = (size_t)1 << (l - 1);
    const size_t chunk = (n / y) >> 1;
    const u128 r = roots[l];
    for (size_t j = 0; j < chunk; ++j) {
      size_t x = j << l;
      u128 u = out[x], v = out[x + y];
      out[x] = f_add(F, u, v);
      out[x + y] = f_sub(F, u, v);
    }
    u128 w = F->one;
    for (size_t i = 1; i < y; ++i) {
      w = f_mul(F, w, r);
      for (size_t j = 0; j < chunk; ++j) {
        size_t x = (j << l) + i;
        u128 u = out[x], v = f_mul(F, w, out[x + y]);
        out[x] = f_add(F, u, v);
        out[x + y] = f_sub(F, u, v);
      }
    }
  }
}
/* prio discrete_fourier_transform_inv_finish */
static void idft_finish(const field* F, u128 ninv, u128* a, size_t n) {
  a[0] = f_mul(F, a[0], ninv);
  a[n >> 1] = f_mul(F, a[n >> 1], ninv);
  for (size_t i = 1; i < (n >> 1); ++i) {
    u128 t = f_mul(F, a[i], ninv);
    a[i] = f_mul(F, a[n - i], ninv);
    a[n - i] = t;
  }
}
static u128 poly_eval(const field* F, const u128* c, size_t n, u128 x) {
  u128 acc = 0;
  for (size_t i = n; i-- > 0;) acc = f_add(F, f_mul(F, acc, x), c[i]);
  return acc;
}

/* ============================ Prio3 types ================================================== */
enum { K_COUNT = 0, K_SUM = 1, K_SUMVEC = 2, K_HIST = 3, K_FPVEC = 4 };
/* gadget kinds (prio src/flp/gadgets.rs): Mul, PolyEval(x^2 - x), ParallelSum(Mul, chunk),
 * ParallelSum(PolyEval(p), chunk) -- all of degree 2 */
enum { G_MUL = 0, G_RANGE2 = 1, G_PSUM_MUL = 2, G_PSUM_POLY = 3 };

typedef struct {
  int kind;
  unsigned chunk, calls, arity, m, logm, gp_len;
  u128 poly[3]; /* G_PSUM_POLY coefficients (Montgomery), ascending */
} gadget;

typedef struct {
  int kind;
  u32 algo_id;
  const field* F;
  unsigned bits, length, chunk;
  unsigned meas_len, out_len, jr_len, qr_len, prove_rand_len;
  unsigned ng;
  gadget g[2];
  unsigned proof_len, ver_len;
  u128 half; /* 1/2 Montgomery */
  u128 roots[24]; /* roots[l] = principal 2^l-th root (Montgomery), prio FieldParameters.roots */
  u128 ninv[24];  /* 1/2^l (Montgomery) */
  u8 vk[16];
} cfgt;

static unsigned npow2(unsigned x) {
  unsigned r = 1;
  while (r < x) r <<= 1;
  return r;
}

/* prio `optimal_chunk_length` (src/vdaf/prio3.rs): gadget_calls = 2^k - 1 from the largest k
 * down, first minimum of the ParallelSum(Mul) proof length */
static unsigned optimal_chunk_length(unsigned len) {
  if (len <= 1) return 1;
  unsigned max_log2 = 0;
  { /* round(log2(len + 1)) */
    double l = 0, x = (double)len + 1.0;
    while (x >= 2.0) { x /= 2.0; l += 1.0; }
    /* x in [1,2): log2(x) >= 0.5 iff x >= sqrt(2) */
    max_log2 = (unsigned)l + (x >= 1.4142135623730951 ? 1 : 0);
  }
  unsigned long long best_cost = ~0ull;
  unsigned best = 1;
  for (unsigned k = max_log2; k >= 1; --k) {
    unsigned long long calls = (1ull << k) - 1, chunk = (len + calls - 1) / calls;
    unsigned long long cost = 2 * chunk + 2 * (npow2((unsigned)(1 + calls)) - 1) + 1;
    if (cost < best_cost) { best_cost = cost; best = (unsigned)chunk; }
  }
  return best;
}

static void gadget_init(gadget* g, int kind, unsigned chunk, unsigned calls) {
  g->kind = kind;
  g->chunk = chunk;
  g->calls = calls;
  g->arity = kind == G_MUL ? 2 : kind == G_RANGE2 ? 1 : kind == G_PSUM_MUL ? 2 * chunk : chunk;
  g->m = npow2(1 + calls);
  g->logm = 0;
  while ((1u << g->logm) < g->m) g->logm++;
  g->gp_len = 2 * (g->m - 1) + 1;
}

int p3ref_cfg_init(cfgt* c, int kind, unsigned bits, unsigned length, unsigned chunk,
                   const u8 vk[16]) {
  memset(c, 0, sizeof *c);
  c->kind = kind;
  c->algo_id = kind == K_FPVEC ? 0xFFFF0000u : (u32)kind;
  c->bits = bits;
  c->length = length;
  c->chunk = chunk;
  c->qr_len = 1;
  c->ng = 1;
  memcpy(c->vk, vk, 16);
  switch (kind) {
    case K_COUNT:
      c->F = &F64; c->meas_len = 1; c->out_len = 1; c->jr_len = 0;
      gadget_init(&c->g[0], G_MUL, 0, 1);
      break;
    case K_SUM:
      c->F = &F128; c->meas_len = bits; c->out_len = 1; c->jr_len = 1;
      gadget_init(&c->g[0], G_RANGE2, 0, bits);
      break;
    case K_SUMVEC:
      c->F = &F128; c->meas_len = bits * length; c->out_len = length; c->jr_len = 1;
      gadget_init(&c->g[0], G_PSUM_MUL, chunk, (c->meas_len + chunk - 1) / chunk);
      break;
    case K_HIST:
      c->F = &F128; c->meas_len = length; c->out_len = length; c->jr_len = 2;
      gadget_init(&c->g[0], G_PSUM_MUL, chunk, (length + chunk - 1) / chunk);
      break;
    case K_FPVEC: {
      if ((bits != 16 && bits != 32 && bits != 64) || length == 0) return -1;
      c->F = &F128; c->meas_len = bits * length + 2 * bits - 2; c->out_len = length;
      c->jr_len = 2; c->qr_len = 2; c->ng = 2;
      unsigned c0 = optimal_chunk_length(c->meas_len), c1 = optimal_chunk_length(length);
      gadget_init(&c->g[0], G_PSUM_MUL, c0, (c->meas_len + c0 - 1) / c0);
      gadget_init(&c->g[1], G_PSUM_POLY, c1, (length + c1 - 1) / c1);
      /* norm summand (z - 2^(n-1))^2 = 2^(2n-2) - 2^n z + z^2 */
      const u128 one = (u128)1 << (bits - 1);
      c->g[1].poly[0] = f_from_int(&F128, one * one);
      c->g[1].poly[1] = f_sub(&F128, 0, f_from_int(&F128, 2 * one));
      c->g[1].poly[2] = F128.one;
      break;
    }
    default:
      return -1;
  }
  c->proof_len = 0;
  c->ver_len = 1;
  c->prove_rand_len = 0;
  for (unsigned i = 0; i < c->ng; ++i) {
    c->proof_len += c->g[i].arity + c->g[i].gp_len;
    c->ver_len += c->g[i].arity + 1;
    c->prove_rand_len += c->g[i].arity;
  }
  c->half = f_inv(c->F, f_from_int(c->F, 2));
  for (unsigned l = 0; l < 24; ++l) {
    c->roots[l] = root_of_unity(c->F, l);
    c->ninv[l] = f_inv(c->F, f_from_int(c->F, (u128)1 << l));
  }
  return 0;
}

static void dst(const cfgt* c, unsigned usage, u8 out[8]) {
  out[0] = 7; out[1] = 0;
  out[2] = (u8)(c->algo_id >> 24); out[3] = (u8)(c->algo_id >> 16);
  out[4] = (u8)(c->algo_id >> 8); out[5] = (u8)c->algo_id;
  out[6] = (u8)(usage >> 8); out[7] = (u8)usage;
}
static void xof_init(const cfgt* c, shake* h, const u8 seed[16], unsigned usage) {
  u8 d[8], l = 8;
  dst(c, usage, d);
  shake_init(h);
  shake_absorb(h, &l, 1);
  shake_absorb(h, d, 8);
  shake_absorb(h, seed, 16);
}

/* ---- gadget records ---------------------------------------------------------------------- */
typedef struct {
  const gadget* g;
  u128* f;      /* arity x (calls+1) wire values */
  unsigned ct;  /* next call index (1-based) */
  const u128* pvals; /* query: gadget poly evaluated at 2m-th roots (query mode) */
  int query;
} shim;

static u128 gadget_eval(const field* F, const gadget* g, const u128* inp) {
  u128 acc = 0;
  switch (g->kind) {
    case G_MUL: return f_mul(F, inp[0], inp[1]);
    case G_RANGE2: return f_sub(F, f_mul(F, inp[0], inp[0]), inp[0]);
    case G_PSUM_MUL:
      for (unsigned j = 0; j < g->chunk; ++j) acc = f_add(F, acc, f_mul(F, inp[2 * j], inp[2 * j + 1]));
      return acc;
    default: /* G_PSUM_POLY, Horner per input */
      for (unsigned j = 0; j < g->chunk; ++j) {
        u128 y = f_add(F, f_mul(F, g->poly[2], inp[j]), g->poly[1]);
        acc = f_add(F, acc, f_add(F, f_mul(F, y, inp[j]), g->poly[0]));
      }
      return acc;
  }
}
static u128 shim_call(const cfgt* c, shim* s, const u128* inp) {
  const gadget* g = s->g;
  for (unsigned w = 0; w < g->arity; ++w) s->f[w * (g->calls + 1) + s->ct] = inp[w];
  u128 out = s->query ? s->pvals[s->ct * 2] : gadget_eval(c->F, g, inp);
  s->ct++;
  return out;
}

/* prio parallel_sum_range_checks: one joint-rand value, r_power across all chunks */
static u128 psum_range_checks(const cfgt* c, shim* g, const u128* x, unsigned len, u128 r,
                              u128 sinv) {
  const field* F = c->F;
  const unsigned chunk = g->g->chunk;
  u128 out = 0, rp = r;
  u128* args = (u128*)malloc(sizeof(u128) * 2 * chunk);
  for (unsigned k = 0; k < g->g->calls; ++k) {
    for (unsigned j = 0; j < chunk; ++j) {
      unsigned idx = k * chunk + j;
      if (idx < len) {
        args[2 * j] = f_mul(F, rp, x[idx]);
        args[2 * j + 1] = f_sub(F, x[idx], sinv);
        rp = f_mul(F, rp, r);
      } else {
        args[2 * j] = 0;
        args[2 * j + 1] = f_sub(F, 0, sinv);
      }
    }
    out = f_add(F, out, shim_call(c, g, args));
  }
  free(args);
  return out;
}

static u128 decode_bits(const field* F, const u128* x, unsigned nb) {
  u128 acc = 0;
  for (unsigned b = nb; b-- > 0;) acc = f_add(F, f_add(F, acc, acc), x[b]);
  return acc;
}

/* validity circuit with shim gadgets (prio Type::valid) */
static u128 valid(const cfgt* c, shim* g, const u128* x, const u128* jr, unsigned num_shares) {
  const field* F = c->F;
  if (c->kind == K_COUNT) {
    u128 in[2] = {x[0], x[0]};
    return f_sub(F, shim_call(c, &g[0], in), x[0]);
  }
  if (c->kind == K_SUM) {
    u128 r = jr[0], out = 0;
    for (unsigned i = 0; i < c->bits; ++i) {
      out = f_add(F, out, f_mul(F, r, shim_call(c, &g[0], &x[i])));
      r = f_mul(F, r, jr[0]);
    }
    return out;
  }
  u128 sinv = num_shares == 2 ? c->half : F->one; /* 1/num_shares */
  u128 out = psum_range_checks(c, &g[0], x, c->meas_len, jr[0], sinv);
  u128 r1 = jr[1];
  if (c->kind == K_HIST) {
    u128 sc = f_sub(F, 0, sinv);
    for (unsigned i = 0; i < c->meas_len; ++i) sc = f_add(F, sc, x[i]);
    out = f_add(F, f_mul(F, r1, out), f_mul(F, f_mul(F, r1, r1), sc));
  } else if (c->kind == K_FPVEC) {
    /* prio FixedPointBoundedL2VecSum::valid: norm of the decoded entries by gadget 1, padded with
     * the share of the encoded zero 2^(n-1)/num_shares; compared with the submitted norm bits */
    const unsigned nb = c->bits, c1 = c->g[1].chunk;
    const u128 zs = f_mul(F, f_from_int(F, (u128)1 << (nb - 1)), sinv);
    u128* args = (u128*)malloc(sizeof(u128) * c1);
    u128 computed = 0;
    for (unsigned k = 0; k < c->g[1].calls; ++k) {
      for (unsigned j = 0; j < c1; ++j) {
        unsigned e = k * c1 + j;
        args[j] = e < c->length ? decode_bits(F, &x[(size_t)e * nb], nb) : zs;
      }
      computed = f_add(F, computed, shim_call(c, &g[1], args));
    }
    free(args);
    u128 submitted = decode_bits(F, &x[(size_t)nb * c->length], 2 * nb - 2);
    u128 nc = f_sub(F, computed, submitted);
    out = f_add(F, f_mul(F, r1, out), f_mul(F, f_mul(F, r1, r1), nc));
  }
  return out;
}

/* FLP prove (prio flp.rs Type::prove) */
static void flp_prove(const cfgt* c, const u128* x, const u128* prove_rand, const u128* jr,
                      u128* proof) {
  const field* F = c->F;
  shim s[2];
  unsigned pr = 0;
  for (unsigned i = 0; i < c->ng; ++i) {
    const gadget* g = &c->g[i];
    const unsigned K = g->calls + 1;
    s[i].g = g;
    s[i].f = (u128*)calloc((size_t)g->arity * K, sizeof(u128));
    s[i].ct = 1;
    s[i].query = 0;
    for (unsigned w = 0; w < g->arity; ++w) s[i].f[w * K] = prove_rand[pr++];
  }
  (void)valid(c, s, x, jr, 1);
  size_t off = 0;
  for (unsigned i = 0; i < c->ng; ++i) {
    const gadget* g = &c->g[i];
    const unsigned m = g->m, K = g->calls + 1;
    /* wire polys: interpolate, then evaluate at 2m points */
    const unsigned n2 = 2 * m;
    u128* coef = (u128*)malloc(sizeof(u128) * m);
    u128* ev = (u128*)malloc(sizeof(u128) * n2 * g->arity);
    for (unsigned w = 0; w < g->arity; ++w) {
      dft(F, c->roots, coef, &s[i].f[w * K], K, m);
      idft_finish(F, c->ninv[g->logm], coef, m);
      proof[off + w] = s[i].f[w * K];
      dft(F, c->roots, &ev[(size_t)w * n2], coef, m, n2);
    }
    /* gadget poly values at 2m points, then interpolate */
    u128* gv = (u128*)malloc(sizeof(u128) * n2);
    u128* inp = (u128*)malloc(sizeof(u128) * g->arity);
    for (unsigned q = 0; q < n2; ++q) {
      for (unsigned w = 0; w < g->arity; ++w) inp[w] = ev[(size_t)w * n2 + q];
      gv[q] = gadget_eval(F, g, inp);
    }
    u128* gp = (u128*)malloc(sizeof(u128) * n2);
    dft(F, c->roots, gp, gv, n2, n2);
    idft_finish(F, c->ninv[g->logm + 1], gp, n2);
    for (unsigned d = 0; d < g->gp_len; ++d) proof[off + g->arity + d] = gp[d];
    off += g->arity + g->gp_len;
    free(gp); free(inp); free(gv); free(ev); free(coef); free(s[i].f);
  }
}

/* FLP query (prio flp.rs Type::query): returns 0 on invalid query randomness */
static int flp_query(const cfgt* c, const u128* x, const u128* proof, const u128* t,
                     const u128* jr, u128* verifier) {
  const field* F = c->F;
  shim s[2];
  u128* pv[2] = {NULL, NULL};
  size_t off = 0;
  int ok = 1;
  for (unsigned i = 0; i < c->ng; ++i) {
    const gadget* g = &c->g[i];
    const unsigned K = g->calls + 1;
    if (f_pow(F, t[i], g->m) == F->one) ok = 0;
    s[i].g = g;
    s[i].f = (u128*)calloc((size_t)g->arity * K, sizeof(u128));
    s[i].ct = 1;
    s[i].query = 1;
    for (unsigned w = 0; w < g->arity; ++w) s[i].f[w * K] = proof[off + w];
    pv[i] = (u128*)malloc(sizeof(u128) * 2 * g->m);
    dft(F, c->roots, pv[i], &proof[off + g->arity], g->gp_len, 2 * g->m);
    s[i].pvals = pv[i];
    off += g->arity + g->gp_len;
  }
  if (!ok) {
    for (unsigned i = 0; i < c->ng; ++i) { free(s[i].f); free(pv[i]); }
    return 0;
  }
  verifier[0] = valid(c, s, x, jr, 2);
  size_t vo = 1;
  off = 0;
  for (unsigned i = 0; i < c->ng; ++i) {
    const gadget* g = &c->g[i];
    const unsigned m = g->m, K = g->calls + 1;
    u128* coef = (u128*)malloc(sizeof(u128) * m);
    for (unsigned w = 0; w < g->arity; ++w) {
      dft(F, c->roots, coef, &s[i].f[w * K], K, m);
      idft_finish(F, c->ninv[g->logm], coef, m);
      verifier[vo++] = poly_eval(F, coef, m, t[i]);
    }
    verifier[vo++] = poly_eval(F, &proof[off + g->arity], g->gp_len, t[i]);
    off += g->arity + g->gp_len;
    free(coef); free(pv[i]); free(s[i].f);
  }
  return 1;
}

static int flp_decide(const cfgt* c, const u128* v) {
  if (v[0] != 0) return 0;
  size_t vo = 1;
  for (unsigned i = 0; i < c->ng; ++i) {
    const gadget* g = &c->g[i];
    if (gadget_eval(c->F, g, &v[vo]) != v[vo + g->arity]) return 0;
    vo += g->arity + 1;
  }
  return 1;
}

/* truncate (prio Type::truncate), Montgomery in/out */
static void truncate_out(const cfgt* c, const u128* x, u128* out) {
  const field* F = c->F;
  if (c->kind == K_SUM || c->kind == K_SUMVEC || c->kind == K_FPVEC) {
    unsigned len = c->kind == K_SUM ? 1 : c->length;
    for (unsigned e = 0; e < len; ++e) out[e] = decode_bits(F, &x[(size_t)e * c->bits], c->bits);
  } else {
    memcpy(out, x, sizeof(u128) * c->out_len);
  }
}

/* ============================ Prio3 ======================================================== */
static void joint_rand_part(const cfgt* c, const u8 blind[16], u8 agg_id, const u8 nonce[16],
                            const u128* meas, u8 out[16]) {
  shake h;
  xof_init(c, &h, blind, 7);
  shake_absorb(&h, &agg_id, 1);
  shake_absorb(&h, nonce, 16);
  u8 enc[16];
  for (unsigned i = 0; i < c->meas_len; ++i) {
    f_encode(c->F, meas[i], enc);
    shake_absorb(&h, enc, c->F->es);
  }
  shake_finish(&h);
  shake_squeeze(&h, out, 16);
}
static void joint_rand_seed(const cfgt* c, const u8 p0[16], const u8 p1[16], u8 out[16]) {
  static const u8 zero[16] = {0};
  shake h;
  xof_init(c, &h, zero, 6);
  shake_absorb(&h, p0, 16);
  shake_absorb(&h, p1, 16);
  shake_finish(&h);
  shake_squeeze(&h, out, 16);
}
static void expand(const cfgt* c, const u8 seed[16], unsigned usage, const u8* binder,
                   size_t blen, u128* out, size_t n) {
  shake h;
  xof_init(c, &h, seed, usage);
  if (blen) shake_absorb(&h, binder, blen);
  shake_finish(&h);
  xof_next_vec(c->F, &h, out, n);
}

unsigned p3ref_random_size(const cfgt* c) { return 16 * (3 + (c->jr_len ? 2 : 0)); }
unsigned p3ref_leader_len(const cfgt* c) {
  return c->F->es * (c->meas_len + c->proof_len) + (c->jr_len ? 16 : 0);
}
unsigned p3ref_helper_len(const cfgt* c) { return c->jr_len ? 48 : 32; }
unsigned p3ref_public_len(const cfgt* c) { return c->jr_len ? 32 : 0; }
unsigned p3ref_prep_len(const cfgt* c) { return c->F->es * c->ver_len + (c->jr_len ? 16 : 0); }

/* Client::shard with explicit randomness (prio shard_with_random order) */
static void shard(const cfgt* c, const u128* encoded, const u8 nonce[16], const u8* rand,
                  u8* pub, u8* leader, u8* helper) {
  const field* F = c->F;
  const u8* k_meas = rand;
  const u8* k_proof = rand + 16;
  const u8* h_blind = c->jr_len ? rand + 32 : NULL;
  const u8* l_blind = c->jr_len ? rand + 48 : NULL;
  const u8* k_prove = rand + (c->jr_len ? 64 : 32);
  u8 one = 1;
  u128* hm = (u128*)malloc(sizeof(u128) * c->meas_len);
  u128* lm = (u128*)malloc(sizeof(u128) * c->meas_len);
  expand(c, k_meas, 1, &one, 1, hm, c->meas_len);
  for (unsigned i = 0; i < c->meas_len; ++i) lm[i] = f_sub(F, encoded[i], hm[i]);
  u128 jr[2] = {0, 0};
  if (c->jr_len) {
    u8 hpart[16], lpart[16], seed[16];
    joint_rand_part(c, h_blind, 1, nonce, hm, hpart);
    joint_rand_part(c, l_blind, 0, nonce, lm, lpart);
    memcpy(pub, lpart, 16);
    memcpy(pub + 16, hpart, 16);
    joint_rand_seed(c, lpart, hpart, seed);
    expand(c, seed, 3, NULL, 0, jr, c->jr_len);
  }
  u128* prove_rand = (u128*)malloc(sizeof(u128) * c->prove_rand_len);
  expand(c, k_prove, 4, NULL, 0, prove_rand, c->prove_rand_len);
  u128* proof = (u128*)malloc(sizeof(u128) * c->proof_len);
  flp_prove(c, encoded, prove_rand, jr, proof);
  u128* hp = (u128*)malloc(sizeof(u128) * c->proof_len);
  expand(c, k_proof, 2, &one, 1, hp, c->proof_len);
  size_t o = 0;
  for (unsigned i = 0; i < c->meas_len; ++i, o += F->es) f_encode(F, lm[i], leader + o);
  for (unsigned i = 0; i < c->proof_len; ++i, o += F->es)
    f_encode(F, f_sub(F, proof[i], hp[i]), leader + o);
  if (c->jr_len) memcpy(leader + o, l_blind, 16);
  memcpy(helper, k_meas, 16);
  memcpy(helper + 16, k_proof, 16);
  if (c->jr_len) memcpy(helper + 32, h_blind, 16);
  free(hm); free(lm); free(prove_rand); free(proof); free(hp);
}

/* prepare_init; returns status (0 ok, 5 prep error, 8 invalid message).
 * out_share (Montgomery, out_len) and seed are the prep state. */
static int prepare_init(const cfgt* c, int agg_id, const u8 nonce[16], const u8* pub,
                        const u8* share, u8* prep_share, u128* out_share, u8 seed[16]) {
  const field* F = c->F;
  u128 t[2];
  {
    shake h;
    xof_init(c, &h, c->vk, 5);
    shake_absorb(&h, nonce, 16);
    shake_finish(&h);
    xof_next_vec(F, &h, t, c->qr_len);
  }
  u128* meas = (u128*)malloc(sizeof(u128) * c->meas_len);
  u128* proof = (u128*)malloc(sizeof(u128) * c->proof_len);
  const u8* blind;
  int st = 0;
  if (agg_id == 0) {
    size_t o = 0;
    for (unsigned i = 0; i < c->meas_len; ++i, o += F->es)
      if (!f_decode(F, share + o, &meas[i])) st = 8;
    for (unsigned i = 0; i < c->proof_len; ++i, o += F->es)
      if (!f_decode(F, share + o, &proof[i])) st = 8;
    blind = share + o;
  } else {
    u8 one = 1;
    expand(c, share, 1, &one, 1, meas, c->meas_len);
    expand(c, share + 16, 2, &one, 1, proof, c->proof_len);
    blind = share + 32;
  }
  if (st) {
    free(meas); free(proof);
    return st;
  }
  u128 jr[2] = {0, 0};
  u8 part[16];
  if (c->jr_len) {
    joint_rand_part(c, blind, (u8)agg_id, nonce, meas, part);
    if (agg_id == 0) joint_rand_seed(c, part, pub + 16, seed);
    else joint_rand_seed(c, pub, part, seed);
    expand(c, seed, 3, NULL, 0, jr, c->jr_len);
  }
  u128* ver = (u128*)malloc(sizeof(u128) * c->ver_len);
  if (!flp_query(c, meas, proof, t, jr, ver)) st = 5;
  size_t o = 0;
  for (unsigned i = 0; i < c->ver_len; ++i, o += F->es) f_encode(F, ver[i], prep_share + o);
  if (c->jr_len) memcpy(prep_share + o, part, 16);
  truncate_out(c, meas, out_share);
  free(ver); free(meas); free(proof);
  return st;
}

static int prep_shares_to_prep(const cfgt* c, const u8* lps, const u8* hps, u8 msg[16]) {
  const field* F = c->F;
  u128* v = (u128*)malloc(sizeof(u128) * c->ver_len);
  int ok = 1;
  for (unsigned i = 0; i < c->ver_len; ++i) {
    u128 a, b;
    if (!f_decode(F, lps + i * F->es, &a) || !f_decode(F, hps + i * F->es, &b)) ok = 0;
    else v[i] = f_add(F, a, b);
  }
  if (ok) ok = flp_decide(c, v);
  free(v);
  if (!ok) return 5;
  if (c->jr_len) joint_rand_seed(c, lps + c->ver_len * F->es, hps + c->ver_len * F->es, msg);
  return 0;
}

/* ============================ batch API (ctypes) =========================================== */
typedef struct {
  cfgt c;
} p3ref;

p3ref* p3ref_new(int kind, unsigned bits, unsigned length, unsigned chunk, const u8 vk[16]) {
  p3ref* r = (p3ref*)calloc(1, sizeof *r);
  if (p3ref_cfg_init(&r->c, kind, bits, length, chunk, vk)) {
    free(r);
    return NULL;
  }
  return r;
}
void p3ref_free(p3ref* r) { free(r); }
void p3ref_sizes(const p3ref* r, unsigned out[8]) {
  const cfgt* c = &r->c;
  out[0] = c->F->es; out[1] = p3ref_leader_len(c); out[2] = p3ref_helper_len(c);
  out[3] = p3ref_public_len(c); out[4] = p3ref_prep_len(c); out[5] = c->jr_len ? 16 : 0;
  out[6] = c->out_len * c->F->es; out[7] = p3ref_random_size(c);
}

/* synthetic report i: stream = SHAKE128("janus-prio3-bench" || cfg_id || u64le(i)),
 * nonce = stream[0:16], rand = next random_size bytes, measurement from the tail. */
static void synth(const cfgt* c, const u8* cfg_id, size_t cfg_len, u64 i, u8 nonce[16], u8* rand,
                  u128* encoded, u64* meas_out) {
  shake h;
  shake_init(&h);
  shake_absorb(&h, (const u8*)"janus-prio3-bench", 17);
  shake_absorb(&h, cfg_id, cfg_len);
  u8 ib[8];
  for (int b = 0; b < 8; ++b) ib[b] = (u8)(i >> (8 * b));
  shake_absorb(&h, ib, 8);
  shake_finish(&h);
  shake_squeeze(&h, nonce, 16);
  unsigned rs = p3ref_random_size(c);
  shake_squeeze(&h, rand, rs);
  const field* F = c->F;
  for (unsigned k = 0; k < c->meas_len; ++k) encoded[k] = 0;
  if (c->kind == K_FPVEC) {
    /* integer entries uniform in [-B, B], entries * B^2 <= (2^(n-1)-1)^2
     * (oracle/prio3.py synth_fixedpoint), 8 stream bytes per entry */
    const unsigned nb = c->bits;
    const u128 one = ((u128)1 << (nb - 1)) - 1;
    const u128 q = one * one / c->length;
    u128 B = 0;
    { /* isqrt */
      u128 lo = 0, hi = (u128)1 << 64;
      while (lo < hi) {
        u128 mid = (lo + hi + 1) / 2;
        if (mid * mid <= q) lo = mid; else hi = mid - 1;
      }
      B = lo;
    }
    u128 norm = 0;
    for (unsigned e = 0; e < c->length; ++e) {
      u8 b[8];
      shake_squeeze(&h, b, 8);
      u64 v = 0;
      for (int k = 0; k < 8; ++k) v |= (u64)b[k] << (8 * k);
      long long sv = (long long)((u128)v % (2 * B + 1)) - (long long)B;
      meas_out[e] = (u64)sv;
      const u64 z = (u64)sv + ((u64)1 << (nb - 1)); /* two's complement with the top bit flipped */
      for (unsigned k = 0; k < nb; ++k) encoded[(size_t)e * nb + k] = (z >> k & 1) ? F->one : 0;
      norm += (u128)((__int128)sv * sv);
    }
    for (unsigned k = 0; k < 2 * nb - 2; ++k)
      encoded[(size_t)nb * c->length + k] = (norm >> k & 1) ? F->one : 0;
    return;
  }
  if (c->kind == K_SUMVEC) {
    unsigned nb = (c->bits + 7) / 8;
    for (unsigned e = 0; e < c->length; ++e) {
      u8 b[8] = {0};
      shake_squeeze(&h, b, nb);
      u64 v = 0;
      for (unsigned q = 0; q < nb; ++q) v |= (u64)b[q] << (8 * q);
      if (c->bits < 64) v &= ((u64)1 << c->bits) - 1;
      meas_out[e] = v;
      for (unsigned q = 0; q < c->bits; ++q) encoded[e * c->bits + q] = (v >> q & 1) ? F->one : 0;
    }
    return;
  }
  u8 b[8];
  shake_squeeze(&h, b, 8);
  u64 v = 0;
  for (int q = 0; q < 8; ++q) v |= (u64)b[q] << (8 * q);
  if (c->kind == K_COUNT) {
    v = b[0] & 1;
    encoded[0] = v ? F->one : 0;
  } else if (c->kind == K_SUM) {
    if (c->bits < 64) v &= ((u64)1 << c->bits) - 1;
    for (unsigned q = 0; q < c->bits; ++q) encoded[q] = (v >> q & 1) ? F->one : 0;
  } else {
    v %= c->length;
    encoded[v] = F->one;
  }
  meas_out[0] = v;
}

typedef struct {
  const p3ref* r;
  const u8* cfg_id;
  size_t cfg_len;
  u64 start;
  size_t lo, hi;
  u8 *nonces, *pub, *leader, *helper;
  u64* meas;
  /* prepare */
  const u8 *c_nonces, *c_pub, *c_leader, *c_helper;
  u8 *lprep, *hprep, *msgs, *status;
  u128* agg_l; /* per-thread aggregates (Montgomery) */
  u128* agg_h;
  unsigned long long count;
} job;

static void* gen_worker(void* arg) {
  job* j = (job*)arg;
  const cfgt* c = &j->r->c;
  const unsigned rs = p3ref_random_size(c);
  const unsigned L = p3ref_leader_len(c), H = p3ref_helper_len(c), P = p3ref_public_len(c);
  const unsigned mw = (c->kind == K_SUMVEC || c->kind == K_FPVEC) ? c->length : 1;
  u8* rand = (u8*)malloc(rs);
  u128* enc = (u128*)malloc(sizeof(u128) * c->meas_len);
  for (size_t k = j->lo; k < j->hi; ++k) {
    synth(c, j->cfg_id, j->cfg_len, j->start + k, j->nonces + 16 * k, rand, enc,
          j->meas + mw * k);
    shard(c, enc, j->nonces + 16 * k, rand, j->pub + (size_t)P * k, j->leader + (size_t)L * k,
          j->helper + (size_t)H * k);
  }
  free(rand);
  free(enc);
  return NULL;
}

static void run_jobs(job* jobs, int threads, void* (*fn)(void*)) {
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * threads);
  for (int t = 0; t < threads; ++t) pthread_create(&th[t], NULL, fn, &jobs[t]);
  for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
  free(th);
}

/* Generate n synthetic reports starting at index `start`.  meas: n x (SumVec ? length : 1). */
int p3ref_gen(const p3ref* r, const u8* cfg_id, size_t cfg_len, u64 start, size_t n, int threads,
              u8* nonces, u8* pub, u8* leader, u8* helper, u64* meas) {
  if (threads < 1) threads = 1;
  job* jobs = (job*)calloc(threads, sizeof(job));
  for (int t = 0; t < threads; ++t) {
    job* j = &jobs[t];
    j->r = r; j->cfg_id = cfg_id; j->cfg_len = cfg_len; j->start = start;
    j->lo = n * t / threads; j->hi = n * (t + 1) / threads;
    j->nonces = nonces; j->pub = pub; j->leader = leader; j->helper = helper; j->meas = meas;
  }
  run_jobs(jobs, threads, gen_worker);
  free(jobs);
  return 0;
}

/* One report prepared by both aggregators and accumulated into both aggregates (the bench unit):
 * leader prepare_init, helper prepare_init + prep_shares_to_prep + prepare_next, leader
 * prepare_next, accumulate. */
static void* prep_worker(void* arg) {
  job* j = (job*)arg;
  const cfgt* c = &j->r->c;
  const field* F = c->F;
  const unsigned L = p3ref_leader_len(c), H = p3ref_helper_len(c), P = p3ref_public_len(c);
  const unsigned PS = p3ref_prep_len(c);
  u8* lps = (u8*)malloc(PS);
  u8* hps = (u8*)malloc(PS);
  u128* lo = (u128*)malloc(sizeof(u128) * c->out_len);
  u128* ho = (u128*)malloc(sizeof(u128) * c->out_len);
  for (size_t k = j->lo; k < j->hi; ++k) {
    u8 lseed[16], hseed[16], msg[16];
    const u8* nonce = j->c_nonces + 16 * k;
    const u8* pub = j->c_pub + (size_t)P * k;
    int st = prepare_init(c, 0, nonce, pub, j->c_leader + (size_t)L * k, lps, lo, lseed);
    if (!st) st = prepare_init(c, 1, nonce, pub, j->c_helper + (size_t)H * k, hps, ho, hseed);
    if (!st) st = prep_shares_to_prep(c, lps, hps, msg);
    if (!st && c->jr_len && memcmp(msg, hseed, 16)) st = 5; /* helper prepare_next */
    if (!st && c->jr_len && memcmp(msg, lseed, 16)) st = 5; /* leader prepare_next */
    if (j->lprep) memcpy(j->lprep + (size_t)PS * k, lps, PS);
    if (j->hprep) memcpy(j->hprep + (size_t)PS * k, hps, PS);
    if (j->msgs && c->jr_len) memcpy(j->msgs + 16 * k, msg, 16);
    if (j->status) j->status[k] = (u8)st;
    if (!st) {
      for (unsigned e = 0; e < c->out_len; ++e) {
        j->agg_l[e] = f_add(F, j->agg_l[e], lo[e]);
        j->agg_h[e] = f_add(F, j->agg_h[e], ho[e]);
      }
      j->count++;
    }
  }
  free(lps); free(hps); free(lo); free(ho);
  return NULL;
}

/* CPU baseline / checker: prepare n reports with `threads` threads (one report per thread at a
 * time), writing optional per-report outputs and the two aggregate shares (encoded). */
long long p3ref_prepare_batch(const p3ref* r, size_t n, int threads, const u8* nonces,
                              const u8* pub, const u8* leader, const u8* helper, u8* lprep,
                              u8* hprep, u8* msgs, u8* status, u8* agg_l, u8* agg_h) {
  const cfgt* c = &r->c;
  const field* F = c->F;
  if (threads < 1) threads = 1;
  job* jobs = (job*)calloc(threads, sizeof(job));
  for (int t = 0; t < threads; ++t) {
    job* j = &jobs[t];
    j->r = r; j->lo = n * t / threads; j->hi = n * (t + 1) / threads;
    j->c_nonces = nonces; j->c_pub = pub; j->c_leader = leader; j->c_helper = helper;
    j->lprep = lprep; j->hprep = hprep; j->msgs = msgs; j->status = status;
    j->agg_l = (u128*)calloc(c->out_len, sizeof(u128));
    j->agg_h = (u128*)calloc(c->out_len, sizeof(u128));
  }
  run_jobs(jobs, threads, prep_worker);
  long long count = 0;
  for (unsigned e = 0; e < c->out_len; ++e) {
    u128 a = 0, b = 0;
    for (int t = 0; t < threads; ++t) {
      a = f_add(F, a, jobs[t].agg_l[e]);
      b = f_add(F, b, jobs[t].agg_h[e]);
    }
    if (agg_l) f_encode(F, a, agg_l + (size_t)e * F->es);
    if (agg_h) f_encode(F, b, agg_h + (size_t)e * F->es);
  }
  for (int t = 0; t < threads; ++t) {
    count += (long long)jobs[t].count;
    free(jobs[t].agg_l);
    free(jobs[t].agg_h);
  }
  free(jobs);
  return count;
}

/* SHAKE128 one-shot (tests cross-check against hashlib / FIPS 202). */
void p3ref_shake128(const u8* msg, size_t len, u8* out, size_t outlen) {
  shake h;
  shake_init(&h);
  shake_absorb(&h, msg, len);
  shake_finish(&h);
  shake_squeeze(&h, out, outlen);
}

/* Synthetic report inputs only (nonce, client randomness, measurement) per the SURVEY §8(d)
 * recipe, for n reports from index `start`; the shares are then produced by prio3gpu_shard. */
typedef struct {
  const p3ref* r;
  const u8* cfg_id;
  size_t cfg_len;
  u64 start;
  size_t lo, hi;
  u8 *nonces, *rand;
  u64* meas;
} synth_job;

static void* synth_worker(void* arg) {
  synth_job* j = (synth_job*)arg;
  const cfgt* c = &j->r->c;
  const unsigned rs = p3ref_random_size(c);
  const unsigned mw = (c->kind == K_SUMVEC || c->kind == K_FPVEC) ? c->length : 1;
  u128* enc = (u128*)malloc(sizeof(u128) * c->meas_len);
  for (size_t k = j->lo; k < j->hi; ++k)
    synth(c, j->cfg_id, j->cfg_len, j->start + k, j->nonces + 16 * k, j->rand + (size_t)rs * k, enc,
          j->meas + (size_t)mw * k);
  free(enc);
  return NULL;
}

int p3ref_synth(const p3ref* r, const u8* cfg_id, size_t cfg_len, u64 start, size_t n, int threads,
                u8* nonces, u8* rand, u64* meas) {
  if (threads < 1) threads = 1;
  synth_job* jobs = (synth_job*)calloc(threads, sizeof(synth_job));
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * threads);
  for (int t = 0; t < threads; ++t) {
    synth_job* j = &jobs[t];
    j->r = r; j->cfg_id = cfg_id; j->cfg_len = cfg_len; j->start = start;
    j->lo = n * t / threads; j->hi = n * (t + 1) / threads;
    j->nonces = nonces; j->rand = rand; j->meas = meas;
    pthread_create(&th[t], NULL, synth_worker, j);
  }
  for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
  free(th);
  free(jobs);
  return 0;
}
