// HPKE (RFC 9180, base mode, single shot) for the helper's aggregate-init input shares, on CPU
// threads in front of the codec edge (the north star keeps HPKE open on the
// host).  Host code, part of libprio3gpu.so, built on the image's OpenSSL 3.0 libcrypto
// primitives (X25519 / P-256 ECDH, SHA-2, AES-GCM, ChaCha20-Poly1305); the HPKE construction
// itself (DHKEM, labeled HKDF, key schedule) is written out here.
//
// Reference behaviour:
//   hpke::open / hpke::seal                         core/src/hpke.rs:158-202 (hpke-dispatch crate,
//                                                    base_mode_open / base_mode_seal)
//   HpkeApplicationInfo = label || sender || recipient  core/src/hpke.rs:44-77
//   supported suites: KEM X25519HkdfSha256 (0x20), P256HkdfSha256 (0x10); KDF HkdfSha256/384/512
//     (1/2/3); AEAD Aes128Gcm / Aes256Gcm / ChaCha20Poly1305 (1/2/3)  messages/src/lib.rs (HpkeKemId,
//     HpkeKdfId, HpkeAeadId); pinned by core/src/hpke.rs:539-615 (RFC 9180 test vectors)
//   helper per-report open: keypair by config id from the task's keys, then the global keys;
//     unknown id -> HpkeUnknownConfigId (3); the task key is tried first and the global key
//     only after a decryption failure; any failure -> HpkeDecryptError (4)
//                                                    aggregator/src/aggregator.rs:1634-1700
//   InputShareAad = TaskId[32] || ReportMetadata{ReportId[16], Time u64 BE} ||
//     u32-prefixed public share                      messages/src/lib.rs:1790-1827
#define OPENSSL_SUPPRESS_DEPRECATED  // low-level SHA-2 / AES / GCM128: no library-context locks
#include <openssl/aes.h>
#include <openssl/bn.h>
#include <openssl/ec.h>
#include <openssl/evp.h>
#include <openssl/obj_mac.h>
#include <openssl/modes.h>
#include <openssl/rand.h>
#include <openssl/sha.h>

#include <immintrin.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/prio3gpu.h"
#include "../../include/prio3gpu_test.h"

namespace {

enum : uint16_t { KEM_P256 = 0x10, KEM_X25519 = 0x20 };
enum : uint16_t { KDF_SHA256 = 1, KDF_SHA384 = 2, KDF_SHA512 = 3 };
enum : uint16_t { AEAD_AES128GCM = 1, AEAD_AES256GCM = 2, AEAD_CHACHA20POLY1305 = 3 };
constexpr size_t kTag = 16, kNonce = 12, kMaxHash = 64;

struct Algs {
  const EVP_MD* md[4] = {};          // by KDF id (1..3)
  const EVP_CIPHER* aead[4] = {};    // by AEAD id (1..3)
  EC_GROUP* p256 = nullptr;
  bool ok = false;
};

// Fetched once: per-call implicit fetches are the slow part of OpenSSL 3 one-shot APIs.
const Algs& algs() {
  static Algs a;
  static std::once_flag once;
  std::call_once(once, [] {
    a.md[1] = EVP_MD_fetch(nullptr, "SHA256", nullptr);
    a.md[2] = EVP_MD_fetch(nullptr, "SHA384", nullptr);
    a.md[3] = EVP_MD_fetch(nullptr, "SHA512", nullptr);
    a.aead[1] = EVP_CIPHER_fetch(nullptr, "AES-128-GCM", nullptr);
    a.aead[2] = EVP_CIPHER_fetch(nullptr, "AES-256-GCM", nullptr);
    a.aead[3] = EVP_CIPHER_fetch(nullptr, "ChaCha20-Poly1305", nullptr);
    a.p256 = EC_GROUP_new_by_curve_name(NID_X9_62_prime256v1);
    a.ok = a.md[1] && a.md[2] && a.md[3] && a.aead[1] && a.aead[2] && a.aead[3] && a.p256;
  });
  return a;
}

struct Suite {
  uint16_t kem, kdf, aead;
  size_t nsecret, nenc, npk, nsk;  // KEM sizes (RFC 9180 §7.1)
  size_t nk;                       // AEAD key size
  size_t nh;                       // KDF output size
};

bool suite_of(uint16_t kem, uint16_t kdf, uint16_t aead, Suite* s) {
  s->kem = kem, s->kdf = kdf, s->aead = aead;
  if (kem == KEM_X25519) { s->nsecret = 32; s->nenc = s->npk = 32; s->nsk = 32; }
  else if (kem == KEM_P256) { s->nsecret = 32; s->nenc = s->npk = 65; s->nsk = 32; }
  else return false;
  if (kdf == KDF_SHA256) s->nh = 32;
  else if (kdf == KDF_SHA384) s->nh = 48;
  else if (kdf == KDF_SHA512) s->nh = 64;
  else return false;
  if (aead == AEAD_AES128GCM) s->nk = 16;
  else if (aead == AEAD_AES256GCM || aead == AEAD_CHACHA20POLY1305) s->nk = 32;
  else return false;
  return algs().ok;
}

// ---- HMAC / HKDF over a pre-fetched digest -------------------------------------------------

struct Bytes {
  std::vector<uint8_t> v;
  Bytes& add(const void* p, size_t n) {
    const uint8_t* b = static_cast<const uint8_t*>(p);
    v.insert(v.end(), b, b + n);
    return *this;
  }
  Bytes& add(const char* s) { return add(s, strlen(s)); }
  Bytes& u16(uint16_t x) {
    uint8_t b[2] = {uint8_t(x >> 8), uint8_t(x)};
    return add(b, 2);
  }
};

// SHA-2 through OpenSSL's low-level (SHA-NI) entry points: the EVP digest path looks the
// algorithm up in the library context under a shared lock on every init, and 16 threads opening
// reports spent most of their time on that lock (measured on the GPU box: 1 thread 5.3 us per
// open, 16 threads 32 us).  Selected by the EVP_MD's output size (32 / 48 / 64).
struct Sha2 {
  size_t hl;
  SHA256_CTX c256;
  SHA512_CTX c512;
  explicit Sha2(size_t h) : hl(h) {
    if (hl == 32) SHA256_Init(&c256);
    else if (hl == 48) SHA384_Init(&c512);
    else SHA512_Init(&c512);
  }
  void update(const void* p, size_t n) {
    if (hl == 32) SHA256_Update(&c256, p, n);
    else if (hl == 48) SHA384_Update(&c512, p, n);
    else SHA512_Update(&c512, p, n);
  }
  void final(uint8_t* out) {
    if (hl == 32) SHA256_Final(out, &c256);
    else if (hl == 48) SHA384_Final(out, &c512);
    else SHA512_Final(out, &c512);
  }
};

struct Seg {
  const void* p;
  size_t n;
};

// HMAC over the concatenation of segs (no intermediate message buffer).
bool hmac_segs(const EVP_MD* md, const uint8_t* key, size_t klen, const Seg* segs, int nseg,
               uint8_t* out) {
  const size_t hl = EVP_MD_get_size(md), bs = hl == 32 ? 64 : 128;
  uint8_t k0[128] = {0}, pad[128];
  if (klen > bs) {
    Sha2 h(hl);
    h.update(key, klen);
    h.final(k0);
  } else if (klen) {
    memcpy(k0, key, klen);
  }
  uint8_t inner[kMaxHash];
  for (size_t i = 0; i < bs; ++i) pad[i] = k0[i] ^ 0x36;
  Sha2 hi(hl);
  hi.update(pad, bs);
  for (int k = 0; k < nseg; ++k)
    if (segs[k].n) hi.update(segs[k].p, segs[k].n);
  hi.final(inner);
  for (size_t i = 0; i < bs; ++i) pad[i] = k0[i] ^ 0x5c;
  Sha2 ho(hl);
  ho.update(pad, bs);
  ho.update(inner, hl);
  ho.final(out);
  return true;
}

bool hmac(const EVP_MD* md, const uint8_t* key, size_t klen, const uint8_t* msg, size_t mlen,
          uint8_t* out) {
  const Seg seg{msg, mlen};
  return hmac_segs(md, key, klen, &seg, 1, out);
}

// LabeledExtract(salt, label, ikm) = HMAC(salt, "HPKE-v1" || suite_id || label || ikm)  (§4)
bool labeled_extract(const EVP_MD* md, const Bytes& suite_id, const uint8_t* salt, size_t slen,
                     const char* label, const uint8_t* ikm, size_t ilen, uint8_t* prk) {
  const Seg segs[4] = {{"HPKE-v1", 7}, {suite_id.v.data(), suite_id.v.size()},
                       {label, strlen(label)}, {ikm, ilen}};
  return hmac_segs(md, salt, slen, segs, 4, prk);
}

// LabeledExpand(prk, label, info, L) = HKDF-Expand(prk, I2OSP(L,2) || "HPKE-v1" || suite_id ||
// label || info, L)
bool labeled_expand(const EVP_MD* md, const Bytes& suite_id, const uint8_t* prk, size_t plen,
                    const char* label, const uint8_t* info, size_t ilen, size_t L, uint8_t* out) {
  const size_t hl = EVP_MD_get_size(md);
  if (L > 255 * hl) return false;
  const uint8_t lbe[2] = {uint8_t(L >> 8), uint8_t(L)};
  uint8_t t[kMaxHash];
  size_t tl = 0, done = 0;
  for (uint8_t i = 1; done < L; ++i) {
    const Seg segs[7] = {{t, tl},     {lbe, 2},     {"HPKE-v1", 7}, {suite_id.v.data(), suite_id.v.size()},
                         {label, strlen(label)}, {info, ilen}, {&i, 1}};
    if (!hmac_segs(md, prk, plen, segs, 7, t)) return false;
    tl = hl;
    const size_t c = std::min(hl, L - done);
    memcpy(out + done, t, c);
    done += c;
  }
  return true;
}

// ---- DHKEM (§4.1) --------------------------------------------------------------------------

// X25519 (RFC 7748 §5), radix 2^51.  Written out rather than taken from EVP_PKEY: OpenSSL
// 3.0's per-call key/ctx construction serialises threads on provider locks (measured: 8 threads
// opened 1.6x what 1 thread did), which is the very scaling the batched open needs.
typedef unsigned __int128 u128;
constexpr uint64_t kM51 = (uint64_t(1) << 51) - 1;
struct Fe { uint64_t v[5]; };

inline void fe_load(Fe& h, const uint8_t* s) {
  uint64_t w[4];
  memcpy(w, s, 32);  // little-endian host
  h.v[0] = w[0] & kM51;
  h.v[1] = ((w[0] >> 51) | (w[1] << 13)) & kM51;
  h.v[2] = ((w[1] >> 38) | (w[2] << 26)) & kM51;
  h.v[3] = ((w[2] >> 25) | (w[3] << 39)) & kM51;
  h.v[4] = (w[3] >> 12) & kM51;  // bit 255 masked (RFC 7748 §5)
}

inline void fe_carry(Fe& h, const u128 r[5]) {
  u128 c = 0, t[5];
  for (int i = 0; i < 5; ++i) {
    t[i] = r[i] + c;
    c = t[i] >> 51;
    t[i] &= kM51;
  }
  const u128 t0 = t[0] + c * 19;
  h.v[0] = uint64_t(t0 & kM51);
  h.v[1] = uint64_t(t[1] + (t0 >> 51));
  for (int i = 2; i < 5; ++i) h.v[i] = uint64_t(t[i]);
}

inline void fe_mul(Fe& h, const Fe& f, const Fe& g) {
  const uint64_t* a = f.v;
  const uint64_t* b = g.v;
  const uint64_t b1 = 19 * b[1], b2 = 19 * b[2], b3 = 19 * b[3], b4 = 19 * b[4];
  u128 r[5];
  r[0] = (u128)a[0] * b[0] + (u128)a[1] * b4 + (u128)a[2] * b3 + (u128)a[3] * b2 + (u128)a[4] * b1;
  r[1] = (u128)a[0] * b[1] + (u128)a[1] * b[0] + (u128)a[2] * b4 + (u128)a[3] * b3 + (u128)a[4] * b2;
  r[2] = (u128)a[0] * b[2] + (u128)a[1] * b[1] + (u128)a[2] * b[0] + (u128)a[3] * b4 +
         (u128)a[4] * b3;
  r[3] = (u128)a[0] * b[3] + (u128)a[1] * b[2] + (u128)a[2] * b[1] + (u128)a[3] * b[0] +
         (u128)a[4] * b4;
  r[4] = (u128)a[0] * b[4] + (u128)a[1] * b[3] + (u128)a[2] * b[2] + (u128)a[3] * b[1] +
         (u128)a[4] * b[0];
  fe_carry(h, r);
}

inline void fe_sq(Fe& h, const Fe& f) {  // 15 products instead of 25
  const uint64_t* a = f.v;
  const uint64_t d0 = 2 * a[0], d1 = 2 * a[1], d2 = 2 * a[2];
  const uint64_t a3_19 = 19 * a[3], a4_19 = 19 * a[4];
  u128 r[5];
  r[0] = (u128)a[0] * a[0] + (u128)d1 * a4_19 + (u128)(2 * a[2]) * a3_19;
  r[1] = (u128)d0 * a[1] + (u128)d2 * a4_19 + (u128)a[3] * a3_19;
  r[2] = (u128)d0 * a[2] + (u128)a[1] * a[1] + (u128)(2 * a[3]) * a4_19;
  r[3] = (u128)d0 * a[3] + (u128)d1 * a[2] + (u128)a[4] * a4_19;
  r[4] = (u128)d0 * a[4] + (u128)d1 * a[3] + (u128)a[2] * a[2];
  fe_carry(h, r);
}

inline void fe_sqn(Fe& h, const Fe& f, int n) {
  fe_sq(h, f);
  for (int i = 1; i < n; ++i) fe_sq(h, h);
}

// z^(p-2) = z^(2^255 - 21): the usual addition chain (254 squarings, 11 multiplications)
void fe_invert(Fe& out, const Fe& z) {
  Fe z2, z9, z11, z_5_0, z_10_0, z_20_0, z_50_0, z_100_0, t;
  fe_sq(z2, z);
  fe_sqn(t, z2, 2);
  fe_mul(z9, t, z);
  fe_mul(z11, z9, z2);
  fe_sq(t, z11);
  fe_mul(z_5_0, t, z9);
  fe_sqn(t, z_5_0, 5);
  fe_mul(z_10_0, t, z_5_0);
  fe_sqn(t, z_10_0, 10);
  fe_mul(z_20_0, t, z_10_0);
  fe_sqn(t, z_20_0, 20);
  fe_mul(t, t, z_20_0);
  fe_sqn(t, t, 10);
  fe_mul(z_50_0, t, z_10_0);
  fe_sqn(t, z_50_0, 50);
  fe_mul(z_100_0, t, z_50_0);
  fe_sqn(t, z_100_0, 100);
  fe_mul(t, t, z_100_0);
  fe_sqn(t, t, 50);
  fe_mul(t, t, z_50_0);
  fe_sqn(t, t, 5);
  fe_mul(out, t, z11);
}

inline void fe_mul_small(Fe& h, const Fe& f, uint64_t k) {
  u128 r[5];
  for (int i = 0; i < 5; ++i) r[i] = (u128)f.v[i] * k;
  fe_carry(h, r);
}

inline void fe_add(Fe& h, const Fe& f, const Fe& g) {
  for (int i = 0; i < 5; ++i) h.v[i] = f.v[i] + g.v[i];
}

// f - g with a 2p bias; g must be a multiplication output (limbs < 2^51 + 2^20).
inline void fe_sub(Fe& h, const Fe& f, const Fe& g) {
  h.v[0] = f.v[0] + 0xFFFFFFFFFFFDAull - g.v[0];
  for (int i = 1; i < 5; ++i) h.v[i] = f.v[i] + 0xFFFFFFFFFFFFEull - g.v[i];
}

inline void fe_cswap(Fe& a, Fe& b, uint64_t swap) {
  const uint64_t m = 0 - swap;
  for (int i = 0; i < 5; ++i) {
    const uint64_t t = m & (a.v[i] ^ b.v[i]);
    a.v[i] ^= t;
    b.v[i] ^= t;
  }
}

void fe_store(uint8_t* s, const Fe& f) {
  Fe h = f;
  for (int pass = 0; pass < 2; ++pass) {
    uint64_t c = 0;
    for (int i = 0; i < 5; ++i) {
      h.v[i] += c;
      c = h.v[i] >> 51;
      h.v[i] &= kM51;
    }
    h.v[0] += 19 * c;
  }
  uint64_t q = (h.v[0] + 19) >> 51;  // q = 1 iff h >= p
  for (int i = 1; i < 5; ++i) q = (h.v[i] + q) >> 51;
  h.v[0] += 19 * q;
  uint64_t c = 0;
  for (int i = 0; i < 5; ++i) {
    h.v[i] += c;
    c = h.v[i] >> 51;
    h.v[i] &= kM51;
  }
  const uint64_t w[4] = {h.v[0] | (h.v[1] << 51), (h.v[1] >> 13) | (h.v[2] << 38),
                         (h.v[2] >> 26) | (h.v[3] << 25), (h.v[3] >> 39) | (h.v[4] << 12)};
  memcpy(s, w, 32);
}

void x25519(uint8_t* out, const uint8_t* scalar, const uint8_t* point) {
  uint8_t k[32];
  memcpy(k, scalar, 32);
  k[0] &= 248;  // decodeScalar25519
  k[31] &= 127;
  k[31] |= 64;
  Fe x1, x2 = {{1, 0, 0, 0, 0}}, z2 = {{0, 0, 0, 0, 0}}, x3, z3 = {{1, 0, 0, 0, 0}};
  fe_load(x1, point);
  x3 = x1;
  uint64_t swap = 0;
  for (int t = 254; t >= 0; --t) {
    const uint64_t kt = (k[t >> 3] >> (t & 7)) & 1;
    swap ^= kt;
    fe_cswap(x2, x3, swap);
    fe_cswap(z2, z3, swap);
    swap = kt;
    Fe A, AA, B, BB, E, C, D, DA, CB, t0, t1;
    fe_add(A, x2, z2);
    fe_sq(AA, A);
    fe_sub(B, x2, z2);
    fe_sq(BB, B);
    fe_sub(E, AA, BB);
    fe_add(C, x3, z3);
    fe_sub(D, x3, z3);
    fe_mul(DA, D, A);
    fe_mul(CB, C, B);
    fe_add(t0, DA, CB);
    fe_sq(x3, t0);
    fe_sub(t1, DA, CB);
    fe_sq(t1, t1);
    fe_mul(z3, x1, t1);
    fe_mul(x2, AA, BB);
    fe_mul_small(t0, E, 121665);
    fe_add(t0, AA, t0);
    fe_mul(z2, E, t0);
  }
  fe_cswap(x2, x3, swap);
  fe_cswap(z2, z3, swap);
  Fe r;
  fe_invert(r, z2);
  fe_mul(x2, x2, r);
  fe_store(out, x2);
}

// ---- 8-way X25519 with AVX-512 IFMA ---------------------------------------------------------
// The helper opens every report of a job with the SAME private key, so the ladder's swap pattern
// is common to all reports: eight DH computations run in lock step, one report per 64-bit lane,
// limb-sliced (Fe8.v[i] = limb i of the eight field elements).  Radix 2^51 with limbs < 2^52 (the
// IFMA input width): vpmadd52lo/hi give the low / high 52 bits of each 52x52 product; a high
// half weighs 2^52 = 2 * 2^51, so column k = L_k + 2 H_(k-1) (< 15 * 2^52), columns 5..9 fold
// with 2^255 = 19 (< 2^61), and one parallel carry brings every limb under 2^51 + 2^15.
// Dispatched at run time (cpuid); both this container's Xeon and the GPU box's EPYC (Zen 5) have
// IFMA.  Checked against the scalar ladder and the RFC 9180 vectors (tests/test_hpke.py).
#define IFMA_FN static inline __attribute__((target("avx512f,avx512ifma"), always_inline))
struct Fe8 { __m512i v[5]; };

IFMA_FN __m512i mul19(__m512i x) {  // x < 2^58
  return _mm512_add_epi64(_mm512_add_epi64(_mm512_slli_epi64(x, 4), _mm512_slli_epi64(x, 1)), x);
}

IFMA_FN void fe8_carry(Fe8& h) {  // limbs < 2^62 -> < 2^51 + (input >> 51)
  const __m512i m = _mm512_set1_epi64(kM51);
  __m512i c[5];
  for (int i = 0; i < 5; ++i) c[i] = _mm512_srli_epi64(h.v[i], 51);
  h.v[0] = _mm512_add_epi64(_mm512_and_si512(h.v[0], m), mul19(c[4]));
  for (int i = 1; i < 5; ++i) h.v[i] = _mm512_add_epi64(_mm512_and_si512(h.v[i], m), c[i - 1]);
}

IFMA_FN void fe8_mul(Fe8& h, const Fe8& f, const Fe8& g) {  // f, g limbs < 2^52
  const __m512i z = _mm512_setzero_si512();
  __m512i L[9], H[9];
  for (int k = 0; k < 9; ++k) L[k] = H[k] = z;
  for (int i = 0; i < 5; ++i)
    for (int j = 0; j < 5; ++j) {
      L[i + j] = _mm512_madd52lo_epu64(L[i + j], f.v[i], g.v[j]);
      H[i + j] = _mm512_madd52hi_epu64(H[i + j], f.v[i], g.v[j]);
    }
  __m512i col[10];
  col[0] = L[0];
  for (int k = 1; k < 9; ++k) col[k] = _mm512_add_epi64(L[k], _mm512_add_epi64(H[k - 1], H[k - 1]));
  col[9] = _mm512_add_epi64(H[8], H[8]);
  for (int k = 0; k < 5; ++k) h.v[k] = _mm512_add_epi64(col[k], mul19(col[k + 5]));
  fe8_carry(h);
}

IFMA_FN void fe8_mul_small(Fe8& h, const Fe8& f, uint64_t k) {  // k < 2^52: 10 products
  const __m512i z = _mm512_setzero_si512(), kk = _mm512_set1_epi64((long long)k);
  __m512i lo[5], hi[5];
  for (int i = 0; i < 5; ++i) {
    lo[i] = _mm512_madd52lo_epu64(z, f.v[i], kk);
    hi[i] = _mm512_madd52hi_epu64(z, f.v[i], kk);
  }
  // column i = lo_i + 2 hi_(i-1); column 5 = 2 hi_4 folds into column 0 with x19
  h.v[0] = _mm512_add_epi64(lo[0], mul19(_mm512_add_epi64(hi[4], hi[4])));
  for (int i = 1; i < 5; ++i) h.v[i] = _mm512_add_epi64(lo[i], _mm512_add_epi64(hi[i - 1], hi[i - 1]));
  fe8_carry(h);
}

IFMA_FN void fe8_sq(Fe8& h, const Fe8& f) {  // 15 products: cross terms doubled in the columns
  const __m512i z = _mm512_setzero_si512();
  __m512i L[9], H[9], LD[9], HD[9];
  for (int k = 0; k < 9; ++k) L[k] = H[k] = LD[k] = HD[k] = z;
  for (int i = 0; i < 5; ++i) {
    L[2 * i] = _mm512_madd52lo_epu64(L[2 * i], f.v[i], f.v[i]);
    H[2 * i] = _mm512_madd52hi_epu64(H[2 * i], f.v[i], f.v[i]);
    for (int j = i + 1; j < 5; ++j) {
      LD[i + j] = _mm512_madd52lo_epu64(LD[i + j], f.v[i], f.v[j]);
      HD[i + j] = _mm512_madd52hi_epu64(HD[i + j], f.v[i], f.v[j]);
    }
  }
  // column k = L_k + 2 LD_k + 2 (H_(k-1) + 2 HD_(k-1));  LD, HD < 2 * 2^52, so col < 2^56
  __m512i col[10];
  for (int k = 0; k < 10; ++k) {
    __m512i c = k < 9 ? _mm512_add_epi64(L[k], _mm512_slli_epi64(LD[k], 1)) : z;
    if (k > 0)
      c = _mm512_add_epi64(
          c, _mm512_slli_epi64(_mm512_add_epi64(H[k - 1], _mm512_slli_epi64(HD[k - 1], 1)), 1));
    col[k] = c;
  }
  for (int k = 0; k < 5; ++k) h.v[k] = _mm512_add_epi64(col[k], mul19(col[k + 5]));
  fe8_carry(h);
}

IFMA_FN void fe8_add(Fe8& h, const Fe8& f, const Fe8& g) {
  for (int i = 0; i < 5; ++i) h.v[i] = _mm512_add_epi64(f.v[i], g.v[i]);
  fe8_carry(h);
}

// f - g + 2p;  g limbs <= 2^52 - 38 (every Fe8 value is a carry output: < 2^51 + 2^15)
IFMA_FN void fe8_sub(Fe8& h, const Fe8& f, const Fe8& g) {
  const __m512i b0 = _mm512_set1_epi64(0xFFFFFFFFFFFDAll), b = _mm512_set1_epi64(0xFFFFFFFFFFFFEll);
  for (int i = 0; i < 5; ++i)
    h.v[i] = _mm512_sub_epi64(_mm512_add_epi64(f.v[i], i ? b : b0), g.v[i]);
  fe8_carry(h);
}

IFMA_FN void fe8_cswap(Fe8& a, Fe8& b, uint64_t swap) {
  const __m512i m = _mm512_set1_epi64((long long)(0 - swap));
  for (int i = 0; i < 5; ++i) {
    const __m512i t = _mm512_and_si512(m, _mm512_xor_si512(a.v[i], b.v[i]));
    a.v[i] = _mm512_xor_si512(a.v[i], t);
    b.v[i] = _mm512_xor_si512(b.v[i], t);
  }
}

IFMA_FN void fe8_sqn(Fe8& h, const Fe8& f, int n) {
  fe8_sq(h, f);
  for (int i = 1; i < n; ++i) fe8_sq(h, h);
}

__attribute__((target("avx512f,avx512ifma"))) void fe8_invert(Fe8& out, const Fe8& z) {
  Fe8 z2, z9, z11, z_5_0, z_10_0, z_20_0, z_50_0, z_100_0, t;
  fe8_sq(z2, z);
  fe8_sqn(t, z2, 2);
  fe8_mul(z9, t, z);
  fe8_mul(z11, z9, z2);
  fe8_sq(t, z11);
  fe8_mul(z_5_0, t, z9);
  fe8_sqn(t, z_5_0, 5);
  fe8_mul(z_10_0, t, z_5_0);
  fe8_sqn(t, z_10_0, 10);
  fe8_mul(z_20_0, t, z_10_0);
  fe8_sqn(t, z_20_0, 20);
  fe8_mul(t, t, z_20_0);
  fe8_sqn(t, t, 10);
  fe8_mul(z_50_0, t, z_10_0);
  fe8_sqn(t, z_50_0, 50);
  fe8_mul(z_100_0, t, z_50_0);
  fe8_sqn(t, z_100_0, 100);
  fe8_mul(t, t, z_100_0);
  fe8_sqn(t, t, 50);
  fe8_mul(t, t, z_50_0);
  fe8_sqn(t, t, 5);
  fe8_mul(out, t, z11);
}

// out[l] = X25519(scalar, points[l]) for l < 8 (one shared scalar)
__attribute__((target("avx512f,avx512ifma"))) void x25519_x8(uint8_t out[8][32],
                                                             const uint8_t* scalar,
                                                             const uint8_t* const points[8]) {
  uint8_t k[32];
  memcpy(k, scalar, 32);
  k[0] &= 248;
  k[31] &= 127;
  k[31] |= 64;
  alignas(64) uint64_t limbs[5][8];
  for (int l = 0; l < 8; ++l) {
    Fe p;
    fe_load(p, points[l]);
    for (int i = 0; i < 5; ++i) limbs[i][l] = p.v[i];
  }
  Fe8 x1, x2, z2, x3, z3;
  const __m512i zero = _mm512_setzero_si512(), one = _mm512_set1_epi64(1);
  for (int i = 0; i < 5; ++i) {
    x1.v[i] = _mm512_load_si512(limbs[i]);
    x2.v[i] = z3.v[i] = i ? zero : one;
    z2.v[i] = zero;
  }
  x3 = x1;
  uint64_t swap = 0;
  for (int t = 254; t >= 0; --t) {
    const uint64_t kt = (k[t >> 3] >> (t & 7)) & 1;
    swap ^= kt;
    fe8_cswap(x2, x3, swap);
    fe8_cswap(z2, z3, swap);
    swap = kt;
    Fe8 A, AA, B, BB, E, C, D, DA, CB, t0, t1;
    fe8_add(A, x2, z2);
    fe8_sq(AA, A);
    fe8_sub(B, x2, z2);
    fe8_sq(BB, B);
    fe8_sub(E, AA, BB);
    fe8_add(C, x3, z3);
    fe8_sub(D, x3, z3);
    fe8_mul(DA, D, A);
    fe8_mul(CB, C, B);
    fe8_add(t0, DA, CB);
    fe8_sq(x3, t0);
    fe8_sub(t1, DA, CB);
    fe8_sq(t1, t1);
    fe8_mul(z3, x1, t1);
    fe8_mul(x2, AA, BB);
    fe8_mul_small(t0, E, 121665);
    fe8_add(t0, AA, t0);
    fe8_mul(z2, E, t0);
  }
  fe8_cswap(x2, x3, swap);
  fe8_cswap(z2, z3, swap);
  Fe8 r;
  fe8_invert(r, z2);
  fe8_mul(x2, x2, r);
  for (int i = 0; i < 5; ++i) _mm512_store_si512(limbs[i], x2.v[i]);
  for (int l = 0; l < 8; ++l) {
    Fe h;
    for (int i = 0; i < 5; ++i) h.v[i] = limbs[i][l];
    fe_store(out[l], h);
  }
}

bool cpu_has_ifma() {
  static const bool ok = __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512ifma");
  return ok;
}

// the 8-report ladder unless prio3gpu_test_hpke_set_ifma(0) switched it off (no environment read)
std::atomic<int> g_use_ifma{1};

bool have_ifma() { return cpu_has_ifma() && g_use_ifma.load(std::memory_order_relaxed) != 0; }

bool x25519_dh(const uint8_t* sk, const uint8_t* pk, uint8_t* dh) {
  x25519(dh, sk, pk);
  uint8_t acc = 0;  // RFC 9180 §7.1.4: an all-zero X25519 output is an error
  for (int i = 0; i < 32; ++i) acc |= dh[i];
  return acc != 0;
}

bool x25519_public(const uint8_t* sk, uint8_t* pk) {
  static const uint8_t kBase[32] = {9};
  x25519(pk, sk, kBase);
  return true;
}

// P-256: sk is a 32-byte big-endian scalar in [1, n); public keys are uncompressed points (65 B,
// on-curve check in oct2point); the DH output is the x coordinate (32 B).
bool p256_mul(const uint8_t* sk, const uint8_t* pk /* nullptr = generator */, uint8_t* out,
              size_t out_len) {
  const EC_GROUP* g = algs().p256;
  BN_CTX* bc = BN_CTX_new();
  BIGNUM* k = BN_bin2bn(sk, 32, nullptr);
  EC_POINT* P = pk ? EC_POINT_new(g) : nullptr;
  EC_POINT* R = EC_POINT_new(g);
  bool ok = bc && k && R && !BN_is_zero(k) && BN_cmp(k, EC_GROUP_get0_order(g)) < 0;
  if (ok && pk) ok = P && EC_POINT_oct2point(g, P, pk, 65, bc) == 1;
  if (ok) ok = EC_POINT_mul(g, R, pk ? nullptr : k, pk ? P : nullptr, pk ? k : nullptr, bc) == 1;
  if (ok) ok = !EC_POINT_is_at_infinity(g, R);
  if (ok) {
    if (out_len == 65) {
      ok = EC_POINT_point2oct(g, R, POINT_CONVERSION_UNCOMPRESSED, out, 65, bc) == 65;
    } else {
      BIGNUM* x = BN_new();
      ok = x && EC_POINT_get_affine_coordinates(g, R, x, nullptr, bc) == 1 &&
           BN_bn2binpad(x, out, 32) == 32;
      BN_free(x);
    }
  }
  EC_POINT_free(R);
  EC_POINT_free(P);
  BN_clear_free(k);
  BN_CTX_free(bc);
  return ok;
}

bool dh(const Suite& s, const uint8_t* sk, const uint8_t* pk, uint8_t* out) {
  return s.kem == KEM_X25519 ? x25519_dh(sk, pk, out) : p256_mul(sk, pk, out, 32);
}

bool public_of(const Suite& s, const uint8_t* sk, uint8_t* pk) {
  return s.kem == KEM_X25519 ? x25519_public(sk, pk) : p256_mul(sk, nullptr, pk, 65);
}

// ExtractAndExpand(dh, enc || pkRm) with suite_id = "KEM" || I2OSP(kem_id, 2); the KEM's KDF is
// HKDF-SHA256 for both supported KEMs.
bool kem_shared_secret(const Suite& s, const uint8_t* dhv, const uint8_t* enc, const uint8_t* pkR,
                       uint8_t* ss) {
  const EVP_MD* md = algs().md[KDF_SHA256];
  Bytes sid;
  sid.add("KEM").u16(s.kem);
  uint8_t prk[kMaxHash];
  if (!labeled_extract(md, sid, nullptr, 0, "eae_prk", dhv, 32, prk)) return false;
  Bytes ctx;
  ctx.add(enc, s.nenc).add(pkR, s.npk);
  return labeled_expand(md, sid, prk, 32, "shared_secret", ctx.v.data(), ctx.v.size(), s.nsecret,
                        ss);
}

// KeySchedule(mode_base, shared_secret, info, "", "") -> (key, base_nonce)  (§5.1)
bool key_schedule(const Suite& s, const uint8_t* ss, const uint8_t* info, size_t ilen,
                  uint8_t* key, uint8_t* nonce) {
  const EVP_MD* md = algs().md[s.kdf];
  Bytes sid;
  sid.add("HPKE").u16(s.kem).u16(s.kdf).u16(s.aead);
  // psk_id_hash and info_hash depend only on the suite and info, which a batch of opens shares:
  // cached per thread (keyed by suite and info bytes).
  struct Cached {
    uint16_t kem = 0, kdf = 0, aead = 0;
    std::vector<uint8_t> info;
    uint8_t psk_id_hash[kMaxHash], info_hash[kMaxHash];
  };
  thread_local Cached cache;
  if (cache.kem != s.kem || cache.kdf != s.kdf || cache.aead != s.aead ||
      cache.info.size() != ilen || (ilen && memcmp(cache.info.data(), info, ilen) != 0)) {
    cache.kem = 0;
    if (!labeled_extract(md, sid, nullptr, 0, "psk_id_hash", nullptr, 0, cache.psk_id_hash) ||
        !labeled_extract(md, sid, nullptr, 0, "info_hash", info, ilen, cache.info_hash))
      return false;
    cache.info.assign(info, info + ilen);
    cache.kem = s.kem, cache.kdf = s.kdf, cache.aead = s.aead;
  }
  const uint8_t* psk_id_hash = cache.psk_id_hash;
  const uint8_t* info_hash = cache.info_hash;
  uint8_t secret[kMaxHash];
  if (!labeled_extract(md, sid, ss, s.nsecret, "secret", nullptr, 0, secret)) return false;
  Bytes ksc;
  const uint8_t mode = 0;
  ksc.add(&mode, 1).add(psk_id_hash, s.nh).add(info_hash, s.nh);
  return labeled_expand(md, sid, secret, s.nh, "key", ksc.v.data(), ksc.v.size(), s.nk, key) &&
         labeled_expand(md, sid, secret, s.nh, "base_nonce", ksc.v.data(), ksc.v.size(), kNonce,
                        nonce);
}

bool aead(const Suite& s, bool encrypt, const uint8_t* key, const uint8_t* nonce,
          const uint8_t* aad, size_t alen, const uint8_t* in, size_t inlen, uint8_t* out) {
  // encrypt: in = plaintext (inlen), out = ciphertext || tag;  decrypt: in = ct || tag.
  if (!encrypt && inlen < kTag) return false;
  const size_t body = encrypt ? inlen : inlen - kTag;
  if (s.aead == AEAD_AES128GCM || s.aead == AEAD_AES256GCM) {  // low-level GCM128, as for SHA-2
    AES_KEY ks;
    if (AES_set_encrypt_key(key, int(s.nk * 8), &ks) != 0) return false;
    GCM128_CONTEXT* g = CRYPTO_gcm128_new(&ks, reinterpret_cast<block128_f>(AES_encrypt));
    if (!g) return false;
    CRYPTO_gcm128_setiv(g, nonce, kNonce);
    bool ok = !alen || CRYPTO_gcm128_aad(g, aad, alen) == 0;
    if (encrypt) {
      ok = ok && CRYPTO_gcm128_encrypt(g, in, out, body) == 0;
      if (ok) CRYPTO_gcm128_tag(g, out + body, kTag);
    } else {
      ok = ok && CRYPTO_gcm128_decrypt(g, in, out, body) == 0 &&
           CRYPTO_gcm128_finish(g, in + body, kTag) == 0;
    }
    CRYPTO_gcm128_release(g);
    OPENSSL_cleanse(&ks, sizeof ks);
    return ok;
  }
  EVP_CIPHER_CTX* c = EVP_CIPHER_CTX_new();
  int l = 0;
  bool ok = c && EVP_CipherInit_ex2(c, algs().aead[s.aead], key, nonce, encrypt ? 1 : 0,
                                    nullptr) == 1;
  if (ok && alen) ok = EVP_CipherUpdate(c, nullptr, &l, aad, int(alen)) == 1;
  if (ok && body) ok = EVP_CipherUpdate(c, out, &l, in, int(body)) == 1;
  if (ok && !encrypt)
    ok = EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_AEAD_SET_TAG, int(kTag),
                             const_cast<uint8_t*>(in + body)) == 1;
  uint8_t fin[16];
  if (ok) ok = EVP_CipherFinal_ex(c, fin, &l) == 1;
  if (ok && encrypt) ok = EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_AEAD_GET_TAG, int(kTag), out + body) == 1;
  EVP_CIPHER_CTX_free(c);
  return ok;
}

// dh_pre: the DH value already computed for (skR, enc) by the 8-way ladder, or null.
int open_one(const Suite& s, const uint8_t* skR, size_t sk_len, const uint8_t* pkR, size_t pk_len,
             const uint8_t* enc, size_t enc_len, const uint8_t* info, size_t ilen,
             const uint8_t* aad, size_t alen, const uint8_t* ct, size_t ct_len, uint8_t* pt,
             const uint8_t* dh_pre = nullptr) {
  if (sk_len != s.nsk || pk_len != s.npk) return PRIO3GPU_E_ARG;
  if (enc_len != s.nenc || ct_len < kTag) return PRIO3GPU_E_HPKE;
  uint8_t dhv[32], ss[32], key[32], nonce[kNonce];
  bool dh_ok;
  if (dh_pre) {
    uint8_t acc = 0;  // RFC 9180 §7.1.4: an all-zero X25519 output is an error
    for (int i = 0; i < 32; ++i) acc |= dh_pre[i];
    memcpy(dhv, dh_pre, 32);
    dh_ok = acc != 0;
  } else {
    dh_ok = dh(s, skR, enc, dhv);
  }
  if (!dh_ok || !kem_shared_secret(s, dhv, enc, pkR, ss) ||
      !key_schedule(s, ss, info, ilen, key, nonce) ||
      !aead(s, false, key, nonce, aad, alen, ct, ct_len, pt))
    return PRIO3GPU_E_HPKE;
  return 0;
}

// parallel_for over [0, n) on `threads` host threads (chunks of 8 reports).
template <class F>
void parallel_for(size_t n, int threads, F&& f) {
  size_t t = threads > 0 ? size_t(threads) : std::max(1u, std::thread::hardware_concurrency());
  t = std::min(t, (n + 7) / 8);
  if (t <= 1) {
    for (size_t i = 0; i < n; ++i) f(i);
    return;
  }
  std::atomic<size_t> next{0};
  auto work = [&] {
    for (;;) {
      const size_t b = next.fetch_add(8);
      if (b >= n) return;
      for (size_t i = b; i < std::min(n, b + 8); ++i) f(i);
    }
  };
  std::vector<std::thread> pool;
  for (size_t k = 1; k < t; ++k) pool.emplace_back(work);
  work();
  for (auto& th : pool) th.join();
}

}  // namespace

extern "C" {

int prio3gpu_hpke_open(uint16_t kem_id, uint16_t kdf_id, uint16_t aead_id, const uint8_t* sk,
                       size_t sk_len, const uint8_t* pk, size_t pk_len, const uint8_t* enc,
                       size_t enc_len, const uint8_t* info, size_t info_len, const uint8_t* aad,
                       size_t aad_len, const uint8_t* ct, size_t ct_len, uint8_t* pt, size_t cap,
                       size_t* pt_len) {
  Suite s;
  if (!suite_of(kem_id, kdf_id, aead_id, &s)) return PRIO3GPU_E_UNSUPPORTED;
  if (!sk || !pk || !enc || !ct || !pt_len) return PRIO3GPU_E_ARG;
  if (ct_len < kTag) return PRIO3GPU_E_HPKE;
  *pt_len = ct_len - kTag;
  if (!pt || cap < ct_len - kTag) return PRIO3GPU_E_CAPACITY;
  return open_one(s, sk, sk_len, pk, pk_len, enc, enc_len, info, info_len, aad, aad_len, ct,
                  ct_len, pt);
}

int prio3gpu_hpke_seal(uint16_t kem_id, uint16_t kdf_id, uint16_t aead_id, const uint8_t* pk,
                       size_t pk_len, const uint8_t* sk_e, size_t sk_e_len, const uint8_t* info,
                       size_t info_len, const uint8_t* aad, size_t aad_len, const uint8_t* pt,
                       size_t pt_len, uint8_t* enc, size_t enc_cap, size_t* enc_len, uint8_t* ct,
                       size_t ct_cap, size_t* ct_len) {
  Suite s;
  if (!suite_of(kem_id, kdf_id, aead_id, &s)) return PRIO3GPU_E_UNSUPPORTED;
  if (!pk || !enc_len || !ct_len || (pt_len && !pt)) return PRIO3GPU_E_ARG;
  *enc_len = s.nenc;
  *ct_len = pt_len + kTag;
  if (!enc || !ct || enc_cap < s.nenc || ct_cap < pt_len + kTag) return PRIO3GPU_E_CAPACITY;
  if (pk_len != s.npk) return PRIO3GPU_E_ARG;
  uint8_t ske[32];
  if (sk_e) {
    if (sk_e_len != s.nsk) return PRIO3GPU_E_ARG;
    memcpy(ske, sk_e, 32);
  } else {  // fresh ephemeral key (P-256: retry until the scalar is in [1, n))
    for (int tries = 0;; ++tries) {
      if (tries > 64 || RAND_bytes(ske, 32) != 1) return PRIO3GPU_E_HPKE;
      if (s.kem == KEM_X25519 || public_of(s, ske, enc)) break;
    }
  }
  uint8_t dhv[32], ss[32], key[32], nonce[kNonce];
  if (!public_of(s, ske, enc) || !dh(s, ske, pk, dhv) || !kem_shared_secret(s, dhv, enc, pk, ss) ||
      !key_schedule(s, ss, info, info_len, key, nonce) ||
      !aead(s, true, key, nonce, aad, aad_len, pt, pt_len, ct))
    return PRIO3GPU_E_HPKE;
  return 0;
}

int prio3gpu_x25519_batch(const uint8_t* sk, const uint8_t* points, size_t n, uint8_t* out,
                          int simd) {
  if (n && (!sk || !points || !out)) return PRIO3GPU_E_ARG;
  if (simd && !have_ifma()) return PRIO3GPU_E_UNSUPPORTED;
  size_t i = 0;
  if (simd) {
    for (; i < n; i += 8) {
      const uint8_t* pts[8];
      const size_t m = std::min<size_t>(8, n - i);
      for (size_t l = 0; l < 8; ++l) pts[l] = points + 32 * (i + (l < m ? l : 0));
      uint8_t o[8][32];
      x25519_x8(o, sk, pts);
      for (size_t l = 0; l < m; ++l) memcpy(out + 32 * (i + l), o[l], 32);
    }
    return 0;
  }
  for (; i < n; ++i) x25519(out + 32 * i, sk, points + 32 * i);
  return 0;
}

int prio3gpu_hpke_public_key(uint16_t kem_id, const uint8_t* sk, size_t sk_len, uint8_t* pk,
                             size_t cap, size_t* pk_len) {
  Suite s;
  if (!suite_of(kem_id, KDF_SHA256, AEAD_AES128GCM, &s)) return PRIO3GPU_E_UNSUPPORTED;
  if (!sk || !pk_len) return PRIO3GPU_E_ARG;
  *pk_len = s.npk;
  if (!pk || cap < s.npk) return PRIO3GPU_E_CAPACITY;
  if (sk_len != s.nsk) return PRIO3GPU_E_ARG;
  return public_of(s, sk, pk) ? 0 : PRIO3GPU_E_HPKE;
}

int prio3gpu_hpke_open_report_shares(const uint8_t* task_id, const prio3gpu_hpke_keypair* task_keys,
                                     size_t n_task_keys, const prio3gpu_hpke_keypair* global_keys,
                                     size_t n_global_keys, uint8_t sender_role,
                                     uint8_t recipient_role, const uint8_t* msg,
                                     const prio3gpu_prepare_init_view* views, size_t n,
                                     uint8_t* plaintexts, uint64_t* offsets, uint8_t* status,
                                     int threads) {
  if (n == 0) {
    if (offsets) offsets[0] = 0;
    return 0;
  }
  if (!msg || !views || !offsets) return PRIO3GPU_E_ARG;
  offsets[0] = 0;
  for (size_t i = 0; i < n; ++i)
    offsets[i + 1] = offsets[i] + (views[i].payload_len >= kTag ? views[i].payload_len - kTag : 0);
  if (!plaintexts) return 0;  // sizing call
  if (!task_id || !status) return PRIO3GPU_E_ARG;
  if (!algs().ok) return PRIO3GPU_E_UNSUPPORTED;
  static const char kLabel[] = "dap-07 input share";  // Label::InputShare, hpke.rs:52-57
  Bytes info;
  info.add(kLabel).add(&sender_role, 1).add(&recipient_role, 1);
  auto find = [](const prio3gpu_hpke_keypair* ks, size_t nk, uint8_t id) {
    for (size_t k = 0; k < nk; ++k)
      if (ks[k].config_id == id) return &ks[k];
    return static_cast<const prio3gpu_hpke_keypair*>(nullptr);
  };
  // One report: InputShareAad, the first-choice key (with its DH precomputed by the 8-way
  // ladder when dh_pre is set), then the global key after a decryption failure.
  auto open_i = [&](size_t i, const uint8_t* dh_pre) {
    if (status[i]) return;
    const prio3gpu_prepare_init_view& v = views[i];
    const prio3gpu_hpke_keypair* tk = find(task_keys, n_task_keys, v.hpke_config_id);
    const prio3gpu_hpke_keypair* gk = find(global_keys, n_global_keys, v.hpke_config_id);
    if (!tk && !gk) {
      status[i] = 3;  // PrepareError::HpkeUnknownConfigId
      return;
    }
    Bytes aad;  // InputShareAad
    uint8_t tbe[8];
    for (int b = 0; b < 8; ++b) tbe[b] = uint8_t(v.time >> (56 - 8 * b));
    const uint32_t pl = v.public_share_len;
    const uint8_t plbe[4] = {uint8_t(pl >> 24), uint8_t(pl >> 16), uint8_t(pl >> 8), uint8_t(pl)};
    aad.add(task_id, 32).add(msg + v.report_id_off, 16).add(tbe, 8).add(plbe, 4);
    aad.add(msg + v.public_share_off, pl);
    uint8_t* out = plaintexts + offsets[i];
    auto try_open = [&](const prio3gpu_hpke_keypair* kp, const uint8_t* pre) -> int {
      Suite s;
      if (!suite_of(kp->kem_id, kp->kdf_id, kp->aead_id, &s)) return PRIO3GPU_E_UNSUPPORTED;
      return open_one(s, kp->private_key, kp->private_key_len, kp->public_key,
                      kp->public_key_len, msg + v.enc_off, v.enc_len, info.v.data(),
                      info.v.size(), aad.v.data(), aad.v.size(), msg + v.payload_off,
                      v.payload_len, out, pre);
    };
    int rc = try_open(tk ? tk : gk, dh_pre);
    if (rc == PRIO3GPU_E_HPKE && tk && gk) rc = try_open(gk, nullptr);  // second trial
    if (rc != 0) status[i] = 4;  // PrepareError::HpkeDecryptError
  };
  auto primary = [&](size_t i) {
    const uint8_t id = views[i].hpke_config_id;
    const prio3gpu_hpke_keypair* tk = find(task_keys, n_task_keys, id);
    return tk ? tk : find(global_keys, n_global_keys, id);
  };
  const bool simd = have_ifma();
  // Chunks of 8 reports: the X25519 DH of every report whose first-choice key is the chunk's
  // common X25519 key runs in the 8-way ladder; the rest (P-256, mixed keys, the global-key
  // retry) take the scalar path inside open_one.
  parallel_for((n + 7) / 8, threads, [&](size_t ch) {
    const size_t b = ch * 8, e = std::min(n, b + 8);
    uint8_t dh8[8][32];
    bool pre[8] = {};
    if (simd) {
      const prio3gpu_hpke_keypair* kp0 = nullptr;
      const uint8_t* pts[8];
      int lanes = 0;
      for (size_t i = b; i < e; ++i) {
        if (status[i]) continue;
        const prio3gpu_hpke_keypair* kp = primary(i);
        if (!kp || kp->kem_id != KEM_X25519 || kp->private_key_len != 32 || views[i].enc_len != 32)
          continue;
        if (!kp0) kp0 = kp;
        if (kp != kp0) continue;
        pre[i - b] = true;
        pts[lanes++] = msg + views[i].enc_off;
      }
      if (lanes >= 2) {
        for (int l = lanes; l < 8; ++l) pts[l] = pts[0];
        uint8_t out[8][32];
        x25519_x8(out, kp0->private_key, pts);
        int l = 0;
        for (size_t i = b; i < e; ++i)
          if (pre[i - b]) memcpy(dh8[i - b], out[l++], 32);
      } else {
        for (bool& p : pre) p = false;
      }
    }
    for (size_t i = b; i < e; ++i) open_i(i, pre[i - b] ? dh8[i - b] : nullptr);
  });
  return 0;
}

int prio3gpu_test_hpke_set_ifma(int on) {
  if (on && !cpu_has_ifma()) return PRIO3GPU_E_UNSUPPORTED;
  return g_use_ifma.exchange(on ? 1 : 0);
}

}  // extern "C"
