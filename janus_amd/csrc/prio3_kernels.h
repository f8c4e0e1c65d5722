// Batched Prio3 preparation kernels for gfx950 (MI355X).
//
// The reference runs Prio3 one report at a time inside prio 0.15.1 (ext crate) from
//   helper:  aggregator/src/aggregator.rs:1613-1848  (helper_initialized + evaluate, :1775-1797)
//   leader:  aggregator/src/aggregator/aggregation_job_driver.rs:329-402 (:362-380) and
//            :566-686 (leader_continued, :579-593)
//   accumulate: aggregator/src/aggregator/accumulator.rs:76-122
// Here a whole aggregation job (or several) is one batch, processed by these kernels:
//
//   k_query_rand   lane/report  XOF(verify_key, dst5, nonce) -> t                     (1 perm)
//   k_expand       lane/report  helper: XOF(seed, dst1|dst2, [1]) -> meas/proof share (MEAS/10.5 perms)
//   k_jr           lane/report  joint-rand part over the encoded meas share, corrected seed,
//                               joint randomness                                      (MEAS/10.5 perms)
//   k_flp_query_lane  lane/report  FLP query of Count / Sum in registers
//   k_flp_weights  lane/report  ParallelSum types: Lagrange weights at t (one batched inversion),
//                               gadget poly at t, circuit output; k_flp_wires_cols /
//                               k_flp_wires_mfma (wires_mfma.h) / k_flp_wires then stream the
//                               measurement share once for the wire values
//   k_decide       lane/report  sum verifier shares, decide, prep msg (1 perm)
//   k_prepare_next lane/report  prep msg == corrected seed
//   k_accum_*      segmented modular sum of truncated output shares into per-batch aggregates
//   k_merge        aggregate += other aggregate (mod p) after the RCCL all-gather
#pragma once
#include <type_traits>

#include "field.h"
#include "keccak.h"
#include "wide.h"
#include "mont3.h"
#include "mont_fma.h"

namespace p3g {

enum Kind : uint32_t {
  KIND_COUNT = 0,
  KIND_SUM = 1,
  KIND_SUMVEC = 2,
  KIND_HISTOGRAM = 3,
  KIND_FPVEC = 4  // FixedPointBoundedL2VecSum (bits = 16/32/64 per entry, length = entries)
};

// Per-report status codes = DAP PrepareError (messages/src/lib.rs:2288-2298) + 0 = ok.
enum Status : uint8_t { ST_OK = 0, ST_VDAF_PREP_ERROR = 5, ST_INVALID_MESSAGE = 8, ST_SKIPPED = 0xFF };

enum Usage : uint32_t {
  DST_MEASUREMENT_SHARE = 1,
  DST_PROOF_SHARE = 2,
  DST_JOINT_RANDOMNESS = 3,
  DST_PROVE_RANDOMNESS = 4,
  DST_QUERY_RANDOMNESS = 5,
  DST_JOINT_RAND_SEED = 6,
  DST_JOINT_RAND_PART = 7,
};

struct Cfg {
  uint32_t kind, algo_id, es;
  uint32_t meas_len, proof_len, verifier_len, jr_len, out_len, prove_rand_len;
  uint32_t bits, length, chunk, calls, m, logm, arity, gp_len;
  uint32_t leader_share_len, helper_share_len, public_share_len, prep_share_len, prep_msg_len;
  uint32_t qr_len;          // query-randomness elements (one per gadget)
  uint32_t exact_squeeze;   // test switch: every XOF squeeze takes the per-element path
  // engine option wave_prio: FixedPoint chain waves issue at s_setprio 3 and its matrix-core wire
  // passes at 2, over whatever co-runs on their SIMDs (the other aggregator's query, k_fpv_regen)
  uint32_t wave_prio;
  Xof xof;                  // XofShake128 (default) or XofTurboShake128
  const uint8_t* twiddles;  // device: alpha_m^k, k < m, Montgomery form, ES bytes each
  // FixedPointBoundedL2VecSum's second gadget, ParallelSum(PolyEval(norm poly), chunk1)
  uint32_t chunk1, calls1, m1, logm1, gp_len1;
  const uint8_t* twiddles1;  // same table layout as `twiddles`, for m1 / calls1
};

// A per-report byte array: element r at base + r*stride.
struct Rows {
  uint8_t* base;
  size_t stride;
  DEVI uint8_t* at(size_t r) const { return base + r * stride; }
};
struct CRows {
  const uint8_t* base;
  size_t stride;
  DEVI const uint8_t* at(size_t r) const { return base + r * stride; }
};

// FLP weight matrix (k_flp_weights* -> k_flp_wires): element e of report r at base + r rs + e es
// (row-major: rs = row bytes, es = ES).
struct WMat {
  uint8_t* base;
  size_t rs, es;
  DEVI uint8_t* el(size_t r, uint32_t e) const { return base + r * rs + (size_t)e * es; }
};

DEVI uint64_t ld64(const uint8_t* p) { return *reinterpret_cast<const uint64_t*>(p); }
DEVI void st64(uint8_t* p, uint64_t v) { *reinterpret_cast<uint64_t*>(p) = v; }

// ------------------------------------------------------------------------------------------------
// Squeeze n field elements (prio `into_field_vec`: ES-byte LE chunks, reject >= p) from a state
// that has just been permuted after absorbing.  Accepted element i goes to out + i*ES.
// `next(s)` produces the next rate block (keccak_x for the XOF; the test kernel
// k_test_squeeze feeds caller-crafted blocks instead).  `exact` forces the per-element
// rejection-sampling path for every block (PRIO3GPU_EXACT_SQUEEZE=1, a test switch).
// ------------------------------------------------------------------------------------------------
template <class FO>
struct SqueezeVec;

// One permutation per loop iteration (a single inlined Keccak-f per loop: ~35 KB of VOP3 code, so
// two hot copies would not fit the instruction cache).  168-byte blocks alternate parity: even
// blocks hold 10 whole elements + the low half of the next, odd blocks start with its high half.
// Fast path: an element whose high 64 bits are below 2^64 - 28 is canonical (< p), which fails with
// probability 28 / 2^64 per element; when every element of the block passes and all fit, they are
// stored unconditionally at immediate offsets from one address.  Otherwise the block takes the
// exact per-element path (prio's rejection sampling), so the output is the same either way.
DEVI bool hi_ok(uint64_t hi) { return hi < 0xFFFFFFFFFFFFFFE4ull; }

template <>
struct SqueezeVec<Field128Ops> {
  // ESTR: bytes from one output element to the next (16: a report's row).
  // PRE: the state holds the absorbed (unpermuted) message block; every block's permutation,
  // the first included, runs at the top of the one loop (a single Keccak copy per call site).
  template <class Next, uint32_t ESTR = 16, bool PRE = false>
  static DEVI void run(uint64_t s[25], uint32_t n, uint8_t* out, bool exact, Next next) {
    using FO = Field128Ops;
    uint32_t cnt = 0;
    uint32_t parity = 0;
    uint64_t carry = 0;
    while (true) {
      if constexpr (PRE) next(s);
      bool fast = !exact && cnt + 11u <= n;
      if (parity == 0) {
#pragma unroll
        for (int k = 0; k < 10; ++k) fast &= hi_ok(s[2 * k + 1]);
      } else {
        fast &= hi_ok(s[0]);
#pragma unroll
        for (int k = 0; k < 10; ++k) fast &= hi_ok(s[2 * k + 2]);
      }
      if (fast) {
        uint8_t* o = out + (size_t)cnt * ESTR;
        if (parity == 0) {
#pragma unroll
          for (int k = 0; k < 10; ++k)
            *reinterpret_cast<ulonglong2*>(o + k * ESTR) = make_ulonglong2(s[2 * k], s[2 * k + 1]);
          carry = s[20];
          cnt += 10u;
        } else {
          *reinterpret_cast<ulonglong2*>(o) = make_ulonglong2(carry, s[0]);
#pragma unroll
          for (int k = 0; k < 10; ++k)
            *reinterpret_cast<ulonglong2*>(o + (k + 1) * ESTR) =
                make_ulonglong2(s[2 * k + 1], s[2 * k + 2]);
          cnt += 11u;
        }
      } else if (parity == 0) {
#pragma unroll
        for (int k = 0; k < 10; ++k) {
          F128 e = FO::from_u64x2(s[2 * k], s[2 * k + 1]);
          if (cnt < n && FO::is_canonical(e)) {
            FO::store(out + (size_t)cnt * ESTR, e);
            ++cnt;
          }
        }
        carry = s[20];
      } else {
        {
          F128 e = FO::from_u64x2(carry, s[0]);
          if (cnt < n && FO::is_canonical(e)) {
            FO::store(out + (size_t)cnt * ESTR, e);
            ++cnt;
          }
        }
#pragma unroll
        for (int k = 0; k < 10; ++k) {
          F128 e = FO::from_u64x2(s[2 * k + 1], s[2 * k + 2]);
          if (cnt < n && FO::is_canonical(e)) {
            FO::store(out + (size_t)cnt * ESTR, e);
            ++cnt;
          }
        }
      }
      if (cnt >= n) break;
      parity ^= 1u;
      if constexpr (!PRE) next(s);
    }
  }
};

// Field64: 21 whole elements per block, always the per-element path.
template <>
struct SqueezeVec<Field64Ops> {
  template <class Next, uint32_t ESTR = 8, bool PRE = false>
  static DEVI void run(uint64_t s[25], uint32_t n, uint8_t* out, bool /*exact*/, Next next) {
    using FO = Field64Ops;
    uint32_t cnt = 0;
    while (true) {
      if constexpr (PRE) next(s);
#pragma unroll
      for (int k = 0; k < 21; ++k) {
        if (cnt < n && s[k] < FO::P) {
          st64(out + (size_t)cnt * 8, s[k]);
          ++cnt;
        }
      }
      if (cnt >= n) break;
      if constexpr (!PRE) next(s);
    }
  }
};

struct KeccakNext {
  Xof x;
  DEVI void operator()(uint64_t s[25]) const { keccak_x(s, x); }
};

template <class FO, uint32_t ESTR = FO::ES>
DEVI void squeeze_vec(uint64_t s[25], uint32_t n, uint8_t* out, const Xof& x, bool exact = false) {
  if constexpr (ESTR == FO::ES)
    SqueezeVec<FO>::run(s, n, out, exact, KeccakNext{x});
  else
    SqueezeVec<FO>::template run<KeccakNext, ESTR>(s, n, out, exact, KeccakNext{x});
}

// XOF(seed, dst(usage), binder=[byte]) expanded into n elements (helper share expansion).
template <class FO, uint32_t ESTR = FO::ES>
DEVI void xof_expand_byte_binder(uint32_t algo_id, uint32_t usage, uint64_t seed_lo,
                                 uint64_t seed_hi, uint32_t binder_byte, uint32_t n,
                                 uint8_t* out, const Xof& x, bool exact) {
  MsgBlock m;
  m.clear();
  m.header(algo_id, usage, seed_lo, seed_hi);
  m.put8(25, binder_byte);
  m.pad(26, x);
  uint64_t s[25];
  sponge_one_block(s, m, x);
  squeeze_vec<FO, ESTR>(s, n, out, x, exact);
}

// derive_seed(0^16, dst6, part0 || part1)   (prio Prio3::derive_joint_rand_seed)
DEVI void derive_jr_seed(const Xof& x, uint32_t algo_id, uint64_t p0lo, uint64_t p0hi,
                         uint64_t p1lo, uint64_t p1hi, uint64_t& olo, uint64_t& ohi) {
  MsgBlock m;
  m.clear();
  m.header(algo_id, DST_JOINT_RAND_SEED, 0ull, 0ull);
  m.put64(25, p0lo);
  m.put64(33, p0hi);
  m.put64(41, p1lo);
  m.put64(49, p1hi);
  m.pad(57, x);
  uint64_t s[25];
  sponge_one_block(s, m, x);
  olo = s[0];
  ohi = s[1];
}

// ------------------------------------------------------------------------------------------------
// Joint-randomness part (prio prepare_init / shard):
//   derive_seed(blind, dst7, [agg_id] || nonce || encode(meas_share))
// Message = 42-byte prefix || data (nbytes, multiple of 8) || SHAKE padding.  Stream word g >= 5 is
// (D[g-6] >> 48) | (D[g-5] << 16) with D[-1] = the top 16 bits of the nonce's high word.
// ------------------------------------------------------------------------------------------------
// Words 21b .. 21b+20 of block b (b >= 0; words < 5 of block 0 are the caller's prefix), cut from
// the 22 data words D[21b-6 .. 21b+15]: loaded in two batches of 11 from clamped addresses (one
// wait per batch instead of a load-use wait per word), selected, funnel-shifted and handed to
// emit(w, word) as soon as formed, so at most one batch is live (k_jr stays within 168 VGPRs).
template <class Emit>
DEVI void jr_block_words(int64_t b, const uint8_t* data, int64_t nd, uint64_t nonce_hi,
                         Emit&& emit) {
  const int64_t j0 = 21 * b - 6;
  auto ld = [&](int k) {
    const int64_t j = j0 + k;
    return ld64(data + 8 * (j < 0 ? 0 : (j < nd ? j : nd - 1)));
  };
  auto fix = [&](int k, uint64_t d) {
    const int64_t j = j0 + k;
    return (j >= 0 && j < nd) ? d : (j == -1 ? nonce_hi : 0ull);
  };
  uint64_t D[11];
#pragma unroll
  for (int k = 0; k < 11; ++k) D[k] = ld(k);
#pragma unroll
  for (int w = 0; w < 10; ++w) emit(w, (fix(w, D[w]) >> 48) | (fix(w + 1, D[w + 1]) << 16));
  const uint64_t d10 = fix(10, D[10]);
  asm volatile("" ::: "memory");  // the second batch is not hoisted above the first one's use
#pragma unroll
  for (int k = 0; k < 11; ++k) D[k] = ld(11 + k);
  emit(10, (d10 >> 48) | (fix(11, D[0]) << 16));
#pragma unroll
  for (int w = 11; w < 21; ++w)
    emit(w, (fix(w, D[w - 11]) >> 48) | (fix(w + 1, D[w - 10]) << 16));
}

DEVI void jr_part(const Xof& x, uint32_t algo_id, uint32_t agg_id, uint64_t blind_lo, uint64_t blind_hi,
                  uint64_t nonce_lo, uint64_t nonce_hi, const uint8_t* data, uint32_t nbytes,
                  uint64_t& olo, uint64_t& ohi) {
  MsgBlock pre;
  pre.clear();
  pre.header(algo_id, DST_JOINT_RAND_PART, blind_lo, blind_hi);
  pre.put8(25, agg_id);
  pre.put64(26, nonce_lo);
  pre.put64(34, nonce_hi);
  // bytes 40,41 (top of nonce_hi) live in word 5 together with data; words 0..4 are pure prefix
  const int64_t nd = nbytes / 8;
  const int64_t total = 42 + (int64_t)nbytes;   // message bytes before padding
  const int64_t nblocks = total / 168 + 1;
  const int64_t padw = total >> 3;              // word holding the 0x1F pad byte
  const uint64_t padv = (uint64_t)x.pad << ((total & 7) * 8);
  uint64_t s[25];
#pragma unroll
  for (int i = 0; i < 25; ++i) s[i] = 0ull;
  // One permutation per iteration (single inlined Keccak-f, see squeeze_vec).  Block 0 carries the
  // 42-byte prefix; "fast" blocks are pure data (the common case); the last block(s) are padded.
  for (int64_t b = 0; b < nblocks; ++b) {
    const bool fast = (b >= 1) && (21 * b + 15 < nd) && (21 * b + 20 < padw);
    if (fast) {
      const uint64_t* D = reinterpret_cast<const uint64_t*>(data) + (21 * b - 6);
      uint64_t prev = D[0];
#pragma unroll
      for (int w = 0; w < 21; ++w) {
        const uint64_t cur = D[w + 1];
        s[w] ^= (prev >> 48) | (cur << 16);
        prev = cur;
      }
    } else if (b == 0) {
#pragma unroll
      for (int w = 0; w < 5; ++w) s[w] ^= (padw == w) ? pre.w[w] ^ padv : pre.w[w];
      asm volatile("" ::: "memory");  // the prefix is absorbed before the data words load
      jr_block_words(0, data, nd, nonce_hi, [&](int w, uint64_t v) {
        if (w < 5) return;
        if (padw == w) v ^= padv;
        if (nblocks == 1 && w == 20) v ^= 0x8000000000000000ull;
        s[w] ^= v;
      });
    } else {
      jr_block_words(b, data, nd, nonce_hi, [&](int w, uint64_t v) {
        const int64_t g = 21 * b + w;
        if (padw == g) v ^= padv;
        if (b == nblocks - 1 && w == 20) v ^= 0x8000000000000000ull;
        s[w] ^= v;
      });
    }
    keccak_x(s, x);
  }
  olo = s[0];
  ohi = s[1];
}

// ================================================================================================
// Kernels
// ================================================================================================

// t = XOF(verify_key, dst5, nonce).next_vec(1)    (prio prepare_init, query randomness)
template <class FO>
__global__ void __launch_bounds__(256) k_query_rand(Cfg cfg, uint32_t n, uint64_t vk_lo,
                                                    uint64_t vk_hi, CRows nonces, Rows out_t,
                                                    const uint8_t* status) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  if (status && status[r] != ST_OK) return;
  const uint8_t* nz = nonces.at(r);
  MsgBlock m;
  m.clear();
  m.header(cfg.algo_id, DST_QUERY_RANDOMNESS, vk_lo, vk_hi);
  m.put64(25, ld64(nz));
  m.put64(33, ld64(nz + 8));
  m.pad(41, cfg.xof);
  uint64_t s[25];
  sponge_one_block(s, m, cfg.xof);
  squeeze_vec<FO>(s, cfg.qr_len, out_t.at(r), cfg.xof, cfg.exact_squeeze);
}

// Helper share expansion: meas share XOF(k_meas, dst1, [agg_id]) and proof share
// XOF(k_proof, dst2, [agg_id]) (prio prepare_init, Share::Helper arms).
template <class FO>
#ifndef P3G_EXPAND_WAVES  // min waves per SIMD for k_expand (A/B knob; 0 = compiler's choice)
#define P3G_EXPAND_WAVES 0
#endif
__global__ void __launch_bounds__(256, P3G_EXPAND_WAVES) k_expand(Cfg cfg, uint32_t n, uint32_t agg_id,
                                                CRows helper_shares, Rows out_meas,
                                                Rows out_proof, const uint8_t* status) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  if (status && status[r] != ST_OK) return;
  const uint8_t* hs = helper_shares.at(r);
#ifndef P3G_EXPAND_ONECOPY
#define P3G_EXPAND_ONECOPY 1
#endif
#if P3G_EXPAND_ONECOPY
  // proof share, then measurement share, through ONE loop body: the absorb permutation runs inside
  // the squeeze loop (PRE), so the kernel holds one copy of the unrolled permutation, not four
  uint32_t ph = 0;
  asm volatile("" : "+s"(ph));  // opaque trip count: the phase loop is not unrolled
  for (; ph < 2u; ++ph) {
    const bool pf = ph == 0u;
    MsgBlock m;
    m.clear();
    m.header(cfg.algo_id, pf ? DST_PROOF_SHARE : DST_MEASUREMENT_SHARE, ld64(hs + (pf ? 16 : 0)),
             ld64(hs + (pf ? 24 : 8)));
    m.put8(25, agg_id);
    m.pad(26, cfg.xof);
    uint64_t s[25];
#pragma unroll
    for (int i = 0; i < 25; ++i) s[i] = i < kRateWords ? m.w[i] : 0ull;
    SqueezeVec<FO>::template run<KeccakNext, FO::ES, true>(
        s, pf ? cfg.proof_len : cfg.meas_len, pf ? out_proof.at(r) : out_meas.at(r),
        cfg.exact_squeeze, KeccakNext{cfg.xof});
  }
  return;
#endif
  xof_expand_byte_binder<FO>(cfg.algo_id, DST_PROOF_SHARE, ld64(hs + 16), ld64(hs + 24), agg_id,
                             cfg.proof_len, out_proof.at(r), cfg.xof, cfg.exact_squeeze);
  xof_expand_byte_binder<FO>(cfg.algo_id, DST_MEASUREMENT_SHARE, ld64(hs), ld64(hs + 8), agg_id,
                             cfg.meas_len, out_meas.at(r), cfg.xof, cfg.exact_squeeze);
}

// Joint randomness (prio prepare_init): own part over the encoded meas share, corrected seed
// (public-share parts with this aggregator's part replaced), joint_rand = XOF(seed, dst3, "").
//
// The meas share is streamed through LDS: each wave owns a 64 x 176-byte window (one 168-byte
// rate block of every lane's report plus the preceding word), filled for block b+1 by 11 LDS-DMA
// instructions (global_load_lds_dwordx4, 16 B/lane, ~6 rows per instruction instead of 64) while
// block b is permuted.  All lanes of a wave take part in the fill, so lanes past n or with a
// failed status still run the loop (on a clamped row) and just do not store.
// lo:hi += x (64-bit), cy += carry out.  s_nop 1: gfx950 wants two wait states between a VALU
// that writes VCC and a VALU that reads it as carry-in (hipcc pads its own chains the same way).
DEVI void acc_u64(uint32_t& lo, uint32_t& hi, uint32_t& cy, uint64_t x) {
  asm("v_add_co_u32 %0, vcc, %0, %3\n\t"
      "s_nop 1\n\t"
      "v_addc_co_u32 %1, vcc, %1, %4, vcc\n\t"
      "s_nop 1\n\t"
      "v_addc_co_u32 %2, vcc, 0, %2, vcc"
      : "+v"(lo), "+v"(hi), "+v"(cy)
      : "v"((uint32_t)x), "v"((uint32_t)(x >> 32))
      : "vcc");
}

// Buffer resource word 3 for raw (stride 0) buffer loads on gfx9-family parts (gfx950):
// DATA_FORMAT = 32, everything else 0.
constexpr int kBufRsrcWord3 = 0x00020000;

constexpr uint32_t kJrWin = 176;  // bytes per report in the LDS window (22 words)
constexpr uint32_t kJrWaveLds = 64 * kJrWin;

template <class FO>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) k_jr(Cfg cfg, uint32_t n, uint32_t agg_id, CRows nonces,
                                            CRows public_shares, CRows blinds, CRows meas,
                                            Rows out_part, Rows out_seed, Rows out_jr,
                                            const uint8_t* status, uint64_t* spec_lo,
                                            uint8_t* spec_cy) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t tid = threadIdx.x, lane = tid & 63u;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave in block (uniform)
  const uint32_t r0w = blockIdx.x * blockDim.x + 64u * wv;       // first report of this wave
  if (r0w >= n) return;                                          // wave-uniform
  const uint32_t r = r0w + lane;
  const bool live = r < n && (!status || status[r] == ST_OK);
  const uint32_t rr = r < n ? r : n - 1u;
  uint8_t* win = smem + wv * kJrWaveLds;

  const uint8_t* data = meas.at(rr);
  const uint32_t nbytes = cfg.meas_len * cfg.es;
  const int64_t nd = nbytes / 8;
  const int64_t total = 42 + (int64_t)nbytes;
  const int64_t nblocks = total / 168 + 1;
  const int64_t padw = total >> 3;
  const uint64_t padv = (uint64_t)cfg.xof.pad << ((total & 7) * 8);

  // LDS-DMA piece q of this lane: flat piece P = 64q + lane = (row, k) with 11 pieces per row,
  // lane = 11 la + lb:  row = la + cq + wrap, k = lb + dq - 11 wrap, wrap = (lb + dq >= 11),
  // where 64q = 11 cq + dq.  A full wave (64 live rows) reads piece q at the per-lane offset
  //   la mstride + 16 lb  +  (cq mstride + 16 dq)  +  wrap (mstride - 176)
  // = one loop-invariant VGPR + a scalar + a select: buffer_load ... lds with the window's source
  // as the (scalar) buffer base, 2 VALU per piece (the general form, kept for the last partial
  // wave whose rows clamp at rlim, spends ~14 incl. a quarter-rate v_mul_lo_u32 and two 64-bit
  // adds).  k_jr must stay <= 168 VGPRs (3 waves per SIMD).
  const uint32_t la0 = lane / 11u, lb0 = lane - 11u * la0;
  const uint32_t rlim = (n - r0w < 64u ? n - r0w : 64u) - 1u;  // last valid row of the wave
  const bool full_wave = rlim == 63u;                             // wave-uniform
  const uint32_t mstride = (uint32_t)meas.stride;
  const uint8_t* wbase = meas.base + (size_t)r0w * meas.stride;
  const uint32_t lofs = la0 * mstride + 16u * lb0;
  const uint32_t wdelta = mstride - 176u;
  auto is_fast = [&](int64_t b) { return (b >= 1) && (21 * b + 15 < nd) && (21 * b + 20 < padw); };
  // one LDS-DMA piece q (1 KB: 64 lanes x 16 B) of the window of block b, any wave
  auto stage_piece = [&](int64_t b, int q) {
    const uint8_t* src = wbase + 8 * (21 * b - 6);
    // opaque copies: keep LICM from hoisting the 11 per-lane offsets out of the loop
    uint32_t la, lb;
    asm volatile("v_mov_b32 %0, %1" : "=v"(la) : "v"(la0));
    asm volatile("v_mov_b32 %0, %1" : "=v"(lb) : "v"(lb0));
    const uint32_t cq = (64u * q) / 11u, dq = (64u * q) % 11u;  // 64q = 11 cq + dq
    const uint32_t t = lb + dq;
    const uint32_t wrap = t >= 11u ? 1u : 0u;
    const uint32_t row = min(la + cq + wrap, rlim);
    const uint32_t k = t - 11u * wrap;
    __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(src + (row * mstride + 16u * k)),
          (__attribute__((address_space(3))) void*)(win + 1024 * q), 16, 0, 0);
  };
  auto stage_full = [&](int64_t b) {  // a full wave: scalar base + 2 VALU per piece
    const uint8_t* src = wbase + 8 * (21 * b - 6);
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, 64u * mstride, kBufRsrcWord3);
    uint32_t lo, lb;
    asm volatile("v_mov_b32 %0, %1" : "=v"(lo) : "v"(lofs));
    asm volatile("v_mov_b32 %0, %1" : "=v"(lb) : "v"(lb0));
#pragma unroll
    for (int q = 0; q < 11; ++q) {
      const uint32_t cq = (64u * q) / 11u, dq = (64u * q) % 11u;
      const uint32_t vo = lo + (lb + dq >= 11u ? wdelta : 0u);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rs, (__attribute__((address_space(3))) void*)(win + 1024 * q), 16, vo,
            cq * mstride + 16u * dq, 0, 0);
    }
  };
  auto stage = [&](int64_t b) {  // window <- words [21b-6, 21b+16) of every row of the wave
    if (full_wave) {
      stage_full(b);
    } else {
#pragma unroll
      for (int q = 0; q < 11; ++q) stage_piece(b, q);
    }
  };


  uint64_t s[25];
#pragma unroll
  for (int i = 0; i < 25; ++i) s[i] = 0ull;
  for (int64_t b = 0; b < nblocks; ++b) {
    if (is_fast(b)) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      // the lane index re-read per block (2 VALU): nothing lane-derived stays live across the
      // permutation, so the window and column-sum addresses need no spill slots
      uint32_t ln;
      asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
      const uint64_t* L = reinterpret_cast<const uint64_t*>(win + ln * kJrWin);
      uint64_t prev = L[0];
#pragma unroll
      for (int w = 0; w < 21; ++w) {
        const uint64_t cur = L[w + 1];
        s[w] ^= (prev >> 48) | (cur << 16);
        prev = cur;
      }
      if (spec_lo != nullptr) {
        // Speculative accumulation: column sums of the window's 21 new words over the wave's 64
        // rows (lane = word wc + 21 gq, rows gq, gq+3, ...; lane 63's sums are never used), as a
        // 64-bit sum plus carry count.  All reads of a half are issued before the adds.
        const uint32_t gq = ln / 21u, wc = ln - 21u * gq;
        // rows gq + 3i: one base address, the row steps are immediate offsets of ds_read_b64
        const uint8_t* colp = win + 8u * (1u + wc) + gq * kJrWin;
        uint32_t l32 = 0, h32 = 0, cy = 0;
#pragma unroll
        for (int i0 = 0; i0 < 22; i0 += 11) {
          uint64_t xs[11];
#pragma unroll
          for (int i = 0; i < 11; ++i) {
            const int ii = i0 + i;
            if (ii < 21) {
              xs[i] = *reinterpret_cast<const uint64_t*>(colp + 3u * (uint32_t)ii * kJrWin);
            } else {  // row 63 exists only for gq == 0
              xs[i] = *reinterpret_cast<const uint64_t*>(win + 8u * (1u + wc) + 63u * kJrWin);
              if (gq != 0u) xs[i] = 0ull;
            }
          }
#pragma unroll
          for (int i = 0; i < 11; ++i) acc_u64(l32, h32, cy, xs[i]);
        }
        // partial sums of lanes ln + 21 and ln + 42 (byte addresses for ds_bpermute)
        const int s1 = (int)(((ln + 21u) & 63u) << 2), s2 = (int)(((ln + 42u) & 63u) << 2);
        const uint32_t la = (uint32_t)__builtin_amdgcn_ds_bpermute(s1, (int)l32);
        const uint32_t ha = (uint32_t)__builtin_amdgcn_ds_bpermute(s1, (int)h32);
        const uint32_t ca = (uint32_t)__builtin_amdgcn_ds_bpermute(s1, (int)cy);
        const uint32_t lb = (uint32_t)__builtin_amdgcn_ds_bpermute(s2, (int)l32);
        const uint32_t hb = (uint32_t)__builtin_amdgcn_ds_bpermute(s2, (int)h32);
        const uint32_t cb = (uint32_t)__builtin_amdgcn_ds_bpermute(s2, (int)cy);
        if (ln < 21u) {
          acc_u64(l32, h32, cy, ((uint64_t)ha << 32) | la);
          acc_u64(l32, h32, cy, ((uint64_t)hb << 32) | lb);
          // buffer stores: the wave's row (scalar base) + a 32-bit per-lane offset
          const size_t wrow = (size_t)(r0w >> 6) * (size_t)nd;
          const uint32_t at = (uint32_t)(21 * b - 5) + ln;
          const __amdgpu_buffer_rsrc_t rlo = __builtin_amdgcn_make_buffer_rsrc(
              (void*)(spec_lo + wrow), (short)0, (uint32_t)(8 * nd), kBufRsrcWord3);
          const __amdgpu_buffer_rsrc_t rcy = __builtin_amdgcn_make_buffer_rsrc(
              (void*)(spec_cy + wrow), (short)0, (uint32_t)nd, kBufRsrcWord3);
          typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
          __builtin_amdgcn_raw_buffer_store_b64(u32x2{l32, h32}, rlo, 8u * at, 0, 0);
          __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(cy + ca + cb), rcy, at, 0, 0);
        }
      }
    } else if (b == 0) {
      // prefix [agg_id] || nonce, built here so none of it stays live across the loop
      const uint8_t* nz = nonces.at(rr);
      const uint8_t* bl = blinds.at(rr);
      const uint64_t nonce_hi = ld64(nz + 8);
      MsgBlock pre;
      pre.clear();
      pre.header(cfg.algo_id, DST_JOINT_RAND_PART, ld64(bl), ld64(bl + 8));
      pre.put8(25, agg_id);
      pre.put64(26, ld64(nz));
      pre.put64(34, nonce_hi);
#pragma unroll
      for (int w = 0; w < 5; ++w) s[w] ^= (padw == w) ? pre.w[w] ^ padv : pre.w[w];
      asm volatile("" ::: "memory");  // the prefix is absorbed before the data words load
      jr_block_words(0, data, nd, nonce_hi, [&](int w, uint64_t v) {
        if (w < 5) return;
        if (padw == w) v ^= padv;
        if (nblocks == 1 && w == 20) v ^= 0x8000000000000000ull;
        s[w] ^= v;
      });
    } else {
      jr_block_words(b, data, nd, 0ull, [&](int w, uint64_t v) {  // b >= 1: no nonce word
        const int64_t g = 21 * b + w;
        if (padw == g) v ^= padv;
        if (b == nblocks - 1 && w == 20) v ^= 0x8000000000000000ull;
        s[w] ^= v;
      });
    }
    if (is_fast(b + 1)) {  // refill the window (its reads above have completed) under the permutation
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      stage(b + 1);
    }
    keccak_x(s, cfg.xof);
  }
  if (!live) return;
  const uint64_t plo = s[0], phi = s[1];
  st64(out_part.at(r), plo);
  st64(out_part.at(r) + 8, phi);
  const uint8_t* ps = public_shares.at(r);
  uint64_t p0lo = ld64(ps), p0hi = ld64(ps + 8), p1lo = ld64(ps + 16), p1hi = ld64(ps + 24);
  if (agg_id == 0) {
    p0lo = plo;
    p0hi = phi;
  } else {
    p1lo = plo;
    p1hi = phi;
  }
  uint64_t slo, shi;
  derive_jr_seed(cfg.xof, cfg.algo_id, p0lo, p0hi, p1lo, p1hi, slo, shi);
  st64(out_seed.at(r), slo);
  st64(out_seed.at(r) + 8, shi);
  MsgBlock m;
  m.clear();
  m.header(cfg.algo_id, DST_JOINT_RANDOMNESS, slo, shi);
  m.pad(25, cfg.xof);
  uint64_t s2[25];
  sponge_one_block(s2, m, cfg.xof);
  squeeze_vec<FO>(s2, cfg.jr_len, out_jr.at(r), cfg.xof, cfg.exact_squeeze);
}

// ------------------------------------------------------------------------------------------------
// LDS helpers
// ------------------------------------------------------------------------------------------------
DEVI uint32_t bitrev(uint32_t x, uint32_t logn) {
  return logn == 0 ? 0u : (__builtin_bitreverse32(x) >> (32 - logn));
}

template <class FO>
DEVI typename FO::T ld_tw(const Cfg& cfg, uint32_t i) {
  // through the constant address space: a wave-uniform index becomes a scalar load (s_load_dwordx4),
  // so no vector-memory wait (vmcnt) is spent on the tables -- one would also wait for the LDS-DMA
  // fills in flight
  using CP = const __attribute__((address_space(4))) uint32_t*;
  const CP p = (CP)(cfg.twiddles + (size_t)i * FO::ES);
  typename FO::T v;
#pragma unroll
  for (int k = 0; k < FO::ES / 4; ++k) v.w[k] = p[k];
  return v;
}

// 16-byte LDS store the compiler's wait-count pass does not see (see k_flp_weights' put); the
// caller orders it against LDS-DMA fills and reads of the same bytes with explicit s_waitcnt
DEVI void lds_store16(uint8_t* p, const F128& v) {
  typedef uint32_t v4u __attribute__((ext_vector_type(4)));
  const v4u d = {v.w[0], v.w[1], v.w[2], v.w[3]};
  const uint32_t a = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)p;
  asm volatile("ds_write_b128 %0, %1" : : "v"(a), "v"(d) : "memory");
}

// Two in-place radix-2 DIT NTTs of size m (inputs already bit-reversed) over LDS arrays A and B,
// twiddles in Montgomery form:  X[k] = sum_i x[i] alpha_m^(ik).
template <class FO>
DEVI void ntt2_lds(const Cfg& cfg, typename FO::T* A, typename FO::T* B, uint32_t tid,
                   uint32_t nthr) {
  const uint32_t m = cfg.m, logm = cfg.logm;
  for (uint32_t st = 1; st <= logm; ++st) {
    const uint32_t half = 1u << (st - 1);
    for (uint32_t q = tid; q < m; q += nthr) {  // q < m/2: array A, else array B
      typename FO::T* a = q < (m >> 1) ? A : B;
      const uint32_t bq = q & ((m >> 1) - 1u);
      const uint32_t grp = bq >> (st - 1), k = bq & (half - 1u);
      const uint32_t i = grp * 2u * half + k, j = i + half;
      const typename FO::T w = ld_tw<FO>(cfg, k << (logm - st));
      const typename FO::T u = a[i];
      const typename FO::T v = FO::mul(w, a[j]);
      a[i] = FO::add(u, v);
      a[j] = FO::sub(u, v);
    }
    __syncthreads();
  }
}

// Block-wide modular sum of one value per thread (all threads call; result valid in all threads).
template <class FO>
DEVI typename FO::T block_sum(typename FO::T x, typename FO::T* red, uint32_t tid, uint32_t nthr) {
  red[tid] = x;
  __syncthreads();
  for (uint32_t s = 1; s < nthr; s <<= 1) {
    typename FO::T y = FO::zero();
    const bool act = (tid % (2 * s) == 0) && (tid + s < nthr);
    if (act) y = FO::add(red[tid], red[tid + s]);
    __syncthreads();
    if (act) red[tid] = y;
    __syncthreads();
  }
  typename FO::T out = red[0];
  __syncthreads();
  return out;
}

// ------------------------------------------------------------------------------------------------
// FLP query (prio src/flp.rs Type::query with QueryShimGadget), one block per report.
//
// For every wire i:  wire_i(t) = sum_{k=0}^{calls} L_k(t) f_{i,k},  f_{i,0} = proof seed,
//   L_k(t) = alpha^k (t^m - 1) / (m (t - alpha^k)) = (alpha^k/m) * NTT_m(t^(m-1-i))[k]
// which equals prio's iDFT + Horner evaluation bit for bit (same polynomial).  The gadget outputs
// p(alpha^k) come from one size-m NTT of the gadget poly folded mod x^m - 1.
//
// ParallelSum(Mul, c) types (SumVec, Histogram), column j, row k, idx = (k-1)c + j:
//   f_{2j,k}   = r^(idx+1) x_idx  (0 if padded)    -> wire_2j   = L0 s_2j   + r^(j+1) sum_k (L_k r^(c(k-1))) x
//   f_{2j+1,k} = x_idx - 1/2      (-1/2 if padded) -> wire_2j+1 = L0 s_2j+1 + sum_k L_k x - 1/2 sum_k L_k
// LDS layout (dynamic):  TP[2m] | NA[m] | NB[m] | LM[m] | MM[m] | RP[c+1] | PA[H*c] | PB[H*c] | RED[nthr] | flag
// ------------------------------------------------------------------------------------------------
// Wave-level inclusive product scan (6 shuffle steps): lane l returns base^(l+1).
template <class FO>
DEVI typename FO::T wave_pow_scan(typename FO::T base, uint32_t lane) {
  typename FO::T v = base;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    typename FO::T y;
#pragma unroll
    for (int w = 0; w < FO::NW; ++w) y.w[w] = __shfl_up(v.w[w], off, 64);
    if (lane >= (uint32_t)off) v = FO::mul(v, y);
  }
  return v;
}

// tab[i] = base^i (Montgomery) for i < n (n <= 4096), built by ONE wave with two product scans:
// base^1..base^64 by lanes, giant steps (base^64)^q by lanes, then tab[64q + l] = base^(64q) base^l.
// No barriers inside (the caller synchronises).
template <class FO>
DEVI void wave_pow_table(typename FO::T* tab, typename FO::T base, uint32_t n, uint32_t lane) {
  using T = typename FO::T;
  const T v = wave_pow_scan<FO>(base, lane);  // base^(lane+1)
  if (lane == 0) tab[0] = FO::one_mont();
  if (lane + 1 < n) tab[lane + 1] = v;
  const uint32_t nq = (n + 63) >> 6;
  if (nq > 1) {
    T b64, bl;
#pragma unroll
    for (int w = 0; w < FO::NW; ++w) {
      b64.w[w] = __shfl(v.w[w], 63, 64);
      bl.w[w] = __shfl(v.w[w], (int)((lane + 63) & 63), 64);  // base^lane (lane 0: fixed below)
    }
    if (lane == 0) bl = FO::one_mont();
    const T g = wave_pow_scan<FO>(b64, lane);  // base^(64 (lane+1))
    for (uint32_t q = 1; q < nq; ++q) {
      T gq;
#pragma unroll
      for (int w = 0; w < FO::NW; ++w) gq.w[w] = __shfl(g.w[w], (int)(q - 1), 64);
      const uint32_t i = 64 * q + lane;
      if (i < n && lane != 0) tab[i] = FO::mul(gq, bl);
      if (i < n && lane == 0) tab[i] = gq;
    }
  }
}

// Block-wide modular sums of three values per thread (wave shuffles, then across waves in LDS).
template <class FO>
DEVI void block_sum3(typename FO::T& a, typename FO::T& b, typename FO::T& c, typename FO::T* red,
                     uint32_t tid, uint32_t nthr) {
  using T = typename FO::T;
  T v[3] = {a, b, c};
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      T o;
#pragma unroll
      for (int w = 0; w < FO::NW; ++w) o.w[w] = __shfl_xor(v[q].w[w], off, 64);
      v[q] = FO::add(v[q], o);
    }
  }
  const uint32_t wave = tid >> 6, nw = (nthr + 63) >> 6;
  if ((tid & 63) == 0) {
    red[3 * wave + 0] = v[0];
    red[3 * wave + 1] = v[1];
    red[3 * wave + 2] = v[2];
  }
  __syncthreads();
  T r0 = red[0], r1 = red[1], r2 = red[2];
  for (uint32_t w = 1; w < nw; ++w) {
    r0 = FO::add(r0, red[3 * w + 0]);
    r1 = FO::add(r1, red[3 * w + 1]);
    r2 = FO::add(r2, red[3 * w + 2]);
  }
  __syncthreads();
  a = r0;
  b = r1;
  c = r2;
}

struct FlpDims {
  uint32_t H;       // row groups in the main loop
  uint32_t cols;    // columns (chunk) for ParallelSum, 1 for Sum, 1 for Count
  uint32_t rp_len;  // entries of the r-power table RP
};

// W row written by k_flp_weights (ParallelSum types) and read by the wire passes (Montgomery form):
//   MM[k] = L_k r^(c(k-1)) | LM[k] = L_k (k = 1..calls) | RP[j] = r^(j+1) (j < c) |
//   L0 | HL = (1/2) sum_(k>=1) L_k | gsum (circuit output before the range/sum mix) |
//   SMM = sum_k MM[k] | SLM = sum_k LM[k]   (mod p: k_flp_wires_mfma's offset correction)
// The wire passes finish  wire_2j = L0 s_2j + RP[j] a_j,  wire_2j+1 = L0 s_2j+1 - HL + b_j  from the
// proof share's wire seeds s themselves (and check them canonical).
// Every section starts at a multiple of 8 entries (128 B) and a row is a multiple of 8 entries, so
// k_flp_weights' 8-entry flushes write whole 128-B lines (a flush that straddled two lines left
// partial lines to be written back twice: 4.23 GB per SumVec launch against 3.52 algorithmic).
__host__ __device__ inline uint32_t round8(uint32_t x) { return (x + 7u) & ~7u; }
struct WRow {
  uint32_t C8, c8;
  DEVI explicit WRow(const Cfg& cfg) : C8(round8(cfg.calls)), c8(round8(cfg.chunk)) {}
  DEVI uint32_t mm(uint32_t k0) const { return k0; }  // k0 = k - 1
  DEVI uint32_t lm(uint32_t k0) const { return C8 + k0; }
  DEVI uint32_t rp(uint32_t j) const { return 2 * C8 + j; }
  DEVI uint32_t l0() const { return 2 * C8 + c8; }
  DEVI uint32_t hl() const { return 2 * C8 + c8 + 1; }
  DEVI uint32_t gsum() const { return 2 * C8 + c8 + 2; }
  DEVI uint32_t smm() const { return 2 * C8 + c8 + 3; }
  DEVI uint32_t slm() const { return 2 * C8 + c8 + 4; }
};
__host__ __device__ inline uint32_t flp_w_len(const Cfg& cfg) {
  return 2 * round8(cfg.calls) + round8(cfg.chunk) + 8;
}
// k_flp_weights' LDS windows and backward blocks: kFwChunk elements / calls
constexpr uint32_t kFwChunk = 4;
// entries of k_flp_weights' element-major scratch per report: the prefix product at the start of
// every kFwChunk-call block of the batched inversion
__host__ __device__ inline uint32_t flp_scratch_len(const Cfg& cfg) {
  return (cfg.calls + kFwChunk - 1) / kFwChunk;
}

// Wire-seed terms of column j (wire_2j, wire_2j+1 without the measurement sums): L0 s_2j and
// L0 s_2j+1 - HL, from the proof share's seeds; `bad` if a seed is not canonical.
DEVI void wire_seed_terms(const WMat& wm, const WRow& W, uint32_t r, const uint8_t* seeds,
                          uint32_t j, F128& t0, F128& t1, bool& bad) {
  using FO = Field128Ops;
  const F128 l0 = FO::load(wm.el(r, W.l0()));
  const F128 s0 = FO::load(seeds + (size_t)(2 * j) * 16), s1 = FO::load(seeds + (size_t)(2 * j + 1) * 16);
  bad |= !FO::is_canonical(s0) || !FO::is_canonical(s1);
  t0 = FO::mul(l0, s0);
  t1 = FO::sub(FO::mul(l0, s1), FO::load(wm.el(r, W.hl())));
}

// ------------------------------------------------------------------------------------------------
// FLP query for Count (Mul, 1 call) and Sum (PolyEval(x^2 - x), `bits` calls), one LANE per report:
// registers only, no LDS, no barriers, no NTT.  With L_k(t) = (t^m - 1)/m * alpha^k / (t - alpha^k):
//   wire_w(t) = C * sum_{k=0..calls} a_{w,k} / (t - alpha^k),   C = (t^m - 1)/m,
//     a_{w,0} = proof seed s_w,  a_{w,k} = alpha^k * (input of call k on wire w)
//   Sum:   v = sum_{k=1..calls} r^k p(alpha^k) = sum_{i<m} F_i G(r alpha^i),
//          F = the gadget poly folded mod x^m - 1,  G(y) = sum_{k=1..calls} y^k
//            = y (y^calls - 1)/(y - 1)  (= calls if y == 1),  y^calls = r^calls alpha^(i calls mod m)
//   Count: v = p(alpha) - x_0
//   p(t) by Horner.
// Both sums of fractions are accumulated as one numerator / denominator pair (N d + a D, D d: three
// multiplications per term), and the two denominators share ONE inversion (Montgomery's trick), so
// Sum32 costs ~900 multiplications per report where the block kernel ran two size-64 NTTs across
// 64 threads with a barrier per stage.  A zero t - alpha^k means t^m == 1: VdafPrepError (prio's
// "root of unity" rejection); the values computed then are discarded.
// ------------------------------------------------------------------------------------------------
// three independent Montgomery products: mont_mul3 for Field128, plain products for Field64
template <class FO>
DEVI void mul3(const typename FO::T& a0, const typename FO::T& b0, const typename FO::T& a1,
               const typename FO::T& b1, const typename FO::T& a2, const typename FO::T& b2,
               typename FO::T& r0, typename FO::T& r1, typename FO::T& r2) {
  if constexpr (FO::ES == 16) {
    F128 t0, t1, t2;
    mont_mul3(a0, b0, a1, b1, a2, b2, t0, t1, t2);
    r0 = t0;
    r1 = t1;
    r2 = t2;
  } else {
    const typename FO::T t0 = FO::mul(a0, b0), t1 = FO::mul(a1, b1), t2 = FO::mul(a2, b2);
    r0 = t0;
    r1 = t1;
    r2 = t2;
  }
}

#ifndef FLPQ_MUL3
#define FLPQ_MUL3 1
#endif

template <class FO>
DEVI typename FO::T inv_mont(const typename FO::T& x) {
  if constexpr (FO::ES == 16) return inv_mont128(x);
  else return inv_mont64(x);
}

// Sum's FLP query when calls = m/2 (power-of-two bits, m >= 8) and r^m != 1, Field128, one lane
// per report: the same field values as the generic loop below, from fewer products.  With
// h = m/2 = calls, alpha^h = -1, beta_i = alpha^-i (tables, Montgomery):
//   * gadget-output sum  v = sum_i F_i G(y_i),  F_i = c_i + c_(i+m),  y_i = r alpha^i,
//     G(y) = y (y^calls - 1)/(y - 1).  y_i^calls = r^calls (-1)^i =: s_i and
//     y_i/(y_i - 1) = r/(r - beta_i), so  v = r sum_par c_par Q_par,  c_par = s_par - 1,
//     Q_par = sum_(i = par) F_i/(r - beta_i): the denominators are r minus a constant.  Pairing
//     i with j = i + h (same parity, beta_j = -beta_i):
//       F_i/(r - beta) + F_j/(r + beta) = (r (F_i + F_j) + beta (F_i - F_j)) / (r^2 - beta^2),
//     so each of the h iterations adds ONE pair to its parity's fraction N/D;
//   * the wire  sum_(k=0..calls) alpha^k x_k/(t - alpha^k) = t sum_k x_k/(t - alpha^k) - sum_k x_k:
//     iteration i takes k = i (x_0 = the proof seed), k = calls is the fraction's start;
//   * p(t) = sum_(i<h) (A_i + t^h A_(i+h)) t^i,  A_i = c_i + t^m c_(i+m): one Horner step per pair;
//   * the three denominators share one inversion.
// Per iteration 7 Montgomery products (mont_fma.h, two interleaved calls: the Horner step's four
// products share ONE reduction, the numerator and wire fractions are fused pairs) against 10 for
// two iterations of the unpaired form (gadget fraction over y_i - 1 with y_i advanced by a
// product) and 24 of the mul3 loop.
// Domains: values marked M are Montgomery form (x R), the rest plain; mont(M, plain) is plain.
// Operands: iteration i reads c_i, c_(i+m), c_(i+h), c_(i+h+m) (gadget coefficients, proof
// elements 1 + .) and x_i (measurement element i - 1; x_0 = the proof seed).  A loop trip (i0 + 3
// down to i0, i0 = 0 mod 4) takes four consecutive elements (64 B) of each of these five streams,
// which arrive by LDS-DMA into a per-wave window of 5 x 4 KB (kSqWin): instruction k of a stream
// fills 1 KB = 16 reports x 4 elements, slot 4q + (u ^ ((q >> 1) & 3)) holding element u of report
// q (each lane's ds_read_b128 of its own report is then bank-conflict-free).  The next trip's DMA
// is issued once the trip's last operands sit in registers, so it lands under that iteration's
// products; no VGPRs are held by loads in flight.  64-B runs per report (rather than 32) halve the
// HBM sectors fetched per byte used (PMC: 12.4 GB per 1M-report launch with 2-element windows
// against 2.6 GB of operands).  Every lane of the wave takes part (dead lanes compute on a clamped
// row).
constexpr uint32_t kSqEl = 4u;                      // elements per stream per trip
constexpr uint32_t kSqWin = 5u * 64u * 16u * kSqEl;  // bytes per wave (20 KB)

DEVI void sum_query_pair(const Cfg& cfg, uint32_t n, uint32_t r0w, uint32_t lane, CRows meas,
                         CRows proof, uint8_t* win, const F128& tm, const F128& th,
                         const F128& tmm, const F128& rm, const F128& rc, const F128& s0,
                         bool& bad, F128& pt_out, F128& w0_out, F128& v_out) {
  using FO = Field128Ops;
  using T = F128;
  const uint32_t m = cfg.m, h = cfg.calls, gp_len = cfg.gp_len;
  const T one = FO::one_mont();
  const T t3h = FO::mul(tmm, th);                    // M(t^(m + h))
  const T r2 = FO::mul(rm, rm);                      // M(r^2)
  constexpr uint32_t SB = 64u * 16u * kSqEl;          // bytes per stream window
  // DMA of the trip covering elements i0 .. i0 + 3 of the five streams
  auto stage = [&](uint32_t i0) {
    uint32_t ln;  // opaque copy: the row addresses are recomputed per trip, never held
    asm volatile("v_mov_b32 %0, %1" : "=v"(ln) : "v"(lane));
    const uint32_t e = i0 + ((ln & 3u) ^ ((ln >> 3) & 3u));  // this lane's element
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
      const uint32_t row = min(r0w + 16u * k + (ln >> 2), n - 1u);
      const uint8_t* pr = proof.base + (size_t)row * proof.stride;
      const uint8_t* xr = meas.base + (size_t)row * meas.stride;
      const uint32_t off[4] = {e, e + m, e + h, (uint32_t)min(e + h + m, gp_len - 1u)};
#pragma unroll
      for (uint32_t s = 0; s < 4; ++s)
        __builtin_amdgcn_global_load_lds(
            (const __attribute__((address_space(1))) void*)(pr + 16u * (1u + off[s])),
            (__attribute__((address_space(3))) void*)(win + SB * s + 1024u * k), 16, 0, 0);
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(xr + 16u * (e ? e - 1u : 0u)),
          (__attribute__((address_space(3))) void*)(win + SB * 4u + 1024u * k), 16, 0, 0);
    }
  };
  const uint32_t sl = 64u * lane, sw = (lane >> 1) & 3u;
  auto rd = [&](uint32_t s, uint32_t u) { return FO::load(win + SB * s + sl + 16u * (u ^ sw)); };
  T N[2] = {FO::zero(), FO::zero()};                 // gadget-output fractions by parity, plain
  T D[2] = {one, one};                               // their denominators, M
  T X = FO::load(meas.at(min(r0w + lane, n - 1u)) + (size_t)(h - 1) * 16);  // x_calls
  bad |= !FO::is_canonical(X);
  T Nw = X, Dw = FO::sub(tm, ld_tw<FO>(cfg, h));     // plain / M(t - alpha^calls)
  // Horner's p_(i+1) = PQ + c_(i+1) is finished inside iteration i's additions
  T PQ = FO::zero(), cprev = FO::zero();
  stage(h - kSqEl);
  auto step = [&](uint32_t i, auto PAR) {
    constexpr uint32_t par = decltype(PAR)::value;  // = i & 1
    const uint32_t u = i & (kSqEl - 1u);               // window slot (wave-uniform)
    if (u == kSqEl - 1u) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the window landed
    const T ci = rd(0, u), cim = rd(1, u), cj = rd(2, u);
    const T cjm = i + h + m < gp_len ? rd(3, u) : FO::zero();
    const T x = i ? rd(4, u) : s0;
    if (u == 0u && i) {  // the trip's operands in registers: the window is free for the next one
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      stage(i - kSqEl);
    }
    bad |= !FO::is_canonical(ci) | !FO::is_canonical(cim) | !FO::is_canonical(cj) |
           !FO::is_canonical(cjm) | !FO::is_canonical(x);
    const uint32_t mi = (m - i) & (m - 1u), m2i = (m - 2u * i) & (m - 1u);
    const T beta = ld_tw<FO>(cfg, mi);                              // M(alpha^-i)
    T fi, fj, d2, dw;
    // F_i, F_j, M(r^2 - beta^2), M(t - alpha^i)
    modaddsub_AASS(ci, cim, fi, cj, cjm, fj, r2, ld_tw<FO>(cfg, m2i), d2, tm, ld_tw<FO>(cfg, i),
                   dw);
    T fs, fd, Xn, pt;
    modaddsub_ASAA(fi, fj, fs, fi, fj, fd, X, x, Xn, PQ, cprev, pt);
    // Horner: t p_(i+1) + t^m c_(i+m) + t^h c_(i+h) + t^(m+h) c_(i+h+m), one reduction
    T U, DN;
    mont_q1_fma1_mul1(tm, pt, tmm, cim, th, cj, t3h, cjm, PQ, rm, fs, beta, fd, U, D[par], d2,
                      DN);
    T NN, NW, DW;
    mont_fma2_mul1(N[par], d2, U, D[par], NN, Nw, dw, x, Dw, NW, Dw, dw, DW);
    N[par] = NN;
    D[par] = DN;
    Nw = NW;
    Dw = DW;
    X = Xn;
    cprev = ci;
  };
  // h = 0 mod 4: a window serves two loop bodies of (odd i, even i - 1), constant parities
  for (uint32_t i = h - 1;; i -= 2) {
    step(i, std::integral_constant<uint32_t, 1>{});
    step(i - 1, std::integral_constant<uint32_t, 0>{});
    if (i == 1) break;
  }
  T pt;
  modaddsub_A(PQ, cprev, pt);
  // one inversion for Dw, D0, D1
  T t1, t2, t3;
  mul3<FO>(D[0], D[1], Dw, D[1], Dw, D[0], t1, t2, t3);  // M(D0 D1), M(Dw D1), M(Dw D0)
  const T inv = inv_mont128(FO::mul(Dw, t1));            // M(1 / (Dw D0 D1))
  T iw, i0, i1;
  mul3<FO>(inv, t1, inv, t2, inv, t3, iw, i0, i1);       // M(1/Dw), M(1/D0), M(1/D1)
  T qw, q0, q1;
  mul3<FO>(Nw, iw, N[0], i0, N[1], i1, qw, q0, q1);      // plain fractions
  const T cm = FO::mul(FO::sub(tmm, one), ld_tw<FO>(cfg, m));  // M((t^m - 1)/m)
  const T c0 = FO::sub(rc, one), c1 = FO::sub(FO::sub(FO::zero(), rc), one);  // M(s_par - 1)
  T tq, v0, v1;
  mul3<FO>(tm, qw, c0, q0, c1, q1, tq, v0, v1);
  w0_out = FO::mul(cm, FO::sub(tq, X));
  v_out = FO::mul(rm, FO::add(v0, v1));
  pt_out = pt;
}

// The paired Sum query's shape (calls = m/2, Field128; sum_query_pair): the launch gives the
// kernel its LDS-DMA windows (4 waves x kSqWin of dynamic LDS) only then, so the other shapes
// (e.g. sum5) keep the CU's LDS for more blocks.
__host__ __device__ inline bool flpq_pair(const Cfg& cfg) {
  return cfg.es == 16 && cfg.kind == KIND_SUM && 2u * cfg.calls == cfg.m && cfg.m >= 8u &&
         cfg.arity == 1u;
}
constexpr uint32_t kFlpqPairLds = 4u * kSqWin;  // per 256-thread block

#ifndef FLPQ_WAVES  // at least 2 waves/SIMD (<= 256 VGPRs) for the Field128 paired Sum query
#define FLPQ_WAVES __attribute__((amdgpu_waves_per_eu(2)))
#endif
// Count's query randomness inline (k_query_rand's XOF, prio prepare_init): the first canonical
// word of XOF(verify_key, dst5, nonce), one Keccak copy for the absorb and any further squeeze.
DEVI F64 query_rand_f64(const Cfg& cfg, uint64_t vk_lo, uint64_t vk_hi, const uint8_t* nz) {
  MsgBlock mb;
  mb.clear();
  mb.header(cfg.algo_id, DST_QUERY_RANDOMNESS, vk_lo, vk_hi);
  mb.put64(25, ld64(nz));
  mb.put64(33, ld64(nz + 8));
  mb.pad(41, cfg.xof);
  uint64_t s[25];
#pragma unroll
  for (int i = 0; i < 25; ++i) s[i] = i < kRateWords ? mb.w[i] : 0ull;
  uint64_t v = 0ull;
  bool found = false;
  do {
    keccak_x(s, cfg.xof);
#pragma unroll
    for (int k = 0; k < kRateWords; ++k)
      if (!found && s[k] < Field64Ops::P) {
        v = s[k];
        found = true;
      }
  } while (!found);
  return Field64Ops::mk(v);
}

// qr_nonces != nullptr (Count): t is derived here from the nonce (the XOF phase launches this
// kernel instead of k_query_rand + a query-phase launch); otherwise t is read from tq.
template <class FO>
__global__ void __launch_bounds__(256) FLPQ_WAVES k_flp_query_lane(Cfg cfg, uint32_t n, CRows meas,
                                                        CRows proof, CRows tq, CRows jr,
                                                        CRows part, Rows out_prep,
                                                        uint8_t* status, const uint8_t* qr_nonces,
                                                        uint64_t vk_lo, uint64_t vk_hi) {
  using T = typename FO::T;
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  const bool live = r < n && status[r] == ST_OK;
  // Sum with calls = m/2 (Field128): the paired query, whole waves (its operands arrive by
  // LDS-DMA for all 64 lanes); every other shape: one independent lane per live report
  bool pair = false;
  if constexpr (FO::ES == 16) pair = flpq_pair(cfg);
  if (!pair && !live) return;
  const uint32_t lane = threadIdx.x & 63u, r0w = r - lane;
  if (pair && r0w >= n) return;  // wave-uniform
  const uint32_t rr = r < n ? r : n - 1u;  // = r on the generic path
  const size_t ES = FO::ES;
  const uint32_t m = cfg.m, calls = cfg.calls, arity = cfg.arity, gp_len = cfg.gp_len;
  const uint8_t* xr = meas.at(rr);
  const uint8_t* pr = proof.at(rr);
  const uint8_t* gp = pr + (size_t)arity * ES;  // gadget poly coefficients
  bool bad = false;
  const T one = FO::one_mont();
  T traw;
  if constexpr (FO::ES == 8) {
    traw = qr_nonces ? query_rand_f64(cfg, vk_lo, vk_hi, qr_nonces + 16u * rr) : FO::load(tq.at(rr));
  } else {
    traw = FO::load(tq.at(rr));
  }
  const T tm = FO::to_mont(traw);
  T tmm = tm;
  // Sum: t^m, r^m and r^calls (calls < m, right-to-left square-and-multiply) advance together,
  // one triple per bit: t and r squared, r^calls times r^(2^q) (or times one)
  T rm = FO::zero(), rmm = FO::zero(), rc = one, th = tm;
  if (cfg.kind == KIND_SUM) {
    rm = FO::to_mont(FO::load(jr.at(rr)));
    rmm = rm;
    for (uint32_t q = 0; q < cfg.logm; ++q) {  // rmm = r^(2^q) before the step
      T nrc;
      mul3<FO>(tmm, tmm, rmm, rmm, rc, ((calls >> q) & 1u) ? rmm : one, tmm, rmm, nrc);
      rc = nrc;
      if (q + 2u == cfg.logm) th = tmm;  // t^(m/2)
    }
  } else {
    for (uint32_t i = 0; i < cfg.logm; ++i) tmm = FO::mul(tmm, tmm);  // t^m
  }
  const bool root = FO::eq(tmm, one);
  const T cm = FO::mul(FO::sub(tmm, one), ld_tw<FO>(cfg, m));  // (t^m - 1)/m, Montgomery

  // wires: N_w / D over k = 0..calls
  T nw0 = FO::zero(), nw1 = FO::zero(), dw = one;
  const T s0 = FO::load(pr), s1 = arity > 1 ? FO::load(pr + ES) : FO::zero();
  bad |= !FO::is_canonical(s0) || !FO::is_canonical(s1);
  if constexpr (FO::ES == 16) {
    if (pair) {
      extern __shared__ __attribute__((aligned(16))) uint8_t sqlds[];  // kFlpqPairLds
      const bool r_root = FO::eq(rmm, one);  // y_i = 1 for some i: the generic loop below
      bool pbad = bad;
      T pt, w0, v;
      sum_query_pair(cfg, n, r0w, lane, meas, proof, sqlds + (threadIdx.x >> 6) * kSqWin, tm, th,
                     tmm, rm, rc, s0, pbad, pt, w0, v);
      if (!live) return;
      if (!r_root) {
        uint8_t* outp = out_prep.at(r);
        FO::store(outp, v);
        FO::store(outp + ES, w0);
        FO::store(outp + (size_t)(1 + arity) * ES, pt);
        const uint8_t* pp = part.at(r);
        uint8_t* dst = outp + (size_t)cfg.verifier_len * ES;
        st64(dst, ld64(pp));
        st64(dst + 8, ld64(pp + 8));
        if (pbad) status[r] = ST_INVALID_MESSAGE;
        else if (root) status[r] = ST_VDAF_PREP_ERROR;
        return;
      }
    }
  }
  T x0 = FO::zero();
  if (cfg.kind == KIND_COUNT) {
    x0 = FO::load(xr);
    bad |= !FO::is_canonical(x0);
  }
  // k-th term of the wire fraction (k >= 1; k = 0 is peeled: a = the proof seed)
  auto wire_step = [&](uint32_t k) {
    const T ak = ld_tw<FO>(cfg, k);  // alpha^k, Montgomery
    const T d = FO::sub(tm, ak);
    T x = x0;
    if (cfg.kind != KIND_COUNT) {
      x = FO::load(xr + (size_t)(k - 1) * ES);
      bad |= !FO::is_canonical(x);
    }
    const T a = FO::mul(ak, x);
    nw0 = FO::add(FO::mul(nw0, d), FO::mul(a, dw));
    if (arity > 1) nw1 = FO::add(FO::mul(nw1, d), FO::mul(a, dw));
    dw = FO::mul(dw, d);
  };

  T pt = FO::zero();
  T vn = FO::zero(), vd = one, extra = FO::zero();
  if (cfg.kind == KIND_COUNT) {
    for (uint32_t k = calls; k >= 1; --k) wire_step(k);
    for (uint32_t d = gp_len; d-- > 0;) {  // p(t) by Horner
      const T c = FO::load(gp + (size_t)d * ES);
      bad |= !FO::is_canonical(c);
      pt = FO::add(FO::mul(tm, pt), c);
    }
    const T al = ld_tw<FO>(cfg, 1);
    T pa = FO::zero();
    for (uint32_t d = gp_len; d-- > 0;) pa = FO::add(FO::mul(al, pa), FO::load(gp + (size_t)d * ES));
    extra = FO::sub(pa, x0);
  } else {  // KIND_SUM: one pass over i = m-1 .. 0 carrying three independent chains
    // (Horner on p(t) = sum_i (c_i + c_(i+m) t^m) t^i, the v fraction over G(r alpha^i), and for
    // i <= calls the wire fraction), so the Montgomery carry chains of one fill the other's
    // hazard slots; y_i = r alpha^i == 1 needs r^m == 1, handled outside the loop.
    const bool r_root = FO::eq(rmm, one);
    auto coeffs = [&](uint32_t i, T& ci, T& ch) {
      ci = FO::load(gp + (size_t)i * ES);
      ch = i + m < gp_len ? FO::load(gp + (size_t)(i + m) * ES) : FO::zero();
      bad |= !FO::is_canonical(ci) || !FO::is_canonical(ch);
    };
    auto v_step = [&](uint32_t i, const T& f) {
      const T y = FO::mul(rm, ld_tw<FO>(cfg, i));
      const T e = FO::sub(y, one);
      const T yc = FO::mul(rc, ld_tw<FO>(cfg, (uint32_t)(((uint64_t)i * calls) % m)));
      const T b = FO::mul(FO::mul(y, f), FO::sub(yc, one));
      vn = FO::add(FO::mul(vn, e), FO::mul(b, vd));
      vd = FO::mul(vd, e);
    };
    if (!r_root && FLPQ_MUL3) {
      // the same three chains, every iteration's products issued as hazard-free triples
      // (mont_mul3, Field128).  b_i * vd is refactored as (y f) * ((yc - 1) vd) so the
      // 12 (13) products of a wire iteration form 4 triples (+1 single); when calls == m / 2
      // (Sum with power-of-two bits) yc = r^calls alpha^(i calls) = +-r^calls needs no product.
      const bool half = 2u * calls == m;
      const T ycm_even = FO::sub(rc, one), ycm_odd = FO::sub(FO::sub(FO::zero(), rc), one);
      for (uint32_t i = m - 1;; --i) {
        const bool wire = i >= 1 && i <= calls;
        T ci, ch;
        coeffs(i, ci, ch);
        T x = FO::zero();
        if (wire) {
          x = FO::load(xr + (size_t)(i - 1) * ES);
          bad |= !FO::is_canonical(x);
        }
        const T f = FO::add(ci, ch);
        const T twi = ld_tw<FO>(cfg, i);
        const T d = FO::sub(tm, twi);
        T q, y, u, a, P, dwn, g, yf, vde, vne, adw, nwd, yfg;
        // triple 1: q = t^m c_(i+m), y = r alpha^i, u = (half ? g : yc)
        if (half) {
          const T ycm = (i & 1u) ? ycm_odd : ycm_even;
          mul3<FO>(tmm, ch, rm, twi, ycm, vd, q, y, g);
        } else {
          mul3<FO>(tmm, ch, rm, twi, rc, ld_tw<FO>(cfg, (uint32_t)(((uint64_t)i * calls) % m)), q,
                   y, u);
        }
        const T e = FO::sub(y, one);
        if (wire) {
          // P = t pt, a = alpha^i x, dw d;  y f, vd e, vn e;  a dw, nw0 d, (y f) g
          mul3<FO>(tm, pt, twi, x, dw, d, P, a, dwn);
          if (!half) g = FO::mul(FO::sub(u, one), vd);
          mul3<FO>(y, f, vd, e, vn, e, yf, vde, vne);
          mul3<FO>(a, dw, nw0, d, yf, g, adw, nwd, yfg);
          nw0 = FO::add(nwd, adw);
          dw = dwn;
        } else if (half) {
          // y f, vd e, vn e;  P = t pt, (y f) g (+ an idle slot: still cheaper than two singles)
          mul3<FO>(y, f, vd, e, vn, e, yf, vde, vne);
          T idle;
          mul3<FO>(tm, pt, yf, g, one, one, P, yfg, idle);
        } else {
          // g = (yc - 1) vd, P = t pt, y f;  vd e, vn e, (y f) g
          mul3<FO>(FO::sub(u, one), vd, tm, pt, y, f, g, P, yf);
          mul3<FO>(vd, e, vn, e, yf, g, vde, vne, yfg);
        }
        pt = FO::add(P, FO::add(ci, q));
        vn = FO::add(vne, yfg);
        vd = vde;
        if (i == 0) break;
      }
    } else if (!r_root) {
      for (uint32_t i = m - 1; i > calls; --i) {
        T ci, ch;
        coeffs(i, ci, ch);
        pt = FO::add(FO::mul(tm, pt), FO::add(ci, FO::mul(tmm, ch)));
        v_step(i, FO::add(ci, ch));
      }
      for (uint32_t i = calls; i >= 1; --i) {
        T ci, ch;
        coeffs(i, ci, ch);
        pt = FO::add(FO::mul(tm, pt), FO::add(ci, FO::mul(tmm, ch)));
        v_step(i, FO::add(ci, ch));
        wire_step(i);
      }
      T ci, ch;
      coeffs(0, ci, ch);
      pt = FO::add(FO::mul(tm, pt), FO::add(ci, FO::mul(tmm, ch)));
      v_step(0, FO::add(ci, ch));
    } else {  // r^m == 1 (probability ~m / p): some y_i == 1, where G = calls
      for (uint32_t k = calls; k >= 1; --k) wire_step(k);
      const T calls_m = FO::to_mont(FO::from_u32(calls));
      for (uint32_t i = m; i-- > 0;) {
        T ci, ch;
        coeffs(i, ci, ch);
        pt = FO::add(FO::mul(tm, pt), FO::add(ci, FO::mul(tmm, ch)));
        const T f = FO::add(ci, ch);
        if (FO::is_zero(FO::sub(FO::mul(rm, ld_tw<FO>(cfg, i)), one)))
          extra = FO::add(extra, FO::mul(calls_m, f));
        else
          v_step(i, f);
      }
    }
  }
  // the k = 0 wire term: a = the proof seed
  {
    const T d = FO::sub(tm, one);
    nw0 = FO::add(FO::mul(nw0, d), FO::mul(s0, dw));
    if (arity > 1) nw1 = FO::add(FO::mul(nw1, d), FO::mul(s1, dw));
    dw = FO::mul(dw, d);
  }

  T w0, w1 = FO::zero(), v;
  if (cfg.kind == KIND_COUNT && calls + 1u == m) {
    // Count: the wire terms run over every m-th root of unity, so dw = t^m - 1 and the wire is
    // (t^m - 1)/m N/dw = N/m; vn = 0, vd = 1: v = extra.  No inversion (the values of a root
    // t, rejected below, are those of the general path: inv(0) = 0).
    const T im = ld_tw<FO>(cfg, m);  // 1/m
    w0 = root ? FO::zero() : FO::mul(nw0, im);
    if (arity > 1) w1 = root ? FO::zero() : FO::mul(nw1, im);
    v = extra;
  } else {
    // one inversion for both denominators
    const T inv = inv_mont<FO>(FO::mul(dw, vd));
    const T dinv = FO::mul(inv, vd), vinv = FO::mul(inv, dw);
    w0 = FO::mul(cm, FO::mul(nw0, dinv));
    if (arity > 1) w1 = FO::mul(cm, FO::mul(nw1, dinv));
    v = FO::add(FO::mul(vn, vinv), extra);
  }

  uint8_t* outp = out_prep.at(r);
  FO::store(outp, v);
  FO::store(outp + ES, w0);
  if (arity > 1) FO::store(outp + 2 * ES, w1);
  FO::store(outp + (size_t)(1 + arity) * ES, pt);
  if (cfg.jr_len > 0) {
    const uint8_t* pp = part.at(r);
    uint8_t* dst = outp + (size_t)cfg.verifier_len * ES;
    st64(dst, ld64(pp));
    st64(dst + 8, ld64(pp + 8));
  }
  if (bad) status[r] = ST_INVALID_MESSAGE;
  else if (root) status[r] = ST_VDAF_PREP_ERROR;
}

// ------------------------------------------------------------------------------------------------
// Cross-lane helpers for Field elements.
// ------------------------------------------------------------------------------------------------
template <class FO>
DEVI typename FO::T shfl_T(const typename FO::T& v, int src) {
  typename FO::T o;
#pragma unroll
  for (int w = 0; w < FO::NW; ++w) o.w[w] = __shfl(v.w[w], src, 64);
  return o;
}
template <class FO>
DEVI typename FO::T shfl_xor_T(const typename FO::T& v, int mask) {
  typename FO::T o;
#pragma unroll
  for (int w = 0; w < FO::NW; ++w) o.w[w] = __shfl_xor(v.w[w], mask, 64);
  return o;
}
template <class FO>
DEVI typename FO::T wave_sum(typename FO::T v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v = FO::add(v, shfl_xor_T<FO>(v, off));
  return v;
}
template <class FO>
DEVI typename FO::T sel(bool c, const typename FO::T& a, const typename FO::T& b) {
  typename FO::T o;
#pragma unroll
  for (int w = 0; w < FO::NW; ++w) o.w[w] = c ? a.w[w] : b.w[w];
  return o;
}

// ------------------------------------------------------------------------------------------------
// FLP query, ParallelSum types, first half, one LANE per report (Field128):
//   * Lagrange weights L_k(t) = (alpha^k/m) (t^m - 1) / (t - alpha^k), k = 0..calls, from ONE
//     batched inversion (Montgomery's trick over d_k = t - alpha^k) whose prefix products are kept
//     only at the start of every kFwChunk-call block (element-major scratch) and recomputed inside
//     a block on the way back; r^c is folded into the same inversion, so MM[k] = L_k r^(c(k-1))
//     comes out of the backward pass directly (descending powers);
//   * RP[j] = r^(j+1) by a running product beside the prefix products;
//   * p(t) by three Horner chains in t^3 and the gadget-output sum sum_d c_d S[d mod m] as a lazily
//     reduced dot product, over the gadget-poly part of the proof share only (the wire seeds are
//     read by the wire passes, which finish wire_2j = L0 s_2j + ..., see WRow);
//   * serial chains issue as hazard-free Field128 pairs / triples (mont_mul2, mont_mul3).
// Sized for 3 waves per SIMD (<= 168 VGPRs, 8 KB of LDS per wave): a backward block of 4 calls
// first runs its L chain (three products per step: L_k = inv P_(k-1) alpha^k/m, inv <- inv d_k and
// the next entry's P_(k-2) alpha^(k-1)/m), parks the L_k in the output window and flushes them as
// LM, then forms MM_k = L_k q and q <- q / r^c as pairs from the window (two products per step).
// Table entries (alpha^k, alpha^k/m, S_i) are wave-uniform (scalar loads).  Memory moves coalesced
// through two per-wave LDS windows of 4 elements x 64 reports (slot 4q + (u ^ ((q >> 2) & 3))
// holds element u of report q: each lane's ds_read/write_b128 of its own row is bank-conflict-free,
// and 4 lanes cover 64 contiguous bytes of one report's row): the proof share arrives by LDS-DMA,
// the weight rows leave 4 entries (half a line; the next flush completes the line) at a time.  Per
// SumVec(8,1000) report it reads the 255 gadget coefficients (4 KB) and writes MM, LM, RP and five
// scalars (4.4 KB) plus 0.4 KB of scratch.
// ------------------------------------------------------------------------------------------------
#ifndef P3G_FLP_PRIO
#define P3G_FLP_PRIO 0  // A/B knob: s_setprio of the FLP kernels (schedules that co-run them)
#endif
constexpr uint32_t kFwWin = 64 * kFwChunk * 16;  // bytes per window (one wave)
constexpr uint32_t kFwThreads = 128;

__global__ void __launch_bounds__(kFwThreads) __attribute__((amdgpu_waves_per_eu(3)))
k_flp_weights(Cfg cfg, uint32_t n, CRows proof, CRows tq, CRows jr, CRows part, Rows out_prep,
              uint8_t* status, WMat wm, uint8_t* scr) {
  using FO = Field128Ops;
  using T = F128;
  if constexpr (P3G_FLP_PRIO > 0) __builtin_amdgcn_s_setprio(P3G_FLP_PRIO);
  __shared__ __attribute__((aligned(16))) uint8_t lds[(kFwThreads / 64) * 2 * kFwWin];
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  const uint32_t r0w = blockIdx.x * blockDim.x + 64u * wv;
  if (r0w >= n) return;  // wave-uniform
  uint8_t* win = lds + wv * 2u * kFwWin;  // proof window; later the MM output window
  uint8_t* wout = win + kFwWin;           // output window (RP, LM)
  const uint32_t r = r0w + lane;
  const bool live = r < n && status[r] == ST_OK;
  const uint64_t livemask = __ballot(live);
  const uint32_t rr = r < n ? r : n - 1u;  // clamped: dead lanes compute on a valid row
  const uint32_t m = cfg.m, logm = cfg.logm, C = cfg.calls, c = cfg.chunk;
  const uint32_t arity = cfg.arity, gp_len = cfg.gp_len;
  const WRow W(cfg);
  constexpr uint32_t K = kFwChunk;
  const uint32_t sw = (lane >> 2) & (K - 1u);  // this lane's swizzle
  const T one = FO::one_mont();
  bool bad = false;
  // block-start prefix products, element-major: entry b holds P_(Kb) of report rr
  auto S = [&](uint32_t b) { return scr + ((size_t)b * n + rr) * 16u; };
  // this lane's slot u of a window.  An inline-asm ds_write: hipcc cannot tell a plain LDS store
  // from a write the earlier LDS-DMA fills might race with, and put a vmcnt(0) in front of every
  // one -- a wait for the flush's global stores (the fills themselves are waited for explicitly
  // before the window is read, and are all done before the backward pass writes win)
  auto put = [&](uint8_t* w, uint32_t u, const T& v) {
    lds_store16(w + 16u * K * lane + 16u * (u ^ sw), v);
  };
  auto get = [&](const uint8_t* w, uint32_t u) {
    return FO::load(w + 16u * K * lane + 16u * (u ^ sw));
  };
  // gadget-poly window <- coefficients [K ch, K ch + K) of the wave's 64 rows (LDS-DMA instruction
  // i fills slots [64i, 64i + 64): report 16i + lane/4, element (lane & 3) ^ swizzle)
  auto stage = [&](uint32_t ch) {
    uint32_t ln;  // opaque copy (see flush)
    asm volatile("v_mov_b32 %0, %1" : "=v"(ln) : "v"(lane));
    const uint32_t ql = ln / K;
#pragma unroll
    for (uint32_t i = 0; i < K; ++i) {
      const uint32_t q = (64u / K) * i + ql;
      const uint32_t u = (ln & (K - 1u)) ^ ((q >> 2) & (K - 1u));
      const uint32_t row = min(r0w + q, n - 1u);
      const uint32_t e = arity + min(K * ch + u, gp_len - 1u);
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(proof.base + (size_t)row * proof.stride +
                                                          16u * e),
          (__attribute__((address_space(3))) void*)(win + 1024u * i), 16, 0, 0);
    }
  };
  // weight-row entries [pos, pos + cnt) (cnt <= K) of every live report of the wave <- window w
  auto flush = [&](uint8_t* w, uint32_t pos, uint32_t cnt) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    uint32_t ln;  // opaque copy: keeps LICM from hoisting the row addresses out of the callers' loops
    asm volatile("v_mov_b32 %0, %1" : "=v"(ln) : "v"(lane));
    const uint32_t ql = ln / K, u = ln & (K - 1u);
#pragma unroll
    for (uint32_t i = 0; i < K; ++i) {
      const uint32_t q = (64u / K) * i + ql;
      const T x = FO::load(w + 16u * (K * q + (u ^ ((q >> 2) & (K - 1u)))));
      if (u < cnt && ((livemask >> q) & 1ull)) FO::store(wm.el(r0w + q, pos + u), x);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  };
  const uint32_t nch = (gp_len + K - 1u) / K;
  stage(nch - 1u);  // in flight under the prefix products

  const T tm = FO::to_mont(FO::load(tq.at(rr)));
  const T rm = FO::to_mont(FO::load(jr.at(rr)));
  T tmm = tm;
  for (uint32_t i = 0; i < logm; ++i) tmm = FO::mul(tmm, tmm);  // t^m
  const bool tbad = FO::eq(tmm, one);

  // ---- forward: P_k = d_0 ... d_k (k <= C; P_(Kb) parked for block b) beside RP[j] = r^(j+1) ----
  T P = FO::sub(tm, one);  // d_0 (alpha^0 = 1)
  T rp = one;
  const uint32_t steps = C > c ? C : c;
  for (uint32_t k = 1; k <= steps; ++k) {
    if (k <= C && ((k - 1u) & (K - 1u)) == 0u) FO::store(S((k - 1u) / K), P);
    const T d = FO::sub(tm, ld_tw<FO>(cfg, k <= C ? k : 1u));
    T nP, nrp;
    mont_mul2(P, d, nP, rp, rm, nrp);
    if (k <= C) P = nP;
    if (k <= c) {
      rp = nrp;
      const uint32_t u = (k - 1u) & (K - 1u);
      put(wout, u, rp);
      if (u == K - 1u || k == c) flush(wout, W.rp((k - 1u) & ~(K - 1u)), u + 1u);
    }
  }
  const T rc = rp;  // r^c

  // ---- p(t) and the gadget-output sum over the gadget coefficients, last window first ----
  // p(t) = A0(t^3) + t A1(t^3) + t^2 A2(t^3): three Horner chains in t^3 advanced as one triple per
  // group of coefficients (3g+2, 3g+1, 3g); c2/c1 park the group's first two
  const T t3 = FO::mul(FO::mul(tm, tm), tm);
  T A0 = FO::zero(), A1 = FO::zero(), A2 = FO::zero(), c2 = FO::zero(), c1 = FO::zero();
  Wide gw;
  wide_zero(gw);
  for (int ch = (int)nch - 1; ch >= 0; --ch) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    T xb[K];
#pragma unroll
    for (uint32_t u = 0; u < K; ++u) xb[u] = get(win, u);
    if (ch > 0) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      stage((uint32_t)ch - 1u);
    }
    const uint32_t e0 = K * (uint32_t)ch;
#pragma unroll
    for (int u = K - 1; u >= 0; --u) {
      const uint32_t e = e0 + (uint32_t)u;  // coefficient index (wave-uniform)
      if (e >= gp_len) continue;
      bad |= !FO::is_canonical(xb[u]);
      const uint32_t g3 = e % 3u;
      if (g3 == 2u) {
        c2 = xb[u];
      } else if (g3 == 1u) {
        c1 = xb[u];
      } else {
        T n2, n1, n0;
        mul3<FO>(A2, t3, A1, t3, A0, t3, n2, n1, n0);
        A2 = FO::add(n2, c2);
        A1 = FO::add(n1, c1);
        A0 = FO::add(n0, xb[u]);
      }
      wide_mac(gw, ld_tw<FO>(cfg, m + 1u + (e & (m - 1u))), xb[u]);
    }
  }
  const T pt = FO::add(FO::mul(FO::add(FO::mul(A2, tm), A1), tm), A0);
  const T gsum = wide_reduce(gw);

  // ---- one inversion for 1/(d_0 ... d_C) and 1/r^c; q = (r^c)^(C-1) for the descending MM ----
  const bool rz = FO::is_zero(rc);  // r = 0: MM[1] = L_1, every other MM[k] = 0
  T q = one;
  {
    T b = rc;
    for (uint32_t e = C - 1u; e != 0u; e >>= 1) {
      T nq, nb, idle;
      mul3<FO>(q, b, b, b, one, one, nq, nb, idle);
      if (e & 1u) q = nq;
      b = nb;
    }
  }
  const T iv = inv_mont128(rz ? P : FO::mul(P, rc));
  T ivP, ivrc, idle0;
  mul3<FO>(iv, P, iv, rc, one, one, ivP, ivrc, idle0);
  const T rcinv = rz ? FO::zero() : ivP;
  T inv = FO::mul(rz ? iv : ivrc, FO::sub(tmm, one));  // (t^m - 1) / (d_0 ... d_C)

  // ---- backward, k = C .. 1 in blocks of K: L_k = inv P_(k-1) alpha^k/m, inv <- inv d_k (LM
  //      through wout), then MM_k = L_k (r^c)^(k-1), q <- q / r^c (MM through win) ----
  T lsum = FO::zero(), smm = FO::zero();
  for (int blk = (int)((C - 1u) / K); blk >= 0; --blk) {
    const uint32_t lo = K * (uint32_t)blk + 1u;
    const uint32_t nb = C - lo + 1u < K ? C - lo + 1u : K;
    T pb[K];
    pb[0] = FO::load(S((uint32_t)blk));  // P_(lo - 1)
#pragma unroll
    for (uint32_t u = 1; u < K; ++u)
      if (u < nb) pb[u] = FO::mul(pb[u - 1], FO::sub(tm, ld_tw<FO>(cfg, lo + u - 1u)));
    T ptw = one;
#pragma unroll
    for (int u = K - 1; u >= 0; --u) {
      if ((uint32_t)u < nb) {
        const uint32_t k = lo + (uint32_t)u;
        if ((uint32_t)u + 1u == nb) ptw = FO::mul(pb[u], ld_tw<FO>(cfg, 2u * m + 1u + k));
        const T d = FO::sub(tm, ld_tw<FO>(cfg, k));
        const T pn = u > 0 ? pb[u > 0 ? u - 1 : 0] : one;
        const T tn = u > 0 ? ld_tw<FO>(cfg, 2u * m + k) : one;
        // the chain step {inv pt_k, inv d_k} and the next entry's P_(k-2) alpha^(k-1)/m
        T lk, ninv, nptw;
        mul3<FO>(inv, ptw, inv, d, pn, tn, lk, ninv, nptw);
        inv = ninv;
        ptw = nptw;
        put(wout, (uint32_t)u, lk);
        lsum = FO::add(lsum, lk);
      }
    }
    flush(wout, W.lm(lo - 1u), nb);
#pragma unroll
    for (int u = K - 1; u >= 0; --u) {
      if ((uint32_t)u < nb) {
        const T lk = get(wout, (uint32_t)u);
        T mm, nq;
        mont_mul2(lk, q, mm, q, rcinv, nq);
        if (rz) mm = lo + (uint32_t)u == 1u ? lk : FO::zero();
        q = nq;
        put(win, (uint32_t)u, mm);
        smm = FO::add(smm, mm);
      }
    }
    flush(win, W.mm(lo - 1u), nb);
  }
  const T l0 = FO::mul(inv, ld_tw<FO>(cfg, 2u * m + 1u));  // k = 0
  const T hl = FO::mul(lsum, FO::half());

  if (!live) return;
  FO::store(wm.el(rr, W.l0()), l0);
  FO::store(wm.el(rr, W.hl()), hl);
  FO::store(wm.el(rr, W.gsum()), gsum);
  FO::store(wm.el(rr, W.smm()), smm);
  FO::store(wm.el(rr, W.slm()), lsum);
  uint8_t* outp = out_prep.at(rr);
  if (cfg.kind != KIND_HISTOGRAM) FO::store(outp, gsum);  // v (Histogram: the wire pass)
  FO::store(outp + (size_t)(1 + arity) * 16, pt);
  const uint8_t* pp = part.at(rr);
  uint8_t* dst = outp + (size_t)cfg.verifier_len * 16;
  st64(dst, ld64(pp));
  st64(dst + 8, ld64(pp + 8));
  if (bad) status[rr] = ST_INVALID_MESSAGE;
  else if (tbad) status[rr] = ST_VDAF_PREP_ERROR;
}

// ------------------------------------------------------------------------------------------------
// FLP query, ParallelSum types, second half: stream the measurement share once and form the wires
//   wire_2j   = B0[j] + r^(j+1) sum_k MM[k] x_(k-1)c+j      wire_2j+1 = B1[j] + sum_k LM[k] x_(k-1)c+j
// (weights from k_flp_query's split mode).  Block per report, thread (h, j): column j, calls
// k = 1+h, 1+h+H, ...; lazy-reduced 256-bit MACs, two measurement loads in flight per thread.
// ------------------------------------------------------------------------------------------------
template <class FO>
__global__ void __launch_bounds__(1024) k_flp_wires(Cfg cfg, uint32_t n, FlpDims dims, CRows meas,
                                                   CRows proof, WMat wm, CRows jr, Rows out_prep,
                                                   uint8_t* status) {
  using T = typename FO::T;
  static_assert(FO::ES == 16, "ParallelSum types are Field128");
  const WRow W(cfg);
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t r = blockIdx.x;
  if (r >= n) return;
  if (status[r] != ST_OK) return;
  const uint32_t tid = threadIdx.x, nthr = blockDim.x;
  const uint32_t C = cfg.calls, c = dims.cols, H = dims.H;
  const size_t ES = FO::ES;
  T* MM = reinterpret_cast<T*>(smem);
  T* LM = MM + C;
  T* PA = LM + C;
  T* PB = PA + H * c;
  T* RED = PB + H * c;
  uint32_t* flag = reinterpret_cast<uint32_t*>(RED + nthr);
  if (tid == 0) *flag = 0u;
  for (uint32_t k = tid; k < 2 * C; k += nthr)
    MM[k] = FO::load(wm.el(r, k < C ? W.mm(k) : W.lm(k - C)));
  __syncthreads();
  const uint8_t* xr = meas.at(r);
  bool bad = false;
  T xsum = FO::zero();
  for (uint32_t slot = tid; slot < H * c; slot += nthr) {
    const uint32_t j = slot % c, h = slot / c;
    T accA, accB;
    if constexpr (FO::ES == 16) {
      Wide wa, wb;
      wide_zero(wa);
      wide_zero(wb);
      // each element is loaded just before its MACs: the pass hides HBM latency with occupancy
      // (78 VGPRs); loading one or three calls ahead (84-88 VGPRs) ran 5-8 % slower
      // (profiles/r03/ab_wires_ahead*.log).  The canonical check is a one-compare pre-filter (an
      // element >= p has its top word 2^32 - 1), the exact comparison only for a thread that saw
      // such a word.
      uint64_t maybe = 0ull;  // lane mask (SGPRs)
      uint32_t k = h;
      for (; k + H < C; k += 2 * H) {  // calls k and k+H; only the last call can be padded
        const uint32_t i0 = k * c + j, i1 = (k + H) * c + j;
        const T x0 = FO::load(xr + (size_t)i0 * ES);
        const T x1 = i1 < cfg.meas_len ? FO::load(xr + (size_t)i1 * ES) : FO::zero();
        maybe |= __ballot(x0.w[3] == 0xFFFFFFFFu || x1.w[3] == 0xFFFFFFFFu);
        wide_mac(wa, MM[k], x0);
        wide_mac(wb, LM[k], x0);
        wide_mac(wa, MM[k + H], x1);
        wide_mac(wb, LM[k + H], x1);
        if (cfg.kind == KIND_HISTOGRAM) xsum = FO::add(FO::add(xsum, x0), x1);
      }
      if (k < C) {
        const uint32_t i0 = k * c + j;
        if (i0 < cfg.meas_len) {
          const T x0 = FO::load(xr + (size_t)i0 * ES);
          maybe |= __ballot(x0.w[3] == 0xFFFFFFFFu);
          wide_mac(wa, MM[k], x0);
          wide_mac(wb, LM[k], x0);
          if (cfg.kind == KIND_HISTOGRAM) xsum = FO::add(xsum, x0);
        }
      }
      if (maybe) {  // rare: the exact check over this wave's elements
        for (uint32_t kk = h; kk < C; kk += H) {
          const uint32_t ii = kk * c + j;
          if (ii < cfg.meas_len) bad |= !FO::is_canonical(FO::load(xr + (size_t)ii * ES));
        }
      }
      accA = wide_reduce(wa);
      accB = wide_reduce(wb);
    } else {
      accA = FO::zero();
      accB = FO::zero();
      for (uint32_t k = h; k < C; k += H) {
        const uint32_t idx = k * c + j;
        if (idx < cfg.meas_len) {
          const T x = FO::load(xr + (size_t)idx * ES);
          bad |= !FO::is_canonical(x);
          accA = FO::add(accA, FO::mul(MM[k], x));
          accB = FO::add(accB, FO::mul(LM[k], x));
          if (cfg.kind == KIND_HISTOGRAM) xsum = FO::add(xsum, x);
        }
      }
    }
    PA[h * c + j] = accA;
    PB[h * c + j] = accB;
  }
  __syncthreads();
  uint8_t* outp = out_prep.at(r);
  for (uint32_t j = tid; j < c; j += nthr) {
    T a = FO::zero(), b = FO::zero();
    for (uint32_t h = 0; h < H; ++h) {
      a = FO::add(a, PA[h * c + j]);
      b = FO::add(b, PB[h * c + j]);
    }
    T b0, b1;
    wire_seed_terms(wm, W, r, proof.at(r), j, b0, b1, bad);
    const T rp = FO::load(wm.el(r, W.rp(j)));  // Montgomery
    FO::store(outp + (size_t)(1 + 2 * j) * ES, FO::add(b0, FO::mul(rp, a)));
    FO::store(outp + (size_t)(2 + 2 * j) * ES, FO::add(b1, b));
  }
  if (bad) atomicOr(flag, 1u);
  if (cfg.kind == KIND_HISTOGRAM) xsum = block_sum<FO>(xsum, RED, tid, nthr);
  __syncthreads();
  if (tid == 0) {
    if (cfg.kind == KIND_HISTOGRAM) {
      // v = jr[1] * range + jr[1]^2 * (sum x - 1/2)
      const T gsum = FO::load(wm.el(r, W.gsum()));
      const T r1m = FO::to_mont(FO::load(jr.at(r) + ES));
      const T sc = FO::sub(xsum, FO::half());
      FO::store(outp, FO::add(FO::mul(r1m, gsum), FO::mul(FO::mul(r1m, r1m), sc)));
    }
    if (*flag & 1u) status[r] = ST_INVALID_MESSAGE;
  }
}

// sum_q xs[q] 2^(32 q) mod p, the xs[q] being sums of < 2^32 32-bit words (canonical result)
DEVI F128 f128_reduce_limb_sums(const uint64_t (&xs)[4]) {
  typedef unsigned __int128 u128;
  const u128 CC = ((u128)28u << 64) - 1u;  // 2^128 - p
  const u128 P = ~(u128)0 - CC + 1u;
  // exact value = lo + top 2^128
  u128 acc = (u128)xs[0] + ((u128)xs[1] << 32);
  u128 c64 = acc >> 64;
  uint64_t w0 = (uint64_t)acc;
  u128 hi = c64 + (u128)xs[2] + ((u128)xs[3] << 32);  // < 2^97
  const u128 lo = ((u128)(uint64_t)hi << 64) | w0;
  const uint64_t top = (uint64_t)(hi >> 64);
  // 2^128 = CC (mod p): lo + top CC < 2^128 + 2^102, then at most one wrap and one subtraction
  u128 v = lo + (u128)top * CC;
  if (v < lo) v += CC;  // wrapped past 2^128 (v is tiny now)
  if (v >= P) v -= P;
  return F128{{(uint32_t)v, (uint32_t)(v >> 32), (uint32_t)(v >> 64), (uint32_t)(v >> 96)}};
}

// ------------------------------------------------------------------------------------------------
// k_flp_wires for short rows (chunk <= 64, Field128: Histogram, small SumVec/CountVec): a group of
// G = next_pow2(chunk) lanes per report, lane j = column j, every call k in that lane:
//   a_j = sum_k MM[k] x_(kc+j),  b_j = sum_k LM[k] x_(kc+j)   (lazy 256-bit MACs, one REDC each)
// For fixed k the group's x loads are one contiguous 16c-byte run and the weight loads a broadcast;
// no LDS, no barrier.  Histogram's sum x (for v) is an xor-shuffle reduction inside the group.
// Same outputs as k_flp_wires, which spends a 64-thread block (4 row groups x 16 columns, LDS
// partials, three barriers, a one-thread tail) on each Histogram(256) report.
// ------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_flp_wires_cols(Cfg cfg, uint32_t n, uint32_t lg, CRows meas,
                                                        CRows proof, WMat wm, CRows jr,
                                                        Rows out_prep, uint8_t* status) {
  using FO = Field128Ops;
  const WRow W(cfg);
  using T = F128;
  constexpr size_t ES = 16;
  const uint32_t G = 1u << lg;
  const uint32_t gt = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t r = gt >> lg, j = gt & (G - 1u);
  const uint32_t rr = r < n ? r : n - 1u;  // dead lanes read a valid row and store nothing
  const bool live = r < n && status[rr] == ST_OK;
  const uint32_t C = cfg.calls, c = cfg.chunk;
  const bool col = live && j < c;
  const uint8_t* xr = meas.at(rr);
  Wide wa, wb;
  wide_zero(wa);
  wide_zero(wb);
  // Histogram's sum x: 32-bit limbs summed into 64-bit words, reduced once after the loop
  uint64_t xs[4] = {0ull, 0ull, 0ull, 0ull};
  // canonical check, one compare per element: only a word 2^32 - 1 on top can make x >= p; the
  // exact test runs after the loop, over this lane's elements, only when some lane saw one
  bool maybe = false;
  for (uint32_t k = 0; k < C; ++k) {
    const uint32_t idx = k * c + j;
    T x = FO::zero();
    if (col && idx < cfg.meas_len) {
      x = FO::load(xr + (size_t)idx * ES);
      maybe |= x.w[3] == 0xFFFFFFFFu;
    }
    const T mm = FO::load(wm.el(rr, W.mm(k))), lm = FO::load(wm.el(rr, W.lm(k)));
    wide_mac(wa, mm, x);
    wide_mac(wb, lm, x);
    if (cfg.kind == KIND_HISTOGRAM) {
#pragma unroll
      for (int q = 0; q < 4; ++q) xs[q] += x.w[q];
    }
  }
  bool bad = false;
  if (__ballot(maybe)) {  // rare (probability ~2^-32 per element): the exact test
    for (uint32_t k = 0; k < C; ++k) {
      const uint32_t idx = k * c + j;
      if (col && idx < cfg.meas_len) bad |= !FO::is_canonical(FO::load(xr + (size_t)idx * ES));
    }
  }
  T xsum = FO::zero();
  if (cfg.kind == KIND_HISTOGRAM) xsum = f128_reduce_limb_sums(xs);
  const T a = wide_reduce(wa), b = wide_reduce(wb);
  uint8_t* outp = out_prep.at(rr);
  if (col) {
    T b0, b1;
    wire_seed_terms(wm, W, rr, proof.at(rr), j, b0, b1, bad);
    const T rp = FO::load(wm.el(rr, W.rp(j)));  // Montgomery
    FO::store(outp + (size_t)(1 + 2 * j) * ES, FO::add(b0, FO::mul(rp, a)));
    FO::store(outp + (size_t)(2 + 2 * j) * ES, FO::add(b1, b));
  }
  if (cfg.kind == KIND_HISTOGRAM) {
    for (uint32_t sft = G >> 1; sft > 0; sft >>= 1) {
      xsum = FO::add(xsum, shfl_xor_T<FO>(xsum, (int)sft));
    }
  }
  const uint64_t bm = __ballot(bad);
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t gmask = (G >= 64u ? ~0ull : ((1ull << G) - 1ull)) << (lane & ~(G - 1u));
  if (!live || j != 0u) return;
  if (cfg.kind == KIND_HISTOGRAM) {
    // v = jr[1] * range + jr[1]^2 * (sum x - 1/2)
    const T gsum = FO::load(wm.el(rr, W.gsum()));
    const T r1m = FO::to_mont(FO::load(jr.at(rr) + ES));
    const T sc = FO::sub(xsum, FO::half());
    FO::store(outp, FO::add(FO::mul(r1m, gsum), FO::mul(FO::mul(r1m, r1m), sc)));
  }
  if (bm & gmask) status[rr] = ST_INVALID_MESSAGE;
}

// ------------------------------------------------------------------------------------------------
// prepare_shares_to_prepare_message (prio): verifier = sum of shares; decide; msg = derive_seed(
// 0^16, dst6, part_0 || part_1).  decide: v == 0 and G(wires) == p(t),
//   G = Mul / ParallelSum(Mul): sum_j w_2j w_2j+1 ;  PolyEval(x^2 - x): w^2 - w.
// ------------------------------------------------------------------------------------------------
template <class FO>
__global__ void __launch_bounds__(256) k_decide(Cfg cfg, uint32_t n, CRows leader_prep,
                                                CRows helper_prep, Rows out_msg, uint8_t* status) {
  // One wave per 64 reports: the wave walks its reports one at a time, reading the two verifier
  // shares coalesced (lane i takes wire pairs i, i + 64, ...) and reducing G across the wave; lane q
  // keeps report q's decision.  Then every lane derives its own report's prep msg (1 Keccak-f).
  using T = typename FO::T;
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t r0 = blockIdx.x * blockDim.x + (threadIdx.x & ~63u);
  if (r0 >= n) return;  // wave-uniform
  const uint32_t nr = n - r0 < 64u ? n - r0 : 64u;
  const size_t ES = FO::ES;
  const uint32_t npairs = cfg.kind == KIND_SUM ? 1u : cfg.arity / 2u;
  bool mine = false;
  if (npairs == 1u) {  // Count / Sum: one gadget evaluation, each lane decides its own report
    const uint32_t rq = r0 + lane;
    if (lane < nr && status[rq] == ST_OK) {
      const uint8_t* a = leader_prep.at(rq);
      const uint8_t* b = helper_prep.at(rq);
      const T x0 = FO::load(a + ES), y0 = FO::load(b + ES);
      bool bad = !FO::is_canonical(x0) || !FO::is_canonical(y0);
      const T w0 = FO::add(x0, y0);
      T g;
      if (cfg.kind == KIND_SUM) {
        g = FO::sub(FO::mul(FO::to_mont(w0), w0), w0);
      } else {
        const T x1 = FO::load(a + 2 * ES), y1 = FO::load(b + 2 * ES);
        bad |= !FO::is_canonical(x1) || !FO::is_canonical(y1);
        g = FO::mul(FO::to_mont(w0), FO::add(x1, y1));
      }
      const T va = FO::load(a), vb = FO::load(b);
      const T pa = FO::load(a + (size_t)(1u + cfg.arity) * ES);
      const T pb = FO::load(b + (size_t)(1u + cfg.arity) * ES);
      bad |= !FO::is_canonical(va) || !FO::is_canonical(vb) || !FO::is_canonical(pa) ||
             !FO::is_canonical(pb);
      mine = !bad && FO::is_zero(FO::add(va, vb)) && FO::eq(g, FO::add(pa, pb));
    }
  }
  // npairs <= 32 (Histogram256: 16): several reports per pass, a power-of-two lane group each,
  // reduced with in-group xor shuffles
  uint32_t G = 1u;
  while (G < npairs) G <<= 1;
  if (npairs > 1u && G < 64u) {
    const uint32_t rpi = 64u / G, sub = lane / G, lj = lane % G;
    for (uint32_t q0 = 0; q0 < nr; q0 += rpi) {
      const uint32_t rq = r0 + q0 + sub;
      const bool on = q0 + sub < nr && status[rq] == ST_OK;
      bool bad = false;
      T g = FO::zero();
      const uint8_t* a = leader_prep.at(on ? rq : r0);
      const uint8_t* b = helper_prep.at(on ? rq : r0);
      if (on && lj < npairs) {
        const uint8_t* pa = a + (size_t)(1u + 2u * lj) * ES;
        const uint8_t* pb = b + (size_t)(1u + 2u * lj) * ES;
        const T x0 = FO::load(pa), x1 = FO::load(pa + ES);
        const T y0 = FO::load(pb), y1 = FO::load(pb + ES);
        bad = !FO::is_canonical(x0) || !FO::is_canonical(x1) || !FO::is_canonical(y0) ||
              !FO::is_canonical(y1);
        g = FO::mul(FO::to_mont(FO::add(x0, y0)), FO::add(x1, y1));
      }
      uint32_t badw = bad ? 1u : 0u;
      for (uint32_t off = G >> 1; off >= 1u; off >>= 1) {
        g = FO::add(g, shfl_xor_T<FO>(g, (int)off));
        badw |= (uint32_t)__shfl_xor((int)badw, (int)off, 64);
      }
      bool ok = false;
      if (on) {
        const T va = FO::load(a), vb = FO::load(b);
        const T pa = FO::load(a + (size_t)(1u + cfg.arity) * ES);
        const T pb = FO::load(b + (size_t)(1u + cfg.arity) * ES);
        const bool bad2 = !FO::is_canonical(va) || !FO::is_canonical(vb) ||
                          !FO::is_canonical(pa) || !FO::is_canonical(pb);
        ok = !badw && !bad2 && FO::is_zero(FO::add(va, vb)) && FO::eq(g, FO::add(pa, pb));
      }
      // report q0 + s's decision sits in every lane of group s: lane q0 + s takes it
      const uint32_t src = lane >= q0 && lane < q0 + rpi ? (lane - q0) * G : 0u;
      const bool got = __shfl((int)ok, (int)src, 64) != 0;
      if (lane >= q0 && lane < q0 + rpi) mine = got;
    }
  }
  for (uint32_t q = 0; q < (npairs == 1u || G < 64u ? 0u : nr); ++q) {
    const uint32_t rq = r0 + q;
    if (__builtin_amdgcn_readfirstlane(status[rq]) != ST_OK) continue;  // wave-uniform
    const uint8_t* a = leader_prep.at(rq);
    const uint8_t* b = helper_prep.at(rq);
    bool bad = false;
    T g = FO::zero();
    for (uint32_t j = lane; j < npairs; j += 64u) {
      if (cfg.kind == KIND_SUM) {  // PolyEval(x^2 - x) on the single wire
        const T x = FO::load(a + ES), y = FO::load(b + ES);
        bad |= !FO::is_canonical(x) || !FO::is_canonical(y);
        const T w = FO::add(x, y);
        g = FO::sub(FO::mul(FO::to_mont(w), w), w);
      } else {  // Mul / ParallelSum(Mul): sum_j w_2j w_2j+1
        const uint8_t* pa = a + (size_t)(1u + 2u * j) * ES;
        const uint8_t* pb = b + (size_t)(1u + 2u * j) * ES;
        const T x0 = FO::load(pa), x1 = FO::load(pa + ES);
        const T y0 = FO::load(pb), y1 = FO::load(pb + ES);
        bad |= !FO::is_canonical(x0) || !FO::is_canonical(x1) || !FO::is_canonical(y0) ||
               !FO::is_canonical(y1);
        g = FO::add(g, FO::mul(FO::to_mont(FO::add(x0, y0)), FO::add(x1, y1)));
      }
    }
    g = wave_sum<FO>(g);
    const T va = FO::load(a), vb = FO::load(b);
    const T pa = FO::load(a + (size_t)(1u + cfg.arity) * ES);
    const T pb = FO::load(b + (size_t)(1u + cfg.arity) * ES);
    bad |= !FO::is_canonical(va) || !FO::is_canonical(vb) || !FO::is_canonical(pa) ||
           !FO::is_canonical(pb);
    const bool ok = !__any(bad) && FO::is_zero(FO::add(va, vb)) && FO::eq(g, FO::add(pa, pb));
    if (lane == q) mine = ok;
  }
  const uint32_t r = r0 + lane;
  if (r >= n || status[r] != ST_OK) return;
  if (!mine) {
    status[r] = ST_VDAF_PREP_ERROR;
    return;
  }
  const uint8_t* a = leader_prep.at(r);
  const uint8_t* b = helper_prep.at(r);
  if (cfg.jr_len > 0) {
    const uint8_t* pa = a + (size_t)cfg.verifier_len * ES;
    const uint8_t* pb = b + (size_t)cfg.verifier_len * ES;
    uint64_t lo, hi;
    derive_jr_seed(cfg.xof, cfg.algo_id, ld64(pa), ld64(pa + 8), ld64(pb), ld64(pb + 8), lo, hi);
    st64(out_msg.at(r), lo);
    st64(out_msg.at(r) + 8, hi);
  }
}

// prepare_next (prio): the prep msg must equal the corrected joint-rand seed.
__global__ void __launch_bounds__(256) k_prepare_next(Cfg cfg, uint32_t n, CRows msgs, CRows seeds,
                                                      uint8_t* status) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  if (status[r] != ST_OK || cfg.jr_len == 0) return;
  const uint8_t* a = msgs.at(r);
  const uint8_t* b = seeds.at(r);
  if (ld64(a) != ld64(b) || ld64(a + 8) != ld64(b + 8)) status[r] = ST_VDAF_PREP_ERROR;
}

// ------------------------------------------------------------------------------------------------
// Output shares and aggregation (prio Type::truncate + Aggregatable::accumulate; Janus
// Accumulator::update accumulator.rs:76-122 / BatchAggregation::merged_with models.rs:962-991).
// ------------------------------------------------------------------------------------------------
template <class FO>
DEVI typename FO::T out_elem(const Cfg& cfg, const uint8_t* x, uint32_t e) {
  using T = typename FO::T;
  if (cfg.kind == KIND_SUMVEC || cfg.kind == KIND_SUM || cfg.kind == KIND_FPVEC) {
    // sum_b 2^b x_b over `bits` consecutive elements, Horner from the top bit
    const uint8_t* p = x + (size_t)e * cfg.bits * FO::ES;
    T acc = FO::zero();
    for (int b = (int)cfg.bits - 1; b >= 0; --b) {
      acc = FO::add(FO::dbl(acc), FO::load(p + (size_t)b * FO::ES));
    }
    return acc;
  }
  return FO::load(x + (size_t)e * FO::ES);
}

// Segmented partial sums of the raw MEASUREMENT-share elements.  truncate() is linear, so
//   sum_r truncate(meas_r) = truncate(sum_r meas_r)
// and the per-report truncation is applied once per chunk sum in k_accum_merge.  Thread e reads
// element e of every report in its chunk: 16 B per lane, consecutive lanes consecutive elements
// (fully coalesced).  chunk c covers perm[chunk_begin[c] .. chunk_begin[c+1]); all reports of a
// chunk share one batch slot.  Block (chunk, tile): EPB elements x G report groups.
template <class FO>
__global__ void __launch_bounds__(256) k_accum_partial(Cfg cfg, CRows meas, const uint32_t* perm,
                                                       const uint32_t* chunk_begin,
                                                       const uint8_t* status, uint32_t epb,
                                                       uint8_t* partials, uint32_t* part_counts,
                                                       const uint32_t* chunk_ids, uint32_t e_head,
                                                       uint32_t e_tail) {
  using T = typename FO::T;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  T* red = reinterpret_cast<T*>(smem);
  const uint32_t ch = chunk_ids ? chunk_ids[blockIdx.x] : blockIdx.x;
  const uint32_t tid = threadIdx.x;
  const uint32_t G = blockDim.x / epb;
  const uint32_t el = tid % epb, g = tid / epb;
  // logical element li -> measurement element: [0, e_head) then [e_tail, meas_len)
  const uint32_t li = blockIdx.y * epb + el;
  const uint32_t e = li < e_head ? li : e_tail + (li - e_head);
  const uint32_t b0 = chunk_begin[ch], b1 = chunk_begin[ch + 1];
  T acc = FO::zero();
  if (g < G && e < cfg.meas_len) {
    const size_t off = (size_t)e * FO::ES;
    uint32_t i = b0 + g;
    // 4 independent loads in flight per thread
    for (; i + 3 * G < b1; i += 4 * G) {
      const uint32_t r0 = perm[i], r1 = perm[i + G], r2 = perm[i + 2 * G], r3 = perm[i + 3 * G];
      const T x0 = FO::load(meas.at(r0) + off), x1 = FO::load(meas.at(r1) + off);
      const T x2 = FO::load(meas.at(r2) + off), x3 = FO::load(meas.at(r3) + off);
      if (status[r0] == ST_OK) acc = FO::add(acc, x0);
      if (status[r1] == ST_OK) acc = FO::add(acc, x1);
      if (status[r2] == ST_OK) acc = FO::add(acc, x2);
      if (status[r3] == ST_OK) acc = FO::add(acc, x3);
    }
    for (; i < b1; i += G) {
      const uint32_t r = perm[i];
      const T x = FO::load(meas.at(r) + off);
      if (status[r] == ST_OK) acc = FO::add(acc, x);
    }
  }
  if (G > 1) {
    red[tid] = acc;
    __syncthreads();
    if (g == 0) {
      for (uint32_t q = 1; q < G; ++q) acc = FO::add(acc, red[q * epb + el]);
    }
  }
  if (g == 0 && e < cfg.meas_len)
    FO::store(partials + ((size_t)ch * cfg.meas_len + e) * FO::ES, acc);
  if (blockIdx.y == 0) {  // accepted-report count of this chunk (LDS word after `red`)
    uint32_t* rc = reinterpret_cast<uint32_t*>(smem + 256 * sizeof(T));
    if (tid == 0) *rc = 0;
    __syncthreads();
    uint32_t cnt = 0;
    for (uint32_t i = b0 + tid; i < b1; i += blockDim.x) cnt += (status[perm[i]] == ST_OK);
    if (cnt) atomicAdd(rc, cnt);
    __syncthreads();
    if (tid == 0) part_counts[ch] = *rc;
  }
}

// Speculative chunks: the measurement-share words [2 e0, 2 e1) were column-summed per wave by
// k_jr (spec_lo/spec_cy).  Sum them over the chunk's waves, subtract the rows that did not end
// with status OK (and the clamped rows past n), and fold the two 64-bit word sums of element e into
// one canonical element:  x = A + 2^64 B,  2^128 = 28 2^64 - 1 (mod p).  Thread pair (2t, 2t+1)
// = the two words of element e0 + 128 blockIdx.y + t.
template <class FO>
__global__ void __launch_bounds__(256) k_accum_spec(Cfg cfg, uint32_t n, CRows meas,
                                                    const uint32_t* chunk_ids,
                                                    const uint32_t* chunk_wbegin,
                                                    const uint32_t* waves, const uint64_t* spec_lo,
                                                    const uint8_t* spec_cy, uint32_t nd,
                                                    uint32_t e0, uint32_t e1,
                                                    const uint8_t* status, uint8_t* partials) {
  typedef unsigned __int128 u128;
  const uint32_t ch = chunk_ids[blockIdx.x];
  const uint32_t tid = threadIdx.x, lane = tid & 63u;
  const uint32_t e = e0 + blockIdx.y * 128u + (tid >> 1);
  const uint32_t wd = 2u * e + (tid & 1u);
  const bool act = e < e1;
  u128 acc = 0;
  const uint32_t wb = chunk_wbegin[blockIdx.x], we = chunk_wbegin[blockIdx.x + 1];
  for (uint32_t q = wb; q < we; ++q) {
    const uint32_t w = waves[q];
    if (act) {
      const size_t at = (size_t)w * nd + wd;
      acc += (u128)spec_lo[at] + ((u128)spec_cy[at] << 64);
    }
    const uint32_t r = w * 64u + lane;
    const bool fail = (r >= n) || status[r] != ST_OK;
    uint64_t mask = __ballot(fail);
    while (mask) {
      const uint32_t i = (uint32_t)__builtin_ctzll(mask);
      mask &= mask - 1ull;
      const uint32_t rr = w * 64u + i < n ? w * 64u + i : n - 1u;
      if (act) acc -= (u128)ld64(meas.at(rr) + (size_t)wd * 8u);
    }
  }
  const uint64_t alo = (uint64_t)acc, ahi = (uint64_t)(acc >> 64);
  const uint64_t blo = __shfl_xor(alo, 1, 64), bhi = __shfl_xor(ahi, 1, 64);
  if (act && (tid & 1u) == 0u) {
    // value = alo + 2^64 (ahi + blo) + 2^128 bhi
    const u128 P = ((u128)0xFFFFFFFFFFFFFFFFull << 64) - ((u128)27ull << 64) + 1;  // 2^128-28*2^64+1
    const u128 x1 = (u128)ahi + blo;                  // < 2^65
    const u128 x2 = (u128)bhi + (uint64_t)(x1 >> 64);  // small
    const u128 v = ((u128)(uint64_t)x1 << 64) | alo;   // < 2^128
    const u128 k = (u128)(uint64_t)x2 * 28u;           // 2^128 x2 = x2 (28 2^64 - 1)
    u128 t = v + (k << 64);
    if (t < v) t += ((u128)28u << 64) - 1;              // carry out of 2^128
    t -= (uint64_t)x2;                                  // no underflow: k << 64 >= x2
    while (t >= P) t -= P;
    uint8_t* dst = partials + ((size_t)ch * cfg.meas_len + e) * 16u;
    st64(dst, (uint64_t)t);
    st64(dst + 8, (uint64_t)(t >> 64));
  }
}

// agg[slot(c)] += truncate(sum of partial[c]) for every slot run of chunks (chunks of one slot
// are contiguous), in chunk order (deterministic).  Block = 256 threads over `bpe`-element groups
// (bpe = bits for Sum/SumVec, 1 otherwise): each thread sums one measurement element over the run,
// then one thread per output element applies truncate (sum_b 2^b x_b) and adds into agg.
template <class FO>
__global__ void __launch_bounds__(256) k_accum_merge(Cfg cfg, uint32_t nchunks,
                                                     const uint32_t* chunk_slot,
                                                     const uint8_t* partials,
                                                     const uint32_t* part_counts, uint8_t* agg,
                                                     unsigned long long* counts) {
  using T = typename FO::T;
  __shared__ T part[256];
  __shared__ T tot[256];
  const uint32_t bpe =
      (cfg.kind == KIND_SUMVEC || cfg.kind == KIND_SUM || cfg.kind == KIND_FPVEC) ? cfg.bits : 1u;
  const uint32_t opb = 256 / bpe;  // output elements per block
  const uint32_t o0 = blockIdx.x * opb;
  const uint32_t nout = min(opb, cfg.out_len - o0);
  // ne measurement elements in this block; when they leave threads idle (Count, Sum: one output)
  // L threads share an element, each summing every L-th chunk of a run, then an LDS fold
  const uint32_t ne = nout * bpe;
  const uint32_t L = 256 / ne;
  const uint32_t tid = threadIdx.x;
  const uint32_t el = tid % ne, g = tid / ne;
  const bool act = g < L;
  const uint32_t o = o0 + el / bpe, b = el % bpe;
  const uint32_t e = o * bpe + b;
  uint32_t c = 0;
  while (c < nchunks) {
    const uint32_t slot = chunk_slot[c];
    // end of this slot's run: a slot's chunks are contiguous, so "== slot" holds exactly on
    // [c, c1) of [c, nchunks) and a binary search finds c1
    uint32_t lo = c + 1, hi = nchunks;
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (chunk_slot[mid] == slot) lo = mid + 1;
      else hi = mid;
    }
    const uint32_t c1 = lo;
    T acc = FO::zero();
    if (act) {
#pragma unroll 4
      for (uint32_t q = c + g; q < c1; q += L)
        acc = FO::add(acc, FO::load(partials + ((size_t)q * cfg.meas_len + e) * FO::ES));
    }
    part[tid] = acc;
    __syncthreads();
    if (g == 0) {
      for (uint32_t gg = 1; gg < L; ++gg) acc = FO::add(acc, part[gg * ne + el]);
      tot[el] = acc;
    }
    __syncthreads();
    if (g == 0 && b == 0) {
      T t = FO::zero();
      for (int k = (int)bpe - 1; k >= 0; --k) t = FO::add(FO::dbl(t), tot[el + k]);
      uint8_t* dst = agg + ((size_t)slot * cfg.out_len + o) * FO::ES;
      FO::store(dst, FO::add(FO::load(dst), t));
    }
    __syncthreads();
    c = c1;
  }
  if (blockIdx.x == 0) {  // report counts: integer adds, order-free
    for (uint32_t q = tid; q < nchunks; q += blockDim.x)
      if (part_counts[q]) atomicAdd(&counts[chunk_slot[q]], (unsigned long long)part_counts[q]);
  }
}

// Per-report output shares (optional debugging/parity output of prepare_next).
template <class FO>
__global__ void __launch_bounds__(256) k_out_shares(Cfg cfg, uint32_t n, CRows meas,
                                                    Rows out, const uint8_t* status) {
  const uint32_t r = blockIdx.y;
  const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n || e >= cfg.out_len) return;
  typename FO::T v = FO::zero();
  if (status[r] == ST_OK) v = out_elem<FO>(cfg, meas.at(r), e);
  FO::store(out.at(r) + (size_t)e * FO::ES, v);
}

// dst[i] += src[i] (mod p) over `nelems` field elements (RCCL all-gather merge, K6).
// ------------------------------------------------------------------------------------------------
// Accumulator::update's report bookkeeping (aggregator/src/aggregator/accumulator.rs:76-122):
// per batch slot, checksum ^= SHA-256(report_id) (ReportIdChecksum::updated_with,
// core/src/report_id.rs:18-44) and client_timestamp_interval merged with [time, time + 1)
// (Interval::merged_with / from_time, core/src/time.rs:289-312).  Slot meta = 8 checksum words
// (SHA-256 state words) + u64 min time + u64 max time.  A wave whose live reports share one slot
// (the common case) reduces with shuffles and issues one set of atomics.
// ------------------------------------------------------------------------------------------------
struct SlotMeta {
  uint32_t ck[8];
  unsigned long long tmin, tmax;
};

__constant__ uint32_t kSha256K[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

DEVI uint32_t rotr32(uint32_t x, uint32_t n) { return __builtin_amdgcn_alignbit(x, x, n); }
DEVI uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

// SHA-256 of a 16-byte message (one padded block): h = digest as 8 big-endian state words.
DEVI void sha256_16(const uint8_t* m, uint32_t h[8]) {
  uint32_t w[16];
#pragma unroll
  for (int i = 0; i < 4; ++i) w[i] = bswap32(*reinterpret_cast<const uint32_t*>(m + 4 * i));
  w[4] = 0x80000000u;
#pragma unroll
  for (int i = 5; i < 15; ++i) w[i] = 0u;
  w[15] = 128u;  // message length in bits
  const uint32_t iv[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                          0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  uint32_t a = iv[0], b = iv[1], c = iv[2], d = iv[3], e = iv[4], f = iv[5], g = iv[6], hh = iv[7];
#pragma unroll
  for (int t = 0; t < 64; ++t) {
    uint32_t wt;
    if (t < 16) {
      wt = w[t];
    } else {
      const uint32_t w15 = w[(t + 1) & 15], w2 = w[(t + 14) & 15];
      const uint32_t s0 = rotr32(w15, 7) ^ rotr32(w15, 18) ^ (w15 >> 3);
      const uint32_t s1 = rotr32(w2, 17) ^ rotr32(w2, 19) ^ (w2 >> 10);
      wt = w[t & 15] = w[t & 15] + s0 + w[(t + 9) & 15] + s1;
    }
    const uint32_t S1 = rotr32(e, 6) ^ rotr32(e, 11) ^ rotr32(e, 25);
    const uint32_t ch = (e & f) ^ (~e & g);
    const uint32_t t1 = hh + S1 + ch + kSha256K[t] + wt;
    const uint32_t S0 = rotr32(a, 2) ^ rotr32(a, 13) ^ rotr32(a, 22);
    const uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
    const uint32_t t2 = S0 + mj;
    hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  h[0] = iv[0] + a; h[1] = iv[1] + b; h[2] = iv[2] + c; h[3] = iv[3] + d;
  h[4] = iv[4] + e; h[5] = iv[5] + f; h[6] = iv[6] + g; h[7] = iv[7] + hh;
}

struct WaveMeta {
  SlotMeta m;
  uint32_t slot;  // 0xFFFFFFFF: no partial (empty or mixed-slot wave)
  uint32_t pad[3];
};

__global__ void __launch_bounds__(256) k_report_meta(uint32_t n, CRows ids, const uint64_t* times,
                                                     const uint8_t* status, const uint32_t* slots,
                                                     uint32_t nslots, SlotMeta* meta,
                                                     WaveMeta* partial) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  const bool ok = r < n && (!status || status[r] == ST_OK) && (!slots || slots[r] < nslots);
  const unsigned long long act = __ballot(ok);
  if (act == 0ull) {  // wave-uniform
    if ((threadIdx.x & 63u) == 0u) partial[r >> 6].slot = 0xFFFFFFFFu;
    return;
  }
  uint32_t h[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long t = ok ? times[r] : 0ull;
  uint32_t slot = 0;
  if (ok) {
    sha256_16(ids.at(r), h);
    slot = slots ? slots[r] : 0u;
  }
  const int lead = __ffsll(act) - 1;
  const uint32_t s0 = __shfl(slot, lead, 64);
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (__ballot(ok && slot != s0) == 0ull) {
    unsigned long long tmin = ok ? t : ~0ull, tmax = t;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
#pragma unroll
      for (int i = 0; i < 8; ++i) h[i] ^= __shfl_xor(h[i], off, 64);
      const unsigned long long a = __shfl_xor(tmin, off, 64), b = __shfl_xor(tmax, off, 64);
      tmin = a < tmin ? a : tmin;
      tmax = b > tmax ? b : tmax;
    }
    // one partial per wave; k_report_meta_fold folds them per slot (atomics on one slot's
    // words from every wave would serialise in L2)
    if ((int)(threadIdx.x & 63u) == lead) {
      WaveMeta& pw = partial[wave];
#pragma unroll
      for (int i = 0; i < 8; ++i) pw.m.ck[i] = h[i];
      pw.m.tmin = tmin;
      pw.m.tmax = tmax;
      pw.slot = s0;
    }
    return;
  }
  if ((threadIdx.x & 63u) == 0u) partial[wave].slot = 0xFFFFFFFFu;  // mixed slots: direct atomics
  if (ok) {
#pragma unroll
    for (int i = 0; i < 8; ++i) atomicXor(&meta[slot].ck[i], h[i]);
    atomicMin(&meta[slot].tmin, t);
    atomicMax(&meta[slot].tmax, t);
  }
}

// Fold the per-wave partials of k_report_meta: block per slot, one set of atomics per slot.
__global__ void __launch_bounds__(256) k_report_meta_fold(uint32_t nwaves, const WaveMeta* partial,
                                                          SlotMeta* meta) {
  const uint32_t slot = blockIdx.x;
  uint32_t h[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long tmin = ~0ull, tmax = 0ull;
  for (uint32_t w = blockIdx.y * blockDim.x + threadIdx.x; w < nwaves;
       w += blockDim.x * gridDim.y) {
    const WaveMeta& p = partial[w];
    if (p.slot != slot) continue;
#pragma unroll
    for (int i = 0; i < 8; ++i) h[i] ^= p.m.ck[i];
    tmin = p.m.tmin < tmin ? p.m.tmin : tmin;
    tmax = p.m.tmax > tmax ? p.m.tmax : tmax;
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
#pragma unroll
    for (int i = 0; i < 8; ++i) h[i] ^= __shfl_xor(h[i], off, 64);
    const unsigned long long a = __shfl_xor(tmin, off, 64), b = __shfl_xor(tmax, off, 64);
    tmin = a < tmin ? a : tmin;
    tmax = b > tmax ? b : tmax;
  }
  if ((threadIdx.x & 63u) == 0u && tmin <= tmax) {
#pragma unroll
    for (int i = 0; i < 8; ++i) atomicXor(&meta[slot].ck[i], h[i]);
    atomicMin(&meta[slot].tmin, tmin);
    atomicMax(&meta[slot].tmax, tmax);
  }
}

template <class FO>
__global__ void __launch_bounds__(256) k_merge(uint8_t* dst, const uint8_t* src, size_t nelems) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nelems) return;
  FO::store(dst + i * FO::ES, FO::add(FO::load(dst + i * FO::ES), FO::load(src + i * FO::ES)));
}

// The RCCL flush in one launch (prio3gpu_agg_allreduce): blocks [0, nb) grid-stride over the
// nelems aggregate elements, dst[i] = (accumulate ? dst[i] : 0) + sum over ranks r of
// gathered[r * nelems + i] in rank order; block nb folds the slots: counts (already summed by
// RCCL) and the all-gathered slot meta, checksum XOR + interval union per slot
// (BatchAggregation::merged_with, aggregator_core/src/datastore/models.rs:962-991).
template <class FO>
__global__ void __launch_bounds__(256) k_merge_ranks(uint8_t* dst, const uint8_t* gathered,
                                                     size_t nelems, uint32_t nranks,
                                                     uint32_t accumulate,
                                                     unsigned long long* counts,
                                                     const unsigned long long* count_sums,
                                                     SlotMeta* meta, const SlotMeta* gmeta,
                                                     uint32_t nslots, uint32_t nb) {
  if (blockIdx.x < nb) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < nelems;
         i += (size_t)nb * blockDim.x) {
      typename FO::T acc = accumulate ? FO::load(dst + i * FO::ES) : FO::zero();
      for (uint32_t r = 0; r < nranks; ++r)
        acc = FO::add(acc, FO::load(gathered + ((size_t)r * nelems + i) * FO::ES));
      FO::store(dst + i * FO::ES, acc);
    }
    return;
  }
  for (uint32_t s = threadIdx.x; s < nslots; s += blockDim.x) {
    counts[s] = (accumulate ? counts[s] : 0ull) + count_sums[s];
    SlotMeta m;
    if (accumulate) {
      m = meta[s];
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) m.ck[i] = 0u;
      m.tmin = ~0ull;
      m.tmax = 0ull;
    }
    for (uint32_t r = 0; r < nranks; ++r) {
      const SlotMeta& x = gmeta[(size_t)r * nslots + s];
#pragma unroll
      for (int i = 0; i < 8; ++i) m.ck[i] ^= x.ck[i];
      m.tmin = x.tmin < m.tmin ? x.tmin : m.tmin;  // an empty interval is tmin > tmax
      m.tmax = x.tmax > m.tmax ? x.tmax : m.tmax;
    }
    meta[s] = m;
  }
}

// Epoch merge staging (prio3gpu_agg_epoch_merge): local slot s (blockIdx.y) is copied to the
// union table's slot map[s] -- share row (8-byte words), count, slot meta -- of a staging
// aggregate that starts empty; union slots no local slot maps to stay empty.
__global__ void __launch_bounds__(256) k_agg_scatter(uint64_t* dst_share,
                                                     unsigned long long* dst_counts,
                                                     SlotMeta* dst_meta, const uint64_t* src_share,
                                                     const unsigned long long* src_counts,
                                                     const SlotMeta* src_meta, const uint32_t* map,
                                                     size_t row_words) {
  const uint32_t s = blockIdx.y, d = map[s];
  if (d == 0xFFFFFFFFu) return;  // PRIO3GPU_SLOT_UNUSED: a pooled slot no job of the epoch used
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < row_words;
       i += (size_t)gridDim.x * blockDim.x)
    dst_share[(size_t)d * row_words + i] = src_share[(size_t)s * row_words + i];
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    dst_counts[d] = src_counts[s];
    dst_meta[d] = src_meta[s];
  }
}

__global__ void __launch_bounds__(256) k_meta_reset(SlotMeta* meta, uint32_t nslots) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nslots) return;
#pragma unroll
  for (int i = 0; i < 8; ++i) meta[s].ck[i] = 0u;
  meta[s].tmin = ~0ull;
  meta[s].tmax = 0ull;
}

}  // namespace p3g

namespace p3g {

// =================================================================================================
// Client: batched Prio3 shard + FLP prove (prio 0.15.1 Prio3::shard_with_random,
// flp.rs Type::prove).  Used to generate inputs at scale; the aggregator path does not depend on it.
// =================================================================================================

// Encoded measurement element i (0/1 for every type here) from the raw measurement row
// (SumVec: `length` u64 entries, others: one u64).  prio Type::encode_measurement.
// Bit i of the encoded measurement.  FixedPointBoundedL2VecSum (prio fixedpoint_l2.rs encode):
// entry e contributes the n bits of z_e = v_e + 2^(n-1) (v_e the raw two's-complement fixed-point
// value), then the 2n-2 bits of the squared norm sum_e v_e^2 (`norm`: two LE u64 words).
DEVI uint32_t enc_meas_bit(const Cfg& cfg, const uint64_t* m, uint32_t i,
                           const uint64_t* norm = nullptr) {
  switch (cfg.kind) {
    case KIND_COUNT: return (uint32_t)(m[0] & 1u);
    case KIND_SUM: return (uint32_t)((m[0] >> i) & 1u);
    case KIND_SUMVEC: return (uint32_t)((m[i / cfg.bits] >> (i % cfg.bits)) & 1u);
    case KIND_FPVEC: {
      const uint32_t nb = cfg.bits, ent = i / nb;
      if (ent < cfg.length) {
        const uint64_t z = m[ent] + (1ull << (nb - 1));
        return (uint32_t)((z >> (i - ent * nb)) & 1u);
      }
      const uint32_t b = i - cfg.length * nb;  // norm bit
      return (uint32_t)((norm[b >> 6] >> (b & 63u)) & 1u);
    }
    default: return m[0] == i ? 1u : 0u;  // Histogram one-hot
  }
}

// FixedPointBoundedL2VecSum client: squared L2 norm sum_e v_e^2 of each measurement (u128, two LE
// words; the caller's entries satisfy the norm bound < 2^(2n-2), which prio's shard checks).
// Block per report.
__global__ void __launch_bounds__(256) k_shard_norm(Cfg cfg, uint32_t n, const uint64_t* meas,
                                                    uint64_t* norms) {
  typedef unsigned __int128 u128;
  __shared__ uint64_t red[2 * 256];
  const uint32_t r = blockIdx.x;
  if (r >= n) return;
  const int64_t* mr = reinterpret_cast<const int64_t*>(meas) + (size_t)r * cfg.length;
  u128 acc = 0;
  for (uint32_t e = threadIdx.x; e < cfg.length; e += blockDim.x) {
    const int64_t v = mr[e];
    const uint64_t a = v < 0 ? (uint64_t)0 - (uint64_t)v : (uint64_t)v;
    acc += (u128)a * a;
  }
  red[2 * threadIdx.x] = (uint64_t)acc;
  red[2 * threadIdx.x + 1] = (uint64_t)(acc >> 64);
  __syncthreads();
  for (uint32_t sft = blockDim.x / 2; sft > 0; sft >>= 1) {
    if (threadIdx.x < sft) {
      const u128 a = ((u128)red[2 * threadIdx.x + 1] << 64) | red[2 * threadIdx.x];
      const u128 b = ((u128)red[2 * (threadIdx.x + sft) + 1] << 64) | red[2 * (threadIdx.x + sft)];
      const u128 c = a + b;
      red[2 * threadIdx.x] = (uint64_t)c;
      red[2 * threadIdx.x + 1] = (uint64_t)(c >> 64);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    norms[2 * r] = red[0];
    norms[2 * r + 1] = red[1];
  }
}

// Radix-2 DIT NTT of size n over up to two LDS arrays (inputs bit-reversed), twiddles
// omega_N^(k*stride) from a table of N-th roots (Montgomery).  All threads call.
template <class FO>
DEVI void ntt_lds(typename FO::T* A, typename FO::T* B, uint32_t n, uint32_t logn,
                  const uint8_t* tw, uint32_t stride, uint32_t tid, uint32_t nthr) {
  const uint32_t na = B ? 2u : 1u;
  for (uint32_t st = 1; st <= logn; ++st) {
    const uint32_t half = 1u << (st - 1);
    for (uint32_t q = tid; q < na * (n >> 1); q += nthr) {
      typename FO::T* a = q < (n >> 1) ? A : B;
      const uint32_t bq = q & ((n >> 1) - 1u);
      const uint32_t grp = bq >> (st - 1), k = bq & (half - 1u);
      const uint32_t i = grp * 2u * half + k, j = i + half;
      const typename FO::T w = FO::load(tw + (size_t)((k << (logn - st)) * stride) * FO::ES);
      const typename FO::T u = a[i];
      const typename FO::T v = FO::mul(w, a[j]);
      a[i] = FO::add(u, v);
      a[j] = FO::sub(u, v);
    }
    __syncthreads();
  }
}

// FLP prove, one block per report.  Everything in Montgomery form until the final conversion.
// Wire polys interpolate f_{w,k} (k = 0: prove rand seed; 1..calls: recorded gadget inputs with
// num_shares = 1; zero above).  The gadget poly G(f_0..f_{arity-1}) has degree 2(m-1): its values
// at the 2m-th roots are, at even points, G of the recorded values and, at odd points w*alpha^k,
// G of the wire polys' values there (iNTT -> twist by w^d / m -> NTT).  Interpolating those 2m
// values gives the 2m-1 proof coefficients.
// tw2 = [w^0 .. w^(2m-1), 1/m, 1/(2m)] (w = primitive 2m-th root), Montgomery.
// LDS: FA[m] FB[m] GA[m] GB[m] PE[m] PO[m] RP[c+1] RR[calls+1]; G[2m] reuses FA..GB at the end.
// FixedPointBoundedL2VecSum: gadget 0 is the ParallelSum(Mul) range check above (chunk c0 over
// the entry and norm bits); gadget 1, ParallelSum(PolyEval(x^2 - 2^n x + 2^(2n-2)), c1) =
// sum_j (w_j - 2^(n-1))^2 over the decoded entries z_e (padding 2^(n-1) = the encoded zero, with
// num_shares = 1), follows in the same block with m1 | m, its roots taken from tw2 at stride m/m1.
template <class FO>
__global__ void __launch_bounds__(256) k_flp_prove(Cfg cfg, uint32_t n, const uint8_t* tw2,
                                                   const uint64_t* meas, uint32_t meas_words,
                                                   CRows prove_rand, CRows jr, Rows proof_out,
                                                   const uint64_t* norms) {
  using T = typename FO::T;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t r = blockIdx.x;
  if (r >= n) return;
  const uint32_t tid = threadIdx.x, nthr = blockDim.x;
  const uint32_t m = cfg.m, logm = cfg.logm, calls = cfg.calls;
  const bool psum =
      (cfg.kind == KIND_SUMVEC || cfg.kind == KIND_HISTOGRAM || cfg.kind == KIND_FPVEC);
  const uint32_t c = psum ? cfg.chunk : 1u;
  T* FA = reinterpret_cast<T*>(smem);
  T* FB = FA + m;
  T* GA = FB + m;
  T* GB = GA + m;
  T* PE = GB + m;
  T* PO = PE + m;
  T* G = FA;  // after the wire loop
  T* RP = PO + m;
  T* RR = RP + (c + 1);
  const uint64_t* mrow = meas + (size_t)r * meas_words;
  const uint64_t* nrm = norms ? norms + 2 * (size_t)r : nullptr;
  const uint8_t* pr = prove_rand.at(r);
  const T one = FO::one_mont();
  const T inv_m = FO::load(tw2 + (size_t)(2 * m) * FO::ES);
  const T inv_2m = FO::load(tw2 + (size_t)(2 * m + 1) * FO::ES);
  // r powers for the a-wires (ParallelSum types): RP[i] = r^i (i <= c), RR[q] = (r^c)^q
  {
    const uint32_t wave = tid >> 6, lane = tid & 63;
    T rm = one;
    if (psum) rm = FO::to_mont(FO::load(jr.at(r)));
    if (psum && wave == 0) wave_pow_table<FO>(RP, rm, c + 1, lane);
    if (psum && wave == (nthr > 64 ? 1u : 0u)) {
      const T rc = mont_pow<FO>(rm, c);
      wave_pow_table<FO>(RR, rc, calls, lane);
    }
  }
  for (uint32_t k = tid; k < m; k += nthr) {
    PE[k] = FO::zero();
    PO[k] = FO::zero();
  }
  __syncthreads();
  const uint32_t npairs = psum ? c : 1u;  // Sum: one wire; Count: one (x, x) pair
  for (uint32_t j = 0; j < npairs; ++j) {
    // wire values at alpha^k, written bit-reversed for the interpolating NTT
    for (uint32_t k = tid; k < m; k += nthr) {
      T a = FO::zero(), b = FO::zero();
      if (k == 0) {
        if (cfg.kind == KIND_SUM) {
          a = FO::to_mont(FO::load(pr));
        } else {
          a = FO::to_mont(FO::load(pr + (size_t)(2 * j) * FO::ES));
          b = FO::to_mont(FO::load(pr + (size_t)(2 * j + 1) * FO::ES));
        }
      } else if (k <= calls) {
        if (psum) {
          const uint32_t idx = (k - 1) * c + j;
          if (idx < cfg.meas_len) {
            const uint32_t x = enc_meas_bit(cfg, mrow, idx, nrm);
            a = x ? FO::mul(RP[j + 1], RR[k - 1]) : FO::zero();  // r^(idx+1) x
            b = x ? FO::zero() : FO::neg(one);                  // x - 1
          } else {
            b = FO::neg(one);  // padding (0, -1/num_shares), num_shares = 1
          }
        } else if (cfg.kind == KIND_SUM) {
          a = enc_meas_bit(cfg, mrow, k - 1) ? one : FO::zero();
        } else {  // Count: Mul(x, x)
          a = enc_meas_bit(cfg, mrow, 0) ? one : FO::zero();
          b = a;
        }
      }
      // even gadget values
      if (cfg.kind == KIND_SUM) PE[k] = FO::add(PE[k], FO::sub(FO::mul(a, a), a));
      else PE[k] = FO::add(PE[k], FO::mul(a, b));
      const uint32_t br = bitrev(k, logm);
      FA[br] = a;
      FB[br] = b;
    }
    __syncthreads();
    ntt_lds<FO>(FA, cfg.kind == KIND_SUM ? nullptr : FB, m, logm, tw2, 2, tid, nthr);
    // coefficients c_d = X[(m-d) mod m] / m ; twist by w^d ; bit-reverse for the next NTT
    for (uint32_t d = tid; d < m; d += nthr) {
      const uint32_t src = (m - d) & (m - 1);
      const T s = FO::mul(FO::load(tw2 + (size_t)d * FO::ES), inv_m);
      const uint32_t br = bitrev(d, logm);
      GA[br] = FO::mul(FA[src], s);
      if (cfg.kind != KIND_SUM) GB[br] = FO::mul(FB[src], s);
    }
    __syncthreads();
    ntt_lds<FO>(GA, cfg.kind == KIND_SUM ? nullptr : GB, m, logm, tw2, 2, tid, nthr);
    for (uint32_t k = tid; k < m; k += nthr) {
      const T a = GA[k];
      if (cfg.kind == KIND_SUM) PO[k] = FO::add(PO[k], FO::sub(FO::mul(a, a), a));
      else PO[k] = FO::add(PO[k], FO::mul(a, GB[k]));
    }
    __syncthreads();
  }
  // interpolate the gadget poly from its 2m values: G[2k] = PE[k], G[2k+1] = PO[k]
  const uint32_t logm2 = logm + 1, m2 = 2 * m;
  for (uint32_t i = tid; i < m2; i += nthr) G[bitrev(i, logm2)] = (i & 1) ? PO[i >> 1] : PE[i >> 1];
  __syncthreads();
  ntt_lds<FO>(G, nullptr, m2, logm2, tw2, 1, tid, nthr);
  uint8_t* out = proof_out.at(r);
  const uint32_t arity = cfg.arity;
  for (uint32_t d = tid; d < cfg.gp_len; d += nthr) {
    const T v = FO::mul(G[(m2 - d) & (m2 - 1)], inv_2m);
    FO::store(out + (size_t)(arity + d) * FO::ES, FO::from_mont(v));
  }
  for (uint32_t w = tid; w < arity; w += nthr)
    FO::store(out + (size_t)w * FO::ES, FO::load(pr + (size_t)w * FO::ES));
  if constexpr (FO::ES == 16) {
  if (cfg.kind != KIND_FPVEC) return;

  // ---- gadget 1 (FixedPointBoundedL2VecSum): sum_j (w_j - 2^(n-1))^2, m1 | m ----
  __syncthreads();
  const uint32_t m1 = cfg.m1, logm1 = cfg.logm1, calls1 = cfg.calls1, c1 = cfg.chunk1;
  const uint32_t q = m / m1;  // tw2 stride for the 2*m1-th roots is q, for the m1-th roots 2q
  const T qm = FO::to_mont(FO::from_u32(q));
  const T inv_m1 = FO::mul(inv_m, qm), inv_2m1 = FO::mul(inv_2m, qm);
  const uint32_t nb = cfg.bits;
  const T half_one = FO::to_mont(FO::from_u64x2(1ull << (nb - 1), 0ull));  // 2^(n-1)
  for (uint32_t k = tid; k < m1; k += nthr) {
    PE[k] = FO::zero();
    PO[k] = FO::zero();
  }
  __syncthreads();
  const uint8_t* pr1 = pr + (size_t)arity * FO::ES;  // gadget-1 wire seeds
  for (uint32_t j = 0; j < c1; ++j) {
    for (uint32_t k = tid; k < m1; k += nthr) {
      T a = FO::zero();
      if (k == 0) {
        a = FO::to_mont(FO::load(pr1 + (size_t)j * FO::ES));
      } else if (k <= calls1) {
        const uint32_t e = (k - 1) * c1 + j;
        a = e < cfg.length ? FO::to_mont(FO::from_u64x2(mrow[e] + (1ull << (nb - 1)), 0ull))
                           : half_one;
      }
      const T d = FO::sub(a, half_one);
      PE[k] = FO::add(PE[k], FO::mul(d, d));
      FA[bitrev(k, logm1)] = a;
    }
    __syncthreads();
    ntt_lds<FO>(FA, nullptr, m1, logm1, tw2, 2 * q, tid, nthr);
    for (uint32_t d = tid; d < m1; d += nthr) {
      const uint32_t src = (m1 - d) & (m1 - 1);
      const T s = FO::mul(FO::load(tw2 + (size_t)(d * q) * FO::ES), inv_m1);
      GA[bitrev(d, logm1)] = FO::mul(FA[src], s);
    }
    __syncthreads();
    ntt_lds<FO>(GA, nullptr, m1, logm1, tw2, 2 * q, tid, nthr);
    for (uint32_t k = tid; k < m1; k += nthr) {
      const T dd = FO::sub(GA[k], half_one);
      PO[k] = FO::add(PO[k], FO::mul(dd, dd));
    }
    __syncthreads();
  }
  const uint32_t m12 = 2 * m1, logm12 = logm1 + 1;
  for (uint32_t i = tid; i < m12; i += nthr)
    G[bitrev(i, logm12)] = (i & 1) ? PO[i >> 1] : PE[i >> 1];
  __syncthreads();
  ntt_lds<FO>(G, nullptr, m12, logm12, tw2, q, tid, nthr);
  uint8_t* out1 = out + (size_t)(arity + cfg.gp_len) * FO::ES;
  for (uint32_t d = tid; d < cfg.gp_len1; d += nthr) {
    const T v = FO::mul(G[(m12 - d) & (m12 - 1)], inv_2m1);
    FO::store(out1 + (size_t)(c1 + d) * FO::ES, FO::from_mont(v));
  }
  for (uint32_t w = tid; w < c1; w += nthr)
    FO::store(out1 + (size_t)w * FO::ES, FO::load(pr1 + (size_t)w * FO::ES));
  }
}

// Shard helpers (lane per report).  rand row = [k_meas, k_proof, (blind_h, blind_l,) k_prove].
// helper share = [k_meas, k_proof, (blind_h)], leader share tail = blind_l.
__global__ void __launch_bounds__(256) k_shard_seeds(Cfg cfg, uint32_t n, CRows rand,
                                                     Rows helper, Rows leader) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  const uint8_t* rd = rand.at(r);
  uint8_t* h = helper.at(r);
  for (int i = 0; i < 4; ++i) st64(h + 8 * i, ld64(rd + 8 * i));
  if (cfg.jr_len) {
    st64(h + 32, ld64(rd + 32));
    st64(h + 40, ld64(rd + 40));
    uint8_t* l = leader.at(r) + (size_t)(cfg.meas_len + cfg.proof_len) * cfg.es;
    st64(l, ld64(rd + 48));
    st64(l + 8, ld64(rd + 56));
  }
}

// leader meas share = encode(measurement) - helper meas share   (elementwise; thread per element)
template <class FO>
__global__ void __launch_bounds__(256) k_shard_meas(Cfg cfg, uint32_t n, const uint64_t* meas,
                                                    uint32_t meas_words, CRows helper_meas,
                                                    Rows leader, const uint64_t* norms) {
  const uint32_t r = blockIdx.y;
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n || i >= cfg.meas_len) return;
  const uint32_t x = enc_meas_bit(cfg, meas + (size_t)r * meas_words, i,
                                  norms ? norms + 2 * (size_t)r : nullptr);
  const typename FO::T h = FO::load(helper_meas.at(r) + (size_t)i * FO::ES);
  FO::store(leader.at(r) + (size_t)i * FO::ES, FO::sub(FO::from_u32(x), h));
}

// Both joint-rand parts, the public share, the joint-rand seed and the joint randomness; then the
// prove randomness XOF(k_prove, dst4, "").  Lane per report.
template <class FO>
__global__ void __launch_bounds__(256) k_shard_jr(Cfg cfg, uint32_t n, CRows nonces, CRows rand,
                                                  CRows helper_meas, CRows leader, Rows pub,
                                                  Rows jr_out, Rows prove_rand_out) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  const uint8_t* nz = nonces.at(r);
  const uint8_t* rd = rand.at(r);
  const uint32_t kp = cfg.jr_len ? 64u : 32u;  // offset of k_prove in the rand row
  if (cfg.jr_len) {
    uint64_t hlo, hhi, llo, lhi;
    jr_part(cfg.xof, cfg.algo_id, 1, ld64(rd + 32), ld64(rd + 40), ld64(nz), ld64(nz + 8),
            helper_meas.at(r), cfg.meas_len * cfg.es, hlo, hhi);
    jr_part(cfg.xof, cfg.algo_id, 0, ld64(rd + 48), ld64(rd + 56), ld64(nz), ld64(nz + 8), leader.at(r),
            cfg.meas_len * cfg.es, llo, lhi);
    uint8_t* p = pub.at(r);
    st64(p, llo);
    st64(p + 8, lhi);
    st64(p + 16, hlo);
    st64(p + 24, hhi);
    uint64_t slo, shi;
    derive_jr_seed(cfg.xof, cfg.algo_id, llo, lhi, hlo, hhi, slo, shi);
    MsgBlock mb;
    mb.clear();
    mb.header(cfg.algo_id, DST_JOINT_RANDOMNESS, slo, shi);
    mb.pad(25, cfg.xof);
    uint64_t s[25];
    sponge_one_block(s, mb, cfg.xof);
    squeeze_vec<FO>(s, cfg.jr_len, jr_out.at(r), cfg.xof, cfg.exact_squeeze);
  }
  MsgBlock mb;
  mb.clear();
  mb.header(cfg.algo_id, DST_PROVE_RANDOMNESS, ld64(rd + kp), ld64(rd + kp + 8));
  mb.pad(25, cfg.xof);
  uint64_t s[25];
  sponge_one_block(s, mb, cfg.xof);
  squeeze_vec<FO>(s, cfg.prove_rand_len, prove_rand_out.at(r), cfg.xof, cfg.exact_squeeze);
}

// leader proof share = proof - helper proof share   (thread per element)
template <class FO>
__global__ void __launch_bounds__(256) k_shard_proof(Cfg cfg, uint32_t n, CRows proof,
                                                     CRows helper_proof, Rows leader) {
  const uint32_t r = blockIdx.y;
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n || i >= cfg.proof_len) return;
  const typename FO::T a = FO::load(proof.at(r) + (size_t)i * FO::ES);
  const typename FO::T h = FO::load(helper_proof.at(r) + (size_t)i * FO::ES);
  FO::store(leader.at(r) + (size_t)(cfg.meas_len + i) * FO::ES, FO::sub(a, h));
}

}  // namespace p3g
