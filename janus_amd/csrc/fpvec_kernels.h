// FLP query + decide for Prio3FixedPointBoundedL2VecSum (prio 0.15.1
// src/flp/types/fixedpoint_l2.rs, ext; Janus VdafInstance::Prio3FixedPoint{16,32,64}BitBoundedL2VecSum,
// aggregator/src/aggregator.rs:839-861, dispatched at :1115-1145).
//
// The type's circuit has TWO gadgets (restated in oracle/prio3.py FixedPointBoundedL2VecSum):
//   gadget 0 = ParallelSum(Mul, c0) range check over all bits x_0..x_{L0-1}
//              (L0 = n*entries + 2n-2; parallel_sum_range_checks on jr[0]),
//   gadget 1 = ParallelSum(PolyEval([2^(2n-2), -2^n, 1]), c1) over the decoded entries
//              z_e = sum_l 2^l x_{ne+l}  (padding: the share of the encoded zero, 2^(n-1)/2),
//   v = jr[1] * sum_k p0(alpha0^k) + jr[1]^2 * (sum_k p1(alpha1^k) - sum_l 2^l x_{n entries + l}).
// The verifier share is [v, wires0 (2 c0), p0(t0), wires1 (c1), p1(t1)] and decide checks
// v == 0, G0(wires0) == p0(t0), G1(wires1) == p1(t1).
//
// Shapes are large and reports few (entries = 100k: 1.6M-element shares, 25.6 MB per report), so
// unlike the ParallelSum kernels for SumVec (a wave per report), every step here spreads ONE
// report over many blocks:
//   k_fpv_weights   block per (report, gadget): power tables, one size-m NTT for the Lagrange
//                   weights at t_g, gadget-output sum as a dot product with the host S table, p(t)
//   k_fpv_wires0    block per (report, 256 columns, row group): lazily reduced dot products
//                   sum_k (L_k r^(c(k-1))) x and sum_k L_k x over the measurement share (HBM stream)
//   k_fpv_wires1    block per (report, 256 columns): decode z_e on the fly, sum_k L_k z
//   k_fpv_finalize  block per (report, 256 columns): fold the row groups, v, p(t), joint-rand part
//   k_fpv_decide    block per report
#pragma once
#include "prio3_kernels.h"
#include "keccak_pair.h"

namespace p3g {

// ------------------------------------------------------------------------------------------------
// Pipelined helper XOF for few, huge reports (k_helper_xof): the helper's measurement-share
// expansion XOF(k_meas, dst1, [1]) and its joint-rand part derive_seed(blind, dst7, [1] || nonce ||
// encode(meas share)) are two 152K-permutation chains per report at entries = 100k, and with
// only a few waves in flight the step is their latency.  Run one after the other (k_expand, then
// k_jr) they cost two chains; here a 2-wave workgroup runs them as a producer/consumer pipeline:
// producer waves squeeze block i of the expansion (store it, and hand it over through an LDS
// ring of kHxDepth slots) while consumer waves absorb earlier blocks into the joint-rand sponge.
// Both waves run the SAME permutation code on their own state (one hot Keccak copy: two would
// not fit the instruction cache; a two-state single wave measured 20 % slower than serial).
//
// Exactness: when every squeezed element is canonical (< p; fails with probability ~28/2^64 per
// element) the encoded measurement share IS the XOF byte stream, so the consumer absorbs the
// producer's words directly: its block b needs stream words [21b-6, 21b+15], i.e. words 15..20 of
// block b-1 (carried in registers) and words 0..15 of block b.  A report that meets a
// non-canonical element bumps `fallback`; the engine then re-runs the exact k_expand + k_jr for
// the batch, so outputs are identical either way.
// ------------------------------------------------------------------------------------------------
// Absorb block b of a joint-rand-part message  header(blind) || agg_id || nonce || share  into
// s, given share words [21b, 21b + 16) (A; zeros past the share) and carry = share words
// [21b - 6, 21b) (for b = 0: carry[5] = the nonce's high word).  The 42-byte prefix puts share
// word j at message bytes 42 + 8j, so message word w of block b is the 16-bit shifted pair
// (D[21b + w - 6] >> 48) | (D[21b + w - 5] << 16).
DEVI void jrp_absorb(uint64_t s[25], const uint64_t carry[6], const uint64_t A[16], int64_t b,
                     int64_t nblocks, int64_t padw, uint64_t padv, const Cfg& cfg,
                     uint32_t agg_id, const uint8_t* blind, const uint8_t* nonce) {
#pragma unroll
  for (int w = 0; w < 21; ++w) {
    uint64_t v;
    if (b == 0 && w < 5) {  // prefix: header(blind) || agg_id || nonce
      MsgBlock m;
      m.clear();
      m.header(cfg.algo_id, DST_JOINT_RAND_PART, ld64(blind), ld64(blind + 8));
      m.put8(25, agg_id);
      m.put64(26, ld64(nonce));
      m.put64(34, carry[5]);
      v = m.w[w];
    } else {
      const uint64_t dlo = w <= 5 ? carry[w] : A[w - 6];
      const uint64_t dhi = w <= 4 ? carry[w + 1] : A[w - 5];
      v = (dlo >> 48) | (dhi << 16);
    }
    const int64_t g = 21 * b + w;
    if (padw == g) v ^= padv;
    if (b == nblocks - 1 && w == 20) v ^= 0x8000000000000000ull;
    s[w] ^= v;
  }
}



// Ring counters in LDS.  kLds: read and written with ds instructions; else through a volatile
// generic pointer, which compiles to FLAT (sc0 sc1) with an s_waitcnt vmcnt(0) lgkmcnt(0) that
// also waits for every global access the wave has in flight.  LDS operations of one wave complete
// in order, so a counter written after a slot's data publishes that data.  Measured at 10,240
// config E reports (profiles/r05/fpvec2/r5_ctr_*.log): the helper's chains run 1,383 -> 1,277 ms
// alone and 1,469 -> 1,306 beside the leader with ds counters, while the leader's k_jr_ring goes
// 1,234 -> 1,371 and 1,314 -> 1,486 -- so k_helper_xof takes ds counters (P3G_HX_CTR_LDS) and
// k_jr_ring keeps the FLAT form (P3G_JR_CTR_LDS).
#ifndef P3G_HX_CTR_LDS
#define P3G_HX_CTR_LDS 1
#endif
#ifndef P3G_JR_CTR_LDS
#define P3G_JR_CTR_LDS 0
#endif
constexpr bool kHxLds = P3G_HX_CTR_LDS != 0, kJrLds = P3G_JR_CTR_LDS != 0;
// A/B split of k_jr_ring's counter accesses by wave and direction (default: all kJrLds)
#ifndef P3G_JR_LOADER_LDS
#define P3G_JR_LOADER_LDS P3G_JR_CTR_LDS
#endif
#ifndef P3G_JR_SPONGE_LD_LDS
#define P3G_JR_SPONGE_LD_LDS P3G_JR_CTR_LDS
#endif
#ifndef P3G_JR_SPONGE_ST_LDS
#define P3G_JR_SPONGE_ST_LDS P3G_JR_CTR_LDS
#endif
constexpr bool kJrLoaderLds = P3G_JR_LOADER_LDS != 0, kJrSpongeLdLds = P3G_JR_SPONGE_LD_LDS != 0,
               kJrSpongeStLds = P3G_JR_SPONGE_ST_LDS != 0;
#ifndef P3G_HX_CONS_ST_LDS  // A/B: k_helper_xof's consumer / producer publish
#define P3G_HX_CONS_ST_LDS P3G_HX_CTR_LDS
#endif
#ifndef P3G_HX_PROD_ST_LDS
#define P3G_HX_PROD_ST_LDS P3G_HX_CTR_LDS
#endif
constexpr bool kHxConsStLds = P3G_HX_CONS_ST_LDS != 0, kHxProdStLds = P3G_HX_PROD_ST_LDS != 0;
#ifndef P3G_JR_LOADER_SLEEP
#define P3G_JR_LOADER_SLEEP 1  // A/B: s_sleep quanta of k_jr_ring's loader while the ring is full
#endif
template <bool kLds>
DEVI uint32_t ctr_ld(uint32_t* p) {
  if constexpr (!kLds) {
    return *reinterpret_cast<volatile uint32_t*>(p);
  } else {
    const uint32_t a = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint32_t*)p;
    uint32_t v;
    asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a) : "memory");
    return __builtin_amdgcn_readfirstlane(v);
  }
}
template <bool kLds>
DEVI void ctr_st(uint32_t* p, uint32_t v) {
  if constexpr (!kLds) {
    *reinterpret_cast<volatile uint32_t*>(p) = v;
  } else {
    const uint32_t a = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint32_t*)p;
    asm volatile("ds_write_b32 %0, %1" : : "v"(a), "v"(v) : "memory");
  }
}

constexpr uint32_t kHxRows = 64;              // reports per producer/consumer pair (a wave each)
constexpr uint32_t kHxDepth = 4;              // ring slots: the producer may run 4 blocks ahead
// LDS ring bytes of one pair (slot rows kHxRows + 1 words apart; see k_helper_xof)
constexpr size_t kHxRingBytes = (size_t)kHxDepth * 21 * (kHxRows + 1) * 8;

// Snapshot mode (engine option helper_snap, the default for FixedPoint vectors): instead of
// storing the 25.6 MB expanded measurement share of every report (entries = 100k), the producer
// keeps the 200-byte sponge state of every kSnapEvery-th block, and k_fpv_regen rewrites any
// range of reports' shares from those snapshots -- in parallel over the snapshots, so the
// rewrite is throughput-bound (a 64-permutation chain per lane), not a 152K-permutation chain.
// The share then costs 200 B per 10.75 KB (1/54) in HBM and twice as many reports fit in flight.
constexpr uint32_t kSnapEvery = 64;  // producer blocks per state snapshot
__host__ __device__ inline uint32_t snap_count(const Cfg& g) {
  const uint32_t nprod = (2u * g.meas_len + 20u) / 21u;
  return (nprod + kSnapEvery - 1u) / kSnapEvery;
}
constexpr size_t kSnapBytes = 25 * 8;  // one Keccak state

// kPairs producer/consumer/storer triples per workgroup (waves p, kPairs + p, 2 kPairs + p for
// pair p), each with its own ring: the waves of ONE workgroup sit on distinct SIMDs, while two
// workgroups sharing a CU put their first waves on the same SIMD, so when there are more pairs
// than CUs (or the other aggregator's chains share the GPU) two pairs per workgroup keep one
// sponge wave per SIMD.  The ring lives in dynamic LDS (kPairs * kHxRingBytes at launch).
template <uint32_t kDepth, uint32_t kPairs>
__global__ void __launch_bounds__(3 * kHxRows * kPairs) k_helper_xof(Cfg cfg, uint32_t n, CRows helper_shares,
                                                    CRows nonces, CRows public_shares,
                                                    Rows out_meas, Rows out_proof, Rows out_part,
                                                    Rows out_seed, Rows out_jr,
                                                    const uint8_t* status, uint32_t* fallback,
                                                    uint64_t* spec_lo, uint8_t* spec_cy,
                                                    uint64_t* snaps) {
  using FO = Field128Ops;
  // slot rows are kHxRows + 1 words apart: the storer's column reads (words x rows) hit distinct
  // banks; the producer's and consumer's row accesses stay conflict-free
  constexpr uint32_t kStride = kHxRows + 1, kSlot = 21 * kStride;
  static_assert(kDepth == kHxDepth, "kHxRingBytes assumes kHxDepth slots");
  extern __shared__ __attribute__((aligned(16))) uint64_t hx_dyn[];
  // Ring handoff through LDS counters instead of a per-block s_barrier: the producer publishes
  // `produced` after its slot writes have landed (lgkmcnt(0)); the consumer publishes `consumed`
  // (the storer `stored`) after its slot reads have returned.  Neither wave waits for the other's
  // permutation unless the ring is full / empty, so each runs at its own pace.
  __shared__ uint32_t counters[3 * kPairs];
  const uint32_t lane = threadIdx.x & (kHxRows - 1u);
  const uint32_t wave = threadIdx.x / kHxRows;  // wave-uniform roles
  const uint32_t pair = wave % kPairs, role = wave / kPairs;
  uint64_t* ring = hx_dyn + (size_t)pair * (kDepth * kSlot);
  uint32_t* vprod = &counters[3 * pair];
  uint32_t* vcons = &counters[3 * pair + 1];
  uint32_t* vstor = &counters[3 * pair + 2];
  if (threadIdx.x < 3 * kPairs) counters[threadIdx.x] = 0u;
  __syncthreads();
  // role 0 produces, role 1 consumes, role 2 stores the expanded share to HBM / sums its columns
  const bool producer = role == 0u, storer = role == 2u;
  const uint32_t r0 = (blockIdx.x * kPairs + pair) * kHxRows;
  if (r0 >= n) return;  // a whole pair past the batch (no barrier follows)
  if (cfg.wave_prio) __builtin_amdgcn_s_setprio(3);  // the chain first on its SIMD
  const uint32_t r = r0 + lane;
  const bool live = r < n && (!status || status[r] == ST_OK);
  const uint32_t rr = r < n ? r : n - 1u;  // every lane runs the loop, clamped row
  const uint8_t* hs = helper_shares.at(rr);
  const int64_t nd = (int64_t)cfg.meas_len * 2;    // meas-share words
  const int64_t total = 42 + 8 * nd;                // consumer's message bytes before padding
  const int64_t nblocks = total / 168 + 1;          // consumer blocks
  const int64_t nprod = (nd + 20) / 21;             // producer blocks
  const int64_t padw = total >> 3;
  const uint64_t padv = (uint64_t)cfg.xof.pad << ((total & 7) * 8);
  const uint64_t nonce_hi = ld64(nonces.at(rr) + 8);
  uint64_t s[25];
  if (producer) {
    MsgBlock m;
    m.clear();
    m.header(cfg.algo_id, DST_MEASUREMENT_SHARE, ld64(hs), ld64(hs + 8));
    m.put8(25, 1u);
    m.pad(26, cfg.xof);
    sponge_one_block(s, m, cfg.xof);  // s = expansion block 0
  } else {
#pragma unroll
    for (int i = 0; i < 25; ++i) s[i] = 0ull;
  }
  uint64_t carry[6];  // consumer: stream words 21(b-1)+15 .. 21(b-1)+20; D[-1] = nonce_hi
#pragma unroll
  for (int i = 0; i < 6; ++i) carry[i] = 0ull;
  carry[5] = nonce_hi;
  bool bad = false;
  uint8_t* om = out_meas.at(rr);
  // One loop for all roles so the waves share ONE inlined permutation (two copies would not
  // fit the instruction cache).
  const int64_t iters = producer || storer ? nprod : nblocks;
  for (int64_t i = 0; i < iters; ++i) {
    bool perm = true;
    if (producer) {
      const int64_t j0 = 21 * i;
      if (snaps != nullptr && (i % kSnapEvery) == 0 && r < n) {
        uint64_t* sp = snaps + ((size_t)r * snap_count(cfg) + (size_t)(i / kSnapEvery)) * 25;
#pragma unroll
        for (int w = 0; w < 25; ++w) sp[w] = s[w];
      }
      while (i - (int64_t)min(ctr_ld<kHxLds>(vcons), ctr_ld<kHxLds>(vstor)) >= (int64_t)kDepth)
        __builtin_amdgcn_s_sleep(1);
      asm volatile("" ::: "memory");
      uint64_t* slot = ring + (i % kDepth) * kSlot;
#pragma unroll
      for (int w = 0; w < 21; ++w) slot[w * kStride + lane] = j0 + w < nd ? s[w] : 0ull;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // slot written before it is published
      ctr_st<kHxProdStLds>(vprod, (uint32_t)(i + 1));
      perm = 21 * (i + 1) < nd;
    } else if (storer) {
      // store block i of the expanded share and check its elements are canonical
      const int64_t j0 = 21 * i;
      while ((int64_t)ctr_ld<kHxLds>(vprod) <= i) __builtin_amdgcn_s_sleep(1);
      asm volatile("" ::: "memory");
      const uint64_t* slot = ring + (i % kDepth) * kSlot;
#pragma unroll
      for (int w = 0; w < 21; ++w) s[w] = slot[w * kStride + lane];
      // speculative accumulation (k_jr's layout): column sums of the block's 21 words over the
      // wave's 64 rows, lane = word wc + 21 gq summing rows gq, gq + 3, ... (lane 63 idle)
      const uint32_t gq = lane / 21u, wc = lane - 21u * gq;
      uint64_t xs[22];
      if (spec_lo != nullptr) {
        const uint64_t* col = slot + (gq < 3u ? wc : 0u) * kStride;
#pragma unroll
        for (int k = 0; k < 22; ++k) {
          const uint32_t row = gq + 3u * (uint32_t)k;
          xs[k] = (gq < 3u && row < 64u) ? col[row] : 0ull;
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // slot read before it is released
      ctr_st<kHxLds>(vstor, (uint32_t)(i + 1));
      if (spec_lo != nullptr) {
        uint32_t l32 = 0, h32 = 0, cy = 0;
#pragma unroll
        for (int k = 0; k < 22; ++k) acc_u64(l32, h32, cy, xs[k]);
        const uint32_t s1 = (lane + 21u) & 63u, s2 = (lane + 42u) & 63u;
        const uint32_t la = __shfl(l32, (int)s1, 64), ha = __shfl(h32, (int)s1, 64);
        const uint32_t ca = __shfl(cy, (int)s1, 64);
        const uint32_t lb = __shfl(l32, (int)s2, 64), hb = __shfl(h32, (int)s2, 64);
        const uint32_t cb = __shfl(cy, (int)s2, 64);
        if (lane < 21u && j0 + lane < nd) {
          acc_u64(l32, h32, cy, ((uint64_t)ha << 32) | la);
          acc_u64(l32, h32, cy, ((uint64_t)hb << 32) | lb);
          const size_t at = (size_t)(r0 >> 6) * (size_t)nd + (size_t)(j0 + lane);
          spec_lo[at] = ((uint64_t)h32 << 32) | l32;
          spec_cy[at] = (uint8_t)(cy + ca + cb);
        }
      }
      // every row below n is stored (also reports rejected before this kernel): k_accum_spec
      // subtracts a rejected row's stored words from the column sums, which include it
      // (snapshot mode: nothing is stored, k_fpv_regen rewrites rows when they are needed)
      const bool st_row = snaps != nullptr ? false : spec_lo != nullptr ? r < n : live;
      if (j0 + 21 <= nd) {  // whole block: 16-B stores (block i starts 16-B aligned iff i even)
        if (st_row) {
          uint8_t* o = om + 8 * j0;
          if ((i & 1) == 0) {
#pragma unroll
            for (int w = 0; w < 20; w += 2)
              *reinterpret_cast<ulonglong2*>(o + 8 * w) = make_ulonglong2(s[w], s[w + 1]);
            st64(o + 160, s[20]);
          } else {
            st64(o, s[0]);
#pragma unroll
            for (int w = 1; w < 21; w += 2)
              *reinterpret_cast<ulonglong2*>(o + 8 * w) = make_ulonglong2(s[w], s[w + 1]);
          }
        }
#pragma unroll
        for (int w = 0; w < 21; ++w)
          if (((j0 + w) & 1) && !hi_ok(s[w])) bad = true;
      } else {
#pragma unroll
        for (int w = 0; w < 21; ++w) {
          const bool in = j0 + w < nd;
          if (in && st_row) st64(om + 8 * (j0 + w), s[w]);
          if (in && ((j0 + w) & 1) && !hi_ok(s[w])) bad = true;
        }
      }
      perm = false;
    } else {
      const int64_t b = i;
      const bool data = 21 * b < nd;  // else the block is past the share: zeros
      uint64_t A[16];
      if (data) {
        while ((int64_t)ctr_ld<kHxLds>(vprod) <= b) __builtin_amdgcn_s_sleep(1);
        asm volatile("" ::: "memory");
        const uint64_t* slot = ring + (b % kDepth) * kSlot;
#pragma unroll
        for (int w = 0; w < 16; ++w) A[w] = slot[w * kStride + lane];
      } else {
#pragma unroll
        for (int w = 0; w < 16; ++w) A[w] = 0ull;
      }
      jrp_absorb(s, carry, A, b, nblocks, padw, padv, cfg, 1u, hs + 32, nonces.at(rr));
      if (data) {
        const uint64_t* slot = ring + (b % kDepth) * kSlot;
#pragma unroll
        for (int k = 0; k < 6; ++k) carry[k] = slot[(15 + k) * kStride + lane];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // slot read before it is released
        ctr_st<kHxConsStLds>(vcons, (uint32_t)(b + 1));
      } else {
#pragma unroll
        for (int k = 0; k < 6; ++k) carry[k] = 0ull;
      }
    }
    if (perm) keccak_x(s, cfg.xof);
  }
  if (storer) {
    if (live && bad) atomicAdd(fallback, 1u);
    return;
  }
  if (producer) {
    if (live) {
      xof_expand_byte_binder<FO>(cfg.algo_id, DST_PROOF_SHARE, ld64(hs + 16), ld64(hs + 24), 1u,
                                 cfg.proof_len, out_proof.at(r), cfg.xof, cfg.exact_squeeze);
    }
    return;
  }
  if (!live) return;
  const uint64_t plo = s[0], phi = s[1];
  st64(out_part.at(r), plo);
  st64(out_part.at(r) + 8, phi);
  const uint8_t* ps = public_shares.at(r);
  uint64_t slo, shi;
  derive_jr_seed(cfg.xof, cfg.algo_id, ld64(ps), ld64(ps + 8), plo, phi, slo, shi);
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

// The helper's expanded measurement shares of reports [r0, r0 + nr) rewritten into rows 0..nr-1
// of `out` from k_helper_xof's state snapshots: lane = (report, snapshot), each lane stores its
// kSnapEvery blocks exactly as the storer wave would have (the share is the raw XOF stream; the
// fused path checked every element canonical) and permutes between them.
// kPair: the snapshots hold (even half, odd half) dword pairs (k_helper_xof_pair, fpvec_pair.h).
template <bool kPair>
__global__ void __launch_bounds__(256) k_fpv_regen(Cfg cfg, uint32_t nr, uint32_t r0,
                                                   const uint64_t* snaps, Rows out) {
  const uint32_t nsnap = snap_count(cfg);
  const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (uint64_t)nr * nsnap) return;
  const uint32_t q = (uint32_t)(gid / nsnap), k = (uint32_t)(gid - (uint64_t)q * nsnap);
  const int64_t nd = (int64_t)cfg.meas_len * 2, nprod = (nd + 20) / 21;
  const uint64_t* sp = snaps + ((size_t)(r0 + q) * nsnap + k) * 25;
  uint64_t s[25];
#pragma unroll
  for (int w = 0; w < 25; ++w) {
    const uint64_t v = sp[w];
    s[w] = kPair ? kp_zip((uint32_t)v, (uint32_t)(v >> 32)) : v;
  }
  uint8_t* om = out.at(q);
  const int64_t i0 = (int64_t)k * kSnapEvery;
  const int64_t i1 = i0 + kSnapEvery < nprod ? i0 + kSnapEvery : nprod;
  for (int64_t i = i0;; ++i) {
    const int64_t j0 = 21 * i;
    if (j0 + 21 <= nd) {  // whole block: 16-B stores (block i starts 16-B aligned iff i even)
      uint8_t* o = om + 8 * j0;
      if ((i & 1) == 0) {
#pragma unroll
        for (int w = 0; w < 20; w += 2)
          *reinterpret_cast<ulonglong2*>(o + 8 * w) = make_ulonglong2(s[w], s[w + 1]);
        st64(o + 160, s[20]);
      } else {
        st64(o, s[0]);
#pragma unroll
        for (int w = 1; w < 21; w += 2)
          *reinterpret_cast<ulonglong2*>(o + 8 * w) = make_ulonglong2(s[w], s[w + 1]);
      }
    } else {
#pragma unroll
      for (int w = 0; w < 21; ++w)
        if (j0 + w < nd) st64(om + 8 * (j0 + w), s[w]);
    }
    if (i + 1 >= i1) break;
    keccak_x(s, cfg.xof);
  }
}

// Joint-rand part of an aggregator's own (given) measurement share for few, huge reports
// (k_jr_ring; the leader side of config E): k_jr's sponge wave stalls on its LDS-DMA window
// refills and does the speculative column sums itself.  Here a loader wave streams share blocks
// from HBM into an LDS ring (the same counter handoff as k_helper_xof) and writes the
// speculative column sums k_accum_spec consumes (every share word, same layout and row clamp as
// k_jr), while the sponge wave only absorbs and permutes.  Ring rows are 65 words apart so the
// loader's column reads (lane = word) hit distinct banks.
// kPairs sponge/loader pairs per workgroup (waves p and kPairs + p), rings in dynamic LDS
// (kPairs * kHxRingBytes at launch), for the reason k_helper_xof gives.
constexpr uint32_t kJrRingStride = kHxRows + 1;

template <uint32_t kPairs>
__global__ void __launch_bounds__(2 * kHxRows * kPairs) k_jr_ring(Cfg cfg, uint32_t n, uint32_t agg_id,
                                                 CRows nonces, CRows public_shares,
                                                 CRows blinds, CRows meas, Rows out_part,
                                                 Rows out_seed, Rows out_jr,
                                                 const uint8_t* status, uint64_t* spec_lo,
                                                 uint8_t* spec_cy) {
  using FO = Field128Ops;
  constexpr uint32_t kSlot = 21 * kJrRingStride;
  extern __shared__ __attribute__((aligned(16))) uint64_t jr_dyn[];
  __shared__ uint32_t counters[2 * kPairs];
  const uint32_t lane = threadIdx.x & (kHxRows - 1u);
  const uint32_t wave = threadIdx.x / kHxRows;
  const uint32_t pair = wave % kPairs;
  const bool loader = wave >= kPairs;  // waves 0..kPairs-1: sponges, then the loaders
  uint64_t* ring = jr_dyn + (size_t)pair * (kHxDepth * kSlot);
  uint32_t* vprod = &counters[2 * pair];
  uint32_t* vcons = &counters[2 * pair + 1];
  if (threadIdx.x < 2 * kPairs) counters[threadIdx.x] = 0u;
  __syncthreads();
  const uint32_t r0 = (blockIdx.x * kPairs + pair) * kHxRows;
  if (r0 >= n) return;  // a whole pair past the batch (no barrier follows)
  if (cfg.wave_prio) __builtin_amdgcn_s_setprio(3);  // the chain first on its SIMD
  const uint32_t r = r0 + lane;
  const bool live = r < n && (!status || status[r] == ST_OK);
  const uint32_t rr = r < n ? r : n - 1u;  // rows past n: the last row (k_jr's clamp)
  const uint8_t* data = meas.at(rr);
  const int64_t nd = (int64_t)cfg.meas_len * 2;  // share words
  const int64_t total = 42 + 8 * nd;
  const int64_t nblocks = total / 168 + 1;
  const int64_t nprod = (nd + 20) / 21;
  const int64_t padw = total >> 3;
  const uint64_t padv = (uint64_t)cfg.xof.pad << ((total & 7) * 8);
  uint64_t s[25];
#pragma unroll
  for (int i = 0; i < 25; ++i) s[i] = 0ull;
  uint64_t carry[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) carry[i] = 0ull;
  carry[5] = ld64(nonces.at(rr) + 8);
  const int64_t iters = loader ? nprod : nblocks;
  for (int64_t i = 0; i < iters; ++i) {
    bool perm = true;
    if (loader) {
      const int64_t j0 = 21 * i;
      const uint8_t* src = data + 8 * j0;  // loads first: in flight while the ring is full
      if (j0 + 21 <= nd) {  // whole block: 16-B loads (block i starts 16-B aligned iff i even)
        if ((i & 1) == 0) {
#pragma unroll
          for (int w = 0; w < 20; w += 2) {
            const ulonglong2 v = *reinterpret_cast<const ulonglong2*>(src + 8 * w);
            s[w] = v.x;
            s[w + 1] = v.y;
          }
          s[20] = ld64(src + 160);
        } else {
          s[0] = ld64(src);
#pragma unroll
          for (int w = 1; w < 21; w += 2) {
            const ulonglong2 v = *reinterpret_cast<const ulonglong2*>(src + 8 * w);
            s[w] = v.x;
            s[w + 1] = v.y;
          }
        }
      } else {
#pragma unroll
        for (int w = 0; w < 21; ++w) s[w] = j0 + w < nd ? ld64(src + 8 * w) : 0ull;
      }
      while (i - (int64_t)ctr_ld<kJrLoaderLds>(vcons) >= (int64_t)kHxDepth)
        __builtin_amdgcn_s_sleep(P3G_JR_LOADER_SLEEP);
      asm volatile("" ::: "memory");
      uint64_t* slot = ring + (i % kHxDepth) * kSlot;
#pragma unroll
      for (int w = 0; w < 21; ++w) slot[w * kJrRingStride + lane] = s[w];
      if (spec_lo != nullptr && lane < 21u && j0 + lane < nd) {
        // column sum of word j0 + lane over the wave's 64 rows (this wave's own LDS writes
        // above complete first: one wave's LDS operations execute in order)
        const uint64_t* col = slot + lane * kJrRingStride;
        uint32_t l32 = 0, h32 = 0, cy = 0;
#pragma unroll 16
        for (int k = 0; k < 64; ++k) acc_u64(l32, h32, cy, col[k]);
        const size_t at = (size_t)(r0 >> 6) * (size_t)nd + (size_t)(j0 + lane);
        spec_lo[at] = ((uint64_t)h32 << 32) | l32;
        spec_cy[at] = (uint8_t)cy;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // slot written before it is published
      ctr_st<kJrLoaderLds>(vprod, (uint32_t)(i + 1));
      perm = false;
    } else {
      const int64_t b = i;
      const bool has = 21 * b < nd;  // else the block is past the share: zeros
      uint64_t A[16];
      if (has) {
        while ((int64_t)ctr_ld<kJrSpongeLdLds>(vprod) <= b) __builtin_amdgcn_s_sleep(1);
        asm volatile("" ::: "memory");
        const uint64_t* slot = ring + (b % kHxDepth) * kSlot;
#pragma unroll
        for (int w = 0; w < 16; ++w) A[w] = slot[w * kJrRingStride + lane];
      } else {
#pragma unroll
        for (int w = 0; w < 16; ++w) A[w] = 0ull;
      }
      jrp_absorb(s, carry, A, b, nblocks, padw, padv, cfg, agg_id, blinds.at(rr), nonces.at(rr));
      if (has) {
        const uint64_t* slot = ring + (b % kHxDepth) * kSlot;
#pragma unroll
        for (int k = 0; k < 6; ++k) carry[k] = slot[(15 + k) * kJrRingStride + lane];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // slot read before it is released
        ctr_st<kJrSpongeStLds>(vcons, (uint32_t)(b + 1));
      } else {
#pragma unroll
        for (int k = 0; k < 6; ++k) carry[k] = 0ull;
      }
    }
    if (perm) keccak_x(s, cfg.xof);
  }
  if (loader || !live) return;
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

// Per-report weight row ("W"), element offsets (Field128 elements).
struct FpvW {
  uint32_t mm, lm, rp, b0, b1, g0, l1, c1, g1, len;
};
__host__ __device__ inline FpvW fpv_w_layout(const Cfg& g) {
  FpvW w;
  w.mm = 0;                       // L_k r^(c0 (k-1)), k = 1..calls0     (Montgomery)
  w.lm = w.mm + g.calls;          // L_k, k = 1..calls0                  (Montgomery)
  w.rp = w.lm + g.calls;          // r^(j+1), j < c0                     (Montgomery)
  w.b0 = w.rp + g.chunk;          // L_0 s_2j                            (canonical)
  w.b1 = w.b0 + g.chunk;          // L_0 s_2j+1 - (1/2) sum_k L_k        (canonical)
  w.g0 = w.b1 + g.chunk;          // sum_k p0(alpha0^k)                  (canonical)
  w.l1 = w.g0 + 1;                // L'_k, k = 1..calls1                 (Montgomery)
  w.c1 = w.l1 + g.calls1;         // L'_0 s'_j + [padded] L'_calls1 z0   (canonical)
  w.g1 = w.c1 + g.chunk1;         // sum_k p1(alpha1^k)                  (canonical)
  w.len = w.g1 + 1;
  return w;
}

// Row groups of k_fpv_wires0 (calls split H ways so one report fills many blocks).
__host__ __device__ inline uint32_t fpv_rows(const Cfg& g) { return g.calls < 32u ? g.calls : 32u; }

// Flag bits per report (OR-ed by every kernel of the query, turned into a status by finalize).
enum : uint32_t { FPV_BAD_ENCODING = 1u, FPV_ROOT_OF_UNITY = 2u };

// One in-place radix-2 DIT NTT of size m (input bit-reversed) in LDS, twiddles `tw` (Montgomery).
DEVI void ntt1_lds(F128* A, uint32_t m, uint32_t logm, const uint8_t* tw, uint32_t tid,
                   uint32_t nthr) {
  using FO = Field128Ops;
  for (uint32_t st = 1; st <= logm; ++st) {
    const uint32_t half = 1u << (st - 1);
    for (uint32_t q = tid; q < (m >> 1); q += nthr) {
      const uint32_t grp = q >> (st - 1), k = q & (half - 1u);
      const uint32_t i = grp * 2u * half + k, j = i + half;
      const F128 w = FO::load(tw + (size_t)(k << (logm - st)) * 16u);
      const F128 u = A[i];
      const F128 v = FO::mul(w, A[j]);
      A[i] = FO::add(u, v);
      A[j] = FO::sub(u, v);
    }
    __syncthreads();
  }
}

// grid (n, 2), 256 threads.  LDS: TP[m] | NA[m] | RC[m] | RP[c0+1] | RED[3*4] | flag
__global__ void __launch_bounds__(256) k_fpv_weights(Cfg cfg, uint32_t n, CRows proof, CRows tq,
                                                     CRows jr, Rows prep, const uint8_t* status,
                                                     Rows wrows, uint32_t* flags) {
  using FO = Field128Ops;
  using T = F128;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t r = blockIdx.x, gi = blockIdx.y;
  if (r >= n || status[r] != ST_OK) return;
  const uint32_t tid = threadIdx.x, nthr = blockDim.x, lane = tid & 63u, wave = tid >> 6;
  const uint32_t m = gi ? cfg.m1 : cfg.m, logm = gi ? cfg.logm1 : cfg.logm;
  const uint32_t calls = gi ? cfg.calls1 : cfg.calls, c = gi ? cfg.chunk1 : cfg.chunk;
  const uint32_t arity = gi ? cfg.chunk1 : cfg.arity, gp_len = gi ? cfg.gp_len1 : cfg.gp_len;
  const uint8_t* tw = gi ? cfg.twiddles1 : cfg.twiddles;
  const size_t ES = 16;
  const FpvW W = fpv_w_layout(cfg);
  T* TP = reinterpret_cast<T*>(smem);
  T* NA = TP + m;
  T* RC = NA + m;
  T* RP = RC + m;
  T* RED = RP + (cfg.chunk + 1);
  uint32_t* flag = reinterpret_cast<uint32_t*>(RED + 12);
  if (tid == 0) *flag = 0u;

  // proof block of this gadget: [seeds (arity)] || [gadget poly (gp_len)]
  const uint8_t* pr = proof.at(r) + (gi ? (size_t)(cfg.arity + cfg.gp_len) * ES : 0);
  const T tm = FO::to_mont(FO::load(tq.at(r) + (size_t)gi * ES));
  const T rm = FO::to_mont(FO::load(jr.at(r)));  // jr[0]: the range check's joint randomness
  if (wave == 0) wave_pow_table<FO>(TP, tm, m, lane);
  if (gi == 0 && wave == 1) wave_pow_table<FO>(RP, rm, c + 1, lane);
  if (gi == 0 && wave == 2) wave_pow_table<FO>(RC, mont_pow<FO>(rm, c), calls, lane);
  __syncthreads();
  const T tmm = FO::mul(TP[m - 1], tm);  // t^m (Montgomery)
  if (tid == 0 && FO::eq(tmm, FO::one_mont())) atomicOr(flag, FPV_ROOT_OF_UNITY);
  for (uint32_t i = tid; i < m; i += nthr) NA[bitrev(i, logm)] = TP[m - 1 - i];
  __syncthreads();
  ntt1_lds(NA, m, logm, tw, tid, nthr);
  // Lagrange weights L_k(t) = NTT(t^(m-1-i))[k] * alpha^k / m (table entry 2m+1+k), Montgomery.
  uint8_t* wr = wrows.at(r);
  T lsum = FO::zero();
  for (uint32_t k = tid; k <= calls; k += nthr) {
    const T L = FO::mul(NA[k], FO::load(tw + (size_t)(2 * m + 1 + k) * ES));
    NA[k] = L;
    if (k >= 1) {
      lsum = FO::add(lsum, L);
      if (gi == 0) {
        FO::store(wr + (size_t)(W.mm + k - 1) * ES, FO::mul(L, RC[k - 1]));
        FO::store(wr + (size_t)(W.lm + k - 1) * ES, L);
      } else {
        FO::store(wr + (size_t)(W.l1 + k - 1) * ES, L);
      }
    }
  }
  // p(t) = sum_{d<m} c_d t^d + t^m sum_{d>=m} c_d t^(d-m);  gsum = sum_d c_d S[d mod m]
  bool bad = false;
  T plo = FO::zero(), phi = FO::zero(), gsum = FO::zero();
  for (uint32_t d = tid; d < gp_len; d += nthr) {
    const T cd = FO::load(pr + (size_t)(arity + d) * ES);
    bad |= !FO::is_canonical(cd);
    const uint32_t dm = d & (m - 1u);
    if (d < m) plo = FO::add(plo, FO::mul(TP[dm], cd));
    else phi = FO::add(phi, FO::mul(TP[dm], cd));
    gsum = FO::add(gsum, FO::mul(FO::load(tw + (size_t)(m + 1 + dm) * ES), cd));
  }
  T hsum = FO::zero();
  block_sum3<FO>(plo, phi, gsum, RED, tid, nthr);
  block_sum3<FO>(lsum, hsum, hsum, RED, tid, nthr);  // also orders the NA[k] = L writes
  const T L0 = NA[0], Lc = NA[calls];
  uint8_t* outp = prep.at(r);
  if (gi == 0) {
    const T half_l = FO::mul(lsum, FO::half());
    for (uint32_t j = tid; j < c; j += nthr) {
      const T s0 = FO::load(pr + (size_t)(2 * j) * ES);
      const T s1 = FO::load(pr + (size_t)(2 * j + 1) * ES);
      bad |= !FO::is_canonical(s0) || !FO::is_canonical(s1);
      FO::store(wr + (size_t)(W.rp + j) * ES, RP[j + 1]);
      FO::store(wr + (size_t)(W.b0 + j) * ES, FO::mul(L0, s0));
      FO::store(wr + (size_t)(W.b1 + j) * ES, FO::sub(FO::mul(L0, s1), half_l));
    }
  } else {
    // padded slots of the last call hold the share of the encoded zero: 2^(n-1) / 2 = 2^(n-2)
    const uint32_t rem = cfg.length - (calls - 1) * c;
    const uint32_t zb = cfg.bits - 2;
    const T z0 = FO::from_u64x2(zb < 64 ? 1ull << zb : 0ull, zb >= 64 ? 1ull << (zb - 64) : 0ull);
    const T pad = FO::mul(Lc, z0);
    for (uint32_t j = tid; j < c; j += nthr) {
      const T s = FO::load(pr + (size_t)j * ES);
      bad |= !FO::is_canonical(s);
      T v = FO::mul(L0, s);
      if (j >= rem) v = FO::add(v, pad);
      FO::store(wr + (size_t)(W.c1 + j) * ES, v);
    }
  }
  if (bad) atomicOr(flag, FPV_BAD_ENCODING);
  __syncthreads();
  if (tid == 0) {
    const T pt = FO::add(plo, FO::mul(tmm, phi));
    FO::store(wr + (size_t)(gi ? W.g1 : W.g0) * ES, gsum);
    const size_t pt_at = gi ? (size_t)(1 + cfg.arity + 1 + cfg.chunk1) : (size_t)(1 + cfg.arity);
    FO::store(outp + pt_at * ES, pt);
    if (*flag) atomicOr(&flags[r], *flag);
  }
}

// grid (ceil(c0/256), H, n), 256 threads: thread = column j, block row group h: calls k = 1+h+qH.
// part[(r*H + h)*c0 + j] = (sum_k MM_k x_idx, sum_k LM_k x_idx), idx = (k-1) c0 + j.
__global__ void __launch_bounds__(256) k_fpv_wires0(Cfg cfg, uint32_t n, uint32_t H, CRows meas,
                                                    CRows wrows, const uint8_t* status,
                                                    uint8_t* part, uint32_t* flags) {
  using FO = Field128Ops;
  const uint32_t r = blockIdx.z, h = blockIdx.y;
  if (r >= n || status[r] != ST_OK) return;
  const uint32_t c = cfg.chunk;
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= c) return;
  const FpvW W = fpv_w_layout(cfg);
  const uint8_t* xr = meas.at(r);
  const uint8_t* wr = wrows.at(r);
  Wide wa, wb;
  wide_zero(wa);
  wide_zero(wb);
  bool bad = false;
  for (uint32_t k = 1 + h; k <= cfg.calls; k += H) {
    const uint32_t idx = (k - 1) * c + j;
    if (idx >= cfg.meas_len) break;  // only the last call is partial
    const F128 x = FO::load(xr + (size_t)idx * 16u);
    bad |= !FO::is_canonical(x);
    wide_mac(wa, FO::load(wr + (size_t)(W.mm + k - 1) * 16u), x);
    wide_mac(wb, FO::load(wr + (size_t)(W.lm + k - 1) * 16u), x);
  }
  uint8_t* dst = part + (((size_t)r * H + h) * c + j) * 32u;
  FO::store(dst, wide_reduce(wa));
  FO::store(dst + 16, wide_reduce(wb));
  if (bad) atomicOr(&flags[r], FPV_BAD_ENCODING);
}

// grid (ceil(c1/256), n), 256 threads: wire1_j = C1[j] + sum_k L'_k z_((k-1) c1 + j) with
// z_e = sum_l 2^l x_(n e + l) (the entry decoded from its n bits).  Linearity moves the decoding
// into the weights: sum_k L'_k z_e = sum_k sum_l (2^l L'_k) x_(ne+l), so each bit is one lazily
// reduced MAC against a weight from an LDS table 2^l L'_k (built per k-chunk by doubling) -- n
// independent MACs per entry instead of a 2n-long serial double-and-add chain.
constexpr uint32_t kW1Tab = 4096;  // table entries (64 KiB) per k-chunk

__global__ void __launch_bounds__(256) k_fpv_wires1(Cfg cfg, uint32_t n, CRows meas, CRows wrows,
                                                    Rows prep, const uint8_t* status) {
  using FO = Field128Ops;
  __shared__ F128 tab[kW1Tab];
  const uint32_t r = blockIdx.y;
  if (r >= n || status[r] != ST_OK) return;  // block-uniform
  const uint32_t c = cfg.chunk1, nb = cfg.bits;
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  const FpvW W = fpv_w_layout(cfg);
  const uint8_t* xr = meas.at(r);
  const uint8_t* wr = wrows.at(r);
  const uint32_t kc = kW1Tab / nb;  // calls per table fill
  Wide acc;
  wide_zero(acc);
  for (uint32_t k0 = 1; k0 <= cfg.calls1; k0 += kc) {
    const uint32_t k1 = min(cfg.calls1 + 1u, k0 + kc);
    __syncthreads();  // the previous chunk's table is no longer read
    for (uint32_t k = k0 + threadIdx.x; k < k1; k += blockDim.x) {
      F128 w = FO::load(wr + (size_t)(W.l1 + k - 1) * 16u);  // L'_k (Montgomery)
      F128* t = tab + (size_t)(k - k0) * nb;
      for (uint32_t l = 0; l < nb; ++l) {
        t[l] = w;
        w = FO::dbl(w);
      }
    }
    __syncthreads();
    if (j < c) {
      for (uint32_t k = k0; k < k1; ++k) {
        const uint32_t e = (k - 1) * c + j;
        if (e >= cfg.length) break;
        const uint8_t* xe = xr + (size_t)e * nb * 16u;
        const F128* t = tab + (size_t)(k - k0) * nb;
        for (uint32_t l0 = 0; l0 < nb; l0 += 8) {
          F128 xb[8];
#pragma unroll
          for (uint32_t u = 0; u < 8; ++u) xb[u] = FO::load(xe + (size_t)(l0 + u) * 16u);
#pragma unroll
          for (uint32_t u = 0; u < 8; ++u) wide_mac(acc, t[l0 + u], xb[u]);
        }
      }
    }
  }
  if (j >= c) return;
  const F128 w = FO::add(FO::load(wr + (size_t)(W.c1 + j) * 16u), wide_reduce(acc));
  FO::store(prep.at(r) + (size_t)(1 + cfg.arity + 1 + j) * 16u, w);
}

// grid (ceil(c0/256), n), 256 threads: wires0 from the row-group partials; block x = 0 also writes
// v, the joint-rand part and the report's status.
__global__ void __launch_bounds__(256) k_fpv_finalize(Cfg cfg, uint32_t n, uint32_t H, CRows meas,
                                                      CRows wrows, CRows jr, CRows part_in,
                                                      const uint8_t* part, Rows prep,
                                                      uint8_t* status, const uint32_t* flags) {
  using FO = Field128Ops;
  const uint32_t r = blockIdx.y;
  if (r >= n || status[r] != ST_OK) return;
  const uint32_t c = cfg.chunk;
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  const FpvW W = fpv_w_layout(cfg);
  const uint8_t* wr = wrows.at(r);
  uint8_t* outp = prep.at(r);
  if (j < c) {
    F128 a = FO::zero(), b = FO::zero();
    for (uint32_t h = 0; h < H; ++h) {
      const uint8_t* src = part + (((size_t)r * H + h) * c + j) * 32u;
      a = FO::add(a, FO::load(src));
      b = FO::add(b, FO::load(src + 16));
    }
    const F128 w0 = FO::add(FO::load(wr + (size_t)(W.b0 + j) * 16u),
                            FO::mul(FO::load(wr + (size_t)(W.rp + j) * 16u), a));
    const F128 w1 = FO::add(FO::load(wr + (size_t)(W.b1 + j) * 16u), b);
    FO::store(outp + (size_t)(1 + 2 * j) * 16u, w0);
    FO::store(outp + (size_t)(2 + 2 * j) * 16u, w1);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    // submitted norm = sum_l 2^l x_(n entries + l), l < 2n - 2
    const uint8_t* xn = meas.at(r) + (size_t)cfg.bits * cfg.length * 16u;
    F128 sn = FO::zero();
    for (int l = (int)(2 * cfg.bits - 3); l >= 0; --l)
      sn = FO::add(FO::dbl(sn), FO::load(xn + (size_t)l * 16u));
    const F128 r1 = FO::to_mont(FO::load(jr.at(r) + 16));
    const F128 norm_check = FO::sub(FO::load(wr + (size_t)W.g1 * 16u), sn);
    const F128 v = FO::add(FO::mul(r1, FO::load(wr + (size_t)W.g0 * 16u)),
                           FO::mul(FO::mul(r1, r1), norm_check));
    FO::store(outp, v);
    const uint8_t* pp = part_in.at(r);
    uint8_t* dst = outp + (size_t)cfg.verifier_len * 16u;
    st64(dst, ld64(pp));
    st64(dst + 8, ld64(pp + 8));
    const uint32_t f = flags[r];
    if (f & FPV_BAD_ENCODING) status[r] = ST_INVALID_MESSAGE;
    else if (f & FPV_ROOT_OF_UNITY) status[r] = ST_VDAF_PREP_ERROR;
  }
}

// prepare_shares_to_prepare_message for FixedPointBoundedL2VecSum: block per report.
//   G0 = sum_j w_2j w_2j+1 (ParallelSum(Mul)),  G1 = sum_j (w_j^2 - 2^n w_j + 2^(2n-2)).
__global__ void __launch_bounds__(256) k_fpv_decide(Cfg cfg, uint32_t n, CRows leader_prep,
                                                    CRows helper_prep, Rows out_msg,
                                                    uint8_t* status) {
  using FO = Field128Ops;
  using T = F128;
  __shared__ T red[12];
  __shared__ uint32_t sbad;
  const uint32_t r = blockIdx.x;
  if (r >= n || status[r] != ST_OK) return;
  const uint32_t tid = threadIdx.x, nthr = blockDim.x;
  if (tid == 0) sbad = 0u;
  __syncthreads();
  const uint8_t* a = leader_prep.at(r);
  const uint8_t* b = helper_prep.at(r);
  const uint32_t nb = cfg.bits;
  // 2^n (Montgomery) and 2^(2n-2) (canonical)
  const T k1 = FO::to_mont(FO::from_u64x2(nb < 64 ? 1ull << nb : 0ull, nb >= 64 ? 1ull : 0ull));
  const uint32_t e2 = 2 * nb - 2;
  const T k0 = FO::from_u64x2(e2 < 64 ? 1ull << e2 : 0ull, e2 >= 64 ? 1ull << (e2 - 64) : 0ull);
  bool bad = false;
  auto wire = [&](uint32_t i) {
    const T x = FO::load(a + (size_t)i * 16u), y = FO::load(b + (size_t)i * 16u);
    bad |= !FO::is_canonical(x) || !FO::is_canonical(y);
    return FO::add(x, y);
  };
  T g0 = FO::zero(), g1 = FO::zero(), z = FO::zero();
  for (uint32_t j = tid; j < cfg.chunk; j += nthr) {
    const T w0 = wire(1 + 2 * j), w1 = wire(2 + 2 * j);
    g0 = FO::add(g0, FO::mul(FO::to_mont(w0), w1));
  }
  const uint32_t base1 = 1 + cfg.arity + 1;
  for (uint32_t j = tid; j < cfg.chunk1; j += nthr) {
    const T w = wire(base1 + j);
    g1 = FO::add(g1, FO::add(FO::sub(FO::mul(FO::to_mont(w), w), FO::mul(k1, w)), k0));
  }
  if (bad) atomicOr(&sbad, 1u);
  block_sum3<FO>(g0, g1, z, red, tid, nthr);
  if (tid != 0) return;
  const T v = wire(0), p0 = wire(1 + cfg.arity), p1 = wire(base1 + cfg.chunk1);
  const bool ok = !sbad && !bad && FO::is_zero(v) && FO::eq(g0, p0) && FO::eq(g1, p1);
  if (!ok) {
    status[r] = ST_VDAF_PREP_ERROR;
    return;
  }
  const uint8_t* pa = a + (size_t)cfg.verifier_len * 16u;
  const uint8_t* pb = b + (size_t)cfg.verifier_len * 16u;
  uint64_t lo, hi;
  derive_jr_seed(cfg.xof, cfg.algo_id, ld64(pa), ld64(pa + 8), ld64(pb), ld64(pb + 8), lo, hi);
  st64(out_msg.at(r), lo);
  st64(out_msg.at(r) + 8, hi);
}

}  // namespace p3g
