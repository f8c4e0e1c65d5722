// Config E chains on lane PAIRS (engine option pair_chains, keccak_pair.h): the FixedPoint
// helper's two 152K-permutation chains per report (k_helper_xof_pair) and the leader's joint-rand
// chain (k_jr_ring_pair) with each sponge state spread bit-interleaved over two lanes, 32 reports
// per sponge wave.  A lone wave issues a VALU every ~4 cycles whatever its lane count, so the
// chain's length is its instruction count: 4.87 vs 9.40 us per permutation at one wave per SIMD
// (tools/mb_pair.hip, profiles/r05/pair/).  The byte stream, the ring handoff and the outputs are
// k_helper_xof's / k_jr_ring's (fpvec_kernels.h); only the sponge words are halves:
//   * the producer squeezes halves into its ring; the consumer absorbs them as they are (the
//     joint-rand message's 2-byte misalignment, (D[j] >> 48) | (D[j+1] << 16), is one alignbit by
//     24 on each half); the storer zips each row's words back to 64 bits for the canonical checks,
//     the rows and the column sums;
//   * snapshots keep the state as 25 (even half, odd half) dword pairs (k_fpv_regen<true>);
//   * the leader's loader unzips each share word into the two halves its sponge absorbs.
// Spec column sums keep the 64-row groups of k_jr's layout (one storer / loader per 64 rows).
#pragma once
#include "fpvec_kernels.h"
#include "keccak_pair.h"

namespace p3g {

// Ring counters of k_jr_ring_pair through ds instructions (ctr_ld / ctr_st): its leader chains
// ran 1,037 -> 975 ms at 10,752 reports against the FLAT form k_jr_ring keeps
// (profiles/r05/pair/r5_pair5).
#ifndef P3G_JRP_CTR_LDS
#define P3G_JRP_CTR_LDS 1
#endif
constexpr bool kJrpLds = P3G_JRP_CTR_LDS != 0;

// The ring counters are LDS words written with ds_write after the slot accesses they publish, and
// one wave's LDS operations are performed in order: a publish needs no s_waitcnt before it, and a
// sponge reads a slot's 21 words (the block's 16 and the next carry) in one go and releases the
// slot at once (P3G_PAIR_NOWAIT 0: the waits of k_helper_xof / k_jr_ring, for A/B).
#ifndef P3G_PAIR_NOWAIT
#define P3G_PAIR_NOWAIT 1
#endif
#if P3G_PAIR_NOWAIT
#define P3G_PAIR_PUBLISH_WAIT() asm volatile("" ::: "memory")
#else
#define P3G_PAIR_PUBLISH_WAIT() asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory")
#endif

// P3G_JRP_PREFETCH 1: k_jr_ring_pair's loaders load block i + 1's share words while they unzip
// and publish block i (0: load, wait, unzip in turn; A/B)
#ifndef P3G_JRP_PREFETCH
#define P3G_JRP_PREFETCH 1
#endif

constexpr uint32_t kPrRows = 32;                 // reports per sponge wave (two lanes each)
constexpr uint32_t kPrStride = 65;               // ring row pitch (dwords): conflict-free columns
constexpr uint32_t kPrSlot = 21 * kPrStride;     // dwords per ring slot
constexpr size_t kPrRingBytes = (size_t)kHxDepth * kPrSlot * 4;  // one sponge's ring
constexpr size_t kPrStageBytes = (size_t)21 * (kHxRows + 1) * 8;  // 64 rows of 64-bit words
// dynamic LDS of the two kernels' workgroups (64 and 128 reports)
constexpr size_t kHxPairLds = 2 * kPrRingBytes + kPrStageBytes;
constexpr size_t kJrPairLds = 4 * kPrRingBytes + 2 * kPrStageBytes;

// jrp_absorb on halves: pre = the halves of the block-0 prefix words, carry / A the halves of the
// share words, padh / lasth this lane's halves of the padding and the final bit.
DEVI void jrp_absorb_pair(uint32_t s[25], const uint32_t carry[6], const uint32_t A[16], int64_t b,
                          int64_t nblocks, int64_t padw, uint32_t padh, uint32_t lasth,
                          const uint32_t pre[5]) {
#pragma unroll
  for (int w = 0; w < 21; ++w) {
    uint32_t v;
    if (b == 0 && w < 5) {
      v = pre[w];
    } else {
      const uint32_t dlo = w <= 5 ? carry[w] : A[w - 6];
      const uint32_t dhi = w <= 4 ? carry[w + 1] : A[w - 5];
      v = abit(dhi, dlo, 24);  // (dlo >> 48) | (dhi << 16) on each half
    }
    if (padw == 21 * b + w) v ^= padh;
    if (b == nblocks - 1 && w == 20) v ^= lasth;
    s[w] ^= v;
  }
}

// The halves of a joint-rand-part message's first five words: header(blind) || agg_id || nonce.
DEVI void jrp_prefix_pair(const Cfg& cfg, uint32_t agg_id, const uint8_t* blind,
                          const uint8_t* nonce, uint32_t p, uint32_t pre[5]) {
  MsgBlock m;
  m.clear();
  m.header(cfg.algo_id, DST_JOINT_RAND_PART, ld64(blind), ld64(blind + 8));
  m.put8(25, agg_id);
  m.put64(26, ld64(nonce));
  m.put64(34, ld64(nonce + 8));
#pragma unroll
  for (int w = 0; w < 5; ++w) pre[w] = kp_half(m.w[w], p);
}

// The joint-rand tail of a finished part sponge (both lanes of a pair call it; the even lane
// stores): part = the first 16 squeezed bytes, then seed and joint randomness (k_jr_ring's tail).
DEVI void jrp_finish_pair(const Cfg& cfg, const uint32_t s[25], const KpLane& ln, bool live,
                          uint32_t r, uint32_t agg_id, CRows public_shares, Rows out_part,
                          Rows out_seed, Rows out_jr) {
  using FO = Field128Ops;
  const uint64_t plo = kp_merge(s[0], ln), phi = kp_merge(s[1], ln);
  if (!live || ln.p) return;
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

// The storer's speculative column sums of one block (k_helper_xof's layout): stage = the block's
// 21 words x 64 rows (row pitch kHxRows + 1), lane = word wc + 21 gq summing rows gq, gq + 3, ..
DEVI void pair_column_sums(const uint64_t* stage, uint32_t lane, uint32_t r0, int64_t j0,
                           int64_t nd, uint64_t* spec_lo, uint8_t* spec_cy) {
  constexpr uint32_t kS = kHxRows + 1;
  const uint32_t gq = lane / 21u, wc = lane - 21u * gq;
  const uint64_t* col = stage + (gq < 3u ? wc : 0u) * kS;
  uint32_t l32 = 0, h32 = 0, cy = 0;
#pragma unroll
  for (int k = 0; k < 22; ++k) {
    const uint32_t row = gq + 3u * (uint32_t)k;
    acc_u64(l32, h32, cy, (gq < 3u && row < 64u) ? col[row] : 0ull);
  }
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

// Helper: one workgroup = 64 reports = waves {producer 0, producer 1, consumer 0, consumer 1,
// storer}; producer / consumer h take reports r0 + 32 h + (lane >> 1), the storer every row.
// Ring h (dynamic LDS) carries producer h's squeezed halves to consumer h and the storer.
template <uint32_t kDepth>
__global__ void __launch_bounds__(5 * kHxRows) k_helper_xof_pair(Cfg cfg, uint32_t n, CRows helper_shares,
                                                  CRows nonces, CRows public_shares,
                                                  Rows out_meas, Rows out_proof, Rows out_part,
                                                  Rows out_seed, Rows out_jr,
                                                  const uint8_t* status, uint32_t* fallback,
                                                  uint64_t* spec_lo, uint8_t* spec_cy,
                                                  uint64_t* snaps) {
  using FO = Field128Ops;
  static_assert(kDepth == kHxDepth, "kPrRingBytes assumes kHxDepth slots");
  extern __shared__ __attribute__((aligned(16))) uint64_t hp_dyn[];
  __shared__ uint32_t counters[6];  // per ring: produced, consumed, stored
  uint32_t* rings = reinterpret_cast<uint32_t*>(hp_dyn);
  uint64_t* stage = reinterpret_cast<uint64_t*>(rings + 2 * kDepth * kPrSlot);
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  if (threadIdx.x < 6) counters[threadIdx.x] = 0u;
  __syncthreads();
  const uint32_t r0 = blockIdx.x * kHxRows;
  if (r0 >= n) return;
  const bool producer = wave < 2u, storer = wave == 4u;
  // wave_prio 1: the sponge waves first on their SIMDs (the storer shares one); 2: every wave
  if (cfg.wave_prio == 2u || (cfg.wave_prio == 1u && !storer)) __builtin_amdgcn_s_setprio(3);
  const uint32_t h = wave & 1u;  // the sponge waves' ring
  const uint32_t p = lane & 1u;
  const KpLane ln = kp_lane(p);
  // sponge waves: report r0 + 32 h + lane / 2; the storer: row r0 + lane
  const uint32_t r = storer ? r0 + lane : r0 + kPrRows * h + (lane >> 1);
  const bool live = r < n && (!status || status[r] == ST_OK);
  const uint32_t rr = r < n ? r : n - 1u;
  const uint8_t* hs = helper_shares.at(rr);
  const int64_t nd = (int64_t)cfg.meas_len * 2;
  const int64_t total = 42 + 8 * nd;
  const int64_t nblocks = total / 168 + 1;
  const int64_t nprod = (nd + 20) / 21;
  const int64_t padw = total >> 3;
  const uint32_t padh = kp_half((uint64_t)cfg.xof.pad << ((total & 7) * 8), p);
  const uint32_t lasth = 0x80000000u & ln.pm;
  uint32_t* ring = rings + (size_t)h * (kDepth * kPrSlot);
  uint32_t s[25];
  uint32_t pre[5] = {0u, 0u, 0u, 0u, 0u};
  uint32_t carry[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) carry[i] = 0u;
  if (producer) {
    MsgBlock m;
    m.clear();
    m.header(cfg.algo_id, DST_MEASUREMENT_SHARE, ld64(hs), ld64(hs + 8));
    m.put8(25, 1u);
    m.pad(26, cfg.xof);
#pragma unroll
    for (int i = 0; i < 25; ++i) s[i] = i < kRateWords ? kp_half(m.w[i], p) : 0u;
    keccak_pair_x(s, ln, cfg.xof);  // s = expansion block 0
  } else {
#pragma unroll
    for (int i = 0; i < 25; ++i) s[i] = 0u;
    if (!storer) {
      jrp_prefix_pair(cfg, 1u, hs + 32, nonces.at(rr), p, pre);
      carry[5] = kp_half(ld64(nonces.at(rr) + 8), p);
    }
  }
  bool bad = false;
  uint8_t* om = out_meas.at(rr);
  const uint32_t nsnap = snap_count(cfg);
  const int64_t iters = producer || storer ? nprod : nblocks;
  for (int64_t i = 0; i < iters; ++i) {
    bool perm = true;
    if (producer) {
      const int64_t j0 = 21 * i;
      if (snaps != nullptr && (i % kSnapEvery) == 0 && r < n) {
        uint32_t* sp = reinterpret_cast<uint32_t*>(snaps + ((size_t)r * nsnap + (size_t)(i / kSnapEvery)) * 25);
#pragma unroll
        for (int w = 0; w < 25; ++w) sp[2 * w + p] = s[w];
      }
      while (i - (int64_t)min(ctr_ld<true>(&counters[3 * h + 1]), ctr_ld<true>(&counters[3 * h + 2])) >=
             (int64_t)kDepth)
        __builtin_amdgcn_s_sleep(1);
      asm volatile("" ::: "memory");
      uint32_t* slot = ring + (i % kDepth) * kPrSlot;
#pragma unroll
      for (int w = 0; w < 21; ++w) slot[w * kPrStride + lane] = j0 + w < nd ? s[w] : 0u;
      P3G_PAIR_PUBLISH_WAIT();  // slot written before it is published
      ctr_st<true>(&counters[3 * h], (uint32_t)(i + 1));
      perm = 21 * (i + 1) < nd;
    } else if (storer) {
      const int64_t j0 = 21 * i;
      while ((int64_t)min(ctr_ld<true>(&counters[0]), ctr_ld<true>(&counters[3])) <= i)
        __builtin_amdgcn_s_sleep(1);
      asm volatile("" ::: "memory");
      // this row's halves: ring (row >> 5), lanes 2 (row & 31) and 2 (row & 31) + 1
      const uint32_t* slot = rings + (size_t)(lane >> 5) * (kDepth * kPrSlot) + (i % kDepth) * kPrSlot +
                             2u * (lane & 31u);
      uint32_t he[21], ho[21];
#pragma unroll
      for (int w = 0; w < 21; ++w) {
        he[w] = slot[w * kPrStride];
        ho[w] = slot[w * kPrStride + 1];
      }
      P3G_PAIR_PUBLISH_WAIT();  // slots read before they are released
      ctr_st<true>(&counters[2], (uint32_t)(i + 1));
      ctr_st<true>(&counters[5], (uint32_t)(i + 1));
      uint64_t x[21];
#pragma unroll
      for (int w = 0; w < 21; ++w)
        x[w] = kp_zip(he[w], ho[w]);
      if (spec_lo != nullptr) {
#pragma unroll
        for (int w = 0; w < 21; ++w) stage[w * (kHxRows + 1) + lane] = x[w];
        // this wave's own LDS writes complete before its reads below (in-order LDS)
        pair_column_sums(stage, lane, r0, j0, nd, spec_lo, spec_cy);
      }
      const bool st_row = snaps != nullptr ? false : spec_lo != nullptr ? r < n : live;
      if (j0 + 21 <= nd) {
        if (st_row) {
          uint8_t* o = om + 8 * j0;
          if ((i & 1) == 0) {
#pragma unroll
            for (int w = 0; w < 20; w += 2)
              *reinterpret_cast<ulonglong2*>(o + 8 * w) = make_ulonglong2(x[w], x[w + 1]);
            st64(o + 160, x[20]);
          } else {
            st64(o, x[0]);
#pragma unroll
            for (int w = 1; w < 21; w += 2)
              *reinterpret_cast<ulonglong2*>(o + 8 * w) = make_ulonglong2(x[w], x[w + 1]);
          }
        }
#pragma unroll
        for (int w = 0; w < 21; ++w)
          if (((j0 + w) & 1) && !hi_ok(x[w])) bad = true;
      } else {
#pragma unroll
        for (int w = 0; w < 21; ++w) {
          const bool in = j0 + w < nd;
          if (in && st_row) st64(om + 8 * (j0 + w), x[w]);
          if (in && ((j0 + w) & 1) && !hi_ok(x[w])) bad = true;
        }
      }
      perm = false;
    } else {
      const int64_t b = i;
      const bool data = 21 * b < nd;
      uint32_t A[16], nc[6];
      if (data) {
        while ((int64_t)ctr_ld<true>(&counters[3 * h]) <= b) __builtin_amdgcn_s_sleep(1);
        asm volatile("" ::: "memory");
        const uint32_t* slot = ring + (b % kDepth) * kPrSlot;
#pragma unroll
        for (int w = 0; w < 16; ++w) A[w] = slot[w * kPrStride + lane];
#pragma unroll
        for (int k = 1; k < 6; ++k) nc[k] = slot[(15 + k) * kPrStride + lane];
        nc[0] = A[15];
        P3G_PAIR_PUBLISH_WAIT();  // slot read before it is released
        ctr_st<true>(&counters[3 * h + 1], (uint32_t)(b + 1));
      } else {
#pragma unroll
        for (int w = 0; w < 16; ++w) A[w] = 0u;
#pragma unroll
        for (int k = 0; k < 6; ++k) nc[k] = 0u;
      }
      jrp_absorb_pair(s, carry, A, b, nblocks, padw, padh, lasth, pre);
#pragma unroll
      for (int k = 0; k < 6; ++k) carry[k] = nc[k];
    }
    if (perm) keccak_pair_x(s, ln, cfg.xof);
  }
  if (storer) {
    if (live && bad) atomicAdd(fallback, 1u);
    return;
  }
  if (producer) {
    if (live && p == 0u)
      xof_expand_byte_binder<FO>(cfg.algo_id, DST_PROOF_SHARE, ld64(hs + 16), ld64(hs + 24), 1u,
                                 cfg.proof_len, out_proof.at(r), cfg.xof, cfg.exact_squeeze);
    return;
  }
  jrp_finish_pair(cfg, s, ln, live, r, 1u, public_shares, out_part, out_seed, out_jr);
}

// Leader: one workgroup = 128 reports = waves {sponge 0..3, loader 0, loader 1}; sponge g takes
// reports r0 + 32 g + (lane >> 1), loader L rows r0 + 64 L + lane (sponges 2L and 2L + 1).  The
// loader unzips each share word into the two halves of its sponge's ring and keeps the 64-bit
// words in its stage for the column sums (k_jr_ring's layout).
__global__ void __launch_bounds__(6 * kHxRows) k_jr_ring_pair(Cfg cfg, uint32_t n, uint32_t agg_id,
                                                CRows nonces, CRows public_shares,
                                                CRows blinds, CRows meas, Rows out_part,
                                                Rows out_seed, Rows out_jr,
                                                const uint8_t* status, uint64_t* spec_lo,
                                                uint8_t* spec_cy) {
  extern __shared__ __attribute__((aligned(16))) uint64_t jp_dyn[];
  __shared__ uint32_t counters[8];  // per sponge ring: produced, consumed
  uint32_t* rings = reinterpret_cast<uint32_t*>(jp_dyn);
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  if (threadIdx.x < 8) counters[threadIdx.x] = 0u;
  __syncthreads();
  const uint32_t rb = blockIdx.x * (2 * kHxRows);
  if (rb >= n) return;
  const bool loader = wave >= 4u;
  if (cfg.wave_prio == 2u || (cfg.wave_prio == 1u && !loader)) __builtin_amdgcn_s_setprio(3);
  const uint32_t L = loader ? wave & 1u : wave >> 1;  // the 64-row group (a loader's, a sponge's)
  // a group wholly past the batch: its loader and both its sponges leave (no spec column-sum
  // group exists for it); a partial group runs on clamped rows like k_jr_ring
  if (rb + kHxRows * L >= n) return;
  const uint32_t p = lane & 1u;
  const KpLane ln = kp_lane(p);
  const uint32_t r = loader ? rb + kHxRows * L + lane : rb + kPrRows * wave + (lane >> 1);
  const bool live = r < n && (!status || status[r] == ST_OK);
  const uint32_t rr = r < n ? r : n - 1u;
  const int64_t nd = (int64_t)cfg.meas_len * 2;
  const int64_t total = 42 + 8 * nd;
  const int64_t nblocks = total / 168 + 1;
  const int64_t nprod = (nd + 20) / 21;
  const int64_t padw = total >> 3;
  const uint32_t padh = kp_half((uint64_t)cfg.xof.pad << ((total & 7) * 8), p);
  const uint32_t lasth = 0x80000000u & ln.pm;
  uint32_t s[25];
#pragma unroll
  for (int i = 0; i < 25; ++i) s[i] = 0u;
  uint32_t pre[5] = {0u, 0u, 0u, 0u, 0u};
  uint32_t carry[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) carry[i] = 0u;
  if (!loader) {
    jrp_prefix_pair(cfg, agg_id, blinds.at(rr), nonces.at(rr), p, pre);
    carry[5] = kp_half(ld64(nonces.at(rr) + 8), p);
  }
  const uint8_t* data = meas.at(rr);
  // loader: its row's sponge ring and lane pair; its stage
  const uint32_t sg = 2u * L + (lane >> 5);
  uint32_t* lring = rings + (size_t)sg * (kHxDepth * kPrSlot) + 2u * (lane & 31u);
  uint64_t* stage = reinterpret_cast<uint64_t*>(rings + 4 * kHxDepth * kPrSlot) +
                    (size_t)L * (21 * (kHxRows + 1));
  uint32_t* ring = rings + (size_t)wave * (kHxDepth * kPrSlot);  // a sponge's own ring
  // share words [21 i, 21 i + 21) of the loader's row (zeros past the share)
  auto load_block = [&](int64_t i, uint64_t x[21]) {
    const int64_t j0 = 21 * i;
    const uint8_t* src = data + 8 * j0;
    if (j0 + 21 <= nd) {
      if ((i & 1) == 0) {  // whole block: 16-B loads (block i starts 16-B aligned iff i even)
#pragma unroll
        for (int w = 0; w < 20; w += 2) {
          const ulonglong2 v = *reinterpret_cast<const ulonglong2*>(src + 8 * w);
          x[w] = v.x;
          x[w + 1] = v.y;
        }
        x[20] = ld64(src + 160);
      } else {
        x[0] = ld64(src);
#pragma unroll
        for (int w = 1; w < 21; w += 2) {
          const ulonglong2 v = *reinterpret_cast<const ulonglong2*>(src + 8 * w);
          x[w] = v.x;
          x[w + 1] = v.y;
        }
      }
    } else {
#pragma unroll
      for (int w = 0; w < 21; ++w) x[w] = j0 + w < nd ? ld64(src + 8 * w) : 0ull;
    }
  };
  uint64_t xn[21];
  if (P3G_JRP_PREFETCH && loader) load_block(0, xn);
  const int64_t iters = loader ? nprod : nblocks;
  for (int64_t i = 0; i < iters; ++i) {
    bool perm = true;
    if (loader) {
      const int64_t j0 = 21 * i;
      uint64_t x[21];
      if (P3G_JRP_PREFETCH) {
#pragma unroll
        for (int w = 0; w < 21; ++w) x[w] = xn[w];
        if (i + 1 < iters) load_block(i + 1, xn);  // in flight under this block's work
      } else {
        load_block(i, x);
      }
      uint32_t he[21], ho[21];
#pragma unroll
      for (int w = 0; w < 21; ++w) kp_unzip(x[w], he[w], ho[w]);
      while (i - (int64_t)min(ctr_ld<kJrpLds>(&counters[2 * (2 * L) + 1]),
                              ctr_ld<kJrpLds>(&counters[2 * (2 * L + 1) + 1])) >= (int64_t)kHxDepth)
        __builtin_amdgcn_s_sleep(P3G_JR_LOADER_SLEEP);
      asm volatile("" ::: "memory");
      uint32_t* slot = lring + (i % kHxDepth) * kPrSlot;
#pragma unroll
      for (int w = 0; w < 21; ++w) {
        slot[w * kPrStride] = he[w];
        slot[w * kPrStride + 1] = ho[w];
      }
      if (!kJrpLds) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // FLAT counters
      P3G_PAIR_PUBLISH_WAIT();  // slots written before they are published
      ctr_st<kJrpLds>(&counters[2 * (2 * L)], (uint32_t)(i + 1));
      ctr_st<kJrpLds>(&counters[2 * (2 * L + 1)], (uint32_t)(i + 1));
      if (spec_lo != nullptr) {
#pragma unroll
        for (int w = 0; w < 21; ++w) stage[w * (kHxRows + 1) + lane] = x[w];
        pair_column_sums(stage, lane, rb + kHxRows * L, j0, nd, spec_lo, spec_cy);
      }
      perm = false;
    } else {
      const int64_t b = i;
      const bool has = 21 * b < nd;
      uint32_t A[16], nc[6];
      if (has) {
        while ((int64_t)ctr_ld<kJrpLds>(&counters[2 * wave]) <= b) __builtin_amdgcn_s_sleep(1);
        asm volatile("" ::: "memory");
        const uint32_t* slot = ring + (b % kHxDepth) * kPrSlot;
#pragma unroll
        for (int w = 0; w < 16; ++w) A[w] = slot[w * kPrStride + lane];
#pragma unroll
        for (int k = 1; k < 6; ++k) nc[k] = slot[(15 + k) * kPrStride + lane];
        nc[0] = A[15];
        if (!kJrpLds || !P3G_PAIR_NOWAIT)  // FLAT counters: the reads must have returned
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        asm volatile("" ::: "memory");
        ctr_st<kJrpLds>(&counters[2 * wave + 1], (uint32_t)(b + 1));
      } else {
#pragma unroll
        for (int w = 0; w < 16; ++w) A[w] = 0u;
#pragma unroll
        for (int k = 0; k < 6; ++k) nc[k] = 0u;
      }
      jrp_absorb_pair(s, carry, A, b, nblocks, padw, padh, lasth, pre);
#pragma unroll
      for (int k = 0; k < 6; ++k) carry[k] = nc[k];
    }
    if (perm) keccak_pair_x(s, ln, cfg.xof);
  }
  if (loader) return;
  jrp_finish_pair(cfg, s, ln, live, r, agg_id, public_shares, out_part, out_seed, out_jr);
}

}  // namespace p3g
