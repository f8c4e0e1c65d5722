// The helper's two measurement-share sponges in one pass (k_helper_sponge, Field128 types with
// joint randomness: Sum, SumVec, Histogram).
//
// prio's helper prepare_init (Share::Helper arm, reached from aggregator.rs:1775-1797) expands
// its measurement share  XOF(k_meas, dst1, [1]).next_vec(MEAS)  and then hashes the encoded share
// into its joint-rand part  derive_seed(blind, dst7, [1] || nonce || encode(meas share)).  Run as
// k_expand then k_jr that is two sponges over the same 128 KB per report, with the share written
// to HBM, read back through LDS-DMA windows and column-summed there.  Here one lane runs both
// sponges over each 168-byte block while it is still in registers:
//
//   S1: expansion sponge (squeeze).   S2: joint-rand-part sponge (absorb).
//   step 2b   : S1 holds stream block b -> store its elements, column-sum its words (speculative
//               accumulation, k_jr's layout and word range), absorb message block b into S2
//               (stream words [21b-6, 21b+15], the 42-byte prefix puts share word j at message
//               byte 42 + 8j; words 15..20 carry to the next block), then permute S2
//   step 2b+1 : permute S1 (stream block b+1)
// ONE inlined Keccak-f serves both: every step swaps the two states and permutes the first
// (a second inlined copy would overflow the instruction cache).
//
// Exactness: when every squeezed element is canonical (< p; fails with probability ~28/2^64 per
// element) the encoded share IS the stream, so S2 absorbs the stream words directly.  A lane that
// meets a non-canonical element sets *fallback; k_expand and k_jr then run gated on that flag
// (they return at once when it is 0) and recompute the whole batch on the exact path, so the
// outputs are identical either way.  Rows past n run the last report (clamped, like k_jr's
// cooperative window) so the column sums carry the same duplicates k_accum_spec subtracts; they
// store nothing.
#pragma once
#include "fpvec_kernels.h"

namespace p3g {

#ifndef P3G_TEST_FORCE_FALLBACK
#define P3G_TEST_FORCE_FALLBACK 0
#endif

__global__ void __launch_bounds__(256) k_helper_sponge(Cfg cfg, uint32_t n, CRows helper_shares,
                                                       CRows nonces, CRows public_shares,
                                                       Rows out_meas, Rows out_proof, Rows out_part,
                                                       Rows out_seed, Rows out_jr,
                                                       const uint8_t* status, uint32_t* fallback,
                                                       uint64_t* spec_lo, uint8_t* spec_cy,
                                                       uint32_t spec_w0, uint32_t spec_w1,
                                                       uint32_t force_fallback) {
  using FO = Field128Ops;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t tid = threadIdx.x, lane = tid & 63u;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t r0w = blockIdx.x * blockDim.x + 64u * wv;
  if (r0w >= n) return;  // wave-uniform
  const uint32_t r = r0w + lane;
  const bool in = r < n;
  const bool live = in && (!status || status[r] == ST_OK);
  const uint32_t rr = in ? r : n - 1u;
  uint8_t* win = smem + wv * kJrWaveLds;  // this wave's 64 rows x 176 B (21 words used)
  const uint8_t* hs = helper_shares.at(rr);

  // proof share first (42 permutations for SumVec), as k_expand does
  if (in)
    xof_expand_byte_binder<FO>(cfg.algo_id, DST_PROOF_SHARE, ld64(hs + 16), ld64(hs + 24), 1u,
                               cfg.proof_len, out_proof.at(r), cfg.xof, false);

  const uint32_t nelem = cfg.meas_len;
  const int64_t nd = (int64_t)nelem * 2;        // share words
  const int64_t total = 42 + nd * 8;            // joint-rand-part message bytes before padding
  const int64_t nblocks = total / 168 + 1;      // its rate blocks
  const int64_t padw = total >> 3;
  const uint64_t padv = (uint64_t)cfg.xof.pad << ((total & 7) * 8);
  const uint8_t* nz = nonces.at(rr);
  const uint8_t* blind = hs + 32;

  uint64_t a[25], o[25];  // a: the state the next permutation runs on; o: the other one
  {
    MsgBlock m;
    m.clear();
    m.header(cfg.algo_id, DST_MEASUREMENT_SHARE, ld64(hs), ld64(hs + 8));
    m.put8(25, 1u);
    m.pad(26, cfg.xof);
    sponge_one_block(a, m, cfg.xof);  // S1 = stream block 0
  }
#pragma unroll
  for (int i = 0; i < 25; ++i) o[i] = 0ull;  // S2
  uint64_t carry[6];
#pragma unroll
  for (int i = 0; i < 5; ++i) carry[i] = 0ull;
  carry[5] = ld64(nz + 8);  // block 0: the nonce's high word precedes share word 0
  uint8_t* mout = out_meas.at(in ? r : 0u);
  uint32_t cnt = 0;        // elements stored
  uint64_t half = 0;       // low word of the element straddling two blocks
  bool bad = force_fallback != 0u;

  for (int64_t step = 0; step < 2 * nblocks - 1; ++step) {
    if ((step & 1) == 0) {  // wave-uniform: S1 = a holds stream block b, S2 = o
      const int64_t b = step >> 1;
      const int64_t w0 = 21 * b;  // first share word of this stream block
      if (w0 < nd) {
        // store the block's elements (even b: 10 whole + the low half of the next; odd b: the
        // carried low half + word 0, then 10 whole); only elements < MEAS, canonical ones only
        bool ok = true;
        if ((b & 1) == 0) {
#pragma unroll
          for (int k = 0; k < 10; ++k) {
            if (cnt + k < nelem) {
              ok &= hi_ok(a[2 * k + 1]);
              if (in)
                *reinterpret_cast<ulonglong2*>(mout + (size_t)(cnt + k) * 16) =
                    make_ulonglong2(a[2 * k], a[2 * k + 1]);
            }
          }
          half = a[20];
          cnt += 10u;
        } else {
          if (cnt < nelem) {
            ok &= hi_ok(a[0]);
            if (in)
              *reinterpret_cast<ulonglong2*>(mout + (size_t)cnt * 16) = make_ulonglong2(half, a[0]);
          }
#pragma unroll
          for (int k = 0; k < 10; ++k) {
            if (cnt + 1u + k < nelem) {
              ok &= hi_ok(a[2 * k + 2]);
              if (in)
                *reinterpret_cast<ulonglong2*>(mout + (size_t)(cnt + 1u + k) * 16) =
                    make_ulonglong2(a[2 * k + 1], a[2 * k + 2]);
            }
          }
          cnt += 11u;
        }
        bad |= !ok;
        // speculative accumulation: column sums of the block's words over the wave's 64 rows
        // (the words in [spec_w0, spec_w1), k_jr's range), through this wave's LDS rows
        if (spec_lo != nullptr && w0 + 21 > (int64_t)spec_w0 && w0 < (int64_t)spec_w1) {
          uint64_t* row = reinterpret_cast<uint64_t*>(win + lane * kJrWin);
#pragma unroll
          for (int w = 0; w < 21; ++w) row[w] = a[w];
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          const uint32_t gq = lane / 21u, wc = lane - 21u * gq;
          const uint8_t* colp = win + 8u * wc + gq * kJrWin;
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
                xs[i] = *reinterpret_cast<const uint64_t*>(win + 8u * wc + 63u * kJrWin);
                if (gq != 0u) xs[i] = 0ull;
              }
            }
#pragma unroll
            for (int i = 0; i < 11; ++i) acc_u64(l32, h32, cy, xs[i]);
          }
          const uint32_t s1 = (lane + 21u) & 63u, s2 = (lane + 42u) & 63u;
          const uint32_t la = __shfl(l32, (int)s1, 64), ha = __shfl(h32, (int)s1, 64);
          const uint32_t ca = __shfl(cy, (int)s1, 64);
          const uint32_t lb = __shfl(l32, (int)s2, 64), hb = __shfl(h32, (int)s2, 64);
          const uint32_t cb = __shfl(cy, (int)s2, 64);
          const int64_t wd = w0 + lane;
          if (lane < 21u && wd >= (int64_t)spec_w0 && wd < (int64_t)spec_w1) {
            acc_u64(l32, h32, cy, ((uint64_t)ha << 32) | la);
            acc_u64(l32, h32, cy, ((uint64_t)hb << 32) | lb);
            const size_t at = (size_t)(r0w >> 6) * (size_t)nd + (size_t)wd;
            spec_lo[at] = ((uint64_t)h32 << 32) | l32;
            spec_cy[at] = (uint8_t)(cy + ca + cb);
          }
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // rows reused next block
        }
      }
      // absorb message block b into S2: stream words [21b-6, 21b+15] (zero past the share)
      uint64_t A[16];
#pragma unroll
      for (int w = 0; w < 16; ++w) A[w] = (w0 + w < nd) ? a[w] : 0ull;
      jrp_absorb(o, carry, A, b, nblocks, padw, padv, cfg, 1u, blind, nz);
#pragma unroll
      for (int i = 0; i < 6; ++i) carry[i] = (w0 + 15 + i < nd) ? a[15 + i] : 0ull;
    }
    // swap: the other state is permuted next (S2 after an absorb, S1 after S2)
#pragma unroll
    for (int i = 0; i < 25; ++i) {
      const uint64_t t = a[i];
      a[i] = o[i];
      o[i] = t;
    }
    keccak_x(a, cfg.xof);
  }
  // a = S2 after its last block: the joint-rand part
  if (bad && in) atomicOr(fallback, 1u);
  if (!live) return;
  const uint64_t plo = a[0], phi = a[1];
  st64(out_part.at(r), plo);
  st64(out_part.at(r) + 8, phi);
  const uint8_t* ps = public_shares.at(r);
  const uint64_t p0lo = ld64(ps), p0hi = ld64(ps + 8);
  uint64_t slo, shi;
  derive_jr_seed(cfg.xof, cfg.algo_id, p0lo, p0hi, plo, phi, slo, shi);
  st64(out_seed.at(r), slo);
  st64(out_seed.at(r) + 8, shi);
  MsgBlock m;
  m.clear();
  m.header(cfg.algo_id, DST_JOINT_RANDOMNESS, slo, shi);
  m.pad(25, cfg.xof);
  uint64_t s2[25];
  sponge_one_block(s2, m, cfg.xof);
  squeeze_vec<FO>(s2, cfg.jr_len, out_jr.at(r), cfg.xof, false);
}

}  // namespace p3g
