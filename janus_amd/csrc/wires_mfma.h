// FLP wire pass for ParallelSum(Mul) (SumVec, chunk > 64) on the matrix cores.
//
// Same outputs as k_flp_wires (prio3_kernels.h), i.e. the query side of prio 0.15.1's
// ParallelSum(Mul) gadget wires that Janus reaches through Prio3::prepare_init
// (aggregator/src/aggregator.rs:1777-1786; leader: aggregation_job_driver.rs:362-380):
//   a_j = REDC( sum_k MM[k] x_(k c + j) ),   b_j = REDC( sum_k LM[k] x_(k c + j) )
//   wire_2j = B0[j] + RP[j] a_j,              wire_2j+1 = B1[j] + b_j
// with the weights MM, LM (Montgomery form, < p) from k_flp_weights.
//
// The Field128 products are computed EXACTLY as integers by byte-limb convolution on
// v_mfma_i32_32x32x32_i8 instead of 2 x 16 v_mad_u64_u32 per element on the VALU:
//   * x (measurement share element, 16 canonical bytes) enters as x' = x - K128 with
//     K128 = 0x8080...80: byte-wise x'_a = x_a ^ 0x80 in [-128, 127] (4 v_xor per element);
//   * a weight w enters as 17 signed digits d_b in [-128, 127] (w + K128, bytes ^ 0x80, the carry
//     out as d_16), converted once per report into LDS;
//   * for call k the A operand is the 32 x 16 Toeplitz matrix T_k[s][a] = d_(k, s-a), the B
//     operand the 16 bytes of x'_(k, j) for 32 columns j, so one MFMA (K = 32 = two calls)
//     accumulates acc[s][j] += sum_(a+b=s) x'_(k,j,a) d_(k,b) for s = 0..31;
//   * sum_s acc[s][j] 2^(8s) = sum_k w_k x'_(k,j) exactly (|acc| <= calls 2^18 < 2^31), and
//     adding K128 * sum_k w_k gives sum_k w_k x_(k,j), REDC'd by wide_reduce like the VALU path
//     (sum_k w_k enters as (its value mod p, from k_flp_weights) + calls p: same residue, and
//     never below the integer sum, so the total stays non-negative).
// Every A/B element pair the hardware multiplies shares its K index by construction, so the
// result does not depend on the i8 operand's k order; the C/D map is the documented one
// (col = lane & 31, row = (reg & 3) + 8 (reg >> 2) + 4 (lane >> 5)).
//
// Shape: block per report, wave per 32-column tile (up to 4 waves, then tiles loop; chunk 89:
// 3 waves), lane (n = lane & 31,
// h = lane >> 5) loads element (2q + h, 32 t + n) at K-step q: each half-wave reads 512
// contiguous bytes per K-step, every element exactly once.  The VALU keeps 4 xors, a compare and
// the Toeplitz fragment (5 LDS dwords + 4 v_alignbit, per wire) per element pair; the MFMA work
// (2 x 32 cycles per K-step per wave) is far below the HBM time.
#pragma once
#include "field.h"
#include "wide.h"

namespace p3g {

typedef int i32x4_t __attribute__((ext_vector_type(4)));
typedef int i32x16_t __attribute__((ext_vector_type(16)));

#ifndef WM_PREFETCH
#define WM_PREFETCH 1
#endif
#ifndef WM_U
#define WM_U 4  // K-steps whose loads are issued together
#endif
constexpr uint32_t kWmEDwords = 12;     // 48-byte reversed digit window per (call, wire)
constexpr uint32_t kWmMaxCalls = 8000;  // |acc| <= calls * 16 * 2^14 < 2^31

DEVI uint64_t shfl_xor_u64(uint64_t v, int m) {
  const uint32_t lo = __shfl_xor((uint32_t)v, m), hi = __shfl_xor((uint32_t)(v >> 32), m);
  return ((uint64_t)hi << 32) | lo;
}


// One column's wire from its exact MFMA sum: T[w] = signed 32-bit word w (rows 4w .. 4w + 3 of
// the C/D fragment) of sum_k w_k x'_k.  Adds K128 * W' with W' = (sum_k w_k mod p) + calls p
// (>= the integer sum of the weights, so the total is >= 0 and == sum_k w_k x_k mod p; `wsum` is
// the weights' sum mod p) and REDCs it like the VALU path.
DEVI F128 wires_mfma_finish(const int64_t T[8], const F128& wsum, uint32_t calls) {
  uint32_t S[10];
  {
    int64_t cr = 0;
#pragma unroll
    for (int w = 0; w < 8; ++w) {
      const int64_t v = T[w] + cr;
      S[w] = (uint32_t)v;
      cr = v >> 32;
    }
    S[8] = (uint32_t)cr;
    S[9] = (uint32_t)(cr >> 32);
  }
  uint32_t Wd[6];
  {
    const int64_t CC = (int64_t)calls;
    const int64_t v[5] = {(int64_t)wsum.w[0] + CC, (int64_t)wsum.w[1],
                          (int64_t)wsum.w[2] - 28 * CC, (int64_t)wsum.w[3], CC};
    int64_t cr = 0;
#pragma unroll
    for (int q = 0; q < 5; ++q) {
      const int64_t t = v[q] + cr;
      Wd[q] = (uint32_t)t;
      cr = t >> 32;
    }
    Wd[5] = (uint32_t)cr;
  }
  uint32_t M[7];
  uint64_t mc = 0;
#pragma unroll
  for (int q = 0; q < 6; ++q) {
    const uint64_t v = (uint64_t)Wd[q] * 0x80808080u + mc;
    M[q] = (uint32_t)v;
    mc = v >> 32;
  }
  M[6] = (uint32_t)mc;
  uint64_t sc = 0;
#pragma unroll
  for (int w = 0; w < 10; ++w) {
    uint64_t v = (uint64_t)S[w] + sc;
#pragma unroll
    for (int sft = 0; sft < 4; ++sft)
      if (w - sft >= 0 && w - sft < 7) v += M[w - sft];
    S[w] = (uint32_t)v;
    sc = v >> 32;
  }
  Wide wd;
  wide_zero(wd);
#pragma unroll
  for (int w = 0; w < 6; ++w) wd.lo[w] = S[w];
  wd.lo[6] = ((uint64_t)S[7] << 32) | S[6];
  wd.hi[6] = S[8];
  return wide_reduce(wd);
}

// Block per report, a wave per 32-column tile (<= 4 waves, then tiles loop).  (A wave-per-report
// form for short rows, chunk 8..32, measured slower than k_flp_wires_cols -- 3.9 vs 1.66 ms per
// launch on Histogram256, profiles/r03/ab_wires_mfma_short_r3u.log -- and was removed.)
__host__ __device__ inline size_t wires_mfma_e_bytes(uint32_t calls) {
  return (size_t)(2 * ((calls + 1) / 2)) * 2 * kWmEDwords * 4;
}

// 4 waves per SIMD (<= 128 VGPRs): the pass hides HBM latency with occupancy
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) k_flp_wires_mfma(Cfg cfg, uint32_t n, CRows meas, CRows proof,
                                                         WMat wm, Rows out_prep, uint8_t* status) {
  using FO = Field128Ops;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = tid & 63u;
  if constexpr (P3G_FLP_PRIO > 0) __builtin_amdgcn_s_setprio(P3G_FLP_PRIO);
  const uint32_t r = blockIdx.x;
  if (r >= n) return;
  if (status[r] != ST_OK) return;
  const uint32_t nw = blockDim.x >> 6;  // waves sharing the report
  const uint32_t wv = wave;             // this wave's first tile
  const uint32_t pt = tid, npt = blockDim.x;  // weight conversion
  const uint32_t C = cfg.calls, c = cfg.chunk, KQ = (C + 1) / 2;
  const WRow W(cfg);
  uint32_t* E = reinterpret_cast<uint32_t*>(smem);
  uint32_t* flag = reinterpret_cast<uint32_t*>(smem + wires_mfma_e_bytes(C));
  if (tid == 0) *flag = 0u;

  const uint32_t nn = lane & 31u, h = lane >> 5;
  const uint32_t o = 31u - nn;  // A row s = nn: the fragment is E[o .. o + 15]
  const uint32_t sh = 8u * (o & 3u);
  const uint32_t* Eh = E + (size_t)h * 2 * kWmEDwords + (o >> 2);
  const uint8_t* xr = meas.at(r);
  const uint32_t ML = cfg.meas_len;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc((void*)xr, (short)0, ML * 16u, kBufRsrcWord3);
  const uint32_t NT = (c + 31u) / 32u;
  // B fragments of K-steps [q0, q0 + U) of a tile.  Raw buffer loads: a dead slot (padding, column
  // >= chunk, K-step >= KQ) gets an offset past the row and reads zero, so no branch (a branch
  // around each load made the compiler wait for every load before issuing the next).
  constexpr uint32_t U = WM_U;
  auto load_batch = [&](uint32_t tile, uint32_t q0, uint4* xv) {
    const uint32_t j = tile * 32u + nn;
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
      const uint32_t idx = (2 * (q0 + u) + h) * c + j;
      const bool v = j < c && idx < ML && q0 + u < KQ;
      const auto t = __builtin_amdgcn_raw_buffer_load_b128(rs, v ? idx * 16u : 0xFFFFFFF0u, 0, 0);
      xv[u] = make_uint4(t[0], t[1], t[2], t[3]);
    }
  };
  uint4 xv[U];
  if (WM_PREFETCH) load_batch(wv, 0, xv);  // in flight while the weights are converted

  // ---- weights -> signed byte digits (reversed, zero-padded windows) ----
  for (uint32_t k = pt; k < 2 * KQ; k += npt) {
#pragma unroll
    for (uint32_t w = 0; w < 2; ++w) {
      F128 x = FO::zero();
      if (k < C) x = FO::load(wm.el(r, w ? W.lm(k) : W.mm(k)));
      // y = x + K128; digits d_b = y_b - 128 (b < 16), d_16 = carry out
      uint32_t D[4], cy = 0u;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint64_t s = (uint64_t)x.w[q] + 0x80808080u + cy;
        D[q] = (uint32_t)s ^ 0x80808080u;
        cy = (uint32_t)(s >> 32);
      }
      uint4* row = reinterpret_cast<uint4*>(E + ((size_t)k * 2 + w) * kWmEDwords);
      // E[m] = d_(31 - m): bytes 15..31 hold d_16..d_0, the rest zero
      row[0] = make_uint4(0u, 0u, 0u, cy << 24);
      row[1] = make_uint4(__builtin_bswap32(D[3]), __builtin_bswap32(D[2]),
                          __builtin_bswap32(D[1]), __builtin_bswap32(D[0]));
      row[2] = make_uint4(0u, 0u, 0u, 0u);
    }
  }
  __syncthreads();

  // ---- main loop: wave = 32-column tile, K-step q covers calls 2q (h = 0) and 2q + 1 (h = 1) ----
  bool bad = false;
  for (uint32_t tile = wv; tile < NT; tile += nw) {  // 32-column tiles
    const uint32_t j = tile * 32u + nn;
    const bool colok = j < c;
    i32x16_t acc_a, acc_b;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      acc_a[i] = 0;
      acc_b[i] = 0;
    }
    uint64_t maybe = 0ull;  // lane mask: some element with top word 2^32 - 1 (exact check below)
    for (uint32_t q0 = 0; q0 < KQ; q0 += U) {
      if (!WM_PREFETCH || q0 > 0 || tile != wv) load_batch(tile, q0, xv);
#pragma unroll
      for (uint32_t u = 0; u < U; ++u) {
        if (q0 + u < KQ) {
          maybe |= __ballot(xv[u].w == 0xFFFFFFFFu);
          const i32x4_t b = {(int)(xv[u].x ^ 0x80808080u), (int)(xv[u].y ^ 0x80808080u),
                             (int)(xv[u].z ^ 0x80808080u), (int)(xv[u].w ^ 0x80808080u)};
          const uint32_t* ea = Eh + (size_t)(q0 + u) * 4 * kWmEDwords;
          const uint32_t* eb = ea + kWmEDwords;
          const i32x4_t fa = {(int)__builtin_amdgcn_alignbit(ea[1], ea[0], sh),
                              (int)__builtin_amdgcn_alignbit(ea[2], ea[1], sh),
                              (int)__builtin_amdgcn_alignbit(ea[3], ea[2], sh),
                              (int)__builtin_amdgcn_alignbit(ea[4], ea[3], sh)};
          const i32x4_t fb = {(int)__builtin_amdgcn_alignbit(eb[1], eb[0], sh),
                              (int)__builtin_amdgcn_alignbit(eb[2], eb[1], sh),
                              (int)__builtin_amdgcn_alignbit(eb[3], eb[2], sh),
                              (int)__builtin_amdgcn_alignbit(eb[4], eb[3], sh)};
          acc_a = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa, b, acc_a, 0, 0, 0);
          acc_b = __builtin_amdgcn_mfma_i32_32x32x32_i8(fb, b, acc_b, 0, 0, 0);
        }
      }
    }
    if (maybe) {  // rare: exact canonical check over this lane's elements
      for (uint32_t q = 0; q < KQ; ++q) {
        const uint32_t idx = (2 * q + h) * c + j;
        if (colok && idx < ML) bad |= !FO::is_canonical(FO::load(xr + (size_t)idx * 16));
      }
    }

    // ---- epilogue: lane h finishes wire h of column j ----
    // Lane half h holds rows 8g + 4h + i (g, i < 4) = bytes 4i of 32-bit word 2g + h.
    int64_t gown[4], goth[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      int64_t va = 0, vb = 0;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        va += (int64_t)acc_a[4 * g + i] << (8 * i);
        vb += (int64_t)acc_b[4 * g + i] << (8 * i);
      }
      gown[g] = h ? vb : va;
      goth[g] = h ? va : vb;
    }
    int64_t T[8];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int64_t rv = (int64_t)shfl_xor_u64((uint64_t)goth[g], 32);
      T[2 * g] = h ? rv : gown[g];
      T[2 * g + 1] = h ? gown[g] : rv;
    }
    const F128 v = wires_mfma_finish(T, FO::load(wm.el(r, h ? W.slm() : W.smm())), C);
    if (colok) {
      // wire 2j + h = L0 s_(2j+h) (- HL for h = 1) + (RP[j] a_j | b_j)
      uint8_t* outp = out_prep.at(r);
      const F128 l0 = FO::load(wm.el(r, W.l0()));
      const F128 sd = FO::load(proof.at(r) + (size_t)(2 * j + h) * 16);
      bad |= !FO::is_canonical(sd);
      if (h == 0) {
        const F128 rp = FO::load(wm.el(r, W.rp(j)));  // Montgomery
        FO::store(outp + (size_t)(1 + 2 * j) * 16, FO::add(FO::mul(l0, sd), FO::mul(rp, v)));
      } else {
        FO::store(outp + (size_t)(2 + 2 * j) * 16,
                  FO::add(FO::sub(FO::mul(l0, sd), FO::load(wm.el(r, W.hl()))), v));
      }
    }
  }
  if (bad) atomicOr(flag, 1u);
  __syncthreads();
  if (tid == 0 && (*flag & 1u)) status[r] = ST_INVALID_MESSAGE;
}

}  // namespace p3g
