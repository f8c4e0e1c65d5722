// FixedPointBoundedL2VecSum wire passes on the matrix cores (config E's FLP query; prio 0.15.1
// src/flp/types/fixedpoint_l2.rs, reached from Janus's Prio3::prepare_init at
// aggregator/src/aggregator.rs:1777-1786 for VdafInstance::Prio3FixedPoint*BitBoundedL2VecSum).
//
// Same outputs as k_fpv_wires0 / k_fpv_wires1 (fpvec_kernels.h), computed with wires_mfma.h's exact
// byte-limb convolution on v_mfma_i32_32x32x32_i8 instead of lazily reduced 256-bit VALU MACs --
// those passes issue 2 (gadget 0) and 1 (gadget 1) 128 x 128-bit products per share element and
// are VALU-bound at 3-4 TB/s; here the VALU keeps the byte flips and the fragment gathers.
//   k_fpv_wires0_mfma  gadget 0, ParallelSum(Mul, c0) over all x: block per (call range, report),
//                      the range's partial a_j = sum_k MM_k x_(k c0 + j), b_j = sum_k LM_k x_(...)
//                      (REDC'd, the VALU pass's `part` layout; k_fpv_finalize folds the ranges)
//   k_fpv_wires1_mfma  gadget 1, ParallelSum(PolyEval) over the decoded entries: block per report;
//                      the same shape over the raw bits (column = bit of an entry), then
//                      wire1_j = C1[j] + sum_l 2^l P_(n j + l) across the entry's lanes (prep
//                      share, as k_fpv_wires1)
// Weight digits live in LDS per call (wires_mfma.h layout: 48-byte reversed windows), and the
// correction term K128 * W' uses the weights' sum over the block's calls, reduced over the block.
#pragma once
#include "fpvec_kernels.h"
#include "wires_mfma.h"

namespace p3g {

constexpr uint32_t kFpvMfmaH = 4;  // gadget-0 call ranges (blocks) per report

// calls per gadget-0 range: even, so a K-step's two calls stay inside one range
__host__ __device__ inline uint32_t fpv_mfma_range(uint32_t calls, uint32_t H) {
  const uint32_t cr = (calls + H - 1) / H;
  return (cr + 1u) & ~1u;
}
// dynamic LDS of k_fpv_wires0_mfma / k_fpv_wires1_mfma: digit windows + block-sum scratch + flag
__host__ __device__ inline size_t fpv_w0m_lds(const Cfg& g) {
  return (size_t)fpv_mfma_range(g.calls, kFpvMfmaH) * 2 * kWmEDwords * 4 + 12 * 16 + 16;
}
__host__ __device__ inline size_t fpv_w1m_lds(const Cfg& g) {
  return (size_t)(2 * ((g.calls1 + 1) / 2)) * kWmEDwords * 4 + 12 * 16 + 16;
}

// Weight w (< p, Montgomery form) -> its 17 signed digits as one reversed 48-byte window at `row`
// (wires_mfma.h: E[m] = d_(31 - m), bytes 15..31 hold d_16..d_0).
DEVI void fpv_put_digits(uint32_t* rowp, const F128& x) {
  uint32_t D[4], cy = 0u;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint64_t s = (uint64_t)x.w[q] + 0x80808080u + cy;
    D[q] = (uint32_t)s ^ 0x80808080u;
    cy = (uint32_t)(s >> 32);
  }
  uint4* row = reinterpret_cast<uint4*>(rowp);
  row[0] = make_uint4(0u, 0u, 0u, cy << 24);
  row[1] = make_uint4(__builtin_bswap32(D[3]), __builtin_bswap32(D[2]), __builtin_bswap32(D[1]),
                      __builtin_bswap32(D[0]));
  row[2] = make_uint4(0u, 0u, 0u, 0u);
}

// The Toeplitz A fragment of one (call, wire) window for this lane (row s = 31 - o).
DEVI i32x4_t fpv_frag(const uint32_t* e, uint32_t sh) {
  const i32x4_t f = {(int)__builtin_amdgcn_alignbit(e[1], e[0], sh),
                     (int)__builtin_amdgcn_alignbit(e[2], e[1], sh),
                     (int)__builtin_amdgcn_alignbit(e[3], e[2], sh),
                     (int)__builtin_amdgcn_alignbit(e[4], e[3], sh)};
  return f;
}

// Column sums (signed 32-bit words) of a C/D fragment, split over the two lane halves: lane half
// h holds rows 8g + 4h + i = byte i of word 2g + h; returns word 2g + h' for the half's own wire.
DEVI void fpv_words(const i32x16_t& acc, int64_t v[4]) {
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    int64_t s = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) s += (int64_t)acc[4 * g + i] << (8 * i);
    v[g] = s;
  }
}

// grid (H, n), 256 threads: block (hr, r) = calls [hr CR, hr CR + CR) of report r; wave = 32-column
// tile (tiles loop over the waves); K-step q covers calls ka + 2q (lane half 0) and ka + 2q + 1.
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4)))
k_fpv_wires0_mfma(Cfg cfg, uint32_t n, CRows meas, CRows wrows, const uint8_t* status, uint8_t* part,
                  uint32_t* flags) {
  using FO = Field128Ops;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t hr = blockIdx.x, r = blockIdx.y, H = gridDim.x;
  if (r >= n || status[r] != ST_OK) return;  // block-uniform
  if (cfg.wave_prio) __builtin_amdgcn_s_setprio(2);  // loads issue ahead of k_fpv_regen's VALU
  const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = tid & 63u, nw = blockDim.x >> 6;
  const uint32_t C = cfg.calls, c = cfg.chunk, ML = cfg.meas_len;
  const uint32_t CR = fpv_mfma_range(C, H);
  const uint32_t ka = min(C, hr * CR), kb = min(C, ka + CR);
  const uint32_t KQ = (kb - ka + 1u) / 2u;
  const FpvW W = fpv_w_layout(cfg);
  uint32_t* E = reinterpret_cast<uint32_t*>(smem);
  F128* RED = reinterpret_cast<F128*>(smem + (size_t)CR * 2 * kWmEDwords * 4);
  uint32_t* flag = reinterpret_cast<uint32_t*>(RED + 12);
  if (tid == 0) *flag = 0u;
  const uint8_t* wr = wrows.at(r);
  const uint8_t* xr = meas.at(r);

  const uint32_t nn = lane & 31u, h = lane >> 5;
  const uint32_t o = 31u - nn;
  const uint32_t sh = 8u * (o & 3u);
  const uint32_t* Eh = E + (size_t)h * 2 * kWmEDwords + (o >> 2);
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc((void*)xr, (short)0, ML * 16u, kBufRsrcWord3);
  const uint32_t NT = (c + 31u) / 32u;
  constexpr uint32_t U = 4;  // K-steps whose loads are issued together
  auto load_batch = [&](uint32_t tile, uint32_t q0, uint4* xv) {
    const uint32_t j = tile * 32u + nn;
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
      const uint32_t k = ka + 2 * (q0 + u) + h;
      const uint32_t idx = k * c + j;
      const bool v = j < c && k < kb && idx < ML;
      const auto t = __builtin_amdgcn_raw_buffer_load_b128(rs, v ? idx * 16u : 0xFFFFFFF0u, 0, 0);
      xv[u] = make_uint4(t[0], t[1], t[2], t[3]);
    }
  };
  uint4 xv[U];
  load_batch(wave, 0, xv);  // in flight while the weights are converted

  // weights MM_k, LM_k of the range -> digits; their sums mod p
  F128 s0 = FO::zero(), s1 = FO::zero(), s2 = FO::zero();
  for (uint32_t kk = tid; kk < 2 * KQ; kk += blockDim.x) {
    F128 mm = FO::zero(), lm = FO::zero();
    if (ka + kk < kb) {
      mm = FO::load(wr + (size_t)(W.mm + ka + kk) * 16u);
      lm = FO::load(wr + (size_t)(W.lm + ka + kk) * 16u);
      s0 = FO::add(s0, mm);
      s1 = FO::add(s1, lm);
    }
    fpv_put_digits(E + ((size_t)kk * 2 + 0) * kWmEDwords, mm);
    fpv_put_digits(E + ((size_t)kk * 2 + 1) * kWmEDwords, lm);
  }
  block_sum3<FO>(s0, s1, s2, RED, tid, blockDim.x);  // its barriers also publish the digits

  bool bad = false;
  for (uint32_t tile = wave; tile < NT; tile += nw) {
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
      if (q0 > 0 || tile != wave) load_batch(tile, q0, xv);
#pragma unroll
      for (uint32_t u = 0; u < U; ++u) {
        if (q0 + u < KQ) {
          maybe |= __ballot(xv[u].w == 0xFFFFFFFFu);
          const i32x4_t b = {(int)(xv[u].x ^ 0x80808080u), (int)(xv[u].y ^ 0x80808080u),
                             (int)(xv[u].z ^ 0x80808080u), (int)(xv[u].w ^ 0x80808080u)};
          const uint32_t* ea = Eh + (size_t)(q0 + u) * 4 * kWmEDwords;
          acc_a = __builtin_amdgcn_mfma_i32_32x32x32_i8(fpv_frag(ea, sh), b, acc_a, 0, 0, 0);
          acc_b = __builtin_amdgcn_mfma_i32_32x32x32_i8(fpv_frag(ea + kWmEDwords, sh), b, acc_b, 0,
                                                        0, 0);
        }
      }
    }
    if (maybe) {  // rare: exact canonical check over this lane's elements of the range
      for (uint32_t q = 0; q < KQ; ++q) {
        const uint32_t k = ka + 2 * q + h, idx = k * c + j;
        if (colok && k < kb && idx < ML) bad |= !FO::is_canonical(FO::load(xr + (size_t)idx * 16));
      }
    }
    // lane half h finishes wire h (a: MM, b: LM) of column j
    int64_t va[4], vb[4];
    fpv_words(acc_a, va);
    fpv_words(acc_b, vb);
    int64_t T[8];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int64_t own = h ? vb[g] : va[g], oth = h ? va[g] : vb[g];
      const int64_t rv = (int64_t)shfl_xor_u64((uint64_t)oth, 32);
      T[2 * g] = h ? rv : own;
      T[2 * g + 1] = h ? own : rv;
    }
    const F128 v = wires_mfma_finish(T, h ? s1 : s0, kb - ka);
    if (colok) FO::store(part + (((size_t)r * H + hr) * c + j) * 32u + 16u * h, v);
  }
  if (bad) atomicOr(flag, 1u);
  __syncthreads();
  if (tid == 0 && *flag) atomicOr(&flags[r], FPV_BAD_ENCODING);
}

// Gadget 1 on the raw bits: with sum_k L'_k z_(k c1 + j) = sum_l 2^l sum_k L'_k x_(n(k c1 + j) + l),
// the pass is the gadget-0 shape over a (calls1 x n c1) element matrix -- row k is call k's n c1
// contiguous elements, column u = n j + l -- with one weight vector L'; the MFMA gives
// P_u = sum_k L'_k x_(k, u) per column, and the epilogue folds wire1_j = C1[j] + sum_l 2^l P_(nj+l)
// over the n adjacent lanes of entry j.  Entry widths n that divide a 32-column tile: 16, 32.
__host__ __device__ inline bool fpv_w1m_bits_ok(uint32_t bits) { return bits == 16 || bits == 32; }

// grid (n, S), 256 threads: block (r, s) takes the 32-column tiles s nw + wave + k S nw (every
// block of a report converts the same weights), K-step q covers calls 2q (lane half 0) and 2q + 1;
// each half-wave reads 512 contiguous bytes per K-step.
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4)))
k_fpv_wires1_mfma(Cfg cfg, uint32_t n, CRows meas, CRows wrows, Rows prep, const uint8_t* status) {
  using FO = Field128Ops;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t r = blockIdx.x;
  if (r >= n || status[r] != ST_OK) return;  // block-uniform
  if (cfg.wave_prio) __builtin_amdgcn_s_setprio(2);  // loads issue ahead of k_fpv_regen's VALU
  const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = tid & 63u, nw = blockDim.x >> 6;
  const uint32_t C = cfg.calls1, nb = cfg.bits, len = cfg.length, ML = cfg.meas_len;
  const uint32_t c = nb * cfg.chunk1;  // columns: the elements of one call
  const uint32_t KQ = (C + 1u) / 2u;
  const FpvW W = fpv_w_layout(cfg);
  uint32_t* E = reinterpret_cast<uint32_t*>(smem);
  F128* RED = reinterpret_cast<F128*>(smem + (size_t)2 * KQ * kWmEDwords * 4);
  const uint8_t* wr = wrows.at(r);
  const uint8_t* xr = meas.at(r);

  const uint32_t nn = lane & 31u, h = lane >> 5;
  const uint32_t o = 31u - nn;
  const uint32_t sh = 8u * (o & 3u);
  const uint32_t* Eh = E + (size_t)h * kWmEDwords + (o >> 2);
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc((void*)xr, (short)0, ML * 16u, kBufRsrcWord3);
  const uint32_t NT = (c + 31u) / 32u;
  constexpr uint32_t U = 4;  // K-steps whose loads are issued together
  auto load_batch = [&](uint32_t tile, uint32_t q0, uint4* xv) {
    const uint32_t u0 = tile * 32u + nn;  // column
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
      const uint32_t k = 2 * (q0 + u) + h;
      const uint32_t e = k * cfg.chunk1 + u0 / nb;  // entry (past `length`: the norm bits)
      const bool v = u0 < c && k < C && e < len;
      const auto t = __builtin_amdgcn_raw_buffer_load_b128(rs, v ? (k * c + u0) * 16u : 0xFFFFFFF0u,
                                                           0, 0);
      xv[u] = make_uint4(t[0], t[1], t[2], t[3]);
    }
  };
  uint4 xv[U];
  const uint32_t t0 = blockIdx.y * nw + wave, tstep = gridDim.y * nw;  // this wave's tiles
  load_batch(t0, 0, xv);  // in flight while the weights are converted

  F128 s0 = FO::zero(), s1 = FO::zero(), s2 = FO::zero();
  for (uint32_t kk = tid; kk < 2 * KQ; kk += blockDim.x) {
    F128 w = FO::zero();
    if (kk < C) {
      w = FO::load(wr + (size_t)(W.l1 + kk) * 16u);  // L'_(kk+1), Montgomery
      s0 = FO::add(s0, w);
    }
    fpv_put_digits(E + (size_t)kk * kWmEDwords, w);
  }
  block_sum3<FO>(s0, s1, s2, RED, tid, blockDim.x);  // its barriers also publish the digits

  // 2^l (Montgomery) for this lane's bit l = column mod n (tiles start at multiples of n)
  const uint32_t l = nn & (nb - 1u);
  const F128 two_l = FO::to_mont(FO::from_u64x2(1ull << l, 0ull));
  for (uint32_t tile = t0; tile < NT; tile += tstep) {
    i32x16_t acc;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0;
    for (uint32_t q0 = 0; q0 < KQ; q0 += U) {
      if (q0 > 0 || tile != t0) load_batch(tile, q0, xv);
#pragma unroll
      for (uint32_t u = 0; u < U; ++u) {
        if (q0 + u < KQ) {
          const i32x4_t b = {(int)(xv[u].x ^ 0x80808080u), (int)(xv[u].y ^ 0x80808080u),
                             (int)(xv[u].z ^ 0x80808080u), (int)(xv[u].w ^ 0x80808080u)};
          acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(
              fpv_frag(Eh + (size_t)(q0 + u) * 2 * kWmEDwords, sh), b, acc, 0, 0, 0);
        }
      }
    }
    int64_t va[4];
    fpv_words(acc, va);
    int64_t T[8];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int64_t rv = (int64_t)shfl_xor_u64((uint64_t)va[g], 32);
      T[2 * g] = h ? rv : va[g];
      T[2 * g + 1] = h ? va[g] : rv;
    }
    // P_u (both lane halves hold it), times 2^l, summed over the entry's n lanes
    F128 q = FO::mul(wires_mfma_finish(T, s0, C), two_l);
    for (uint32_t off = nb >> 1; off >= 1u; off >>= 1) q = FO::add(q, shfl_xor_T<FO>(q, (int)off));
    const uint32_t u0 = tile * 32u + nn, j = u0 / nb;
    if (h == 0 && l == 0 && u0 < c) {
      FO::store(prep.at(r) + (size_t)(1 + cfg.arity + 1 + j) * 16u,
                FO::add(FO::load(wr + (size_t)(W.c1 + j) * 16u), q));
    }
  }
}

}  // namespace p3g
