// Keccak-p[1600, nr] on a lane PAIR (gfx950): lanes 2q and 2q + 1 hold one state in
// bit-interleaved halves -- the even lane bits 0, 2, .., 62 of every 64-bit word, the odd lane
// bits 1, 3, .., 63 -- 25 VGPRs per lane.  For a latency-bound sponge chain (a lone wave issues a
// VALU every ~4 cycles whatever its lane count) this halves the instructions on the chain:
//   theta parities, theta's XOR and chi: one op per word instead of two;
//   rotl64 by n = 2k: rotl32 by k on both lanes (one alignbit, none for n = 0);
//   rotl64 by n = 2k + 1: the even word takes rotl32(odd word, k + 1), the odd word
//     rotl32(even word, k) -- each lane rotates its OWN word (by k + 1 if odd, k if even, a per-lane
//     alignbit amount) and the pair swaps through one DPP quad_perm [1, 0, 3, 2] move.
// => 10 + 15 + 25 + 60 + 25 + ~2 = ~137 issue slots per round (alignbit at half rate) against
// keccak.h's ~238 (keccak_round32, 64-bit words as two 32-bit halves).  A wave then carries 32
// sponges instead of 64, so throughput-bound kernels keep keccak.h; this form is for chains.
// Words enter and leave through kp_half / kp_merge (bit compress / expand, off the chain).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "keccak.h"
#include "kp_bits.h"

#ifndef DEVI
#define DEVI __device__ __forceinline__
#endif

struct KpLane {
  uint32_t p;   // 0 even lane, 1 odd lane
  uint32_t pm;  // p ? ~0 : 0
};
DEVI KpLane kp_lane(uint32_t p) { return KpLane{p, 0u - p}; }

// the partner lane's value (quad_perm [1, 0, 3, 2])
DEVI uint32_t kp_swap(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, true);
}
// the pair's 64-bit word from its two halves (both lanes get it)
DEVI uint64_t kp_merge(uint32_t own, const KpLane& ln) {
  const uint32_t o = kp_swap(own);
  return ln.p ? kp_zip(o, own) : kp_zip(own, o);
}

namespace kp {
constexpr int kRho[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43, 25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};
constexpr int pi_dst(int i) { return (i / 5) + 5 * ((2 * (i % 5) + 3 * (i / 5)) % 5); }
}  // namespace kp

// rotl64 by n of the pair's word, on this lane's half
template <int N>
DEVI uint32_t kp_rotl(uint32_t v, const KpLane& ln) {
  if constexpr (N == 0) {
    return v;
  } else if constexpr ((N & 1) == 0) {
    return abit(v, v, 32 - N / 2);
  } else {
    constexpr uint32_t k = (uint32_t)(N - 1) / 2;
    // own word rotated by k (even lane) or k + 1 (odd lane): alignbit by (32 - k - p) mod 32
    return kp_swap(abit(v, v, 32u - k - ln.p));
  }
}

template <int R>
DEVI void kp_round(uint32_t s[25], const KpLane& ln) {
  uint32_t c[5], rc1[5], b[25];
#pragma unroll
  for (int x = 0; x < 5; ++x) c[x] = xor3(xor3(s[x], s[x + 5], s[x + 10]), s[x + 15], s[x + 20]);
#pragma unroll
  for (int x = 0; x < 5; ++x) rc1[x] = kp_rotl<1>(c[x], ln);
#pragma unroll
  for (int i = 0; i < 25; ++i) {
    const int x = i % 5;
    const uint32_t v = xor3(s[i], c[(x + 4) % 5], rc1[(x + 1) % 5]);
    switch (kp::kRho[i]) {  // constant per unrolled i
#define KP_CASE(n) case n: b[kp::pi_dst(i)] = kp_rotl<n>(v, ln); break;
      KP_CASE(0) KP_CASE(1) KP_CASE(62) KP_CASE(28) KP_CASE(27) KP_CASE(36) KP_CASE(44) KP_CASE(6)
      KP_CASE(55) KP_CASE(20) KP_CASE(3) KP_CASE(10) KP_CASE(43) KP_CASE(25) KP_CASE(39) KP_CASE(41)
      KP_CASE(45) KP_CASE(15) KP_CASE(21) KP_CASE(8) KP_CASE(18) KP_CASE(2) KP_CASE(61) KP_CASE(56)
      KP_CASE(14)
#undef KP_CASE
    }
  }
#pragma unroll
  for (int y = 0; y < 5; ++y)
#pragma unroll
    for (int x = 0; x < 5; ++x)
      s[x + 5 * y] = chi3(b[x + 5 * y], b[(x + 1) % 5 + 5 * y], b[(x + 2) % 5 + 5 * y]);
  constexpr uint32_t rce = kp_half(kRC[R], 0), rco = kp_half(kRC[R], 1);
  if constexpr (rce == rco) {
    if constexpr (rce != 0u) s[0] ^= rce;
  } else {
    s[0] ^= (rco & ln.pm) | (rce & ~ln.pm);
  }
}

template <int R, int END>
DEVI void kp_rounds(uint32_t s[25], const KpLane& ln) {
  if constexpr (R < END) {
    kp_round<R>(s, ln);
    kp_rounds<R + 1, END>(s, ln);
  }
}

// keccak_x on the pair: 24 rounds (SHAKE128) or the last 12 (TurboSHAKE128)
DEVI void keccak_pair_x(uint32_t s[25], const KpLane& ln, const Xof& x) {
  if (x.full) kp_rounds<0, 12>(s, ln);
  kp_rounds<12, 24>(s, ln);
}
