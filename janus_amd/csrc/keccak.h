// Keccak-p[1600, nr] for gfx950: one sponge per lane (state = 25 x u64 = 50 VGPRs).
// Replaces `keccak 0.1.4` / `sha3 0.10.8` behind prio 0.15.1's XofShake128 (ext crates,
// Cargo.lock:2190-2194, :3687-3691), which the reference reaches through Prio3 prepare
// (aggregator/src/aggregator.rs:1777-1786).
//
// 64-bit rotations lower to two v_alignbit_b32; chi (a ^ (~b & c)) and the 3-way theta parities
// lower to v_bitop3_b32 (gfx950).  Rounds are fully unrolled so pi is pure register renaming.
// NR = 24 is SHAKE128 (parity with prio 0.15.1 / VDAF-07); NR = 12 is TurboSHAKE128 (VDAF-08+).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#ifndef DEVI
#define DEVI __device__ __forceinline__
#endif

__device__ __constant__ static const uint64_t kKeccakRC[24] = {
    0x0000000000000001ull, 0x0000000000008082ull, 0x800000000000808aull, 0x8000000080008000ull,
    0x000000000000808bull, 0x0000000080000001ull, 0x8000000080008081ull, 0x8000000000008009ull,
    0x000000000000008aull, 0x0000000000000088ull, 0x0000000080008009ull, 0x000000008000000aull,
    0x000000008000808bull, 0x800000000000008bull, 0x8000000000008089ull, 0x8000000000008003ull,
    0x8000000000008002ull, 0x8000000000000080ull, 0x000000000000800aull, 0x800000008000000aull,
    0x8000000080008081ull, 0x8000000000008080ull, 0x0000000080000001ull, 0x8000000080008008ull};

DEVI uint64_t rotl64(uint64_t x, int n) { return (x << n) | (x >> (64 - n)); }

// One round on state a (indices x + 5y).
#define KECCAK_ROUND(a, rc)                                                                     \
  do {                                                                                          \
    uint64_t c0 = a[0] ^ a[5] ^ a[10] ^ a[15] ^ a[20];                                          \
    uint64_t c1 = a[1] ^ a[6] ^ a[11] ^ a[16] ^ a[21];                                          \
    uint64_t c2 = a[2] ^ a[7] ^ a[12] ^ a[17] ^ a[22];                                          \
    uint64_t c3 = a[3] ^ a[8] ^ a[13] ^ a[18] ^ a[23];                                          \
    uint64_t c4 = a[4] ^ a[9] ^ a[14] ^ a[19] ^ a[24];                                          \
    uint64_t d0 = c4 ^ rotl64(c1, 1);                                                           \
    uint64_t d1 = c0 ^ rotl64(c2, 1);                                                           \
    uint64_t d2 = c1 ^ rotl64(c3, 1);                                                           \
    uint64_t d3 = c2 ^ rotl64(c4, 1);                                                           \
    uint64_t d4 = c3 ^ rotl64(c0, 1);                                                           \
    /* theta + rho + pi: b[y][2x+3y] = rot(a[x][y] ^ d[x], r[x][y]) ; b index = y + 5*(2x+3y) */ \
    uint64_t b0 = a[0] ^ d0;                                                                    \
    uint64_t b10 = rotl64(a[1] ^ d1, 1);                                                        \
    uint64_t b20 = rotl64(a[2] ^ d2, 62);                                                       \
    uint64_t b5 = rotl64(a[3] ^ d3, 28);                                                        \
    uint64_t b15 = rotl64(a[4] ^ d4, 27);                                                       \
    uint64_t b16 = rotl64(a[5] ^ d0, 36);                                                       \
    uint64_t b1 = rotl64(a[6] ^ d1, 44);                                                        \
    uint64_t b11 = rotl64(a[7] ^ d2, 6);                                                        \
    uint64_t b21 = rotl64(a[8] ^ d3, 55);                                                       \
    uint64_t b6 = rotl64(a[9] ^ d4, 20);                                                        \
    uint64_t b7 = rotl64(a[10] ^ d0, 3);                                                        \
    uint64_t b17 = rotl64(a[11] ^ d1, 10);                                                      \
    uint64_t b2 = rotl64(a[12] ^ d2, 43);                                                       \
    uint64_t b12 = rotl64(a[13] ^ d3, 25);                                                      \
    uint64_t b22 = rotl64(a[14] ^ d4, 39);                                                      \
    uint64_t b23 = rotl64(a[15] ^ d0, 41);                                                      \
    uint64_t b8 = rotl64(a[16] ^ d1, 45);                                                       \
    uint64_t b18 = rotl64(a[17] ^ d2, 15);                                                      \
    uint64_t b3 = rotl64(a[18] ^ d3, 21);                                                       \
    uint64_t b13 = rotl64(a[19] ^ d4, 8);                                                       \
    uint64_t b14 = rotl64(a[20] ^ d0, 18);                                                      \
    uint64_t b24 = rotl64(a[21] ^ d1, 2);                                                       \
    uint64_t b9 = rotl64(a[22] ^ d2, 61);                                                       \
    uint64_t b19 = rotl64(a[23] ^ d3, 56);                                                      \
    uint64_t b4 = rotl64(a[24] ^ d4, 14);                                                       \
    /* chi + iota */                                                                            \
    a[0] = b0 ^ (~b1 & b2) ^ (rc);                                                              \
    a[1] = b1 ^ (~b2 & b3);                                                                     \
    a[2] = b2 ^ (~b3 & b4);                                                                     \
    a[3] = b3 ^ (~b4 & b0);                                                                     \
    a[4] = b4 ^ (~b0 & b1);                                                                     \
    a[5] = b5 ^ (~b6 & b7);                                                                     \
    a[6] = b6 ^ (~b7 & b8);                                                                     \
    a[7] = b7 ^ (~b8 & b9);                                                                     \
    a[8] = b8 ^ (~b9 & b5);                                                                     \
    a[9] = b9 ^ (~b5 & b6);                                                                     \
    a[10] = b10 ^ (~b11 & b12);                                                                 \
    a[11] = b11 ^ (~b12 & b13);                                                                 \
    a[12] = b12 ^ (~b13 & b14);                                                                 \
    a[13] = b13 ^ (~b14 & b10);                                                                 \
    a[14] = b14 ^ (~b10 & b11);                                                                 \
    a[15] = b15 ^ (~b16 & b17);                                                                 \
    a[16] = b16 ^ (~b17 & b18);                                                                 \
    a[17] = b17 ^ (~b18 & b19);                                                                 \
    a[18] = b18 ^ (~b19 & b15);                                                                 \
    a[19] = b19 ^ (~b15 & b16);                                                                 \
    a[20] = b20 ^ (~b21 & b22);                                                                 \
    a[21] = b21 ^ (~b22 & b23);                                                                 \
    a[22] = b22 ^ (~b23 & b24);                                                                 \
    a[23] = b23 ^ (~b24 & b20);                                                                 \
    a[24] = b24 ^ (~b20 & b21);                                                                 \
  } while (0)

// Keccak-p[1600, NR]: the last NR rounds of Keccak-f (round constants RC[24-NR .. 23]).
template <int NR = 24>
DEVI void keccak_p(uint64_t a[25]) {
#pragma unroll
  for (int r = 24 - NR; r < 24; ++r) {
    KECCAK_ROUND(a, kKeccakRC[r]);
  }
}

// ------------------------------------------------------------------------------------------------
// XofShake128 message framing (prio src/vdaf/xof.rs; VDAF-07 §6.2.1):
//   SHAKE128( u8(8) || dst[8] || seed[16] || binder )       rate 168 B = 21 words, pad 0x1F..0x80
// dst = [7, 0, algo_id (u32 BE), usage (u16 BE)].
// ------------------------------------------------------------------------------------------------
constexpr int kRateWords = 21;
constexpr uint8_t kShakePad = 0x1F;

// Word 0 and the low byte of word 1 of every XOF message: [8, 7, 0, id BE(4), usage_hi] [usage_lo].
DEVI uint64_t xof_word0(uint32_t algo_id, uint32_t usage) {
  uint64_t w = 8ull | (7ull << 8) | (0ull << 16);
  w |= (uint64_t)((algo_id >> 24) & 0xFF) << 24;
  w |= (uint64_t)((algo_id >> 16) & 0xFF) << 32;
  w |= (uint64_t)((algo_id >> 8) & 0xFF) << 40;
  w |= (uint64_t)(algo_id & 0xFF) << 48;
  w |= (uint64_t)((usage >> 8) & 0xFF) << 56;
  return w;
}

// A short message (< 168 bytes) assembled in registers as up to 21 LE words, XORed at byte offsets.
struct MsgBlock {
  uint64_t w[kRateWords];
  DEVI void clear() {
#pragma unroll
    for (int i = 0; i < kRateWords; ++i) w[i] = 0ull;
  }
  // XOR 8 LE bytes `v` at byte offset `off` (off compile-time after inlining).
  DEVI void put64(int off, uint64_t v) {
    const int wi = off >> 3, sh = (off & 7) * 8;
    if (sh == 0) {
      w[wi] ^= v;
    } else {
      w[wi] ^= v << sh;
      if (wi + 1 < kRateWords) w[wi + 1] ^= v >> (64 - sh);
    }
  }
  DEVI void put8(int off, uint32_t v) { w[off >> 3] ^= (uint64_t)(v & 0xFF) << ((off & 7) * 8); }
  // Standard XOF header: len(dst) || dst || seed  -> 25 bytes
  DEVI void header(uint32_t algo_id, uint32_t usage, uint64_t seed_lo, uint64_t seed_hi) {
    w[0] ^= xof_word0(algo_id, usage);
    put8(8, usage & 0xFF);
    put64(9, seed_lo);
    put64(17, seed_hi);
  }
  // SHAKE padding for a message of `len` bytes (< 168)
  DEVI void pad(int len) {
    put8(len, kShakePad);
    w[kRateWords - 1] ^= 0x8000000000000000ull;
  }
};

// Absorb a single padded block into a fresh state and permute.
template <int NR = 24>
DEVI void sponge_one_block(uint64_t s[25], const MsgBlock& m) {
#pragma unroll
  for (int i = 0; i < kRateWords; ++i) s[i] = m.w[i];
#pragma unroll
  for (int i = kRateWords; i < 25; ++i) s[i] = 0ull;
  keccak_p<NR>(s);
}
