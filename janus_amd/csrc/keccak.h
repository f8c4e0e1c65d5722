// Keccak-p[1600, nr] for gfx950: one sponge per lane (state = 25 x u64 = 50 VGPRs).
// Replaces `keccak 0.1.4` / `sha3 0.10.8` behind prio 0.15.1's XofShake128 (ext crates,
// Cargo.lock:2190-2194, :3687-3691), which the reference reaches through Prio3 prepare
// (aggregator/src/aggregator.rs:1777-1786).
//
// 64-bit rotations lower to two v_alignbit_b32; chi (a ^ (~b & c)) and the 3-way theta parities
// lower to v_bitop3_b32 (gfx950).  Rounds are fully unrolled so pi is pure register renaming.
// NR = 24 is SHAKE128 (parity with prio 0.15.1 / VDAF-07); NR = 12 is TurboSHAKE128 (VDAF-08+).
// The kernels choose at run time (Xof below): the 12 rounds TurboSHAKE128 uses are the LAST 12 of
// Keccak-f, so one unrolled copy of rounds 12..23 serves both and rounds 0..11 sit behind a
// wave-uniform branch -- no second copy of the permutation in the instruction cache.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#ifndef DEVI
#define DEVI __device__ __forceinline__
#endif

constexpr uint64_t kRC[24] = {
    0x0000000000000001ull, 0x0000000000008082ull, 0x800000000000808aull, 0x8000000080008000ull,
    0x000000000000808bull, 0x0000000080000001ull, 0x8000000080008081ull, 0x8000000000008009ull,
    0x000000000000008aull, 0x0000000000000088ull, 0x0000000080008009ull, 0x000000008000000aull,
    0x000000008000808bull, 0x800000000000008bull, 0x8000000000008089ull, 0x8000000000008003ull,
    0x8000000000008002ull, 0x8000000000000080ull, 0x000000000000800aull, 0x800000008000000aull,
    0x8000000080008081ull, 0x8000000000008080ull, 0x0000000080000001ull, 0x8000000080008008ull};

// 3-input bitwise ops (gfx950 v_bitop3_b32; LUT index = (src0<<2)|(src1<<1)|src2).
DEVI uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); }
DEVI uint32_t chi3(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0xD2); }  // a ^ (~b & c)
// v_alignbit_b32: ((hi:lo) >> s)[31:0]
DEVI uint32_t abit(uint32_t hi, uint32_t lo, uint32_t s) { return __builtin_amdgcn_alignbit(hi, lo, s); }

// One Keccak round on a state split into 32-bit halves (l = low words, h = high words).
//   theta: C[x] = xor of column (2 xor3 per half); lane ^= C[x-1] ^ rotl1(C[x+1]) (1 xor3 per half)
//   rho:   rotl64 by r = 2 v_alignbit_b32 (swap when r = 32; none when r = 0)
//   pi:    register renaming
//   chi:   1 bitop3 per half;  iota: xor of the round constant halves
// => 20 + 10 + 50 + 48 + 50 + 2 = 180 VALU ops per round.
template <int R>
DEVI void keccak_round32(uint32_t l[25], uint32_t h[25]) {
  uint32_t cl[5], ch[5], rl[5], rh[5];
#pragma unroll
  for (int x = 0; x < 5; ++x) {
    cl[x] = xor3(xor3(l[x], l[x + 5], l[x + 10]), l[x + 15], l[x + 20]);
    ch[x] = xor3(xor3(h[x], h[x + 5], h[x + 10]), h[x + 15], h[x + 20]);
  }
#pragma unroll
  for (int x = 0; x < 5; ++x) {  // rotl64(C[x], 1)
    rl[x] = abit(cl[x], ch[x], 31);
    rh[x] = abit(ch[x], cl[x], 31);
  }
  uint32_t bl[25], bh[25];

  { const uint32_t tl = xor3(l[0], cl[4], rl[1]), th = xor3(h[0], ch[4], rh[1]);
    bl[0] = tl; bh[0] = th; }
  { const uint32_t tl = xor3(l[1], cl[0], rl[2]), th = xor3(h[1], ch[0], rh[2]);
    bl[10] = abit(tl, th, 31); bh[10] = abit(th, tl, 31); }
  { const uint32_t tl = xor3(l[2], cl[1], rl[3]), th = xor3(h[2], ch[1], rh[3]);
    bl[20] = abit(th, tl, 2); bh[20] = abit(tl, th, 2); }
  { const uint32_t tl = xor3(l[3], cl[2], rl[4]), th = xor3(h[3], ch[2], rh[4]);
    bl[5] = abit(tl, th, 4); bh[5] = abit(th, tl, 4); }
  { const uint32_t tl = xor3(l[4], cl[3], rl[0]), th = xor3(h[4], ch[3], rh[0]);
    bl[15] = abit(tl, th, 5); bh[15] = abit(th, tl, 5); }
  { const uint32_t tl = xor3(l[5], cl[4], rl[1]), th = xor3(h[5], ch[4], rh[1]);
    bl[16] = abit(th, tl, 28); bh[16] = abit(tl, th, 28); }
  { const uint32_t tl = xor3(l[6], cl[0], rl[2]), th = xor3(h[6], ch[0], rh[2]);
    bl[1] = abit(th, tl, 20); bh[1] = abit(tl, th, 20); }
  { const uint32_t tl = xor3(l[7], cl[1], rl[3]), th = xor3(h[7], ch[1], rh[3]);
    bl[11] = abit(tl, th, 26); bh[11] = abit(th, tl, 26); }
  { const uint32_t tl = xor3(l[8], cl[2], rl[4]), th = xor3(h[8], ch[2], rh[4]);
    bl[21] = abit(th, tl, 9); bh[21] = abit(tl, th, 9); }
  { const uint32_t tl = xor3(l[9], cl[3], rl[0]), th = xor3(h[9], ch[3], rh[0]);
    bl[6] = abit(tl, th, 12); bh[6] = abit(th, tl, 12); }
  { const uint32_t tl = xor3(l[10], cl[4], rl[1]), th = xor3(h[10], ch[4], rh[1]);
    bl[7] = abit(tl, th, 29); bh[7] = abit(th, tl, 29); }
  { const uint32_t tl = xor3(l[11], cl[0], rl[2]), th = xor3(h[11], ch[0], rh[2]);
    bl[17] = abit(tl, th, 22); bh[17] = abit(th, tl, 22); }
  { const uint32_t tl = xor3(l[12], cl[1], rl[3]), th = xor3(h[12], ch[1], rh[3]);
    bl[2] = abit(th, tl, 21); bh[2] = abit(tl, th, 21); }
  { const uint32_t tl = xor3(l[13], cl[2], rl[4]), th = xor3(h[13], ch[2], rh[4]);
    bl[12] = abit(tl, th, 7); bh[12] = abit(th, tl, 7); }
  { const uint32_t tl = xor3(l[14], cl[3], rl[0]), th = xor3(h[14], ch[3], rh[0]);
    bl[22] = abit(th, tl, 25); bh[22] = abit(tl, th, 25); }
  { const uint32_t tl = xor3(l[15], cl[4], rl[1]), th = xor3(h[15], ch[4], rh[1]);
    bl[23] = abit(th, tl, 23); bh[23] = abit(tl, th, 23); }
  { const uint32_t tl = xor3(l[16], cl[0], rl[2]), th = xor3(h[16], ch[0], rh[2]);
    bl[8] = abit(th, tl, 19); bh[8] = abit(tl, th, 19); }
  { const uint32_t tl = xor3(l[17], cl[1], rl[3]), th = xor3(h[17], ch[1], rh[3]);
    bl[18] = abit(tl, th, 17); bh[18] = abit(th, tl, 17); }
  { const uint32_t tl = xor3(l[18], cl[2], rl[4]), th = xor3(h[18], ch[2], rh[4]);
    bl[3] = abit(tl, th, 11); bh[3] = abit(th, tl, 11); }
  { const uint32_t tl = xor3(l[19], cl[3], rl[0]), th = xor3(h[19], ch[3], rh[0]);
    bl[13] = abit(tl, th, 24); bh[13] = abit(th, tl, 24); }
  { const uint32_t tl = xor3(l[20], cl[4], rl[1]), th = xor3(h[20], ch[4], rh[1]);
    bl[14] = abit(tl, th, 14); bh[14] = abit(th, tl, 14); }
  { const uint32_t tl = xor3(l[21], cl[0], rl[2]), th = xor3(h[21], ch[0], rh[2]);
    bl[24] = abit(tl, th, 30); bh[24] = abit(th, tl, 30); }
  { const uint32_t tl = xor3(l[22], cl[1], rl[3]), th = xor3(h[22], ch[1], rh[3]);
    bl[9] = abit(th, tl, 3); bh[9] = abit(tl, th, 3); }
  { const uint32_t tl = xor3(l[23], cl[2], rl[4]), th = xor3(h[23], ch[2], rh[4]);
    bl[19] = abit(th, tl, 8); bh[19] = abit(tl, th, 8); }
  { const uint32_t tl = xor3(l[24], cl[3], rl[0]), th = xor3(h[24], ch[3], rh[0]);
    bl[4] = abit(tl, th, 18); bh[4] = abit(th, tl, 18); }
#pragma unroll
  for (int y = 0; y < 5; ++y) {
#pragma unroll
    for (int x = 0; x < 5; ++x) {
      l[x + 5 * y] = chi3(bl[x + 5 * y], bl[(x + 1) % 5 + 5 * y], bl[(x + 2) % 5 + 5 * y]);
      h[x + 5 * y] = chi3(bh[x + 5 * y], bh[(x + 1) % 5 + 5 * y], bh[(x + 2) % 5 + 5 * y]);
    }
  }
  constexpr uint64_t rc = kRC[R];
  if constexpr ((uint32_t)rc != 0u) l[0] ^= (uint32_t)rc;
  if constexpr ((uint32_t)(rc >> 32) != 0u) h[0] ^= (uint32_t)(rc >> 32);
}

template <int R, int END>
DEVI void keccak_rounds32(uint32_t l[25], uint32_t h[25]) {
  if constexpr (R < END) {
    keccak_round32<R>(l, h);
    keccak_rounds32<R + 1, END>(l, h);
  }
}

// Keccak-p[1600, NR]: the last NR rounds of Keccak-f (round constants RC[24-NR .. 23]).
template <int NR = 24>
DEVI void keccak_p(uint64_t a[25]) {
  uint32_t l[25], h[25];
#pragma unroll
  for (int i = 0; i < 25; ++i) {
    l[i] = (uint32_t)a[i];
    h[i] = (uint32_t)(a[i] >> 32);
  }
  keccak_rounds32<24 - NR, 24>(l, h);
#pragma unroll
  for (int i = 0; i < 25; ++i) a[i] = ((uint64_t)h[i] << 32) | l[i];
}

// The XOF of a context: XofShake128 (Keccak-f[1600] = 24 rounds, SHAKE padding byte 0x1F; prio
// 0.15.1 / VDAF-07, Janus 0.6) or XofTurboShake128 (Keccak-p[1600, 12], domain byte 0x01;
// draft-irtf-cfrg-vdaf-08+).  Both absorb the same message u8(len(dst)) || dst || seed || binder.
struct Xof {
  uint32_t full;  // 1: 24 rounds (SHAKE128), 0: 12 rounds (TurboSHAKE128)
  uint32_t pad;   // first padding byte: 0x1F (SHAKE128) or the TurboSHAKE domain byte 0x01
};
constexpr Xof kXofShake128{1u, 0x1Fu};
constexpr Xof kXofTurboShake128{0u, 0x01u};

DEVI void keccak_x(uint64_t a[25], const Xof& x) {
  uint32_t l[25], h[25];
#pragma unroll
  for (int i = 0; i < 25; ++i) {
    l[i] = (uint32_t)a[i];
    h[i] = (uint32_t)(a[i] >> 32);
  }
  if (x.full) keccak_rounds32<0, 12>(l, h);
  keccak_rounds32<12, 24>(l, h);
#pragma unroll
  for (int i = 0; i < 25; ++i) a[i] = ((uint64_t)h[i] << 32) | l[i];
}

// ------------------------------------------------------------------------------------------------
// XofShake128 message framing (prio src/vdaf/xof.rs; VDAF-07 §6.2.1):
//   SHAKE128( u8(8) || dst[8] || seed[16] || binder )       rate 168 B = 21 words, pad 0x1F..0x80
// dst = [7, 0, algo_id (u32 BE), usage (u16 BE)].
// ------------------------------------------------------------------------------------------------
constexpr int kRateWords = 21;

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
  // sponge padding for a message of `len` bytes (< 168): the XOF's first pad byte .. 0x80
  DEVI void pad(int len, const Xof& x) {
    put8(len, x.pad);
    w[kRateWords - 1] ^= 0x8000000000000000ull;
  }
};

// Absorb a single padded block into a fresh state and permute.
DEVI void sponge_one_block(uint64_t s[25], const MsgBlock& m, const Xof& x) {
#pragma unroll
  for (int i = 0; i < kRateWords; ++i) s[i] = m.w[i];
#pragma unroll
  for (int i = kRateWords; i < 25; ++i) s[i] = 0ull;
  keccak_x(s, x);
}
