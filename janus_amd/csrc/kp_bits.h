// Bit-interleaving helpers of the lane-pair Keccak (keccak_pair.h): a 64-bit word as its even-bit
// and odd-bit halves.  Host + device (tests/test_keccak_pair.py builds it with g++).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define KP_HD __host__ __device__ __forceinline__
#else
#define KP_HD inline
#endif

// bits p, p + 2, .., p + 62 of w packed into 32 bits
constexpr uint32_t kp_half(uint64_t w, uint32_t p) {
  uint64_t x = (w >> p) & 0x5555555555555555ull;
  x = (x | (x >> 1)) & 0x3333333333333333ull;
  x = (x | (x >> 2)) & 0x0F0F0F0F0F0F0F0Full;
  x = (x | (x >> 4)) & 0x00FF00FF00FF00FFull;
  x = (x | (x >> 8)) & 0x0000FFFF0000FFFFull;
  x = (x | (x >> 16)) & 0x00000000FFFFFFFFull;
  return (uint32_t)x;
}
// the inverse for one half: its bits spread to positions p, p + 2, .. (OR the two halves)
constexpr uint64_t kp_spread(uint32_t h, uint32_t p) {
  uint64_t x = h;
  x = (x | (x << 16)) & 0x0000FFFF0000FFFFull;
  x = (x | (x << 8)) & 0x00FF00FF00FF00FFull;
  x = (x | (x << 4)) & 0x0F0F0F0F0F0F0F0Full;
  x = (x | (x << 2)) & 0x3333333333333333ull;
  x = (x | (x << 1)) & 0x5555555555555555ull;
  return x << p;
}

// the middle-byte swap (the 8-bit delta stage): one v_perm_b32 on the device
KP_HD uint32_t kp_swap_mid_bytes(uint32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_perm(x, x, 0x03010200u);
#else
  const uint32_t t = (x ^ (x >> 8)) & 0x0000FF00u;
  return x ^ t ^ (t << 8);
#endif
}
KP_HD uint32_t kp_unshuffle32(uint32_t x) {
  uint32_t t = (x ^ (x >> 1)) & 0x22222222u;
  x ^= t ^ (t << 1);
  t = (x ^ (x >> 2)) & 0x0C0C0C0Cu;
  x ^= t ^ (t << 2);
  t = (x ^ (x >> 4)) & 0x00F000F0u;
  x ^= t ^ (t << 4);
  return kp_swap_mid_bytes(x);  // even bits in the low 16, odd bits in the high 16
}
KP_HD uint32_t kp_shuffle32(uint32_t x) {  // the inverse
  x = kp_swap_mid_bytes(x);
  uint32_t t = (x ^ (x >> 4)) & 0x00F000F0u;
  x ^= t ^ (t << 4);
  t = (x ^ (x >> 2)) & 0x0C0C0C0Cu;
  x ^= t ^ (t << 2);
  t = (x ^ (x >> 1)) & 0x22222222u;
  x ^= t ^ (t << 1);
  return x;
}
// low halves (lo16(a) | lo16(b) << 16) and high halves (hi16(a) | hi16(b) << 16): one v_perm_b32 each
KP_HD uint32_t kp_lo16s(uint32_t a, uint32_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_perm(b, a, 0x05040100u);
#else
  return (a & 0xFFFFu) | (b << 16);
#endif
}
KP_HD uint32_t kp_hi16s(uint32_t a, uint32_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_perm(b, a, 0x07060302u);
#else
  return (a >> 16) | (b & 0xFFFF0000u);
#endif
}
// Both halves of a 64-bit word at once (32-bit delta swaps, Hacker's Delight 7-2 unshuffle, on
// each 32-bit half, then byte selects): e = kp_half(x, 0), o = kp_half(x, 1); kp_zip inverts it.
KP_HD void kp_unzip(uint64_t x, uint32_t& e, uint32_t& o) {
  const uint32_t u = kp_unshuffle32((uint32_t)x), v = kp_unshuffle32((uint32_t)(x >> 32));
  e = kp_lo16s(u, v);
  o = kp_hi16s(u, v);
}
KP_HD uint64_t kp_zip(uint32_t e, uint32_t o) {
  const uint32_t lo = kp_shuffle32(kp_lo16s(e, o));
  const uint32_t hi = kp_shuffle32(kp_hi16s(e, o));
  return ((uint64_t)hi << 32) | lo;
}
