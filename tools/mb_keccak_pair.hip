// Keccak-f[1600] CHAIN LATENCY and throughput: one state per lane vs one state per lane PAIR
// (keccak_pair_x below: low halves in the even lane, high halves in the odd lane, DPP swap for
// the rotations), gfx950.  Measured (profiles/r02/microbench_keccak_pair.log): 6.33 vs 7.39 us per
// permutation at one wave per CU -- only 1.17x, because the v_mov_b32_dpp feeding each rotation
// costs a lone wave ~8 cycles instead of 4 -- so the product kernels keep a state per lane.  Config E runs a few thousand sequential 152K-permutation sponges, so
// the time per permutation of ONE state bounds it.
//   mode 0: lane per state,  mode 1: lane pair per state;  W waves per CU (1 = one wave per CU)
// Checked against a host Keccak-f.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/mb_keccak_pair tools/mb_keccak_pair.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

#include "../janus_amd/csrc/keccak.h"

// ------------------------------------------------------------------------------------------------
// Keccak on a lane PAIR (latency-bound chains, e.g. FixedPoint config E): the even lane holds the
// low 32-bit halves of the 25 words, the odd lane the high halves.  XORs and chi are local; a 64-bit
// rotation needs the partner's half, one DPP quad_perm swap (v_mov_b32_dpp, full rate) and one
// v_alignbit_b32:  rotl64(v, n) own half = alignbit(own, partner, 32 - n) for n < 32, and
// alignbit(partner, own, 64 - n) for n > 32 -- the same formula in both lanes.  Per round and lane:
// 10 (theta parities) + 5 + 5 (rotl1) + 25 (theta xor3) + 24 + 24 (rho) + 25 (chi) + 1-2 (iota)
// = 120 VALU vs 180 for a whole state in one lane: a lone wave issues one VALU per 4 cycles, so a
// chain runs ~1.5x faster at 1.33x the total work.
// ------------------------------------------------------------------------------------------------
constexpr int kRho[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43,
                          25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};

// the other lane of the pair (quad_perm [1, 0, 3, 2])
DEVI uint32_t pair_swap(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);
}

template <int N>
DEVI uint32_t pair_rotl(uint32_t v) {
  if constexpr (N == 0) {
    return v;
  } else {
    const uint32_t p = pair_swap(v);
    if constexpr (N < 32) return abit(v, p, 32 - N);
    else if constexpr (N == 32) return p;
    else return abit(p, v, 64 - N);
  }
}

template <int I>
DEVI void pair_theta_rho_pi(const uint32_t s[25], const uint32_t c[5], const uint32_t r1[5],
                            uint32_t b[25]) {
  if constexpr (I < 25) {
    constexpr int x = I % 5, y = I / 5;
    const uint32_t t = xor3(s[I], c[(x + 4) % 5], r1[(x + 1) % 5]);
    b[y + 5 * ((2 * x + 3 * y) % 5)] = pair_rotl<kRho[I]>(t);
    pair_theta_rho_pi<I + 1>(s, c, r1, b);
  }
}

template <int R>
DEVI void keccak_round_pair(uint32_t s[25], bool odd) {
  uint32_t c[5], r1[5], b[25];
#pragma unroll
  for (int x = 0; x < 5; ++x) c[x] = xor3(xor3(s[x], s[x + 5], s[x + 10]), s[x + 15], s[x + 20]);
#pragma unroll
  for (int x = 0; x < 5; ++x) r1[x] = abit(c[x], pair_swap(c[x]), 31);
  pair_theta_rho_pi<0>(s, c, r1, b);
#pragma unroll
  for (int y = 0; y < 5; ++y) {
#pragma unroll
    for (int x = 0; x < 5; ++x)
      s[x + 5 * y] = chi3(b[x + 5 * y], b[(x + 1) % 5 + 5 * y], b[(x + 2) % 5 + 5 * y]);
  }
  constexpr uint32_t lo = (uint32_t)kRC[R], hi = (uint32_t)(kRC[R] >> 32);
  if constexpr (lo != 0u || hi != 0u) s[0] ^= odd ? hi : lo;
}

template <int R, int END>
DEVI void keccak_rounds_pair(uint32_t s[25], bool odd) {
  if constexpr (R < END) {
    keccak_round_pair<R>(s, odd);
    keccak_rounds_pair<R + 1, END>(s, odd);
  }
}

// Keccak-f[1600] (SHAKE128) or Keccak-p[1600, 12] (TurboSHAKE128) on a lane pair; `odd` = this
// lane holds the high halves.  Every lane of the wave must execute it (DPP reads the partner).
DEVI void keccak_pair_x(uint32_t s[25], bool odd, const Xof& x) {
  if (x.full) keccak_rounds_pair<0, 12>(s, odd);
  keccak_rounds_pair<12, 24>(s, odd);
}


#define CK(x)                                                       \
  do {                                                              \
    hipError_t e = (x);                                             \
    if (e != hipSuccess) {                                          \
      printf("%s: %s\n", #x, hipGetErrorString(e));                 \
      return 1;                                                     \
    }                                                               \
  } while (0)

__global__ void __launch_bounds__(64) k_lane(uint64_t* io, int nperm) {
  const size_t st = (size_t)blockIdx.x * 64 + threadIdx.x;
  uint64_t s[25];
#pragma unroll
  for (int i = 0; i < 25; ++i) s[i] = io[st * 25 + i];
  for (int k = 0; k < nperm; ++k) keccak_x(s, kXofShake128);
#pragma unroll
  for (int i = 0; i < 25; ++i) io[st * 25 + i] = s[i];
}

__global__ void __launch_bounds__(64) k_pair(uint64_t* io, int nperm) {
  const uint32_t lane = threadIdx.x;
  const size_t st = (size_t)blockIdx.x * 32 + (lane >> 1);
  const bool odd = lane & 1u;
  uint32_t s[25];
  const uint32_t* p = reinterpret_cast<const uint32_t*>(io + st * 25);
#pragma unroll
  for (int i = 0; i < 25; ++i) s[i] = p[2 * i + (odd ? 1 : 0)];
  for (int k = 0; k < nperm; ++k) keccak_pair_x(s, odd, kXofShake128);
  uint32_t* q = reinterpret_cast<uint32_t*>(io + st * 25);
#pragma unroll
  for (int i = 0; i < 25; ++i) q[2 * i + (odd ? 1 : 0)] = s[i];
}

static const int kR[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43,
                           25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};
static uint64_t rotl(uint64_t v, int n) { return n ? (v << n) | (v >> (64 - n)) : v; }
static void host_keccak(uint64_t a[25]) {
  for (int R = 0; R < 24; ++R) {
    uint64_t c[5], b[25];
    for (int x = 0; x < 5; ++x) c[x] = a[x] ^ a[x + 5] ^ a[x + 10] ^ a[x + 15] ^ a[x + 20];
    for (int i = 0; i < 25; ++i) a[i] ^= c[(i % 5 + 4) % 5] ^ rotl(c[(i % 5 + 1) % 5], 1);
    for (int x = 0; x < 5; ++x)
      for (int y = 0; y < 5; ++y) b[y + 5 * ((2 * x + 3 * y) % 5)] = rotl(a[x + 5 * y], kR[x + 5 * y]);
    for (int i = 0; i < 25; ++i)
      a[i] = b[i] ^ (~b[(i % 5 + 1) % 5 + 5 * (i / 5)] & b[(i % 5 + 2) % 5 + 5 * (i / 5)]);
    a[0] ^= kRC[R];
  }
}

int main() {
  const int NPERM = 2000;
  const int MAXB = 256 * 16;
  const int NST = MAXB * 64;
  uint64_t* h = (uint64_t*)malloc((size_t)NST * 25 * 8);
  for (size_t i = 0; i < (size_t)NST * 25; ++i) h[i] = 0x9E3779B97F4A7C15ull * (i + 1);
  uint64_t* d;
  CK(hipMalloc(&d, (size_t)NST * 25 * 8));
  uint64_t* o = (uint64_t*)malloc((size_t)NST * 25 * 8);
  uint64_t ref[4][25];
  for (int sidx = 0; sidx < 4; ++sidx) {
    memcpy(ref[sidx], h + (size_t)sidx * 25, 200);
    for (int k = 0; k < NPERM; ++k) host_keccak(ref[sidx]);
  }
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int waves[] = {1, 4, 8, 16};
  for (int wi = 0; wi < 4; ++wi) {
    const int NB = 256 * waves[wi];
    for (int mode = 0; mode < 2; ++mode) {
      CK(hipMemcpy(d, h, (size_t)NST * 25 * 8, hipMemcpyHostToDevice));
      if (mode == 0) k_lane<<<NB, 64>>>(d, 1); else k_pair<<<NB, 64>>>(d, 1);
      CK(hipMemcpy(d, h, (size_t)NST * 25 * 8, hipMemcpyHostToDevice));
      CK(hipEventRecord(a));
      if (mode == 0) k_lane<<<NB, 64>>>(d, NPERM); else k_pair<<<NB, 64>>>(d, NPERM);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      CK(hipMemcpy(o, d, (size_t)NST * 25 * 8, hipMemcpyDeviceToHost));
      int bad = 0;
      for (int sidx = 0; sidx < 4; ++sidx) bad += memcmp(ref[sidx], o + (size_t)sidx * 25, 200) != 0;
      const double states = (double)NB * (mode ? 32 : 64);
      printf("{\"bench\": \"keccak_chain\", \"mode\": \"%s\", \"waves_per_cu\": %d, "
             "\"us_per_perm_chain\": %.3f, \"perm_per_s\": %.4g, \"check\": \"%s\"}\n",
             mode ? "lane_pair" : "lane", waves[wi], ms * 1e3 / NPERM,
             states * NPERM / (ms * 1e-3), bad ? "FAILED" : "ok");
    }
  }
  return 0;
}
