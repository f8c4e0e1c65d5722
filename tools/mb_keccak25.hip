// Keccak-f[1600] CHAIN LATENCY, one state per lane vs one state spread over 25 lanes (a lane per
// 64-bit word, ds_bpermute for theta's columns and pi/chi), gfx950.  Measurement infrastructure
// for the latency-bound FixedPoint pipeline: config E runs a few thousand sequential
// 152K-permutation sponges, so the time per permutation of ONE state is what bounds it.
//   mode 0: lane = state (the product kernels' form), 1 wave per CU
//   mode 1: 25 lanes = state (lanes 0..24 and 32..56 of a wave: 2 states per wave), 1 wave per CU
// Checked against a host Keccak-f.  Build: hipcc --offload-arch=gfx950 -O3 -o tools/mb_keccak25 tools/mb_keccak25.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

#include "../janus_amd/csrc/keccak.h"

#define CK(x)                                                       \
  do {                                                              \
    hipError_t e = (x);                                             \
    if (e != hipSuccess) {                                          \
      printf("%s: %s\n", #x, hipGetErrorString(e));                 \
      return 1;                                                     \
    }                                                               \
  } while (0)

__constant__ uint32_t kRot[25] = {0,  1,  62, 28, 27, 36, 44, 6,  55, 20, 3,  10, 43,
                                  25, 39, 41, 45, 15, 21, 8,  18, 2,  61, 56, 14};

DEVI uint32_t bperm(uint32_t v, uint32_t lane) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(lane << 2), (int)v);
}

// one Keccak-f on a state held one word per lane (word i = x + 5y in lane base + i, i < 25)
DEVI void keccak25(uint32_t& lo, uint32_t& hi, uint32_t lane) {
  const uint32_t base = lane & 32u, i = lane & 31u;
  const uint32_t ii = i < 25u ? i : 0u;
  const uint32_t x = ii % 5u, y = ii / 5u;
  uint32_t col[4];
#pragma unroll
  for (uint32_t d = 1; d < 5; ++d) col[d - 1] = base + x + 5u * ((y + d) % 5u);
  const uint32_t lm1 = base + (x + 4u) % 5u + 5u * y, lp1 = base + (x + 1u) % 5u + 5u * y;
  // rho: rotl64 by r = kRot[i] (kRot is indexed by x + 5y with the usual Keccak offsets)
  const uint32_t r = kRot[ii];
  const bool swp = r >= 32u;
  const uint32_t rr = r & 31u, sh = 32u - rr;
  // pi: B(X, Y) = rho(A(x_s, y_s)) with X = y_s, Y = 2 x_s + 3 y_s  =>  y_s = X, x_s = 3 (Y - 3X)
  uint32_t src[3];
#pragma unroll
  for (uint32_t k = 0; k < 3; ++k) {
    const uint32_t X = (x + k) % 5u, Y = y;
    const uint32_t xs = (3u * ((Y + 15u - 3u * X) % 5u)) % 5u, ys = X;
    src[k] = base + xs + 5u * ys;
  }
  for (int R = 0; R < 24; ++R) {
    // theta
    uint32_t cl = lo, ch = hi;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      cl ^= bperm(lo, col[d]);
      ch ^= bperm(hi, col[d]);
    }
    const uint32_t ml = bperm(cl, lm1), mh = bperm(ch, lm1);
    const uint32_t pl = bperm(cl, lp1), ph = bperm(ch, lp1);
    lo = xor3(lo, ml, abit(pl, ph, 31));
    hi = xor3(hi, mh, abit(ph, pl, 31));
    // rho
    uint32_t a = swp ? hi : lo, b = swp ? lo : hi;
    if (rr) {
      const uint32_t na = abit(a, b, sh), nb = abit(b, a, sh);
      a = na;
      b = nb;
    }
    lo = a;
    hi = b;
    // pi + chi
    const uint32_t b0l = bperm(lo, src[0]), b0h = bperm(hi, src[0]);
    const uint32_t b1l = bperm(lo, src[1]), b1h = bperm(hi, src[1]);
    const uint32_t b2l = bperm(lo, src[2]), b2h = bperm(hi, src[2]);
    lo = chi3(b0l, b1l, b2l);
    hi = chi3(b0h, b1h, b2h);
    // iota
    const uint64_t rc = kRC[R];
    if (i == 0u) {
      lo ^= (uint32_t)rc;
      hi ^= (uint32_t)(rc >> 32);
    }
  }
}

__global__ void __launch_bounds__(64) k_lane(uint64_t* io, int nperm) {
  const size_t st = (size_t)blockIdx.x * 64 + threadIdx.x;
  uint64_t s[25];
#pragma unroll
  for (int i = 0; i < 25; ++i) s[i] = io[st * 25 + i];
  for (int k = 0; k < nperm; ++k) keccak_p<24>(s);
#pragma unroll
  for (int i = 0; i < 25; ++i) io[st * 25 + i] = s[i];
}

__global__ void __launch_bounds__(64) k_25(uint64_t* io, int nperm) {
  const uint32_t lane = threadIdx.x;
  const size_t st = (size_t)blockIdx.x * 2 + (lane >> 5);
  const uint32_t i = lane & 31u;
  uint64_t w = i < 25u ? io[st * 25 + i] : 0ull;
  uint32_t lo = (uint32_t)w, hi = (uint32_t)(w >> 32);
  for (int k = 0; k < nperm; ++k) keccak25(lo, hi, lane);
  if (i < 25u) io[st * 25 + i] = ((uint64_t)hi << 32) | lo;
}

// host Keccak-f
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
  const int NB = 256;         // blocks of one wave: one wave per CU
  const int NPERM = 4000;
  const int NST = NB * 64;    // states in mode 0 (mode 1 uses the first NB * 2)
  uint64_t* h = (uint64_t*)malloc((size_t)NST * 25 * 8);
  for (size_t i = 0; i < (size_t)NST * 25; ++i) h[i] = 0x9E3779B97F4A7C15ull * (i + 1);
  uint64_t* d;
  CK(hipMalloc(&d, (size_t)NST * 25 * 8));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int mode = 0; mode < 2; ++mode) {
    CK(hipMemcpy(d, h, (size_t)NST * 25 * 8, hipMemcpyHostToDevice));
    // warm-up launch with 1 permutation, then the timed chain
    if (mode == 0) k_lane<<<NB, 64>>>(d, 1); else k_25<<<NB, 64>>>(d, 1);
    CK(hipMemcpy(d, h, (size_t)NST * 25 * 8, hipMemcpyHostToDevice));
    CK(hipEventRecord(a));
    if (mode == 0) k_lane<<<NB, 64>>>(d, NPERM); else k_25<<<NB, 64>>>(d, NPERM);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    uint64_t* o = (uint64_t*)malloc((size_t)NST * 25 * 8);
    CK(hipMemcpy(o, d, (size_t)NST * 25 * 8, hipMemcpyDeviceToHost));
    int bad = 0;
    for (int sidx = 0; sidx < 4; ++sidx) {
      uint64_t s[25];
      memcpy(s, h + (size_t)sidx * 25, 200);
      for (int k = 0; k < NPERM; ++k) host_keccak(s);
      if (memcmp(s, o + (size_t)sidx * 25, 200)) ++bad;
    }
    printf("mode %d (%s): %d permutations in %.2f ms = %.3f us per permutation per state chain; "
           "host check %s\n", mode, mode ? "25 lanes per state" : "lane per state", NPERM, ms,
           ms * 1e3 / NPERM, bad ? "FAILED" : "ok");
    free(o);
  }
  return 0;
}
