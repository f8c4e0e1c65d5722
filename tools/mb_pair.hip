// Lane-pair Keccak microbenchmark (measurement tooling, not product code): a latency-bound sponge
// chain (config E) issues one VALU every ~4 cycles per lone wave, so a permutation's latency is
// its instruction count.  Here two lanes hold one state in bit-interleaved halves (even lane: the
// even bits of every 64-bit word, odd lane: the odd bits), so XOR / chi / theta take one op per
// word, an even rotation two half-rate alignbits' worth on each lane, and an odd rotation one
// per-lane-amount alignbit plus a DPP swap with the partner lane.  Checks the pair result against
// keccak.h's permutation and times NP permutations per chain, one or two waves per SIMD.
// Build: hipcc --offload-arch=gfx950 -O3 -I janus_amd/csrc -o tools/mb_pair tools/mb_pair.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include <vector>
#include "keccak.h"
#include "keccak_pair.h"
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__host__ __device__ inline uint64_t init_word(uint32_t r, uint32_t i) {
  uint64_t z = 0x9E3779B97F4A7C15ull * (uint64_t)(r * 25u + i + 1u);
  z ^= z >> 29;
  z *= 0xBF58476D1CE4E5B9ull;
  return z ^ (z >> 32);
}

__global__ void __launch_bounds__(64) k_std(uint64_t* out, int np) {
  const uint32_t r = blockIdx.x * 64u + threadIdx.x;
  uint64_t a[25];
  for (int i = 0; i < 25; ++i) a[i] = init_word(r, i);
  for (int q = 0; q < np; ++q) keccak_x(a, kXofShake128);
  for (int i = 0; i < 25; ++i) out[(size_t)r * 25 + i] = a[i];
}

__global__ void __launch_bounds__(64) k_pair(uint32_t* out, int np) {
  const uint32_t g = blockIdx.x * 64u + threadIdx.x, r = g >> 1, p = g & 1u;
  uint32_t s[25];
  for (int i = 0; i < 25; ++i) s[i] = kp_half(init_word(r, i), p);
  const KpLane ln = kp_lane(p);
  for (int q = 0; q < np; ++q) keccak_pair_x(s, ln, kXofShake128);
  for (int i = 0; i < 25; ++i) out[((size_t)r * 25 + i) * 2 + p] = s[i];
}

static uint64_t merge(uint32_t e, uint32_t o) {
  uint64_t v = 0;
  for (int j = 0; j < 32; ++j) v |= ((uint64_t)((e >> j) & 1u) << (2 * j)) | ((uint64_t)((o >> j) & 1u) << (2 * j + 1));
  return v;
}

int main() {
  const int blocks_check = 4;
  uint64_t* d64;
  uint32_t* d32;
  CK(hipMalloc(&d64, (size_t)4096 * 64 * 25 * 8));
  CK(hipMalloc(&d32, (size_t)4096 * 64 * 25 * 8));
  // correctness: 3 permutations of 128 reports
  hipLaunchKernelGGL(k_std, dim3(2), dim3(64), 0, 0, d64, 3);
  hipLaunchKernelGGL(k_pair, dim3(blocks_check), dim3(64), 0, 0, d32, 3);
  CK(hipDeviceSynchronize());
  std::vector<uint64_t> hs(128 * 25);
  std::vector<uint32_t> hp(128 * 25 * 2);
  CK(hipMemcpy(hs.data(), d64, hs.size() * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hp.data(), d32, hp.size() * 4, hipMemcpyDeviceToHost));
  int bad = 0;
  for (int r = 0; r < 128; ++r)
    for (int i = 0; i < 25; ++i)
      if (merge(hp[(r * 25 + i) * 2], hp[(r * 25 + i) * 2 + 1]) != hs[r * 25 + i]) ++bad;
  printf("pair vs std mismatches: %d of %d words\n", bad, 128 * 25);
  if (bad) return 2;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int np = 2000;
  for (int waves : {1, 1024, 2048, 4096}) {
    for (int kind = 0; kind < 2; ++kind) {
      for (int rep = 0; rep < 2; ++rep) {
        CK(hipEventRecord(a));
        if (kind == 0) hipLaunchKernelGGL(k_std, dim3(waves), dim3(64), 0, 0, d64, np);
        else hipLaunchKernelGGL(k_pair, dim3(waves), dim3(64), 0, 0, d32, np);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        const double reports = waves * (kind ? 32.0 : 64.0);
        if (rep)
          printf("%-5s waves %5d  %8.3f ms  chain %6.3f us/perm (%6.0f cyc @2.4GHz)  %6.2f G perm/s\n",
                 kind ? "pair" : "std", waves, ms, ms * 1e3 / np, ms * 1e6 / np * 2.4,
                 reports * np / (ms * 1e-3) * 1e-9);
      }
    }
  }
  return 0;
}
