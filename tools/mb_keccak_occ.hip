// Keccak-f[1600] throughput vs waves per SIMD on gfx950 (measurement infrastructure, not product).
// Occupancy is pinned with dynamic LDS: 160 KiB / k per 256-thread block -> k blocks per CU ->
// k waves per SIMD; the grid is exactly 256 CUs x k blocks x ROUNDS.  Variants:
//   reg    : state in registers only (the permutation alone)
//   store  : + 168 B of squeezed output per permutation, one row per lane (k_expand's pattern)
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/mb_keccak_occ tools/mb_keccak_occ.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "../janus_amd/csrc/keccak.h"

#define CK(x)                                                         \
  do {                                                                \
    hipError_t e = (x);                                               \
    if (e != hipSuccess) {                                            \
      printf("%s: %s\n", #x, hipGetErrorString(e));                   \
      return 1;                                                       \
    }                                                                 \
  } while (0)

constexpr int PERMS = 96;

__global__ void __launch_bounds__(256) k_reg(uint32_t* out, uint32_t seed, uint8_t* rows) {
  extern __shared__ uint8_t lds[];
  (void)lds;
  (void)rows;
  uint64_t s[25];
#pragma unroll
  for (int i = 0; i < 25; ++i) s[i] = (uint64_t)(seed + threadIdx.x) * (i + 1);
  for (int it = 0; it < PERMS; ++it) keccak_p<24>(s);
  uint64_t r = 0;
#pragma unroll
  for (int i = 0; i < 25; ++i) r ^= s[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)r;
}

__global__ void __launch_bounds__(256) k_store(uint32_t* out, uint32_t seed, uint8_t* rows) {
  extern __shared__ uint8_t lds[];
  (void)lds;
  const size_t gid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint8_t* row = rows + gid * (size_t)(PERMS * 168 + 8);
  uint64_t s[25];
#pragma unroll
  for (int i = 0; i < 25; ++i) s[i] = (uint64_t)(seed + threadIdx.x) * (i + 1);
  for (int it = 0; it < PERMS; ++it) {
    keccak_p<24>(s);
    uint64_t* o = reinterpret_cast<uint64_t*>(row + (size_t)it * 168);
#pragma unroll
    for (int w = 0; w < 21; ++w) o[w] = s[w];
  }
  out[gid] = (uint32_t)s[0];
}

typedef void (*kfn)(uint32_t*, uint32_t, uint8_t*);

static int run(const char* name, kfn k, int per_cu, uint32_t* d, uint8_t* rows, int rounds) {
  const int blocks = 256 * per_cu * rounds;
  const size_t lds = (160 * 1024) / per_cu;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  hipLaunchKernelGGL(k, dim3(blocks), dim3(256), lds, 0, d, 1u, rows);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a, 0));
  const int reps = 3;
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), lds, 0, d, 2u + r, rows);
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  const double perms = (double)PERMS * 256.0 * blocks * reps;
  printf("{\"bench\": \"keccak_%s\", \"waves_per_simd\": %d, \"perm_per_s\": %.4g, \"ms\": %.3f}\n",
         name, per_cu, perms / (ms * 1e-3), ms / reps);
  return 0;
}

int main() {
  const int rounds = 4;
  const size_t max_lanes = (size_t)256 * 6 * rounds * 256;
  uint32_t* d;
  uint8_t* rows;
  CK(hipMalloc(&d, max_lanes * 4));
  CK(hipMalloc(&rows, max_lanes / 2 * (size_t)(PERMS * 168 + 8)));  // store variant: <= 3 waves
  for (int k = 1; k <= 6; ++k) run("reg", k_reg, k, d, rows, rounds);
  for (int k = 1; k <= 3; ++k) run("store", k_store, k, d, rows, rounds);
  CK(hipFree(d));
  CK(hipFree(rows));
  return 0;
}
