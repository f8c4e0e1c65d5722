// VALU microbenchmarks on gfx950 (measurement infrastructure, not product code):
//   - int32 bitop3 / alignbit throughput (the Keccak instruction mix) -> confirms the int32 VALU
//     peak used as the roofline denominator
//   - v_mad_u64_u32 throughput (Field128 Montgomery building block)
//   - Field128 Montgomery multiply throughput (janus_amd/csrc/field.h)
//   - Keccak-f[1600] permutations/s (janus_amd/csrc/keccak.h)
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/microbench tools/microbench.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "../janus_amd/csrc/field.h"
#include "../janus_amd/csrc/keccak.h"

#define CK(x)                                                         \
  do {                                                                \
    hipError_t e = (x);                                               \
    if (e != hipSuccess) {                                            \
      printf("%s: %s\n", #x, hipGetErrorString(e));                   \
      return 1;                                                       \
    }                                                                 \
  } while (0)

constexpr int ITERS = 4096;

__global__ void __launch_bounds__(256) k_bitop3(uint32_t* out, uint32_t seed) {
  uint32_t v[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = seed * (threadIdx.x + 1) + i;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = __builtin_amdgcn_bitop3_b32(v[i], v[(i + 1) & 15], v[(i + 5) & 15], 0x96);
  }
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) r ^= v[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void __launch_bounds__(256) k_alignbit(uint32_t* out, uint32_t seed) {
  uint32_t v[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = seed * (threadIdx.x + 1) + i;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = __builtin_amdgcn_alignbit(v[i], v[(i + 3) & 15], 7 + (i & 7));
  }
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) r ^= v[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void __launch_bounds__(256) k_perm(uint32_t* out, uint32_t seed) {
  uint32_t v[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = seed * (threadIdx.x + 1) + i;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 16; ++i)
      v[i] = __builtin_amdgcn_perm(v[i], v[(i + 3) & 15], 0x04030201u + 0x01010101u * (i & 3));
  }
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) r ^= v[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void __launch_bounds__(256) k_mad64(uint32_t* out, uint32_t seed) {
  uint64_t v[8];
  uint32_t m[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    v[i] = seed * (threadIdx.x + 1) + i;
    m[i] = seed ^ (i * 0x9E3779B9u);
  }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (uint64_t)m[i] * (uint32_t)v[(i + 1) & 7] + v[i];
  }
  uint64_t r = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) r ^= v[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)r ^ (uint32_t)(r >> 32);
}

__global__ void __launch_bounds__(256) k_f128mul(uint32_t* out, uint32_t seed) {
  using FO = Field128Ops;
  F128 a[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) a[i] = F128{{seed + threadIdx.x, (uint32_t)i, 7u, 0x1000u}};
  const F128 b = F128{{seed, 3u, 5u, 0x7FFu}};
  for (int it = 0; it < ITERS / 16; ++it) {
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] = FO::mul(a[i], b);
  }
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) r ^= a[i].w[0] ^ a[i].w[3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void __launch_bounds__(256) k_keccak(uint32_t* out, uint32_t seed) {
  uint64_t s[25];
#pragma unroll
  for (int i = 0; i < 25; ++i) s[i] = (uint64_t)(seed + threadIdx.x) * (i + 1);
  for (int it = 0; it < ITERS / 64; ++it) keccak_p<24>(s);
  uint64_t r = 0;
#pragma unroll
  for (int i = 0; i < 25; ++i) r ^= s[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)r;
}

typedef void (*kfn)(uint32_t*, uint32_t);

static int run(const char* name, kfn k, double ops_per_thread, const char* unit, int blocks,
               uint32_t* d) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, d, 1u);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a, 0));
  const int reps = 5;
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, d, 2u + r);
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  double total = ops_per_thread * 256.0 * blocks * reps;
  printf("{\"bench\": \"%s\", \"rate\": %.4g, \"unit\": \"%s\", \"ms\": %.3f}\n", name,
         total / (ms * 1e-3), unit, ms / reps);
  return 0;
}

int main() {
  int blocks = 256 * 8 * 4;  // 8 blocks of 256 threads per CU x 4 rounds
  uint32_t* d;
  CK(hipMalloc(&d, (size_t)blocks * 256 * 4));
  run("int32 bitop3 (xor3)", k_bitop3, 16.0 * ITERS, "lane-ops/s", blocks, d);
  run("int32 alignbit", k_alignbit, 16.0 * ITERS, "lane-ops/s", blocks, d);
  run("int32 v_perm_b32", k_perm, 16.0 * ITERS, "lane-ops/s", blocks, d);
  run("v_mad_u64_u32", k_mad64, 8.0 * ITERS, "lane-ops/s", blocks, d);
  run("Field128 mont mul", k_f128mul, 4.0 * (ITERS / 16), "mul/s", blocks, d);
  run("Keccak-f[1600]", k_keccak, (double)(ITERS / 64), "perm/s", blocks, d);
  CK(hipFree(d));
  return 0;
}
