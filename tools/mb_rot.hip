// Issue-rate microbenchmark of the VALU instructions a Keccak-f[1600] rotation can be built from
// on gfx950 (measurement tooling, not product code): 32-bit funnel shifts (v_alignbit_b32,
// v_alignbyte_b32), 32-bit shift/or forms, and the 64-bit shifts (v_lshlrev_b64,
// v_lshrrev_b64, v_lshl_add_u64).  Each kernel streams independent instructions over 16 registers
// (inline asm, so the compiler cannot substitute), every CU busy.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/mb_rot tools/mb_rot.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CK(x)                                                         \
  do {                                                                \
    hipError_t e = (x);                                               \
    if (e != hipSuccess) {                                            \
      printf("%s: %s\n", #x, hipGetErrorString(e));                   \
      return 1;                                                       \
    }                                                                 \
  } while (0)

constexpr int ITERS = 2048;

#define K32(NAME, ASM)                                                                  \
  __global__ void __launch_bounds__(256) NAME(uint32_t* out, uint32_t seed) {            \
    uint32_t v[16];                                                                     \
    _Pragma("unroll") for (int i = 0; i < 16; ++i) v[i] = seed * (threadIdx.x + 1) + i; \
    for (int it = 0; it < ITERS; ++it) {                                                \
      _Pragma("unroll") for (int i = 0; i < 16; ++i) {                                  \
        uint32_t a = v[i], b = v[(i + 3) & 15], c = v[(i + 7) & 15];                    \
        asm volatile(ASM : "+v"(a) : "v"(b), "v"(c));                                   \
        v[i] = a;                                                                       \
      }                                                                                 \
    }                                                                                   \
    uint32_t r = 0;                                                                     \
    _Pragma("unroll") for (int i = 0; i < 16; ++i) r ^= v[i];                           \
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;                                     \
  }

#define K64(NAME, ASM)                                                                  \
  __global__ void __launch_bounds__(256) NAME(uint32_t* out, uint32_t seed) {            \
    uint64_t v[8];                                                                      \
    _Pragma("unroll") for (int i = 0; i < 8; ++i) v[i] = (uint64_t)seed * (threadIdx.x + 1) + i; \
    for (int it = 0; it < ITERS; ++it) {                                                \
      _Pragma("unroll") for (int i = 0; i < 8; ++i) {                                   \
        uint64_t a = v[i], b = v[(i + 3) & 7];                                          \
        asm volatile(ASM : "+v"(a) : "v"(b));                                           \
        v[i] = a;                                                                       \
      }                                                                                 \
    }                                                                                   \
    uint64_t r = 0;                                                                     \
    _Pragma("unroll") for (int i = 0; i < 8; ++i) r ^= v[i];                            \
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(r ^ (r >> 32));             \
  }

K32(k_xor, "v_xor_b32 %0, %0, %1")
K32(k_bitop3, "v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96")
K32(k_alignbit, "v_alignbit_b32 %0, %0, %1, 13")
K32(k_alignbyte, "v_alignbyte_b32 %0, %0, %1, 3")
K32(k_lshl_or, "v_lshl_or_b32 %0, %0, 13, %1")
K32(k_lshr, "v_lshrrev_b32 %0, 13, %0")
K32(k_perm, "v_perm_b32 %0, %0, %1, %2")
K64(k_lshl64, "v_lshlrev_b64 %0, 13, %0")
K64(k_lshr64, "v_lshrrev_b64 %0, 13, %0")
K64(k_lshl_add64, "v_lshl_add_u64 %0, %0, 13, %1")
// a whole 64-bit rotate, two ways (2 instructions each)
__global__ void __launch_bounds__(256) k_rot_align(uint32_t* out, uint32_t seed) {
  uint32_t lo[8], hi[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    lo[i] = seed * (threadIdx.x + 1) + i;
    hi[i] = lo[i] ^ 0x5555u;
  }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      uint32_t a = lo[i], b = hi[i], na, nb;
      asm volatile("v_alignbit_b32 %0, %2, %3, 13\n\tv_alignbit_b32 %1, %3, %2, 13"
                   : "=&v"(na), "=&v"(nb) : "v"(a), "v"(b));
      lo[i] = na;
      hi[i] = nb;
    }
  }
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) r ^= lo[i] ^ hi[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
__global__ void __launch_bounds__(256) k_rot_lshl_add(uint32_t* out, uint32_t seed) {
  uint64_t v[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = (uint64_t)seed * (threadIdx.x + 1) + i;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      uint64_t a = v[i], t;
      asm volatile("v_lshrrev_b64 %1, 51, %0\n\tv_lshl_add_u64 %0, %0, 13, %1"
                   : "+v"(a), "=&v"(t));
      v[i] = a;
    }
  }
  uint64_t r = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) r ^= v[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(r ^ (r >> 32));
}

int run(const char* name, void (*k)(uint32_t*, uint32_t), double ops_per_thread, uint32_t* d,
        int blocks) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, d, 1u);
  CK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int rep = 0; rep < 5; ++rep) {
    CK(hipEventRecord(a, 0));
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, d, 1u + rep);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    if (ms < best) best = ms;
  }
  const double lane_ops = ops_per_thread * 256.0 * blocks;
  printf("{\"bench\": \"%s\", \"lane_ops_per_s\": %.4g, \"wave_instr_per_cu_per_ns\": %.4f, "
         "\"ms\": %.3f}\n",
         name, lane_ops / (best * 1e-3), lane_ops / 64.0 / 256.0 / (best * 1e6), best);
  return 0;
}

int main() {
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int blocks = cus * 16;  // 16 waves per CU
  uint32_t* d;
  CK(hipMalloc(&d, (size_t)blocks * 256 * 4));
  const double n32 = 16.0 * ITERS, n64 = 8.0 * ITERS;
  run("v_xor_b32", k_xor, n32, d, blocks);
  run("v_bitop3_b32", k_bitop3, n32, d, blocks);
  run("v_alignbit_b32", k_alignbit, n32, d, blocks);
  run("v_alignbyte_b32", k_alignbyte, n32, d, blocks);
  run("v_lshl_or_b32", k_lshl_or, n32, d, blocks);
  run("v_lshrrev_b32", k_lshr, n32, d, blocks);
  run("v_perm_b32", k_perm, n32, d, blocks);
  run("v_lshlrev_b64", k_lshl64, n64, d, blocks);
  run("v_lshrrev_b64", k_lshr64, n64, d, blocks);
  run("v_lshl_add_u64", k_lshl_add64, n64, d, blocks);
  run("rot64 = 2 x v_alignbit_b32 (per rotate)", k_rot_align, n64, d, blocks);
  run("rot64 = v_lshrrev_b64 + v_lshl_add_u64 (per rotate)", k_rot_lshl_add, n64, d, blocks);
  CK(hipFree(d));
  return 0;
}
