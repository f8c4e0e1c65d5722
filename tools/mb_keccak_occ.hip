// Keccak-f[1600] throughput vs waves per SIMD and per-permutation memory traffic, gfx950
// (measurement infrastructure, not product code).  Occupancy is pinned with dynamic LDS:
// 160 KiB / k per 256-thread block -> k blocks per CU -> k waves per SIMD; the grid is exactly
// 256 CUs x k blocks x ROUNDS.  Variants (one 168-byte rate block per permutation and lane):
//   reg      : state in registers only (the permutation alone)
//   st8      : + 21 x 8-B stores to the lane's own row (row-strided: 64 rows per store)
//   st16     : + 10 x 16-B stores to the lane's own row (k_expand's pattern)
//   st16nt   : st16 with non-temporal stores
//   ld16     : + 11 x 16-B loads of the lane's own row, absorbed (per-lane row-strided loads)
//   lds      : + 10 ds_write_b128 + 10 ds_read_b128 of a 160-B LDS row (no global traffic)
//   st16c    : + 10 x 16-B stores, COALESCED: the wave's 64 lanes write 1 KB contiguous per store
//              (a 64-report tile, element-major), instead of one row per lane
//   ld16c    : + 11 x 16-B loads, coalesced the same way
//   *_stg    : the same with odd blocks starting half a permutation late (breaks the lockstep of
//              the waves that share a SIMD, so their memory phases do not coincide)
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
constexpr size_t ROW = PERMS * 168 + 16;

template <int V, bool STG = false>
__global__ void __launch_bounds__(256) k_var(uint32_t* out, uint32_t seed, uint8_t* rows) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const size_t gid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint8_t* row = rows + gid * ROW;
  uint64_t s[25];
#pragma unroll
  for (int i = 0; i < 25; ++i) s[i] = (uint64_t)(seed + threadIdx.x) * (i + 1);
  if (STG && (blockIdx.x & 1)) keccak_p<12>(s);
  for (int it = 0; it < PERMS; ++it) {
    if constexpr (V == 7) {  // ld16c
      const ulonglong2* src = reinterpret_cast<const ulonglong2*>(
          rows + (gid >> 6) * 64 * ROW + ((size_t)it * 10 * 64 + (gid & 63)) * 16);
#pragma unroll
      for (int k = 0; k < 10; ++k) {
        const ulonglong2 v = src[k * 64];
        s[2 * k] ^= v.x;
        s[2 * k + 1] ^= v.y;
      }
    }
    if constexpr (V == 4) {  // ld16
      const ulonglong2* src = reinterpret_cast<const ulonglong2*>(row + (size_t)it * 168);
#pragma unroll
      for (int k = 0; k < 10; ++k) {
        const ulonglong2 v = src[k];
        s[2 * k] ^= v.x;
        s[2 * k + 1] ^= v.y;
      }
    }
    keccak_p<24>(s);
    uint8_t* o = row + (size_t)it * 168;
    if constexpr (V == 1) {
#pragma unroll
      for (int w = 0; w < 21; ++w) reinterpret_cast<uint64_t*>(o)[w] = s[w];
    } else if constexpr (V == 2) {
      ulonglong2* d = reinterpret_cast<ulonglong2*>(row + (size_t)(it & ~1) * 168);
#pragma unroll
      for (int k = 0; k < 10; ++k) d[k] = make_ulonglong2(s[2 * k], s[2 * k + 1]);
    } else if constexpr (V == 6) {
      ulonglong2* d = reinterpret_cast<ulonglong2*>(
          rows + (gid >> 6) * 64 * ROW + ((size_t)(it & ~1) * 10 * 64 + (gid & 63)) * 16);
#pragma unroll
      for (int k = 0; k < 10; ++k) d[k * 64] = make_ulonglong2(s[2 * k], s[2 * k + 1]);
    } else if constexpr (V == 3) {
      ulonglong2* d = reinterpret_cast<ulonglong2*>(row + (size_t)(it & ~1) * 168);
#pragma unroll
      for (int k = 0; k < 10; ++k) {
        __builtin_nontemporal_store(s[2 * k], &d[k].x);
        __builtin_nontemporal_store(s[2 * k + 1], &d[k].y);
      }
    } else if constexpr (V == 5) {
      ulonglong2* w = reinterpret_cast<ulonglong2*>(lds + (threadIdx.x & 63) * 160 +
                                                    (threadIdx.x >> 6) * 10240);
#pragma unroll
      for (int k = 0; k < 10; ++k) w[k] = make_ulonglong2(s[2 * k], s[2 * k + 1]);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      const ulonglong2* r = reinterpret_cast<const ulonglong2*>(
          lds + ((threadIdx.x + 7) & 63) * 160 + (threadIdx.x >> 6) * 10240);
#pragma unroll
      for (int k = 0; k < 10; ++k) {
        const ulonglong2 v = r[k];
        s[2 * k + 1] ^= v.x & 1ull;
        s[2 * k] ^= v.y & 1ull;
      }
    }
  }
  uint64_t r = 0;
#pragma unroll
  for (int i = 0; i < 25; ++i) r ^= s[i];
  out[gid] = (uint32_t)r;
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
  const size_t lanes = (size_t)256 * 4 * rounds * 256;  // up to 4 waves per SIMD
  uint32_t* d;
  uint8_t* rows;
  CK(hipMalloc(&d, lanes * 4));
  CK(hipMalloc(&rows, lanes * ROW));
  CK(hipMemset(rows, 0, lanes * ROW));
  const char* names[6] = {"reg", "st16", "st16c", "ld16", "ld16c", "lds"};
  kfn ks[6] = {k_var<0>, k_var<2>, k_var<6>, k_var<4>, k_var<7>, k_var<5>};
  for (int v = 0; v < 6; ++v)
    for (int k = 2; k <= 4; ++k) run(names[v], ks[v], k, d, rows, rounds);
  CK(hipFree(d));
  CK(hipFree(rows));
  return 0;
}
