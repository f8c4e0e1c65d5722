// Where do the waves of a multi-wave workgroup run?  Each wave records HW_ID (SIMD, CU, SE) and
// runs a Keccak-f chain on its own lane states; if the two waves of a 2-wave workgroup shared a
// SIMD the chain time per permutation would double against 1-wave workgroups.  Diagnostic for
// k_helper_xof's producer/consumer pair.
//   hipcc --offload-arch=gfx950 -O3 -o tools/mb_wave_place tools/mb_wave_place.hip
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

__global__ void k_chain(uint64_t* io, uint32_t* hwid, int nperm) {
  const size_t st = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if ((threadIdx.x & 63u) == 0u)
    hwid[st >> 6] = __builtin_amdgcn_s_getreg(4 | (31 << 11));  // HW_REG_HW_ID, 32 bits
  uint64_t s[25];
#pragma unroll
  for (int i = 0; i < 25; ++i) s[i] = io[st * 25 + i];
  for (int k = 0; k < nperm; ++k) keccak_p<24>(s);
#pragma unroll
  for (int i = 0; i < 25; ++i) io[st * 25 + i] = s[i];
}

int main() {
  const int NB = 128, NPERM = 4000, MAXT = 256;
  const size_t NST = (size_t)NB * MAXT;
  uint64_t* h = (uint64_t*)malloc(NST * 25 * 8);
  for (size_t i = 0; i < NST * 25; ++i) h[i] = 0x9E3779B97F4A7C15ull * (i + 1);
  uint64_t* d;
  uint32_t* dh;
  CK(hipMalloc(&d, NST * 25 * 8));
  CK(hipMalloc(&dh, NST / 64 * 4));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int thr = 64; thr <= MAXT; thr *= 2) {
    CK(hipMemcpy(d, h, NST * 25 * 8, hipMemcpyHostToDevice));
    k_chain<<<NB, thr>>>(d, dh, 1);
    CK(hipEventRecord(a));
    k_chain<<<NB, thr>>>(d, dh, NPERM);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    const int nw = NB * thr / 64;
    uint32_t* hw = (uint32_t*)malloc(nw * 4);
    CK(hipMemcpy(hw, dh, nw * 4, hipMemcpyDeviceToHost));
    int same_simd = 0, same_cu = 0;
    const int wpb = thr / 64;
    for (int blk = 0; blk < NB; ++blk)
      for (int w = 1; w < wpb; ++w) {
        const uint32_t x = hw[blk * wpb], y = hw[blk * wpb + w];
        const uint32_t cux = x >> 8 & 0xFF, cuy = y >> 8 & 0xFF;  // CU, SH, SE bits
        if (cux == cuy) {
          ++same_cu;
          if ((x >> 4 & 3) == (y >> 4 & 3)) ++same_simd;
        }
      }
    printf("waves/workgroup %d: %.3f us per permutation; wave pairs in one workgroup: same CU %d, "
           "same SIMD %d of %d; block0 hwids:", wpb, ms * 1e3 / NPERM, same_cu, same_simd,
           NB * (wpb - 1));
    for (int w = 0; w < wpb; ++w) printf(" %08x", hw[w]);
    printf("\n");
    free(hw);
  }
  return 0;
}
