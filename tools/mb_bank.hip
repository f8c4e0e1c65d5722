// VGPR bank microbenchmark (measurement tooling, not product code): 16 independent v_bitop3_b32 /
// v_alignbit_b32 per asm block with explicit registers whose source operands sit in distinct or
// in the same VGPR bank (register index mod 4), one wave per SIMD and four.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/mb_bank tools/mb_bank.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
constexpr int ITERS = 4096;
#define CLOB "v0","v1","v2","v3","v4","v5","v6","v7","v8","v9","v10","v11","v12","v13","v14","v15","v16","v17","v18","v19","v20","v21","v22","v23","v24","v25","v26","v27","v28","v29","v30","v31","v32","v33","v34","v35","v36","v37","v38","v39","v40","v41","v42","v43","v44","v45","v46","v47","v48","v49","v50","v51","v52","v53","v54","v55"
__global__ void __launch_bounds__(64) k_bitop3_nb(uint32_t* out) {
  for (int it = 0; it < ITERS; ++it) {
    asm volatile("v_bitop3_b32 v40, v1, v2, v3 bitop3:0x96\n\tv_bitop3_b32 v41, v5, v6, v7 bitop3:0x96\n\tv_bitop3_b32 v42, v9, v10, v11 bitop3:0x96\n\tv_bitop3_b32 v43, v13, v14, v15 bitop3:0x96\n\tv_bitop3_b32 v44, v1, v2, v3 bitop3:0x96\n\tv_bitop3_b32 v45, v5, v6, v7 bitop3:0x96\n\tv_bitop3_b32 v46, v9, v10, v11 bitop3:0x96\n\tv_bitop3_b32 v47, v13, v14, v15 bitop3:0x96\n\tv_bitop3_b32 v48, v1, v2, v3 bitop3:0x96\n\tv_bitop3_b32 v49, v5, v6, v7 bitop3:0x96\n\tv_bitop3_b32 v50, v9, v10, v11 bitop3:0x96\n\tv_bitop3_b32 v51, v13, v14, v15 bitop3:0x96\n\tv_bitop3_b32 v52, v1, v2, v3 bitop3:0x96\n\tv_bitop3_b32 v53, v5, v6, v7 bitop3:0x96\n\tv_bitop3_b32 v54, v9, v10, v11 bitop3:0x96\n\tv_bitop3_b32 v55, v13, v14, v15 bitop3:0x96" ::: CLOB);
  }
  if (threadIdx.x == 0) out[blockIdx.x] = 1u;
}
__global__ void __launch_bounds__(64) k_bitop3_b2(uint32_t* out) {
  for (int it = 0; it < ITERS; ++it) {
    asm volatile("v_bitop3_b32 v40, v1, v5, v3 bitop3:0x96\n\tv_bitop3_b32 v41, v5, v9, v7 bitop3:0x96\n\tv_bitop3_b32 v42, v9, v13, v11 bitop3:0x96\n\tv_bitop3_b32 v43, v13, v17, v15 bitop3:0x96\n\tv_bitop3_b32 v44, v1, v5, v3 bitop3:0x96\n\tv_bitop3_b32 v45, v5, v9, v7 bitop3:0x96\n\tv_bitop3_b32 v46, v9, v13, v11 bitop3:0x96\n\tv_bitop3_b32 v47, v13, v17, v15 bitop3:0x96\n\tv_bitop3_b32 v48, v1, v5, v3 bitop3:0x96\n\tv_bitop3_b32 v49, v5, v9, v7 bitop3:0x96\n\tv_bitop3_b32 v50, v9, v13, v11 bitop3:0x96\n\tv_bitop3_b32 v51, v13, v17, v15 bitop3:0x96\n\tv_bitop3_b32 v52, v1, v5, v3 bitop3:0x96\n\tv_bitop3_b32 v53, v5, v9, v7 bitop3:0x96\n\tv_bitop3_b32 v54, v9, v13, v11 bitop3:0x96\n\tv_bitop3_b32 v55, v13, v17, v15 bitop3:0x96" ::: CLOB);
  }
  if (threadIdx.x == 0) out[blockIdx.x] = 1u;
}
__global__ void __launch_bounds__(64) k_bitop3_b3(uint32_t* out) {
  for (int it = 0; it < ITERS; ++it) {
    asm volatile("v_bitop3_b32 v40, v1, v5, v9 bitop3:0x96\n\tv_bitop3_b32 v41, v5, v9, v13 bitop3:0x96\n\tv_bitop3_b32 v42, v9, v13, v17 bitop3:0x96\n\tv_bitop3_b32 v43, v13, v17, v21 bitop3:0x96\n\tv_bitop3_b32 v44, v1, v5, v9 bitop3:0x96\n\tv_bitop3_b32 v45, v5, v9, v13 bitop3:0x96\n\tv_bitop3_b32 v46, v9, v13, v17 bitop3:0x96\n\tv_bitop3_b32 v47, v13, v17, v21 bitop3:0x96\n\tv_bitop3_b32 v48, v1, v5, v9 bitop3:0x96\n\tv_bitop3_b32 v49, v5, v9, v13 bitop3:0x96\n\tv_bitop3_b32 v50, v9, v13, v17 bitop3:0x96\n\tv_bitop3_b32 v51, v13, v17, v21 bitop3:0x96\n\tv_bitop3_b32 v52, v1, v5, v9 bitop3:0x96\n\tv_bitop3_b32 v53, v5, v9, v13 bitop3:0x96\n\tv_bitop3_b32 v54, v9, v13, v17 bitop3:0x96\n\tv_bitop3_b32 v55, v13, v17, v21 bitop3:0x96" ::: CLOB);
  }
  if (threadIdx.x == 0) out[blockIdx.x] = 1u;
}
__global__ void __launch_bounds__(64) k_align_nb(uint32_t* out) {
  for (int it = 0; it < ITERS; ++it) {
    asm volatile("v_alignbit_b32 v40, v1, v2, 13\n\tv_alignbit_b32 v41, v5, v6, 13\n\tv_alignbit_b32 v42, v9, v10, 13\n\tv_alignbit_b32 v43, v13, v14, 13\n\tv_alignbit_b32 v44, v1, v2, 13\n\tv_alignbit_b32 v45, v5, v6, 13\n\tv_alignbit_b32 v46, v9, v10, 13\n\tv_alignbit_b32 v47, v13, v14, 13\n\tv_alignbit_b32 v48, v1, v2, 13\n\tv_alignbit_b32 v49, v5, v6, 13\n\tv_alignbit_b32 v50, v9, v10, 13\n\tv_alignbit_b32 v51, v13, v14, 13\n\tv_alignbit_b32 v52, v1, v2, 13\n\tv_alignbit_b32 v53, v5, v6, 13\n\tv_alignbit_b32 v54, v9, v10, 13\n\tv_alignbit_b32 v55, v13, v14, 13" ::: CLOB);
  }
  if (threadIdx.x == 0) out[blockIdx.x] = 1u;
}
__global__ void __launch_bounds__(64) k_align_b2(uint32_t* out) {
  for (int it = 0; it < ITERS; ++it) {
    asm volatile("v_alignbit_b32 v40, v1, v5, 13\n\tv_alignbit_b32 v41, v5, v9, 13\n\tv_alignbit_b32 v42, v9, v13, 13\n\tv_alignbit_b32 v43, v13, v17, 13\n\tv_alignbit_b32 v44, v1, v5, 13\n\tv_alignbit_b32 v45, v5, v9, 13\n\tv_alignbit_b32 v46, v9, v13, 13\n\tv_alignbit_b32 v47, v13, v17, 13\n\tv_alignbit_b32 v48, v1, v5, 13\n\tv_alignbit_b32 v49, v5, v9, 13\n\tv_alignbit_b32 v50, v9, v13, 13\n\tv_alignbit_b32 v51, v13, v17, 13\n\tv_alignbit_b32 v52, v1, v5, 13\n\tv_alignbit_b32 v53, v5, v9, 13\n\tv_alignbit_b32 v54, v9, v13, 13\n\tv_alignbit_b32 v55, v13, v17, 13" ::: CLOB);
  }
  if (threadIdx.x == 0) out[blockIdx.x] = 1u;
}
int main() {
  uint32_t* d;
  CK(hipMalloc(&d, 1 << 20));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  typedef void (*K)(uint32_t*);
  const K ks[] = {k_bitop3_nb, k_bitop3_b2, k_bitop3_b3, k_align_nb, k_align_b2};
  const char* names[] = {"bitop3_nb", "bitop3_b2", "bitop3_b3", "align_nb", "align_b2"};
  for (int waves : {1024, 4096}) {
    for (int i = 0; i < 5; ++i) {
      hipLaunchKernelGGL(ks[i], dim3(waves), dim3(64), 0, 0, d);
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(a));
      for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(ks[i], dim3(waves), dim3(64), 0, 0, d);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      const double instr = 5.0 * waves * ITERS * 16.0;  // wave-instructions
      // per SIMD (1024 SIMDs): wave-instructions per microsecond; cycles at 2.4 GHz per instr
      const double per_simd = instr / 1024.0;
      printf("waves %5d %-10s %8.3f ms  %6.2f ns/wave-instr/SIMD  (%.2f cyc @2.4GHz)\n", waves, names[i], ms / 5,
             ms * 1e6 / per_simd, ms * 1e6 / per_simd * 2.4);
    }
  }
  return 0;
}
