// Field128 Montgomery multiplication throughput/latency on gfx950: the compiler's Field128Ops::mul
// vs mont_mul3 (three products interleaved in one hazard-free asm stream, tools/gen_mont3.py).
// Each lane runs three independent chains x_s <- x_s * y_s; results must agree bit for bit.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/mb_mont3 tools/mb_mont3.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "../janus_amd/csrc/mont3.h"

#define CK(x)                                                   \
  do {                                                          \
    hipError_t e = (x);                                         \
    if (e != hipSuccess) {                                      \
      printf("%s: %s\n", #x, hipGetErrorString(e));             \
      return 1;                                                 \
    }                                                           \
  } while (0)

template <int V>
__global__ void __launch_bounds__(256) k_chain(F128* io, int iters) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  F128 x0 = io[6 * t], x1 = io[6 * t + 1], x2 = io[6 * t + 2];
  const F128 y0 = io[6 * t + 3], y1 = io[6 * t + 4], y2 = io[6 * t + 5];
  for (int i = 0; i < iters; ++i) {
    if constexpr (V == 0) {
      x0 = Field128Ops::mul(x0, y0);
      x1 = Field128Ops::mul(x1, y1);
      x2 = Field128Ops::mul(x2, y2);
    } else {
      F128 r0, r1, r2;
      mont_mul3(x0, y0, x1, y1, x2, y2, r0, r1, r2);
      x0 = r0;
      x1 = r1;
      x2 = r2;
    }
  }
  io[6 * t] = x0;
  io[6 * t + 1] = x1;
  io[6 * t + 2] = x2;
}

int main() {
  const int maxb = 256 * 16;
  const size_t nl = (size_t)maxb * 256;
  F128* h = (F128*)malloc(nl * 6 * sizeof(F128));
  uint64_t s = 0x9E3779B97F4A7C15ull;
  for (size_t i = 0; i < nl * 6; ++i) {
    for (int w = 0; w < 4; ++w) {
      s ^= s << 13; s ^= s >> 7; s ^= s << 17;
      h[i].w[w] = (uint32_t)s;
    }
    h[i].w[3] &= 0x7FFFFFFFu;  // < p
  }
  F128 *d0, *d1;
  CK(hipMalloc(&d0, nl * 6 * sizeof(F128)));
  CK(hipMalloc(&d1, nl * 6 * sizeof(F128)));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int iters = 400;
  const int blocks[] = {256, 1024, 4096};
  int bad = 0;
  for (int bi = 0; bi < 3; ++bi) {
    const int nb = blocks[bi];
    float ms[2];
    for (int v = 0; v < 2; ++v) {
      F128* d = v ? d1 : d0;
      CK(hipMemcpy(d, h, nl * 6 * sizeof(F128), hipMemcpyHostToDevice));
      if (v == 0) k_chain<0><<<nb, 256>>>(d, 2); else k_chain<1><<<nb, 256>>>(d, 2);
      CK(hipMemcpy(d, h, nl * 6 * sizeof(F128), hipMemcpyHostToDevice));
      CK(hipEventRecord(a));
      if (v == 0) k_chain<0><<<nb, 256>>>(d, iters); else k_chain<1><<<nb, 256>>>(d, iters);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      CK(hipEventElapsedTime(&ms[v], a, b));
    }
    F128* o0 = (F128*)malloc((size_t)nb * 256 * 6 * sizeof(F128));
    F128* o1 = (F128*)malloc((size_t)nb * 256 * 6 * sizeof(F128));
    CK(hipMemcpy(o0, d0, (size_t)nb * 256 * 6 * sizeof(F128), hipMemcpyDeviceToHost));
    CK(hipMemcpy(o1, d1, (size_t)nb * 256 * 6 * sizeof(F128), hipMemcpyDeviceToHost));
    size_t diff = 0;
    for (size_t i = 0; i < (size_t)nb * 256 * 6; ++i)
      for (int w = 0; w < 4; ++w) diff += o0[i].w[w] != o1[i].w[w];
    bad += diff != 0;
    const double mults = 3.0 * iters * nb * 256;
    printf("{\"bench\": \"mont_mul\", \"blocks\": %d, \"compiler_mul_per_s\": %.4g, "
           "\"mont_mul3_per_s\": %.4g, \"speedup\": %.3f, \"mismatched_words\": %zu}\n",
           nb, mults / (ms[0] * 1e-3), mults / (ms[1] * 1e-3), ms[0] / ms[1], diff);
    free(o0);
    free(o1);
  }
  return bad;
}
