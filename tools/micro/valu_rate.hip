// VALU issue-rate probe (gfx950): scalar v_fma_f32 vs packed v_pk_fma_f32 chains, 8 independent
// chains per lane, W waves per SIMD.  Prints G FMA-lanes/s per variant.
//   hipcc -O3 -fno-slp-vectorize --offload-arch=gfx950 valu_rate.hip -o valu_rate && ./valu_rate
// (-fno-slp-vectorize keeps the scalar variant scalar: SLP would pack it into v_pk_fma_f32)
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256) void k_fma(float* out, float s, int iters) {
  float a[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = threadIdx.x * 1e-3f + i;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 16; ++r)
#pragma unroll
      for (int i = 0; i < 8; ++i) a[i] = __builtin_fmaf(a[i], s, 0.5f);
  }
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) t += a[i];
  out[blockIdx.x * 256 + threadIdx.x] = t;
}

__global__ __launch_bounds__(256) void k_pkfma(float* out, float s, int iters) {
  f2 a[8];
  const f2 sv = {s, s}, h = {0.5f, 0.5f};
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = (f2){threadIdx.x * 1e-3f + i, threadIdx.x * 2e-3f + i};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 16; ++r)
#pragma unroll
      for (int i = 0; i < 8; ++i) a[i] = __builtin_elementwise_fma(a[i], sv, h);
  }
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) t += a[i].x + a[i].y;
  out[blockIdx.x * 256 + threadIdx.x] = t;
}

int main() {
  float* d;
  const int blocks = 256 * 8;   // 8 blocks/CU of 4 waves = 8 waves/SIMD
  hipMalloc(&d, blocks * 256 * 4);
  const int iters = 4000;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int rep = 0; rep < 2; ++rep) {
    for (int v = 0; v < 2; ++v) {
      for (int bl : {256 * 1, 256 * 2, 256 * 8}) {
        hipEventRecord(e0);
        if (v == 0) hipLaunchKernelGGL(k_fma, dim3(bl), dim3(256), 0, 0, d, 0.999f, iters);
        else hipLaunchKernelGGL(k_pkfma, dim3(bl), dim3(256), 0, 0, d, 0.999f, iters);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        const double lanes_fma = (double)bl * 256 * iters * 16 * 8 * (v ? 2 : 1);
        if (rep) printf("%s waves/SIMD=%d: %.1f G lane-FMA/s = %.1f TFLOP/s\n", v ? "v_pk_fma_f32" : "v_fma_f32   ",
                        bl / 256, lanes_fma / ms / 1e6, 2 * lanes_fma / ms / 1e9);
      }
    }
  }
  hipFree(d);
  return 0;
}
