// Bias of the device math the decoder's activations use (parity diagnostics): ELU = expm1f(x)
// for x < 0, sigmoid = 1 / (1 + expf(-x)), over dense grids; mean signed error and RMS in ulps
// of the result against fp64, and the fraction correctly rounded.
//   hipcc -O3 --offload-arch=gfx950 act_round.hip -o act_round && ./act_round
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <vector>

__global__ void k_act(const float* x, float* elu, float* sig, float* ex, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float v = x[i];
  elu[i] = expm1f(v);
  sig[i] = 1.f / (1.f + expf(-v));
  ex[i] = expf(v);
}

static double ulp(float f) { return std::ldexp(1.0, std::ilogb(f == 0.f ? 1e-30f : f) - 23); }

static void stat(const char* name, const std::vector<float>& got, const std::vector<double>& ex) {
  double s = 0, s2 = 0;
  long eq = 0;
  for (size_t i = 0; i < got.size(); ++i) {
    const float r = (float)ex[i];
    eq += got[i] == r;
    const double e = ((double)got[i] - ex[i]) / ulp(r);
    s += e;
    s2 += e * e;
  }
  printf("%-28s n=%zu  correctly rounded %.4f  mean %+.4f ulp  rms %.4f ulp\n", name, got.size(),
         (double)eq / got.size(), s / got.size(), std::sqrt(s2 / got.size()));
}

int main() {
  const int n = 1 << 22;
  std::vector<float> x(n);
  for (int i = 0; i < n; ++i) x[i] = -8.f + 8.f * (float)i / n;       // ELU's negative side
  float *dx, *de, *ds, *dq;
  hipMalloc(&dx, n * 4);
  hipMalloc(&de, n * 4);
  hipMalloc(&ds, n * 4);
  hipMalloc(&dq, n * 4);
  hipMemcpy(dx, x.data(), n * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_act, dim3(n / 256), dim3(256), 0, 0, dx, de, ds, dq, n);
  std::vector<float> e(n), s(n), q(n);
  hipMemcpy(e.data(), de, n * 4, hipMemcpyDeviceToHost);
  hipMemcpy(s.data(), ds, n * 4, hipMemcpyDeviceToHost);
  hipMemcpy(q.data(), dq, n * 4, hipMemcpyDeviceToHost);
  std::vector<double> re(n), rs(n), rq(n);
  for (int i = 0; i < n; ++i) {
    re[i] = std::expm1((double)x[i]);
    rs[i] = 1.0 / (1.0 + std::exp(-(double)x[i]));
    rq[i] = std::exp((double)x[i]);
  }
  stat("expm1f on [-8, 0)", e, re);
  stat("1/(1+expf(-x)) on [-8, 0)", s, rs);
  stat("expf on [-8, 0)", q, rq);
  // sigmoid on the positive side too
  for (int i = 0; i < n; ++i) x[i] = 8.f * (float)i / n;
  hipMemcpy(dx, x.data(), n * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_act, dim3(n / 256), dim3(256), 0, 0, dx, de, ds, dq, n);
  hipMemcpy(s.data(), ds, n * 4, hipMemcpyDeviceToHost);
  for (int i = 0; i < n; ++i) rs[i] = 1.0 / (1.0 + std::exp(-(double)x[i]));
  stat("1/(1+expf(-x)) on [0, 8)", s, rs);
  hipFree(dx); hipFree(de); hipFree(ds); hipFree(dq);
  return 0;
}
