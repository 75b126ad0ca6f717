// Rounding of the MFMA accumulation on gfx950 (parity diagnostics): is D = A*B + C of
// v_mfma_f32_32x32x16_bf16 (and of v_mfma_f32_32x32x2_f32) the round-to-nearest-even fp32 of
// the exact value, and is its error biased?  Random bf16 / fp32 operands (exact products and
// sums in fp64), one wave per trial; prints the fraction of results equal to RNE(exact), the
// mean and RMS of the signed error in ulps of the result, and the same for a single fp32 fma
// chain (the reference rounding).
//   hipcc -O3 --offload-arch=gfx950 mfma_round.hip -o mfma_round && ./mfma_round
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// A [T][32][16] bf16 (as uint16), B [T][16][32], C/D [T][32][32]
__global__ __launch_bounds__(64) void k_bf16(const uint16_t* A, const uint16_t* B, const float* C, float* D, int chain) {
  const int t = blockIdx.x, l = threadIdx.x, i = l & 31, h = l >> 5;
  bf16x8 a, b;
  for (int q = 0; q < 8; ++q) {
    uint16_t av = A[(size_t)t * 512 + i * 16 + 8 * h + q], bv = B[(size_t)t * 512 + (8 * h + q) * 32 + i];
    a[q] = __builtin_bit_cast(__bf16, av);
    b[q] = __builtin_bit_cast(__bf16, bv);
  }
  f32x16 c;
  for (int r = 0; r < 16; ++r) c[r] = C[(size_t)t * 1024 + ((r & 3) + 8 * (r >> 2) + 4 * h) * 32 + i];
  for (int k = 0; k < chain; ++k) c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  for (int r = 0; r < 16; ++r) D[(size_t)t * 1024 + ((r & 3) + 8 * (r >> 2) + 4 * h) * 32 + i] = c[r];
}

// f32: A [T][32][2], B [T][2][32]
__global__ __launch_bounds__(64) void k_f32(const float* A, const float* B, const float* C, float* D) {
  const int t = blockIdx.x, l = threadIdx.x, i = l & 31, h = l >> 5;
  const float a = A[(size_t)t * 64 + i * 2 + h], b = B[(size_t)t * 64 + h * 32 + i];
  f32x16 c;
  for (int r = 0; r < 16; ++r) c[r] = C[(size_t)t * 1024 + ((r & 3) + 8 * (r >> 2) + 4 * h) * 32 + i];
  c = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
  for (int r = 0; r < 16; ++r) D[(size_t)t * 1024 + ((r & 3) + 8 * (r >> 2) + 4 * h) * 32 + i] = c[r];
}

static float bf(uint16_t u) {
  uint32_t v = (uint32_t)u << 16;
  float f;
  std::memcpy(&f, &v, 4);
  return f;
}
static double ulp(float f) { return std::ldexp(1.0, std::ilogb(f) - 23); }

struct Stat {
  long n = 0, rne = 0;
  double sum = 0, sum2 = 0;
  void add(float got, double exact) {
    const float r = (float)exact;   // host RNE
    ++n;
    rne += got == r;
    const double e = ((double)got - exact) / ulp(r == 0.f ? 1e-30f : r);
    sum += e;
    sum2 += e * e;
  }
  void print(const char* name) const {
    printf("%-34s n=%ld  equal to RNE %.4f  mean err %+.4f ulp  rms %.4f ulp\n", name, n, (double)rne / n,
           sum / n, std::sqrt(sum2 / n));
  }
};

int main() {
  const int T = 2048;
  std::mt19937 g(7);
  std::uniform_real_distribution<float> U(0.5f, 2.f);
  std::bernoulli_distribution S(0.5);
  auto rnd = [&](bool pos) { const float v = U(g); return (pos || S(g)) ? v : -v; };
  auto to_bf = [](float f) { uint32_t v; std::memcpy(&v, &f, 4); return (uint16_t)(v >> 16); };
  for (int pos = 0; pos < 2; ++pos) {
    std::vector<uint16_t> A((size_t)T * 512), B((size_t)T * 512);
    std::vector<float> C((size_t)T * 1024), D((size_t)T * 1024);
    for (auto& v : A) v = to_bf(rnd(pos));
    for (auto& v : B) v = to_bf(rnd(pos));
    for (auto& v : C) v = rnd(pos) * 8.f;
    uint16_t *dA, *dB;
    float *dC, *dD;
    hipMalloc(&dA, A.size() * 2);
    hipMalloc(&dB, B.size() * 2);
    hipMalloc(&dC, C.size() * 4);
    hipMalloc(&dD, D.size() * 4);
    hipMemcpy(dA, A.data(), A.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(dB, B.data(), B.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(dC, C.data(), C.size() * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_bf16, dim3(T), dim3(64), 0, 0, dA, dB, dC, dD, 1);
    hipMemcpy(D.data(), dD, D.size() * 4, hipMemcpyDeviceToHost);
    Stat s, sf;
    for (int t = 0; t < T; ++t)
      for (int i = 0; i < 32; ++i)
        for (int j = 0; j < 32; ++j) {
          double ex = C[(size_t)t * 1024 + i * 32 + j];
          float fc = C[(size_t)t * 1024 + i * 32 + j];   // sequential fp32 fma chain (reference rounding)
          for (int k = 0; k < 16; ++k) {
            const double p = (double)bf(A[(size_t)t * 512 + i * 16 + k]) * bf(B[(size_t)t * 512 + k * 32 + j]);
            ex += p;
            fc = std::fma(bf(A[(size_t)t * 512 + i * 16 + k]), bf(B[(size_t)t * 512 + k * 32 + j]), fc);
          }
          s.add(D[(size_t)t * 1024 + i * 32 + j], ex);
          sf.add(fc, ex);
        }
    printf("operands %s:\n", pos ? "all positive" : "random signs");
    s.print("  v_mfma_f32_32x32x16_bf16");
    sf.print("  16 sequential fp32 fma (reference)");
    // f32 MFMA (2-deep K)
    std::vector<float> Af((size_t)T * 64), Bf((size_t)T * 64);
    for (auto& v : Af) v = rnd(pos);
    for (auto& v : Bf) v = rnd(pos);
    float *dAf, *dBf;
    hipMalloc(&dAf, Af.size() * 4);
    hipMalloc(&dBf, Bf.size() * 4);
    hipMemcpy(dAf, Af.data(), Af.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(dBf, Bf.data(), Bf.size() * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_f32, dim3(T), dim3(64), 0, 0, dAf, dBf, dC, dD);
    hipMemcpy(D.data(), dD, D.size() * 4, hipMemcpyDeviceToHost);
    Stat s2, sf2;
    for (int t = 0; t < T; ++t)
      for (int i = 0; i < 32; ++i)
        for (int j = 0; j < 32; ++j) {
          double ex = C[(size_t)t * 1024 + i * 32 + j];
          float fc = C[(size_t)t * 1024 + i * 32 + j];
          for (int k = 0; k < 2; ++k) {
            ex += (double)Af[(size_t)t * 64 + i * 2 + k] * Bf[(size_t)t * 64 + k * 32 + j];
            fc = std::fma(Af[(size_t)t * 64 + i * 2 + k], Bf[(size_t)t * 64 + k * 32 + j], fc);
          }
          s2.add(D[(size_t)t * 1024 + i * 32 + j], ex);
          sf2.add(fc, ex);
        }
    s2.print("  v_mfma_f32_32x32x2_f32");
    sf2.print("  2 sequential fp32 fma (reference)");
    hipFree(dA); hipFree(dB); hipFree(dC); hipFree(dD); hipFree(dAf); hipFree(dBf);
  }
  return 0;
}
