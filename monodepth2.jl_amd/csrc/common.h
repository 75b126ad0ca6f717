// Shared helpers for libmd2hip (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <string>

#include "../../include/md2.h"

namespace md2 {

// ---------------------------------------------------------------------------------------------
// error state (md2_last_error)
// ---------------------------------------------------------------------------------------------
void set_error(const std::string& msg);
const char* last_error();


#define MD2_CHECK_ARG(cond, msg)                                  \
  do {                                                            \
    if (!(cond)) {                                                \
      ::md2::set_error(std::string("invalid argument: ") + (msg)); \
      return MD2_EINVAL;                                   \
    }                                                             \
  } while (0)

#define MD2_HIP(expr)                                                                   \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    if (_e != hipSuccess) {                                                             \
      ::md2::set_error(std::string("HIP error ") + hipGetErrorString(_e) + " at " +     \
                       __FILE__ + ":" + std::to_string(__LINE__) + " (" #expr ")");     \
      return MD2_EHIP;                                                           \
    }                                                                                   \
  } while (0)

#define MD2_LAUNCH_CHECK() MD2_HIP(hipGetLastError())

#define MD2_TRY(expr)                    \
  do {                                   \
    int _rc = (expr);                    \
    if (_rc != 0) return _rc;            \
  } while (0)

inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }

// ---------------------------------------------------------------------------------------------
// device helpers
// ---------------------------------------------------------------------------------------------

// Unsigned division by a runtime constant via a precomputed magic number (Granlund-Montgomery,
// round-up variant).  Exact for 0 <= n < 2^31 and 1 <= d < 2^31.
struct FastDiv {
  uint32_t d;
  uint32_t mul;
  uint32_t shift;
};

inline FastDiv make_fastdiv(uint32_t d) {
  FastDiv f;
  f.d = d;
  if (d == 1) {
    f.mul = 0;
    f.shift = 0;
    return f;
  }
  uint32_t l = 0;
  while ((1ull << l) < d) ++l;
  uint64_t m = ((1ull << 32) * ((1ull << l) - d)) / d + 1;
  f.mul = (uint32_t)m;
  f.shift = l;
  return f;
}

__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
  if (f.d == 1) return n;
  uint32_t t = __umulhi(n, f.mul);
  return (t + ((n - t) >> 1)) >> (f.shift - 1);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Deterministic block sum of NV values per thread (blockDim.x == 256).  Result valid in
// threadIdx.x == 0 only.  `red` must hold 4*NV floats of LDS.
template <int NV>
__device__ __forceinline__ void block_sum256(float (&v)[NV], float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < NV; ++i) v[i] = wave_sum(v[i]);
  if (lane == 0) {
#pragma unroll
    for (int i = 0; i < NV; ++i) red[wid * NV + i] = v[i];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int i = 0; i < NV; ++i) v[i] = red[i] + red[NV + i] + red[2 * NV + i] + red[3 * NV + i];
  }
  __syncthreads();
}

}  // namespace md2
