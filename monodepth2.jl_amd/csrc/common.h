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

// Kernel / planner tuning knobs (tools/*_sweep.sh, tools/ab_*.sh): MD2_<name>=<int> is honoured
// ONLY when MD2_TUNING=1 is also set; otherwise every knob is its measured default and the
// library's kernels and plans do not depend on the environment.  (The fusion switches
// MD2_FUSE_* are separate: each is tested for bit-identity, tests/test_gpu_fusion.py.)
int tuning_knob(const char* name, int dflt);

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
// ---- raw buffer loads: scalar resource + 32-bit per-lane byte offset (+ wave-uniform soffset)
constexpr uint32_t OOB = 0x7ffffff0u;   // byte offset that is out of range for every tensor

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ float bload(__amdgpu_buffer_rsrc_t r, uint32_t off_bytes) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, (int)off_bytes, 0, 0));
}
// voffset (per lane; OOB for padding) + soffset (wave-uniform channel step); OOB + soffset stays
// below 2^32 and beyond every extent, whether or not the range check includes soffset
__device__ __forceinline__ float bload_s(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, (int)voff, (int)soff, 0));
}
// two consecutive floats at a 4-byte-aligned offset (the two taps of a bilinear row pair)
__device__ __forceinline__ float2 bload2_s(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
  const auto v = __builtin_amdgcn_raw_buffer_load_b64(r, (int)voff, (int)soff, 0);
  return make_float2(__uint_as_float(v[0]), __uint_as_float(v[1]));
}
__device__ __forceinline__ float4 bload4(__amdgpu_buffer_rsrc_t r, uint32_t off_bytes) {
  const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off_bytes, 0, 0);
  return make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]),
                     __uint_as_float(v[3]));
}

// Wave sum by DPP (no LDS traffic): quad permutes and row shifts form the 16-lane row sums,
// row_bcast:15 / row_bcast:31 fold the four rows into lane 63, which is broadcast.
__device__ __forceinline__ float dpp_add(float v, int ctrl_sel) {
  int r;
  const int x = __builtin_bit_cast(int, v);
  switch (ctrl_sel) {
    case 0: r = __builtin_amdgcn_update_dpp(0, x, 0xb1, 0xf, 0xf, true); break;    // quad 1,0,3,2
    case 1: r = __builtin_amdgcn_update_dpp(0, x, 0x4e, 0xf, 0xf, true); break;    // quad 2,3,0,1
    case 2: r = __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, true); break;   // row_shr:4
    case 3: r = __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, true); break;   // row_shr:8
    case 4: r = __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false); break;  // row_bcast:15
    default: r = __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false); break; // row_bcast:31
  }
  return v + __builtin_bit_cast(float, r);
}
__device__ __forceinline__ float wave_sum_dpp(float v) {
#pragma unroll
  for (int k = 0; k < 6; ++k) v = dpp_add(v, k);
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 63));
}

// threadIdx.x == 0 only.  `red` must hold 4*NV floats of LDS.
template <int NV>
__device__ __forceinline__ void block_sum256(float (&v)[NV], float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < NV; ++i) v[i] = wave_sum_dpp(v[i]);
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

// the same in fp64 (shuffle tree; `red` holds 4*NV doubles): the cancelling global sums of the
// loss tail (disparity means, the smoothness normalisation constant)
template <int NV>
__device__ __forceinline__ void block_sum256_d(double (&v)[NV], double* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < NV; ++i) v[i] = wave_sum_d(v[i]);
  if (lane == 0) {
#pragma unroll
    for (int i = 0; i < NV; ++i) red[wid * NV + i] = v[i];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int i = 0; i < NV; ++i) v[i] = (red[i] + red[NV + i]) + (red[2 * NV + i] + red[3 * NV + i]);
  }
  __syncthreads();
}

}  // namespace md2
