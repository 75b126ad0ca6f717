// Non-GEMM layers of the train step (see nn.h).  All are HBM-bound streaming kernels; channel
// reductions are deterministic two-stage (per-block fp64 partials, then a per-channel finalise).
#include "nn.h"

namespace md2 {

// ---------------------------------------------------------------------------------------------
// BatchNorm (Flux BatchNorm in trainmode!: batch statistics, biased variance, eps = 1e-5)
// ---------------------------------------------------------------------------------------------
int bn_parts(int C, long N, long HW) {
  long total = N * HW;
  int parts = (int)std::max(1L, std::min(1024L / std::max(1, C) + 1, total / 2048 + 1));
  return (int)std::min<long>(std::min(parts, 256), std::max(1L, N));   // parts split images
}

// Element index helpers: every activation here is < 2^31 elements (checked on the host), so
// indices are 32-bit and divisions by runtime extents use magic numbers (FastDiv).
static FastDiv fd(long d) { return make_fastdiv((uint32_t)d); }
static int check_u31(long n) {
  MD2_CHECK_ARG(n >= 0 && n < (1L << 31), "tensor larger than 2^31 elements");
  return MD2_OK;
}

// units in flight per thread and trip in the BN reduction passes (all loads issued before the
// first is summed; the sums take the units in the one-unit-per-trip order: bit-identical)
constexpr int BN_INFLIGHT = 4;

// One block per (channel c, image group p): the group's images x HW elements of channel c,
// walked as a flat range (float4 units when HW % 4 == 0); fp64 accumulation.
// SLAB: y is not read but formed here from the split-K slabs of the conv that produced it
// (sum in split order = the conv's own reduction, bit-identical) and written to yout -- the
// conv's separate reduction launch and one read of y disappear
template <bool VEC, bool SLAB = false>
__global__ __launch_bounds__(256) void bn_stats_partial_kernel(const float* __restrict__ y, int C,
                                                               int HW, int N, int parts,
                                                               FastDiv fdu, double* __restrict__ part,
                                                               SlabIn sl = SlabIn{},
                                                               float* __restrict__ yout = nullptr) {
  __shared__ double red[8];
  const int c = blockIdx.x, p = blockIdx.y;
  const int i0 = (int)((long)N * p / parts), i1 = (int)((long)N * (p + 1) / parts);
  const int U = VEC ? HW / 4 : HW;                 // units per image
  const uint32_t nu = (uint32_t)(i1 - i0) * U;
  const long sstride = (long)C * N * HW;           // one slab [C][N*HW]
  double s = 0.0, ss = 0.0;
  // BN_INFLIGHT units per thread and trip (all loads in flight first), summed in the one-unit order
  for (uint32_t e0 = threadIdx.x; e0 < nu; e0 += 256u * BN_INFLIGHT) {
    float4 vv[BN_INFLIGHT];
    bool live[BN_INFLIGHT];
#pragma unroll
    for (int h = 0; h < BN_INFLIGHT; ++h) {
      const uint32_t e = e0 + 256u * h;
      live[h] = e < nu;
      vv[h] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (!live[h]) continue;
      const uint32_t im = fdiv(e, fdu), k = e - im * U;
      const long base = ((long)(i0 + im) * C + c) * HW;
      if (SLAB) {
        const long si = (long)c * N * HW + (long)(i0 + im) * HW + (VEC ? 4 * k : k);
        if (VEC) {
#pragma unroll 4
          for (int q = 0; q < sl.splits; ++q) {
            const float4 t = *reinterpret_cast<const float4*>(sl.slab + q * sstride + si);
            vv[h].x += t.x; vv[h].y += t.y; vv[h].z += t.z; vv[h].w += t.w;
          }
          *reinterpret_cast<float4*>(yout + base + 4 * k) = vv[h];
        } else {
          for (int q = 0; q < sl.splits; ++q) vv[h].x += sl.slab[q * sstride + si];
          yout[base + k] = vv[h].x;
        }
      } else if (VEC) {
        vv[h] = *reinterpret_cast<const float4*>(y + base + 4 * k);
      } else {
        vv[h].x = y[base + k];
      }
    }
#pragma unroll
    for (int h = 0; h < BN_INFLIGHT; ++h) {
      if (!live[h]) continue;
      const float4 v = vv[h];
      if (VEC) {
        s += (double)v.x + (double)v.y + (double)v.z + (double)v.w;
        ss += (double)v.x * v.x + (double)v.y * v.y + (double)v.z * v.z + (double)v.w * v.w;
      } else {
        const double d = v.x;
        s += d;
        ss += d * d;
      }
    }
  }
  s = wave_sum_d(s);
  ss = wave_sum_d(ss);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) {
    red[wid] = s;
    red[4 + wid] = ss;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    part[((long)c * parts + p) * 2 + 0] = red[0] + red[1] + red[2] + red[3];
    part[((long)c * parts + p) * 2 + 1] = red[4] + red[5] + red[6] + red[7];
  }
}

__global__ void bn_stats_final_kernel(const double* __restrict__ part, int C, int parts,
                                      long total, float eps, float momentum, float* mean,
                                      float* invstd, float* run_mean, float* run_var) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double s = 0.0, ss = 0.0;
  for (int p = 0; p < parts; ++p) {
    s += part[((long)c * parts + p) * 2];
    ss += part[((long)c * parts + p) * 2 + 1];
  }
  const double mu = s / (double)total;
  const double var = fmax(ss / (double)total - mu * mu, 0.0);
  mean[c] = (float)mu;
  invstd[c] = (float)(1.0 / sqrt(var + (double)eps));
  if (run_mean) {
    run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * (float)mu;
    run_var[c] = (1.f - momentum) * run_var[c] +
                 momentum * (float)(var * (double)total / (double)std::max(total - 1, 1L));
  }
}

__global__ __launch_bounds__(64) void bn_partials_collapse_kernel(const double* __restrict__ part, int parts,
                                                                  double* __restrict__ out) {
  const int c = blockIdx.x;
  double a = 0.0, aa = 0.0;
  const double* q = part + (long)c * parts * 2;
  for (int p = threadIdx.x; p < parts; p += 64) {
    a += q[2 * p];
    aa += q[2 * p + 1];
  }
  a = wave_sum_d(a);
  aa = wave_sum_d(aa);
  if (threadIdx.x == 0) {
    out[2 * c] = a;
    out[2 * c + 1] = aa;
  }
}

int bn_partials_collapse(const double* part, int C, int parts, double* out, hipStream_t st) {
  MD2_CHECK_ARG(part && out && C >= 1 && parts >= 1, "bn_partials_collapse: arguments");
  hipLaunchKernelGGL(bn_partials_collapse_kernel, dim3(C), dim3(64), 0, st, part, parts, out);
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

int bn_stats_partial(const float* y, int N, int C, long HW, BNStatsWs ws, hipStream_t st) {
  MD2_TRY(check_u31((long)N * C * HW));
  MD2_CHECK_ARG(ws.parts >= 1 && ws.parts <= N, "bn_stats: parts must split the images");
  const int vec = HW % 4 == 0;
  const FastDiv fdu = fd(vec ? HW / 4 : HW);
  if (vec)
    hipLaunchKernelGGL(bn_stats_partial_kernel<true>, dim3(C, ws.parts), dim3(256), 0, st, y, C,
                       (int)HW, N, ws.parts, fdu, ws.partials);
  else
    hipLaunchKernelGGL(bn_stats_partial_kernel<false>, dim3(C, ws.parts), dim3(256), 0, st, y, C,
                       (int)HW, N, ws.parts, fdu, ws.partials);
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

int bn_stats_partial_slabs(SlabIn sl, float* y, int N, int C, long HW, BNStatsWs ws, hipStream_t st) {
  MD2_TRY(check_u31((long)N * C * HW));
  MD2_CHECK_ARG(ws.parts >= 1 && ws.parts <= N, "bn_stats: parts must split the images");
  MD2_CHECK_ARG(sl.slab && sl.splits >= 1 && y, "bn_stats_partial_slabs: slabs / output");
  const int vec = HW % 4 == 0;
  const FastDiv fdu = fd(vec ? HW / 4 : HW);
  if (vec)
    hipLaunchKernelGGL((bn_stats_partial_kernel<true, true>), dim3(C, ws.parts), dim3(256), 0, st,
                       (const float*)nullptr, C, (int)HW, N, ws.parts, fdu, ws.partials, sl, y);
  else
    hipLaunchKernelGGL((bn_stats_partial_kernel<false, true>), dim3(C, ws.parts), dim3(256), 0, st,
                       (const float*)nullptr, C, (int)HW, N, ws.parts, fdu, ws.partials, sl, y);
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

int bn_stats(const float* y, int N, int C, long HW, float eps, float momentum, float* mean,
             float* invstd, float* run_mean, float* run_var, BNStatsWs ws, hipStream_t st) {
  MD2_TRY(check_u31((long)N * C * HW));
  MD2_CHECK_ARG(ws.parts >= 1 && ws.parts <= N, "bn_stats: parts must split the images");
  const long total = (long)N * HW;
  const int vec = HW % 4 == 0;
  const FastDiv fdu = fd(vec ? HW / 4 : HW);
  if (vec)
    hipLaunchKernelGGL(bn_stats_partial_kernel<true>, dim3(C, ws.parts), dim3(256), 0, st, y, C,
                       (int)HW, N, ws.parts, fdu, ws.partials);
  else
    hipLaunchKernelGGL(bn_stats_partial_kernel<false>, dim3(C, ws.parts), dim3(256), 0, st, y, C,
                       (int)HW, N, ws.parts, fdu, ws.partials);
  MD2_LAUNCH_CHECK();
  hipLaunchKernelGGL(bn_stats_final_kernel, dim3(cdiv(C, 64)), dim3(64), 0, st, ws.partials, C,
                     ws.parts, total, eps, momentum, mean, invstd, run_mean, run_var);
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

// channel of element unit u (float4 or scalar units): plane = u / U, c = plane % C
__device__ __forceinline__ int unit_channel(uint32_t u, const FastDiv& fdU, const FastDiv& fdC) {
  const uint32_t plane = fdiv(u, fdU);
  return (int)(plane - fdiv(plane, fdC) * fdC.d);
}

template <bool VEC>
__global__ __launch_bounds__(256) void bn_apply_kernel(BNApply p, float* __restrict__ out,
                                                       uint32_t nu, FastDiv fdU, FastDiv fdC) {
  const uint32_t u = blockIdx.x * 256 + threadIdx.x;
  if (u >= nu) return;
  const int c = unit_channel(u, fdU, fdC);
  const float sc = p.gamma[c] * p.invstd[c], sh = p.beta[c] - p.mean[c] * sc;
  float sc2 = 0.f, sh2 = 0.f;
  if (p.y2) {
    sc2 = p.gamma2[c] * p.invstd2[c];
    sh2 = p.beta2[c] - p.mean2[c] * sc2;
  }
  if (VEC) {
    const long i = 4L * u;
    float4 v = *reinterpret_cast<const float4*>(p.y + i);
    float r[4] = {v.x * sc + sh, v.y * sc + sh, v.z * sc + sh, v.w * sc + sh};
    if (p.y2) {
      const float4 q = *reinterpret_cast<const float4*>(p.y2 + i);
      r[0] += q.x * sc2 + sh2; r[1] += q.y * sc2 + sh2; r[2] += q.z * sc2 + sh2; r[3] += q.w * sc2 + sh2;
    }
    if (p.res) {
      const float4 q = *reinterpret_cast<const float4*>(p.res + i);
      r[0] += q.x; r[1] += q.y; r[2] += q.z; r[3] += q.w;
    }
    if (p.relu) {
#pragma unroll
      for (int k = 0; k < 4; ++k) r[k] = fmaxf(r[k], 0.f);
    }
    *reinterpret_cast<float4*>(out + i) = make_float4(r[0], r[1], r[2], r[3]);
  } else {
    float r = p.y[u] * sc + sh;
    if (p.y2) r += p.y2[u] * sc2 + sh2;
    if (p.res) r += p.res[u];
    if (p.relu) r = fmaxf(r, 0.f);
    out[u] = r;
  }
}

int bn_apply(const BNApply& p, float* out, int N, int C, long HW, hipStream_t st) {
  const long n = (long)N * C * HW;
  MD2_TRY(check_u31(n));
  if (HW % 4 == 0) {
    hipLaunchKernelGGL(bn_apply_kernel<true>, dim3(cdiv(n / 4, 256)), dim3(256), 0, st, p, out,
                       (uint32_t)(n / 4), fd(HW / 4), fd(C));
  } else {
    hipLaunchKernelGGL(bn_apply_kernel<false>, dim3(cdiv(n, 256)), dim3(256), 0, st, p, out,
                       (uint32_t)n, fd(HW), fd(C));
  }
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}


// ---- fused finalise + apply.  A block covers 256 consecutive units (float4 or scalar), i.e. the
// planes pl0..pl1 (plane = image*C + channel, <= 256 of them); wave w finalises the channels of
// planes pl0+w, pl0+w+4, ... from the partials (lane-parallel fixed-order sum + wave reduction,
// same result in every block), the scale/shift go through LDS.  The block holding the first unit of image 0's plane of channel c writes mean[c],
// invstd[c] and the running statistics.
// called by a whole wave: lane l sums partials l, l+64, ... (fixed order), then a wave reduction
// -- one partial-load latency per plane instead of `parts` dependent ones
__device__ __forceinline__ void bn_finalise_plane(const BNStatsIn& s, int c, double total,
                                                  bool owner, float& sc, float& sh) {
  double a = 0.0, aa = 0.0;
  const double* q = s.part + (long)c * s.parts * 2;
  for (int p = threadIdx.x & 63; p < s.parts; p += 64) {
    a += q[2 * p];
    aa += q[2 * p + 1];
  }
  a = wave_sum_d(a);
  aa = wave_sum_d(aa);
  const double mu = a / total;
  const double var = fmax(aa / total - mu * mu, 0.0);
  const float meanf = (float)mu;
  const float isf = (float)(1.0 / sqrt(var + (double)s.eps));
  // explicit roundings: bn_bwd_* re-derive relu(y*sc + sh) > 0 from y with the same operations
  sc = __fmul_rn(s.gamma[c], isf);
  sh = __fmaf_rn(-meanf, sc, s.beta[c]);
  if (owner && (threadIdx.x & 63) == 0) {
    s.mean[c] = meanf;
    s.invstd[c] = isf;
    if (s.run_mean) {
      const float m = s.momentum;
      s.run_mean[c] = (1.f - m) * s.run_mean[c] + m * meanf;
      s.run_var[c] = (1.f - m) * s.run_var[c] + m * (float)(var * total / fmax(total - 1.0, 1.0));
    }
  }
}

// Units per thread of the fused apply passes: a block covers 256 * UPT consecutive units, so the
// per-block finalise (one wave per plane) is paid once per 256 * UPT units and a thread has UPT
// independent loads in flight.  UPT only regroups the same per-element arithmetic (bit-identical
// for every UPT).  The host picks the largest UPT that keeps >= BN_MIN_BLOCKS blocks and the
// block's plane count within the 256-entry LDS tables.
constexpr int BN_MIN_BLOCKS = 1024;
static int bn_upt(long units, long U) {
  int upt = 8;
  while (upt > 1 && (units / (256L * upt) < BN_MIN_BLOCKS || 256L * upt / U + 2 > 256)) upt /= 2;
  return upt;
}

template <bool VEC, int UPT = 1>
__global__ __launch_bounds__(256) void bn_apply_fused_kernel(BNApplyFused p, float* __restrict__ out,
                                                             uint32_t nu, FastDiv fdU, FastDiv fdC,
                                                             double total) {
  __shared__ float s_sc[256], s_sh[256], s_sc2[256], s_sh2[256];
  const uint32_t u0 = blockIdx.x * (256u * UPT);
  const uint32_t pl0 = fdiv(u0, fdU);
  const uint32_t npl = fdiv(min(u0 + 256u * UPT - 1u, nu - 1u), fdU) - pl0 + 1u;
  // the block's loads are issued before the per-plane finalise (independent of it): its partial
  // sums -- up to one per 256-pixel tile when the conv epilogue took the statistics -- are read
  // while the tensor's bytes are in flight
  float4 v[UPT], q2[UPT], qr[UPT];
  if (VEC) {
#pragma unroll
    for (int j = 0; j < UPT; ++j) {
      const uint32_t u = u0 + threadIdx.x + 256u * j;
      const long i = 4L * (u < nu ? u : 0u);
      v[j] = *reinterpret_cast<const float4*>(p.y + i);
      if (p.y2) q2[j] = *reinterpret_cast<const float4*>(p.y2 + i);
      if (p.res) qr[j] = *reinterpret_cast<const float4*>(p.res + i);
    }
  }
  for (uint32_t t = threadIdx.x >> 6; t < npl; t += 4) {   // wave-uniform plane loop
    const uint32_t pl = pl0 + t;
    const int c = (int)(pl - fdiv(pl, fdC) * fdC.d);
    const bool owner = pl < fdC.d && pl * fdU.d >= u0;
    float sc, sh;
    bn_finalise_plane(p.s1, c, total, owner, sc, sh);
    float sc2 = 0.f, sh2 = 0.f;
    if (p.y2) bn_finalise_plane(p.s2, c, total, owner, sc2, sh2);
    if ((threadIdx.x & 63) == 0) {
      s_sc[t] = sc;
      s_sh[t] = sh;
      s_sc2[t] = sc2;
      s_sh2[t] = sh2;
    }
  }
  __syncthreads();
  if (VEC) {
#pragma unroll
    for (int j = 0; j < UPT; ++j) {
      const uint32_t u = u0 + threadIdx.x + 256u * j;
      if (u >= nu) break;
      const uint32_t li = fdiv(u, fdU) - pl0;
      const float sc = s_sc[li], sh = s_sh[li];
      float r[4] = {__fmaf_rn(v[j].x, sc, sh), __fmaf_rn(v[j].y, sc, sh), __fmaf_rn(v[j].z, sc, sh),
                    __fmaf_rn(v[j].w, sc, sh)};
      if (p.y2) {
        const float sc2 = s_sc2[li], sh2 = s_sh2[li];
        const float4 q = q2[j];
        r[0] += q.x * sc2 + sh2; r[1] += q.y * sc2 + sh2; r[2] += q.z * sc2 + sh2; r[3] += q.w * sc2 + sh2;
      }
      if (p.res) {
        const float4 q = qr[j];
        r[0] += q.x; r[1] += q.y; r[2] += q.z; r[3] += q.w;
      }
      if (p.relu) {
#pragma unroll
        for (int k = 0; k < 4; ++k) r[k] = fmaxf(r[k], 0.f);
      }
      *reinterpret_cast<float4*>(out + 4L * u) = make_float4(r[0], r[1], r[2], r[3]);
    }
  } else {
#pragma unroll
    for (int j = 0; j < UPT; ++j) {
      const uint32_t u = u0 + threadIdx.x + 256u * j;
      if (u >= nu) break;
      const uint32_t li = fdiv(u, fdU) - pl0;
      const float sc = s_sc[li], sh = s_sh[li];
      float r = __fmaf_rn(p.y[u], sc, sh);
      if (p.y2) r += p.y2[u] * s_sc2[li] + s_sh2[li];
      if (p.res) r += p.res[u];
      if (p.relu) r = fmaxf(r, 0.f);
      out[u] = r;
    }
  }
}

int bn_apply_fused(const BNApplyFused& p, float* out, int N, int C, long HW, hipStream_t st) {
  const long n = (long)N * C * HW;
  MD2_TRY(check_u31(n));
  MD2_CHECK_ARG(p.s1.part && p.s1.parts >= 1 && (!p.y2 || (p.s2.part && p.s2.parts >= 1)),
                "bn_apply_fused: missing statistics partials");
  const double total = (double)((long)N * HW);
  if (HW % 4 == 0) {
    const long nu = n / 4;
    const int upt = bn_upt(nu, HW / 4);
    const dim3 grid(cdiv(nu, 256L * upt));
    if (upt == 8)
      hipLaunchKernelGGL((bn_apply_fused_kernel<true, 8>), grid, dim3(256), 0, st, p, out, (uint32_t)nu,
                         fd(HW / 4), fd(C), total);
    else if (upt == 4)
      hipLaunchKernelGGL((bn_apply_fused_kernel<true, 4>), grid, dim3(256), 0, st, p, out, (uint32_t)nu,
                         fd(HW / 4), fd(C), total);
    else if (upt == 2)
      hipLaunchKernelGGL((bn_apply_fused_kernel<true, 2>), grid, dim3(256), 0, st, p, out, (uint32_t)nu,
                         fd(HW / 4), fd(C), total);
    else
      hipLaunchKernelGGL((bn_apply_fused_kernel<true, 1>), grid, dim3(256), 0, st, p, out, (uint32_t)nu,
                         fd(HW / 4), fd(C), total);
  } else {
    hipLaunchKernelGGL(bn_apply_fused_kernel<false>, dim3(cdiv(n, 256)), dim3(256), 0, st, p, out,
                       (uint32_t)n, fd(HW), fd(C), total);
  }
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

// ReLU mask of a BN+ReLU output without a residual, re-derived from the pre-BN y: the forward's
// relu(fma(y, sc, sh)) with sc = gamma*invstd, sh = beta - mean*sc in the same explicit roundings
// (bn_finalise_plane), so the mask is bit-identical and the activation is not read back
struct YMask {
  float sc, sh;
  bool on;
};
__device__ __forceinline__ YMask ymask(const float* mgamma, const float* mbeta, int c, float mu, float is) {
  YMask m{0.f, 0.f, mbeta != nullptr};
  if (m.on) {
    m.sc = __fmul_rn(mgamma[c], is);
    m.sh = __fmaf_rn(-mu, m.sc, mbeta[c]);
  }
  return m;
}
__device__ __forceinline__ float ymasked(float g, float y, const YMask& m) {
  return (m.on && !(__fmaf_rn(y, m.sc, m.sh) > 0.f)) ? 0.f : g;
}

__device__ __forceinline__ float4 add_skip4(const SkipSrc& q, uint32_t i, float4 g) {
  if (i >= q.skip_lo && i < q.skip_hi) {
    const float4 k = *reinterpret_cast<const float4*>(q.skip + (i - q.skip_lo));
    g.x += k.x; g.y += k.y; g.z += k.z; g.w += k.w;
  }
  return g;
}

// SLAB: dout formed from the dgrad conv's split-K slabs and written (see bn_stats_partial_kernel)
// SKIP: dout + pd.skip over flat elements [pd.skip_lo, pd.skip_hi) (the decoder skip gradient,
// added where axpy used to add it before this pass; same fp add, bit-identical)
template <bool VEC, bool SLAB = false, bool SKIP = false>
__global__ __launch_bounds__(256) void bn_bwd_partial_kernel(
    const float* __restrict__ dout, const float* __restrict__ mask, const float* __restrict__ y,
    const float* __restrict__ mean, const float* __restrict__ invstd, const float* __restrict__ mgamma,
    const float* __restrict__ mbeta, int C, int HW, int N, int parts, FastDiv fdu,
    double* __restrict__ part, SlabIn sl = SlabIn{}, float* __restrict__ dout_w = nullptr,
    SkipSrc pd = SkipSrc{}) {
  static_assert(!SKIP || (VEC && !SLAB), "SKIP: float4 units of a read dout");
  __shared__ double red[8];
  const int c = blockIdx.x, p = blockIdx.y;
  const int i0 = (int)((long)N * p / parts), i1 = (int)((long)N * (p + 1) / parts);
  const int U = VEC ? HW / 4 : HW;
  const uint32_t nu = (uint32_t)(i1 - i0) * U;
  const float mu = mean[c], is = invstd[c];
  const YMask ym = ymask(mgamma, mbeta, c, mu, is);
  const long sstride = (long)C * N * HW;
  double sg = 0.0, sgx = 0.0;
  // BN_INFLIGHT units per thread and trip (all loads in flight before any is used); the sums take
  // them in the same order as one unit per trip
  for (uint32_t e0 = threadIdx.x; e0 < nu; e0 += 256u * BN_INFLIGHT) {
    float4 gv[BN_INFLIGHT], yv[BN_INFLIGHT];
    bool live[BN_INFLIGHT];
#pragma unroll
    for (int h = 0; h < BN_INFLIGHT; ++h) {
      const uint32_t e = e0 + 256u * h;
      live[h] = e < nu;
      gv[h] = yv[h] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (!live[h]) continue;
      const uint32_t im = fdiv(e, fdu), k = e - im * U;
      const long base = ((long)(i0 + im) * C + c) * HW;
      if (SLAB) {
        const long si = (long)c * N * HW + (long)(i0 + im) * HW + (VEC ? 4 * k : k);
        if (VEC) {
#pragma unroll 4
          for (int q = 0; q < sl.splits; ++q) {
            const float4 t = *reinterpret_cast<const float4*>(sl.slab + q * sstride + si);
            gv[h].x += t.x; gv[h].y += t.y; gv[h].z += t.z; gv[h].w += t.w;
          }
          *reinterpret_cast<float4*>(dout_w + base + 4 * k) = gv[h];
        } else {
          for (int q = 0; q < sl.splits; ++q) gv[h].x += sl.slab[q * sstride + si];
          dout_w[base + k] = gv[h].x;
        }
      }
      if (VEC) {
        const long i = base + 4 * k;
        if (!SLAB) gv[h] = *reinterpret_cast<const float4*>(dout + i);
        if (SKIP) gv[h] = add_skip4(pd, (uint32_t)i, gv[h]);
        yv[h] = *reinterpret_cast<const float4*>(y + i);
        if (mask) {
          const float4 m = *reinterpret_cast<const float4*>(mask + i);
          if (!(m.x > 0.f)) gv[h].x = 0.f;
          if (!(m.y > 0.f)) gv[h].y = 0.f;
          if (!(m.z > 0.f)) gv[h].z = 0.f;
          if (!(m.w > 0.f)) gv[h].w = 0.f;
        }
      } else {
        const long i = base + k;
        if (!SLAB) gv[h].x = dout[i];
        yv[h].x = y[i];
        if (mask && !(mask[i] > 0.f)) gv[h].x = 0.f;
      }
    }
#pragma unroll
    for (int h = 0; h < BN_INFLIGHT; ++h) {
      if (!live[h]) continue;
      float4 g = gv[h];
      const float4 v = yv[h];
      if (VEC) {
        g.x = ymasked(g.x, v.x, ym);
        g.y = ymasked(g.y, v.y, ym);
        g.z = ymasked(g.z, v.z, ym);
        g.w = ymasked(g.w, v.w, ym);
        sg += (double)g.x + (double)g.y + (double)g.z + (double)g.w;
        sgx += (double)g.x * (double)((v.x - mu) * is) + (double)g.y * (double)((v.y - mu) * is) +
               (double)g.z * (double)((v.z - mu) * is) + (double)g.w * (double)((v.w - mu) * is);
      } else {
        g.x = ymasked(g.x, v.x, ym);
        sg += g.x;
        sgx += (double)g.x * (double)((v.x - mu) * is);
      }
    }
  }
  sg = wave_sum_d(sg);
  sgx = wave_sum_d(sgx);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) {
    red[wid] = sg;
    red[4 + wid] = sgx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    part[((long)c * parts + p) * 2 + 0] = red[0] + red[1] + red[2] + red[3];
    part[((long)c * parts + p) * 2 + 1] = red[4] + red[5] + red[6] + red[7];
  }
}

__global__ void bn_bwd_final_kernel(const double* __restrict__ part, int C, int parts,
                                    float* dgamma, float* dbeta) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double sg = 0.0, sgx = 0.0;
  for (int p = 0; p < parts; ++p) {
    sg += part[((long)c * parts + p) * 2];
    sgx += part[((long)c * parts + p) * 2 + 1];
  }
  dbeta[c] = (float)sg;
  dgamma[c] = (float)sgx;
}

static SkipSrc skip_src(const SkipAdd& sk) {
  SkipSrc pd{};
  pd.skip = sk.skip;
  pd.skip_lo = (uint32_t)sk.lo;
  pd.skip_hi = (uint32_t)sk.hi;
  return pd;
}

int bn_bwd_partial(const float* dout, const float* mask_out, const float* y, const float* mean,
                   const float* invstd, int N, int C, long HW, BNStatsWs ws, hipStream_t st,
                   const float* mgamma, const float* mbeta, SkipAdd sk) {
  MD2_TRY(check_u31((long)N * C * HW));
  MD2_CHECK_ARG(ws.parts >= 1 && ws.parts <= N, "bn_bwd: parts must split the images");
  const int vec = HW % 4 == 0;
  const FastDiv fdu = fd(vec ? HW / 4 : HW);
  MD2_CHECK_ARG(!sk.skip || (vec && sk.lo >= 0 && sk.lo <= sk.hi && sk.hi <= (long)N * C * HW),
                "bn_bwd: skip range / HW % 4");
  if (sk.skip)
    hipLaunchKernelGGL((bn_bwd_partial_kernel<true, false, true>), dim3(C, ws.parts), dim3(256), 0,
                       st, dout, mask_out, y, mean, invstd, mgamma, mbeta, C, (int)HW, N, ws.parts, fdu,
                       ws.partials, SlabIn{}, (float*)nullptr, skip_src(sk));
  else if (vec)
    hipLaunchKernelGGL(bn_bwd_partial_kernel<true>, dim3(C, ws.parts), dim3(256), 0, st, dout,
                       mask_out, y, mean, invstd, mgamma, mbeta, C, (int)HW, N, ws.parts, fdu,
                       ws.partials);
  else
    hipLaunchKernelGGL(bn_bwd_partial_kernel<false>, dim3(C, ws.parts), dim3(256), 0, st, dout,
                       mask_out, y, mean, invstd, mgamma, mbeta, C, (int)HW, N, ws.parts, fdu,
                       ws.partials);
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

int bn_bwd_partial_slabs(SlabIn sl, float* dout, const float* y, const float* mean,
                         const float* invstd, int N, int C, long HW, BNStatsWs ws, hipStream_t st,
                         const float* mgamma, const float* mbeta) {
  MD2_TRY(check_u31((long)N * C * HW));
  MD2_CHECK_ARG(ws.parts >= 1 && ws.parts <= N, "bn_bwd: parts must split the images");
  MD2_CHECK_ARG(sl.slab && sl.splits >= 1 && dout, "bn_bwd_partial_slabs: slabs / output");
  const int vec = HW % 4 == 0;
  const FastDiv fdu = fd(vec ? HW / 4 : HW);
  if (vec)
    hipLaunchKernelGGL((bn_bwd_partial_kernel<true, true>), dim3(C, ws.parts), dim3(256), 0, st,
                       (const float*)nullptr, (const float*)nullptr, y, mean, invstd, mgamma, mbeta, C,
                       (int)HW, N, ws.parts, fdu, ws.partials, sl, dout);
  else
    hipLaunchKernelGGL((bn_bwd_partial_kernel<false, true>), dim3(C, ws.parts), dim3(256), 0, st,
                       (const float*)nullptr, (const float*)nullptr, y, mean, invstd, mgamma, mbeta, C,
                       (int)HW, N, ws.parts, fdu, ws.partials, sl, dout);
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

int bn_bwd_reduce(const float* dout, const float* mask_out, const float* y, const float* mean,
                  const float* invstd, int N, int C, long HW, float* dgamma, float* dbeta,
                  BNStatsWs ws, hipStream_t st) {
  MD2_TRY(check_u31((long)N * C * HW));
  MD2_CHECK_ARG(ws.parts >= 1 && ws.parts <= N, "bn_bwd: parts must split the images");
  const int vec = HW % 4 == 0;
  const FastDiv fdu = fd(vec ? HW / 4 : HW);
  if (vec)
    hipLaunchKernelGGL(bn_bwd_partial_kernel<true>, dim3(C, ws.parts), dim3(256), 0, st, dout,
                       mask_out, y, mean, invstd, (const float*)nullptr, (const float*)nullptr, C, (int)HW, N, ws.parts, fdu,
                       ws.partials);
  else
    hipLaunchKernelGGL(bn_bwd_partial_kernel<false>, dim3(C, ws.parts), dim3(256), 0, st, dout,
                       mask_out, y, mean, invstd, (const float*)nullptr, (const float*)nullptr, C, (int)HW, N, ws.parts, fdu,
                       ws.partials);
  MD2_LAUNCH_CHECK();
  hipLaunchKernelGGL(bn_bwd_final_kernel, dim3(cdiv(C, 64)), dim3(64), 0, st, ws.partials, C,
                     ws.parts, dgamma, dbeta);
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

template <bool VEC>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(
    const float* __restrict__ dout, const float* __restrict__ mask, const float* __restrict__ y,
    const float* __restrict__ mean, const float* __restrict__ invstd,
    const float* __restrict__ gamma, const float* __restrict__ dgamma,
    const float* __restrict__ dbeta, uint32_t nu, FastDiv fdU, FastDiv fdC, float invL,
    float* __restrict__ dy, float* __restrict__ dres, int dres_acc) {
  const uint32_t u = blockIdx.x * 256 + threadIdx.x;
  if (u >= nu) return;
  const int c = unit_channel(u, fdU, fdC);
  const float is = invstd[c], mu = mean[c];
  const float k0 = gamma[c] * is, db = dbeta[c] * invL, dg = dgamma[c] * invL;
  if (VEC) {
    const long i = 4L * u;
    float g[4];
    {
      const float4 t = *reinterpret_cast<const float4*>(dout + i);
      g[0] = t.x; g[1] = t.y; g[2] = t.z; g[3] = t.w;
    }
    if (mask) {
      const float4 m = *reinterpret_cast<const float4*>(mask + i);
      if (!(m.x > 0.f)) g[0] = 0.f;
      if (!(m.y > 0.f)) g[1] = 0.f;
      if (!(m.z > 0.f)) g[2] = 0.f;
      if (!(m.w > 0.f)) g[3] = 0.f;
    }
    const float4 v = *reinterpret_cast<const float4*>(y + i);
    const float yv[4] = {v.x, v.y, v.z, v.w};
    float r[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) r[k] = k0 * (g[k] - db - (yv[k] - mu) * is * dg);
    *reinterpret_cast<float4*>(dy + i) = make_float4(r[0], r[1], r[2], r[3]);
    if (dres) {
      float4 o = make_float4(g[0], g[1], g[2], g[3]);
      if (dres_acc) {
        const float4 q = *reinterpret_cast<const float4*>(dres + i);
        o.x += q.x; o.y += q.y; o.z += q.z; o.w += q.w;
      }
      *reinterpret_cast<float4*>(dres + i) = o;
    }
  } else {
    float g = dout[u];
    if (mask && !(mask[u] > 0.f)) g = 0.f;
    const float xh = (y[u] - mu) * is;
    dy[u] = k0 * (g - db - xh * dg);
    if (dres) {
      if (dres_acc)
        dres[u] += g;
      else
        dres[u] = g;
    }
  }
}

int bn_bwd_apply(const float* dout, const float* mask_out, const float* y, const float* mean,
                 const float* invstd, const float* gamma, const float* dgamma,
                 const float* dbeta, int N, int C, long HW, float* dy, float* dres,
                 int dres_accumulate, hipStream_t st) {
  const long n = (long)N * C * HW;
  MD2_TRY(check_u31(n));
  const float invL = 1.f / (float)((long)N * HW);
  if (HW % 4 == 0)
    hipLaunchKernelGGL(bn_bwd_apply_kernel<true>, dim3(cdiv(n / 4, 256)), dim3(256), 0, st, dout,
                       mask_out, y, mean, invstd, gamma, dgamma, dbeta, (uint32_t)(n / 4), fd(HW / 4),
                       fd(C), invL, dy, dres, dres_accumulate);
  else
    hipLaunchKernelGGL(bn_bwd_apply_kernel<false>, dim3(cdiv(n, 256)), dim3(256), 0, st, dout,
                       mask_out, y, mean, invstd, gamma, dgamma, dbeta, (uint32_t)n, fd(HW), fd(C),
                       invL, dy, dres, dres_accumulate);
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}


// ---- fused finalise + backward apply: per block the channels of its planes sum the backward
// partials in bn_bwd_final_kernel's order (bit-identical dgamma/dbeta), the owner block of each
// channel (first unit of image 0's plane) stores dgamma[c]/dbeta[c].
template <bool VEC, bool SKIP = false, int UPT = 1>
__global__ __launch_bounds__(256) void bn_bwd_apply_fused_kernel(
    const float* __restrict__ dout, const float* __restrict__ mask, const float* __restrict__ y,
    const float* __restrict__ mean, const float* __restrict__ invstd,
    const float* __restrict__ gamma, const double* __restrict__ part, int parts,
    float* __restrict__ dgamma, float* __restrict__ dbeta, uint32_t nu, FastDiv fdU, FastDiv fdC,
    float invL, float* __restrict__ dy, float* __restrict__ dres, int dres_acc,
    const float* __restrict__ mbeta, SkipSrc pd = SkipSrc{}) {
  static_assert(!SKIP || VEC, "SKIP: float4 units of a read dout");
  static_assert(VEC || UPT == 1, "scalar units: one per thread");
  __shared__ float s_k0[256], s_db[256], s_dg[256], s_mu[256], s_is[256], s_msc[256], s_msh[256];
  const uint32_t u0 = blockIdx.x * (256u * UPT);
  const uint32_t pl0 = fdiv(u0, fdU);
  const uint32_t npl = fdiv(min(u0 + 256u * UPT - 1u, nu - 1u), fdU) - pl0 + 1u;
  for (uint32_t t = threadIdx.x >> 6; t < npl; t += 4) {   // one wave per plane (see bn_finalise_plane)
    const uint32_t pl = pl0 + t;
    const int c = (int)(pl - fdiv(pl, fdC) * fdC.d);
    double sg = 0.0, sgx = 0.0;
    const double* q = part + (long)c * parts * 2;
    for (int p = threadIdx.x & 63; p < parts; p += 64) {
      sg += q[2 * p];
      sgx += q[2 * p + 1];
    }
    sg = wave_sum_d(sg);
    sgx = wave_sum_d(sgx);
    if ((threadIdx.x & 63) == 0) {
      const float dbf = (float)sg, dgf = (float)sgx;
      if (pl < fdC.d && pl * fdU.d >= u0) {
        dbeta[c] = dbf;
        dgamma[c] = dgf;
      }
      const float is = invstd[c];
      s_k0[t] = gamma[c] * is;
      s_db[t] = dbf * invL;
      s_dg[t] = dgf * invL;
      s_mu[t] = mean[c];
      s_is[t] = is;
      const YMask ym = ymask(gamma, mbeta, c, mean[c], is);
      s_msc[t] = ym.sc;
      s_msh[t] = ym.sh;
    }
  }
  __syncthreads();
  if (VEC) {
    // every load of the thread's UPT units in flight before the first is used
    float4 t[UPT], mv[UPT], v[UPT], qd[UPT];
#pragma unroll
    for (int j = 0; j < UPT; ++j) {
      const uint32_t u = u0 + threadIdx.x + 256u * j;
      const long i = 4L * (u < nu ? u : 0u);
      t[j] = *reinterpret_cast<const float4*>(dout + i);
      if (SKIP) t[j] = add_skip4(pd, (uint32_t)i, t[j]);
      if (mask) mv[j] = *reinterpret_cast<const float4*>(mask + i);
      v[j] = *reinterpret_cast<const float4*>(y + i);
      if (dres && dres_acc) qd[j] = *reinterpret_cast<const float4*>(dres + i);
    }
#pragma unroll
    for (int j = 0; j < UPT; ++j) {
      const uint32_t u = u0 + threadIdx.x + 256u * j;
      if (u >= nu) break;
      const long i = 4L * u;
      const uint32_t li = fdiv(u, fdU) - pl0;
      const float k0 = s_k0[li], db = s_db[li], dg = s_dg[li], mu = s_mu[li], is = s_is[li];
      const YMask ym{s_msc[li], s_msh[li], mbeta != nullptr};
      float g[4] = {t[j].x, t[j].y, t[j].z, t[j].w};
      if (mask) {
        const float4 m = mv[j];
        if (!(m.x > 0.f)) g[0] = 0.f;
        if (!(m.y > 0.f)) g[1] = 0.f;
        if (!(m.z > 0.f)) g[2] = 0.f;
        if (!(m.w > 0.f)) g[3] = 0.f;
      }
      const float yv[4] = {v[j].x, v[j].y, v[j].z, v[j].w};
#pragma unroll
      for (int k = 0; k < 4; ++k) g[k] = ymasked(g[k], yv[k], ym);
      float r[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) r[k] = k0 * (g[k] - db - (yv[k] - mu) * is * dg);
      *reinterpret_cast<float4*>(dy + i) = make_float4(r[0], r[1], r[2], r[3]);
      if (dres) {
        float4 o = make_float4(g[0], g[1], g[2], g[3]);
        if (dres_acc) {
          const float4 q = qd[j];
          o.x += q.x; o.y += q.y; o.z += q.z; o.w += q.w;
        }
        *reinterpret_cast<float4*>(dres + i) = o;
      }
    }
  } else {
    const uint32_t u = u0 + threadIdx.x;
    if (u >= nu) return;
    const uint32_t li = fdiv(u, fdU) - pl0;
    const float k0 = s_k0[li], db = s_db[li], dg = s_dg[li], mu = s_mu[li], is = s_is[li];
    const YMask ym{s_msc[li], s_msh[li], mbeta != nullptr};
    float g = dout[u];
    if (mask && !(mask[u] > 0.f)) g = 0.f;
    g = ymasked(g, y[u], ym);
    const float xh = (y[u] - mu) * is;
    dy[u] = k0 * (g - db - xh * dg);
    if (dres) {
      if (dres_acc)
        dres[u] += g;
      else
        dres[u] = g;
    }
  }
}

int bn_bwd_apply_fused(const float* dout, const float* mask_out, const float* y, const float* mean,
                       const float* invstd, const float* gamma, BNStatsWs ws, float* dgamma,
                       float* dbeta, int N, int C, long HW, float* dy, float* dres,
                       int dres_accumulate, hipStream_t st, const float* mbeta, SkipAdd sk) {
  const long n = (long)N * C * HW;
  MD2_TRY(check_u31(n));
  MD2_CHECK_ARG(ws.partials && ws.parts >= 1, "bn_bwd_apply_fused: missing partials");
  MD2_CHECK_ARG(!sk.skip || (HW % 4 == 0 && sk.lo >= 0 && sk.lo <= sk.hi && sk.hi <= n),
                "bn_bwd: skip range / HW % 4");
  const float invL = 1.f / (float)((long)N * HW);
  if (HW % 4 == 0) {
    const long nu = n / 4;
    const int upt = bn_upt(nu, HW / 4);
    const dim3 grid(cdiv(nu, 256L * upt));
#define MD2_BWDA(SK, U)                                                                              \
  hipLaunchKernelGGL((bn_bwd_apply_fused_kernel<true, SK, U>), grid, dim3(256), 0, st, dout, mask_out, y, \
                     mean, invstd, gamma, ws.partials, ws.parts, dgamma, dbeta, (uint32_t)nu, fd(HW / 4), \
                     fd(C), invL, dy, dres, dres_accumulate, mbeta, skip_src(sk))
    if (sk.skip) {
      if (upt == 8) MD2_BWDA(true, 8);
      else if (upt == 4) MD2_BWDA(true, 4);
      else if (upt == 2) MD2_BWDA(true, 2);
      else MD2_BWDA(true, 1);
    } else {
      if (upt == 8) MD2_BWDA(false, 8);
      else if (upt == 4) MD2_BWDA(false, 4);
      else if (upt == 2) MD2_BWDA(false, 2);
      else MD2_BWDA(false, 1);
    }
#undef MD2_BWDA
  } else
    hipLaunchKernelGGL(bn_bwd_apply_fused_kernel<false>, dim3(cdiv(n, 256)), dim3(256), 0, st,
                       dout, mask_out, y, mean, invstd, gamma, ws.partials, ws.parts, dgamma, dbeta,
                       (uint32_t)n, fd(HW), fd(C), invL, dy, dres, dres_accumulate, mbeta);
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

// ---------------------------------------------------------------------------------------------
// MaxPool 3x3 / stride 2 / pad 1 (ResNet stem); argmax kept as the window index 0..8
// ---------------------------------------------------------------------------------------------
// one output per thread; with an even input width the window columns 2ow, 2ow+1 are one float2
template <bool EVENW>
__global__ __launch_bounds__(256) void maxpool_fwd_kernel(const float* __restrict__ x, int H, int W,
                                                          float* __restrict__ y,
                                                          unsigned char* __restrict__ arg, int Ho,
                                                          FastDiv fdWo, FastDiv fdHo, uint32_t n) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint32_t r = fdiv(i, fdWo), plane = fdiv(r, fdHo);
  const int ow = (int)(i - r * fdWo.d), oh = (int)(r - plane * fdHo.d);
  const float* p = x + plane * (uint32_t)(H * W);
  float best = -INFINITY;
  int bi = 0;
  const int iw = ow * 2;
#pragma unroll
  for (int kh = 0; kh < 3; ++kh) {
    const int ih = oh * 2 - 1 + kh;
    if (ih < 0 || ih >= H) continue;
    const float* row = p + ih * W;
    float v0 = -INFINITY, v1, v2 = -INFINITY;
    if (iw > 0) v0 = row[iw - 1];
    if (EVENW) {
      const float2 t = *reinterpret_cast<const float2*>(row + iw);
      v1 = t.x;
      v2 = t.y;
    } else {
      v1 = row[iw];
      if (iw + 1 < W) v2 = row[iw + 1];
    }
    // strict '>' in (kh, kw) scan order: the first maximum wins (NNlib maxpool)
    if (v0 > best) { best = v0; bi = kh * 3; }
    if (v1 > best) { best = v1; bi = kh * 3 + 1; }
    if (v2 > best) { best = v2; bi = kh * 3 + 2; }
  }
  y[i] = best;
  arg[i] = (unsigned char)bi;
}

// Gather over 2x2 input blocks: input rows {2i, 2i+1} x columns {2j, 2j+1} are touched only by
// outputs (i..i+1, j..j+1) -- even rows/columns are tap 1 of output i, odd ones tap 2 of output
// i and tap 0 of output i+1 -- so each thread reads 4 (arg, dy) pairs and writes 4 inputs.
// SKIP (even W): dx += skip over flat elements [sk.skip_lo, sk.skip_hi) -- the decoder skip
// gradient on the target images, added here instead of by a separate axpy (same fp add)
template <bool EVENW, bool SKIP = false>
__global__ __launch_bounds__(256) void maxpool_bwd_kernel(const float* __restrict__ dy,
                                                          const unsigned char* __restrict__ arg,
                                                          int H, int W, int Ho, FastDiv fdWo,
                                                          FastDiv fdHo, float* __restrict__ dx,
                                                          uint32_t n, SkipSrc sk = SkipSrc{}) {
  static_assert(!SKIP || EVENW, "SKIP: even width");
  const uint32_t t = blockIdx.x * 256 + threadIdx.x;
  if (t >= n) return;
  const uint32_t r = fdiv(t, fdWo), plane = fdiv(r, fdHo);
  const int Wo = (int)fdWo.d;
  const int j = (int)(t - r * fdWo.d), i = (int)(r - plane * fdHo.d);
  const bool hasr = i + 1 < Ho, hasc = j + 1 < Wo;
  const uint32_t o = t;
  const int a00 = arg[o];
  const float g00 = dy[o];
  int a01 = -1, a10 = -1, a11 = -1;
  float g01 = 0.f, g10 = 0.f, g11 = 0.f;
  if (hasc) { a01 = arg[o + 1]; g01 = dy[o + 1]; }
  if (hasr) { a10 = arg[o + Wo]; g10 = dy[o + Wo]; }
  if (hasr && hasc) { a11 = arg[o + Wo + 1]; g11 = dy[o + Wo + 1]; }
  const float e00 = a00 == 4 ? g00 : 0.f;
  const float e01 = (a00 == 5 ? g00 : 0.f) + (a01 == 3 ? g01 : 0.f);
  const float e10 = (a00 == 7 ? g00 : 0.f) + (a10 == 1 ? g10 : 0.f);
  const float e11 = (a00 == 8 ? g00 : 0.f) + (a01 == 6 ? g01 : 0.f) + (a10 == 2 ? g10 : 0.f) +
                    (a11 == 0 ? g11 : 0.f);
  const uint32_t qi = plane * (uint32_t)(H * W) + (2 * i) * W + 2 * j;
  float* q = dx + qi;
  if (EVENW) {
    float2 r0 = make_float2(e00, e01), r1 = make_float2(e10, e11);
    if (SKIP && qi >= sk.skip_lo && qi < sk.skip_hi) {   // image-uniform: both rows in range
      const float2 k0 = *reinterpret_cast<const float2*>(sk.skip + (qi - sk.skip_lo));
      r0.x += k0.x; r0.y += k0.y;
      if (2 * i + 1 < H) {
        const float2 k1 = *reinterpret_cast<const float2*>(sk.skip + (qi + W - sk.skip_lo));
        r1.x += k1.x; r1.y += k1.y;
      }
    }
    *reinterpret_cast<float2*>(q) = r0;
    if (2 * i + 1 < H) *reinterpret_cast<float2*>(q + W) = r1;
  } else {
    q[0] = e00;
    if (2 * j + 1 < W) q[1] = e01;
    if (2 * i + 1 < H) {
      q[W] = e10;
      if (2 * j + 1 < W) q[W + 1] = e11;
    }
  }
}

// ResNet stem tail in one pass: BN (batch statistics finalised per block, bn_apply_fused's
// explicit roundings) + ReLU + MaxPool 3x3/2/pad 1.  One pooled output per thread: it evaluates
// relu(fma(y, sc, sh)) over its window (bit-identical to bn_apply_fused then maxpool_fwd), stores
// the window's own 2x2 block of the activation (rows 2oh..2oh+1, columns 2ow..2ow+1: every
// activation exactly once, even H and W) and the max / argmax -- the activation is written but
// never read back (the pool used to re-read it: one full read of the stem output less).
__global__ __launch_bounds__(256) void bn_relu_maxpool_kernel(BNApplyFused p, float* __restrict__ act,
                                                              int H, int W, float* __restrict__ y,
                                                              unsigned char* __restrict__ arg,
                                                              FastDiv fdWo, FastDiv fdHo, FastDiv fdU,
                                                              FastDiv fdC, uint32_t n, double total) {
  __shared__ float s_sc[256], s_sh[256];
  const uint32_t u0 = blockIdx.x * 256u;
  const uint32_t pl0 = fdiv(u0, fdU);
  const uint32_t npl = fdiv(min(u0 + 255u, n - 1u), fdU) - pl0 + 1u;
  for (uint32_t t = threadIdx.x >> 6; t < npl; t += 4) {   // wave-uniform plane loop
    const uint32_t pl = pl0 + t;
    const int c = (int)(pl - fdiv(pl, fdC) * fdC.d);
    const bool owner = pl < fdC.d && pl * fdU.d >= u0;
    float sc, sh;
    bn_finalise_plane(p.s1, c, total, owner, sc, sh);
    if ((threadIdx.x & 63) == 0) {
      s_sc[t] = sc;
      s_sh[t] = sh;
    }
  }
  __syncthreads();
  const uint32_t i = u0 + threadIdx.x;
  if (i >= n) return;
  const uint32_t r = fdiv(i, fdWo), plane = fdiv(r, fdHo);
  const int ow = (int)(i - r * fdWo.d), oh = (int)(r - plane * fdHo.d);
  const float sc = s_sc[plane - pl0], sh = s_sh[plane - pl0];
  const uint32_t base = plane * (uint32_t)(H * W);
  const float* src = p.y + base;
  float best = -INFINITY;
  int bi = 0;
  const int iw = ow * 2;
#pragma unroll
  for (int kh = 0; kh < 3; ++kh) {
    const int ih = oh * 2 - 1 + kh;
    if (ih < 0) continue;                       // ih <= 2*oh + 1 < H (even H)
    const float* row = src + ih * W;
    float v0 = -INFINITY;
    if (iw > 0) v0 = fmaxf(__fmaf_rn(row[iw - 1], sc, sh), 0.f);
    const float2 t = *reinterpret_cast<const float2*>(row + iw);
    const float v1 = fmaxf(__fmaf_rn(t.x, sc, sh), 0.f);
    const float v2 = fmaxf(__fmaf_rn(t.y, sc, sh), 0.f);
    if (kh > 0) *reinterpret_cast<float2*>(act + base + ih * W + iw) = make_float2(v1, v2);
    // strict '>' in (kh, kw) scan order: the first maximum wins (NNlib maxpool)
    if (v0 > best) { best = v0; bi = kh * 3; }
    if (v1 > best) { best = v1; bi = kh * 3 + 1; }
    if (v2 > best) { best = v2; bi = kh * 3 + 2; }
  }
  y[i] = best;
  arg[i] = (unsigned char)bi;
}

int bn_relu_maxpool(const BNApplyFused& p, float* act, int N, int C, int H, int W, float* y,
                    unsigned char* arg, int Ho, int Wo, hipStream_t st) {
  MD2_CHECK_ARG(H % 2 == 0 && W % 2 == 0 && Ho == H / 2 && Wo == W / 2,
                "bn_relu_maxpool: even input, 3x3/2 pad-1 output shape");
  MD2_CHECK_ARG(p.y && p.s1.part && p.s1.parts >= 1 && !p.y2 && !p.res && p.relu,
                "bn_relu_maxpool: BN+ReLU without residual / second branch");
  const long n = (long)N * C * Ho * Wo;
  MD2_TRY(check_u31((long)N * C * H * W));
  const double total = (double)((long)N * H * W);
  hipLaunchKernelGGL(bn_relu_maxpool_kernel, dim3(cdiv(n, 256)), dim3(256), 0, st, p, act, H, W, y,
                     arg, fd(Wo), fd(Ho), fd((long)Ho * Wo), fd(C), (uint32_t)n, total);
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

int maxpool_fwd(const float* x, int N, int C, int H, int W, float* y, unsigned char* arg, int Ho,
                int Wo, hipStream_t st) {
  const long n = (long)N * C * Ho * Wo;
  MD2_TRY(check_u31((long)N * C * H * W));
  if (W % 2 == 0)
    hipLaunchKernelGGL(maxpool_fwd_kernel<true>, dim3(cdiv(n, 256)), dim3(256), 0, st, x, H, W, y,
                       arg, Ho, fd(Wo), fd(Ho), (uint32_t)n);
  else
    hipLaunchKernelGGL(maxpool_fwd_kernel<false>, dim3(cdiv(n, 256)), dim3(256), 0, st, x, H, W, y,
                       arg, Ho, fd(Wo), fd(Ho), (uint32_t)n);
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

int maxpool_bwd(const float* dy, const unsigned char* arg, int N, int C, int H, int W, int Ho,
                int Wo, float* dx, hipStream_t st, SkipAdd skip) {
  MD2_CHECK_ARG(Ho == (H + 1) / 2 && Wo == (W + 1) / 2, "maxpool_bwd: 3x3/2 pad-1 output shape");
  const long n = (long)N * C * Ho * Wo;
  MD2_TRY(check_u31((long)N * C * H * W));
  MD2_CHECK_ARG(!skip.skip || (W % 2 == 0 && skip.lo >= 0 && skip.lo <= skip.hi &&
                               skip.hi <= (long)N * C * H * W && skip.lo % ((long)H * W) == 0 &&
                               skip.hi % ((long)H * W) == 0),
                "maxpool_bwd: skip range (whole images, even W)");
  if (skip.skip)
    hipLaunchKernelGGL((maxpool_bwd_kernel<true, true>), dim3(cdiv(n, 256)), dim3(256), 0, st, dy, arg, H,
                       W, Ho, fd(Wo), fd(Ho), dx, (uint32_t)n, skip_src(skip));
  else if (W % 2 == 0)
    hipLaunchKernelGGL(maxpool_bwd_kernel<true>, dim3(cdiv(n, 256)), dim3(256), 0, st, dy, arg, H,
                       W, Ho, fd(Wo), fd(Ho), dx, (uint32_t)n);
  else
    hipLaunchKernelGGL(maxpool_bwd_kernel<false>, dim3(cdiv(n, 256)), dim3(256), 0, st, dy, arg, H,
                       W, Ho, fd(Wo), fd(Ho), dx, (uint32_t)n);
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

// ---------------------------------------------------------------------------------------------
// upsample_bilinear(x, (2,2)) with align_corners = true (src/depth_decoder.jl:18-19)
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ void src_idx(int o, float r, int in, int& i0, int& i1, float& f) {
  const float s = r * (float)o;
  i0 = min((int)s, in - 1);
  i1 = min(i0 + 1, in - 1);
  f = s - (float)i0;
}

__global__ __launch_bounds__(256) void upsample2_fwd_kernel(const float* __restrict__ x, int h,
                                                            int w, float ry, float rx, FastDiv fdW2,
                                                            FastDiv fdH2, float* __restrict__ y,
                                                            uint32_t n) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint32_t r = fdiv(i, fdW2), plane = fdiv(r, fdH2);
  const int ox = (int)(i - r * fdW2.d), oy = (int)(r - plane * fdH2.d);
  const float* p = x + (long)plane * h * w;
  int y0, y1, x0, x1;
  float fy, fx;
  src_idx(oy, ry, h, y0, y1, fy);
  src_idx(ox, rx, w, x0, x1, fx);
  y[i] = (1.f - fy) * ((1.f - fx) * p[y0 * w + x0] + fx * p[y0 * w + x1]) +
         fy * ((1.f - fx) * p[y1 * w + x0] + fx * p[y1 * w + x1]);
}

// Adjoint as a gather.  For the x2 align-corners map s = r*o, r = (n-1)/(2n-1), 1/r = 2+1/(n-1):
// input i receives from outputs with floor(s) in {i-1, i}, i.e. o in [2i-2, 2i+3] (r*o is never
// within float rounding of an integer except at the end points, which stay inside the range).
// The six per-axis weights are computed once, with the forward's exact float arithmetic.
__device__ __forceinline__ void up_adj_weights(int i, float r, int in, int out, int& o0,
                                               float wv[6]) {
  o0 = 2 * i - 2;
#pragma unroll
  for (int q = 0; q < 6; ++q) {
    const int o = o0 + q;
    float wq = 0.f;
    if (o >= 0 && o < out) {
      int i0, i1;
      float f;
      src_idx(o, r, in, i0, i1, f);
      wq = (i0 == i ? 1.f - f : 0.f) + (i1 == i ? f : 0.f);
    }
    wv[q] = wq;
  }
}

__global__ __launch_bounds__(256) void upsample2_bwd_kernel(const float* __restrict__ dy, int h,
                                                            int w, float ry, float rx, FastDiv fdw,
                                                            FastDiv fdh, float* __restrict__ dx,
                                                            uint32_t n) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int W2 = 2 * w, H2 = 2 * h;
  const uint32_t r = fdiv(i, fdw), plane = fdiv(r, fdh);
  const int ix = (int)(i - r * fdw.d), iy = (int)(r - plane * fdh.d);
  const float* g = dy + plane * (uint32_t)(H2 * W2);
  int oy0, ox0;
  float wy[6], wx[6];
  up_adj_weights(iy, ry, h, H2, oy0, wy);
  up_adj_weights(ix, rx, w, W2, ox0, wx);
  // explicit fmas (the tiled kernel's order and roundings; a skipped zero weight is an exact
  // fma(0, x, acc) = acc there)
  float s = 0.f;
#pragma unroll
  for (int a = 0; a < 6; ++a) {
    if (wy[a] == 0.f) continue;
    const float* row = g + (oy0 + a) * W2;
    float acc = 0.f;
#pragma unroll
    for (int b = 0; b < 6; ++b)
      if (wx[b] != 0.f) acc = fmaf(wx[b], row[ox0 + b], acc);
    s = fmaf(wy[a], acc, s);
  }
  dx[i] = s;
}

// MPI-mode decoder input: repeat(target features, planes) ++ repeat(embed(bins), h, w) along
// channels, planes merged into the batch (src/model.jl:39-50, embed :4-15).  One thread per
// output element; the embedding channel is recomputed per element (2 transcendental ops at most).
__global__ __launch_bounds__(256) void mpi_embed_kernel(const float* __restrict__ feat, long sstride,
                                                        int C, int hw, const float* __restrict__ bins,
                                                        int P, int E, int Ctot, float* __restrict__ out,
                                                        long n) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int px = (int)(i % hw);
  const long t = i / hw;
  const int c = (int)(t % Ctot);
  const long img = t / Ctot;            // b * P + p
  const int b = (int)(img / P), p = (int)(img - (long)b * P);
  float v;
  if (c < C) {
    v = feat[(long)b * sstride + (long)c * hw + px];
  } else if (c >= C + E) {
    v = 0.f;                            // zero padding channels (Ctot > C + E)
  } else {
    const int e = c - C;
    const float x = bins[(long)b * P + p];
    if (e == 0) {
      v = x;
    } else {
      const float a = ldexpf(x, (e - 1) >> 1);  // 2^i x, exact in fp32 like the reference's 2^i .* x
      v = (e & 1) ? sinf(a) : cosf(a);
    }
  }
  out[i] = v;
}

// The _repeat pullback over the plane axis (src/repeat.jl:44-53, block sum): for the first C of
// the Cin channels of every decoder input image, out[b][c][q] (+)= sum_p in[b*P + p][c][q], in the
// fixed order p = 0..P-1 (the embedding channels c >= C get no gradient: embed is
// @non_differentiable, src/model.jl:15).  4 pixels per thread.
__global__ __launch_bounds__(256) void plane_sum_kernel(const float* __restrict__ in, int P, int Cin,
                                                        int C, int hw4, float* __restrict__ out,
                                                        int acc, long n4) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  const int q = (int)(i % hw4);
  const long t = i / hw4;
  const int c = (int)(t % C);
  const long b = t / C;
  const long pstride = (long)Cin * hw4;
  const float4* src = reinterpret_cast<const float4*>(in) + ((b * P) * Cin + c) * (long)hw4 + q;
  float4 s = src[0];
  for (int p = 1; p < P; ++p) {
    const float4 v = src[(long)p * pstride];
    s.x += v.x;
    s.y += v.y;
    s.z += v.z;
    s.w += v.w;
  }
  float4* dst = reinterpret_cast<float4*>(out) + i;
  if (acc) {
    const float4 o = *dst;
    s.x += o.x;
    s.y += o.y;
    s.z += o.z;
    s.w += o.w;
  }
  *dst = s;
}

// the same block sum one pixel per thread, for maps whose h*w is not a multiple of 4 (e.g. the
// 3x10 level-4 map of a 96x320 input)
__global__ __launch_bounds__(256) void plane_sum1_kernel(const float* __restrict__ in, int P, int Cin,
                                                         int C, int hw, float* __restrict__ out,
                                                         int acc, long n) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int q = (int)(i % hw);
  const long t = i / hw;
  const int c = (int)(t % C);
  const long b = t / C;
  const float* src = in + ((b * P) * Cin + c) * (long)hw + q;
  float s = src[0];
  for (int p = 1; p < P; ++p) s += src[(long)p * Cin * hw];
  if (acc) s += out[i];
  out[i] = s;
}

int plane_sum(const float* in, int N, int P, int Cin, int C, long hw, float* out, int accumulate,
              hipStream_t st) {
  if (hw % 4 != 0) {
    const long n = (long)N * C * hw;
    MD2_TRY(check_u31(n));
    hipLaunchKernelGGL(plane_sum1_kernel, dim3(cdiv(n, 256)), dim3(256), 0, st, in, P, Cin, C, (int)hw,
                       out, accumulate, n);
    MD2_LAUNCH_CHECK();
    return MD2_OK;
  }
  const long n4 = (long)N * C * (hw / 4);
  MD2_TRY(check_u31(4 * n4));
  hipLaunchKernelGGL(plane_sum_kernel, dim3(cdiv(n4, 256)), dim3(256), 0, st, in, P, Cin, C,
                     (int)(hw / 4), out, accumulate, n4);
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

// rows of a [R][cols] matrix repeated P times (row r -> rows r*P .. r*P+P-1) and the adjoint sum
__global__ __launch_bounds__(256) void repeat_rows_kernel(const float* __restrict__ src, int cols,
                                                          int P, float* __restrict__ dst, long n) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const long row = i / cols;
  dst[i] = src[(row / P) * cols + (i - row * cols)];
}
__global__ __launch_bounds__(256) void repeat_rows_adj_kernel(const float* __restrict__ src, int cols,
                                                              int P, float* __restrict__ dst, long n) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const long row = i / cols, col = i - row * cols;
  float s = 0.f;
  for (int p = 0; p < P; ++p) s += src[(row * P + p) * cols + col];
  dst[i] = s;
}

int repeat_rows(const float* src, long rows, int cols, int P, float* dst, hipStream_t st) {
  const long n = rows * P * cols;
  MD2_TRY(check_u31(n));
  if (n == 0) return MD2_OK;
  hipLaunchKernelGGL(repeat_rows_kernel, dim3(cdiv(n, 256)), dim3(256), 0, st, src, cols, P, dst, n);
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}
int repeat_rows_adjoint(const float* src, long rows, int cols, int P, float* dst, hipStream_t st) {
  const long n = rows * cols;
  MD2_TRY(check_u31(n * P));
  if (n == 0) return MD2_OK;
  hipLaunchKernelGGL(repeat_rows_adj_kernel, dim3(cdiv(n, 256)), dim3(256), 0, st, src, cols, P, dst, n);
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

int mpi_embed_features(const float* feat, long sample_stride, int N, int C, int h, int w,
                       const float* bins, int P, int L, float* out, hipStream_t st, int Ctot) {
  const int E = 2 * L + 1;
  if (Ctot <= 0) Ctot = C + E;
  if (Ctot < C + E) {
    set_error("mpi_embed_features: output channels < C + 2L + 1");
    return MD2_EINVAL;
  }
  const long n = (long)N * P * Ctot * h * w;
  MD2_TRY(check_u31(n));
  hipLaunchKernelGGL(mpi_embed_kernel, dim3(cdiv(n, 256)), dim3(256), 0, st, feat, sample_stride, C,
                     h * w, bins, P, E, Ctot, out, n);
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

__global__ __launch_bounds__(256) void concat_kernel(const float* __restrict__ a, int ca,
                                                     const float* __restrict__ b, int cb, long hw,
                                                     float* __restrict__ out, long n) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const long px = i % hw, t = i / hw;
  const int c = (int)(t % (ca + cb));
  const long img = t / (ca + cb);
  out[i] = c < ca ? a[(img * ca + c) * hw + px] : b[(img * cb + (c - ca)) * hw + px];
}

int concat_channels(const float* a, int ca, const float* b, int cb, int N, long hw, float* out,
                    hipStream_t st) {
  const long n = (long)N * (ca + cb) * hw;
  MD2_TRY(check_u31(n));
  hipLaunchKernelGGL(concat_kernel, dim3(cdiv(n, 256)), dim3(256), 0, st, a, ca, b, cb, hw, out, n);
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

// Tiled adjoint over the STACKED planes: the N*C input planes of h rows are one (N*C*h) x w
// image, and input row r (plane r / h, local row r % h) reads output rows 2r-2 .. 2r+3 of the
// equally stacked (N*C*2h) x 2w gradient, whatever plane they belong to -- an output row of a
// neighbouring plane gets weight 0 from up_adj_weights (local index outside [0, 2h)), so a tile
// may straddle planes and the small coarse levels (13 x 4 planes) fill whole blocks.  A block of
// TW x (RPT * 256 / TW) input pixels stages its (2 TH + 4) x (2 TW + 4) output window in LDS with
// every thread's loads issued before any LDS store, then each thread contracts RPT vertically
// adjacent input pixels of one column (its six column weights computed once) from LDS with the
// same weights and the same summation order as upsample2_bwd_kernel (bit-identical).  RPT = 4
// (round 6): a quarter of the blocks, 4x the loads in flight per block and 4.5 instead of 5.3
// staged floats per input pixel -- the one-row tiles were latency-bound (~1 TB/s).
template <int TW, int RPT>
__global__ __launch_bounds__(256) void upsample2_bwd_tile_kernel(const float* __restrict__ dy, int h,
                                                                 int w, long rows, float ry, float rx,
                                                                 float* __restrict__ dx) {
  constexpr int TY = 256 / TW, TH = TY * RPT, FR = 2 * TH + 4, FC = 2 * TW + 4;
  constexpr int NL = (FR * FC + 255) / 256;
  __shared__ float t[FR][FC + 1];
  const int W2 = 2 * w;
  const int ix0 = blockIdx.x * TW;
  const long r0 = (long)blockIdx.y * TH;
  const long oyb = 2 * r0 - 2, orows = 2 * rows;
  const int oxb = 2 * ix0 - 2;
  float v[NL];
#pragma unroll
  for (int q = 0; q < NL; ++q) {
    const int e = threadIdx.x + 256 * q;
    const int r = e / FC, c = e - r * FC;
    const long oy = oyb + r;
    const int ox = oxb + c;
    v[q] = (e < FR * FC && oy >= 0 && oy < orows && ox >= 0 && ox < W2) ? dy[oy * W2 + ox] : 0.f;
  }
#pragma unroll
  for (int q = 0; q < NL; ++q) {
    const int e = threadIdx.x + 256 * q;
    const int r = e / FC, c = e - r * FC;
    if (e < FR * FC) t[r][c] = v[q];
  }
  __syncthreads();
  const int tx = threadIdx.x % TW, ty = threadIdx.x / TW;
  const int ix = ix0 + tx;
  if (ix >= w) return;
  int ox0;
  float wx[6];
  up_adj_weights(ix, rx, w, W2, ox0, wx);
#pragma unroll
  for (int k = 0; k < RPT; ++k) {
    const int ly = ty * RPT + k;
    const long row = r0 + ly;
    if (row >= rows) break;
    const int iy = (int)(row % h);
    int oy0;
    float wy[6];
    up_adj_weights(iy, ry, h, 2 * h, oy0, wy);
    float s = 0.f;
#pragma unroll
    for (int a = 0; a < 6; ++a) {
      float acc = 0.f;
#pragma unroll
      for (int b = 0; b < 6; ++b) acc = fmaf(wx[b], t[2 * ly + a][2 * tx + b], acc);
      s = fmaf(wy[a], acc, s);
    }
    dx[row * w + ix] = s;
  }
}

static inline float up_ratio(int in, int out) { return out > 1 ? (float)(in - 1) / (float)(out - 1) : 0.f; }

int upsample2_fwd(const float* x, int N, int C, int h, int w, float* y, hipStream_t st) {
  const long n = (long)N * C * 4 * h * w;
  MD2_TRY(check_u31(n));
  hipLaunchKernelGGL(upsample2_fwd_kernel, dim3(cdiv(n, 256)), dim3(256), 0, st, x, h, w,
                     up_ratio(h, 2 * h), up_ratio(w, 2 * w), fd(2 * w), fd(2 * h), y, (uint32_t)n);
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

int upsample2_bwd(const float* dy, int N, int C, int h, int w, float* dx, hipStream_t st) {
  const long n = (long)N * C * h * w;
  MD2_TRY(check_u31(4 * n));
  static const int tiled = tuning_knob("MD2_UP_TILED", 1);
  const long rows = (long)N * C * h;
  if (tiled && w > 16 && cdiv(rows, 32) <= 65535)
    hipLaunchKernelGGL((upsample2_bwd_tile_kernel<32, 4>), dim3(cdiv(w, 32), cdiv(rows, 32)), dim3(256), 0, st, dy,
                       h, w, rows, up_ratio(h, 2 * h), up_ratio(w, 2 * w), dx);
  else if (tiled && cdiv(rows, 16) <= 65535)   // (4 rows per thread: 13.7 vs 10.3 us on the 4x13 maps)
    hipLaunchKernelGGL((upsample2_bwd_tile_kernel<16, 1>), dim3(cdiv(w, 16), cdiv(rows, 16)), dim3(256), 0, st, dy,
                       h, w, rows, up_ratio(h, 2 * h), up_ratio(w, 2 * w), dx);
  else
    hipLaunchKernelGGL(upsample2_bwd_kernel, dim3(cdiv(n, 256)), dim3(256), 0, st, dy, h, w,
                       up_ratio(h, 2 * h), up_ratio(w, 2 * w), fd(w), fd(h), dx, (uint32_t)n);
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

// ---------------------------------------------------------------------------------------------
// Pose head: Conv((1,1), 256=>6) + mean over (w,h) + 1e-2 scale (src/pose_decoder.jl:19,29-30).
// mean(W x + b) = W mean(x) + b, so the 1x1 conv runs on the spatial means.
// ---------------------------------------------------------------------------------------------
// one wave per (pair, channel): lanes stride the plane, then a fixed-order wave sum (one thread
// per channel walking its plane serially was latency-bound: 28 us for 24 x 256 planes of 52)
__global__ __launch_bounds__(256) void pose_means_kernel(const float* __restrict__ x, int C, long HW,
                                                         float* __restrict__ means) {
  const int q = blockIdx.x, c = blockIdx.y * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (c >= C) return;
  const float* p = x + ((long)q * C + c) * HW;
  float s = 0.f;
  for (long i = lane; i < HW; i += 64) s += p[i];
  s = wave_sum(s);
  if (lane == 0) means[(long)q * C + c] = s / (float)HW;
}

__global__ __launch_bounds__(64) void pose_fc_kernel(const float* __restrict__ means, int C,
                                                     const float* __restrict__ w,
                                                     const float* __restrict__ b,
                                                     float* __restrict__ pose) {
  const int q = blockIdx.x, k = blockIdx.y;
  float s = 0.f;
  for (int c = threadIdx.x; c < C; c += 64) s += w[(long)k * C + c] * means[(long)q * C + c];
  s = wave_sum(s);
  if (threadIdx.x == 0) pose[q * 6 + k] = 1e-2f * (s + b[k]);
}

int pose_head_fwd(const float* x, int Q, int C, long HW, const float* w, const float* b,
                  float* means, float* pose, hipStream_t st) {
  hipLaunchKernelGGL(pose_means_kernel, dim3(Q, cdiv(C, 4)), dim3(256), 0, st, x, C, HW, means);
  MD2_LAUNCH_CHECK();
  hipLaunchKernelGGL(pose_fc_kernel, dim3(Q, 6), dim3(64), 0, st, means, C, w, b, pose);
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

__global__ __launch_bounds__(256) void pose_head_dx_kernel(const float* __restrict__ dpose, int C,
                                                           long HW, const float* __restrict__ w,
                                                           FastDiv fdHW, FastDiv fdC,
                                                           float* __restrict__ dx, uint32_t n) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint32_t qc = fdiv(i, fdHW), q = fdiv(qc, fdC);
  const int c = (int)(qc - q * fdC.d);
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < 6; ++k) s += dpose[q * 6 + k] * w[(long)k * C + c];
  dx[i] = s * (1e-2f / (float)HW);
}

__global__ __launch_bounds__(256) void pose_head_dw_kernel(const float* __restrict__ dpose, int Q,
                                                           int C, const float* __restrict__ means,
                                                           float* __restrict__ dw,
                                                           float* __restrict__ db) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx < 6 * C) {
    const int k = idx / C, c = idx % C;
    float s = 0.f;
    for (int q = 0; q < Q; ++q) s += dpose[q * 6 + k] * means[(long)q * C + c];
    dw[idx] = 1e-2f * s;
  }
  if (idx < 6) {
    float s = 0.f;
    for (int q = 0; q < Q; ++q) s += dpose[q * 6 + idx];
    db[idx] = 1e-2f * s;
  }
}

int pose_head_bwd(const float* dpose, int Q, int C, long HW, const float* w, const float* means,
                  float* dx, float* dw, float* db, hipStream_t st) {
  const long n = (long)Q * C * HW;
  MD2_TRY(check_u31(n));
  hipLaunchKernelGGL(pose_head_dx_kernel, dim3(cdiv(n, 256)), dim3(256), 0, st, dpose, C, HW, w,
                     fd(HW), fd(C), dx, (uint32_t)n);
  MD2_LAUNCH_CHECK();
  hipLaunchKernelGGL(pose_head_dw_kernel, dim3(cdiv(6 * C, 256)), dim3(256), 0, st, dpose, Q, C,
                     means, dw, db);
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

// ---------------------------------------------------------------------------------------------
// elementwise helpers
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void axpy_kernel(float* __restrict__ y, const float* __restrict__ x,
                                                   long n) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i < n) y[i] += x[i];
}

int axpy(float* y, const float* x, long n, hipStream_t st) {
  hipLaunchKernelGGL(axpy_kernel, dim3(cdiv(n, 256)), dim3(256), 0, st, y, x, n);
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

// pose pairs q = s*N + n read (sq[q], sq[q+N]) (src/model.jl:65-70 in frame-major order):
// dsq[b] = (b < 2N ? dpin[b][0:C] : 0) + (b >= N ? dpin[b-N][C:2C] : 0)
// Pose pairs (src/model.jl:57-70 _get_pose_features): pair j of sample q = (frame a_j, frame b_j)
// with a_j = min(source_j, target), b_j = max(source_j, target); squeezer outputs are frame-major
// images f*N + q.  pair_gather builds the PoseDecoder input [2N][2C][HW] (only when the pairs are
// not the (q, q+N) zero-copy layout of target 2 / sources 1, 3); pair_grad scatters its gradient
// back: d sq[f*N + q] = sum_j [a_j == f] d pin[jN + q][:C] + [b_j == f] d pin[jN + q][C:].
__global__ __launch_bounds__(256) void pair_gather_kernel(const float* __restrict__ sq, int N,
                                                          FastDiv fdper, int a0, int a1, int b0,
                                                          int b1, float* __restrict__ pin,
                                                          uint32_t n) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;   // over [2N][2][per]
  if (i >= n) return;
  const long per = fdper.d;
  const uint32_t row = fdiv(i, fdper);                // (jN + q)*2 + half
  const long r = i - (long)row * per;
  const int half = row & 1, img = row >> 1, j = img >= N ? 1 : 0, q = img - j * N;
  const int f = half ? (j ? b1 : b0) : (j ? a1 : a0);
  pin[i] = sq[((long)f * N + q) * per + r];
}

__global__ __launch_bounds__(256) void pair_grad_kernel(const float* __restrict__ dpin, int N,
                                                        FastDiv fdper, int a0, int a1, int b0,
                                                        int b1, float* __restrict__ dsq,
                                                        uint32_t n) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;   // over [3N][per]
  if (i >= n) return;
  const long per = fdper.d;
  const uint32_t b = fdiv(i, fdper);
  const long r = i - (long)b * per;
  const int f = (int)b / N, q = (int)b - f * N;
  float s = 0.f;
  if (a0 == f) s += dpin[((long)q * 2) * per + r];
  if (b0 == f) s += dpin[((long)q * 2 + 1) * per + r];
  if (a1 == f) s += dpin[((long)(N + q) * 2) * per + r];
  if (b1 == f) s += dpin[((long)(N + q) * 2 + 1) * per + r];
  dsq[i] = s;
}

int pair_gather(const float* sq, int N, int C, long HW, const int a[2], const int b[2], float* pin,
                hipStream_t st) {
  const long n = 4L * N * C * HW;
  MD2_TRY(check_u31(n));
  hipLaunchKernelGGL(pair_gather_kernel, dim3(cdiv(n, 256)), dim3(256), 0, st, sq, N, fd((long)C * HW),
                     a[0], a[1], b[0], b[1], pin, (uint32_t)n);
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

int pair_grad_gather(const float* dpin, int N, int C, long HW, const int a[2], const int b[2],
                     float* dsq, hipStream_t st) {
  const long n = 3L * N * C * HW;
  MD2_TRY(check_u31(2 * n));
  hipLaunchKernelGGL(pair_grad_kernel, dim3(cdiv(n, 256)), dim3(256), 0, st, dpin, N, fd((long)C * HW),
                     a[0], a[1], b[0], b[1], dsq, (uint32_t)n);
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

// Flux ADAM (Flux.Optimise.apply!): m = b1 m + (1-b1) g; v = b2 v + (1-b2) g^2;
// p -= lr * (m / bc1) / (sqrt(v / bc2) + eps), with bc = 1 - beta^t.
__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v, long n,
                                                   float lr, float b1, float b2, float eps, float bc1,
                                                   float bc2, float gscale) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const float gi = g[i] * gscale;
  const float mi = b1 * m[i] + (1.f - b1) * gi;
  const float vi = b2 * v[i] + (1.f - b2) * gi * gi;
  m[i] = mi;
  v[i] = vi;
  p[i] -= lr * (mi / bc1) / (sqrtf(vi / bc2) + eps);
}

// Graph-replayed ADAM: the step counter lives on the device (adam_prep increments it and forms
// the bias corrections), so one captured step replays for every t.
__global__ void adam_prep_kernel(int* __restrict__ step, float* __restrict__ bc, float b1, float b2) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const int t = step[0] + 1;
  step[0] = t;
  bc[0] = (float)(1.0 - pow((double)b1, (double)t));
  bc[1] = (float)(1.0 - pow((double)b2, (double)t));
}

__global__ void set_int_kernel(int* __restrict__ p, int v) {
  if (threadIdx.x == 0 && blockIdx.x == 0) p[0] = v;
}

__global__ __launch_bounds__(256) void adam_dev_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                       float* __restrict__ m, float* __restrict__ v, long n,
                                                       float lr, float b1, float b2, float eps,
                                                       const float* __restrict__ bc, float gscale) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const float bc1 = bc[0], bc2 = bc[1];
  const float gi = g[i] * gscale;
  const float mi = b1 * m[i] + (1.f - b1) * gi;
  const float vi = b2 * v[i] + (1.f - b2) * gi * gi;
  m[i] = mi;
  v[i] = vi;
  p[i] -= lr * (mi / bc1) / (sqrtf(vi / bc2) + eps);
}

int adam_prep(int* step, float* bc, float b1, float b2, hipStream_t st) {
  hipLaunchKernelGGL(adam_prep_kernel, dim3(1), dim3(64), 0, st, step, bc, b1, b2);
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

int set_device_int(int* p, int v, hipStream_t st) {
  hipLaunchKernelGGL(set_int_kernel, dim3(1), dim3(64), 0, st, p, v);
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

int adam_step_dev(float* p, const float* g, float* m, float* v, long n, float lr, float b1, float b2,
                  float eps, const float* bc, float gscale, hipStream_t st) {
  hipLaunchKernelGGL(adam_dev_kernel, dim3(cdiv(n, 256)), dim3(256), 0, st, p, g, m, v, n, lr, b1, b2,
                     eps, bc, gscale);
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

// x *= s (train_loss pullback cotangent on the loss-tail gradients)
__global__ __launch_bounds__(256) void scale_kernel(float* __restrict__ x, long n, float s) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i < n) x[i] *= s;
}
int scale_inplace(float* x, long n, float s, hipStream_t st) {
  if (n <= 0) return MD2_OK;
  hipLaunchKernelGGL(scale_kernel, dim3(cdiv(n, 256)), dim3(256), 0, st, x, n, s);
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

// d pre = d disp .* (s .* (1 - s)) -- the sigmoid head's pullback of a caller cotangent on the
// disparity (md2_model_set_cotangents); the same rounding as the loss tail's fused form
// (loss_kernels.hip up_adjoint: acc *= sg * (1 - sg)), so a cotangent that equals the loss tail's
// own d disp gives a bit-identical head gradient.  g == nullptr: zero cotangent.
__global__ __launch_bounds__(256) void sigmoid_cot_kernel(const float* __restrict__ g,
                                                          const float* __restrict__ s,
                                                          float* __restrict__ out, long n) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const float sg = s[i];
  out[i] = g ? g[i] * (sg * (1.f - sg)) : 0.f;
}
int sigmoid_cotangent(const float* g, const float* s, float* out, long n, hipStream_t st) {
  if (n <= 0) return MD2_OK;
  hipLaunchKernelGGL(sigmoid_cot_kernel, dim3(cdiv(n, 256)), dim3(256), 0, st, g, s, out, n);
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

// Flux Conv weights (kw,kh,cin,cout) = C-order [cout][cin][kh][kw] of a TRUE convolution ->
// the library's cross-correlation layout (and back: the map is an involution): both spatial axes
// reversed, dst[o][i][y][x] = src[o][i][kh-1-y][kw-1-x]
__global__ __launch_bounds__(256) void flip_taps_kernel(const float* __restrict__ src, float* __restrict__ dst,
                                                        long planes, int kh, int kw) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  const long kk = (long)kh * kw;
  if (i >= planes * kk) return;
  const long pl = i / kk;
  const int t = (int)(i - pl * kk), y = t / kw, x = t - y * kw;
  dst[i] = src[pl * kk + (long)(kh - 1 - y) * kw + (kw - 1 - x)];
}
int flip_taps(const float* src, float* dst, long planes, int kh, int kw, hipStream_t st) {
  hipLaunchKernelGGL(flip_taps_kernel, dim3(cdiv(planes * kh * kw, 256)), dim3(256), 0, st, src, dst,
                     planes, kh, kw);
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

int adam_step(float* p, const float* g, float* m, float* v, long n, float lr, float b1, float b2,
              float eps, float bc1, float bc2, float gscale, hipStream_t st) {
  hipLaunchKernelGGL(adam_kernel, dim3(cdiv(n, 256)), dim3(256), 0, st, p, g, m, v, n, lr, b1, b2,
                     eps, bc1, bc2, gscale);
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

}  // namespace md2
