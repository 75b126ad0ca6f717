// Single-output-channel 3x3 / stride 1 / pad 1 convolutions: the DepthDecoder disparity heads
// Conv((3,3), cin=>1, σ) after pad_reflect (src/depth_decoder.jl:5, 46), forward / ∇conv_data /
// ∇conv_filter.  With one output row an implicit GEMM leaves 31 of 32 MFMA rows idle, while the
// work is 9*Cin MACs per pixel -- far below the HBM time of reading Cin planes -- so these are
// VALU kernels sized for HBM: one pixel per lane, filter taps as wave-uniform scalar loads.
#include "head.h"

namespace md2 {

namespace {

// source row/column of output index o + k - 1 (k = 0..2): reflect (pad_reflect excludes the
// edge: -1 -> 1, n -> n-2) or zero padding (returns -1)
template <bool RFL>
__device__ __forceinline__ int src_of(int o, int k, int n) {
  int v = o + k - 1;
  if (RFL) {
    v = v < 0 ? -v : v;
    v = v >= n ? 2 * n - 2 - v : v;
    return v;
  }
  return (v < 0 || v >= n) ? -1 : v;
}

// image offset of operand b (TensorIn p0 addressing: frame-major stem batches use bdiv/bhi)
__device__ __forceinline__ long img_off(const HeadIn& x, int b) {
  return (long)(b % x.bdiv) * x.bs0 + (long)(b / x.bdiv) * x.bhi;
}

__device__ __forceinline__ float act_f(float v, int act) {
  switch (act) {
    case ACT_RELU: return fmaxf(v, 0.f);
    case ACT_ELU: return v > 0.f ? v : expm1f(v);
    case ACT_SIGMOID: return 1.f / (1.f + expf(-v));
    default: return v;
  }
}

// ---- forward: y[b][p] = act(bias + sum_c sum_tap w[c][tap] x[b][c][src(p, tap)]) -------------
// A block is PX = 256/CG pixels x CG channel groups (CG > 1 on the coarse heads, whose few pixels
// would otherwise leave each lane a long serial channel loop); the group partials are summed in
// fixed order through LDS.
template <bool RFL>
__global__ __launch_bounds__(256) void head_fwd_kernel(HeadIn x, HeadW w, int Cin, int H, int W,
                                                       FastDiv fdW, FastDiv fdH, uint32_t npix,
                                                       int cg_shift, const float* __restrict__ bias,
                                                       int act, float* __restrict__ y, long ybs,
                                                       int accumulate) {
  __shared__ float s_part[256];
  const int px_shift = 8 - cg_shift;
  const int g = threadIdx.x >> px_shift, pl = threadIdx.x & ((1 << px_shift) - 1);
  const uint32_t i = (blockIdx.x << px_shift) + pl;
  const bool live = i < npix;
  const uint32_t ii = live ? i : npix - 1;
  const uint32_t r = fdiv(ii, fdW), b = fdiv(r, fdH);
  const int px = (int)(ii - r * fdW.d), py = (int)(r - b * fdH.d);
  int ro[3], co[3];
  bool rv[3], cv[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const int sy = src_of<RFL>(py, k, H), sx = src_of<RFL>(px, k, W);
    rv[k] = sy >= 0;
    cv[k] = sx >= 0;
    ro[k] = (sy < 0 ? 0 : sy) * W;
    co[k] = sx < 0 ? 0 : sx;
  }
  const float* xb = x.p + img_off(x, (int)b);
  const long HW = (long)H * W;
  const int cpg = (Cin + (1 << cg_shift) - 1) >> cg_shift;
  const int cb = g * cpg, ce = min(Cin, cb + cpg);
  float acc = 0.f;
  for (int c = cb; c < ce; ++c) {
    const float* xc = xb + c * HW;
    const float* wc = w.p + (long)c * w.sc;
#pragma unroll
    for (int kh = 0; kh < 3; ++kh)
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const float v = (RFL || (rv[kh] && cv[kw])) ? xc[ro[kh] + co[kw]] : 0.f;
        acc = fmaf(wc[(long)(kh * 3 + kw) * w.st], v, acc);
      }
  }
  if (cg_shift) {
    s_part[threadIdx.x] = acc;
    __syncthreads();
    if (g != 0) return;
    for (int q = 1; q < (1 << cg_shift); ++q) acc += s_part[(q << px_shift) + pl];
  }
  if (!live) return;
  if (bias) acc += bias[0];
  acc = act_f(acc, act);
  float* dst = y + (long)b * ybs + (long)py * W + px;
  *dst = accumulate ? *dst + acc : acc;
}

// ---- data gradient: dx[b][c][q] = sum over (p, tap) with src(p, tap) = q of w[c][tap] dy[b][p].
// Per axis, q collects from p = q + 1 - k for k = 0..2 (when inside), and under reflection also
// from the folded border taps: q = 1 from (p = 0, k = 0) and q = n-2 from (p = n-1, k = 2).
// The (up to 5 x 5) contributions are first summed into 9 per-tap dy values D[tap], then every
// channel is 9 FMAs: dx[c] = sum_tap w[c][tap] D[tap].
// Channel groups as in the forward (each group re-forms D, then writes its channel range).
template <bool RFL>
__global__ __launch_bounds__(256) void head_dgrad_kernel(const float* __restrict__ dy, HeadW w,
                                                         int Cin, int H, int W, FastDiv fdW,
                                                         FastDiv fdH, uint32_t npix, int cg_shift,
                                                         float* __restrict__ dx, long dxbs,
                                                         int accumulate) {
  const int px_shift = 8 - cg_shift;
  const int grp = threadIdx.x >> px_shift;
  const uint32_t i = (blockIdx.x << px_shift) + (threadIdx.x & ((1 << px_shift) - 1));
  if (i >= npix) return;
  const uint32_t r = fdiv(i, fdW), b = fdiv(r, fdH);
  const int qx = (int)(i - r * fdW.d), qy = (int)(r - b * fdH.d);
  // slots 0..2: tap k = slot, source p = q + 1 - k; slot 3: k = 0 folded; slot 4: k = 2 folded
  int ry[5], rx[5];
  bool vy[5], vx[5];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    ry[k] = qy + 1 - k;
    rx[k] = qx + 1 - k;
    vy[k] = ry[k] >= 0 && ry[k] < H;
    vx[k] = rx[k] >= 0 && rx[k] < W;
  }
  ry[3] = 0;
  rx[3] = 0;
  ry[4] = H - 1;
  rx[4] = W - 1;
  vy[3] = RFL && qy == 1;
  vx[3] = RFL && qx == 1;
  vy[4] = RFL && qy == H - 2;
  vx[4] = RFL && qx == W - 2;
  constexpr int KOF[5] = {0, 1, 2, 0, 2};
  const float* g = dy + (long)b * H * W;
  float D[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) D[t] = 0.f;
#pragma unroll
  for (int a = 0; a < 5; ++a) {
    if (!vy[a]) continue;
    const float* row = g + ry[a] * W;
#pragma unroll
    for (int c = 0; c < 5; ++c)
      if (vx[c]) D[KOF[a] * 3 + KOF[c]] += row[rx[c]];
  }
  float* out = dx + (long)b * dxbs + (long)qy * W + qx;
  const long HW = (long)H * W;
  const int cpg = (Cin + (1 << cg_shift) - 1) >> cg_shift;
  const int cb = grp * cpg, ce = min(Cin, cb + cpg);
  for (int c = cb; c < ce; ++c) {
    const float* wc = w.p + (long)c * w.sc;
    float v = 0.f;
#pragma unroll
    for (int t = 0; t < 9; ++t) v = fmaf(wc[(long)t * w.st], D[t], v);
    float* d = out + c * HW;
    *d = accumulate ? *d + v : v;
  }
}

// ---- filter gradient, pass 1: per-block partial sums of dy[p] * x[c][src(p, tap)] over a
// grid-strided pixel range, for a group of HEAD_CG channels (blockIdx.y); group 0 also sums dy
// (the bias gradient).  Partials [blockIdx.x][Cin*9 + 1]; pass 2 reduces them in fixed order.
constexpr int HEAD_CG = 8;

template <bool RFL>
__global__ __launch_bounds__(256) void head_wgrad_partial_kernel(HeadIn x, const float* __restrict__ dy,
                                                                 int Cin, int H, int W, FastDiv fdW,
                                                                 FastDiv fdH, uint32_t npix,
                                                                 float* __restrict__ part) {
  __shared__ float s_red[4][HEAD_CG * 9 + 1];
  const int c0 = blockIdx.y * HEAD_CG;
  const int ncg = min(HEAD_CG, Cin - c0);
  float acc[HEAD_CG * 9 + 1];
#pragma unroll
  for (int t = 0; t < HEAD_CG * 9 + 1; ++t) acc[t] = 0.f;
  const long HW = (long)H * W;
  const uint32_t stride = gridDim.x * 256;
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < npix; i += stride) {
    const uint32_t r = fdiv(i, fdW), b = fdiv(r, fdH);
    const int px = (int)(i - r * fdW.d), py = (int)(r - b * fdH.d);
    const float g = dy[i];
    acc[HEAD_CG * 9] += g;
    int ro[3], co[3];
    bool rv[3], cv[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const int sy = src_of<RFL>(py, k, H), sx = src_of<RFL>(px, k, W);
      rv[k] = sy >= 0;
      cv[k] = sx >= 0;
      ro[k] = (sy < 0 ? 0 : sy) * W;
      co[k] = sx < 0 ? 0 : sx;
    }
    const float* xb = x.p + img_off(x, (int)b) + c0 * HW;
#pragma unroll
    for (int c = 0; c < HEAD_CG; ++c) {
      if (c < ncg) {
        const float* xc = xb + c * HW;
#pragma unroll
        for (int kh = 0; kh < 3; ++kh)
#pragma unroll
          for (int kw = 0; kw < 3; ++kw) {
            const float v = (RFL || (rv[kh] && cv[kw])) ? xc[ro[kh] + co[kw]] : 0.f;
            acc[c * 9 + kh * 3 + kw] = fmaf(g, v, acc[c * 9 + kh * 3 + kw]);
          }
      }
    }
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int t = 0; t < HEAD_CG * 9 + 1; ++t) {
    const float v = wave_sum(acc[t]);
    if (lane == 0) s_red[wv][t] = v;
  }
  __syncthreads();
  float* dst = part + (long)blockIdx.x * (Cin * 9 + 1);
  for (int t = threadIdx.x; t < ncg * 9; t += 256)
    dst[c0 * 9 + t] = (s_red[0][t] + s_red[1][t]) + (s_red[2][t] + s_red[3][t]);
  if (blockIdx.y == 0 && threadIdx.x == 0) {
    const int t = HEAD_CG * 9;
    dst[Cin * 9] = (s_red[0][t] + s_red[1][t]) + (s_red[2][t] + s_red[3][t]);
  }
}

// pass 2: one block per column (Cin*9 weights + the bias), fixed-order tree over the partials
__global__ __launch_bounds__(256) void head_wgrad_reduce_kernel(const float* __restrict__ part,
                                                                int parts, int ncols,
                                                                float* __restrict__ dw,
                                                                float* __restrict__ db,
                                                                int accumulate) {
  __shared__ float s_red[4];
  const int t = blockIdx.x;
  float v = 0.f;
  for (int k = threadIdx.x; k < parts; k += 256) v += part[(long)k * (ncols + 1) + t];
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x != 0) return;
  v = (s_red[0] + s_red[1]) + (s_red[2] + s_red[3]);
  float* d = t < ncols ? dw + t : db;
  if (!d) return;
  *d = accumulate ? *d + v : v;
}

// pixels per partial block: ~8 per lane (the 73-accumulator block reduction is amortised over
// them), raised toward >= 512 blocks (parts x channel groups) while every lane keeps a pixel
int head_parts(long npix, int Cin) {
  const long groups = cdiv(Cin, HEAD_CG);
  long parts = std::max<long>(cdiv(npix, 256 * 8), 1);
  parts = std::max(parts, std::min<long>(cdiv(512, groups), cdiv(npix, 256)));
  return (int)std::min<long>(parts, 2048);
}

// channel groups (log2) so a launch has >= ~128k lanes, each group keeping >= 4 channels
int head_cg_shift(long npix, int Cin) {
  int sh = 0;
  while (sh < 4 && (npix << sh) < 131072 && (Cin >> (sh + 1)) >= 4) ++sh;
  return sh;
}

}  // namespace

bool head_conv_ok(const ConvShape& s) {
  return s.Cout == 1 && s.KH == 3 && s.KW == 3 && s.stride == 1 && s.pad == 1 && s.H >= 2 &&
         s.W >= 2 && (long)s.N * s.H * s.W < (1L << 31);
}

size_t head_wgrad_workspace(const ConvShape& s) {
  return (size_t)head_parts((long)s.N * s.H * s.W, s.Cin) * (s.Cin * 9 + 1) * sizeof(float);
}

int head_fwd(const ConvShape& s, const HeadIn& x, HeadW w, const float* bias, int act, float* y,
             long ybs, int accumulate, hipStream_t st) {
  const uint32_t npix = (uint32_t)((long)s.N * s.H * s.W);
  const FastDiv fdW = make_fastdiv(s.W), fdH = make_fastdiv(s.H);
  const int sh = head_cg_shift(npix, s.Cin);
  const dim3 grid(cdiv(npix, 256 >> sh));
  if (s.reflect)
    hipLaunchKernelGGL(head_fwd_kernel<true>, grid, dim3(256), 0, st, x, w, s.Cin, s.H, s.W, fdW,
                       fdH, npix, sh, bias, act, y, ybs, accumulate);
  else
    hipLaunchKernelGGL(head_fwd_kernel<false>, grid, dim3(256), 0, st, x, w, s.Cin, s.H, s.W, fdW,
                       fdH, npix, sh, bias, act, y, ybs, accumulate);
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

int head_dgrad(const ConvShape& s, const float* dy, HeadW w, float* dx, long dxbs, int accumulate,
               hipStream_t st) {
  const uint32_t npix = (uint32_t)((long)s.N * s.H * s.W);
  const FastDiv fdW = make_fastdiv(s.W), fdH = make_fastdiv(s.H);
  const int sh = head_cg_shift(npix, s.Cin);
  const dim3 grid(cdiv(npix, 256 >> sh));
  if (s.reflect)
    hipLaunchKernelGGL(head_dgrad_kernel<true>, grid, dim3(256), 0, st, dy, w, s.Cin, s.H, s.W,
                       fdW, fdH, npix, sh, dx, dxbs, accumulate);
  else
    hipLaunchKernelGGL(head_dgrad_kernel<false>, grid, dim3(256), 0, st, dy, w, s.Cin, s.H, s.W,
                       fdW, fdH, npix, sh, dx, dxbs, accumulate);
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

int head_wgrad(const ConvShape& s, const HeadIn& x, const float* dy, float* dw, float* db,
               int accumulate, void* ws, size_t ws_bytes, hipStream_t st) {
  const long np = (long)s.N * s.H * s.W;
  const int parts = head_parts(np, s.Cin);
  MD2_CHECK_ARG(ws && ws_bytes >= head_wgrad_workspace(s), "head_wgrad workspace");
  float* part = (float*)ws;
  const uint32_t npix = (uint32_t)np;
  const FastDiv fdW = make_fastdiv(s.W), fdH = make_fastdiv(s.H);
  const dim3 grid(parts, cdiv(s.Cin, HEAD_CG));
  if (s.reflect)
    hipLaunchKernelGGL(head_wgrad_partial_kernel<true>, grid, dim3(256), 0, st, x, dy, s.Cin, s.H,
                       s.W, fdW, fdH, npix, part);
  else
    hipLaunchKernelGGL(head_wgrad_partial_kernel<false>, grid, dim3(256), 0, st, x, dy, s.Cin, s.H,
                       s.W, fdW, fdH, npix, part);
  MD2_LAUNCH_CHECK();
  const int ncols = s.Cin * 9;
  hipLaunchKernelGGL(head_wgrad_reduce_kernel, dim3(ncols + 1), dim3(256), 0, st, part, parts,
                     ncols, dw, db, accumulate);
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

}  // namespace md2
