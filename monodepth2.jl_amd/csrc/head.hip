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
  __shared__ double s_dred[4];
  const int c0 = blockIdx.y * HEAD_CG;
  const int ncg = min(HEAD_CG, Cin - c0);
  float acc[HEAD_CG * 9 + 1];
#pragma unroll
  for (int t = 0; t < HEAD_CG * 9 + 1; ++t) acc[t] = 0.f;
  double gsum = 0.0;   // bias gradient in fp64 (a long cancelling sum)
  const long HW = (long)H * W;
  const uint32_t stride = gridDim.x * 256;
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < npix; i += stride) {
    const uint32_t r = fdiv(i, fdW), b = fdiv(r, fdH);
    const int px = (int)(i - r * fdW.d), py = (int)(r - b * fdH.d);
    const float g = dy[i];
    gsum += (double)g;
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
  for (int t = 0; t < HEAD_CG * 9; ++t) {
    const float v = wave_sum(acc[t]);
    if (lane == 0) s_red[wv][t] = v;
  }
  {
    const double v = wave_sum_d(gsum);
    if (lane == 0) s_dred[wv] = v;
  }
  __syncthreads();
  float* dst = part + (long)blockIdx.x * (Cin * 9 + 1);
  for (int t = threadIdx.x; t < ncg * 9; t += 256)
    dst[c0 * 9 + t] = (s_red[0][t] + s_red[1][t]) + (s_red[2][t] + s_red[3][t]);
  if (blockIdx.y == 0 && threadIdx.x == 0)
    dst[Cin * 9] = (float)((s_dred[0] + s_dred[1]) + (s_dred[2] + s_dred[3]));
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


// ---------------------------------------------------------------------------------------------
// Column-strip kernels for the wide heads (W >= 64): lane = one image column of a 64-column
// segment, walking R consecutive rows with the three input rows of the 3x3 window held in
// registers, so each input value is loaded once per column offset (3 loads per pixel and channel
// instead of 9).  A unit = (image, row band, column segment).
// ---------------------------------------------------------------------------------------------
struct StripGeo {
  int H, W, nseg, nband;
};

__device__ __forceinline__ void strip_unit(const StripGeo& g, int u, int R, int& b, int& y0, int& xx) {
  const int seg = u % g.nseg;
  u /= g.nseg;
  const int band = u % g.nband;
  b = u / g.nband;
  y0 = band * R;
  xx = seg * 64 + (threadIdx.x & 63);
}

// one input row (reflect / zero padded) at the three column offsets of this lane
template <bool RFL>
__device__ __forceinline__ void strip_row(const float* __restrict__ xc, int yy, int H, int W,
                                          const int (&co)[3], const bool (&cv)[3], float (&v)[3]) {
  int sy = src_of<RFL>(yy, 1, H);
  const bool rv = sy >= 0;
  sy = min(max(sy, 0), H - 1);   // rows past the band end (never stored) stay in bounds
#pragma unroll
  for (int k = 0; k < 3; ++k) v[k] = (RFL || (rv && cv[k])) ? xc[sy * W + co[k]] : 0.f;
}

template <bool RFL>
__device__ __forceinline__ void strip_cols(int xx, int W, int (&co)[3], bool (&cv)[3]) {
  const int xc = min(xx, W - 1);
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const int sx = src_of<RFL>(xc, k, W);
    cv[k] = sx >= 0;
    co[k] = min(max(sx, 0), W - 1);
  }
}

// forward: the block's 4 waves split the channels; partial columns summed in wave order (LDS)
template <bool RFL, int R>
__global__ __launch_bounds__(256) void head_fwd_strip_kernel(HeadIn x, HeadW w, int Cin, StripGeo g,
                                                             const float* __restrict__ bias, int act,
                                                             float* __restrict__ y, long ybs,
                                                             int accumulate) {
  __shared__ float s_part[3][R][64];
  const int lane = threadIdx.x & 63, wq = threadIdx.x >> 6;
  int b, y0, xx;
  strip_unit(g, blockIdx.x, R, b, y0, xx);
  int co[3];
  bool cv[3];
  strip_cols<RFL>(xx, g.W, co, cv);
  const long HW = (long)g.H * g.W;
  const float* xb = x.p + img_off(x, b);
  const int cpw = (Cin + 3) >> 2;
  const int cb = wq * cpw, ce = min(Cin, cb + cpw);
  float out[R];
#pragma unroll
  for (int r = 0; r < R; ++r) out[r] = 0.f;
  for (int c = cb; c < ce; ++c) {
    const float* xc = xb + c * HW;
    float wt[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) wt[t] = w.p[(long)c * w.sc + (long)t * w.st];
    float a0[3], a1[3], a2[3];
    strip_row<RFL>(xc, y0 - 1, g.H, g.W, co, cv, a0);
    strip_row<RFL>(xc, y0, g.H, g.W, co, cv, a1);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      strip_row<RFL>(xc, y0 + r + 1, g.H, g.W, co, cv, a2);
      float v = out[r];
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        v = fmaf(wt[k], a0[k], v);
        v = fmaf(wt[3 + k], a1[k], v);
        v = fmaf(wt[6 + k], a2[k], v);
      }
      out[r] = v;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        a0[k] = a1[k];
        a1[k] = a2[k];
      }
    }
  }
  if (wq > 0) {
#pragma unroll
    for (int r = 0; r < R; ++r) s_part[wq - 1][r][lane] = out[r];
  }
  __syncthreads();
  if (wq > 0 || xx >= g.W) return;
  const float bb = bias ? bias[0] : 0.f;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if (y0 + r >= g.H) break;
    float v = ((out[r] + s_part[0][r][lane]) + s_part[1][r][lane]) + s_part[2][r][lane];
    v = act_f(v + bb, act);
    float* dst = y + (long)b * ybs + (long)(y0 + r) * g.W + xx;
    *dst = accumulate ? *dst + v : v;
  }
}

// filter gradient partials: wave wq of channel block blockIdx.y owns CPW channels; per unit a row
// [Cin*9 + 1] of partials (the last column = sum of dy, the bias gradient)
template <bool RFL, int R, int CPW>
__global__ __launch_bounds__(256) void head_wgrad_strip_kernel(HeadIn x, const float* __restrict__ dy,
                                                               int Cin, StripGeo g,
                                                               float* __restrict__ part) {
  const int lane = threadIdx.x & 63, wq = threadIdx.x >> 6;
  int b, y0, xx;
  strip_unit(g, blockIdx.x, R, b, y0, xx);
  int co[3];
  bool cv[3];
  strip_cols<RFL>(xx, g.W, co, cv);
  const bool live = xx < g.W;
  const long HW = (long)g.H * g.W;
  float gr[R];
  double gs = 0.0;   // bias gradient in fp64: a long cancelling sum
#pragma unroll
  for (int r = 0; r < R; ++r) {
    gr[r] = (live && y0 + r < g.H) ? dy[(long)b * HW + (long)(y0 + r) * g.W + xx] : 0.f;
    gs += (double)gr[r];
  }
  const int c0 = (blockIdx.y * 4 + wq) * CPW;
  const float* xb = x.p + img_off(x, b);
  float acc[CPW][9];
#pragma unroll
  for (int i = 0; i < CPW; ++i)
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[i][t] = 0.f;
#pragma unroll
  for (int i = 0; i < CPW; ++i) {
    if (c0 + i < Cin) {
      const float* xc = xb + (c0 + i) * HW;
      float a0[3], a1[3], a2[3];
      strip_row<RFL>(xc, y0 - 1, g.H, g.W, co, cv, a0);
      strip_row<RFL>(xc, y0, g.H, g.W, co, cv, a1);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        strip_row<RFL>(xc, y0 + r + 1, g.H, g.W, co, cv, a2);
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          acc[i][k] = fmaf(gr[r], a0[k], acc[i][k]);
          acc[i][3 + k] = fmaf(gr[r], a1[k], acc[i][3 + k]);
          acc[i][6 + k] = fmaf(gr[r], a2[k], acc[i][6 + k]);
        }
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          a0[k] = a1[k];
          a1[k] = a2[k];
        }
      }
    }
  }
  float* dst = part + (long)blockIdx.x * (Cin * 9 + 1);
#pragma unroll
  for (int i = 0; i < CPW; ++i)
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const float v = wave_sum(acc[i][t]);
      if (lane == 0 && c0 + i < Cin) dst[(c0 + i) * 9 + t] = v;
    }
  if (blockIdx.y == 0 && wq == 0) {
    const double v = wave_sum_d(gs);
    if (lane == 0) dst[Cin * 9] = (float)v;
  }
}

// data gradient: one unit per WAVE, all channels per lane.  E(yy) = the dy row yy at the three
// column taps with the reflect folds (q = 1 also takes p = 0 through tap 0, q = W-2 takes p = W-1
// through tap 2); D = rows E(qy+1), E(qy), E(qy-1) with the same folds in y; dx[c] = w[c] . D.
template <bool RFL>
__device__ __forceinline__ void strip_erow(const float* __restrict__ g, int yy, int H, int W, int qx,
                                           float (&e)[3]) {
  const bool rv = yy >= 0 && yy < H;
  const int sy = min(max(yy, 0), H - 1);
  const float* row = g + (long)sy * W;
  const int xq = min(qx, W - 1);
  e[0] = (rv && xq + 1 < W) ? row[xq + 1] : 0.f;
  e[1] = rv ? row[xq] : 0.f;
  e[2] = (rv && xq >= 1) ? row[xq - 1] : 0.f;
  if (RFL) {
    if (xq == 1 && rv) e[0] += row[0];
    if (xq == W - 2 && rv) e[2] += row[W - 1];
  }
}

template <bool RFL, int R>
__global__ __launch_bounds__(256) void head_dgrad_strip_kernel(const float* __restrict__ dy, HeadW w,
                                                               int Cin, StripGeo g, int nunits,
                                                               float* __restrict__ dx, long dxbs,
                                                               int accumulate) {
  const int u = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (u >= nunits) return;
  int b, y0, qx;
  strip_unit(g, u, R, b, y0, qx);
  const long HW = (long)g.H * g.W;
  const float* gb = dy + (long)b * HW;
  float D[R][9];
  float e0[3], e1[3], e2[3];   // E(y+1), E(y), E(y-1) of the current row y
  strip_erow<RFL>(gb, y0 + 1, g.H, g.W, qx, e0);
  strip_erow<RFL>(gb, y0, g.H, g.W, qx, e1);
  strip_erow<RFL>(gb, y0 - 1, g.H, g.W, qx, e2);
  float ef0[3] = {0.f, 0.f, 0.f}, efH[3] = {0.f, 0.f, 0.f};
  if (RFL) {
    if (y0 <= 1 && 1 < y0 + R) strip_erow<RFL>(gb, 0, g.H, g.W, qx, ef0);
    if (y0 <= g.H - 2 && g.H - 2 < y0 + R) strip_erow<RFL>(gb, g.H - 1, g.H, g.W, qx, efH);
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int qy = y0 + r;
    const bool f0 = RFL && qy == 1, fH = RFL && qy == g.H - 2;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      D[r][k] = e0[k] + (f0 ? ef0[k] : 0.f);
      D[r][3 + k] = e1[k];
      D[r][6 + k] = e2[k] + (fH ? efH[k] : 0.f);
    }
    if (r + 1 < R) {
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        e2[k] = e1[k];
        e1[k] = e0[k];
      }
      strip_erow<RFL>(gb, qy + 2, g.H, g.W, qx, e0);
    }
  }
  if (qx >= g.W) return;
  float* out = dx + (long)b * dxbs + (long)y0 * g.W + qx;
  const int cpg = (Cin + gridDim.y - 1) / gridDim.y;
  const int cb = blockIdx.y * cpg, ce = min(Cin, cb + cpg);
  for (int c = cb; c < ce; ++c) {
    float wt[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) wt[t] = w.p[(long)c * w.sc + (long)t * w.st];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (y0 + r >= g.H) break;
      float v = 0.f;
#pragma unroll
      for (int t = 0; t < 9; ++t) v = fmaf(wt[t], D[r][t], v);
      float* d = out + c * HW + (long)r * g.W;
      *d = accumulate ? *d + v : v;
    }
  }
}

StripGeo strip_geo(const ConvShape& s, int R) {
  StripGeo g;
  g.H = s.H;
  g.W = s.W;
  g.nseg = cdiv(s.W, 64);
  g.nband = cdiv(s.H, R);
  return g;
}
long strip_units(const ConvShape& s, int R) { return (long)s.N * cdiv(s.H, R) * cdiv(s.W, 64); }

// strip path for the wide heads; MD2_HEAD_STRIP=0 keeps the pixel-per-lane kernels
bool strip_ok(const ConvShape& s) {
  static const int on = tuning_knob("MD2_HEAD_STRIP", 1);
  return on && s.W >= 64 && s.H >= 4;
}
// forward / filter gradient strips only where they give enough blocks (measured: head5, head4;
// the head3 grid of 96-192 blocks ran slower than the pixel-per-lane kernels)
bool strip_fw_ok(const ConvShape& s) { return strip_ok(s) && (long)s.N * s.H * s.W >= 131072; }
// rows per lane: 16 when that still gives >= 512 units, else 8
int strip_rows(const ConvShape& s) { return strip_units(s, 16) >= 512 ? 16 : 8; }
// wgrad channels per wave (8 for Cin >= 32) and channel blocks
int strip_cpw(int Cin) { return Cin >= 32 ? 8 : 4; }

// ---------------------------------------------------------------------------------------------
// Batched heads (all disparity heads of the DepthDecoder in one launch per pass).  Every head is
// an HBM pass over its Cin input planes (9*Cin MACs per pixel), so the kernels are shaped for
// bytes: a lane owns V = 4 (2 when W % 4 != 0) consecutive pixels of one row and moves them as
// ONE float4 (float2) load / store; the +-1 column neighbours come from the adjacent lanes by DPP.
// A wave covers 62 consecutive pixel vectors of the flattened [image][row][vector] index space:
// lanes 0 and 63 are halo loaders only (their vectors belong to the neighbouring tiles), so the
// DPP neighbour of every owning lane is always loaded, with no divergent edge loads.  Where a
// row starts or ends inside the wave the column taps fold by reflection (pad_reflect excludes the
// edge, src/depth_decoder.jl:5) from the lane's own vector.
//   forward   block = one 62-vector tile; wave q of the block sums channel quarter q; the four
//             partial sums are added in wave order through LDS, then bias + sigmoid.
//   backward  ONE pass per (head, 4-channel chunk, run of T tiles) wave item: the 9 tap-shifted
//             dy values D of each pixel (with the reflect folds) are formed once per tile, then
//             per channel dx = w . D is stored and the filter-gradient sums dy * x(window) are
//             accumulated; at the end of the run they are wave-summed into one partial row.
//             The bias gradient (sum of dy, a long cancelling sum) stays fp64.  A fixed-order
//             column reduction finishes dw / db.
// ---------------------------------------------------------------------------------------------
constexpr int HB_TILE = 62;   // owned pixel vectors per wave (lanes 1..62)
constexpr int HB_CH = 2;      // filter gradient: channels per wave item (4: 193 VGPRs)
constexpr int HB_DCH = 16;    // data gradient: channels per wave item

struct HeadBatch {
  HeadJob j[MAX_HEADS];
  int n, act;
  int V[MAX_HEADS];          // pixels per lane
  long ntile[MAX_HEADS];     // 62-vector tiles of the head
  long f0[MAX_HEADS + 1];    // forward: first block of each head
  int T[MAX_HEADS];          // backward: tiles per wave item
  int nrun[MAX_HEADS];       // backward: runs of T tiles
  long d0[MAX_HEADS + 1];    // data gradient: first wave item of each head
  long w0[MAX_HEADS + 1];    // filter gradient: first wave item of each head
  long c0[MAX_HEADS + 1];    // reduction: first column of each head
  long p0[MAX_HEADS];        // partial rows [nrun][Cin*9] (float offset)
  long q0[MAX_HEADS];        // fp64 bias partials [nrun] (double offset, after every float row)
};

__device__ __forceinline__ int hb_find(const long* off, int n, long b) {
  int k = 0;
  while (k + 1 < n && b >= off[k + 1]) ++k;
  return k;
}

template <int V> struct VecT;
template <> struct VecT<4> { using T = float4; };
template <> struct VecT<2> { using T = float2; };

template <int V>
__device__ __forceinline__ void vload(const float* p, float (&v)[V]) {
  const auto t = *reinterpret_cast<const typename VecT<V>::T*>(p);
  v[0] = t.x;
  v[1] = t.y;
  if constexpr (V == 4) {
    v[2] = t.z;
    v[3] = t.w;
  }
}
template <int V>
__device__ __forceinline__ void vstore(float* p, const float (&v)[V]) {
  if constexpr (V == 4)
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  else
    *reinterpret_cast<float2*>(p) = make_float2(v[0], v[1]);
}

__device__ __forceinline__ float hb_from_left(float v) {    // lane i <- lane i-1
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x138, 0xf, 0xf, true));
}
__device__ __forceinline__ float hb_from_right(float v) {   // lane i <- lane i+1
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x130, 0xf, 0xf, true));
}

// The lane's pixel vector: tile t, lane -> flat vector g = 62 t + lane - 1 (clamped into range
// for the loads; `own` = a lane that owns a real vector)
struct HbPix {
  int b, y, cx;
  bool own;
};
template <int V>
__device__ __forceinline__ HbPix hb_pix(const HeadJob& J, long t, int lane) {
  const int Wv = J.W / V;
  const long nv = (long)J.N * J.H * Wv;
  long g = t * HB_TILE + lane - 1;
  HbPix p;
  p.own = lane >= 1 && lane <= HB_TILE && g >= 0 && g < nv;
  g = g < 0 ? 0 : (g >= nv ? nv - 1 : g);
  const long r = g / Wv;
  p.cx = (int)(g - r * Wv);
  p.b = (int)(r / J.H);
  p.y = (int)(r - (long)p.b * J.H);
  return p;
}

// row `row` of plane xc around the lane's vector: a[0] = column 4cx-1, a[1..V] = the vector,
// a[V+1] = column 4cx+V, the outer two folded by reflection at the row ends (mirror excluding the
// edge: -1 -> 1, W -> W-2)
template <int V>
__device__ __forceinline__ void hb_row_reflect(const float* __restrict__ xc, int row, int W, int cx, int Wv,
                                               float (&a)[V + 2]) {
  float v[V];
  vload<V>(xc + (long)row * W + cx * V, v);
  const float l = hb_from_left(v[V - 1]), r = hb_from_right(v[0]);
#pragma unroll
  for (int i = 0; i < V; ++i) a[i + 1] = v[i];
  a[0] = cx == 0 ? v[1] : l;
  a[V + 1] = cx == Wv - 1 ? v[V - 2] : r;
}
// the same with zero padding outside the row and a zero row outside the image (dy)
template <int V>
__device__ __forceinline__ void hb_row_zero(const float* __restrict__ g, int row, int H, int W, int cx, int Wv,
                                            float (&a)[V + 2]) {
  float v[V];
  const bool in = row >= 0 && row < H;
  vload<V>(g + (long)(in ? row : 0) * W + cx * V, v);
#pragma unroll
  for (int i = 0; i < V; ++i) v[i] = in ? v[i] : 0.f;
  const float l = hb_from_left(v[V - 1]), r = hb_from_right(v[0]);
#pragma unroll
  for (int i = 0; i < V; ++i) a[i + 1] = v[i];
  a[0] = cx == 0 ? 0.f : l;
  a[V + 1] = cx == Wv - 1 ? 0.f : r;
}

__device__ __forceinline__ int hb_reflect(int i, int n) {
  i = i < 0 ? -i : i;
  return i >= n ? 2 * n - 2 - i : i;
}

template <int V>
__device__ void heads_fwd_body(const HeadBatch& hb, const HeadJob& J, long t, float (*s_part)[64][4]) {
  const int lane = threadIdx.x & 63, wq = threadIdx.x >> 6;
  const HbPix p = hb_pix<V>(J, t, lane);
  const int Wv = J.W / V;
  const long HW = (long)J.H * J.W;
  const int ym = hb_reflect(p.y - 1, J.H), yp = hb_reflect(p.y + 1, J.H);
  const float* xb = J.x.p + img_off(J.x, p.b);
  const int cpw = (J.Cin + 3) >> 2;
  const int cb = wq * cpw, ce = min(J.Cin, cb + cpw);
  float out[V];
#pragma unroll
  for (int i = 0; i < V; ++i) out[i] = 0.f;
#pragma unroll 2
  for (int c = cb; c < ce; ++c) {
    const float* xc = xb + c * HW;
    float wt[9];
#pragma unroll
    for (int q = 0; q < 9; ++q) wt[q] = J.wf.p[(long)c * J.wf.sc + (long)q * J.wf.st];
    float a0[V + 2], a1[V + 2], a2[V + 2];
    hb_row_reflect<V>(xc, ym, J.W, p.cx, Wv, a0);
    hb_row_reflect<V>(xc, p.y, J.W, p.cx, Wv, a1);
    hb_row_reflect<V>(xc, yp, J.W, p.cx, Wv, a2);
#pragma unroll
    for (int i = 0; i < V; ++i) {
      float v = out[i];
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        v = fmaf(wt[q], a0[i + q], v);
        v = fmaf(wt[3 + q], a1[i + q], v);
        v = fmaf(wt[6 + q], a2[i + q], v);
      }
      out[i] = v;
    }
  }
  if (wq > 0) {
#pragma unroll
    for (int i = 0; i < V; ++i) s_part[wq - 1][lane][i] = out[i];
  }
  __syncthreads();
  if (wq > 0 || !p.own) return;
  const float bb = J.bias ? J.bias[0] : 0.f;
  float y[V];
#pragma unroll
  for (int i = 0; i < V; ++i)
    y[i] = act_f(((out[i] + s_part[0][lane][i]) + s_part[1][lane][i]) + s_part[2][lane][i] + bb, hb.act);
  vstore<V>(J.y + (long)p.b * J.ybs + (long)p.y * J.W + p.cx * V, y);
}

__global__ __launch_bounds__(256) void heads_fwd_kernel(HeadBatch hb) {
  __shared__ float s_part[3][64][4];
  const int k = hb_find(hb.f0, hb.n, blockIdx.x);
  const long t = blockIdx.x - hb.f0[k];
  if (hb.V[k] == 4)
    heads_fwd_body<4>(hb, hb.j[k], t, s_part);
  else
    heads_fwd_body<2>(hb, hb.j[k], t, s_part);
}

// E(row) of the data gradient for pixel i at the three column taps kx (p.x = q.x + 1 - kx), from
// the zero-padded row a (a[i+1] = column of pixel i), with the reflect folds in x: q = 1 also
// takes p = 0 through kx = 0, q = W-2 takes p = W-1 through kx = 2
template <int V>
__device__ __forceinline__ void hb_erow(const float (&a)[V + 2], int cx, int Wv, float (&e)[3][V]) {
#pragma unroll
  for (int i = 0; i < V; ++i) {
    e[0][i] = a[i + 2];
    e[1][i] = a[i + 1];
    e[2][i] = a[i];
  }
  if (cx == 0) e[0][1] += a[1];
  if (cx == Wv - 1) e[2][V - 2] += a[V];
}

// data gradient item: one 62-vector tile x HB_DCH channels.  D[ky][kx][i] = dy(q.y + 1 - ky,
// q.x + 1 - kx) with the folds: q.y = 1 also takes p.y = 0 through ky = 0, q.y = H-2 takes
// p.y = H-1 through ky = 2; then dx[c] = sum_tap w_d[c][tap] D[tap] for each channel.
template <int V>
__device__ void heads_dgrad_body(const HeadBatch& hb, int k, long item) {
  const HeadJob& J = hb.j[k];
  const int lane = threadIdx.x & 63;
  const int nch = (J.Cin + HB_DCH - 1) / HB_DCH;
  const int ch = (int)(item % nch);
  const long t = item / nch;
  const int Wv = J.W / V;
  const long HW = (long)J.H * J.W;
  const HbPix p = hb_pix<V>(J, t, lane);
  const float* gb = J.dy + (long)p.b * HW;
  float dm[V + 2], d0[V + 2], dp[V + 2];
  hb_row_zero<V>(gb, p.y - 1, J.H, J.W, p.cx, Wv, dm);
  hb_row_zero<V>(gb, p.y, J.H, J.W, p.cx, Wv, d0);
  hb_row_zero<V>(gb, p.y + 1, J.H, J.W, p.cx, Wv, dp);
  float D[3][3][V], Em[3][V];
  hb_erow<V>(dp, p.cx, Wv, D[0]);
  hb_erow<V>(d0, p.cx, Wv, D[1]);
  hb_erow<V>(dm, p.cx, Wv, Em);
  const bool f0 = p.y == 1, fH = p.y == J.H - 2;
#pragma unroll
  for (int q = 0; q < 3; ++q)
#pragma unroll
    for (int i = 0; i < V; ++i) {
      D[2][q][i] = Em[q][i] + (fH ? D[0][q][i] : 0.f);
      D[0][q][i] += f0 ? Em[q][i] : 0.f;
    }
  if (!p.own) return;
  float* dxb = J.dx + (long)p.b * J.dxbs + (long)p.y * J.W + p.cx * V;
  const int cb = ch * HB_DCH, ce = min(J.Cin, cb + HB_DCH);
#pragma unroll 4
  for (int c = cb; c < ce; ++c) {
    float wd[9];
#pragma unroll
    for (int q = 0; q < 9; ++q) wd[q] = J.wd.p[(long)c * J.wd.sc + (long)q * J.wd.st];
    float dx[V];
#pragma unroll
    for (int i = 0; i < V; ++i) {
      float v = 0.f;
#pragma unroll
      for (int q = 0; q < 9; ++q) v = fmaf(wd[q], D[q / 3][q % 3][i], v);
      dx[i] = v;
    }
    vstore<V>(dxb + c * HW, dx);
  }
}

// filter gradient item: HB_CH channels x a run of T tiles: sum_p dy[p] x[src(p, tap)] per
// (channel, tap) in lane registers, wave-summed once at the end of the run into partial row
// `run`; the 4-channel chunk 0 also sums dy (the bias gradient) in fp64.
template <int V>
__device__ void heads_wgrad_body(const HeadBatch& hb, int k, long item, float* __restrict__ part) {
  const HeadJob& J = hb.j[k];
  const int lane = threadIdx.x & 63;
  const int nch = (J.Cin + HB_CH - 1) / HB_CH;
  const int ch = (int)(item % nch);
  const int run = (int)(item / nch);
  const long tb = (long)run * hb.T[k], te = min(hb.ntile[k], tb + hb.T[k]);
  const int Wv = J.W / V;
  const long HW = (long)J.H * J.W;
  const int c0 = ch * HB_CH;
  float acc[HB_CH][9];
#pragma unroll
  for (int c = 0; c < HB_CH; ++c)
#pragma unroll
    for (int q = 0; q < 9; ++q) acc[c][q] = 0.f;
  double gs = 0.0;
  for (long t = tb; t < te; ++t) {
    const HbPix p = hb_pix<V>(J, t, lane);
    float g[V];
    vload<V>(J.dy + (long)p.b * HW + (long)p.y * J.W + p.cx * V, g);
#pragma unroll
    for (int i = 0; i < V; ++i) g[i] = p.own ? g[i] : 0.f;    // halo lanes add nothing
    if (ch == 0) {
#pragma unroll
      for (int i = 0; i < V; ++i) gs += (double)g[i];
    }
    const int ym = hb_reflect(p.y - 1, J.H), yp = hb_reflect(p.y + 1, J.H);
    const float* xb = J.x.p + img_off(J.x, p.b);
#pragma unroll
    for (int c = 0; c < HB_CH; ++c) {
      if (c0 + c >= J.Cin) break;
      const float* xc = xb + (c0 + c) * HW;
      float a0[V + 2], a1[V + 2], a2[V + 2];
      hb_row_reflect<V>(xc, ym, J.W, p.cx, Wv, a0);
      hb_row_reflect<V>(xc, p.y, J.W, p.cx, Wv, a1);
      hb_row_reflect<V>(xc, yp, J.W, p.cx, Wv, a2);
#pragma unroll
      for (int i = 0; i < V; ++i)
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          acc[c][q] = fmaf(g[i], a0[i + q], acc[c][q]);
          acc[c][3 + q] = fmaf(g[i], a1[i + q], acc[c][3 + q]);
          acc[c][6 + q] = fmaf(g[i], a2[i + q], acc[c][6 + q]);
        }
    }
  }
  float* dst = part + hb.p0[k] + (long)run * J.Cin * 9;
#pragma unroll
  for (int c = 0; c < HB_CH; ++c)
#pragma unroll
    for (int q = 0; q < 9; ++q) {
      const float v = wave_sum_dpp(acc[c][q]);
      if (lane == 0 && c0 + c < J.Cin) dst[(c0 + c) * 9 + q] = v;
    }
  if (ch == 0) {
    const double v = wave_sum_d(gs);
    if (lane == 0) reinterpret_cast<double*>(part)[hb.q0[k] + run] = v;
  }
}

// one launch, two wave ranges: [0, d0[n]) data-gradient items, then [d0[n], + w0[n]) filter-
// gradient items (both read dy; only the data gradient writes, only the filter gradient reads x)
__global__ __launch_bounds__(256) void heads_bwd_kernel(HeadBatch hb, float* __restrict__ part) {
  long w = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (w < hb.d0[hb.n]) {
    const int k = hb_find(hb.d0, hb.n, w);
    if (hb.V[k] == 4)
      heads_dgrad_body<4>(hb, k, w - hb.d0[k]);
    else
      heads_dgrad_body<2>(hb, k, w - hb.d0[k]);
    return;
  }
  w -= hb.d0[hb.n];
  if (w >= hb.w0[hb.n]) return;                                // wave-uniform
  const int k = hb_find(hb.w0, hb.n, w);
  if (hb.V[k] == 4)
    heads_wgrad_body<4>(hb, k, w - hb.w0[k], part);
  else
    heads_wgrad_body<2>(hb, k, w - hb.w0[k], part);
}

// one block per column of every head (Cin*9 weights + the bias), fixed-order sum over its runs
__global__ __launch_bounds__(256) void heads_wgrad_reduce_kernel(HeadBatch hb, const float* __restrict__ part) {
  __shared__ float s_red[4];
  __shared__ double s_dred[4];
  const int k = hb_find(hb.c0, hb.n, blockIdx.x);
  const HeadJob& J = hb.j[k];
  const int t = (int)(blockIdx.x - hb.c0[k]);
  const int ncol = J.Cin * 9;
  const long runs = hb.nrun[k];
  if (t == ncol) {                  // bias column: fp64 partials, fp64 sum
    const double* bsrc = reinterpret_cast<const double*>(part) + hb.q0[k];
    double d = 0.0;
    for (long q = threadIdx.x; q < runs; q += 256) d += bsrc[q];
    d = wave_sum_d(d);
    if ((threadIdx.x & 63) == 0) s_dred[threadIdx.x >> 6] = d;
    __syncthreads();
    if (threadIdx.x == 0 && J.db) J.db[0] = (float)((s_dred[0] + s_dred[1]) + (s_dred[2] + s_dred[3]));
    return;
  }
  const float* src = part + hb.p0[k] + t;
  float v = 0.f;
  for (long q = threadIdx.x; q < runs; q += 256) v += src[q * ncol];
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x != 0) return;
  J.dw[t] = (s_red[0] + s_red[1]) + (s_red[2] + s_red[3]);
}

// tiles per filter-gradient wave item: 8 (the 18 wave sums of a run amortised over 8 tiles x 2
// channels), 1 on tiny heads
int hb_tiles_per_item(long ntile) {
  static const int T = tuning_knob("MD2_HEAD_T", 8);
  return ntile >= 16L * T ? T : 1;
}

HeadBatch make_batch(const HeadJob* jobs, int n) {
  HeadBatch hb{};
  hb.n = n;
  long f = 0, d = 0, w = 0, c = 0, p = 0;
  for (int k = 0; k < n; ++k) {
    const HeadJob& j = jobs[k];
    hb.j[k] = j;
    hb.V[k] = j.W % 4 == 0 ? 4 : 2;
    const long nv = (long)j.N * j.H * (j.W / hb.V[k]);
    hb.ntile[k] = cdiv(nv, HB_TILE);
    hb.f0[k] = f;
    f += hb.ntile[k];
    hb.T[k] = hb_tiles_per_item(hb.ntile[k]);
    hb.nrun[k] = cdiv(hb.ntile[k], hb.T[k]);
    hb.d0[k] = d;
    d += hb.ntile[k] * cdiv(j.Cin, HB_DCH);
    hb.w0[k] = w;
    w += (long)hb.nrun[k] * cdiv(j.Cin, HB_CH);
    hb.c0[k] = c;
    c += (long)j.Cin * 9 + 1;
    hb.p0[k] = p;
    p += (long)hb.nrun[k] * j.Cin * 9;
  }
  hb.f0[n] = f;
  hb.d0[n] = d;
  hb.w0[n] = w;
  hb.c0[n] = c;
  long q = (p + 1) / 2;             // doubles start after the float rows (8-byte aligned)
  for (int k = 0; k < n; ++k) {
    hb.q0[k] = q;
    q += hb.nrun[k];
  }
  return hb;
}

long heads_parts_floats(const HeadJob* jobs, int n) {
  const HeadBatch hb = make_batch(jobs, n);
  long q = hb.q0[n - 1] + hb.nrun[n - 1];
  return 2 * q;
}

int check_jobs(const HeadJob* jobs, int n) {
  MD2_CHECK_ARG(jobs && n >= 1 && n <= MAX_HEADS, "heads: 1..5 heads");
  for (int k = 0; k < n; ++k) {
    const HeadJob& j = jobs[k];
    MD2_CHECK_ARG(j.Cin >= 1 && j.H >= 2 && j.W >= 4 && j.W % 2 == 0 && j.N >= 1 && j.x.p,
                  "heads: shape (W even, >= 4) / input");
    MD2_CHECK_ARG((long)j.N * j.H * j.W < (1L << 31) && (long)j.Cin * j.H * j.W < (1L << 31),
                  "heads: size");
    const int V = j.W % 4 == 0 ? 4 : 2;
    // vector loads / stores: every plane and image base V-float aligned
    MD2_CHECK_ARG(j.x.bs0 % V == 0 && j.x.bhi % V == 0 && j.dxbs % V == 0 && j.ybs % V == 0 &&
                      ((uintptr_t)j.x.p % (4 * V)) == 0,
                  "heads: vector alignment");
  }
  return MD2_OK;
}
}  // namespace

bool head_conv_ok(const ConvShape& s) {
  return s.Cout == 1 && s.KH == 3 && s.KW == 3 && s.stride == 1 && s.pad == 1 && s.H >= 2 &&
         s.W >= 2 && (long)s.N * s.H * s.W < (1L << 31);
}

size_t head_wgrad_workspace(const ConvShape& s) {
  long parts = head_parts((long)s.N * s.H * s.W, s.Cin);
  if (strip_fw_ok(s)) parts = std::max(parts, strip_units(s, strip_rows(s)));
  return (size_t)parts * (s.Cin * 9 + 1) * sizeof(float);
}

int head_fwd(const ConvShape& s, const HeadIn& x, HeadW w, const float* bias, int act, float* y,
             long ybs, int accumulate, hipStream_t st) {
  if (strip_fw_ok(s)) {
    const int R = strip_rows(s);
    const StripGeo g = strip_geo(s, R);
    const dim3 grid((unsigned)strip_units(s, R));
#define MD2_HF(RF, RR)                                                                             \
  hipLaunchKernelGGL((head_fwd_strip_kernel<RF, RR>), grid, dim3(256), 0, st, x, w, s.Cin, g, bias, \
                     act, y, ybs, accumulate)
    if (s.reflect) {
      if (R == 16) MD2_HF(true, 16); else MD2_HF(true, 8);
    } else {
      if (R == 16) MD2_HF(false, 16); else MD2_HF(false, 8);
    }
#undef MD2_HF
    MD2_LAUNCH_CHECK();
    return MD2_OK;
  }
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
  if (strip_ok(s)) {
    constexpr int R = 4;
    const StripGeo g = strip_geo(s, R);
    const long nu = strip_units(s, R);
    // channel groups (each re-forms D) until ~4096 waves, >= 4 channels per group
    const int G = (int)std::max<long>(1, std::min<long>(cdiv(4096, nu), s.Cin / 4));
    const dim3 grid((unsigned)cdiv(nu, 4), G);
    if (s.reflect)
      hipLaunchKernelGGL((head_dgrad_strip_kernel<true, R>), grid, dim3(256), 0, st, dy, w, s.Cin, g,
                         (int)nu, dx, dxbs, accumulate);
    else
      hipLaunchKernelGGL((head_dgrad_strip_kernel<false, R>), grid, dim3(256), 0, st, dy, w, s.Cin, g,
                         (int)nu, dx, dxbs, accumulate);
    MD2_LAUNCH_CHECK();
    return MD2_OK;
  }
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
  MD2_CHECK_ARG(ws && ws_bytes >= head_wgrad_workspace(s), "head_wgrad workspace");
  float* part = (float*)ws;
  const int ncols = s.Cin * 9;
  if (strip_fw_ok(s)) {
    const int R = strip_rows(s), cpw = strip_cpw(s.Cin);
    const StripGeo g = strip_geo(s, R);
    const long nu = strip_units(s, R);
    const dim3 grid((unsigned)nu, cdiv(s.Cin, 4 * cpw));
#define MD2_HW(RF, RR, CP)                                                                         \
  hipLaunchKernelGGL((head_wgrad_strip_kernel<RF, RR, CP>), grid, dim3(256), 0, st, x, dy, s.Cin, g, part)
    if (s.reflect) {
      if (R == 16) { if (cpw == 8) MD2_HW(true, 16, 8); else MD2_HW(true, 16, 4); }
      else { if (cpw == 8) MD2_HW(true, 8, 8); else MD2_HW(true, 8, 4); }
    } else {
      if (R == 16) { if (cpw == 8) MD2_HW(false, 16, 8); else MD2_HW(false, 16, 4); }
      else { if (cpw == 8) MD2_HW(false, 8, 8); else MD2_HW(false, 8, 4); }
    }
#undef MD2_HW
    MD2_LAUNCH_CHECK();
    hipLaunchKernelGGL(head_wgrad_reduce_kernel, dim3(ncols + 1), dim3(256), 0, st, part, (int)nu,
                       ncols, dw, db, accumulate);
    MD2_LAUNCH_CHECK();
    return MD2_OK;
  }
  const long np = (long)s.N * s.H * s.W;
  const int parts = head_parts(np, s.Cin);
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
  hipLaunchKernelGGL(head_wgrad_reduce_kernel, dim3(ncols + 1), dim3(256), 0, st, part, parts,
                     ncols, dw, db, accumulate);
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

int heads_fwd(const HeadJob* jobs, int n, int act, hipStream_t st) {
  MD2_TRY(check_jobs(jobs, n));
  for (int k = 0; k < n; ++k) MD2_CHECK_ARG(jobs[k].y && jobs[k].wf.p, "heads_fwd: output / weights");
  HeadBatch hb = make_batch(jobs, n);
  hb.act = act;
  hipLaunchKernelGGL(heads_fwd_kernel, dim3((unsigned)hb.f0[n]), dim3(256), 0, st, hb);
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

size_t heads_bwd_workspace(const HeadJob* jobs, int n) {
  return (size_t)heads_parts_floats(jobs, n) * sizeof(float);
}

int heads_bwd(const HeadJob* jobs, int n, void* ws, size_t ws_bytes, hipStream_t st) {
  MD2_TRY(check_jobs(jobs, n));
  for (int k = 0; k < n; ++k)
    MD2_CHECK_ARG(jobs[k].dy && jobs[k].dx && jobs[k].dw && jobs[k].wd.p, "heads_bwd: pointers");
  MD2_CHECK_ARG(ws && ws_bytes >= heads_bwd_workspace(jobs, n), "heads_bwd workspace");
  for (int k = 0; k < n; ++k)
    MD2_CHECK_ARG(((uintptr_t)jobs[k].dx % 16) == 0 && ((uintptr_t)jobs[k].dy % 16) == 0, "heads_bwd: alignment");
  const HeadBatch hb = make_batch(jobs, n);
  hipLaunchKernelGGL(heads_bwd_kernel, dim3((unsigned)cdiv(hb.d0[n] + hb.w0[n], 4)), dim3(256), 0, st, hb,
                     (float*)ws);
  MD2_LAUNCH_CHECK();
  hipLaunchKernelGGL(heads_wgrad_reduce_kernel, dim3((unsigned)hb.c0[n]), dim3(256), 0, st, hb,
                     (const float*)ws);
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

}  // namespace md2
