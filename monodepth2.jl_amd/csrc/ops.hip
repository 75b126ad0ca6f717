// Op-level kernels of the loss primitives, at ChainRulesCore rrule granularity (gfx950):
//   identity-reprojection loss   src/training.jl:9-11   (automasking_loss, also used by the model)
//   SSIM fwd / pullback          src/utils.jl:17-43
//   Backproject fwd / pullback   src/utils.jl:45-69
//   Project fwd / pullback       src/utils.jl:71-103
//   grid_sample(:border) fwd / pullback   NNlib, called at src/training.jl:56
//   smooth_loss fwd / pullback   src/utils.jl:163-177
//   per-scale warp + photometric loss fwd / pullback   src/training.jl:43-62
// The train step itself runs the fused kernels of loss_kernels.hip; these entries let a host
// (the Julia shim, julia/MD2HIP.jl) differentiate the same ops one at a time.  Layouts are the
// Julia column-major arrays read as C-order (see include/md2.h).
#include "loss_kernels.h"

namespace md2 {

namespace {

__device__ __forceinline__ int refl(int i, int n) { return i < 0 ? -i : (i >= n ? 2 * n - 2 - i : i); }

// Tile of TW x TH output pixels per 256-thread block; LDS planes hold the HALO-wide region.
constexpr int OT_W = 32, OT_H = 8;

// SSIM of one window from the 9 reflect-mapped LDS samples of x and y, shifted by the centre
// values (exact algebra; better fp32 conditioning than E[x^2] - E[x]^2).  Returns the unclamped
// value and the window statistics for the pullback.
struct SsimWin {
  float mx, my, vx, vy, cxy, num, den, val;
};
__device__ __forceinline__ SsimWin ssim_window(const float* xs, const float* ys, const int* wi, int ci) {
  const float xc = xs[ci], yc = ys[ci];
  float sx = 0.f, sy = 0.f, sxx = 0.f, syy = 0.f, sxy = 0.f;
#pragma unroll
  for (int q = 0; q < 9; ++q) {
    const float dx = xs[wi[q]] - xc, dy = ys[wi[q]] - yc;
    sx += dx;
    sy += dy;
    sxx += dx * dx;
    syy += dy * dy;
    sxy += dx * dy;
  }
  const float ninth = 1.f / 9.f;
  const float ex = sx * ninth, ey = sy * ninth;
  SsimWin w;
  w.mx = xc + ex;
  w.my = yc + ey;
  w.vx = sxx * ninth - ex * ex;
  w.vy = syy * ninth - ey * ey;
  w.cxy = sxy * ninth - ex * ey;
  const float c1 = 1e-4f, c2 = 9e-4f;
  w.num = (2.f * w.mx * w.my + c1) * (2.f * w.cxy + c2);
  w.den = (w.mx * w.mx + w.my * w.my + c1) * (w.vx + w.vy + c2);
  w.val = (1.f - w.num / w.den) * 0.5f;
  return w;
}

// Load the (OT_W + 2h) x (OT_H + 2h) region of a plane (global coordinates clamped: values at
// out-of-image positions are never read through the reflect map).
template <int HALO>
__device__ __forceinline__ void load_region(const float* __restrict__ src, int W, int H, int x0,
                                            int y0, float* dst) {
  constexpr int RW = OT_W + 2 * HALO, RH = OT_H + 2 * HALO;
  for (int i = threadIdx.x; i < RW * RH; i += 256) {
    const int rx = i % RW, ry = i / RW;
    const int gx = min(max(x0 - HALO + rx, 0), W - 1), gy = min(max(y0 - HALO + ry, 0), H - 1);
    dst[i] = src[(long)gy * W + gx];
  }
}

// LDS indices of the 9 reflect-mapped window samples of global pixel (gx, gy) in a region with
// origin (x0 - HALO, y0 - HALO).
template <int HALO>
__device__ __forceinline__ void window_idx(int gx, int gy, int W, int H, int x0, int y0, int* wi) {
  constexpr int RW = OT_W + 2 * HALO;
#pragma unroll
  for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
    for (int dx = -1; dx <= 1; ++dx)
      wi[(dy + 1) * 3 + dx + 1] = (refl(gy + dy, H) - (y0 - HALO)) * RW + (refl(gx + dx, W) - (x0 - HALO));
}

// ---------------------------------------------------------------------------------------------
// automasking_loss: min over sources of 0.85 mean_c SSIM(src, tgt) + 0.15 mean_c |tgt - src|
// ---------------------------------------------------------------------------------------------
// N0f8 pixels -> Float32 (the data pipeline's `Float32.(channelview(x))`, src/dtk.jl:45,
// src/kitty.jl:58): one byte in, Float32(u) / 255f0 out, 16 bytes per lane per trip.
__global__ __launch_bounds__(256) void unorm8_kernel(const uint8_t* __restrict__ in, long n,
                                                     float* __restrict__ out) {
  const long stride = (long)gridDim.x * 256 * 4;
  for (long i = ((long)blockIdx.x * 256 + threadIdx.x) * 4; i < n; i += stride) {
    if (i + 4 <= n) {
      const uint32_t v = *reinterpret_cast<const uint32_t*>(in + i);
      float4 f;
      f.x = (float)(v & 0xff) / 255.f;
      f.y = (float)((v >> 8) & 0xff) / 255.f;
      f.z = (float)((v >> 16) & 0xff) / 255.f;
      f.w = (float)(v >> 24) / 255.f;
      *reinterpret_cast<float4*>(out + i) = f;
    } else {
      for (long k = i; k < n; ++k) out[k] = (float)in[k] / 255.f;
    }
  }
}

template <int C>
__global__ __launch_bounds__(256) void automask_kernel(const float* __restrict__ x, long x_ss,
                                                       long x_fs, int target, int src0, int src1,
                                                       int W, int H, float* __restrict__ out) {
  constexpr int RW = OT_W + 2, RH = OT_H + 2, NR = RW * RH;
  __shared__ float s_t[C][NR], s_s[2][C][NR];
  const int n = blockIdx.z, x0 = blockIdx.x * OT_W, y0 = blockIdx.y * OT_H;
  const long HW = (long)W * H;
  const float* xb = x + (long)n * x_ss;
#pragma unroll
  for (int c = 0; c < C; ++c) {
    load_region<1>(xb + target * x_fs + c * HW, W, H, x0, y0, s_t[c]);
    load_region<1>(xb + src0 * x_fs + c * HW, W, H, x0, y0, s_s[0][c]);
    load_region<1>(xb + src1 * x_fs + c * HW, W, H, x0, y0, s_s[1][c]);
  }
  __syncthreads();
  const int tx = threadIdx.x % OT_W, ty = threadIdx.x / OT_W;
  const int gx = x0 + tx, gy = y0 + ty;
  if (gx >= W || gy >= H) return;
  int wi[9];
  window_idx<1>(gx, gy, W, H, x0, y0, wi);
  const int ci = (ty + 1) * RW + tx + 1;
  float l[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    float ss = 0.f, l1 = 0.f;
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const SsimWin w = ssim_window(s_s[s][c], s_t[c], wi, ci);
      ss += fminf(fmaxf(w.val, 0.f), 1.f);
      l1 += fabsf(s_t[c][ci] - s_s[s][c][ci]);
    }
    l[s] = 0.85f * (ss / (float)C) + 0.15f * (l1 / (float)C);
  }
  out[((long)n * H + gy) * W + gx] = l[1] < l[0] ? l[1] : l[0];   // first argmin on ties
}

// ---------------------------------------------------------------------------------------------
// SSIM()(x, y) per channel plane, and its pullback to both arguments.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void ssim_fwd_kernel(const float* __restrict__ x,
                                                       const float* __restrict__ y, int W, int H,
                                                       float* __restrict__ out) {
  constexpr int RW = OT_W + 2, NR = RW * (OT_H + 2);
  __shared__ float s_x[NR], s_y[NR];
  const long plane = blockIdx.z, HW = (long)W * H;
  const int x0 = blockIdx.x * OT_W, y0 = blockIdx.y * OT_H;
  load_region<1>(x + plane * HW, W, H, x0, y0, s_x);
  load_region<1>(y + plane * HW, W, H, x0, y0, s_y);
  __syncthreads();
  const int tx = threadIdx.x % OT_W, ty = threadIdx.x / OT_W;
  const int gx = x0 + tx, gy = y0 + ty;
  if (gx >= W || gy >= H) return;
  int wi[9];
  window_idx<1>(gx, gy, W, H, x0, y0, wi);
  const SsimWin w = ssim_window(s_x, s_y, wi, (ty + 1) * RW + tx + 1);
  out[plane * HW + (long)gy * W + gx] = fminf(fmaxf(w.val, 0.f), 1.f);
}

// Pullback: per window centre p the partials of clamp((1 - n/d)/2) w.r.t. (mu_x, mu_y, var_x,
// var_y, cov_xy) (var_x and var_y share d/dB2), then per pixel q the adjoint of the reflect-padded
// 3x3 mean pool  dx_q = 1/9 sum_p m_pq [g_mx + 2 g_v (x_q - mu_x) + g_c (y_q - mu_y)]  (m_pq: how
// often q appears in p's reflect window), symmetrically for dy.
__global__ __launch_bounds__(256) void ssim_bwd_kernel(const float* __restrict__ x,
                                                       const float* __restrict__ y,
                                                       const float* __restrict__ dout, int W,
                                                       int H, float* __restrict__ dx,
                                                       float* __restrict__ dy) {
  constexpr int AW = OT_W + 4, NA = AW * (OT_H + 4);     // halo-2 samples
  constexpr int BW = OT_W + 2, NB = BW * (OT_H + 2);     // halo-1 window centres
  __shared__ float s_x[NA], s_y[NA];
  __shared__ float s_c[6][NB];                           // g_mx, g_my, g_v, g_c, mu_x, mu_y
  const long plane = blockIdx.z, HW = (long)W * H;
  const int x0 = blockIdx.x * OT_W, y0 = blockIdx.y * OT_H;
  load_region<2>(x + plane * HW, W, H, x0, y0, s_x);
  load_region<2>(y + plane * HW, W, H, x0, y0, s_y);
  __syncthreads();
  for (int i = threadIdx.x; i < NB; i += 256) {
    const int bx = i % BW, by = i / BW;
    const int gx = x0 - 1 + bx, gy = y0 - 1 + by;
    float c[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (gx >= 0 && gx < W && gy >= 0 && gy < H) {
      int wi[9];
      window_idx<2>(gx, gy, W, H, x0, y0, wi);
      const SsimWin w = ssim_window(s_x, s_y, wi, (by + 1) * AW + bx + 1);
      const float lv = (w.val >= 0.f && w.val <= 1.f) ? 1.f : 0.f;   // clamp pullback
      const float g = dout[plane * HW + (long)gy * W + gx] * lv * (1.f / 9.f);
      const float c1 = 1e-4f, c2 = 9e-4f;
      const float A1 = 2.f * w.mx * w.my + c1, A2 = 2.f * w.cxy + c2;
      const float B1 = w.mx * w.mx + w.my * w.my + c1, B2 = w.vx + w.vy + c2;
      const float dn = -0.5f / w.den * g, dd = 0.5f * w.num / (w.den * w.den) * g;
      c[0] = dn * 2.f * w.my * A2 + dd * 2.f * w.mx * B2;
      c[1] = dn * 2.f * w.mx * A2 + dd * 2.f * w.my * B2;
      c[2] = dd * B1;
      c[3] = dn * 2.f * A1;
      c[4] = w.mx;
      c[5] = w.my;
    }
#pragma unroll
    for (int k = 0; k < 6; ++k) s_c[k][i] = c[k];
  }
  __syncthreads();
  const int tx = threadIdx.x % OT_W, ty = threadIdx.x / OT_W;
  const int gx = x0 + tx, gy = y0 + ty;
  if (gx >= W || gy >= H) return;
  const int ai = (ty + 2) * AW + tx + 2;
  const float xq = s_x[ai], yq = s_y[ai];
  float gxs = 0.f, gys = 0.f;
#pragma unroll
  for (int oy = -1; oy <= 1; ++oy) {
    const int py = gy + oy;
    if (py < 0 || py >= H) continue;
    const float wy = 1.f + ((gy == 1 && py == 0) ? 1.f : 0.f) + ((gy == H - 2 && py == H - 1) ? 1.f : 0.f);
#pragma unroll
    for (int ox = -1; ox <= 1; ++ox) {
      const int px = gx + ox;
      if (px < 0 || px >= W) continue;
      const float wx = 1.f + ((gx == 1 && px == 0) ? 1.f : 0.f) + ((gx == W - 2 && px == W - 1) ? 1.f : 0.f);
      const int bi = (py - (y0 - 1)) * BW + (px - (x0 - 1));
      const float m = wx * wy;
      gxs += m * (s_c[0][bi] + 2.f * s_c[2][bi] * (xq - s_c[4][bi]) + s_c[3][bi] * (yq - s_c[5][bi]));
      gys += m * (s_c[1][bi] + 2.f * s_c[2][bi] * (yq - s_c[5][bi]) + s_c[3][bi] * (xq - s_c[4][bi]));
    }
  }
  if (dx) dx[plane * HW + (long)gy * W + gx] = gxs;
  if (dy) dy[plane * HW + (long)gy * W + gx] = gys;
}

// ---------------------------------------------------------------------------------------------
// Backproject (src/utils.jl:67-69): out[n][p][k] = depth[n][p] * (invK [w, h, 1])_k, 1-based grid
// ---------------------------------------------------------------------------------------------
struct Mat3 {
  float m[9];   // row-major
};

__global__ __launch_bounds__(256) void backproject_fwd_kernel(const float* __restrict__ depth,
                                                              int W, long P, long total, Mat3 iK,
                                                              float* __restrict__ out) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int p = (int)(i % P);
  const float w = (float)(p % W + 1), h = (float)(p / W + 1);
  const float d = depth[i];
#pragma unroll
  for (int k = 0; k < 3; ++k) out[i * 3 + k] = d * (iK.m[3 * k] * w + iK.m[3 * k + 1] * h + iK.m[3 * k + 2]);
}

__global__ __launch_bounds__(256) void backproject_bwd_kernel(const float* __restrict__ dout,
                                                              int W, long P, long total, Mat3 iK,
                                                              float* __restrict__ d_depth) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int p = (int)(i % P);
  const float w = (float)(p % W + 1), h = (float)(p / W + 1);
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < 3; ++k) s += dout[i * 3 + k] * (iK.m[3 * k] * w + iK.m[3 * k + 1] * h + iK.m[3 * k + 2]);
  d_depth[i] = s;
}

// ---------------------------------------------------------------------------------------------
// Project (src/utils.jl:99-103): cam = K (R X + t); uv = cam[1:2] / (cam[3] + 1e-7);
// normalize: ((uv - 1) / (W-1, H-1) - 0.5) * 2.   points [n][P][3], R [n][9] row-major, t [n][3],
// out [n][P][2].  Pullback to the points and (per-sample deterministic block partials) R, t.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void project_fwd_kernel(const float* __restrict__ pts, long P,
                                                          Mat3 K, const float* __restrict__ R,
                                                          const float* __restrict__ t, float wm1,
                                                          float hm1, float* __restrict__ out) {
  const int n = blockIdx.y;
  const long p = (long)blockIdx.x * 256 + threadIdx.x;
  if (p >= P) return;
  const float* X = pts + ((long)n * P + p) * 3;
  const float* Rn = R + n * 9;
  float Q[3], cam[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) Q[i] = Rn[3 * i] * X[0] + Rn[3 * i + 1] * X[1] + Rn[3 * i + 2] * X[2] + t[n * 3 + i];
#pragma unroll
  for (int i = 0; i < 3; ++i) cam[i] = K.m[3 * i] * Q[0] + K.m[3 * i + 1] * Q[1] + K.m[3 * i + 2] * Q[2];
  const float denom = 1.f / (cam[2] + 1e-7f);
  float* o = out + ((long)n * P + p) * 2;
  o[0] = (((cam[0] * denom - 1.f) / wm1) - 0.5f) * 2.f;
  o[1] = (((cam[1] * denom - 1.f) / hm1) - 0.5f) * 2.f;
}

__global__ __launch_bounds__(256) void project_bwd_kernel(const float* __restrict__ pts, long P,
                                                          Mat3 K, const float* __restrict__ R,
                                                          const float* __restrict__ t, float wm1,
                                                          float hm1, const float* __restrict__ dout,
                                                          float* __restrict__ d_pts,
                                                          float* __restrict__ partials) {
  __shared__ float red[4 * 12];
  const int n = blockIdx.y;
  const long p = (long)blockIdx.x * 256 + threadIdx.x;
  float acc[12];
#pragma unroll
  for (int k = 0; k < 12; ++k) acc[k] = 0.f;
  if (p < P) {
    const float* X = pts + ((long)n * P + p) * 3;
    const float* Rn = R + n * 9;
    float Q[3], cam[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) Q[i] = Rn[3 * i] * X[0] + Rn[3 * i + 1] * X[1] + Rn[3 * i + 2] * X[2] + t[n * 3 + i];
#pragma unroll
    for (int i = 0; i < 3; ++i) cam[i] = K.m[3 * i] * Q[0] + K.m[3 * i + 1] * Q[1] + K.m[3 * i + 2] * Q[2];
    const float denom = 1.f / (cam[2] + 1e-7f);
    const float* g = dout + ((long)n * P + p) * 2;
    const float du = g[0] * 2.f / wm1, dv = g[1] * 2.f / hm1;     // d/d(cam_xy * denom)
    const float dcam[3] = {du * denom, dv * denom, -(du * cam[0] + dv * cam[1]) * denom * denom};
    float dQ[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) dQ[j] = K.m[j] * dcam[0] + K.m[3 + j] * dcam[1] + K.m[6 + j] * dcam[2];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
#pragma unroll
      for (int j = 0; j < 3; ++j) acc[3 * i + j] = dQ[i] * X[j];
      acc[9 + i] = dQ[i];
    }
    float* dX = d_pts + ((long)n * P + p) * 3;
#pragma unroll
    for (int j = 0; j < 3; ++j) dX[j] = Rn[j] * dQ[0] + Rn[3 + j] * dQ[1] + Rn[6 + j] * dQ[2];
  }
  block_sum256<12>(acc, red);
  if (threadIdx.x == 0) {
    float* o = partials + ((long)n * gridDim.x + blockIdx.x) * 12;
#pragma unroll
    for (int k = 0; k < 12; ++k) o[k] = acc[k];
  }
}

// out[n][k] = sum_b part[n][b][k] for k < K (fixed order: deterministic)
__global__ __launch_bounds__(256) void reduce_partials_kernel(const float* __restrict__ part, int nb,
                                                              int K, int stride,
                                                              float* __restrict__ out,
                                                              float* __restrict__ out2, int split) {
  __shared__ float red[4];
  const int n = blockIdx.y, k = blockIdx.x;
  float s = 0.f;
  for (int b = threadIdx.x; b < nb; b += 256) s += part[((long)n * nb + b) * stride + k];
  float v[1] = {s};
  block_sum256<1>(v, red);
  if (threadIdx.x == 0) {
    if (k < split)
      out[n * split + k] = v[0];
    else
      out2[n * (K - split) + (k - split)] = v[0];
  }
}

// ---------------------------------------------------------------------------------------------
// grid_sample(x, grid; padding_mode=:border), align_corners=true (NNlib; src/training.jl:56).
// x [n][c][hi][wi], grid [n][ho][wo][2] = normalised (x, y), out [n][c][ho][wo].
// ---------------------------------------------------------------------------------------------
struct GridAt {
  int x0, y0, x1, y1;
  float fx, fy, mx, my;
};
__device__ __forceinline__ GridAt grid_at(float gxn, float gyn, int wi, int hi) {
  const float ix = (gxn + 1.f) * 0.5f * (float)(wi - 1), iy = (gyn + 1.f) * 0.5f * (float)(hi - 1);
  const float cx = fminf(fmaxf(ix, 0.f), (float)(wi - 1)), cy = fminf(fmaxf(iy, 0.f), (float)(hi - 1));
  GridAt a;
  a.x0 = (int)cx;
  a.y0 = (int)cy;
  a.x1 = min(a.x0 + 1, wi - 1);
  a.y1 = min(a.y0 + 1, hi - 1);
  a.fx = cx - (float)a.x0;
  a.fy = cy - (float)a.y0;
  a.mx = (ix > 0.f && ix < (float)(wi - 1)) ? 1.f : 0.f;   // border clip: no gradient outside
  a.my = (iy > 0.f && iy < (float)(hi - 1)) ? 1.f : 0.f;
  return a;
}

__global__ __launch_bounds__(256) void grid_sample_fwd_kernel(const float* __restrict__ x,
                                                              const float* __restrict__ grid, int C,
                                                              int hi, int wi, long PO,
                                                              float* __restrict__ out) {
  const int n = blockIdx.y;
  const long p = (long)blockIdx.x * 256 + threadIdx.x;
  if (p >= PO) return;
  const float* g = grid + ((long)n * PO + p) * 2;
  const GridAt a = grid_at(g[0], g[1], wi, hi);
  const long HWi = (long)hi * wi;
  for (int c = 0; c < C; ++c) {
    const float* q = x + ((long)n * C + c) * HWi;
    const float v = (1.f - a.fy) * ((1.f - a.fx) * q[a.y0 * wi + a.x0] + a.fx * q[a.y0 * wi + a.x1]) +
                    a.fy * ((1.f - a.fx) * q[a.y1 * wi + a.x0] + a.fx * q[a.y1 * wi + a.x1]);
    out[((long)n * C + c) * PO + p] = v;
  }
}

__global__ __launch_bounds__(256) void grid_sample_bwd_kernel(const float* __restrict__ x,
                                                              const float* __restrict__ grid, int C,
                                                              int hi, int wi, long PO,
                                                              const float* __restrict__ dout,
                                                              float* __restrict__ d_grid,
                                                              float* __restrict__ d_x) {
  const int n = blockIdx.y;
  const long p = (long)blockIdx.x * 256 + threadIdx.x;
  if (p >= PO) return;
  const float* g = grid + ((long)n * PO + p) * 2;
  const GridAt a = grid_at(g[0], g[1], wi, hi);
  const long HWi = (long)hi * wi;
  const bool okx = a.x1 != a.x0, oky = a.y1 != a.y0;   // the far corner lies inside the image
  float gxs = 0.f, gys = 0.f;
  for (int c = 0; c < C; ++c) {
    const float* q = x + ((long)n * C + c) * HWi;
    const float go = dout[((long)n * C + c) * PO + p];
    const float v00 = q[a.y0 * wi + a.x0];
    const float v01 = okx ? q[a.y0 * wi + a.x1] : 0.f;
    const float v10 = oky ? q[a.y1 * wi + a.x0] : 0.f;
    const float v11 = (okx && oky) ? q[a.y1 * wi + a.x1] : 0.f;
    gxs += go * ((v01 - v00) * (1.f - a.fy) + (v11 - v10) * a.fy);
    gys += go * ((v10 - v00) * (1.f - a.fx) + (v11 - v01) * a.fx);
    if (d_x) {   // scatter (atomic: summation order not fixed)
      float* dq = d_x + ((long)n * C + c) * HWi;
      atomicAdd(dq + a.y0 * wi + a.x0, go * (1.f - a.fx) * (1.f - a.fy));
      if (okx) atomicAdd(dq + a.y0 * wi + a.x1, go * a.fx * (1.f - a.fy));
      if (oky) atomicAdd(dq + a.y1 * wi + a.x0, go * (1.f - a.fx) * a.fy);
      if (okx && oky) atomicAdd(dq + a.y1 * wi + a.x1, go * a.fx * a.fy);
    }
  }
  // d ix / d gx = (wi - 1) / 2
  d_grid[((long)n * PO + p) * 2 + 0] = gxs * a.mx * 0.5f * (float)(wi - 1);
  d_grid[((long)n * PO + p) * 2 + 1] = gys * a.my * 0.5f * (float)(hi - 1);
}

}  // namespace

// per-sample mean of an [n][hw] map, one block per sample, fixed summation order (deterministic)
__global__ __launch_bounds__(256) void sample_mean_kernel(const float* __restrict__ m, long hw,
                                                          float* __restrict__ out) {
  __shared__ float red[4];
  const float* p = m + (long)blockIdx.x * hw;
  float s = 0.f;
  for (long i = threadIdx.x; i < hw; i += 256) s += p[i];
  float v[1] = {s};
  block_sum256<1>(v, red);
  if (threadIdx.x == 0) out[blockIdx.x] = v[0] / (float)hw;
}

int launch_automask(const float* x, long x_sample_stride, long x_frame_stride, int target,
                    int src0, int src1, int N, int C, int H, int W, float* out, hipStream_t st) {
  const dim3 grid(cdiv(W, OT_W), cdiv(H, OT_H), N);
  if (C == 3)
    hipLaunchKernelGGL(automask_kernel<3>, grid, dim3(256), 0, st, x, x_sample_stride,
                       x_frame_stride, target, src0, src1, W, H, out);
  else if (C == 1)
    hipLaunchKernelGGL(automask_kernel<1>, grid, dim3(256), 0, st, x, x_sample_stride,
                       x_frame_stride, target, src0, src1, W, H, out);
  else {
    set_error("automask: channels must be 1 or 3");
    return MD2_ENOTSUP;
  }
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

}  // namespace md2

using namespace md2;

namespace {
Mat3 mat3(const float* m) {
  Mat3 r;
  for (int i = 0; i < 9; ++i) r.m[i] = m[i];
  return r;
}
inline size_t a256(size_t b) { return (b + 255) & ~size_t(255); }
}  // namespace

extern "C" {

int md2_automasking_loss(const float* x, int n, int c, int h, int w, int target, int src0,
                         int src1, float* out, void* stream) {
  MD2_CHECK_ARG(x && out && n > 0 && w >= 2 && h >= 2, "automasking_loss args");
  MD2_CHECK_ARG(target >= 0 && target < 3 && src0 >= 0 && src0 < 3 && src1 >= 0 && src1 < 3,
                "frame ids (0-based, < 3)");
  const long fs = (long)c * h * w;
  return launch_automask(x, 3 * fs, fs, target, src0, src1, n, c, h, w, out, (hipStream_t)stream);
}

size_t md2_static_scores_workspace_size(int n, int h, int w) {
  return a256(sizeof(float) * (size_t)n * h * w);
}

// find_static (src/dtk.jl:51-69): score[i] = mean(automasking_loss(ssim, x_i, x_i[target];
// source_ids)); the caller keeps the samples whose score exceeds alpha
int md2_static_scores(const float* x, int n, int c, int h, int w, int target, int src0, int src1,
                      float* scores, void* workspace, void* stream) {
  MD2_CHECK_ARG(x && scores && workspace && n > 0 && w >= 2 && h >= 2, "static_scores args");
  MD2_CHECK_ARG(target >= 0 && target < 3 && src0 >= 0 && src0 < 3 && src1 >= 0 && src1 < 3,
                "frame ids (0-based, < 3)");
  const long fs = (long)c * h * w;
  float* map = (float*)workspace;
  MD2_TRY(launch_automask(x, 3 * fs, fs, target, src0, src1, n, c, h, w, map, (hipStream_t)stream));
  hipLaunchKernelGGL(sample_mean_kernel, dim3(n), dim3(256), 0, (hipStream_t)stream, map,
                     (long)h * w, scores);
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

int md2_ssim_fwd(const float* x, const float* y, int n, int c, int h, int w, float* out,
                 void* stream) {
  MD2_CHECK_ARG(x && y && out && n > 0 && c > 0 && w >= 2 && h >= 2, "ssim_fwd args");
  hipLaunchKernelGGL(ssim_fwd_kernel, dim3(cdiv(w, OT_W), cdiv(h, OT_H), n * c), dim3(256), 0,
                     (hipStream_t)stream, x, y, w, h, out);
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

int md2_ssim_bwd(const float* x, const float* y, const float* dout, int n, int c, int h, int w,
                 float* dx, float* dy, void* stream) {
  MD2_CHECK_ARG(x && y && dout && (dx || dy) && n > 0 && c > 0 && w >= 2 && h >= 2, "ssim_bwd args");
  hipLaunchKernelGGL(ssim_bwd_kernel, dim3(cdiv(w, OT_W), cdiv(h, OT_H), n * c), dim3(256), 0,
                     (hipStream_t)stream, x, y, dout, w, h, dx, dy);
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

int md2_backproject_fwd(const float* depth, int n, int w, int h, const float* invK, float* out,
                        void* stream) {
  MD2_CHECK_ARG(depth && invK && out && n > 0 && w > 0 && h > 0, "backproject_fwd args");
  const long P = (long)w * h, total = P * n;
  hipLaunchKernelGGL(backproject_fwd_kernel, dim3(cdiv(total, 256)), dim3(256), 0,
                     (hipStream_t)stream, depth, w, P, total, mat3(invK), out);
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

int md2_backproject_bwd(const float* dout, int n, int w, int h, const float* invK, float* d_depth,
                        void* stream) {
  MD2_CHECK_ARG(dout && invK && d_depth && n > 0 && w > 0 && h > 0, "backproject_bwd args");
  const long P = (long)w * h, total = P * n;
  hipLaunchKernelGGL(backproject_bwd_kernel, dim3(cdiv(total, 256)), dim3(256), 0,
                     (hipStream_t)stream, dout, w, P, total, mat3(invK), d_depth);
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

int md2_project_fwd(const float* points, int n, int w, int h, const float* K, const float* R,
                    const float* t, float* out, void* stream) {
  MD2_CHECK_ARG(points && K && R && t && out && n > 0 && w > 1 && h > 1, "project_fwd args");
  const long P = (long)w * h;
  hipLaunchKernelGGL(project_fwd_kernel, dim3(cdiv(P, 256), n), dim3(256), 0, (hipStream_t)stream,
                     points, P, mat3(K), R, t, (float)(w - 1), (float)(h - 1), out);
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

size_t md2_project_workspace_size(int n, int w, int h) {
  return a256(sizeof(float) * 12 * (size_t)n * cdiv((long)w * h, 256));
}

int md2_project_bwd(const float* points, int n, int w, int h, const float* K, const float* R,
                    const float* t, const float* dout, float* d_points, float* d_R, float* d_t,
                    void* workspace, void* stream) {
  MD2_CHECK_ARG(points && K && R && t && dout && d_points && d_R && d_t && workspace && n > 0 &&
                    w > 1 && h > 1,
                "project_bwd args");
  const long P = (long)w * h;
  const int nb = cdiv(P, 256);
  hipStream_t st = (hipStream_t)stream;
  float* part = (float*)workspace;
  hipLaunchKernelGGL(project_bwd_kernel, dim3(nb, n), dim3(256), 0, st, points, P, mat3(K), R, t,
                     (float)(w - 1), (float)(h - 1), dout, d_points, part);
  MD2_LAUNCH_CHECK();
  hipLaunchKernelGGL(reduce_partials_kernel, dim3(12, n), dim3(256), 0, st, part, nb, 12, 12, d_R,
                     d_t, 9);
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

int md2_grid_sample_border_fwd(const float* x, const float* grid, int n, int c, int hi, int wi,
                               int ho, int wo, float* out, void* stream) {
  MD2_CHECK_ARG(x && grid && out && n > 0 && c > 0 && hi > 0 && wi > 0 && ho > 0 && wo > 0,
                "grid_sample_fwd args");
  const long PO = (long)ho * wo;
  hipLaunchKernelGGL(grid_sample_fwd_kernel, dim3(cdiv(PO, 256), n), dim3(256), 0,
                     (hipStream_t)stream, x, grid, c, hi, wi, PO, out);
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

int md2_grid_sample_border_bwd(const float* x, const float* grid, const float* dout, int n, int c,
                               int hi, int wi, int ho, int wo, float* d_grid, float* d_x,
                               void* stream) {
  MD2_CHECK_ARG(x && grid && dout && d_grid && n > 0 && c > 0 && hi > 0 && wi > 0 && ho > 0 && wo > 0,
                "grid_sample_bwd args");
  hipStream_t st = (hipStream_t)stream;
  const long PO = (long)ho * wo;
  if (d_x) MD2_HIP(hipMemsetAsync(d_x, 0, sizeof(float) * (size_t)n * c * hi * wi, st));
  hipLaunchKernelGGL(grid_sample_bwd_kernel, dim3(cdiv(PO, 256), n), dim3(256), 0, st, x, grid, c,
                     hi, wi, PO, dout, d_grid, d_x);
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

// smooth_loss(disparity [n][h][w], image [n][c][h][w]) -- the smoothness kernel of the loss tail
// on a full-resolution disparity, no mean normalisation, upstream weight dloss.
int md2_unorm8_to_float(const unsigned char* in, float* out, long long n, void* stream) {
  MD2_CHECK_ARG(in && out && n >= 0, "unorm8_to_float args");
  MD2_CHECK_ARG(((uintptr_t)in & 3) == 0 && ((uintptr_t)out & 15) == 0,
                "unorm8_to_float: in must be 4-byte and out 16-byte aligned");
  if (n == 0) return MD2_OK;
  const long blocks = std::min<long>(4096, cdiv(n, 256 * 4));
  hipLaunchKernelGGL(unorm8_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                     (const uint8_t*)in, (long)n, out);
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

size_t md2_smooth_loss_workspace_size(int n, int w, int h) {
  return a256(sizeof(float) * (size_t)n * w * h) + a256(sizeof(float) * 2 * smooth_blocks(w, h, n));
}

static int smooth_run(const float* disp, const float* img, int n, int c, int h, int w, float dloss,
                      float* loss, float* d_disp, void* workspace, hipStream_t st) {
  MD2_CHECK_ARG(disp && img && workspace && n > 0 && w >= 2 && h >= 2, "smooth_loss args");
  MD2_CHECK_ARG(c == 1 || c == 3, "smooth_loss: channels must be 1 or 3");
  char* ws = (char*)workspace;
  float* g = d_disp ? d_disp : (float*)ws;
  float* part = (float*)(ws + a256(sizeof(float) * (size_t)n * w * h));
  MD2_HIP(hipMemsetAsync(g, 0, sizeof(float) * (size_t)n * w * h, st));
  SmoothArgs sa{};
  sa.disp = disp;
  sa.dw = w;
  sa.dh = h;
  sa.rx = sa.ry = 1.f;
  sa.img = img;
  sa.img_sample_stride = (long)c * h * w;
  sa.mean_partials = nullptr;
  sa.mean_parts = 0;
  sa.ws = dloss;
  sa.g_disp = g;
  sa.partials = part;
  sa.N = n;
  sa.W = w;
  sa.H = h;
  MD2_TRY(launch_smooth(&sa, 1, c, st));
  if (loss) {
    const int nb = (int)smooth_blocks(w, h, n);
    hipLaunchKernelGGL(reduce_partials_kernel, dim3(1, 1), dim3(256), 0, st, part, nb, 1, 2, loss,
                       nullptr, 1);
    MD2_LAUNCH_CHECK();
  }
  return MD2_OK;
}

int md2_smooth_loss_fwd(const float* disp, const float* img, int n, int c, int h, int w,
                        float* loss, void* workspace, void* stream) {
  MD2_CHECK_ARG(loss, "smooth_loss_fwd: loss");
  return smooth_run(disp, img, n, c, h, w, 1.f, loss, nullptr, workspace, (hipStream_t)stream);
}

int md2_smooth_loss_bwd(const float* disp, const float* img, int n, int c, int h, int w,
                        float dloss, float* d_disp, void* workspace, void* stream) {
  MD2_CHECK_ARG(d_disp, "smooth_loss_bwd: d_disp");
  return smooth_run(disp, img, n, c, h, w, dloss, nullptr, d_disp, workspace, (hipStream_t)stream);
}

}  // extern "C"
