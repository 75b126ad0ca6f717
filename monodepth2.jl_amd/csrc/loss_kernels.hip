// Loss-tail kernels of the Monodepth2.jl train step around the photometric pass (photo.hip):
// disparity means, edge-aware smoothness, the upsample adjoint, final reductions, so3/composeT,
// and the visualisation warp (gfx950).
//
// Reference: src/training.jl:21-78 (train_loss), src/utils.jl:106-145 (so3 + hat),
// :163-183 (smooth_loss, disparity_to_depth), :185-192 (composeT).
#include <algorithm>

#include "loss_kernels.h"

namespace md2 {

// Bilinear align_corners=true upsample of one value (NNlib upsample_bilinear(x; size)),
// src/training.jl:45.  ratio = (in-1)/(out-1).
__device__ __forceinline__ float upsample_at(const float* __restrict__ d, int dw, int dh,
                                             float rx, float ry, int X, int Y) {
  const float sx = rx * (float)X, sy = ry * (float)Y;
  int ix0 = (int)sx, iy0 = (int)sy;
  ix0 = min(ix0, dw - 1);
  iy0 = min(iy0, dh - 1);
  const int ix1 = min(ix0 + 1, dw - 1), iy1 = min(iy0 + 1, dh - 1);
  const float fx = sx - (float)ix0, fy = sy - (float)iy0;
  const float v00 = d[iy0 * dw + ix0], v01 = d[iy0 * dw + ix1];
  const float v10 = d[iy1 * dw + ix0], v11 = d[iy1 * dw + ix1];
  return (1.f - fy) * ((1.f - fx) * v00 + fx * v01) + fy * ((1.f - fx) * v10 + fx * v11);
}

__device__ __forceinline__ float disp_at(const float* __restrict__ d, int dw, int dh, float rx,
                                         float ry, int W, int H, int X, int Y) {
  if (dw == W && dh == H) return d[Y * W + X];
  return upsample_at(d, dw, dh, rx, ry, X, Y);
}

struct Proj {
  float X[3];     // camera point  depth * invK * (w, h, 1)
  float P[3];     // R X + t
  float cam[3];   // K P
  float denom;    // 1 / (cam_z + 1e-7)
  float ix, iy;   // unnormalised sample coordinate (0-based), before clamping
};

// src/utils.jl:67-69 (Backproject), :99-103 (Project), :83-85 (normalize), and the NNlib
// grid_sample unnormalisation ((g + 1)/2)(size - 1) for align_corners = true.
__device__ __forceinline__ void project_point(const Geom& g, const float* Rt, float depth,
                                              float ray0, float ray1, float ray2, Proj& p) {
  p.X[0] = depth * ray0;
  p.X[1] = depth * ray1;
  p.X[2] = depth * ray2;
#pragma unroll
  for (int i = 0; i < 3; ++i)
    p.P[i] = Rt[3 * i + 0] * p.X[0] + Rt[3 * i + 1] * p.X[1] + Rt[3 * i + 2] * p.X[2] + Rt[9 + i];
#pragma unroll
  for (int i = 0; i < 3; ++i)
    p.cam[i] = g.K[3 * i + 0] * p.P[0] + g.K[3 * i + 1] * p.P[1] + g.K[3 * i + 2] * p.P[2];
  p.denom = 1.f / (p.cam[2] + 1e-7f);
  const float u = p.cam[0] * p.denom, v = p.cam[1] * p.denom;
  const float gx = (((u - 1.f) / g.wm1) - 0.5f) * 2.f;
  const float gy = (((v - 1.f) / g.hm1) - 0.5f) * 2.f;
  p.ix = ((gx + 1.f) * 0.5f) * g.wm1;
  p.iy = ((gy + 1.f) * 0.5f) * g.hm1;
}

__device__ __forceinline__ void ray_at(const Geom& g, int gx, int gy, float& r0, float& r1,
                                       float& r2) {
  const float w = (float)(gx + 1), h = (float)(gy + 1);   // 1-based grid (src/utils.jl:51-55)
  r0 = g.invK[0] * w + g.invK[1] * h + g.invK[2];
  r1 = g.invK[3] * w + g.invK[4] * h + g.invK[5];
  r2 = g.invK[6] * w + g.invK[7] * h + g.invK[8];
}

// ---------------------------------------------------------------------------------------------
// per-image mean of the (upsampled) disparity -- src/training.jl:64-65
// ---------------------------------------------------------------------------------------------
// all scales in one launch: grid (parts, N, nscales)
__global__ __launch_bounds__(256) void disp_sum_kernel(DispSumBatch b) {
  __shared__ double red[4];
  const int n = blockIdx.y;
  const DispSumArgs a = b.s[blockIdx.z];
  const int W = b.W, H = b.H, parts = b.parts;
  const long P = (long)W * H;
  const float* d = a.disp + (long)n * a.dw * a.dh;
  double s = 0.0;
  for (long q = (long)blockIdx.x * 256 + threadIdx.x; q < P; q += (long)parts * 256) {
    const int X = (int)(q % W), Y = (int)(q / W);
    s += (double)disp_at(d, a.dw, a.dh, a.rx, a.ry, W, H, X, Y);
  }
  double v[1] = {s};
  block_sum256_d<1>(v, red);
  if (threadIdx.x == 0) a.out[n * parts + blockIdx.x] = v[0];
}

// ---------------------------------------------------------------------------------------------
// Edge-aware smoothness on the mean-normalised full-res disparity (src/utils.jl:163-177,
// src/training.jl:64-67), forward + the local part of the backward.
// ---------------------------------------------------------------------------------------------
// A wave owns 62 columns (lanes 1..62; lanes 0 and 63 hold the neighbouring columns x0-1 and
// x0+62) and walks SM_R rows top to bottom (plus the row above its band) with the current and
// the next row in registers: each pixel's disparity (the align-corners upsample) and image
// values are formed ONCE, the right neighbour comes from lane + 1 and the left pair's weight from
// lane - 1 by DPP, the row above's vertical weight from the previous step, the row two ahead is
// loaded while the current one is computed.  4 waves = 4 stacked bands per block.  (The previous
// LDS-tile form evaluated every disparity 2-3 times and every image value 4 times: 55-61 us per
// launch at B=12.)  Same per-pixel arithmetic and evaluation order as before.
constexpr int SM_TW = 62, SM_R = 8, SM_BR = 4 * SM_R;

__device__ __forceinline__ float sm_from_left(float v) {    // lane i <- lane i-1
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x138, 0xf, 0xf, true));
}
__device__ __forceinline__ float sm_from_right(float v) {   // lane i <- lane i+1
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x130, 0xf, 0xf, true));
}

template <int C>
__global__ __launch_bounds__(256) void smooth_kernel(SmoothBatch b) {
  __shared__ float s_red[4 * 3];
  __shared__ double s_redd[4];
  const int sc = blockIdx.z / b.s[0].N;       // scale; every scale shares N, W, H
  const SmoothArgs a = b.s[sc];
  const int W = a.W, H = a.H;
  const long HW = (long)W * H;
  const int n = blockIdx.z - sc * a.N;
  const int lane = threadIdx.x & 63, wq = threadIdx.x >> 6;
  const int x = (int)blockIdx.x * SM_TW + lane - 1;
  const int y0 = (int)blockIdx.y * SM_BR + wq * SM_R;
  const bool colv = x >= 0 && x < W;
  const bool own = colv && lane >= 1 && lane <= SM_TW;
  const bool hpair = colv && x + 1 < W && lane < 63;   // the pair (x, x+1) exists
  const int xc = min(max(x, 0), W - 1);
  const float* dsp = a.disp + (long)n * a.dw * a.dh;
  const float* img = a.img + (long)n * a.img_sample_stride;
  float inv = 1.f;                          // slow_depth: no mean normalisation
  if (a.mean_partials) {
    double m = 0.0;
    for (int k = 0; k < a.mean_parts; ++k) m += a.mean_partials[n * a.mean_parts + k];
    inv = 1.f / ((float)(m / (double)HW) + 1e-7f);
  }
  const float cx = 1.f / ((float)a.N * (float)H * (float)(W - 1));
  const float cy = 1.f / ((float)a.N * (float)(H - 1) * (float)W);
  auto load_row = [&](int r, float& d, float (&im)[C]) {
    const int rc = min(max(r, 0), H - 1);
    d = disp_at(dsp, a.dw, a.dh, a.rx, a.ry, W, H, xc, rc);
#pragma unroll
    for (int c = 0; c < C; ++c) im[c] = img[c * HW + (long)rc * W + xc];
  };
  float lx = 0.f, ly = 0.f, tsum = 0.f;
  double tsumd = 0.0;
  if (y0 < H) {                             // wave-uniform
    const int r1 = min(y0 + SM_R, H);
    float d0, i0[C], d1, i1[C], d2, i2[C];
    load_row(y0 - 1, d0, i0);
    load_row(y0, d1, i1);
    float vyprev = 0.f;
    for (int r = y0 - 1; r < r1; ++r) {     // wave-uniform trip count
      load_row(r + 2, d2, i2);              // two rows ahead
      // differences are formed on the raw disparity and scaled afterwards: (d_q - d_r) * inv is
      // sign-exact (no FMA-contraction residue where d_q == d_r, abs'(0) = 0)
      float vx = 0.f, vy = 0.f;
      {
        const float dr = sm_from_right(d0);
        float gi = 0.f;
#pragma unroll
        for (int c = 0; c < C; ++c) gi += fabsf(i0[c] - sm_from_right(i0[c]));
        const float e = expf(-gi / (float)C) * cx;
        const float df = (d0 - dr) * inv;
        if (r >= 0 && hpair) {
          vx = e * (df > 0.f ? 1.f : (df < 0.f ? -1.f : 0.f));
          if (own && r >= y0) lx += fabsf(df) * e;
        }
      }
      if (r >= 0 && r + 1 < H && colv) {
        float gi = 0.f;
#pragma unroll
        for (int c = 0; c < C; ++c) gi += fabsf(i0[c] - i1[c]);
        const float e = expf(-gi / (float)C) * cy;
        const float df = (d0 - d1) * inv;
        vy = e * (df > 0.f ? 1.f : (df < 0.f ? -1.f : 0.f));
        if (own && r >= y0) ly += fabsf(df) * e;
      }
      const float vxl = sm_from_left(vx);
      if (r >= y0 && own) {
        const float u = vx - vxl + vy - vyprev;
        const long q = ((long)n * H + r) * W + x;
        a.g_disp[q] += a.ws * u * inv;
        tsum += u * d0;
        tsumd += (double)u * (double)d0;
      }
      vyprev = vy;
      d0 = d1;
      d1 = d2;
#pragma unroll
      for (int c = 0; c < C; ++c) {
        i0[c] = i1[c];
        i1[c] = i2[c];
      }
    }
  }
  float v[3] = {lx + ly, tsum, 0.f};
  block_sum256<3>(v, s_red);
  const long blk = ((long)n * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
  if (threadIdx.x == 0) {
    a.partials[blk * 2 + 0] = v[0];
    a.partials[blk * 2 + 1] = v[1];
  }
  if (a.tsum) {                               // block-uniform
    double t[1] = {tsumd};
    block_sum256_d<1>(t, s_redd);
    if (threadIdx.x == 0) a.tsum[blk] = t[0];
  }
}

// ---------------------------------------------------------------------------------------------
// Adjoint of the align_corners bilinear upsample (+ the mean-normalisation constant and the
// optional sigmoid derivative of the disparity head), one low-res pixel per thread.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ void up_range(int j, int in, int out, float r, int& lo, int& hi) {
  if (in == 1) {
    lo = 0;
    hi = out - 1;
    return;
  }
  lo = max(0, (int)floorf((float)(j - 1) / r) - 1);
  hi = min(out - 1, (int)ceilf((float)(j + 1) / r) + 1);
}

__device__ __forceinline__ float up_weight(int X, int j, int in, float r) {
  const float sx = r * (float)X;
  int i0 = (int)sx;
  i0 = min(i0, in - 1);
  const int i1 = min(i0 + 1, in - 1);
  const float f = sx - (float)i0;
  return (i0 == j ? 1.f - f : 0.f) + (i1 == j ? f : 0.f);
}

// One block per (low-res row i, sample n).  The mean-normalisation constant is reduced once
// per block; the row's full-res support rows are contracted column-wise into LDS (coalesced
// reads of g), then each low-res column contracts its support columns from LDS.
// All scales in one launch: grid (max dh, N, nscales); rows past a scale's dh exit at once.
__global__ __launch_bounds__(256) void up_adjoint_kernel(UpAdjBatch b) {
  extern __shared__ float s_col[];           // [W]
  __shared__ double s_red[2][4];
  const UpAdjArgs a = b.s[blockIdx.z];
  const int W = a.W, H = a.H;
  const int i = blockIdx.x, n = blockIdx.y, tid = threadIdx.x;
  if (i >= a.dh) return;                     // block-uniform, before any barrier
  float cn = 0.f;
  if (a.smooth_tsum) {
    // the mean-normalisation constant -ws * sum(u d) / (m^2 W H): sum(u d) is a near-cancelling
    // sum (the normalised disparity is scale invariant, so its gradient is orthogonal to d), so
    // both sums are formed in fp64 from fp64 partials
    double m = 0.0, T = 0.0;
    for (int k = tid; k < a.mean_parts; k += 256) m += a.mean_partials[n * a.mean_parts + k];
    for (int k = tid; k < a.smooth_parts; k += 256) T += a.smooth_tsum[(long)n * a.smooth_parts + k];
    m = wave_sum_d(m);
    T = wave_sum_d(T);
    if ((tid & 63) == 0) {
      s_red[0][tid >> 6] = m;
      s_red[1][tid >> 6] = T;
    }
    __syncthreads();
    m = (s_red[0][0] + s_red[0][1]) + (s_red[0][2] + s_red[0][3]);
    T = (s_red[1][0] + s_red[1][1]) + (s_red[1][2] + s_red[1][3]);
    const double WH = (double)W * (double)H;
    const double mi = 1.0 / ((double)(float)(m / WH) + 1e-7);
    cn = (float)(-(double)a.ws * T * mi * mi / WH);
  }
  const float* g = a.g_full + (long)n * W * H;
  const long orow = ((long)n * a.dh + i) * a.dw;
  const bool direct = a.dw == W && a.dh == H;
  float wys = 0.f;
  if (!direct) {
    int ylo, yhi;
    up_range(i, a.dh, H, a.ry, ylo, yhi);
    for (int Y = ylo; Y <= yhi; ++Y) wys += up_weight(Y, i, a.dh, a.ry);
    for (int X = tid; X < W; X += 256) {
      float c = 0.f;
      for (int Y = ylo; Y <= yhi; ++Y) {
        const float wy = up_weight(Y, i, a.dh, a.ry);
        if (wy != 0.f) c += wy * g[(long)Y * W + X];
      }
      s_col[X] = c;
    }
    __syncthreads();
  }
  for (int j = tid; j < a.dw; j += 256) {
    float acc;
    if (direct) {
      acc = g[(long)i * W + j] + cn;
    } else {
      int xlo, xhi;
      up_range(j, a.dw, W, a.rx, xlo, xhi);
      float row = 0.f, wxs = 0.f;
      for (int X = xlo; X <= xhi; ++X) {
        const float wx = up_weight(X, j, a.dw, a.rx);
        wxs += wx;
        row += wx * s_col[X];
      }
      acc = row + cn * wxs * wys;
    }
    if (a.sigmoid) {
      const float sg = a.disp[orow + j];
      acc *= sg * (1.f - sg);
    }
    if (a.accumulate)
      a.out[orow + j] += acc;
    else
      a.out[orow + j] = acc;
  }
}

// ---------------------------------------------------------------------------------------------
// Final deterministic reductions: loss scalar and per-(source, sample) dR, dt.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void loss_finalize_kernel(FinalizeArgs a) {
  __shared__ float red[4 * 2];
  // one block per scale: sum photometric (col 0 of 25) and smooth (col 0 of 2) partials
  const int s = blockIdx.x;
  float v[2] = {0.f, 0.f};
  for (long k = threadIdx.x; k < a.photo_blocks[s]; k += 256) v[0] += a.photo_partials[s][k * 25];
  for (long k = threadIdx.x; k < a.smooth_blocks[s]; k += 256) v[1] += a.smooth_partials[s][k * 2];
  block_sum256<2>(v, red);
  if (threadIdx.x == 0) {
    a.terms[2 * s + 0] = v[0] * a.photo_scale;         // mean(warp_loss)
    a.terms[2 * s + 1] = v[1] * a.smooth_scale[s];      // smooth * 1e-3 * scale
  }
}

__global__ void loss_total_kernel(const float* terms, int nscales, float divisor, float* loss) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    float l = 0.f;
    for (int s = 0; s < nscales; ++s) l += terms[2 * s] + terms[2 * s + 1];
    loss[0] = l / divisor;
  }
}

// grid: (2*N) blocks; sums the 24 pose values of every block of image n over all scales.
__global__ __launch_bounds__(256) void pose_grad_reduce_kernel(FinalizeArgs a, float* dRt) {
  __shared__ float red[4 * 12];
  const int q = blockIdx.x;            // q = s*N + n
  const int s = q / a.N, n = q % a.N;
  float v[12];
#pragma unroll
  for (int k = 0; k < 12; ++k) v[k] = 0.f;
  for (int sc = 0; sc < a.nscales; ++sc) {
    const long per = a.photo_blocks[sc] / a.N;
    const float* p = a.photo_partials[sc] + (long)n * per * 25;
    for (long b = threadIdx.x; b < per; b += 256) {
#pragma unroll
      for (int k = 0; k < 12; ++k) v[k] += p[b * 25 + 1 + 12 * s + k];
    }
  }
  block_sum256<12>(v, red);
  if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < 12; ++k) dRt[(long)q * 12 + k] = v[k];
  }
}

// ---------------------------------------------------------------------------------------------
// so3_exp_map + composeT forward / backward (src/utils.jl:106-145, 185-192).
// pose [2N][6] = (rvec, tvec) per (source, sample); invert flag per source.
// ---------------------------------------------------------------------------------------------
// fp64 throughout (2N threads): the rotation's rounding perturbs every pixel's warp coherently,
// and 1 - cos(th) cancels at the small angles a pose network emits
struct So3Tmp {
  double S[9], S2[9], f1, f2, th, thi;
};

__device__ __forceinline__ void so3_core(const float* rf, So3Tmp& t) {
  const double r[3] = {rf[0], rf[1], rf[2]};
  t.S[0] = 0.0;   t.S[1] = -r[2]; t.S[2] = r[1];
  t.S[3] = r[2];  t.S[4] = 0.0;   t.S[5] = -r[0];
  t.S[6] = -r[1]; t.S[7] = r[0];  t.S[8] = 0.0;
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j)
      t.S2[3 * i + j] = t.S[3 * i] * t.S[j] + t.S[3 * i + 1] * t.S[3 + j] + t.S[3 * i + 2] * t.S[6 + j];
  t.th = sqrt(r[0] * r[0] + r[1] * r[1] + r[2] * r[2]);
  t.thi = 1.0 / fmax(t.th, 1e-4);
  t.f1 = t.thi * sin(t.th);
  t.f2 = t.thi * t.thi * (1.0 - cos(t.th));
}

__global__ void so3_fwd_kernel(const float* __restrict__ pose, int count, int N, int invert_mask,
                               float* __restrict__ Rt) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= count) return;
  const int s = q / N;
  const float* r = pose + q * 6;
  So3Tmp t;
  so3_core(r, t);
  double R[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) R[k] = t.f1 * t.S[k] + t.f2 * t.S2[k] + ((k % 4) == 0 ? 1.0 : 0.0);
  const double tv[3] = {pose[q * 6 + 3], pose[q * 6 + 4], pose[q * 6 + 5]};
  float* o = Rt + q * 12;
  if ((invert_mask >> s) & 1) {
    // R' = R^T, t' = R' (-t)
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) o[3 * i + j] = (float)R[3 * j + i];
#pragma unroll
    for (int i = 0; i < 3; ++i) o[9 + i] = (float)-(R[i] * tv[0] + R[3 + i] * tv[1] + R[6 + i] * tv[2]);
  } else {
#pragma unroll
    for (int k = 0; k < 9; ++k) o[k] = (float)R[k];
#pragma unroll
    for (int i = 0; i < 3; ++i) o[9 + i] = (float)tv[i];
  }
}

__global__ void so3_bwd_kernel(const float* __restrict__ pose, int count, int N, int invert_mask,
                               const float* __restrict__ dRt, float* __restrict__ dpose,
                               int accumulate) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= count) return;
  const int s = q / N;
  const float* r = pose + q * 6;
  So3Tmp t;
  so3_core(r, t);
  double R[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) R[k] = t.f1 * t.S[k] + t.f2 * t.S2[k] + ((k % 4) == 0 ? 1.0 : 0.0);
  const double tv[3] = {pose[q * 6 + 3], pose[q * 6 + 4], pose[q * 6 + 5]};
  const float* g = dRt + q * 12;
  double dR[9], dt[3];
  if ((invert_mask >> s) & 1) {
    // R' = R^T; t' = -R' t.  dR'_ij += -dt'_i t_j ;  dt = -R'^T dt' = -R dt'
    double dRp[9];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) dRp[3 * i + j] = g[3 * i + j] - g[9 + i] * tv[j];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) dR[3 * i + j] = dRp[3 * j + i];
#pragma unroll
    for (int i = 0; i < 3; ++i) dt[i] = -(R[3 * i] * g[9] + R[3 * i + 1] * g[10] + R[3 * i + 2] * g[11]);
  } else {
#pragma unroll
    for (int k = 0; k < 9; ++k) dR[k] = g[k];
#pragma unroll
    for (int i = 0; i < 3; ++i) dt[i] = g[9 + i];
  }
  // R = f1 S + f2 S^2 + I
  double dS[9];
  double df1 = 0.0, df2 = 0.0;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    df1 += dR[k] * t.S[k];
    df2 += dR[k] * t.S2[k];
  }
  // d/dS <dR, S^2> = dR S^T + S^T dR
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      double a1 = 0.0, a2 = 0.0;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        a1 += dR[3 * i + k] * t.S[3 * j + k];
        a2 += t.S[3 * k + i] * dR[3 * k + j];
      }
      dS[3 * i + j] = t.f1 * dR[3 * i + j] + t.f2 * (a1 + a2);
    }
  // f1 = thi sin(th), f2 = thi^2 (1 - cos th), thi = 1/max(th, 1e-4)
  const double dthi = (t.th > 1e-4) ? -1.0 / (t.th * t.th) : 0.0;
  const double dth = df1 * (dthi * sin(t.th) + t.thi * cos(t.th)) +
                     df2 * (2.0 * t.thi * dthi * (1.0 - cos(t.th)) + t.thi * t.thi * sin(t.th));
  double dr[3];
  dr[0] = dS[7] - dS[5];            // hat rrule, src/utils.jl:139-141
  dr[1] = dS[2] - dS[6];
  dr[2] = dS[3] - dS[1];
#pragma unroll
  for (int k = 0; k < 3; ++k) dr[k] += dth * r[k] / t.th;   // d sqrt(sum r^2)
  float* o = dpose + q * 6;
  if (accumulate) {
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      o[k] = (float)(o[k] + dr[k]);
      o[3 + k] = (float)(o[3 + k] + dt[k]);
    }
  } else {
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      o[k] = (float)dr[k];
      o[3 + k] = (float)dt[k];
    }
  }
}

// ---------------------------------------------------------------------------------------------
// host launchers
// ---------------------------------------------------------------------------------------------
// Visualisation warp (train_loss vis_warped, src/training.jl:48-57,71-73): both sources
// resampled through the scale's depth and pose, no loss, no backward.  One thread per target
// pixel, all C channels of both sources; same geometry helpers as the photometric kernel.
template <int C>
__global__ __launch_bounds__(256) void warp_vis_kernel(PhotoArgs a, int scale, Geom g, float* __restrict__ out) {
  const PhotoScale sc = a.sc[scale];
  const int HW = g.W * g.H;
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long)a.N * HW) return;
  const int n = (int)(idx / HW), pix = (int)(idx - (long)n * HW);
  const int Y = pix / g.W, X = pix - Y * g.W;
  const float d = disp_at(sc.disp + (long)n * sc.dw * sc.dh, sc.dw, sc.dh, sc.rx, sc.ry, g.W, g.H, X, Y);
  const float depth = 1.f / (d * g.disp_range + g.min_disp);
  float r0, r1, r2;
  ray_at(g, X, Y, r0, r1, r2);
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    Proj p;
    project_point(g, a.Rt + ((long)s * a.N + n) * 12, depth, r0, r1, r2, p);
    const float x = fminf(fmaxf(p.ix, 0.f), (float)(g.W - 1));
    const float y = fminf(fmaxf(p.iy, 0.f), (float)(g.H - 1));
    const int x0 = (int)x, y0 = (int)y;
    const int x1 = min(x0 + 1, g.W - 1), y1 = min(y0 + 1, g.H - 1);
    const float fx = x - (float)x0, fy = y - (float)y0;
    const float* src = a.x + (long)n * a.x_sample_stride + (long)(s ? a.src1 : a.src0) * a.x_frame_stride;
    float* o = out + ((long)s * a.N + n) * C * HW + pix;
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const float* q = src + (long)c * HW;
      const float v = (1.f - fy) * ((1.f - fx) * q[y0 * g.W + x0] + fx * q[y0 * g.W + x1]) +
                      fy * ((1.f - fx) * q[y1 * g.W + x0] + fx * q[y1 * g.W + x1]);
      o[(long)c * HW] = v;
    }
  }
}

int launch_warp_vis(const PhotoArgs& a, int scale, const Geom& g, int C, float* out, hipStream_t st) {
  const long n = (long)a.N * g.W * g.H;
  const dim3 grid((unsigned)cdiv(n, 256L));
  if (C == 3)
    hipLaunchKernelGGL(warp_vis_kernel<3>, grid, dim3(256), 0, st, a, scale, g, out);
  else if (C == 1)
    hipLaunchKernelGGL(warp_vis_kernel<1>, grid, dim3(256), 0, st, a, scale, g, out);
  else {
    set_error("warp_vis: channels must be 1 or 3");
    return MD2_ENOTSUP;
  }
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

long smooth_blocks(int W, int H, int N) { return (long)cdiv(W, SM_TW) * cdiv(H, SM_BR) * N; }

int launch_disp_sum(const DispSumBatch& b, int nscales, hipStream_t st) {
  MD2_CHECK_ARG(nscales >= 1 && nscales <= MAX_SCALES, "disp_sum: nscales");
  hipLaunchKernelGGL(disp_sum_kernel, dim3(b.parts, b.N, nscales), dim3(256), 0, st, b);
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

int launch_smooth(const SmoothArgs* a, int nscales, int C, hipStream_t st) {
  MD2_CHECK_ARG(nscales >= 1 && nscales <= MAX_SCALES, "smooth: nscales");
  SmoothBatch b{};
  for (int k = 0; k < nscales; ++k) {
    MD2_CHECK_ARG(a[k].N == a[0].N && a[k].W == a[0].W && a[k].H == a[0].H, "smooth: scales differ in N/W/H");
    b.s[k] = a[k];
  }
  dim3 grid(cdiv(a[0].W, SM_TW), cdiv(a[0].H, SM_BR), a[0].N * nscales);
  if (C == 3)
    hipLaunchKernelGGL(smooth_kernel<3>, grid, dim3(256), 0, st, b);
  else if (C == 1)
    hipLaunchKernelGGL(smooth_kernel<1>, grid, dim3(256), 0, st, b);
  else {
    set_error("smooth: channels must be 1 or 3");
    return MD2_ENOTSUP;
  }
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

int launch_up_adjoint(const UpAdjArgs* a, int nscales, hipStream_t st) {
  MD2_CHECK_ARG(nscales >= 1 && nscales <= MAX_SCALES, "up_adjoint: nscales");
  UpAdjBatch b{};
  int maxdh = 1;
  bool any_lds = false;
  for (int k = 0; k < nscales; ++k) {
    MD2_CHECK_ARG(a[k].N == a[0].N && a[k].W == a[0].W, "up_adjoint: scales differ in N/W");
    b.s[k] = a[k];
    maxdh = std::max(maxdh, a[k].dh);
    any_lds |= !(a[k].dw == a[k].W && a[k].dh == a[k].H);
  }
  const size_t lds = any_lds ? (size_t)a[0].W * sizeof(float) : 0;
  MD2_CHECK_ARG(lds <= 64 * 1024, "up_adjoint: full-res width exceeds the LDS row");
  hipLaunchKernelGGL(up_adjoint_kernel, dim3(maxdh, a[0].N, nscales), dim3(256), lds, st, b);
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

int launch_loss_finalize(const FinalizeArgs& a, float* dRt, float* loss, hipStream_t st) {
  hipLaunchKernelGGL(loss_finalize_kernel, dim3(a.nscales), dim3(256), 0, st, a);
  MD2_LAUNCH_CHECK();
  hipLaunchKernelGGL(loss_total_kernel, dim3(1), dim3(64), 0, st, a.terms, a.nscales, a.divisor,
                     loss);
  MD2_LAUNCH_CHECK();
  if (dRt) {
    hipLaunchKernelGGL(pose_grad_reduce_kernel, dim3(2 * a.N), dim3(256), 0, st, a, dRt);
    MD2_LAUNCH_CHECK();
  }
  return MD2_OK;
}

int launch_pose_grad_reduce(const FinalizeArgs& a, float* dRt, hipStream_t st) {
  hipLaunchKernelGGL(pose_grad_reduce_kernel, dim3(2 * a.N), dim3(256), 0, st, a, dRt);
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

int launch_so3_fwd(const float* pose, int count, int N, int invert_mask, float* Rt,
                   hipStream_t st) {
  hipLaunchKernelGGL(so3_fwd_kernel, dim3(cdiv(count, 64)), dim3(64), 0, st, pose, count, N,
                     invert_mask, Rt);
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

int launch_so3_bwd(const float* pose, int count, int N, int invert_mask, const float* dRt,
                   float* dpose, int accumulate, hipStream_t st) {
  hipLaunchKernelGGL(so3_bwd_kernel, dim3(cdiv(count, 64)), dim3(64), 0, st, pose, count, N,
                     invert_mask, dRt, dpose, accumulate);
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

}  // namespace md2
