// Fused warp + SSIM + L1 photometric loss, forward AND pullback, every scale in one launch
// (gfx950).
//
// Reference: src/training.jl:43-62 (per scale: upsample the disparity to full resolution,
// disparity_to_depth, Backproject, Project, grid_sample(:border), photometric_loss =
// 0.85 mean_c SSIM + 0.15 mean_c |y - x|, minimum over the sources, _apply_mask),
// src/utils.jl:17-43 (SSIM: reflect pad 1, 3x3 mean pools, c1 = 1e-4, c2 = 9e-4, clamp),
// :45-103 (Backproject / Project / normalize), :179-183 (disparity_to_depth).
//
// The loss is a pixel MEAN of per-pixel terms, so the cotangent of every per-pixel term is a
// known constant (or a caller-supplied map): one pass computes the forward value and the whole
// pullback (d disparity, d R, d t) with no saved activations.
//
// Work layout (one wave = one task, no LDS tiles, no barriers):
//   a wave owns 60 output columns x `rows` output rows of one (scale, sample).  Lane l holds
//   column x0 - 2 + l: a 2-column halo on each side.  Halo lanes at the image edge evaluate the
//   REFLECTED column (and rows -1, -2, H, H+1 evaluate rows 1, 2, H-2, H-3), so the reflect-
//   padded 3x3 SSIM windows are plain 3-sums with no edge fix-ups.  The wave walks down its rows:
//     P1 (row r)    warp both sources + read the target: backproject -> project -> border
//                   bilinear gather and the bilinear derivative terms; the warped / target
//                   values go into a 3-row register ring;
//     P2 (row r-1)  the 8 window moments per channel (y, yy, x, xx, xy per source) as vertical
//                   3-sums over the ring (fused multiply-adds), then horizontal 3-sums by DPP
//                   lane shifts -> SSIM and L1 per source, min over sources
//                   (+ automask), and the selected source's adjoint coefficients (A, B, Cc with
//                   d/dx_q = sum over windows p containing q of A_p + x_q B_p + y_q Cc_p),
//                   horizontally 3-summed by DPP with the reflect-adjoint weights;
//     P3 (row r-2)  vertical 3-sum of the coefficient ring -> d/d warped values -> bilinear
//                   derivative -> projection -> d/d depth -> d/d disparity (stored) and the
//                   pose partials (accumulated per lane, reduced per wave at the end).
//   The next row's gathers are issued before P2/P3 of the current row and the disparity two
//   rows ahead (software pipeline); each row's P1 state needed by P3 is parked in the wave's
//   own LDS ring.
// Moments are formed on values shifted by a per-sample constant (the target at the image centre):
// exact algebra, and E[x^2] - E[x]^2 then cancels far less than the reference's unshifted fp32.
// Every sum over a window is taken in a fixed (row, then column) order, so pixels that two waves
// both evaluate (halos) get bit-identical values and decisions.
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "loss_kernels.h"

namespace md2 {
namespace {

constexpr int PW = 60;            // output columns per wave
constexpr int PHOTO_WAVES = 2048; // target tasks per launch: 2 waves per SIMD on 256 CUs

__device__ __forceinline__ float from_left(float v) {    // lane i <- lane i-1 (lane 0 <- 0)
  return __builtin_bit_cast(
      float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x138, 0xf, 0xf, true));
}
__device__ __forceinline__ float from_right(float v) {   // lane i <- lane i+1 (lane 63 <- 0)
  return __builtin_bit_cast(
      float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x130, 0xf, 0xf, true));
}
__device__ __forceinline__ int reflect_clamp(int i, int n) {
  i = i < 0 ? -i : i;
  i = i >= n ? 2 * n - 2 - i : i;
  return min(max(i, 0), n - 1);
}
#ifdef MD2_PHOTO_DIV
__device__ __forceinline__ float frcp(float x) { return 1.f / x; }
#else
__device__ __forceinline__ float frcp(float x) { return __builtin_amdgcn_rcpf(x); }
#endif

#ifndef MD2_PHOTO_NOWPE
#define MD2_PHOTO_WPE __attribute__((amdgpu_waves_per_eu(2)))
#else
#define MD2_PHOTO_WPE
#endif

template <int N_>
using Slot = std::integral_constant<int, N_>;

}  // namespace

// CELLS: also record each owned pixel's bilinear cell / border state (sc.cell_map, parity
// diagnostics).  A separate instantiation so the production kernel's registers are untouched;
// the arithmetic is the same source, so values and decisions are the same.
template <int C, bool CELLS>
__global__ __launch_bounds__(64) MD2_PHOTO_WPE
void photo_stream_kernel(PhotoArgs a, Geom g, PhotoTiling tl) {
  constexpr int NF = 6 * C;       // coefficients per pixel: per source and channel A, B, Cc
  constexpr int NV = 4 * C + 1;   // parked P1 state: Gx0 Gx1 Gy0 Gy1 (C each), depth
  __shared__ float s_v1[3 * NV * 64];

  const int lane = threadIdx.x;
  const int W = g.W, H = g.H;
  int b = blockIdx.x;
  const int tx = b % tl.tiles_x;
  b /= tl.tiles_x;
  const int ty = b % tl.tiles_y;
  b /= tl.tiles_y;
  const int n = b % a.N;
  const int s = b / a.N;
  const PhotoScale sc = a.sc[s];
  const int x0 = tx * PW, y0 = ty * tl.rows;
  const int rows = min(tl.rows, H - y0);
  const int KT = rows + 4;        // P1 rows y0-2 .. y0+rows+1

  const __amdgpu_buffer_rsrc_t rxs =
      make_rsrc(a.x + (long)n * a.x_sample_stride, (uint32_t)(3 * a.x_frame_stride * 4));   // the 3 frames
                                                   // (sample stride 0: MPI planes share them)
  const int dw = sc.dw, dh = sc.dh;
  const __amdgpu_buffer_rsrc_t rdsp =
      make_rsrc(sc.disp + (long)n * dw * dh, (uint32_t)dw * dh * 4u);
  const uint32_t HW4 = (uint32_t)W * H * 4u, W4 = (uint32_t)W * 4u;
  const uint32_t so_t = (uint32_t)(a.target * a.x_frame_stride * 4);
  const uint32_t so_s[2] = {(uint32_t)(a.src0 * a.x_frame_stride * 4),
                            (uint32_t)(a.src1 * a.x_frame_stride * 4)};

  // pixel -> camera map per source (Backproject then Project, src/utils.jl:67-69,99-101), in
  // CENTRED coordinates for fp32 accuracy: pixel p = S (wc, hc, 1) with (wc, hc) = (w, h) - (cx, cy)
  // (1-based w, h), camera cam = T camt with T = [1 0 cx; 0 1 cy; 0 0 1] and Kc = T^-1 K, so
  //   camt = depth * Mc (wc, hc, 1) + Kct,   Mc = Kc R invK S,   Kct = Kc t,
  //   u = cam_0 / (cam_2 + 1e-7) = (camt_0 + cx camt_2) / (camt_2 + 1e-7),
  // and d u / d depth = (mt_0 (Kct_2 + 1e-7) - (Kct_0 - cx 1e-7) mt_2) / (camt_2 + 1e-7)^2 with the
  // depth terms cancelled exactly (mt = Mc (wc, hc, 1)).  For the usual K the maps are near
  // identity and every intermediate is a centred, small quantity.
  // The maps are uniform per (sample, source): formed in fp64 and rounded once, since their
  // rounding is a COHERENT perturbation of every pixel's warp (a tiny pose change), which the
  // cancelling sums downstream (head-bias gradients) would see undiminished.
  const float cxp = g.K[2], cyp = g.K[5];
  float Kc[9];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    Kc[j] = fmaf(-cxp, g.K[6 + j], g.K[j]);
    Kc[3 + j] = fmaf(-cyp, g.K[6 + j], g.K[3 + j]);
    Kc[6 + j] = g.K[6 + j];
  }
  // Mc rows + Kct, invK S rows and the depth-derivative constants in LDS, read where used (keeps
  // ~40 uniform floats out of VGPRs)
  __shared__ float4 s_cam[11];
  if (lane < 11) {
    const double cxd = g.K[2], cyd = g.K[5];
    double Kd[9], iKS[9];                           // Kc and invK S
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      Kd[j] = (double)g.K[j] - cxd * g.K[6 + j];
      Kd[3 + j] = (double)g.K[3 + j] - cyd * g.K[6 + j];
      Kd[6 + j] = g.K[6 + j];
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      iKS[3 * i] = g.invK[3 * i];
      iKS[3 * i + 1] = g.invK[3 * i + 1];
      iKS[3 * i + 2] = (double)g.invK[3 * i] * cxd + (double)g.invK[3 * i + 1] * cyd + g.invK[3 * i + 2];
    }
    float4 v;
    if (lane < 6) {
      const int sp = lane / 3, i = lane % 3;
      const float* rt = a.Rt + ((long)sp * a.N + n) * 12;
      double KR[3], m[3];
#pragma unroll
      for (int j = 0; j < 3; ++j)
        KR[j] = Kd[3 * i] * rt[j] + Kd[3 * i + 1] * rt[3 + j] + Kd[3 * i + 2] * rt[6 + j];
#pragma unroll
      for (int j = 0; j < 3; ++j) m[j] = KR[0] * iKS[j] + KR[1] * iKS[3 + j] + KR[2] * iKS[6 + j];
      const double kt = Kd[3 * i] * rt[9] + Kd[3 * i + 1] * rt[10] + Kd[3 * i + 2] * rt[11];
      v = make_float4((float)m[0], (float)m[1], (float)m[2], (float)kt);
    } else if (lane < 9) {
      const int r = lane - 6;
      v = make_float4((float)iKS[3 * r], (float)iKS[3 * r + 1], (float)iKS[3 * r + 2], 0.f);
    } else {
      const int q = lane - 9;
      const float* rt = a.Rt + ((long)q * a.N + n) * 12;
      double kt[3];
#pragma unroll
      for (int i = 0; i < 3; ++i) kt[i] = Kd[3 * i] * rt[9] + Kd[3 * i + 1] * rt[10] + Kd[3 * i + 2] * rt[11];
      v = make_float4((float)(kt[0] - cxd * 1e-7), (float)(kt[1] - cyd * 1e-7), (float)(kt[2] + 1e-7), 0.f);
    }
    s_cam[lane] = v;
  }
  __syncthreads();
  auto cam_const = [&](int idx) {
    asm volatile("" : "+v"(idx));
    return s_cam[idx];
  };
  // moment shift: the target at the image centre, per channel -- the SAME for every wave of the
  // sample, so the halo rows / columns two waves both evaluate come out bit-identical (the
  // per-pixel argmin and clamp decisions must not depend on which wave made them)
  float cc[C];
  {
    const int cx = W / 2, cy = H / 2;
    const float* tp = a.x + (long)n * a.x_sample_stride + (long)a.target * a.x_frame_stride;
#pragma unroll
    for (int c = 0; c < C; ++c) cc[c] = tp[(long)c * W * H + (long)cy * W + cx];
#ifdef MD2_PHOTO_NOSHIFT
#pragma unroll
    for (int c = 0; c < C; ++c) cc[c] = 0.f;
#endif
  }

  // per-lane constants
  const int col = x0 - 2 + lane;
  const int colr = reflect_clamp(col, W);
  const float wcol = (float)(colr + 1) - cxp;       // centred 1-based pixel grid (src/utils.jl:51-55)
  const bool cvalid = col >= 0 && col < W;          // a real window centre
  const bool outl = lane >= 2 && lane < 2 + PW && col < W;   // owned output column
  const float wl = (col == 1) ? 2.f : 1.f;          // reflect adjoint: x[-1] = x[1]
  const float wr = (col == W - 2) ? 2.f : 1.f;      //                  x[W] = x[W-2]
  // upsample_bilinear to full resolution, align_corners (training.jl:45); the full-resolution
  // scale takes the same path with zero weights (exact)
  const float usx = sc.rx * (float)colr;
  const int ux0 = min((int)usx, dw - 1);
  const float ufx = usx - (float)ux0;
  // the two column taps ux0, min(ux0 + 1, dw - 1) as ONE 8-byte load at min(ux0, dw - 2): at the
  // last column (ux0 = dw - 1) both taps are the pair's right element (dw >= 2)
  const int uxp = min(ux0, dw - 2);
  const bool uedge = ux0 == dw - 1;
  const float kS = a.wloss * (0.85f / (float)C) * (1.f / 9.f);
  const float kL = a.wloss * (0.15f / (float)C);
  const float inv9 = 1.f / 9.f, c1 = 1e-4f, c2 = 9e-4f;
  const float Wm1 = (float)(W - 1), Hm1 = (float)(H - 1);

  // ---- pipeline registers --------------------------------------------------------------------
  float dA[4] = {0.f, 0.f, 0.f, 0.f}, fyA = 0.f;   // stage A: disparity loads (2 rows ahead)
  float gv[2][C][4], tv[C];                         // stage B: gathers (1 row ahead)
  float bfx[2], bfy[2], bmx[2], bmy[2], bdepth = 0.f;
  float xr[3][2][C], yr[3][C];                      // shifted warped / target values, rows r-2..r
  float ch[3][NF];                                  // horizontal coefficient sums, rows r-3..r-1
  float acc[24];                                    // per source: sum dcam_i X_j (9), sum dcam_i (3)
#pragma unroll
  for (int i = 0; i < 24; ++i) acc[i] = 0.f;
  float lsum = 0.f;
  int selc = -1;                                    // P2 decision of the last P2 row
  float gpc = 0.f;                                  // its cotangent

  auto issue_disp = [&](int R) {
    const float sy = sc.ry * (float)reflect_clamp(R, H);
    const int uy0 = min((int)sy, dh - 1), uy1 = min(uy0 + 1, dh - 1);
    fyA = sy - (float)uy0;
    const float2 t = bload2_s(rdsp, (uint32_t)(uy0 * dw + uxp) * 4u, 0u);
    const float2 b = bload2_s(rdsp, (uint32_t)(uy1 * dw + uxp) * 4u, 0u);
    dA[0] = t.x;
    dA[1] = t.y;
    dA[2] = b.x;
    dA[3] = b.y;
  };

  auto issue_gathers = [&](int R) {
    const int Rr = reflect_clamp(R, H);
    const float h = (float)(Rr + 1) - cyp;
    const float d00 = uedge ? dA[1] : dA[0], d10 = uedge ? dA[3] : dA[2];
    const float dtop = fmaf(ufx, dA[1] - d00, d00);
    const float dbot = fmaf(ufx, dA[3] - d10, d10);
    const float d = fmaf(fyA, dbot - dtop, dtop);
    const float depth = frcp(fmaf(d, g.disp_range, g.min_disp));   // disparity_to_depth
    bdepth = depth;
#pragma unroll
    for (int sp = 0; sp < 2; ++sp) {
      float cam[3];
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const float4 mk = cam_const(3 * sp + i);
        cam[i] = fmaf(depth, fmaf(mk.x, wcol, fmaf(mk.y, h, mk.z)), mk.w);
      }
      const float rc = frcp(cam[2] + 1e-7f);
      // normalize + grid_sample unnormalise (align_corners) collapse to u - 1 (0-based)
      const float c2r = cam[2] * rc;
      const float ix = fmaf(cam[0], rc, fmaf(cxp, c2r, -1.f));
      const float iy = fmaf(cam[1], rc, fmaf(cyp, c2r, -1.f));
      const float xc = fminf(fmaxf(ix, 0.f), Wm1), yc = fminf(fmaxf(iy, 0.f), Hm1);  // :border
      const int xi = min((int)xc, W - 2), yi = min((int)yc, H - 2);
      bfx[sp] = xc - (float)xi;
      bfy[sp] = yc - (float)yi;
      bmx[sp] = (ix > 0.f && ix < Wm1) ? 1.f : 0.f;   // clamp gradient masks
      bmy[sp] = (iy > 0.f && iy < Hm1) ? 1.f : 0.f;
      if (CELLS && outl && R >= y0 && R < y0 + rows) {          // parity diagnostics only
        const int fx = ix > 0.f ? (ix < Wm1 ? 0 : 2) : 1, fy = iy > 0.f ? (iy < Hm1 ? 0 : 2) : 1;
        sc.cell_map[(((long)sp * a.N + n) * H + R) * W + col] =
            xi | (yi << PHOTO_CELL_YSHIFT) | (fx << PHOTO_CELL_FXSHIFT) | (fy << PHOTO_CELL_FYSHIFT);
      }
      // xi <= W-2, yi <= H-2: the right / lower taps are always +1 / +W, so each row pair of
      // taps is ONE 8-byte load (half the gather instructions of four dword loads)
      const uint32_t vo = (uint32_t)(yi * W + xi) * 4u;
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const uint32_t so = so_s[sp] + (uint32_t)c * HW4;
        const float2 t = bload2_s(rxs, vo, so), b = bload2_s(rxs, vo, so + W4);
        gv[sp][c][0] = t.x;
        gv[sp][c][1] = t.y;
        gv[sp][c][2] = b.x;
        gv[sp][c][3] = b.y;
      }
    }
    const uint32_t to = (uint32_t)(Rr * W + colr) * 4u;
#pragma unroll
    for (int c = 0; c < C; ++c) tv[c] = bload_s(rxs, to, so_t + (uint32_t)c * HW4);
  };

  // P1 of row R (its gathers have landed): values -> ring slot S, derivative terms -> LDS slot vs
  auto finish_p1 = [&](auto Sc, int vs) {
    constexpr int S = decltype(Sc)::value;
    float* v1 = s_v1 + vs * NV * 64 + lane;
#pragma unroll
    for (int c = 0; c < C; ++c) yr[S][c] = tv[c] - cc[c];
#pragma unroll
    for (int sp = 0; sp < 2; ++sp) {
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const float v00 = gv[sp][c][0], v01 = gv[sp][c][1], v10 = gv[sp][c][2], v11 = gv[sp][c][3];
        const float d0 = v01 - v00, d1 = v11 - v10;
        const float top = fmaf(bfx[sp], d0, v00), bot = fmaf(bfx[sp], d1, v10);
        const float dv = bot - top;
        xr[S][sp][c] = fmaf(bfy[sp], dv, top) - cc[c];
        v1[(sp * C + c) * 64] = fmaf(bfy[sp], d1 - d0, d0) * bmx[sp];      // d val / d ix
        v1[(2 * C + sp * C + c) * 64] = dv * bmy[sp];                      // d val / d iy
      }
    }
    v1[(4 * C) * 64] = bdepth;
  };

  // P2 head for row p (window rows p-1, p, p+1 = all three ring slots; p in slot S+2): SSIM and
  // L1 per source, the adjoint coefficients of both sources (cf), min over sources -> sel
  auto p2_head = [&](auto Sc, int p, float am, float gp, float (&cf)[2][C][3]) -> int {
    constexpr int S = decltype(Sc)::value;
    constexpr int SP = (S + 2) % 3;                // ring slots in row order: S+1, S+2 (= p), S
    constexpr int S0 = (S + 1) % 3;
    // rows -1 and H are not window centres: zero coefficients (reflect adjoint, P3)
    const float kp = (cvalid && p >= 0 && p < H) ? kS * gp : 0.f;
    float loss[2] = {0.f, 0.f};
#pragma unroll
    for (int c = 0; c < C; ++c) {
      // window moments: vertical 3-sums over the ring, then horizontal 3-sums across lanes
      float m[8];
      {
        const float y0v = yr[S0][c], y1v = yr[SP][c], y2v = yr[S][c];
        m[0] = y0v + y1v + y2v;
        m[1] = fmaf(y0v, y0v, fmaf(y1v, y1v, y2v * y2v));
#pragma unroll
        for (int sp = 0; sp < 2; ++sp) {
          const float a0 = xr[S0][sp][c], a1 = xr[SP][sp][c], a2 = xr[S][sp][c];
          m[2 + 3 * sp] = a0 + a1 + a2;
          m[3 + 3 * sp] = fmaf(a0, a0, fmaf(a1, a1, a2 * a2));
          m[4 + 3 * sp] = fmaf(a0, y0v, fmaf(a1, y1v, a2 * y2v));
          loss[sp] = fmaf(0.15f / (float)C, fabsf(yr[SP][c] - xr[SP][sp][c]), loss[sp]);  // L1, centre
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) m[k] = m[k] + from_left(m[k]) + from_right(m[k]);
      }
      const float my = m[0] * inv9;                 // shifted mean of the target window
      const float mty = fmaf(m[0], inv9, cc[c]);
      const float vy = fmaf(m[1], inv9, -my * my);
      const float two_mty = 2.f * mty;
      const float B1y = fmaf(mty, mty, c1), B2y = vy + c2;
#pragma unroll
      for (int sp = 0; sp < 2; ++sp) {
        const float mx = m[2 + 3 * sp] * inv9;
        const float mtx = fmaf(m[2 + 3 * sp], inv9, cc[c]);
        const float vx = fmaf(m[3 + 3 * sp], inv9, -mx * mx);
        const float cxy = fmaf(m[4 + 3 * sp], inv9, -mx * my);
        const float A1 = fmaf(mtx, two_mty, c1), A2 = fmaf(2.f, cxy, c2);
        const float B1 = fmaf(mtx, mtx, B1y), B2 = vx + B2y;
        const float rd = frcp(B1 * B2);
        const float r = (A1 * A2) * rd;
        const float val = fmaf(-0.5f, r, 0.5f);
        const float sv = fminf(fmaxf(val, 0.f), 1.f);
        loss[sp] = fmaf(0.85f / (float)C, sv, loss[sp]);
        // d loss/d (mu_x, var_x, cov_xy) of this window (clamp gradient 1 inside [0, 1]); the
        // adjoint at q is g_m + 2 g_v (x_q - mu_x) + g_c (y_q - mu_y) = A + x_q B + y_q Cc
        const float t1 = (val == sv) ? kp * rd : 0.f;
        const float gm = t1 * fmaf(r * mtx, B2, -mty * A2);
        const float gv2 = (r * t1) * B1;            // 2 d/d var_x
        const float gc = -t1 * A1;                  //   d/d cov_xy
        cf[sp][c][0] = fmaf(-gv2, mx, fmaf(-gc, my, gm));
        cf[sp][c][1] = gv2;
        cf[sp][c][2] = gc;
      }
      __builtin_amdgcn_sched_barrier(0);            // one channel's window state live at a time
    }
    // minimum over sources (first argmin), then the automask (wins ties), training.jl:60-62
    int sel = (loss[1] < loss[0]) ? 1 : 0;
    float lmin = sel ? loss[1] : loss[0];
    if (a.automask && !(lmin < am)) {
      sel = -1;
      lmin = am;
    }
    const bool own = p >= y0 && p < y0 + rows && outl;
    lsum += own ? lmin : 0.f;
    if (own) {
      const long qq = ((long)n * H + p) * W + col;
      if (sc.loss_map) sc.loss_map[qq] = lmin;
      if (sc.sel_map) sc.sel_map[qq] = (signed char)sel;
    }
    return sel;
  };

  // P2 tail (masked coefficients of row q+1, horizontally 3-summed -> ch[S]) fused with P3 of
  // row q (coefficient rows q-1, q, q+1 in ch slots S+1, S+2, S; values in ring slot S+1; P1
  // derivative terms in LDS slot S+1): d/d warped values -> projection pullback
  auto p2_tail_p3 = [&](auto Sc, int sel, const float (&cf)[2][C][3], int q, bool live3, int selq,
                        float gpq) {
    constexpr int S = decltype(Sc)::value;
    constexpr int SA = (S + 1) % 3, SB = (S + 2) % 3;
    const float wa = (q == 1) ? 2.f : 1.f, wb = (q == H - 2) ? 2.f : 1.f;
    const float* v1 = s_v1 + SA * NV * 64 + lane;
    const float kLq = kL * gpq;
    float gx[2] = {0.f, 0.f}, gy[2] = {0.f, 0.f};
    unsigned l1bits = 0;                           // CELLS only: the L1 branches taken at q
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const float yq = yr[SA][c];
      // L1 pullback at q for its selected source: d|y - x|/dx = sign(x - y), abs'(0) = 0
      const float xs = (selq == 1) ? xr[SA][1][c] : xr[SA][0][c];
      const float df = xs - yq;
      const float t = df > 0.f ? kLq : (df < 0.f ? -kLq : 0.f);
      if (CELLS) l1bits |= (df > 0.f ? 2u : (df < 0.f ? 1u : 3u)) << (PHOTO_CELL_L1SHIFT + 2 * c);
#pragma unroll
      for (int sp = 0; sp < 2; ++sp) {
        const int f = (sp * C + c) * 3;
        float sum[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          const float F = (sel == sp) ? cf[sp][c][k] : 0.f;
          ch[S][f + k] = fmaf(wl, from_left(F), fmaf(wr, from_right(F), F));
          sum[k] = fmaf(wa, ch[SA][f + k], fmaf(wb, ch[S][f + k], ch[SB][f + k]));
        }
        float dx = fmaf(xr[SA][sp][c], sum[1], fmaf(yq, sum[2], sum[0]));
        dx += (selq == sp) ? t : 0.f;
        gx[sp] = fmaf(dx, v1[(sp * C + c) * 64], gx[sp]);
        gy[sp] = fmaf(dx, v1[(2 * C + sp * C + c) * 64], gy[sp]);
      }
    }
    const bool live = live3 && outl;
    if (CELLS && live && selq >= 0) {              // parity diagnostics only (same lane wrote it)
      int* cm = sc.cell_map + (((long)selq * a.N + n) * H + q) * W + col;
      *cm = (int)((unsigned)*cm | l1bits);
    }
    const float depth = v1[(4 * C) * 64];
    const float h = (float)(q + 1) - cyp;
    float X[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const float4 ik = cam_const(6 + i);
      X[i] = depth * fmaf(ik.x, wcol, fmaf(ik.y, h, ik.z));
    }
    float ddepth = 0.f;
#pragma unroll
    for (int sp = 0; sp < 2; ++sp) {
      const float ggx = live ? gx[sp] : 0.f, ggy = live ? gy[sp] : 0.f;
      float m[3], cam[3];
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const float4 mk = cam_const(3 * sp + i);
        m[i] = fmaf(mk.x, wcol, fmaf(mk.y, h, mk.z));
        cam[i] = fmaf(depth, m[i], mk.w);
      }
      const float rc = frcp(cam[2] + 1e-7f);
      const float4 kd = cam_const(9 + sp);
      float dc[3];                                 // d loss / d camt
      dc[0] = ggx * rc;
      dc[1] = ggy * rc;
      dc[2] = -fmaf(ggx, cam[0], ggy * cam[1]) * rc * rc;
      const float rc2 = rc * rc;
      ddepth = fmaf(rc2, fmaf(ggx, fmaf(m[0], kd.z, -kd.x * m[2]), ggy * fmaf(m[1], kd.z, -kd.y * m[2])), ddepth);
#pragma unroll
      for (int i = 0; i < 3; ++i) {
#pragma unroll
        for (int j = 0; j < 3; ++j) acc[12 * sp + 3 * i + j] = fmaf(dc[i], X[j], acc[12 * sp + 3 * i + j]);
        acc[12 * sp + 9 + i] += dc[i];
      }
    }
    // depth = 1/(disp*range + min_disp)  =>  d depth/d disp = -range * depth^2
    if (live) sc.g_disp[((long)n * H + q) * W + col] = -ddepth * g.disp_range * depth * depth;
  };

  // one row step: P1 of row R = y0-2+k (ring / LDS slot S = k % 3), P2 of row R-1, P3 of R-2.
  // Every step runs all three phases; the first steps' P2/P3 and the padding steps past KT
  // (KT rounded up to a multiple of 3) work on zero-initialised or clamped rows and are
  // masked out of every output, which keeps the loop body one straight-line block.
  auto step = [&](auto Sc, int k) {
    constexpr int S = decltype(Sc)::value;
    const int R = y0 - 2 + k;
    const int p = min(max(R - 1, 0), H - 1);
    float am = 0.f, gp = 1.f;
    if (a.automask) am = a.automask[((long)n * H + p) * W + colr];
    if (a.gmap) gp = a.gmap[((long)n * H + p) * W + colr];
    finish_p1(Sc, S);
    __builtin_amdgcn_sched_barrier(0);
    float cf[2][C][3];
    const int sel = p2_head(Sc, R - 1, am, gp, cf);
    // the next row's loads may interleave with the SSIM arithmetic (measured: 147 -> 136 us)
    issue_gathers(R + 1);                          // rows past the tile are harmless (clamped)
    issue_disp(R + 2);
    p2_tail_p3(Sc, sel, cf, R - 2, k >= 4 && k < KT, selc, gpc);
    selc = sel;
    gpc = gp;
    __builtin_amdgcn_sched_barrier(0);             // steps do not interleave (register pressure)
  };

  // zero rings and parked state: the first steps read them before P1 has filled them
#pragma unroll
  for (int r = 0; r < 3; ++r) {
#pragma unroll
    for (int c = 0; c < C; ++c) {
      yr[r][c] = 0.f;
      xr[r][0][c] = 0.f;
      xr[r][1][c] = 0.f;
    }
#pragma unroll
    for (int f = 0; f < NF; ++f) ch[r][f] = 0.f;
  }
  for (int i = lane; i < 3 * NV * 64; i += 64) s_v1[i] = 1.f;
  issue_disp(y0 - 2);
  issue_gathers(y0 - 2);
  issue_disp(y0 - 1);
  const int KTp = (KT + 2) / 3 * 3;
  for (int k = 0; k < KTp; k += 3) {
    step(Slot<0>{}, k);
    step(Slot<1>{}, k + 1);
    step(Slot<2>{}, k + 2);
  }

  // ---- per-wave partials: loss sum, then per source dR = Kc^T sum(dcamt X^T), dt = Kc^T sum(dcamt)
  lsum = wave_sum_dpp(lsum);
#pragma unroll
  for (int i = 0; i < 24; ++i) acc[i] = wave_sum_dpp(acc[i]);
  if (lane == 0) {
    float* out = sc.partials + (((long)n * tl.tiles_y + ty) * tl.tiles_x + tx) * 25;
    out[0] = lsum;
#pragma unroll
    for (int sp = 0; sp < 2; ++sp) {
#pragma unroll
      for (int k = 0; k < 3; ++k) {
#pragma unroll
        for (int l = 0; l < 3; ++l)
          out[1 + 12 * sp + 3 * k + l] =
              fmaf(Kc[k], acc[12 * sp + l], fmaf(Kc[3 + k], acc[12 * sp + 3 + l], Kc[6 + k] * acc[12 * sp + 6 + l]));
        out[1 + 12 * sp + 9 + k] =
            fmaf(Kc[k], acc[12 * sp + 9], fmaf(Kc[3 + k], acc[12 * sp + 10], Kc[6 + k] * acc[12 * sp + 11]));
      }
    }
  }
}

PhotoTiling photo_tiling(int W, int H, int N, int nscales) {
  PhotoTiling t;
  t.tiles_x = cdiv(W, PW);
  static const int target = std::max(1, tuning_knob("MD2_PHOTO_WAVES", PHOTO_WAVES));
  const double per_row = (double)nscales * N * t.tiles_x;
  int ty = (int)(target / per_row + 0.5);
  ty = std::max(1, std::min(ty, cdiv(H, 8)));
  t.rows = cdiv(H, ty);
  t.tiles_y = cdiv(H, t.rows);
  return t;
}

long photometric_blocks(int W, int H, int N, int nscales) {
  return (long)photo_tiling(W, H, N, nscales).per_scale() * N;
}

int launch_photometric(const PhotoArgs& a, const Geom& g, int C, hipStream_t st) {
  if (a.nscales < 1 || a.nscales > MAX_SCALES) {
    set_error("photometric: nscales out of range");
    return MD2_EINVAL;
  }
  if (g.W < 3 || g.H < 3) {
    set_error("photometric: image must be at least 3x3");
    return MD2_EINVAL;
  }
  for (int s = 0; s < a.nscales; ++s)
    if (a.sc[s].dw < 2) {   // the disparity column taps are one 8-byte pair load
      set_error("photometric: disparity maps must be at least 2 columns wide");
      return MD2_EINVAL;
    }
  const PhotoTiling tl = photo_tiling(g.W, g.H, a.N, a.nscales);
  const long blocks = tl.per_scale() * a.N * a.nscales;
  bool cells = false;
  for (int s = 0; s < a.nscales; ++s) cells |= a.sc[s].cell_map != nullptr;
  if (cells) {
    for (int s = 0; s < a.nscales; ++s)
      if (!a.sc[s].cell_map) {
        set_error("photometric: cell_map must be given for every scale or none");
        return MD2_EINVAL;
      }
    if (g.W > PHOTO_CELL_MAXDIM || g.H > PHOTO_CELL_MAXDIM) {
      set_error("photometric: cell_map packs 11-bit cells (w, h <= 2048)");
      return MD2_EINVAL;
    }
  }
  // the packed-fp32 form (photo2.hip, bit-identical); MD2_PHOTO_V1=1 (read per launch, for the
  // A/B and the bit-identity test) runs this file's scalar kernel
  const char* v1 = std::getenv("MD2_PHOTO_V1");
  if (!(v1 && v1[0] == '1')) return launch_photo2(a, g, tl, C, cells, blocks, st);
  const dim3 grid((unsigned)blocks), block(64);
  if (C == 3 && !cells)
    hipLaunchKernelGGL((photo_stream_kernel<3, false>), grid, block, 0, st, a, g, tl);
  else if (C == 3)
    hipLaunchKernelGGL((photo_stream_kernel<3, true>), grid, block, 0, st, a, g, tl);
  else if (C == 1 && !cells)
    hipLaunchKernelGGL((photo_stream_kernel<1, false>), grid, block, 0, st, a, g, tl);
  else if (C == 1)
    hipLaunchKernelGGL((photo_stream_kernel<1, true>), grid, block, 0, st, a, g, tl);
  else {
    set_error("photometric: channels must be 1 or 3");
    return MD2_ENOTSUP;
  }
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

}  // namespace md2
