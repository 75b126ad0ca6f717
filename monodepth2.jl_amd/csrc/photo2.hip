// Fused warp + SSIM + L1 photometric loss, forward AND pullback, every scale in one launch --
// round-6 form (gfx950): the per-source arithmetic of photo.hip on PACKED fp32.
//
// Same algorithm, same operations in the same order as photo_stream_kernel (photo.hip, whose
// header describes the work layout: a wave owns 60 output columns of a row band and walks its
// rows through P1 (warp + gathers), P2 (window moments, SSIM, min over sources, adjoint
// coefficients) and P3 (coefficient sums -> projection pullback)), so the outputs are
// bit-identical to it (tests/test_gpu_photo2.py).  What changes is how the VALU issues it:
//
//  * the two SOURCES ride the two halves of v_pk_{fma,mul,add}_f32 (one 4-cycle issue for both):
//    the projection of P1, the window moments / SSIM / adjoint coefficients of P2, the
//    coefficient sums, the bilinear derivative and the projection pullback of P3 -- every
//    per-source quantity is an `f2` = (source 0, source 1).  Only the gathers, the per-source
//    compares / selects / conversions / clamps, the reciprocals and the DPP lane shifts stay
//    scalar.  Uniform operands (pixel coordinates, target moments, weights) are broadcast by
//    op_sel_hi at no cost;
//  * the per-channel scheduling fence of P2 is gone: the three channels' chains interleave,
//    which hides the one wait state a packed result needs before a dependent packed op;
//  * the reflect-adjoint weights of the horizontal coefficient sums are folded into the value a
//    lane SHIPS (x2 at columns 0 and W-1, exact) so each sum is two v_add_f32_dpp instead of two
//    DPP moves and two FMAs -- the same single rounding per add as fma(w, L, fma(w, R, F));
//  * phases run only where their rows exist: the first two row steps are P1 only, the third and
//    fourth skip P3, and the loop leaves at the band's last row (photo.hip ran every phase on
//    every step of a 3-step-padded loop and masked the outputs).
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "loss_kernels.h"

namespace md2 {
namespace {

typedef float f2 __attribute__((ext_vector_type(2)));

constexpr int PW = 60;            // output columns per wave (photo.hip)

__device__ __forceinline__ f2 fma2(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f2 bc(float s) { return (f2){s, s}; }
__device__ __forceinline__ float from_left(float v) {    // lane i <- lane i-1 (lane 0 <- 0)
  return __builtin_bit_cast(
      float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x138, 0xf, 0xf, true));
}
__device__ __forceinline__ float from_right(float v) {   // lane i <- lane i+1 (lane 63 <- 0)
  return __builtin_bit_cast(
      float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x130, 0xf, 0xf, true));
}
// 3-lane window sums in photo.hip's order, (v + left) + right, for NV values at once: all first
// adds, a scheduling fence, then all second adds -- a v_add_f32_dpp reading a VGPR the previous
// VALU wrote costs two wait states (s_nop 1), and this order keeps every such read NV
// instructions away from its write
template <int NV>
__device__ __forceinline__ void hsum3_n(float (&v)[NV]) {
  float t[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) t[i] = v[i] + from_left(v[i]);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int i = 0; i < NV; ++i) v[i] = t[i] + from_right(v[i]);
}
__device__ __forceinline__ int reflect_clamp(int i, int n) {
  i = i < 0 ? -i : i;
  i = i >= n ? 2 * n - 2 - i : i;
  return min(max(i, 0), n - 1);
}
__device__ __forceinline__ float frcp(float x) { return __builtin_amdgcn_rcpf(x); }
// a wave-uniform value held in a VGPR (the kernel is short of SGPRs -- the spills cost VALU
// v_readlane restores in the row loop -- and has VGPRs to spare)
__device__ __forceinline__ float vreg(float x) {
  asm volatile("" : "+v"(x));
  return x;
}
__device__ __forceinline__ f2 frcp(f2 x) { return (f2){frcp(x.x), frcp(x.y)}; }

template <int N_>
using Slot = std::integral_constant<int, N_>;

// which phases a row step runs (P1 always)
constexpr int PH_P2 = 1, PH_P3 = 2, PH_ALL = 3;

}  // namespace

template <int C, bool CELLS>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2)))
void photo2_kernel(PhotoArgs a, Geom g, PhotoTiling tl) {
  constexpr int NP = 2 * C;       // parked P1 pairs: (d val / d ix, d val / d iy) per channel
  __shared__ f2 s_v2[3 * NP * 64];
  __shared__ float s_dep[3 * 64];

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
      make_rsrc(a.x + (long)n * a.x_sample_stride, (uint32_t)(3 * a.x_frame_stride * 4));
  const int dw = sc.dw, dh = sc.dh;
  const __amdgpu_buffer_rsrc_t rdsp =
      make_rsrc(sc.disp + (long)n * dw * dh, (uint32_t)dw * dh * 4u);
  const uint32_t HW4 = (uint32_t)W * H * 4u, W4 = (uint32_t)W * 4u;
  const uint32_t so_t = (uint32_t)(a.target * a.x_frame_stride * 4);
  const uint32_t so_s[2] = {(uint32_t)(a.src0 * a.x_frame_stride * 4),
                            (uint32_t)(a.src1 * a.x_frame_stride * 4)};

  // camera maps of both sources (photo.hip: centred coordinates, formed in fp64, rounded once),
  // stored as (source 0, source 1) pairs: s_pk[4 i + {0,1,2,3}] = Mc row i (x, y, z) and Kct_i,
  // s_pk[12 + {0,1,2}] = the depth-derivative constants (kd.x, kd.y, kd.z); s_iks[i] = invK S row i
  const float cxp = vreg(g.K[2]), cyp = vreg(g.K[5]);
  float Kc[9];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    Kc[j] = fmaf(-cxp, g.K[6 + j], g.K[j]);
    Kc[3 + j] = fmaf(-cyp, g.K[6 + j], g.K[3 + j]);
    Kc[6 + j] = g.K[6 + j];
  }
  __shared__ f2 s_pk[16];
  __shared__ float4 s_iks[3];
  if (lane < 11) {
    const double cxd = g.K[2], cyd = g.K[5];
    double Kd[9], iKS[9];
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
      float* pk = reinterpret_cast<float*>(s_pk);
      pk[2 * (4 * i + 0) + sp] = (float)m[0];
      pk[2 * (4 * i + 1) + sp] = (float)m[1];
      pk[2 * (4 * i + 2) + sp] = (float)m[2];
      pk[2 * (4 * i + 3) + sp] = (float)kt;
    } else if (lane < 9) {
      const int r = lane - 6;
      s_iks[r] = make_float4((float)iKS[3 * r], (float)iKS[3 * r + 1], (float)iKS[3 * r + 2], 0.f);
    } else {
      const int q = lane - 9;
      const float* rt = a.Rt + ((long)q * a.N + n) * 12;
      double kt[3];
#pragma unroll
      for (int i = 0; i < 3; ++i) kt[i] = Kd[3 * i] * rt[9] + Kd[3 * i + 1] * rt[10] + Kd[3 * i + 2] * rt[11];
      float* pk = reinterpret_cast<float*>(s_pk);
      pk[2 * 12 + q] = (float)(kt[0] - cxd * 1e-7);
      pk[2 * 13 + q] = (float)(kt[1] - cyd * 1e-7);
      pk[2 * 14 + q] = (float)(kt[2] + 1e-7);
    }
  }
  __syncthreads();
  // read where used (keeps the ~40 uniform floats out of VGPRs)
  // an opaque LDS base per use site: constant-offset ds_reads, never hoisted out of the row loop
  auto opaque0 = [&]() {
    int z = 0;
    asm volatile("" : "+v"(z));
    return z;
  };
  auto pk_base = [&]() { return s_pk + opaque0(); };
  auto iks_base = [&]() { return s_iks + opaque0(); };
  float cc[C];
  {
    const int cx = W / 2, cy = H / 2;
    const float* tp = a.x + (long)n * a.x_sample_stride + (long)a.target * a.x_frame_stride;
#pragma unroll
    for (int c = 0; c < C; ++c) cc[c] = vreg(tp[(long)c * W * H + (long)cy * W + cx]);
  }

  // per-lane constants
  const int col = x0 - 2 + lane;
  const int colr = reflect_clamp(col, W);
  const float wcol = (float)(colr + 1) - cxp;
  const bool cvalid = col >= 0 && col < W;
  const bool outl = lane >= 2 && lane < 2 + PW && col < W;
  // reflect adjoint x[-1] = x[1], x[W] = x[W-2]: the window centred at column 0 counts column 1
  // twice (likewise W-1 / W-2) -- folded into the value lanes 0 / W-1 ship to their neighbours
  const float wship = (col == 0 || col == W - 1) ? 2.f : 1.f;
  const float usx = sc.rx * (float)colr;
  const int ux0 = min((int)usx, dw - 1);
  const float ufx = usx - (float)ux0;
  const int uxp = min(ux0, dw - 2);
  const bool uedge = ux0 == dw - 1;
  const float kS = a.wloss * (0.85f / (float)C) * (1.f / 9.f);
  const float kL = a.wloss * (0.15f / (float)C);
  const float inv9 = vreg(1.f / 9.f), c1 = vreg(1e-4f), c2 = vreg(9e-4f), eps7 = vreg(1e-7f);
  const float Wm1 = vreg((float)(W - 1)), Hm1 = vreg((float)(H - 1));
  const float disp_range = vreg(g.disp_range), min_disp = vreg(g.min_disp);

  // ---- pipeline registers --------------------------------------------------------------------
  float dA[4] = {0.f, 0.f, 0.f, 0.f}, fyA = 0.f;
  float gv[2][C][4], tv[C];
  float bfx[2], bfy[2], bmx[2], bmy[2], bdepth = 0.f;
  f2 xr[3][C];                                      // shifted warped values (source 0, 1)
  float yr[3][C];                                   // shifted target values
  f2 ch[3][C][3];                                   // horizontal coefficient sums, rows r-3..r-1
  f2 acc[12];                                       // sum dcam_i X_j (9), sum dcam_i (3)
#pragma unroll
  for (int i = 0; i < 12; ++i) acc[i] = bc(0.f);
  float lsum = 0.f;
  int selc = -1;
  float gpc = 0.f;

  auto issue_disp = [&](int R) {
    const float sy = sc.ry * (float)reflect_clamp(R, H);
    const int uy0 = min((int)sy, dh - 1), uy1 = min(uy0 + 1, dh - 1);
    fyA = sy - (float)uy0;
    const float2 t = bload2_s(rdsp, (uint32_t)(uy0 * dw + uxp) * 4u, 0u);
    const float2 bb = bload2_s(rdsp, (uint32_t)(uy1 * dw + uxp) * 4u, 0u);
    dA[0] = t.x;
    dA[1] = t.y;
    dA[2] = bb.x;
    dA[3] = bb.y;
  };

  auto issue_gathers = [&](int R) {
    const int Rr = reflect_clamp(R, H);
    const float h = (float)(Rr + 1) - cyp;
    const float d00 = uedge ? dA[1] : dA[0], d10 = uedge ? dA[3] : dA[2];
    const float dtop = fmaf(ufx, dA[1] - d00, d00);
    const float dbot = fmaf(ufx, dA[3] - d10, d10);
    const float d = fmaf(fyA, dbot - dtop, dtop);
    const float depth = frcp(fmaf(d, disp_range, min_disp));
    bdepth = depth;
    f2 cam[3];
    const f2* pkc = pk_base();
#pragma unroll
    for (int i = 0; i < 3; ++i)
      cam[i] = fma2(bc(depth), fma2(pkc[4 * i], bc(wcol), fma2(pkc[4 * i + 1], bc(h), pkc[4 * i + 2])),
                    pkc[4 * i + 3]);
    const f2 rc = frcp(cam[2] + bc(eps7));
    const f2 c2r = cam[2] * rc;
    const f2 ix = fma2(cam[0], rc, fma2(bc(cxp), c2r, bc(-1.f)));
    const f2 iy = fma2(cam[1], rc, fma2(bc(cyp), c2r, bc(-1.f)));
#pragma unroll
    for (int sp = 0; sp < 2; ++sp) {
      const float ixs = sp ? ix.y : ix.x, iys = sp ? iy.y : iy.x;
      const float xc = fminf(fmaxf(ixs, 0.f), Wm1), yc = fminf(fmaxf(iys, 0.f), Hm1);
      const int xi = min((int)xc, W - 2), yi = min((int)yc, H - 2);
      bfx[sp] = xc - (float)xi;
      bfy[sp] = yc - (float)yi;
      bmx[sp] = (ixs > 0.f && ixs < Wm1) ? 1.f : 0.f;
      bmy[sp] = (iys > 0.f && iys < Hm1) ? 1.f : 0.f;
      if (CELLS && outl && R >= y0 && R < y0 + rows) {
        const int fx = ixs > 0.f ? (ixs < Wm1 ? 0 : 2) : 1, fy = iys > 0.f ? (iys < Hm1 ? 0 : 2) : 1;
        sc.cell_map[(((long)sp * a.N + n) * H + R) * W + col] =
            xi | (yi << PHOTO_CELL_YSHIFT) | (fx << PHOTO_CELL_FXSHIFT) | (fy << PHOTO_CELL_FYSHIFT);
      }
      const uint32_t vo = (uint32_t)(yi * W + xi) * 4u;
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const uint32_t so = so_s[sp] + (uint32_t)c * HW4;
        const float2 t = bload2_s(rxs, vo, so), bb = bload2_s(rxs, vo, so + W4);
        gv[sp][c][0] = t.x;
        gv[sp][c][1] = t.y;
        gv[sp][c][2] = bb.x;
        gv[sp][c][3] = bb.y;
      }
    }
    const uint32_t to = (uint32_t)(Rr * W + colr) * 4u;
#pragma unroll
    for (int c = 0; c < C; ++c) tv[c] = bload_s(rxs, to, so_t + (uint32_t)c * HW4);
  };

  // P1 of row R: values -> ring slot S, derivative pairs + depth -> LDS slot S
  auto finish_p1 = [&](auto Sc) {
    constexpr int S = decltype(Sc)::value;
    f2* v2 = s_v2 + S * NP * 64 + lane;
#pragma unroll
    for (int c = 0; c < C; ++c) yr[S][c] = tv[c] - cc[c];
#pragma unroll
    for (int c = 0; c < C; ++c) {
      float xv[2], dx[2], dy[2];
#pragma unroll
      for (int sp = 0; sp < 2; ++sp) {
        const float v00 = gv[sp][c][0], v01 = gv[sp][c][1], v10 = gv[sp][c][2], v11 = gv[sp][c][3];
        const float d0 = v01 - v00, d1 = v11 - v10;
        const float top = fmaf(bfx[sp], d0, v00), bot = fmaf(bfx[sp], d1, v10);
        const float dv = bot - top;
        xv[sp] = fmaf(bfy[sp], dv, top);
        dx[sp] = fmaf(bfy[sp], d1 - d0, d0);
        dy[sp] = dv;
      }
      xr[S][c] = (f2){xv[0], xv[1]} - bc(cc[c]);
      v2[c * 64] = (f2){dx[0], dx[1]} * (f2){bmx[0], bmx[1]};          // d val / d ix
      v2[(C + c) * 64] = (f2){dy[0], dy[1]} * (f2){bmy[0], bmy[1]};    // d val / d iy
    }
    s_dep[S * 64 + lane] = bdepth;
  };

  // P2 head for row p (window rows in ring slots S+1, S+2 (= p), S): SSIM and L1 of both
  // sources, their adjoint coefficients (cf), min over sources -> sel
  auto p2_head = [&](auto Sc, int p, float am, float gp, f2 (&cf)[C][3]) -> int {
    constexpr int S = decltype(Sc)::value;
    constexpr int SP = (S + 2) % 3;
    constexpr int S0 = (S + 1) % 3;
    const float kp = (cvalid && p >= 0 && p < H) ? kS * gp : 0.f;
    f2 loss = bc(0.f);
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const float y0v = yr[S0][c], y1v = yr[SP][c], y2v = yr[S][c];
      float my0 = y0v + y1v + y2v;
      float my1 = fmaf(y0v, y0v, fmaf(y1v, y1v, y2v * y2v));
      const f2 a0 = xr[S0][c], a1 = xr[SP][c], a2 = xr[S][c];
      f2 mx0 = a0 + a1 + a2;
      f2 mx1 = fma2(a0, a0, fma2(a1, a1, a2 * a2));
      f2 mxy = fma2(a0, bc(y0v), fma2(a1, bc(y1v), a2 * bc(y2v)));
      const f2 dl = bc(y1v) - a1;                    // L1 at the centre
      loss.x = fmaf(0.15f / (float)C, fabsf(dl.x), loss.x);
      loss.y = fmaf(0.15f / (float)C, fabsf(dl.y), loss.y);
      {
        float hv[8] = {my0, my1, mx0.x, mx0.y, mx1.x, mx1.y, mxy.x, mxy.y};
        __builtin_amdgcn_sched_barrier(0);
        hsum3_n(hv);
        __builtin_amdgcn_sched_barrier(0);
        my0 = hv[0];
        my1 = hv[1];
        mx0 = (f2){hv[2], hv[3]};
        mx1 = (f2){hv[4], hv[5]};
        mxy = (f2){hv[6], hv[7]};
      }
      const float my = my0 * inv9;
      const float mty = fmaf(my0, inv9, cc[c]);
      const float vy = fmaf(my1, inv9, -my * my);
      const float two_mty = 2.f * mty;
      const float B1y = fmaf(mty, mty, c1), B2y = vy + c2;
      const f2 mx = mx0 * bc(inv9);
      const f2 mtx = fma2(mx0, bc(inv9), bc(cc[c]));
      const f2 vx = fma2(mx1, bc(inv9), -mx * mx);
      const f2 cxy = fma2(mxy, bc(inv9), -mx * bc(my));
      const f2 A1 = fma2(mtx, bc(two_mty), bc(c1)), A2 = fma2(bc(2.f), cxy, bc(c2));
      const f2 B1 = fma2(mtx, mtx, bc(B1y)), B2 = vx + bc(B2y);
      const f2 rd = frcp(B1 * B2);
      const f2 r = (A1 * A2) * rd;
      const f2 val = fma2(bc(-0.5f), r, bc(0.5f));
      const f2 sv = (f2){fminf(fmaxf(val.x, 0.f), 1.f), fminf(fmaxf(val.y, 0.f), 1.f)};
      loss = fma2(bc(0.85f / (float)C), sv, loss);
      const f2 t1 = (f2){(val.x == sv.x) ? kp * rd.x : 0.f, (val.y == sv.y) ? kp * rd.y : 0.f};
      const f2 gm = t1 * fma2(r * mtx, B2, -bc(mty) * A2);
      const f2 gv2 = (r * t1) * B1;
      const f2 gc = -t1 * A1;
      cf[c][0] = fma2(-gv2, mx, fma2(-gc, bc(my), gm));
      cf[c][1] = gv2;
      cf[c][2] = gc;
    }
    int sel = (loss.y < loss.x) ? 1 : 0;
    float lmin = sel ? loss.y : loss.x;
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

  // P2 tail: the selected source's coefficients of row q+1, horizontally summed -> ch[S]
  auto p2_tail = [&](auto Sc, int sel, const f2 (&cf)[C][3]) {
    constexpr int S = decltype(Sc)::value;
    constexpr int NT = 6 * C;
    float F[NT], G[NT], t[NT];
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const f2 f = (f2){sel == 0 ? cf[c][k].x : 0.f, sel == 1 ? cf[c][k].y : 0.f};
        const f2 gg = f * bc(wship);
        F[2 * (3 * c + k)] = f.x;
        F[2 * (3 * c + k) + 1] = f.y;
        G[2 * (3 * c + k)] = gg.x;
        G[2 * (3 * c + k) + 1] = gg.y;
      }
    // photo.hip: fma(wl, left, fma(wr, right, F)) -- the same two roundings, in two passes
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < NT; ++i) t[i] = from_right(G[i]) + F[i];
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < NT; ++i) t[i] = from_left(G[i]) + t[i];
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int k = 0; k < 3; ++k) ch[S][c][k] = (f2){t[2 * (3 * c + k)], t[2 * (3 * c + k) + 1]};
  };

  // P3 of row q (coefficient rows q-1, q, q+1 in ch slots S+1, S+2, S; values in ring slot S+1;
  // P1 derivative pairs in LDS slot S+1): d/d warped values -> projection pullback
  auto p3 = [&](auto Sc, int q, bool live3, int selq, float gpq) {
    constexpr int S = decltype(Sc)::value;
    constexpr int SA = (S + 1) % 3, SB = (S + 2) % 3;
    const float wa = (q == 1) ? 2.f : 1.f, wb = (q == H - 2) ? 2.f : 1.f;
    const f2* v2 = s_v2 + SA * NP * 64 + lane;
    const float kLq = kL * gpq;
    f2 gx = bc(0.f), gy = bc(0.f);
    unsigned l1bits = 0;
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const float yq = yr[SA][c];
      const f2 xq = xr[SA][c];
      const float xs = (selq == 1) ? xq.y : xq.x;
      const float df = xs - yq;
      const float t = df > 0.f ? kLq : (df < 0.f ? -kLq : 0.f);
      if (CELLS) l1bits |= (df > 0.f ? 2u : (df < 0.f ? 1u : 3u)) << (PHOTO_CELL_L1SHIFT + 2 * c);
      f2 sum[3];
#pragma unroll
      for (int k = 0; k < 3; ++k) sum[k] = fma2(bc(wa), ch[SA][c][k], fma2(bc(wb), ch[S][c][k], ch[SB][c][k]));
      f2 dx = fma2(xq, sum[1], fma2(bc(yq), sum[2], sum[0]));
      dx += (f2){selq == 0 ? t : 0.f, selq == 1 ? t : 0.f};
      gx = fma2(dx, v2[c * 64], gx);
      gy = fma2(dx, v2[(C + c) * 64], gy);
    }
    const bool live = live3 && outl;
    if (CELLS && live && selq >= 0) {
      int* cm = sc.cell_map + (((long)selq * a.N + n) * H + q) * W + col;
      *cm = (int)((unsigned)*cm | l1bits);
    }
    const float depth = s_dep[SA * 64 + lane];
    const float h = (float)(q + 1) - cyp;
    float X[3];
    const float4* ikc = iks_base();
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const float4 ik = ikc[i];
      X[i] = depth * fmaf(ik.x, wcol, fmaf(ik.y, h, ik.z));
    }
    const f2 ggx = live ? gx : bc(0.f), ggy = live ? gy : bc(0.f);
    f2 m[3], cam[3];
    const f2* pkc = pk_base();
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      m[i] = fma2(pkc[4 * i], bc(wcol), fma2(pkc[4 * i + 1], bc(h), pkc[4 * i + 2]));
      cam[i] = fma2(bc(depth), m[i], pkc[4 * i + 3]);
    }
    const f2 rc = frcp(cam[2] + bc(eps7));
    const f2 kdx = pkc[12], kdy = pkc[13], kdz = pkc[14];
    f2 dc[3];
    dc[0] = ggx * rc;
    dc[1] = ggy * rc;
    dc[2] = -fma2(ggx, cam[0], ggy * cam[1]) * rc * rc;
    const f2 rc2 = rc * rc;
    const f2 T = fma2(ggx, fma2(m[0], kdz, -kdx * m[2]), ggy * fma2(m[1], kdz, -kdy * m[2]));
    const float ddepth = fmaf(rc2.y, T.y, fmaf(rc2.x, T.x, 0.f));   // photo.hip's source order
#pragma unroll
    for (int i = 0; i < 3; ++i) {
#pragma unroll
      for (int j = 0; j < 3; ++j) acc[3 * i + j] = fma2(dc[i], bc(X[j]), acc[3 * i + j]);
      acc[9 + i] += dc[i];
    }
    if (live) sc.g_disp[((long)n * H + q) * W + col] = -ddepth * disp_range * depth * depth;
  };

  // one row step k: P1 of row R = y0-2+k (slot S = k % 3), P2 of row R-1, P3 of row R-2
  auto step = [&](auto Sc, auto Pc, int k) {
    constexpr int S = decltype(Sc)::value;
    constexpr int PH = decltype(Pc)::value;
    const int R = y0 - 2 + k;
    finish_p1(Sc);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (PH & PH_P2) {
      const int p = min(max(R - 1, 0), H - 1);
      float am = 0.f, gp = 1.f;
      if (a.automask) am = a.automask[((long)n * H + p) * W + colr];
      if (a.gmap) gp = a.gmap[((long)n * H + p) * W + colr];
      f2 cf[C][3];
      const int sel = p2_head(Sc, R - 1, am, gp, cf);
      issue_gathers(R + 1);
      issue_disp(R + 2);
      p2_tail(Sc, sel, cf);
      if constexpr (PH & PH_P3) p3(Sc, R - 2, k >= 4, selc, gpc);
      selc = sel;
      gpc = gp;
    } else {
      issue_gathers(R + 1);
      issue_disp(R + 2);
    }
    __builtin_amdgcn_sched_barrier(0);
  };

#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int k = 0; k < 3; ++k) ch[r][c][k] = bc(0.f);
  issue_disp(y0 - 2);
  issue_gathers(y0 - 2);
  issue_disp(y0 - 1);
  // rows y0-2, y0-1: P1 only; row y0 (k = 2): + P2 of the halo row y0-1; k = 3: + P2 of row y0
  // (its P3 row y0-1 is a halo row); from k = 4 on every phase, up to the band's last row
  step(Slot<0>{}, std::integral_constant<int, 0>{}, 0);
  step(Slot<1>{}, std::integral_constant<int, 0>{}, 1);
  step(Slot<2>{}, std::integral_constant<int, PH_P2>{}, 2);
  step(Slot<0>{}, std::integral_constant<int, PH_P2>{}, 3);
  for (int k = 4;; k += 3) {
    step(Slot<1>{}, std::integral_constant<int, PH_ALL>{}, k);
    if (k + 1 >= KT) break;
    step(Slot<2>{}, std::integral_constant<int, PH_ALL>{}, k + 1);
    if (k + 2 >= KT) break;
    step(Slot<0>{}, std::integral_constant<int, PH_ALL>{}, k + 2);
    if (k + 3 >= KT) break;
  }

  // ---- per-wave partials (photo.hip's layout and order)
  lsum = wave_sum_dpp(lsum);
  float accs[24];
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    accs[i] = wave_sum_dpp(acc[i].x);
    accs[12 + i] = wave_sum_dpp(acc[i].y);
  }
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
              fmaf(Kc[k], accs[12 * sp + l], fmaf(Kc[3 + k], accs[12 * sp + 3 + l], Kc[6 + k] * accs[12 * sp + 6 + l]));
        out[1 + 12 * sp + 9 + k] =
            fmaf(Kc[k], accs[12 * sp + 9], fmaf(Kc[3 + k], accs[12 * sp + 10], Kc[6 + k] * accs[12 * sp + 11]));
      }
    }
  }
}

int launch_photo2(const PhotoArgs& a, const Geom& g, const PhotoTiling& tl, int C, bool cells, long blocks,
                  hipStream_t st) {
  const dim3 grid((unsigned)blocks), block(64);
  if (C == 3 && !cells)
    hipLaunchKernelGGL((photo2_kernel<3, false>), grid, block, 0, st, a, g, tl);
  else if (C == 3)
    hipLaunchKernelGGL((photo2_kernel<3, true>), grid, block, 0, st, a, g, tl);
  else if (C == 1 && !cells)
    hipLaunchKernelGGL((photo2_kernel<1, false>), grid, block, 0, st, a, g, tl);
  else if (C == 1)
    hipLaunchKernelGGL((photo2_kernel<1, true>), grid, block, 0, st, a, g, tl);
  else {
    set_error("photometric: channels must be 1 or 3");
    return MD2_ENOTSUP;
  }
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

}  // namespace md2
