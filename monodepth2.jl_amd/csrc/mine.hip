// MINE plane rendering of the MPI mode (src/render.jl:21-114), forward, for gfx950.
//
// Layouts are the Julia arrays' bytes read in C order (include/md2.h): q = b*N + n indexes the
// (plane n, batch item b) pairs, pixels run x fastest.
//   rgb (W,H,3,N,B) = [B][N][3][H][W]      sigma (W,H,1,N,B) = [B][N][H][W]
//   xyz (3,W,H,N,B) = [B][N][H][W][3]      disparity / depth (N,B) = [B][N]
//   pose = [B][6] (rvec, tvec)             sample src (W,H,C,N*B) = [B*N][C][H][W]
// The reference's semantics are kept as written, not "fixed":
//   * sample normalises the source coordinate as (u + 0.5) / (W/2) with no -1 before
//     grid_sample (align_corners, :border) -- render.jl:85-86;
//   * its valid mask is Julia's chained comparison `u .< W .* u .>= 0`, i.e.
//     (u < W*u) & (W*u >= 0), which is u > 0 for W > 1 -- render.jl:83;
//   * the last plane's distance is 1e3 and the transmittance product runs over (T + 1e-6),
//     exclusive -- render.jl:35-41;
//   * render_tgt_rgb_depth's "depth" output is the transparency_acc volume -- render.jl:110-113.
//
// render_tgt_rgb_depth is ONE kernel: each thread owns a target pixel of one batch item and walks
// the planes front to back -- homography (H_src_tgt per plane, computed once per block into LDS),
// bilinear taps of the 7 packed channels (rgb, sigma, xyz) read straight from the three inputs,
// and the volume-rendering recurrence with a one-plane delay for the inter-plane distance.  The
// reference's cat -> sample -> slice -> plane_volume_rendering chain (a 7-channel packed copy, the
// sampled volume and the weights volume in HBM) collapses into reads of the inputs plus the depth
// volume write: 28 B read + 4 B written per pixel and plane.
#include "mine.h"

namespace md2 {
namespace {

constexpr int MINE_MAX_PLANES = 512;   // LDS: 9 floats per plane

// so3_exp_map (src/utils.jl:106-121), theta' = max(theta, 1e-4), in fp64
__device__ void so3_exp_d(const float* r, double* R) {
  const double a = r[0], b = r[1], c = r[2];
  const double th = sqrt(a * a + b * b + c * c);
  const double thi = 1.0 / fmax(th, 1e-4);
  const double f1 = thi * sin(th), f2 = thi * thi * (1.0 - cos(th));
  const double S[9] = {0.0, -c, b, c, 0.0, -a, -b, a, 0.0};
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      double s2 = 0.0;
      for (int k = 0; k < 3; ++k) s2 += S[3 * i + k] * S[3 * k + j];
      R[3 * i + j] = f1 * S[3 * i + j] + f2 * s2 + (i == j ? 1.0 : 0.0);
    }
}

// H_src_tgt = inv(K (R - t n^T / (-d)) K^-1), n = (0, 0, 1) (render.jl:72-79), in fp64, into out[9]
__device__ __noinline__ void homography_src_tgt(const float* pose_b, double d, const Mat3& K, const Mat3& invK,
                                   float* out) {
  double R[9];
  so3_exp_d(pose_b, R);
  const double t[3] = {pose_b[3], pose_b[4], pose_b[5]};
  double M[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) M[3 * i + j] = R[3 * i + j] - (j == 2 ? t[i] / (-d) : 0.0);
  double KM[9], Ht[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      double s = 0.0;
      for (int k = 0; k < 3; ++k) s += (double)K.m[3 * i + k] * M[3 * k + j];
      KM[3 * i + j] = s;
    }
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      double s = 0.0;
      for (int k = 0; k < 3; ++k) s += KM[3 * i + k] * (double)invK.m[3 * k + j];
      Ht[3 * i + j] = s;
    }
  // the adjugate inverse (the reference's batched getrf/getri, render.jl:3-17, is the same matrix)
  const double c00 = Ht[4] * Ht[8] - Ht[5] * Ht[7], c01 = Ht[5] * Ht[6] - Ht[3] * Ht[8],
               c02 = Ht[3] * Ht[7] - Ht[4] * Ht[6];
  const double id = 1.0 / (Ht[0] * c00 + Ht[1] * c01 + Ht[2] * c02);
  out[0] = (float)(c00 * id);
  out[1] = (float)((Ht[2] * Ht[7] - Ht[1] * Ht[8]) * id);
  out[2] = (float)((Ht[1] * Ht[5] - Ht[2] * Ht[4]) * id);
  out[3] = (float)(c01 * id);
  out[4] = (float)((Ht[0] * Ht[8] - Ht[2] * Ht[6]) * id);
  out[5] = (float)((Ht[2] * Ht[3] - Ht[0] * Ht[5]) * id);
  out[6] = (float)(c02 * id);
  out[7] = (float)((Ht[1] * Ht[6] - Ht[0] * Ht[7]) * id);
  out[8] = (float)((Ht[0] * Ht[4] - Ht[1] * Ht[3]) * id);
}

// One target pixel through one plane's homography: the 4 bilinear taps of grid_sample(:border)
// at the reference's normalised coordinate, and the valid flag (render.jl:80-90).
struct Taps {
  int i0, i1;               // offsets of the top-left tap of the two rows; the right taps are +1
  float wx, wy;
  bool valid;
};

__device__ __forceinline__ Taps taps_at(const float* h, float fx, float fy, int H, int W) {
  const float a0 = h[0] * fx + h[1] * fy + h[2];
  const float a1 = h[3] * fx + h[4] * fy + h[5];
  const float a2 = h[6] * fx + h[7] * fy + h[8];
  const float u = a0 / a2, v = a1 / a2;
  const float Wf = (float)W, Hf = (float)H;
  Taps t;
  t.valid = (u < Wf * u) && (Wf * u >= 0.f) && (v < Hf * v) && (Hf * v >= 0.f);
  const float gx = (u + 0.5f) / (Wf * 0.5f), gy = (v + 0.5f) / (Hf * 0.5f);
  // grid_sample unnormalise (align_corners) + border clamp
  const float ix = fminf(fmaxf((gx + 1.f) * 0.5f * (Wf - 1.f), 0.f), Wf - 1.f);
  const float iy = fminf(fmaxf((gy + 1.f) * 0.5f * (Hf - 1.f), 0.f), Hf - 1.f);
  // left/top tap clamped to W-2 / H-2: at ix = W-1 the pair (W-2, W-1) with weight 1 on the
  // right tap is the same value as NNlib's (W-1, out-of-range) with weight 0, and the right
  // taps are always x0+1 / y0+1 -- adjacent, so each row pair is one 8-byte load
  const int x0 = min((int)ix, W - 2), y0 = min((int)iy, H - 2);
  t.wx = ix - (float)x0;
  t.wy = iy - (float)y0;
  t.i0 = y0 * W + x0;
  t.i1 = t.i0 + W;
  return t;
}

__device__ __forceinline__ float lerp2(float a, float b, float w) { return a + w * (b - a); }

__device__ __forceinline__ float tap(const float* p, const Taps& t) {
  const float top = lerp2(p[t.i0], p[t.i0 + 1], t.wx);
  const float bot = lerp2(p[t.i1], p[t.i1 + 1], t.wx);
  return lerp2(top, bot, t.wy);
}
// point planes ([H][W][3], xyz): the two taps of a row are 6 consecutive floats
__device__ __forceinline__ void tap3(const float* p, const Taps& t, float& X, float& Y, float& Z) {
  const float* a = p + 3 * t.i0;
  const float* b = p + 3 * t.i1;
  X = lerp2(lerp2(a[0], a[3], t.wx), lerp2(b[0], b[3], t.wx), t.wy);
  Y = lerp2(lerp2(a[1], a[4], t.wx), lerp2(b[1], b[4], t.wx), t.wy);
  Z = lerp2(lerp2(a[2], a[5], t.wx), lerp2(b[2], b[5], t.wx), t.wy);
}

// sample(src, depth_src, pose, K, K_inv) (render.jl:68-94) for C channels.
// grid (x tiles of 64, y tiles of 4, plane*batch); block 256.
__global__ __launch_bounds__(256) void mine_sample_kernel(const float* __restrict__ src, int C, int N,
                                                          int H, int W, const float* __restrict__ depth,
                                                          const float* __restrict__ pose, Mat3 K,
                                                          Mat3 invK, float* __restrict__ out,
                                                          float* __restrict__ valid) {
  __shared__ float hs[9];
  const int q = blockIdx.z;
  if (threadIdx.x == 0) homography_src_tgt(pose + 6 * (q / N), (double)depth[q], K, invK, hs);
  __syncthreads();
  const int x = blockIdx.x * 64 + (threadIdx.x & 63), y = blockIdx.y * 4 + (threadIdx.x >> 6);
  if (x >= W || y >= H) return;
  const Taps t = taps_at(hs, (float)x, (float)y, H, W);
  const long HW = (long)H * W, pix = (long)y * W + x;
  valid[q * HW + pix] = t.valid ? 1.f : 0.f;
  const float* s = src + (long)q * C * HW;
  float* o = out + (long)q * C * HW + pix;
  for (int c = 0; c < C; ++c) o[c * HW] = tap(s + c * HW, t);
}

// plane_volume_rendering(rgb, sigma, xyz) (render.jl:32-49): one thread per (pixel, batch item)
// walking the planes; sigma is used as given.
__global__ __launch_bounds__(256) void plane_render_kernel(const float* __restrict__ rgb,
                                                           const float* __restrict__ sigma,
                                                           const float* __restrict__ xyz, int N, int HW,
                                                           float* __restrict__ rgb_out,
                                                           float* __restrict__ tacc,
                                                           float* __restrict__ weights) {
  const int p = blockIdx.x * 256 + threadIdx.x, b = blockIdx.y;
  if (p >= HW) return;
  float acc = 1.f, o0 = 0.f, o1 = 0.f, o2 = 0.f;
  const float* xb = xyz + (long)b * N * HW * 3 + 3L * p;
  float X0 = xb[0], Y0 = xb[1], Z0 = xb[2];
  for (int n = 0; n < N; ++n) {
    float dist = 1e3f;
    if (n + 1 < N) {
      const float* x1 = xb + (long)(n + 1) * HW * 3;
      const float X1 = x1[0], Y1 = x1[1], Z1 = x1[2];
      const float dx = X1 - X0, dy = Y1 - Y0, dz = Z1 - Z0;
      dist = sqrtf(dx * dx + dy * dy + dz * dz);
      X0 = X1;
      Y0 = Y1;
      Z0 = Z1;
    }
    const long q = ((long)b * N + n) * HW + p;
    const float T = expf(-dist * sigma[q]);
    const float w = acc * (1.f - T);
    tacc[q] = acc;
    weights[q] = w;
    const float* c = rgb + ((long)b * N + n) * 3 * HW + p;
    o0 += w * c[0];
    o1 += w * c[HW];
    o2 += w * c[2 * HW];
    acc *= T + 1e-6f;
  }
  float* o = rgb_out + (long)b * 3 * HW + p;
  o[0] = o0;
  o[HW] = o1;
  o[2 * HW] = o2;
}

// get_src_xyz_from_plane_disparity (render.jl:25-30): K^-1 [w, h, 1] / disparity, 1-based grid
__global__ __launch_bounds__(256) void mine_src_xyz_kernel(const float* __restrict__ disp, Mat3 invK,
                                                           int H, int W, float* __restrict__ xyz) {
  const int p = blockIdx.x * 256 + threadIdx.x, q = blockIdx.y;
  if (p >= H * W) return;
  const int y = p / W, x = p - y * W;
  const float d = 1.f / disp[q];
  const float w = (float)(x + 1), h = (float)(y + 1);
  float* o = xyz + ((long)q * H * W + p) * 3;
#pragma unroll
  for (int i = 0; i < 3; ++i) o[i] = (invK.m[3 * i] * w + invK.m[3 * i + 1] * h + invK.m[3 * i + 2]) * d;
}

// get_tgt_xyz_from_plane_disparity (render.jl:51-64): R(rvec_b) xyz + t_b
__global__ __launch_bounds__(256) void mine_tgt_xyz_kernel(const float* __restrict__ xyz,
                                                           const float* __restrict__ pose, long per_b,
                                                           float* __restrict__ out) {
  __shared__ float rt[12];
  const int b = blockIdx.y;
  if (threadIdx.x == 0) {
    double R[9];
    so3_exp_d(pose + 6 * b, R);
    for (int k = 0; k < 9; ++k) rt[k] = (float)R[k];
    for (int k = 0; k < 3; ++k) rt[9 + k] = pose[6 * b + 3 + k];
  }
  __syncthreads();
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= per_b) return;
  const float* s = xyz + ((long)b * per_b + i) * 3;
  float* o = out + ((long)b * per_b + i) * 3;
  const float X = s[0], Y = s[1], Z = s[2];
#pragma unroll
  for (int k = 0; k < 3; ++k) o[k] = rt[3 * k] * X + rt[3 * k + 1] * Y + rt[3 * k + 2] * Z + rt[9 + k];
}

// the 7 sampled channels of plane q (= b*N + n) at one target pixel
struct PlaneVals {
  float c0, c1, c2, s, X, Y, Z, valid;
};
__device__ __forceinline__ PlaneVals plane_vals(const float* __restrict__ rgb,
                                                const float* __restrict__ sigma,
                                                const float* __restrict__ xyz, const float* h, long q,
                                                float fx, float fy, int H, int W) {
  const Taps t = taps_at(h, fx, fy, H, W);
  const long HW = (long)H * W;
  const float* c = rgb + q * 3 * HW;
  PlaneVals v;
  v.c0 = tap(c, t);
  v.c1 = tap(c + HW, t);
  v.c2 = tap(c + 2 * HW, t);
  v.s = tap(sigma + q * HW, t);
  tap3(xyz + q * 3 * HW, t, v.X, v.Y, v.Z);
  v.valid = t.valid ? 1.f : 0.f;
  return v;
}

// render_tgt_rgb_depth (render.jl:96-114), fused (see the header comment).
// grid (x tiles of 64, y tiles of 4, batch); block 256; dynamic LDS 9*N floats.
// Measured (profiles/r02_mine.json): deeper per-thread prefetch rings (2-4 planes in flight)
// did not beat this one-plane lookahead -- the loop-carried copies of in-flight registers force
// the waits back -- so the kernel stays at ~86 VGPRs (5 waves/SIMD) and lets occupancy hide it.
__global__ __launch_bounds__(256) void mine_render_kernel(const float* __restrict__ rgb,
                                                          const float* __restrict__ sigma,
                                                          const float* __restrict__ disparity,
                                                          const float* __restrict__ xyz,
                                                          const float* __restrict__ pose, Mat3 K,
                                                          Mat3 invK, int N, int H, int W,
                                                          float* __restrict__ rgb_out,
                                                          float* __restrict__ depth,
                                                          float* __restrict__ mask) {
  extern __shared__ float hs[];   // [N][9]
  const int b = blockIdx.z;
  // depth_src = 1 ./ disparity_src (render.jl:102)
  for (int n = threadIdx.x; n < N; n += 256)
    homography_src_tgt(pose + 6 * b, (double)(1.f / disparity[b * N + n]), K, invK, hs + 9 * n);
  __syncthreads();
  const int x = blockIdx.x * 64 + (threadIdx.x & 63), y = blockIdx.y * 4 + (threadIdx.x >> 6);
  if (x >= W || y >= H) return;
  const long HW = (long)H * W, pix = (long)y * W + x;
  const float fx = (float)x, fy = (float)y;
  const long q0 = (long)b * N;
  float* dep = depth + q0 * HW + pix;
  PlaneVals cur = plane_vals(rgb, sigma, xyz, hs, q0, fx, fy, H, W);
  float acc = 1.f, o0 = 0.f, o1 = 0.f, o2 = 0.f, nvalid = 0.f;
  float r0 = 0.f, r1 = 0.f, r2 = 0.f, sg = 0.f, X0 = 0.f, Y0 = 0.f, Z0 = 0.f;
  for (int n = 0; n < N; ++n) {
    PlaneVals nxt;
    if (n + 1 < N) nxt = plane_vals(rgb, sigma, xyz, hs + 9 * (n + 1), q0 + n + 1, fx, fy, H, W);
    nvalid += cur.valid;
    if (n > 0) {   // plane n-1 completes now that its successor's point is known
      const float dx = cur.X - X0, dy = cur.Y - Y0, dz = cur.Z - Z0;
      const float T = expf(-sqrtf(dx * dx + dy * dy + dz * dz) * sg);
      const float w = acc * (1.f - T);
      o0 += w * r0;
      o1 += w * r1;
      o2 += w * r2;
      acc *= T + 1e-6f;
    }
    dep[n * HW] = acc;
    r0 = cur.c0;
    r1 = cur.c1;
    r2 = cur.c2;
    sg = cur.s * (cur.s >= 0.f ? 1.f : 0.f);   // sigma .* (sigma .>= 0)
    X0 = cur.X;
    Y0 = cur.Y;
    Z0 = cur.Z;
    cur = nxt;
  }
  const float T = expf(-1e3f * sg);   // the last plane's distance
  const float w = acc * (1.f - T);
  o0 += w * r0;
  o1 += w * r1;
  o2 += w * r2;
  float* o = rgb_out + (long)b * 3 * HW + pix;
  o[0] = o0;
  o[HW] = o1;
  o[2 * HW] = o2;
  mask[(long)b * HW + pix] = nvalid;
}

}  // namespace

int mine_src_xyz(const float* disp, int N, int B, int H, int W, const Mat3& invK, float* xyz,
                 hipStream_t st) {
  hipLaunchKernelGGL(mine_src_xyz_kernel, dim3(cdiv((long)H * W, 256), N * B), dim3(256), 0, st, disp,
                     invK, H, W, xyz);
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

int mine_tgt_xyz(const float* xyz, const float* pose, int N, int B, int H, int W, float* out,
                 hipStream_t st) {
  const long per_b = (long)N * H * W;
  hipLaunchKernelGGL(mine_tgt_xyz_kernel, dim3(cdiv(per_b, 256), B), dim3(256), 0, st, xyz, pose,
                     per_b, out);
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

int mine_sample(const float* src, int C, const float* depth, const float* pose, int N, int B, int H,
                int W, const Mat3& K, const Mat3& invK, float* out, float* valid, hipStream_t st) {
  hipLaunchKernelGGL(mine_sample_kernel, dim3(cdiv(W, 64), cdiv(H, 4), N * B), dim3(256), 0, st, src,
                     C, N, H, W, depth, pose, K, invK, out, valid);
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

int plane_volume_rendering(const float* rgb, const float* sigma, const float* xyz, int N, int B,
                           int H, int W, float* rgb_out, float* tacc, float* weights,
                           hipStream_t st) {
  const int HW = H * W;
  hipLaunchKernelGGL(plane_render_kernel, dim3(cdiv(HW, 256), B), dim3(256), 0, st, rgb, sigma, xyz,
                     N, HW, rgb_out, tacc, weights);
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

int render_tgt_rgb_depth(const float* rgb, const float* sigma, const float* disparity,
                         const float* xyz_tgt, const float* pose, const Mat3& invK, const Mat3& K,
                         int N, int B, int H, int W, float* rgb_out, float* depth, float* mask,
                         hipStream_t st) {
  MD2_CHECK_ARG(N <= MINE_MAX_PLANES, "render_tgt_rgb_depth: at most 512 planes");
  hipLaunchKernelGGL(mine_render_kernel, dim3(cdiv(W, 64), cdiv(H, 4), B), dim3(256),
                     9 * N * sizeof(float), st, rgb, sigma, disparity, xyz_tgt, pose, K, invK, N, H, W,
                     rgb_out, depth, mask);
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

}  // namespace md2
