// Non-GEMM layers of the train step: BatchNorm (train mode), max-pool, x2 bilinear upsample,
// the pose head (1x1 conv + spatial mean), Adam, small elementwise helpers.
#pragma once
#include "common.h"

namespace md2 {

// ---- BatchNorm, Flux train mode (batch mean / biased var, eps), per channel over N*HW ----
struct BNStatsWs {
  double* partials;   // [C][parts][2]
  int parts;
};
int bn_parts(int C, long N, long HW);
// Split-K slabs [splits][C][N*HW] of the conv that produced a BN input (conv_fwd / conv_dgrad
// with a SplitKDefer): the BN kernels below sum them in split order -- the conv's own reduction,
// bit-identical -- write the tensor and take its partials in the same pass (the launch-boundary
// reduce: one launch and one full read of the tensor fewer)
struct SlabIn {
  const float* slab = nullptr;
  int splits = 0;
};
// optional addend of a BN backward's dout: skip[e - lo] over flat elements [lo, hi)
struct SkipAdd {
  const float* skip = nullptr;
  long lo = 0, hi = 0;
};
// device-side form of a SkipAdd (nn.hip)
struct SkipSrc {
  const float* skip = nullptr;
  uint32_t skip_lo = 0, skip_hi = 0;
};
// mean/invstd [C]; running stats updated when run_mean != nullptr (momentum, unbiased var)
int bn_stats(const float* y, int N, int C, long HW, float eps, float momentum, float* mean,
             float* invstd, float* run_mean, float* run_var, BNStatsWs ws, hipStream_t st);
// out = act(gamma*(y-mean)*invstd + beta [+ gamma2*(y2-mean2)*invstd2 + beta2] [+ res])
struct BNApply {
  const float* y; const float* mean; const float* invstd; const float* gamma; const float* beta;
  const float* y2 = nullptr; const float* mean2 = nullptr; const float* invstd2 = nullptr;
  const float* gamma2 = nullptr; const float* beta2 = nullptr;
  const float* res = nullptr;
  int relu = 0;
};
int bn_apply(const BNApply& p, float* out, int N, int C, long HW, hipStream_t st);

// Fused statistics finalise + apply (the model's path): bn_stats_partial writes the per-(channel,
// image group) fp64 partials; bn_apply_fused derives mean/invstd from them inside every block
// (same summation order as bn_stats' finalise: bit-identical), applies the affine map (+ the
// downsample branch, residual, ReLU) and writes mean/invstd/running stats once per channel.
struct BNStatsIn {
  const double* part = nullptr;   // [C][parts][2] from bn_stats_partial
  int parts = 0;
  float eps = 1e-5f, momentum = 0.1f;
  const float* gamma = nullptr; const float* beta = nullptr;
  float* mean = nullptr; float* invstd = nullptr;          // [C] outputs (for the backward)
  float* run_mean = nullptr; float* run_var = nullptr;     // running stats (nullable)
};
struct BNApplyFused {
  const float* y = nullptr; BNStatsIn s1;
  const float* y2 = nullptr; BNStatsIn s2;                 // downsample branch (nullable y2)
  const float* res = nullptr;
  int relu = 0;
};
int bn_stats_partial(const float* y, int N, int C, long HW, BNStatsWs ws, hipStream_t st);
// [C][parts][2] statistics partials -> [C][1][2] (fixed order per channel), so the apply passes'
// per-block finalise reads one partial instead of `parts` (the conv epilogue's per-tile partials)
int bn_partials_collapse(const double* part, int C, int parts, double* out, hipStream_t st);
int bn_stats_partial_slabs(SlabIn sl, float* y, int N, int C, long HW, BNStatsWs ws, hipStream_t st);
int bn_apply_fused(const BNApplyFused& p, float* out, int N, int C, long HW, hipStream_t st);
// backward reduce: g = dout * (mask_out > 0 if mask_out) ; dgamma = sum g*xhat, dbeta = sum g
int bn_bwd_reduce(const float* dout, const float* mask_out, const float* y, const float* mean,
                  const float* invstd, int N, int C, long HW, float* dgamma, float* dbeta,
                  BNStatsWs ws, hipStream_t st);
// backward partials only (bn_bwd_reduce without its finalise); bn_bwd_apply_fused then sums the
// partials per block (dgamma/dbeta written once per channel) and applies -- model path
// mgamma/mbeta non-null (and mask_out null): the ReLU mask of a residual-free BN+ReLU output is
// re-derived from y bit-exactly (bn_apply_fused's explicit roundings) instead of read back
int bn_bwd_partial(const float* dout, const float* mask_out, const float* y, const float* mean,
                   const float* invstd, int N, int C, long HW, BNStatsWs ws, hipStream_t st,
                   const float* mgamma = nullptr, const float* mbeta = nullptr, SkipAdd sk = SkipAdd{});
// the same with dout formed from the dgrad's split-K slabs (and written to dout)
int bn_bwd_partial_slabs(SlabIn sl, float* dout, const float* y, const float* mean,
                         const float* invstd, int N, int C, long HW, BNStatsWs ws, hipStream_t st,
                         const float* mgamma, const float* mbeta);
int bn_bwd_apply_fused(const float* dout, const float* mask_out, const float* y, const float* mean,
                       const float* invstd, const float* gamma, BNStatsWs ws, float* dgamma,
                       float* dbeta, int N, int C, long HW, float* dy, float* dres,
                       int dres_accumulate, hipStream_t st, const float* mbeta = nullptr,
                       SkipAdd sk = SkipAdd{});
// dy = gamma*invstd*(g - dbeta/L - xhat*dgamma/L); optional dres (=g) store/accumulate
int bn_bwd_apply(const float* dout, const float* mask_out, const float* y, const float* mean,
                 const float* invstd, const float* gamma, const float* dgamma,
                 const float* dbeta, int N, int C, long HW, float* dy, float* dres,
                 int dres_accumulate, hipStream_t st);

// ---- MaxPool((3,3); stride 2, pad 1) ----
// stem tail: act = relu(BN(p.y)) (statistics finalised from p.s1's partials) and its 3x3/2/pad-1
// max pool (y, argmax) in one pass; even H, W; bit-identical to bn_apply_fused + maxpool_fwd
int bn_relu_maxpool(const BNApplyFused& p, float* act, int N, int C, int H, int W, float* y,
                    unsigned char* arg, int Ho, int Wo, hipStream_t st);
int maxpool_fwd(const float* x, int N, int C, int H, int W, float* y, unsigned char* arg,
                int Ho, int Wo, hipStream_t st);
// optional skip: dx += skip over whole images (the decoder skip gradient; even W)
int maxpool_bwd(const float* dy, const unsigned char* arg, int N, int C, int H, int W, int Ho,
                int Wo, float* dx, hipStream_t st, SkipAdd skip = SkipAdd{});

// ---- upsample_bilinear(x, (2,2)), align_corners = true ----
int upsample2_fwd(const float* x, int N, int C, int h, int w, float* y, hipStream_t st);
int upsample2_bwd(const float* dy, int N, int C, int h, int w, float* dx, hipStream_t st);
// MPI-mode decoder input (src/model.jl:39-50): out[(b*P + p)][0:C] = feat[b], out[..][C + e] =
// embed(bins[b][p])[e] broadcast over h x w (e < 2L+1: x, sin(2^i x), cos(2^i x))
// Ctot: channels per output image (>= C + 2L + 1; the channels past C + 2L + 1 are written as
// zeros -- the executor's padded layout); 0 = C + 2L + 1
int mpi_embed_features(const float* feat, long sample_stride, int N, int C, int h, int w,
                       const float* bins, int P, int L, float* out, hipStream_t st, int Ctot = 0);
// the _repeat pullback (src/repeat.jl:44-53): out[b][c] (+)= sum_p in[b*P + p][c] for c < C of the
// Cin channels per image (hw % 4 == 0)
int plane_sum(const float* in, int N, int P, int Cin, int C, long hw, float* out, int accumulate,
              hipStream_t st);
// dst[r*P + p][:] = src[r][:] for a [rows][cols] matrix, and its adjoint dst[r] = sum_p src[r*P + p]
int repeat_rows(const float* src, long rows, int cols, int P, float* dst, hipStream_t st);
int repeat_rows_adjoint(const float* src, long rows, int cols, int P, float* dst, hipStream_t st);
// channel concatenation cat(a, b; dims=3) of [N][ca][hw] and [N][cb][hw]
int concat_channels(const float* a, int ca, const float* b, int cb, int N, long hw, float* out,
                    hipStream_t st);

// ---- pose head: pose[q][k] = 0.01 * (b[k] + sum_c W[k][c] * mean_hw(x[q][c])) ----
int pose_head_fwd(const float* x, int Q, int C, long HW, const float* w, const float* b,
                  float* means, float* pose, hipStream_t st);
int pose_head_bwd(const float* dpose, int Q, int C, long HW, const float* w, const float* means,
                  float* dx, float* dw, float* db, hipStream_t st);

// ---- misc elementwise ----
int axpy(float* y, const float* x, long n, hipStream_t st);               // y += x
// pose pairs (a_j, b_j) of frames: PoseDecoder input gather / its gradient scatter (nn.hip)
int pair_gather(const float* sq, int N, int C, long HW, const int a[2], const int b[2], float* pin,
                hipStream_t st);
int pair_grad_gather(const float* dpin, int N, int C, long HW, const int a[2], const int b[2],
                     float* dsq, hipStream_t st);

// ---- Flux ADAM over the flat parameter vector ----
int scale_inplace(float* x, long n, float s, hipStream_t st);
// out = g .* (s .* (1 - s)) (g == nullptr: 0), the sigmoid head's pullback
int sigmoid_cotangent(const float* g, const float* s, float* out, long n, hipStream_t st);
// [planes][kh][kw] with both spatial axes reversed (Flux true-convolution <-> cross-correlation)
int flip_taps(const float* src, float* dst, long planes, int kh, int kw, hipStream_t st);
// graph-replayable ADAM: *step += 1 and bc = (1 - b1^t, 1 - b2^t) on the device, then the update
int adam_prep(int* step, float* bc, float b1, float b2, hipStream_t st);
int set_device_int(int* p, int v, hipStream_t st);
int adam_step_dev(float* p, const float* g, float* m, float* v, long n, float lr, float b1, float b2,
                  float eps, const float* bc, float gscale, hipStream_t st);
int adam_step(float* p, const float* g, float* m, float* v, long n, float lr, float b1, float b2,
              float eps, float bc1, float bc2, float gscale, hipStream_t st);

}  // namespace md2
