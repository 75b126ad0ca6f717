// Loss-tail kernels: see loss_kernels.hip.
#pragma once
#include "common.h"

namespace md2 {

constexpr int MAX_SCALES = 5;

// Camera / depth constants of one resolution (TrainCache K, invK; Params min/max depth).
struct Geom {
  float K[9];        // row-major
  float invK[9];     // row-major
  float min_disp;    // 1 / max_depth
  float disp_range;  // 1/min_depth - 1/max_depth
  float wm1, hm1;    // W-1, H-1 (normalize / unnormalize)
  int W, H;          // full (target) resolution
};

// One scale of the photometric pass: its disparity (any resolution <= the target's, upsampled
// in-kernel with align_corners) and its outputs.
struct PhotoScale {
  const float* disp;      // [N][dh][dw]  (sigmoid output of one scale)
  int dw, dh;
  float rx, ry;           // (dw-1)/(W-1), (dh-1)/(H-1)  align_corners upsample ratios
  float* g_disp;          // [N][H][W] out: d loss / d full-res disparity (store)
  float* partials;        // [N*tiles][25]: loss sum, dR0(9) dt0(3), dR1(9) dt1(3)
  float* loss_map;        // [N][H][W] per-pixel warp loss (train_loss vis_loss) or nullptr
  signed char* sel_map;   // [N][H][W] chosen source (0/1, -1 = automask) or nullptr
  int* cell_map;          // [2][N][H][W] bilinear cell + border flags per source (parity
                          // diagnostics, PHOTO_CELL_* packing) or nullptr
};

// cell_map packing: x cell (bits 0-10), y cell (11-21), x border state (22-23), y (24-25);
// state 0 = interior (coordinate differentiable), 1 = clamped to 0, 2 = clamped to W-1 / H-1;
// on the SELECTED source of a pixel, bits 26 + 2c: the L1 branch abs' took in channel c
// (1 = warped below the target, 2 = above, 3 = equal: abs'(0) = 0; 0 on the other source)
constexpr int PHOTO_CELL_YSHIFT = 11, PHOTO_CELL_FXSHIFT = 22, PHOTO_CELL_FYSHIFT = 24;
constexpr int PHOTO_CELL_L1SHIFT = 26;
constexpr int PHOTO_CELL_MAXDIM = 2048;

struct PhotoArgs {
  PhotoScale sc[MAX_SCALES];
  int nscales;
  const float* x;         // frames
  long x_sample_stride;   // elements between samples
  long x_frame_stride;    // elements between frames of a sample
  int target, src0, src1; // 0-based frame indices
  const float* Rt;        // [2][N][12]  composed (R row-major, t) per (source, sample)
  const float* automask;  // [N][H][W] identity-reprojection loss or nullptr
  float wloss;            // d(total loss) / d(per-pixel warp loss)
  const float* gmap;      // [N][H][W] per-pixel cotangent (times wloss) or nullptr (uniform)
  int N;
};

// Wave tiling of the photometric pass (photo.hip): 60 output columns x `rows` output rows per
// wave, tiles_x * tiles_y tiles per sample and scale.
struct PhotoTiling {
  int tiles_x, tiles_y, rows;
  long per_scale() const { return (long)tiles_x * tiles_y; }
};
PhotoTiling photo_tiling(int W, int H, int N, int nscales);

struct SmoothArgs {
  const float* disp;
  int dw, dh;
  float rx, ry;
  const float* img;          // target frame of sample 0 ([C][H][W])
  long img_sample_stride;
  const double* mean_partials;  // [N][mean_parts] sums of the upsampled disparity (fp64)
  int mean_parts;
  float ws;                  // d(total)/d(smooth term) = smoothness * scale / nscales * upstream
  float* g_disp;             // [N][H][W] accumulated
  float* partials;           // [blocks][2]: smooth loss sum, sum(u * d) (fp32)
  double* tsum;              // [blocks] sum(u * d) in fp64 (the normalisation constant) or nullptr
  int N, W, H;
};

struct SmoothBatch {
  SmoothArgs s[MAX_SCALES];  // every scale shares N, W, H (full resolution)
};

struct UpAdjArgs {
  const float* g_full;       // [N][H][W]
  const float* disp;         // [N][dh][dw] sigmoid output (for the derivative)
  int dw, dh;
  float rx, ry;
  const double* mean_partials;
  int mean_parts;
  const double* smooth_tsum;     // [N][smooth_parts] fp64 sum(u * d) or nullptr
  int smooth_parts;
  float ws;
  int sigmoid;               // multiply by s(1-s)
  int accumulate;
  float* out;                // [N][dh][dw]
  int N, W, H;
};

struct UpAdjBatch {
  UpAdjArgs s[MAX_SCALES];   // every scale shares N and W
};

// per-image sums of one scale's upsampled disparity (the smoothness mean normalisation)
struct DispSumArgs {
  const float* disp;         // [N][dh][dw]
  int dw, dh;
  float rx, ry;
  double* out;               // [N][parts] (fp64: the mean feeds a cancelling normalisation)
};
struct DispSumBatch {
  DispSumArgs s[MAX_SCALES];
  int W, H, N, parts;
};

struct FinalizeArgs {
  const float* photo_partials[MAX_SCALES];
  long photo_blocks[MAX_SCALES];
  const float* smooth_partials[MAX_SCALES];
  long smooth_blocks[MAX_SCALES];
  float smooth_scale[MAX_SCALES];   // smoothness * scale  (the term's forward weight)
  float photo_scale;                // 1 / (N*H*W)
  float* terms;                     // [nscales][2]
  float divisor;                    // train_loss: nscales; slow_depth: 1
  int nscales;
  int N;
};

// all a.nscales scales in one launch (photo.hip)
int launch_photometric(const PhotoArgs& a, const Geom& g, int C, hipStream_t st);
// the packed-fp32 photometric kernel (photo2.hip), launched by launch_photometric
int launch_photo2(const PhotoArgs& a, const Geom& g, const PhotoTiling& tl, int C, bool cells, long blocks,
                  hipStream_t st);
// identity-reprojection loss (training.jl:9-11): out [N][H][W] = min over the two raw sources of
// photometric_loss(source, target)
int launch_automask(const float* x, long x_sample_stride, long x_frame_stride, int target,
                    int src0, int src1, int N, int C, int H, int W, float* out, hipStream_t st);
// warped sources only (train_loss vis_warped): out [2][N][C][H][W]
int launch_warp_vis(const PhotoArgs& a, int scale, const Geom& g, int C, float* out, hipStream_t st);
// partial rows per scale of the photometric pass run with `nscales` scales
long photometric_blocks(int W, int H, int N, int nscales);
long smooth_blocks(int W, int H, int N);
// the next three run every scale of the loss tail in ONE launch each (scale = grid z)
int launch_disp_sum(const DispSumBatch& b, int nscales, hipStream_t st);
int launch_smooth(const SmoothArgs* a, int nscales, int C, hipStream_t st);
int launch_up_adjoint(const UpAdjArgs* a, int nscales, hipStream_t st);
int launch_loss_finalize(const FinalizeArgs& a, float* dRt, float* loss, hipStream_t st);
// per-(source, sample) sums of the photometric blocks' pose partials -> dRt [2N][12]
int launch_pose_grad_reduce(const FinalizeArgs& a, float* dRt, hipStream_t st);
int launch_so3_fwd(const float* pose, int count, int N, int invert_mask, float* Rt,
                   hipStream_t st);
int launch_so3_bwd(const float* pose, int count, int N, int invert_mask, const float* dRt,
                   float* dpose, int accumulate, hipStream_t st);

}  // namespace md2
