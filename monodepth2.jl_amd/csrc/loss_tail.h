// Host orchestration of the loss tail: composeT -> per scale {mean, warp+SSIM, smoothness,
// upsample adjoint} -> deterministic reductions -> composeT/so3 backward.
#pragma once
#include "loss_kernels.h"

namespace md2 {

struct LossTailCfg {
  int N, C, W, H;             // samples, channels, target resolution
  int nscales;
  int dw[MAX_SCALES], dh[MAX_SCALES];
  float smooth_w[MAX_SCALES]; // forward weight of the smooth term (train_loss: smoothness*scale)
  float divisor;              // train_loss: nscales (src/training.jl:77); slow_depth: 1
  int smooth_normalize;       // divide the disparity by its per-image mean (training.jl:64-65)
  float K[9], invK[9];
  float min_depth, max_depth;
  long x_sample_stride, x_frame_stride;
  int target, src0, src1;     // 0-based frame indices
  int invert_mask;            // bit s: source s uses the inverse transform (src < target)
  int sigmoid_grad;           // 1: d_disp is w.r.t. the head pre-activation (s(1-s) fused)
};

constexpr int MEAN_PARTS = 64;

size_t loss_tail_workspace_bytes(const LossTailCfg& c);

struct LossTailOut {
  float* loss;
  float* terms;
  float* d_disp[MAX_SCALES];
  float* d_pose;
  float* vis_loss;
  signed char* vis_sel;
  float* vis_warped;                    // [2][N][C][H][W] warped sources at the last scale or nullptr
  int* vis_cell;                        // [nscales][2][N][H][W] bilinear cells (diagnostics) or nullptr
  hipEvent_t* photo_events = nullptr;   // optional [2]: around the (all-scale) photometric launch
};

// disp[s]: [N][dh][dw] sigmoid outputs; pose: [2N][6] (rvec, tvec) per (source, sample);
// x: frames; automask: [N][H][W] or nullptr.  dloss: upstream scalar gradient.
int loss_tail_run(const LossTailCfg& c, const float* const* disp, const float* pose,
                  const float* x, const float* automask, float dloss, const LossTailOut& o,
                  void* workspace, hipStream_t st);

// Op-level per-scale warp + photometric loss (md2_warp_photometric_*).
struct WarpOpCfg {
  int N, C, W, H, dw, dh;
  float K[9], invK[9];
  float min_depth, max_depth;
  long x_sample_stride, x_frame_stride;
  int target, src0, src1;
};
size_t warp_op_workspace_bytes(int N, int W, int H);
// d_loss == nullptr: forward only (loss_map / sel_map); else also the pullback of sum(d_loss .*
// warp_loss) into d_disp [N][dh][dw] and d_Rt [2N][12] (each optional).
int warp_op_run(const WarpOpCfg& c, const float* disp, const float* Rt, const float* x,
                const float* automask, const float* d_loss, float* loss_map, signed char* sel_map,
                float* d_disp, float* d_Rt, void* workspace, hipStream_t st);

}  // namespace md2
