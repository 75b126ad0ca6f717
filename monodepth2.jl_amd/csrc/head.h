// Single-output-channel 3x3 convolutions (DepthDecoder disparity heads, src/depth_decoder.jl:46)
// on VALU: forward / data gradient / filter gradient.  conv_fwd / conv_dgrad / conv_wgrad route
// shapes accepted by head_conv_ok here.
#pragma once
#include "conv.h"

namespace md2 {

// input planes of image b start at (b % bdiv) * bs0 + (b / bdiv) * bhi (TensorIn p0 addressing)
struct HeadIn {
  const float* p;
  long bs0;
  int bdiv;
  long bhi;
};
// filter tap (c, tap) = p[c * sc + tap * st] (read straight from the packed GEMM operand)
struct HeadW {
  const float* p;
  long sc, st;
};

bool head_conv_ok(const ConvShape& s);
size_t head_wgrad_workspace(const ConvShape& s);
int head_fwd(const ConvShape& s, const HeadIn& x, HeadW w, const float* bias, int act, float* y,
             long ybs, int accumulate, hipStream_t st);
int head_dgrad(const ConvShape& s, const float* dy, HeadW w, float* dx, long dxbs, int accumulate,
               hipStream_t st);
int head_wgrad(const ConvShape& s, const HeadIn& x, const float* dy, float* dw, float* db,
               int accumulate, void* ws, size_t ws_bytes, hipStream_t st);

// All disparity heads of the DepthDecoder in ONE launch per pass (3x3 reflect-pad, Cout = 1):
// the forward after the whole decoder, the data + filter gradients before the decoder backward.
// Each head is an HBM-bound pass over its input planes; batched, the four heads share one launch
// floor and fill the chip together instead of one small grid at a time.
constexpr int MAX_HEADS = 5;
struct HeadJob {
  HeadIn x;             // input planes (the branch output o2)
  HeadW wf, wd;         // forward / data-gradient views of the packed weights (conv_head_w)
  int Cin, H, W, N;
  const float* bias;
  float* y;             // forward output, image stride ybs
  long ybs;
  const float* dy;      // backward: d loss / d pre-activation, [N][H][W]
  float* dx;            // d loss / d x, image stride dxbs (written, not accumulated)
  long dxbs;
  float* dw;            // [Cin * 9] (written)
  float* db;            // [1] (written) or nullptr
};
int heads_fwd(const HeadJob* jobs, int n, int act, hipStream_t st);
size_t heads_bwd_workspace(const HeadJob* jobs, int n);
int heads_bwd(const HeadJob* jobs, int n, void* ws, size_t ws_bytes, hipStream_t st);
HeadIn conv_head_in(const TensorIn& x);
HeadW conv_head_w(const ConvShape& s, int mode, const float* packed);

}  // namespace md2
