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

}  // namespace md2
