// Implicit-GEMM 2-D convolution on gfx950 fp32 MFMA: forward, data-gradient, filter-gradient.
//
// Replaces NNlib conv / ∇conv_data / ∇conv_filter behind Flux `Conv` (src/depth_decoder.jl:13-14,
// 46; src/pose_decoder.jl:15-19; the ResNet.jl encoder).  Weights are stored as cross-correlation
// kernels [Cout][Cin][KH][KW] (the Julia shim flips Flux's true-convolution kernels).
#pragma once
#include "common.h"

namespace md2 {

enum Act : int { ACT_NONE = 0, ACT_RELU = 1, ACT_ELU = 2, ACT_SIGMOID = 3 };

struct ConvShape {
  int N;            // images
  int Cin, H, W;    // input
  int Cout, Ho, Wo; // output
  int KH, KW, stride, pad;
  int reflect;      // 1: NNlib pad_reflect(x, pad) + valid conv (src/depth_decoder.jl:5)
  int cin_w;        // input channels of the WEIGHT tensor [Cout][cin_w][KH][KW] when the conv runs
                    // on Cin > cin_w channels whose last Cin - cin_w are zero padding (their
                    // packed weights are zero, their filter gradients are not produced); 0: Cin
};
inline int weight_cin(const ConvShape& s) { return s.cin_w > 0 ? s.cin_w : s.Cin; }

// Input operand: channel concat of up to two tensors (cat(..., dims=3)), each [img][c][H][W].
// p0 image offset = (b % bdiv) * bs0 + (b / bdiv) * bhi  (lets the stem read x[n][l] frames
// in frame-major encoder order); p1 image offset = b * bs1.
struct TensorIn {
  const float* p0 = nullptr;
  const float* p1 = nullptr;
  int c0 = 0;          // channels held by p0 (== Cin when p1 is unused)
  long bs0 = 0, bs1 = 0;
  int bdiv = 1 << 30;
  long bhi = 0;
};

// Output: rows m < c0 go to p0, the rest to p1 (channel split for the concat gradient).
struct TensorOut {
  float* p0 = nullptr;
  float* p1 = nullptr;
  int c0 = 1 << 30;
  long bs0 = 0, bs1 = 0;   // image strides
  const float* bias = nullptr;
  int act = ACT_NONE;
  int accumulate = 0;      // out += result
};

// Launch-boundary split-K reduce: with a SplitKDefer, a fwd/dgrad launch that runs split-K into
// a plain output (stride 1, no bias/activation/accumulate/concat, contiguous images) does NOT
// launch its reduction; `slab`/`splits` describe the [splits][M][N] partial slabs in the conv
// workspace and the caller's next kernel sums them (bn_stats_partial_slabs /
// bn_bwd_partial_slabs) before any other conv reuses the workspace.  splits == 0: the output was
// written as usual.
struct SplitKDefer {
  const float* slab = nullptr;
  int splits = 0;
  // BatchNorm statistics from the conv epilogue (conv_fwd only): the caller offers a partials
  // buffer [Cout][>= ceil(N*Ho*Wo / 256)][2] (fp64 sum, sum of squares); when the conv runs the
  // LDS-halo kernel without split-K it writes one partial per 256-pixel tile and sets
  // stats_parts to the tile count (0: not written, run bn_stats_partial as usual)
  double* stats = nullptr;
  int stats_parts = 0;
  bool keep_reduce = false;   // input: never defer the split-K reduction (only the statistics)
};

struct ConvWorkspace {
  void* ptr = nullptr;
  size_t bytes = 0;
};

// GEMM reduction order.  Tap-major (k = tap*C + c, tap = kh*KW + kw) keeps the filter tap
// constant over a K chunk, so the spatial gather address is computed once per chunk and every
// channel step is a scalar offset; it needs the channel count (and a concat split) to be a
// multiple of the chunk.  Otherwise (the 3-channel stem, 1-channel disparity heads) the order is
// channel-major k = c*KK + tap.  mode: 0 forward (C = Cin), 1 dgrad (C = Cout), 2 wgrad columns.
bool conv_tap_major(const ConvShape& s, int mode);
// forward (mode 0) / dgrad (mode 1) run the k-contiguous kernel with packed layout 1
bool conv_px2_used(const ConvShape& s, int mode);
bool conv_px3_used(const ConvShape& s, int mode);    // conv_px2 shapes + 32-row stride-1 forwards on the bf16x6 kernel
bool conv_px16_used(const ConvShape& s, int mode);   // M <= 16 (16x16x4 MFMA kernel)

// packed operand sizes (elements) -- weights are repacked K-major with zero padding
size_t conv_fwd_packed_elems(const ConvShape& s);
size_t conv_dgrad_packed_elems(const ConvShape& s);
int conv_pack_fwd(const ConvShape& s, const float* w, float* packed, hipStream_t st);
int conv_pack_dgrad(const ConvShape& s, const float* w, float* packed, hipStream_t st);

// all packs of a model in ONE launch: a device-resident job table.  A job is one conv weight
// read once in source order [Cout][Cin][KK] and scattered into its forward and (optional) dgrad
// packed layouts; the zero padding of those buffers is written once at allocation
// (conv_pack_zero), not per update.
struct PackDst {
  float* out;          // nullptr: not packed
  int tap;             // tap-major K order (conv_tap_major)
  int layout;          // 0: [Kpad][Mpad]; 1: [Kpad/16][Mpad][16] (k-contiguous chunks, conv_px2)
  int Mpad;
};
struct PackJob {
  const float* w;
  PackDst f, d;        // forward (k over Cin, rows Cout) / dgrad (k over Cout, rows Cin)
  int Cout, Cin, KK;
  int Cinw;            // the source weights' Cin (<= Cin: padded input channels stay zero)
  int tiled;           // both operands tap-major k-contiguous, Cin, Cout % 16 == 0: LDS tiles
  long block_begin;    // first block of this job in the batched grid
};
PackJob conv_pack_job(const ConvShape& s, const float* w, float* out_f, float* out_d);
long conv_pack_job_blocks(const PackJob& j);
int conv_pack_batch(const PackJob* dev_jobs, int njobs, long total_blocks, hipStream_t st);

// workspace needed for split-K slabs (bytes)
size_t conv_fwd_workspace(const ConvShape& s);
size_t conv_dgrad_workspace(const ConvShape& s);
size_t conv_wgrad_workspace(const ConvShape& s);

// arithmetic of the last conv kernel launched by this host thread (profiling labels): 6 = bf16x6
// split products on the bf16 MFMA (issued ceiling 2516 / 6 TFLOP/s fp32-equivalent), 1 = fp32
// MFMA, 0 = VALU (the Cout = 1 heads)
int conv_last_arith();
int conv_fwd(const ConvShape& s, const TensorIn& x, const float* wpacked, const TensorOut& y,
             ConvWorkspace ws, hipStream_t st, SplitKDefer* defer = nullptr);
// dX from dY (dY: [N][Cout][Ho][Wo] pre-activation gradient)
int conv_dgrad(const ConvShape& s, const float* dy, const float* wpacked_d, const TensorOut& dx,
               ConvWorkspace ws, hipStream_t st, SplitKDefer* defer = nullptr);
// dW [Cout][Cin*KH*KW] (store or accumulate) and optional db [Cout]
// db_part/db_parts: bias-gradient partials [Cout][db_parts] already summed by act_backward_bias
// (the bias partial pass over dY is then skipped)
int conv_wgrad(const ConvShape& s, const TensorIn& x, const float* dy, float* dw, float* db,
               int accumulate, ConvWorkspace ws, hipStream_t st, const float* db_part = nullptr,
               int db_parts = 0);

// dPre = dOut * act'(out) (act from the stored post-activation output), elementwise
int act_backward(const float* out, const float* dout, float* dpre, long n, int act, hipStream_t st);
// the same over [N][C][HW] planes fused with the per-channel partial sums of dPre (the bias
// gradient of the conv that produced `out`): part [C][parts], parts = act_bias_parts(C, N, HW)
int act_bias_parts(int C, int N, long HW);
int act_backward_bias(const float* out, const float* dout, float* dpre, int N, int C, long HW,
                      int act, float* part, hipStream_t st);

}  // namespace md2
