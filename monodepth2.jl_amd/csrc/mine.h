// MINE plane rendering of the MPI mode (src/render.jl:21-114), forward.
#pragma once
#include "common.h"

namespace md2 {

struct Mat3 {
  float m[9];   // row-major
};

int mine_src_xyz(const float* disparity, int N, int B, int H, int W, const Mat3& invK, float* xyz,
                 hipStream_t st);
int mine_tgt_xyz(const float* xyz_src, const float* pose, int N, int B, int H, int W, float* xyz_tgt,
                 hipStream_t st);
int mine_sample(const float* src, int C, const float* depth, const float* pose, int N, int B, int H,
                int W, const Mat3& K, const Mat3& invK, float* out, float* valid, hipStream_t st);
int plane_volume_rendering(const float* rgb, const float* sigma, const float* xyz, int N, int B, int H,
                           int W, float* rgb_out, float* transparency_acc, float* weights,
                           hipStream_t st);
int render_tgt_rgb_depth(const float* rgb, const float* sigma, const float* disparity,
                         const float* xyz_tgt, const float* pose, const Mat3& invK, const Mat3& K,
                         int N, int B, int H, int W, float* rgb_out, float* depth, float* mask,
                         hipStream_t st);

}  // namespace md2
