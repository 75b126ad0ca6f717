// Model executor: Model(encoder, DepthDecoder, PoseDecoder) forward + train_loss + backward +
// ADAM on the HIP kernels (src/model.jl, src/depth_decoder.jl, src/pose_decoder.jl,
// src/training.jl; encoder = ResNet.jl ResidualNetwork with torchvision topology).
#pragma once
#include <string>
#include <vector>

#include "conv.h"
#include "loss_tail.h"
#include "nn.h"

namespace md2 {

struct ArchCfg {
  int arch = 18;           // 18 / 34 / 50
  int in_ch = 3;
  int nlevels = 4;
  int levels[MAX_SCALES] = {2, 3, 4, 5};
  int emb = 0;             // DepthDecoder embedding_levels (0: mono mode; 21: MPI mode)
};

struct ParamEntry {
  std::string name;
  int ndim;
  int shape[4];
  long offset;
  long numel;
};

// flat parameter table in the order of oracle/md2_oracle.py param_spec
std::vector<ParamEntry> build_param_table(const ArchCfg& a);

struct ModelCfg {
  ArchCfg arch;
  int N, W, H;             // samples per step, target size
  float K[9], invK[9];
  float min_depth = 0.1f, max_depth = 100.f, smoothness = 1e-3f;
  float scales[MAX_SCALES] = {0.125f, 0.25f, 0.5f, 1.f};
  int automask = 0;
  int target = 1, src0 = 0, src1 = 2;   // 0-based frame ids, L = 3
  int num_bins = 32;       // MPI mode (arch.emb > 0): disparity planes per sample
};

// profiling categories (HIP events around each launch, md2_model_profile_read)
enum ProfCat : int { PROF_CONV3_ENC = 0, PROF_CONV_OTHER = 1, PROF_PHOTO = 2, PROF_NCAT = 3 };

class Model;
int model_set_profiling(Model* m, int on);
// out[cat*3 + {0,1,2}] = {total ms, total algorithmic work (FLOP or bytes), launches}
int model_profile_read(Model* m, double* out, int ncat);
int model_profile_records(Model* m, int max, double* ms, double* work, int* cat, char* tags,
                          int tag_len, int* count);
int model_create(const ModelCfg& cfg, float* params, float* grads, Model** out);
// scale_levels validation shared by the parameter table and the executor (MD2_ENOTSUP for
// non-increasing levels)
int check_scale_levels(const ArchCfg& a);
void model_destroy(Model* m);

// train path
int model_forward_loss(Model* m, const float* x, const float* automask, float* loss, float* terms,
                       hipStream_t st);
// forward only ((m)(x, source_ids, target_id), src/model.jl:31-55): outputs via model_outputs;
// a backward after it needs model_set_cotangents
int model_forward(Model* m, const float* x, hipStream_t st);
// cotangents of the last forward's outputs: d_disp[level] w.r.t. each disparity (nullptr array or
// entry: zero), d_pose [2N][6] (nullptr: zero); then model_backward_segment as after forward_loss
int model_set_cotangents(Model* m, const float* const* d_disp, const float* d_pose, hipStream_t st);
int model_num_segments(Model* m);
// runs backward segment k (0 = pose+decoder ... last = stem); [off, off+len) of the flat gradient
// is final afterwards
int model_backward_segment(Model* m, int k, long* off, long* len, hipStream_t st);
int model_adam(Model* m, float* adam_m, float* adam_v, float lr, float b1, float b2, float eps,
               int step, float grad_scale, hipStream_t st);
int model_repack(Model* m, hipStream_t st);   // after the parameters changed
// ADAM over backward segment k's parameter range + the re-pack of its conv weights, enqueued on
// the executor's update stream after everything enqueued on st so far (call it right after
// model_backward_segment(k) -- and after the bucket's all-reduce in DP); model_adam_join makes st
// wait for all of them (forward_loss, eval, model_adam and the parameter copies join first)
int model_adam_segment(Model* m, int k, float* adam_m, float* adam_v, float lr, float b1, float b2,
                       float eps, int step, float grad_scale, hipStream_t st);
int model_adam_join(Model* m, hipStream_t st);
// whether the train-step entry points use the per-segment update: MD2_SEG_UPDATE=1 (default off --
// at N=1 the concurrent updates slowed the step by 2%, profiles/r04_seg_update_ab.txt)
bool model_segment_update_enabled();
// forward + loss + backward + ADAM(0.9, 0.999, 1e-8) replayed as one captured hipGraph
int model_train_step_graph(Model* m, const float* x, const float* auto_loss, float* adam_m,
                           float* adam_v, float lr, int step, float* loss, hipStream_t st);
// MPI mode: the disparity bins [N][num_bins] of the next forwards (device; copied)
int model_set_bins(Model* m, const float* bins, hipStream_t st);
// outputs of the last forward
int model_outputs(Model* m, const float** disp, int* dw, int* dh, const float** pose);
// the five encoder stage outputs of the last forward: [3N frame-major images][c][h][w]
int model_features(Model* m, const float** feat, int* c, int* h, int* w);
// inference: eval_disparity (src/model.jl:63) on x [n][C][H][W], n <= N*3
int model_eval_disparity(Model* m, const float* x, int n, float** disp_out, hipStream_t st);
int model_debug_tensor(Model* m, int index, const char** name, const void** ptr, int* dims);
long model_param_count(Model* m);
// flat vectors in Flux layout (conv weights as true convolutions: taps reversed)
int model_set_params_flux(Model* m, const float* flux, hipStream_t st);
int model_get_params_flux(Model* m, float* flux, hipStream_t st);
int model_get_grads_flux(Model* m, float* flux, hipStream_t st);
// scale the loss-tail gradients of the last forward by the train_loss cotangent
int model_scale_loss_cotangent(Model* m, float dloss, hipStream_t st);
float* model_grads(Model* m);          // the caller-owned flat gradient vector
size_t model_device_bytes(Model* m);

}  // namespace md2

// opaque handle of the C ABI (include/md2.h)
struct md2_model {
  md2::Model* impl;
};
