/* md2.h -- C ABI of libmd2hip.so, the MI355X (gfx950) hot path of the Monodepth2.jl train step.
 *
 * Every entry point is extern "C", takes plain pointers/sizes (device pointers unless noted),
 * returns 0 on success or an MD2_E* code, and leaves a message for md2_last_error().
 * `stream` is a hipStream_t passed as void* (NULL = the legacy default stream).
 *
 * Layout: Julia column-major (W,H,C,N) arrays are memory-identical to the C-order [N][C][H][W]
 * arrays used here, so a Julia ccall shim passes pointers without transposes.
 * Small matrices (K, invK, R) are ROW-major 3x3 here; the Julia shim passes permutedims(K).
 *
 * Reference interfaces replaced (paths relative to the reference root):
 *   md2_loss_*            src/training.jl:21-78  train_loss after the model call (+ Zygote pullback)
 *   md2_so3_compose_*     src/utils.jl:106-145,185-192  so3_exp_map / hat rrule / composeT
 *   md2_conv2d_*          Flux Conv + NNlib conv / ∇conv_data / ∇conv_filter (depth/pose decoders,
 *                         ResNet.jl encoder)
 *   md2_model_*           src/model.jl:24-70 Model / eval_poses / eval_disparity,
 *                         src/depth_decoder.jl, src/pose_decoder.jl, ResNet.jl ResidualNetwork
 *   md2_model_train_*     the gradient(θ) + update!(ADAM) loop of scripts/script.jl:84-86 and
 *                         src/simple_depth.jl:25-42
 */
#ifndef MD2_H
#define MD2_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Bumped on every change to an exported struct layout or signature.  2: md2_loss_out gained
 * vis_cell; md2_model_cfg gained embedding_levels and num_bins.  Bindings refuse a mismatch. */
#define MD2_ABI_VERSION 2

#define MD2_OK 0
#define MD2_EINVAL 1
#define MD2_EHIP 2
#define MD2_ENOTSUP 3
#define MD2_ENOMEM 4
#define MD2_ESTATE 5

int md2_abi_version(void);
/* hash of the sources the library was built from (csrc/Makefile BUILD_ID): bindings recompute it
 * from their source tree and refuse a stale library */
const char* md2_build_id(void);
/* thread-local message of the last failing call (never NULL). */
const char* md2_last_error(void);
/* number of visible HIP devices (host call; does not initialise a context). */
int md2_device_count(int* count);
/* async device-to-device copy on `stream` (used to hand library-owned outputs to the host) */
int md2_memcpy_d2d(void* dst, const void* src, size_t bytes, void* stream);

/* ------------------------------------------------------------------------------------------
 * Loss tail: src/training.jl:25-77 (given the model's disparities and poses) -- forward value
 * AND the Zygote pullback in one pass per scale.
 * ---------------------------------------------------------------------------------------- */
#define MD2_MAX_SCALES 5

typedef struct md2_loss_cfg {
  int n;                       /* samples (Params.batch_size)                                */
  int c;                       /* image channels (1 or 3)                                    */
  int width, height;           /* Params.target_size                                         */
  int nscales;                 /* length(TrainCache.scales)                                  */
  int scale_w[MD2_MAX_SCALES]; /* disparity resolution of each scale                         */
  int scale_h[MD2_MAX_SCALES];
  float smooth_weight[MD2_MAX_SCALES]; /* train_loss: disparity_smoothness * scale           */
  float divisor;               /* train_loss: nscales (training.jl:77); slow_depth: 1         */
  int smooth_normalize;        /* 1: disparity / (mean + 1e-7) (training.jl:64-65)           */
  float K[9];                  /* TrainCache.K, row-major                                    */
  float invK[9];               /* TrainCache.invK, row-major                                 */
  float min_depth, max_depth;  /* Params                                                      */
  long long x_sample_stride;   /* elements between samples of x (L*C*H*W for x[N][L][C][H][W]) */
  long long x_frame_stride;    /* elements between frames (C*H*W)                            */
  int target, src0, src1;      /* 0-based frame ids (TrainCache.target_id-1, source_ids-1)   */
  int invert_mask;             /* bit s set: source s < target (training.jl:29)              */
  int sigmoid_grad;            /* 1: d_disp w.r.t. the sigmoid head pre-activation           */
} md2_loss_cfg;

size_t md2_loss_workspace_size(const md2_loss_cfg* cfg);

/* Outputs of md2_loss_fwd_bwd (device pointers; NULL = not wanted, except loss). */
typedef struct md2_loss_out {
  float* loss;                       /* [1]  train_loss value                                 */
  float* terms;                      /* [nscales][2] mean warp loss, weighted smooth term     */
  float* d_disp[MD2_MAX_SCALES];     /* d loss / d disp[s] (or / d pre-sigmoid, cfg)          */
  float* d_pose;                     /* [2n][6] d loss / d (rvec, tvec)                       */
  float* vis_loss;                   /* [nscales][n][h][w] per-pixel warp loss (vis_loss)     */
  signed char* vis_sel;              /* [nscales][n][h][w] argmin source (-1 = automask)      */
  float* vis_warped;                 /* [2][n][c][h][w] both sources warped by the LAST scale
                                        (train_loss vis_warped, src/training.jl:71-73)        */
  int* vis_cell;                     /* [nscales][2][n][h][w] parity diagnostics: per pixel and
                                        source the grid_sample bilinear cell and border state,
                                        x | y << 11 | sx << 22 | sy << 24 (0-based cell corner;
                                        s = 0 interior, 1 clamped to 0, 2 clamped to W-1 / H-1);
                                        on the selected source, bits 26 + 2c = the L1 branch of
                                        channel c (1 warped < target, 2 >, 3 equal); w, h <= 2048 */
} md2_loss_out;

/* disp[s]: [n][scale_h][scale_w]; pose: [2n][6] = (rvec, tvec) for (source s, sample i) at row
 * s*n+i; x: frames; automask: [n][h][w] identity-reprojection loss or NULL (Params.automasking).
 * dloss: upstream gradient of the scalar loss (1 for gradient(θ)). */
int md2_loss_fwd_bwd(const md2_loss_cfg* cfg, const float* const* disp, const float* pose,
                     const float* x, const float* automask, float dloss,
                     const md2_loss_out* out, void* workspace, void* stream);

/* composeT(so3_exp_map(rvec), tvec, invert) for 2n poses -> Rt [2n][12] (R row-major, t). */
int md2_so3_compose_fwd(const float* pose, int n, int invert_mask, float* Rt, void* stream);
int md2_so3_compose_bwd(const float* pose, int n, int invert_mask, const float* dRt,
                        float* d_pose, void* stream);

/* ------------------------------------------------------------------------------------------
 * Op-level loss primitives at ChainRulesCore rrule granularity (fwd + pullback pairs), for a host
 * that differentiates the reference's ops one at a time (julia/MD2HIP.jl).  Layouts are the Julia
 * arrays read as C-order; small matrices row-major (the shim passes permutedims).
 *
 * md2_automasking_loss   automasking_loss(ssim, x, target; source_ids)   src/training.jl:9-11
 *   x [n][3][c][h][w]; out [n][h][w] = min over the two raw sources of photometric_loss (ties to
 *   the first source); 0-based frame ids.  Not differentiable (data only).
 * md2_ssim_{fwd,bwd}     (ssim::SSIM)(x, y)                                src/utils.jl:29-43
 *   x, y, out, dout, dx, dy: [n][c][h][w] (Julia (W,H,C,N)); dx or dy may be NULL.
 * md2_backproject_{fwd,bwd}   (b::Backproject)(depth, invK)                src/utils.jl:67-69
 *   depth [n][w*h] (Julia (1,W*H,N)); out [n][w*h][3] (Julia (3,W*H,N)); invK row-major; the
 *   invK cotangent is not formed (TrainCache constant).
 * md2_project_{fwd,bwd}   (p::Project)(points, K, R, t)                    src/utils.jl:99-103
 *   points [n][w*h][3]; R [n][9] row-major; t [n][3]; out [n][w*h][2] normalised (-1, 1);
 *   pullback to points, R, t (deterministic per-sample reductions; K's cotangent not formed).
 * md2_grid_sample_border_{fwd,bwd}   NNlib grid_sample(x, grid; padding_mode=:border),
 *   align_corners=true (src/training.jl:56): x [n][c][hi][wi], grid [n][ho][wo][2] (Julia
 *   (2,W,H,N)), out [n][c][ho][wo]; pullback to grid and (if d_x != NULL, by atomic scatter
 *   whose summation order is not fixed) to x.
 * md2_smooth_loss_{fwd,bwd}   smooth_loss(disparity, image)                 src/utils.jl:163-177
 *   disparity [n][h][w], image [n][c][h][w] (c = 1 or 3); loss: one device float.
 * md2_warp_photometric_{fwd,bwd}   one scale of train_loss's loop body     src/training.jl:43-62
 *   upsample (align_corners) -> disparity_to_depth -> Backproject -> Project(R_s, t_s) ->
 *   grid_sample(:border) -> photometric_loss per source -> min over sources [-> _apply_mask].
 *   disp [n][dh][dw]; Rt [2][n][12] = composeT outputs (R row-major, t) of source 0 then 1
 *   (md2_so3_compose_fwd); loss_map [n][h][w]; sel_map (NULL ok) = argmin (0/1, -1 automask).
 *   Pullback of sum(d_loss .* loss_map): d_disp [n][dh][dw], d_Rt [2n][12] (each NULL ok).
 * ---------------------------------------------------------------------------------------- */
int md2_automasking_loss(const float* x, int n, int c, int h, int w, int target, int src0,
                         int src1, float* out, void* stream);
/* find_static(dataset, alpha) (src/dtk.jl:51-69), the per-sample part: scores[i] =
 * mean(automasking_loss(ssim, x_i, x_i[target]; source_ids)) for the n triplets of x
 * [n][3][c][h][w]; the dataset filter keeps samples with scores[i] > alpha (md2hip.find_static).
 * workspace: md2_static_scores_workspace_size(n, h, w) bytes of device memory. */
size_t md2_static_scores_workspace_size(int n, int h, int w);
int md2_static_scores(const float* x, int n, int c, int h, int w, int target, int src0, int src1,
                      float* scores, void* workspace, void* stream);
int md2_ssim_fwd(const float* x, const float* y, int n, int c, int h, int w, float* out,
                 void* stream);
int md2_ssim_bwd(const float* x, const float* y, const float* dout, int n, int c, int h, int w,
                 float* dx, float* dy, void* stream);
int md2_backproject_fwd(const float* depth, int n, int w, int h, const float* invK, float* out,
                        void* stream);
int md2_backproject_bwd(const float* dout, int n, int w, int h, const float* invK, float* d_depth,
                        void* stream);
int md2_project_fwd(const float* points, int n, int w, int h, const float* K, const float* R,
                    const float* t, float* out, void* stream);
size_t md2_project_workspace_size(int n, int w, int h);
int md2_project_bwd(const float* points, int n, int w, int h, const float* K, const float* R,
                    const float* t, const float* dout, float* d_points, float* d_R, float* d_t,
                    void* workspace, void* stream);
int md2_grid_sample_border_fwd(const float* x, const float* grid, int n, int c, int hi, int wi,
                               int ho, int wo, float* out, void* stream);
int md2_grid_sample_border_bwd(const float* x, const float* grid, const float* dout, int n, int c,
                               int hi, int wi, int ho, int wo, float* d_grid, float* d_x,
                               void* stream);
size_t md2_smooth_loss_workspace_size(int n, int w, int h);
int md2_smooth_loss_fwd(const float* disp, const float* img, int n, int c, int h, int w,
                        float* loss, void* workspace, void* stream);
int md2_smooth_loss_bwd(const float* disp, const float* img, int n, int c, int h, int w,
                        float dloss, float* d_disp, void* workspace, void* stream);

typedef struct md2_warp_cfg {
  int n, c, width, height;       /* samples, channels, full (target) resolution              */
  int dw, dh;                    /* resolution of the disparity of this scale                */
  float K[9], invK[9];           /* row-major                                                 */
  float min_depth, max_depth;    /* Params                                                    */
  long long x_sample_stride;     /* elements between samples of x                            */
  long long x_frame_stride;      /* elements between frames                                  */
  int target, src0, src1;        /* 0-based frame ids                                        */
} md2_warp_cfg;
size_t md2_warp_photometric_workspace_size(const md2_warp_cfg* cfg);
int md2_warp_photometric_fwd(const md2_warp_cfg* cfg, const float* disp, const float* Rt,
                             const float* x, const float* automask, float* loss_map,
                             signed char* sel_map, void* workspace, void* stream);
int md2_warp_photometric_bwd(const md2_warp_cfg* cfg, const float* disp, const float* Rt,
                             const float* x, const float* automask, const float* d_loss,
                             float* d_disp, float* d_Rt, void* workspace, void* stream);

/* Data pipeline, host code: PNG files (8-bit, non-interlaced gray / RGB / RGBA)
 * decoded on `threads` host threads straight into the uint8 batch layout (lossless: the bytes of
 * FileIO/PNGFiles' N0f8 arrays).
 * md2_load_triplets_u8   Depth10k (src/dtk.jl:29-46): file i = three frames side by side (3W x H
 *                        RGB) -> out [n][3][3][H][W], frame j = columns [jW, (j+1)W); flip[i]
 *                        (NULL = none) mirrors every frame of sample i (FlipX).
 * md2_load_kitti_u8      KittyDataset (src/kitty.jl:45-61): paths[3i+k] = frame k of sample i
 *                        (8-bit gray) -> out [n][3][1][h][w], each imresize'd to (h, w) and kept
 *                        N0f8 (md2hip/data.py imresize), then flipped if flip[i].
 * Host pointers; errors name the offending file. */
int md2_png_info(const char* path, int* width, int* height, int* channels);
int md2_load_triplets_u8(const char* const* paths, int n, int width, int height,
                         const unsigned char* flip, unsigned char* out, int threads);
int md2_load_kitti_u8(const char* const* paths, int n, int height, int width,
                      const unsigned char* flip, unsigned char* out, int threads);

/* Data pipeline: N0f8 images -> Float32, out[i] = Float32(in[i]) / 255f0, the
 * `Float32.(channelview(x))` of src/dtk.jl:45 / src/kitty.jl:58 -- batches cross PCIe as bytes.
 * in 4-byte aligned, out 16-byte aligned. */
int md2_unorm8_to_float(const unsigned char* in, float* out, long long n, void* stream);

/* ------------------------------------------------------------------------------------------
 * 2-D convolution (Flux Conv / NNlib conv, ∇conv_data, ∇conv_filter) on gfx950 fp32 MFMA.
 * x [n][cin][h][w], w [cout][cin][kh][kw] (cross-correlation; flip Flux kernels), bias [cout],
 * y [n][cout][ho][wo].  reflect=1: NNlib pad_reflect(x, pad) then a valid conv
 * (src/depth_decoder.jl:5; 3x3, stride 1, pad 1 only).  act: 0 none, 1 relu, 2 elu, 3 sigmoid.
 * ---------------------------------------------------------------------------------------- */
typedef struct md2_conv_desc {
  int n, cin, h, w, cout, kh, kw, stride, pad, reflect;
  int act;
} md2_conv_desc;

size_t md2_conv2d_workspace_size(const md2_conv_desc* d);
int md2_conv2d_fwd(const md2_conv_desc* d, const float* x, const float* w, const float* bias,
                   float* y, void* workspace, void* stream);
/* dx = ∇conv_data(dy_pre) where dy_pre is the gradient w.r.t. the pre-activation output. */
int md2_conv2d_dgrad(const md2_conv_desc* d, const float* dy, const float* w, float* dx,
                     void* workspace, void* stream);
/* dw = ∇conv_filter(x, dy_pre), db = sum(dy_pre) (db may be NULL). */
int md2_conv2d_wgrad(const md2_conv_desc* d, const float* x, const float* dy, float* dw,
                     float* db, void* workspace, void* stream);
/* dpre = dout .* act'(out) from the stored post-activation output (n elements). */
int md2_act_backward(const float* out, const float* dout, float* dpre, long long n, int act,
                     void* stream);

/* ------------------------------------------------------------------------------------------
 * Pooling / resampling layers of the networks, [n][c][h][w] planes.
 * MaxPool((3,3), pad=1, stride=2) of the ResNet.jl stem: y [n][c][ho][wo] with
 * ho = (h+1)/2, wo = (w+1)/2, arg = window index kh*3+kw of the first maximum (uint8, kept for
 * the pullback).  upsample_bilinear(x, (2,2)), align_corners (src/depth_decoder.jl:18-19):
 * y [n][c][2h][2w]; the backward is its exact adjoint dx [n][c][h][w].
 * ---------------------------------------------------------------------------------------- */
int md2_maxpool3s2_fwd(const float* x, int n, int c, int h, int w, float* y, unsigned char* arg,
                       void* stream);
int md2_maxpool3s2_bwd(const float* dy, const unsigned char* arg, int n, int c, int h, int w,
                       float* dx, void* stream);
int md2_upsample2_fwd(const float* x, int n, int c, int h, int w, float* y, void* stream);
int md2_upsample2_bwd(const float* dy, int n, int c, int h, int w, float* dx, void* stream);

/* ------------------------------------------------------------------------------------------
 * MPI mode (src/model.jl:1-55; forward only upstream).  md2_mpi_embed_features
 * builds the DepthDecoder input of one feature level: out [n*num_bins][c + 2L+1][h][w] with
 * image b*num_bins + p = cat(feat[b], repeat(embed(bins[b][p]), h, w)); embed(x) = [x, sin(2^i x),
 * cos(2^i x) for i in 0:L-1] (src/model.jl:4-15); feat[b] at feat + b*sample_stride.
 * md2_concat_channels: cat(a, b; dims=3) for [n][ca][hw] and [n][cb][hw] (BranchBlock skip).
 * ---------------------------------------------------------------------------------------- */
int md2_mpi_embed_features(const float* feat, long long sample_stride, int n, int c, int h, int w,
                           const float* bins, int num_bins, int L, float* out, void* stream);
int md2_concat_channels(const float* a, int ca, const float* b, int cb, int n, long long hw,
                        float* out, void* stream);

/* ------------------------------------------------------------------------------------------
 * MINE plane rendering of the MPI mode (src/render.jl:21-114), forward (the reference defines
 * no pullback).  Arrays are the Julia arrays' bytes (column-major dims listed first):
 *   rgb (W,H,3,N,B)   sigma (W,H,1,N,B)   xyz (3,W,H,N,B)   disparity/depth (N,B)
 *   pose [B][6] = (rvec, tvec) of Pose(rvec (3,B), tvec (3,B))   K, invK 3x3 row-major (host)
 * The reference's semantics are reproduced as written (valid mask = chained comparison
 * u < W*u >= 0, grid normalised (u + 0.5)/(W/2) with no -1, last plane distance 1e3,
 * transmittance over T + 1e-6); see DESIGN.md "MINE rendering".
 * md2_mine_src_xyz   get_src_xyz_from_plane_disparity(create_meshgrid(H,W), disparity, invK)
 *                    (render.jl:21-30) -> xyz (3,W,H,N,B)
 * md2_mine_tgt_xyz   get_tgt_xyz_from_plane_disparity(xyz_src, pose) (render.jl:51-64)
 * md2_mine_sample    sample(src, depth_src, pose, K, K_inv) (render.jl:66-94): src (W,H,c,N*B),
 *                    depth (N,B) -> out (W,H,c,N*B), valid (W*H, N*B) as 0/1 floats
 * md2_plane_volume_rendering  plane_volume_rendering(rgb, sigma, xyz) (render.jl:32-49) ->
 *                    rgb_out (W,H,3,B), transparency_acc (W,H,1,N,B), weights (W,H,1,N,B)
 * md2_render_tgt_rgb_depth  render_tgt_rgb_depth(rgb, sigma, disparity, xyz_tgt, pose, invK, K)
 *                    (render.jl:96-114), one fused kernel, N <= 512 -> rgb (W,H,3,B),
 *                    depth (W,H,1,N,B), mask (W,H,1,1,B) (plane counts of the valid mask)
 * ---------------------------------------------------------------------------------------- */
int md2_mine_src_xyz(const float* disparity, int n_planes, int batch, int h, int w,
                     const float* invK, float* xyz, void* stream);
int md2_mine_tgt_xyz(const float* xyz_src, const float* pose, int n_planes, int batch, int h, int w,
                     float* xyz_tgt, void* stream);
int md2_mine_sample(const float* src, int c, const float* depth, const float* pose, int n_planes,
                    int batch, int h, int w, const float* K, const float* invK, float* out,
                    float* valid, void* stream);
int md2_plane_volume_rendering(const float* rgb, const float* sigma, const float* xyz, int n_planes,
                               int batch, int h, int w, float* rgb_out, float* transparency_acc,
                               float* weights, void* stream);
int md2_render_tgt_rgb_depth(const float* rgb, const float* sigma, const float* disparity,
                             const float* xyz_tgt, const float* pose, const float* invK,
                             const float* K, int n_planes, int batch, int h, int w, float* rgb_out,
                             float* depth, float* mask, void* stream);

/* ------------------------------------------------------------------------------------------
 * Model: Model(ResidualNetwork(arch), DepthDecoder(embedding_levels=0), PoseDecoder) in mono
 * mode (src/model.jl:24-70), train_loss (src/training.jl:21-78), its pullback, Flux ADAM.
 * Parameters / gradients are CALLER-owned flat fp32 device vectors; their order is the table
 * of md2_arch_param_info (conv weights cross-correlation [cout][cin][kh][kw], then bias;
 * BatchNorm gamma, beta).  x is [batch][3][c][h][w] (Julia (W,H,C,3,N)).
 * ---------------------------------------------------------------------------------------- */
typedef struct md2_model_cfg {
  int arch;                             /* ResidualNetwork depth: 18, 34 or 50              */
  int in_channels;                      /* 1 (grayscale) or 3                                */
  int batch;                            /* samples per step (triplets)                       */
  int width, height;                    /* Params.target_size (multiples of 32)              */
  int n_levels;                         /* length(scale_levels)                              */
  int scale_levels[MD2_MAX_SCALES];     /* DepthDecoder scale_levels in 1:5, strictly increasing
                                           (repeated / decreasing: MD2_ENOTSUP)               */
  float K[9], invK[9];                  /* TrainCache.K / invK, row-major                    */
  float min_depth, max_depth, disparity_smoothness;   /* Params                              */
  float scales[MD2_MAX_SCALES];         /* TrainCache.scales                                 */
  int automasking;                      /* Params.automasking                                */
  int target, src0, src1;               /* 0-based frame ids in 0:2 (TrainCache target_id /
                                           source_ids minus 1)                                */
  int embedding_levels;                 /* DepthDecoder(; embedding_levels): 0 = mono mode (the
                                           measured step); 2L+1 (21) = MPI mode, model.jl:31-55 */
  int num_bins;                         /* MPI mode: disparity planes per sample (model.jl:31)  */
} md2_model_cfg;

typedef struct md2_model md2_model;

/* host-only queries of the flat parameter table (no device needed) */
int md2_arch_param_count(const md2_model_cfg* cfg, long long* n_entries, long long* n_elems);
int md2_arch_param_info(const md2_model_cfg* cfg, int idx, char* name, int name_len, int* ndim,
                        int* shape4, long long* offset);

int md2_model_create(const md2_model_cfg* cfg, float* params, float* grads, md2_model** out);
int md2_model_destroy(md2_model* m);
size_t md2_model_device_bytes(md2_model* m);
/* re-pack conv weights after the caller changed `params` directly */
int md2_model_repack(md2_model* m, void* stream);
/* Flux-layout flat vectors (the order of md2_arch_param_info; conv weights as Flux stores them:
 * (kw,kh,cin,cout) TRUE-convolution kernels = C-order [cout][cin][kh][kw] with both spatial axes
 * reversed w.r.t. the library's cross-correlation).  set: copies into the model's params (taps
 * flipped) and re-packs; get: params -> Flux layout; get_grads: the flat gradient -> Flux layout
 * (what Zygote returns for Flux.params).  `flux` must not alias the model's vectors. */
int md2_model_set_params(md2_model* m, const float* flux, void* stream);
int md2_model_get_params(md2_model* m, float* flux, void* stream);
int md2_model_get_grads(md2_model* m, float* flux, void* stream);
/* train_loss pullback with an upstream cotangent (ChainRulesCore rrule): after
 * md2_model_forward_loss and before backward segment 0, scale the loss-tail gradients by dloss */
int md2_model_loss_cotangent(md2_model* m, float dloss, void* stream);
/* forward (encoder on 3*batch frames, decoder on targets, poses) + train_loss value + the
 * loss-tail pullback; terms: [n_levels][2] or NULL.  With cfg.automasking, auto_loss [batch][h][w]
 * is the caller's automasking_loss, or NULL: the library computes it from x (md2_automasking_loss). */
int md2_model_forward_loss(md2_model* m, const float* x, const float* auto_loss, float* loss,
                           float* terms, void* stream);
/* backward in segments (0 = pose+depth decoders, 1..4 = layer4..layer1, 5 = stem); after
 * segment k the flat gradient range [off, off+len) is final (bucket for the DP all-reduce) */
/* (m)(x, source_ids, target_id) -> (disparities, poses) (src/model.jl:31-55; called at
 * src/training.jl:26 and, bare, scripts/script.jl:93): the forward only -- encoder, DepthDecoder,
 * PoseDecoder, no loss tail.  disp[level] ([batch*num_bins][h][w]) and *pose ([2*batch][6]) are
 * set to the model's output buffers (either may be NULL), the values md2_model_forward_loss would
 * produce for the same x, bit for bit.  A backward after it needs the outputs' cotangents. */
int md2_model_forward(md2_model* m, const float* x, const float** disp, const float** pose,
                      void* stream);
/* The pullback of md2_model_forward from caller cotangents (a host that differentiates its own
 * loss, e.g. the reference's train_loss through Zygote): d_disp[level] = d L / d disparity of that
 * level, laid out as the outputs (NULL array or entry: zero), d_pose [2*batch][6] (NULL: zero).
 * md2_model_set_cotangents only installs them -- the backward segments then run as after
 * md2_model_forward_loss (DP buckets unchanged); md2_model_backward_from installs them and runs
 * every segment.  The flat gradient equals the fused path's bit for bit when the cotangents equal
 * the loss tail's own (md2_loss_fwd_bwd with sigmoid_grad = 0). */
int md2_model_set_cotangents(md2_model* m, const float* const* d_disp, const float* d_pose,
                             void* stream);
int md2_model_backward_from(md2_model* m, const float* const* d_disp, const float* d_pose,
                            void* stream);
int md2_model_num_segments(md2_model* m);
int md2_model_backward_segment(md2_model* m, int k, long long* off, long long* len,
                               void* stream);
/* update!(ADAM(lr, (beta1, beta2)), θ, ∇) on any flat fp32 device vector of n elements (Flux
 * ADAM, eps on the bias-corrected sqrt(v)); `step` >= 1 counts updates of this vector; the
 * gradient is scaled by grad_scale first (1/world for a summed DP gradient).  The free-variable
 * loop of slow_depth (src/simple_depth.jl:20-43) uses it directly. */
int md2_adam(float* p, const float* g, float* adam_m, float* adam_v, long long n, float lr,
             float beta1, float beta2, float eps, int step, float grad_scale, void* stream);
/* Flux ADAM step over the flat vectors (bias correction with `step` >= 1); gradients are
 * multiplied by grad_scale first (1/world_size after a sum all-reduce); re-packs weights */
int md2_model_adam(md2_model* m, float* adam_m, float* adam_v, float lr, float beta1,
                   float beta2, float eps, int step, float grad_scale, void* stream);
/* The update of ONE backward segment's parameters (the range model_backward_segment returned):
 * ADAM as md2_model_adam over that range + the re-pack of its conv weights, enqueued on the
 * executor's own update stream ordered after everything enqueued on `stream` so far -- called
 * right after md2_model_backward_segment(segment) (a DP caller: on the stream its bucket's
 * all-reduce ran on) it runs beside the remaining backward.  Every segment of a step takes the
 * same `step`.  md2_model_adam_join makes `stream` wait for all pending segment updates
 * (md2_model_forward_loss, eval_disparity, md2_model_adam and the parameter copies join first). */
int md2_model_adam_segment(md2_model* m, int segment, float* adam_m, float* adam_v, float lr,
                           float beta1, float beta2, float eps, int step, float grad_scale, void* stream);
int md2_model_adam_join(md2_model* m, void* stream);
/* forward_loss + every backward segment + ADAM (single-GPU step).  By default ONE update runs
 * after the last segment; MD2_SEG_UPDATE=1 opts into each segment's update beside the remaining
 * backward (md2_model_adam_segment; measured 2% slower at N=1) */
int md2_model_train_step(md2_model* m, const float* x, const float* auto_loss, float* adam_m,
                         float* adam_v, float lr, int step, float* loss, void* stream);
/* md2_model_train_step as ONE captured hipGraph (forward, loss, every backward segment, ADAM,
 * weight repack): captured on the executor's own stream at the first call and again when adam_m,
 * adam_v, lr or the presence of auto_loss change; x / auto_loss are copied into executor-owned
 * buffers each call (any pointer may be passed), the loss is copied out; `step` may jump (the
 * device step counter is re-set).  Same arithmetic, same results as md2_model_train_step. */
int md2_model_train_step_graph(md2_model* m, const float* x, const float* auto_loss, float* adam_m,
                               float* adam_v, float lr, int step, float* loss, void* stream);
/* ------------------------------------------------------------------------------------------
 * Data parallelism over RCCL (xGMI), one process (rank) per GPU -- SURVEY.md 8(e).  The
 * reference has no collectives; these replace the torch.distributed plumbing so a Julia host
 * needs only this library.  RCCL is dlopen'ed on first use (MD2_ENOTSUP if absent).
 * md2_comm_get_unique_id: rank 0 creates the 128-byte id and ships it to the other ranks (file,
 * MPI, a TCP store ...); md2_comm_init then joins (collective over all ranks) on `device` (the
 * caller's current device is restored before it returns).
 * md2_model_backward_allreduce: every backward segment on `stream`, each followed by the RCCL
 * sum of its (final) gradient range on the communicator's own stream -- bucketed, overlapped with
 * the rest of the backward; `stream` waits for all buckets before returning.  comm == NULL:
 * plain backward.  md2_model_train_step_dp: forward_loss + that + ADAM with grad_scale 1/nranks
 * (one update after the last bucket by default; MD2_SEG_UPDATE=1: each bucket's ADAM + re-pack
 * on the update stream right after its all-reduce).
 * ---------------------------------------------------------------------------------------- */
#define MD2_COMM_ID_BYTES 128
typedef struct md2_comm md2_comm;
int md2_comm_get_unique_id(char* id);
int md2_comm_init(int rank, int nranks, const char* id, int device, md2_comm** out);
int md2_comm_destroy(md2_comm* comm);
/* rank and size as the RCCL communicator reports them (ncclCommUserRank / ncclCommCount) */
int md2_comm_rank(const md2_comm* comm, int* rank, int* nranks);
/* all-reduces enqueued through this communicator and their payload bytes, cumulative */
int md2_comm_stats(const md2_comm* comm, long long* calls, long long* bytes);
/* in-place sum all-reduce of n floats, on `stream` (RCCL's ordering) */
int md2_comm_allreduce_sum(md2_comm* comm, float* buf, long long n, void* stream);
int md2_model_backward_allreduce(md2_model* m, md2_comm* comm, void* stream);
int md2_model_train_step_dp(md2_model* m, md2_comm* comm, const float* x, const float* auto_loss,
                            float* adam_m, float* adam_v, float lr, float beta1, float beta2,
                            float eps, int step, float* loss, void* stream);

/* MPI mode (embedding_levels > 0; src/model.jl:31-55, batch 1): the decoder runs on
 * num_bins*batch plane images, image n*num_bins + p = cat(target features of sample n,
 * repeat(embed(bins[n][p]), h, w)); the loss treats the planes as the batch, each warped with
 * its sample's poses against its sample's frames (the broadcast of src/training.jl:42-56); the
 * backward block-sums the planes' feature gradients (_repeat pullback, src/repeat.jl:44-53).
 * bins [batch][num_bins] (device or host): uniformly_sample_disparity_from_linspace_bins's draw
 * (src/model.jl:17-21, CUDA.rand there), used by every following forward until set again. */
int md2_model_set_disparity_bins(md2_model* m, const float* bins, void* stream);

/* device pointers of the last forward: disparities per level ([batch*num_bins][h][w] in MPI
 * mode) and poses [2*batch][6] */
int md2_model_outputs(md2_model* m, const float** disp, int* w, int* h, const float** pose);
/* The five encoder stage outputs of the last forward (device memory owned by the model):
 * feat[k] = [3n frame-major images][c[k]][h[k]][w[k]] (image l*n + i = frame l of sample i). */
int md2_model_features(md2_model* m, const float** feat, int* c, int* h, int* w);
/* HIP-event profiling of the hot kernels on the model's stream (bench roofline): categories
 * 0 = zero-padded 3x3 convs (encoder + pose decoder; fwd/dgrad/wgrad incl. their split-K
 * reductions, work = algorithmic FLOP), 1 = other convs,
 * 2 = fused warp+SSIM photometric kernel (work = algorithmic HBM bytes).
 * out[cat*3 + {0,1,2}] = {total ms, total work, launches}; read() clears. */
#define MD2_PROF_NCAT 3
int md2_model_set_profiling(md2_model* m, int on);
int md2_model_profile_read(md2_model* m, double* out, int ncat);
/* the same events one record at a time (per-layer table): ms, work, category and a tag ("fwd
 * 3x3/1 64->64 32x104 n36" for a conv: pass, kernel/stride[r = reflect pad], channels, input
 * size, images); up to `max` records, *count set; clears like md2_model_profile_read. */
int md2_model_profile_records(md2_model* m, int max, double* ms, double* work, int* cat, char* tags,
                              int tag_len, int* count);
/* Diagnostics (parity tests): named internal buffers of the last forward / backward, by index
 * 0..count-1 (MD2_EINVAL past the end): encoder activations ("stem.y", "stem.out",
 * "maxpool.out", "maxpool.arg" = window index kh*3+kw as uint8, "layer<s>.<b>.conv<k>.y",
 * "...relu1", "....out", "....down.y"), block-output gradients "....d_out", pose activations
 * "pose.sq", "pose.conv1", "pose.conv2", decoder skip gradients "d_skip<f>", "d_mp", "d_f0".
 * Images are in the encoder's frame-major order (image = frame*batch + n).
 * dims = {images, channels, height, width, dtype (0 float32, 1 uint8)}; *name valid until the
 * next call. */
int md2_model_debug_tensor(md2_model* m, int index, const char** name, const void** ptr,
                           int* dims);
/* eval_disparity (src/model.jl:63) on x [n][c][h][w], n <= batch; disp: per-level pointers.
 * It reuses the executor's activation buffers: a pending forward_loss is discarded and a later
 * md2_model_backward_segment returns MD2_ESTATE until the next forward_loss. */
int md2_model_eval_disparity(md2_model* m, const float* x, int n, const float** disp,
                             void* stream);

#ifdef __cplusplus
}
#endif

#endif /* MD2_H */
