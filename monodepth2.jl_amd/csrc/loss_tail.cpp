// Loss-tail orchestration (src/training.jl:21-78 after the model call).
#include "loss_tail.h"

#include <cstring>

namespace md2 {

namespace {
inline size_t align256(size_t b) { return (b + 255) & ~size_t(255); }

struct TailLayout {
  size_t Rt, dRt, g_full[MAX_SCALES], mean, photo[MAX_SCALES], smooth[MAX_SCALES], tsum[MAX_SCALES],
      terms, total;
};

TailLayout layout(const LossTailCfg& c) {
  TailLayout L{};
  size_t off = 0;
  auto take = [&](size_t bytes) {
    size_t o = off;
    off += align256(bytes);
    return o;
  };
  L.Rt = take(sizeof(float) * 2 * c.N * 12);
  L.dRt = take(sizeof(float) * 2 * c.N * 12);
  L.mean = take(sizeof(double) * (size_t)c.nscales * c.N * MEAN_PARTS);
  for (int s = 0; s < c.nscales; ++s) {
    L.g_full[s] = take(sizeof(float) * (size_t)c.N * c.W * c.H);
    L.photo[s] = take(sizeof(float) * 25 * photometric_blocks(c.W, c.H, c.N, c.nscales));
    L.smooth[s] = take(sizeof(float) * 2 * smooth_blocks(c.W, c.H, c.N));
    L.tsum[s] = take(sizeof(double) * smooth_blocks(c.W, c.H, c.N));
  }
  L.terms = take(sizeof(float) * 2 * MAX_SCALES);
  L.total = off;
  return L;
}

inline float ratio(int in, int out) { return out > 1 ? (float)(in - 1) / (float)(out - 1) : 0.f; }
}  // namespace

size_t loss_tail_workspace_bytes(const LossTailCfg& c) { return layout(c).total; }

int loss_tail_run(const LossTailCfg& c, const float* const* disp, const float* pose,
                  const float* x, const float* automask, float dloss, const LossTailOut& o,
                  void* workspace, hipStream_t st) {
  float* loss = o.loss;
  float* terms = o.terms;
  const float* const* d_disp = o.d_disp;
  float* d_pose = o.d_pose;
  MD2_CHECK_ARG(c.N > 0 && c.W > 2 && c.H > 2, "loss tail dims");
  MD2_CHECK_ARG(c.nscales >= 1 && c.nscales <= MAX_SCALES, "nscales");
  MD2_CHECK_ARG(c.C == 1 || c.C == 3, "channels must be 1 or 3");
  MD2_CHECK_ARG(workspace != nullptr && disp != nullptr && pose != nullptr && x != nullptr,
                "null pointer");
  const TailLayout L = layout(c);
  char* ws = (char*)workspace;
  float* Rt = (float*)(ws + L.Rt);
  float* dRt = (float*)(ws + L.dRt);
  double* mean = (double*)(ws + L.mean);
  float* tterms = terms ? terms : (float*)(ws + L.terms);

  Geom g;
  std::memcpy(g.K, c.K, sizeof(g.K));
  std::memcpy(g.invK, c.invK, sizeof(g.invK));
  g.min_disp = (float)(1.0 / c.max_depth);
  g.disp_range = (float)(1.0 / c.min_depth - 1.0 / c.max_depth);
  g.W = c.W;
  g.H = c.H;
  g.wm1 = (float)(c.W - 1);
  g.hm1 = (float)(c.H - 1);

  MD2_TRY(launch_so3_fwd(pose, 2 * c.N, c.N, c.invert_mask, Rt, st));

  const float up = dloss / c.divisor;
  const long photo_blk = photometric_blocks(c.W, c.H, c.N, c.nscales);
  const long smooth_blk = smooth_blocks(c.W, c.H, c.N);
  FinalizeArgs fa{};
  fa.nscales = c.nscales;
  fa.N = c.N;
  fa.photo_scale = 1.f / ((float)c.N * c.W * c.H);
  fa.terms = tterms;
  fa.divisor = c.divisor;

  // all scales' warp + SSIM + L1 forward and pullback in one launch (photo.hip)
  PhotoArgs pa{};
  pa.nscales = c.nscales;
  pa.x = x;
  pa.x_sample_stride = c.x_sample_stride;
  pa.x_frame_stride = c.x_frame_stride;
  pa.target = c.target;
  pa.src0 = c.src0;
  pa.src1 = c.src1;
  pa.Rt = Rt;
  pa.automask = automask;
  pa.wloss = up / ((float)c.N * c.W * c.H);
  pa.N = c.N;
  const size_t plane = (size_t)c.N * c.W * c.H;
  DispSumBatch db{};
  db.W = c.W;
  db.H = c.H;
  db.N = c.N;
  db.parts = MEAN_PARTS;
  for (int s = 0; s < c.nscales; ++s) {
    MD2_CHECK_ARG(c.dw[s] >= 1 && c.dh[s] >= 1 && c.dw[s] <= c.W && c.dh[s] <= c.H, "scale dims");
    PhotoScale& ps = pa.sc[s];
    ps.disp = disp[s];
    ps.dw = c.dw[s];
    ps.dh = c.dh[s];
    ps.rx = ratio(c.dw[s], c.W);
    ps.ry = ratio(c.dh[s], c.H);
    ps.g_disp = (float*)(ws + L.g_full[s]);
    ps.partials = (float*)(ws + L.photo[s]);
    ps.loss_map = o.vis_loss ? o.vis_loss + s * plane : nullptr;
    ps.sel_map = o.vis_sel ? o.vis_sel + s * plane : nullptr;
    ps.cell_map = o.vis_cell ? o.vis_cell + 2 * s * plane : nullptr;
    db.s[s] = DispSumArgs{disp[s], c.dw[s], c.dh[s], ps.rx, ps.ry, mean + (size_t)s * c.N * MEAN_PARTS};
  }
  MD2_TRY(launch_disp_sum(db, c.nscales, st));   // every scale's mean in one launch
  if (o.photo_events) MD2_HIP(hipEventRecord(o.photo_events[0], st));
  MD2_TRY(launch_photometric(pa, g, c.C, st));
  if (o.photo_events) MD2_HIP(hipEventRecord(o.photo_events[1], st));
  if (o.vis_warped) MD2_TRY(launch_warp_vis(pa, c.nscales - 1, g, c.C, o.vis_warped, st));

  // smoothness and the upsample adjoint: every scale in one launch each (scale = grid z)
  SmoothArgs sas[MAX_SCALES];
  UpAdjArgs uas[MAX_SCALES];
  int nua = 0;
  for (int s = 0; s < c.nscales; ++s) {
    const PhotoScale& ps = pa.sc[s];
    double* mp = mean + (size_t)s * c.N * MEAN_PARTS;
    float* sp = (float*)(ws + L.smooth[s]);
    double* tp = (double*)(ws + L.tsum[s]);
    SmoothArgs& sa = sas[s];
    sa = SmoothArgs{};
    sa.disp = disp[s];
    sa.dw = c.dw[s];
    sa.dh = c.dh[s];
    sa.rx = ps.rx;
    sa.ry = ps.ry;
    sa.img = x + (long)c.target * c.x_frame_stride;
    sa.img_sample_stride = c.x_sample_stride;
    sa.mean_partials = c.smooth_normalize ? mp : nullptr;
    sa.mean_parts = c.smooth_normalize ? MEAN_PARTS : 0;
    sa.ws = up * c.smooth_w[s];
    sa.g_disp = ps.g_disp;
    sa.partials = sp;
    sa.tsum = c.smooth_normalize ? tp : nullptr;
    sa.N = c.N;
    sa.W = c.W;
    sa.H = c.H;

    UpAdjArgs ua{};
    ua.g_full = ps.g_disp;
    ua.disp = disp[s];
    ua.dw = c.dw[s];
    ua.dh = c.dh[s];
    ua.rx = ps.rx;
    ua.ry = ps.ry;
    ua.mean_partials = mp;
    ua.mean_parts = MEAN_PARTS;
    ua.smooth_tsum = c.smooth_normalize ? tp : nullptr;
    ua.smooth_parts = (int)(smooth_blk / c.N);
    ua.ws = sa.ws;
    ua.sigmoid = c.sigmoid_grad;
    ua.accumulate = 0;
    ua.out = (float*)d_disp[s];
    ua.N = c.N;
    ua.W = c.W;
    ua.H = c.H;
    if (d_disp[s]) uas[nua++] = ua;

    fa.photo_partials[s] = ps.partials;
    fa.photo_blocks[s] = photo_blk;
    fa.smooth_partials[s] = sp;
    fa.smooth_blocks[s] = smooth_blk;
    fa.smooth_scale[s] = c.smooth_w[s];
  }
  MD2_TRY(launch_smooth(sas, c.nscales, c.C, st));
  if (nua > 0) MD2_TRY(launch_up_adjoint(uas, nua, st));
  MD2_TRY(launch_loss_finalize(fa, d_pose ? dRt : nullptr, loss, st));
  if (d_pose) MD2_TRY(launch_so3_bwd(pose, 2 * c.N, c.N, c.invert_mask, dRt, d_pose, 0, st));
  return MD2_OK;
}


// ---------------------------------------------------------------------------------------------
// Op-level warp + photometric loss of ONE scale (src/training.jl:43-62): upsample the disparity,
// depth, backproject, project with each composed pose, border grid_sample, SSIM + L1, min over
// the two sources (and the automask).  Forward: the per-pixel warp_loss map; pullback: from a
// per-pixel cotangent map to the disparity and to the composed poses Rt.
// ---------------------------------------------------------------------------------------------
size_t warp_op_workspace_bytes(int N, int W, int H) {
  return align256(sizeof(float) * (size_t)N * W * H) +
         align256(sizeof(float) * 25 * photometric_blocks(W, H, N, 1));
}

int warp_op_run(const WarpOpCfg& c, const float* disp, const float* Rt, const float* x,
                const float* automask, const float* d_loss, float* loss_map, signed char* sel_map,
                float* d_disp, float* d_Rt, void* workspace, hipStream_t st) {
  MD2_CHECK_ARG(c.N > 0 && c.W > 2 && c.H > 2 && c.dw >= 1 && c.dh >= 1 && c.dw <= c.W && c.dh <= c.H,
                "warp_photometric dims");
  MD2_CHECK_ARG(c.C == 1 || c.C == 3, "channels must be 1 or 3");
  MD2_CHECK_ARG(disp && Rt && x && workspace, "warp_photometric: null pointer");
  char* ws = (char*)workspace;
  float* g_full = (float*)ws;
  float* part = (float*)(ws + align256(sizeof(float) * (size_t)c.N * c.W * c.H));
  Geom g;
  std::memcpy(g.K, c.K, sizeof(g.K));
  std::memcpy(g.invK, c.invK, sizeof(g.invK));
  g.min_disp = (float)(1.0 / c.max_depth);
  g.disp_range = (float)(1.0 / c.min_depth - 1.0 / c.max_depth);
  g.W = c.W;
  g.H = c.H;
  g.wm1 = (float)(c.W - 1);
  g.hm1 = (float)(c.H - 1);
  PhotoArgs pa{};
  pa.nscales = 1;
  PhotoScale& ps = pa.sc[0];
  ps.disp = disp;
  ps.dw = c.dw;
  ps.dh = c.dh;
  ps.rx = ratio(c.dw, c.W);
  ps.ry = ratio(c.dh, c.H);
  ps.g_disp = g_full;
  ps.partials = part;
  ps.loss_map = loss_map;
  ps.sel_map = sel_map;
  pa.x = x;
  pa.x_sample_stride = c.x_sample_stride;
  pa.x_frame_stride = c.x_frame_stride;
  pa.target = c.target;
  pa.src0 = c.src0;
  pa.src1 = c.src1;
  pa.Rt = Rt;
  pa.automask = automask;
  pa.wloss = d_loss ? 1.f : 0.f;
  pa.gmap = d_loss;
  pa.N = c.N;
  MD2_TRY(launch_photometric(pa, g, c.C, st));
  if (!d_loss) return MD2_OK;
  if (d_disp) {
    UpAdjArgs ua{};
    ua.g_full = g_full;
    ua.disp = disp;
    ua.dw = c.dw;
    ua.dh = c.dh;
    ua.rx = ps.rx;
    ua.ry = ps.ry;
    ua.out = d_disp;
    ua.N = c.N;
    ua.W = c.W;
    ua.H = c.H;
    MD2_TRY(launch_up_adjoint(&ua, 1, st));
  }
  if (d_Rt) {
    FinalizeArgs fa{};
    fa.nscales = 1;
    fa.N = c.N;
    fa.photo_partials[0] = part;
    fa.photo_blocks[0] = photometric_blocks(c.W, c.H, c.N, 1);
    MD2_TRY(launch_pose_grad_reduce(fa, d_Rt, st));
  }
  return MD2_OK;
}

}  // namespace md2
