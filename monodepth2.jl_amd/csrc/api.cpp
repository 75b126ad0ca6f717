// C ABI of libmd2hip.so (include/md2.h).
#include "../../include/md2.h"

#include <cstring>
#include <string>

#include "loss_tail.h"

namespace md2 {
static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }
const char* last_error() { return g_last_error.c_str(); }

static LossTailCfg to_tail_cfg(const md2_loss_cfg* c) {
  LossTailCfg t{};
  t.N = c->n;
  t.C = c->c;
  t.W = c->width;
  t.H = c->height;
  t.nscales = c->nscales;
  for (int s = 0; s < MAX_SCALES; ++s) {
    t.dw[s] = c->scale_w[s];
    t.dh[s] = c->scale_h[s];
    t.smooth_w[s] = c->smooth_weight[s];
  }
  t.divisor = c->divisor;
  t.smooth_normalize = c->smooth_normalize;
  std::memcpy(t.K, c->K, sizeof(t.K));
  std::memcpy(t.invK, c->invK, sizeof(t.invK));
  t.min_depth = c->min_depth;
  t.max_depth = c->max_depth;
  t.x_sample_stride = (long)c->x_sample_stride;
  t.x_frame_stride = (long)c->x_frame_stride;
  t.target = c->target;
  t.src0 = c->src0;
  t.src1 = c->src1;
  t.invert_mask = c->invert_mask;
  t.sigmoid_grad = c->sigmoid_grad;
  return t;
}
}  // namespace md2

using namespace md2;

extern "C" {

int md2_abi_version(void) { return MD2_ABI_VERSION; }

const char* md2_last_error(void) { return md2::last_error(); }

int md2_device_count(int* count) {
  MD2_CHECK_ARG(count != nullptr, "count");
  MD2_HIP(hipGetDeviceCount(count));
  return MD2_OK;
}

size_t md2_loss_workspace_size(const md2_loss_cfg* cfg) {
  if (!cfg) return 0;
  return loss_tail_workspace_bytes(to_tail_cfg(cfg));
}

int md2_loss_fwd_bwd(const md2_loss_cfg* cfg, const float* const* disp, const float* pose,
                     const float* x, const float* automask, float dloss,
                     const md2_loss_out* out, void* workspace, void* stream) {
  MD2_CHECK_ARG(cfg != nullptr && out != nullptr && out->loss != nullptr, "cfg/out/loss");
  LossTailOut o{};
  o.loss = out->loss;
  o.terms = out->terms;
  for (int s = 0; s < MAX_SCALES; ++s) o.d_disp[s] = out->d_disp[s];
  o.d_pose = out->d_pose;
  o.vis_loss = out->vis_loss;
  o.vis_sel = out->vis_sel;
  return loss_tail_run(to_tail_cfg(cfg), disp, pose, x, automask, dloss, o, workspace,
                       (hipStream_t)stream);
}

int md2_so3_compose_fwd(const float* pose, int n, int invert_mask, float* Rt, void* stream) {
  MD2_CHECK_ARG(pose && Rt && n > 0, "so3 fwd args");
  return launch_so3_fwd(pose, 2 * n, n, invert_mask, Rt, (hipStream_t)stream);
}

int md2_so3_compose_bwd(const float* pose, int n, int invert_mask, const float* dRt,
                        float* d_pose, void* stream) {
  MD2_CHECK_ARG(pose && dRt && d_pose && n > 0, "so3 bwd args");
  return launch_so3_bwd(pose, 2 * n, n, invert_mask, dRt, d_pose, 0, (hipStream_t)stream);
}

}  // extern "C"
