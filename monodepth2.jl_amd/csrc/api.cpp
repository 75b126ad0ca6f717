// C ABI of libmd2hip.so (include/md2.h).
#include "../../include/md2.h"

#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>

#include "conv.h"
#include "loss_tail.h"
#include "mine.h"
#include "model.h"
#include "nn.h"

#include <algorithm>

#include <dlfcn.h>
#include <execinfo.h>
#include <csignal>
#include <unistd.h>

namespace md2 {
// MD2_SEGV_TRACE=1: on SIGSEGV / SIGABRT print the native backtrace (and this library's load base,
// so `addr2line -e libmd2hip.so <pc - base>` maps the frames) before the default action -- host
// debugging on a box where no debugger may attach to a GPU process.
// The handler is installed with sigaction and chains to whatever handler was there before
// (pytest's faulthandler prints the Python traceback); backtrace() is called once at install time
// so libgcc's unwinder is already loaded when a crash happens (its first call may allocate).
static struct sigaction g_prev_segv, g_prev_abrt;
static void segv_trace(int sig, siginfo_t* info, void* uctx) {
  void* frames[64];
  const int n = backtrace(frames, 64);
  Dl_info di{};
  if (dladdr((void*)&segv_trace, &di) && di.dli_fbase) {
    char buf[96];
    const int k = snprintf(buf, sizeof buf, "libmd2hip base %p\n", di.dli_fbase);
    if (k > 0) (void)!write(2, buf, (size_t)k);
  }
  backtrace_symbols_fd(frames, n, 2);
  const struct sigaction& prev = sig == SIGSEGV ? g_prev_segv : g_prev_abrt;
  if ((prev.sa_flags & SA_SIGINFO) && prev.sa_sigaction) {
    prev.sa_sigaction(sig, info, uctx);
    return;
  }
  if (prev.sa_handler != SIG_DFL && prev.sa_handler != SIG_IGN && prev.sa_handler) {
    prev.sa_handler(sig);
    return;
  }
  struct sigaction dfl {};
  dfl.sa_handler = SIG_DFL;
  sigemptyset(&dfl.sa_mask);
  sigaction(sig, &dfl, nullptr);
  raise(sig);
}
__attribute__((constructor)) static void install_segv_trace() {
  const char* e = std::getenv("MD2_SEGV_TRACE");
  if (e && std::atoi(e) == 1) {
    void* warm[4];
    (void)backtrace(warm, 4);
    struct sigaction sa {};
    sa.sa_sigaction = segv_trace;
    sa.sa_flags = SA_SIGINFO;
    sigemptyset(&sa.sa_mask);
    sigaction(SIGSEGV, &sa, &g_prev_segv);
    sigaction(SIGABRT, &sa, &g_prev_abrt);
  }
}

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

namespace md2 {
int tuning_knob(const char* name, int dflt) {
  static const bool on = [] {
    const char* t = std::getenv("MD2_TUNING");
    return t && std::atoi(t) == 1;
  }();
  if (!on) return dflt;
  const char* e = std::getenv(name);
  return e ? std::atoi(e) : dflt;
}
}  // namespace md2

extern "C" {

int md2_abi_version(void) { return MD2_ABI_VERSION; }
const char* md2_build_id(void) { return MD2_BUILD_ID; }

const char* md2_last_error(void) { return md2::last_error(); }

int md2_device_count(int* count) {
  MD2_CHECK_ARG(count != nullptr, "count");
  MD2_HIP(hipGetDeviceCount(count));
  return MD2_OK;
}

int md2_memcpy_d2d(void* dst, const void* src, size_t bytes, void* stream) {
  MD2_CHECK_ARG(dst && src, "memcpy pointers");
  MD2_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream));
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
  o.vis_warped = out->vis_warped;
  o.vis_cell = out->vis_cell;
  return loss_tail_run(to_tail_cfg(cfg), disp, pose, x, automask, dloss, o, workspace,
                       (hipStream_t)stream);
}

static WarpOpCfg to_warp_cfg(const md2_warp_cfg* c) {
  WarpOpCfg w{};
  w.N = c->n;
  w.C = c->c;
  w.W = c->width;
  w.H = c->height;
  w.dw = c->dw;
  w.dh = c->dh;
  std::memcpy(w.K, c->K, sizeof(w.K));
  std::memcpy(w.invK, c->invK, sizeof(w.invK));
  w.min_depth = c->min_depth;
  w.max_depth = c->max_depth;
  w.x_sample_stride = (long)c->x_sample_stride;
  w.x_frame_stride = (long)c->x_frame_stride;
  w.target = c->target;
  w.src0 = c->src0;
  w.src1 = c->src1;
  return w;
}

size_t md2_warp_photometric_workspace_size(const md2_warp_cfg* cfg) {
  return cfg ? warp_op_workspace_bytes(cfg->n, cfg->width, cfg->height) : 0;
}

int md2_warp_photometric_fwd(const md2_warp_cfg* cfg, const float* disp, const float* Rt,
                             const float* x, const float* automask, float* loss_map,
                             signed char* sel_map, void* workspace, void* stream) {
  MD2_CHECK_ARG(cfg && loss_map, "warp_photometric_fwd: cfg/loss_map");
  return warp_op_run(to_warp_cfg(cfg), disp, Rt, x, automask, nullptr, loss_map, sel_map, nullptr,
                     nullptr, workspace, (hipStream_t)stream);
}

int md2_warp_photometric_bwd(const md2_warp_cfg* cfg, const float* disp, const float* Rt,
                             const float* x, const float* automask, const float* d_loss,
                             float* d_disp, float* d_Rt, void* workspace, void* stream) {
  MD2_CHECK_ARG(cfg && d_loss, "warp_photometric_bwd: cfg/d_loss");
  return warp_op_run(to_warp_cfg(cfg), disp, Rt, x, automask, d_loss, nullptr, nullptr, d_disp,
                     d_Rt, workspace, (hipStream_t)stream);
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

static ConvShape to_shape(const md2_conv_desc* d) {
  ConvShape s{};
  s.N = d->n;
  s.Cin = d->cin;
  s.H = d->h;
  s.W = d->w;
  s.Cout = d->cout;
  s.KH = d->kh;
  s.KW = d->kw;
  s.stride = d->stride;
  s.pad = d->pad;
  s.reflect = d->reflect;
  s.Ho = (d->h + 2 * d->pad - d->kh) / d->stride + 1;
  s.Wo = (d->w + 2 * d->pad - d->kw) / d->stride + 1;
  return s;
}

static size_t align_up(size_t b) { return (b + 255) & ~size_t(255); }

size_t md2_conv2d_workspace_size(const md2_conv_desc* d) {
  if (!d) return 0;
  const ConvShape s = to_shape(d);
  size_t packed = std::max(conv_fwd_packed_elems(s), conv_dgrad_packed_elems(s)) * sizeof(float);
  size_t slab = std::max(conv_fwd_workspace(s), std::max(conv_dgrad_workspace(s), conv_wgrad_workspace(s)));
  return align_up(packed) + align_up(slab);
}

int md2_conv2d_fwd(const md2_conv_desc* d, const float* x, const float* w, const float* bias,
                   float* y, void* workspace, void* stream) {
  MD2_CHECK_ARG(d && x && w && y && workspace, "conv2d_fwd args");
  const ConvShape s = to_shape(d);
  hipStream_t st = (hipStream_t)stream;
  float* packed = (float*)workspace;
  const size_t pbytes = align_up(std::max(conv_fwd_packed_elems(s), conv_dgrad_packed_elems(s)) * sizeof(float));
  MD2_TRY(conv_pack_fwd(s, w, packed, st));
  TensorIn in;
  in.p0 = x;
  in.c0 = s.Cin;
  in.bs0 = (long)s.Cin * s.H * s.W;
  TensorOut out;
  out.p0 = y;
  out.bs0 = (long)s.Cout * s.Ho * s.Wo;
  out.bias = bias;
  out.act = d->act;
  ConvWorkspace ws{(char*)workspace + pbytes, md2_conv2d_workspace_size(d) - pbytes};
  return conv_fwd(s, in, packed, out, ws, st);
}

int md2_conv2d_dgrad(const md2_conv_desc* d, const float* dy, const float* w, float* dx,
                     void* workspace, void* stream) {
  MD2_CHECK_ARG(d && dy && w && dx && workspace, "conv2d_dgrad args");
  const ConvShape s = to_shape(d);
  hipStream_t st = (hipStream_t)stream;
  float* packed = (float*)workspace;
  const size_t pbytes = align_up(std::max(conv_fwd_packed_elems(s), conv_dgrad_packed_elems(s)) * sizeof(float));
  MD2_TRY(conv_pack_dgrad(s, w, packed, st));
  TensorOut out;
  out.p0 = dx;
  out.bs0 = (long)s.Cin * s.H * s.W;
  ConvWorkspace ws{(char*)workspace + pbytes, md2_conv2d_workspace_size(d) - pbytes};
  return conv_dgrad(s, dy, packed, out, ws, st);
}

int md2_conv2d_wgrad(const md2_conv_desc* d, const float* x, const float* dy, float* dw,
                     float* db, void* workspace, void* stream) {
  MD2_CHECK_ARG(d && x && dy && dw && workspace, "conv2d_wgrad args");
  const ConvShape s = to_shape(d);
  const size_t pbytes = align_up(std::max(conv_fwd_packed_elems(s), conv_dgrad_packed_elems(s)) * sizeof(float));
  TensorIn in;
  in.p0 = x;
  in.c0 = s.Cin;
  in.bs0 = (long)s.Cin * s.H * s.W;
  ConvWorkspace ws{(char*)workspace + pbytes, md2_conv2d_workspace_size(d) - pbytes};
  return conv_wgrad(s, in, dy, dw, db, 0, ws, (hipStream_t)stream);
}

int md2_act_backward(const float* out, const float* dout, float* dpre, long long n, int act,
                     void* stream) {
  MD2_CHECK_ARG(out && dout && dpre && n >= 0, "act_backward args");
  return act_backward(out, dout, dpre, (long)n, act, (hipStream_t)stream);
}

// ---- optimiser ---------------------------------------------------------------------------------
int md2_adam(float* p, const float* g, float* adam_m, float* adam_v, long long n, float lr,
             float beta1, float beta2, float eps, int step, float grad_scale, void* stream) {
  MD2_CHECK_ARG(p && g && adam_m && adam_v && n > 0 && step >= 1, "adam args");
  const double bc1 = 1.0 - std::pow((double)beta1, step), bc2 = 1.0 - std::pow((double)beta2, step);
  return adam_step(p, g, adam_m, adam_v, (long)n, lr, beta1, beta2, eps, (float)bc1, (float)bc2,
                   grad_scale, (hipStream_t)stream);
}

// ---- pooling / resampling --------------------------------------------------------------------
int md2_maxpool3s2_fwd(const float* x, int n, int c, int h, int w, float* y, unsigned char* arg,
                       void* stream) {
  MD2_CHECK_ARG(x && y && arg && n > 0 && c > 0 && h > 0 && w > 0, "maxpool3s2_fwd args");
  return maxpool_fwd(x, n, c, h, w, y, arg, (h + 1) / 2, (w + 1) / 2, (hipStream_t)stream);
}
int md2_maxpool3s2_bwd(const float* dy, const unsigned char* arg, int n, int c, int h, int w,
                       float* dx, void* stream) {
  MD2_CHECK_ARG(dy && arg && dx && n > 0 && c > 0 && h > 0 && w > 0, "maxpool3s2_bwd args");
  return maxpool_bwd(dy, arg, n, c, h, w, (h + 1) / 2, (w + 1) / 2, dx, (hipStream_t)stream);
}
int md2_upsample2_fwd(const float* x, int n, int c, int h, int w, float* y, void* stream) {
  MD2_CHECK_ARG(x && y && n > 0 && c > 0 && h > 0 && w > 0, "upsample2_fwd args");
  return upsample2_fwd(x, n, c, h, w, y, (hipStream_t)stream);
}
int md2_mpi_embed_features(const float* feat, long long sample_stride, int n, int c, int h, int w,
                           const float* bins, int num_bins, int L, float* out, void* stream) {
  MD2_CHECK_ARG(feat && bins && out && n > 0 && c > 0 && h > 0 && w > 0 && num_bins > 0 && L >= 0 &&
                    sample_stride >= (long long)c * h * w, "mpi_embed_features args");
  return mpi_embed_features(feat, (long)sample_stride, n, c, h, w, bins, num_bins, L, out,
                            (hipStream_t)stream);
}
int md2_concat_channels(const float* a, int ca, const float* b, int cb, int n, long long hw,
                        float* out, void* stream) {
  MD2_CHECK_ARG(a && b && out && ca > 0 && cb > 0 && n > 0 && hw > 0, "concat_channels args");
  return concat_channels(a, ca, b, cb, n, (long)hw, out, (hipStream_t)stream);
}
// ---- MINE rendering (src/render.jl:21-114) -------------------------------------------------
static md2::Mat3 mat3(const float* m) {
  md2::Mat3 r;
  std::memcpy(r.m, m, sizeof(r.m));
  return r;
}
int md2_mine_src_xyz(const float* disparity, int n_planes, int batch, int h, int w,
                     const float* invK, float* xyz, void* stream) {
  MD2_CHECK_ARG(disparity && invK && xyz && n_planes > 0 && batch > 0 && h > 0 && w > 0,
                "mine_src_xyz args");
  return mine_src_xyz(disparity, n_planes, batch, h, w, mat3(invK), xyz, (hipStream_t)stream);
}
int md2_mine_tgt_xyz(const float* xyz_src, const float* pose, int n_planes, int batch, int h, int w,
                     float* xyz_tgt, void* stream) {
  MD2_CHECK_ARG(xyz_src && pose && xyz_tgt && n_planes > 0 && batch > 0 && h > 0 && w > 0,
                "mine_tgt_xyz args");
  return mine_tgt_xyz(xyz_src, pose, n_planes, batch, h, w, xyz_tgt, (hipStream_t)stream);
}
int md2_mine_sample(const float* src, int c, const float* depth, const float* pose, int n_planes,
                    int batch, int h, int w, const float* K, const float* invK, float* out,
                    float* valid, void* stream) {
  MD2_CHECK_ARG(src && depth && pose && K && invK && out && valid && c > 0 && n_planes > 0 &&
                    batch > 0 && h >= 2 && w >= 2, "mine_sample args (h, w >= 2)");
  return mine_sample(src, c, depth, pose, n_planes, batch, h, w, mat3(K), mat3(invK), out, valid,
                     (hipStream_t)stream);
}
int md2_plane_volume_rendering(const float* rgb, const float* sigma, const float* xyz, int n_planes,
                               int batch, int h, int w, float* rgb_out, float* transparency_acc,
                               float* weights, void* stream) {
  MD2_CHECK_ARG(rgb && sigma && xyz && rgb_out && transparency_acc && weights && n_planes > 0 &&
                    batch > 0 && h > 0 && w > 0, "plane_volume_rendering args");
  return plane_volume_rendering(rgb, sigma, xyz, n_planes, batch, h, w, rgb_out, transparency_acc,
                                weights, (hipStream_t)stream);
}
int md2_render_tgt_rgb_depth(const float* rgb, const float* sigma, const float* disparity,
                             const float* xyz_tgt, const float* pose, const float* invK,
                             const float* K, int n_planes, int batch, int h, int w, float* rgb_out,
                             float* depth, float* mask, void* stream) {
  MD2_CHECK_ARG(rgb && sigma && disparity && xyz_tgt && pose && invK && K && rgb_out && depth &&
                    mask && n_planes > 0 && batch > 0 && h >= 2 && w >= 2,
                "render_tgt_rgb_depth args (h, w >= 2)");
  return render_tgt_rgb_depth(rgb, sigma, disparity, xyz_tgt, pose, mat3(invK), mat3(K), n_planes,
                              batch, h, w, rgb_out, depth, mask, (hipStream_t)stream);
}
int md2_upsample2_bwd(const float* dy, int n, int c, int h, int w, float* dx, void* stream) {
  MD2_CHECK_ARG(dy && dx && n > 0 && c > 0 && h > 0 && w > 0, "upsample2_bwd args");
  return upsample2_bwd(dy, n, c, h, w, dx, (hipStream_t)stream);
}

// ---- model -----------------------------------------------------------------------------------
static ArchCfg to_arch(const md2_model_cfg* c) {
  ArchCfg a;
  a.arch = c->arch;
  a.in_ch = c->in_channels;
  a.nlevels = c->n_levels;
  for (int i = 0; i < MAX_SCALES; ++i) a.levels[i] = c->scale_levels[i];
  a.emb = c->embedding_levels;
  return a;
}

int md2_arch_param_count(const md2_model_cfg* cfg, long long* n_entries, long long* n_elems) {
  MD2_CHECK_ARG(cfg != nullptr, "cfg");
  MD2_CHECK_ARG(cfg->embedding_levels >= 0, "embedding_levels >= 0");
  MD2_CHECK_ARG(cfg->arch == 18 || cfg->arch == 34 || cfg->arch == 50, "arch 18/34/50");
  MD2_TRY(check_scale_levels(to_arch(cfg)));
  const auto t = build_param_table(to_arch(cfg));
  if (n_entries) *n_entries = (long long)t.size();
  if (n_elems) *n_elems = t.empty() ? 0 : (long long)(t.back().offset + t.back().numel);
  return MD2_OK;
}

int md2_arch_param_info(const md2_model_cfg* cfg, int idx, char* name, int name_len, int* ndim,
                        int* shape4, long long* offset) {
  MD2_CHECK_ARG(cfg != nullptr, "cfg");
  MD2_TRY(check_scale_levels(to_arch(cfg)));
  const auto t = build_param_table(to_arch(cfg));
  MD2_CHECK_ARG(idx >= 0 && idx < (int)t.size(), "param index");
  const ParamEntry& e = t[idx];
  if (name && name_len > 0) {
    std::strncpy(name, e.name.c_str(), name_len - 1);
    name[name_len - 1] = 0;
  }
  if (ndim) *ndim = e.ndim;
  if (shape4)
    for (int i = 0; i < 4; ++i) shape4[i] = e.shape[i];
  if (offset) *offset = e.offset;
  return MD2_OK;
}

int md2_model_create(const md2_model_cfg* c, float* params, float* grads, md2_model** out) {
  MD2_CHECK_ARG(c && params && grads && out, "model_create args");
  ModelCfg mc;
  mc.arch = to_arch(c);
  mc.N = c->batch;
  mc.W = c->width;
  mc.H = c->height;
  std::memcpy(mc.K, c->K, sizeof(mc.K));
  std::memcpy(mc.invK, c->invK, sizeof(mc.invK));
  mc.min_depth = c->min_depth;
  mc.max_depth = c->max_depth;
  mc.smoothness = c->disparity_smoothness;
  for (int i = 0; i < MAX_SCALES; ++i) mc.scales[i] = c->scales[i];
  mc.automask = c->automasking;
  mc.target = c->target;
  mc.src0 = c->src0;
  mc.src1 = c->src1;
  mc.num_bins = c->num_bins;
  Model* m = nullptr;
  MD2_TRY(model_create(mc, params, grads, &m));
  *out = new md2_model{m};
  return MD2_OK;
}

int md2_model_destroy(md2_model* m) {
  if (m) {
    model_destroy(m->impl);
    delete m;
  }
  return MD2_OK;
}

size_t md2_model_device_bytes(md2_model* m) { return m ? model_device_bytes(m->impl) : 0; }

int md2_model_repack(md2_model* m, void* stream) {
  MD2_CHECK_ARG(m, "model");
  return model_repack(m->impl, (hipStream_t)stream);
}

int md2_model_forward_loss(md2_model* m, const float* x, const float* auto_loss, float* loss,
                           float* terms, void* stream) {
  MD2_CHECK_ARG(m, "model");
  return model_forward_loss(m->impl, x, auto_loss, loss, terms, (hipStream_t)stream);
}

int md2_model_forward(md2_model* m, const float* x, const float** disp, const float** pose,
                      void* stream) {
  MD2_CHECK_ARG(m, "model");
  MD2_TRY(model_forward(m->impl, x, (hipStream_t)stream));
  return model_outputs(m->impl, disp, nullptr, nullptr, pose);
}

int md2_model_set_cotangents(md2_model* m, const float* const* d_disp, const float* d_pose,
                             void* stream) {
  MD2_CHECK_ARG(m, "model");
  return model_set_cotangents(m->impl, d_disp, d_pose, (hipStream_t)stream);
}

int md2_model_backward_from(md2_model* m, const float* const* d_disp, const float* d_pose,
                            void* stream) {
  MD2_CHECK_ARG(m, "model");
  MD2_TRY(model_set_cotangents(m->impl, d_disp, d_pose, (hipStream_t)stream));
  for (int k = 0; k < model_num_segments(m->impl); ++k)
    MD2_TRY(model_backward_segment(m->impl, k, nullptr, nullptr, (hipStream_t)stream));
  return MD2_OK;
}

int md2_model_num_segments(md2_model* m) { return m ? model_num_segments(m->impl) : 0; }

int md2_model_backward_segment(md2_model* m, int k, long long* off, long long* len,
                               void* stream) {
  MD2_CHECK_ARG(m, "model");
  long o = 0, l = 0;
  MD2_TRY(model_backward_segment(m->impl, k, &o, &l, (hipStream_t)stream));
  if (off) *off = o;
  if (len) *len = l;
  return MD2_OK;
}

int md2_model_adam(md2_model* m, float* adam_m, float* adam_v, float lr, float beta1,
                   float beta2, float eps, int step, float grad_scale, void* stream) {
  MD2_CHECK_ARG(m, "model");
  return model_adam(m->impl, adam_m, adam_v, lr, beta1, beta2, eps, step, grad_scale,
                    (hipStream_t)stream);
}

int md2_model_adam_segment(md2_model* m, int segment, float* adam_m, float* adam_v, float lr,
                           float beta1, float beta2, float eps, int step, float grad_scale, void* stream) {
  MD2_CHECK_ARG(m, "model");
  return model_adam_segment(m->impl, segment, adam_m, adam_v, lr, beta1, beta2, eps, step, grad_scale,
                            (hipStream_t)stream);
}

int md2_model_adam_join(md2_model* m, void* stream) {
  MD2_CHECK_ARG(m, "model");
  return model_adam_join(m->impl, (hipStream_t)stream);
}

int md2_model_train_step(md2_model* m, const float* x, const float* auto_loss, float* adam_m,
                         float* adam_v, float lr, int step, float* loss, void* stream) {
  MD2_CHECK_ARG(m && adam_m && adam_v && step >= 1, "train_step args");
  hipStream_t st = (hipStream_t)stream;
  MD2_TRY(model_forward_loss(m->impl, x, auto_loss, loss, nullptr, st));
  if (!model_segment_update_enabled()) {   // measured default: one update after the backward
    for (int k = 0; k < model_num_segments(m->impl); ++k)
      MD2_TRY(model_backward_segment(m->impl, k, nullptr, nullptr, st));
    return model_adam(m->impl, adam_m, adam_v, lr, 0.9f, 0.999f, 1e-8f, step, 1.f, st);
  }
  // each segment's update runs beside the remaining backward (model_adam_segment)
  for (int k = 0; k < model_num_segments(m->impl); ++k) {
    MD2_TRY(model_backward_segment(m->impl, k, nullptr, nullptr, st));
    MD2_TRY(model_adam_segment(m->impl, k, adam_m, adam_v, lr, 0.9f, 0.999f, 1e-8f, step, 1.f, st));
  }
  return model_adam_join(m->impl, st);
}

int md2_model_train_step_graph(md2_model* m, const float* x, const float* auto_loss, float* adam_m,
                               float* adam_v, float lr, int step, float* loss, void* stream) {
  MD2_CHECK_ARG(m, "model");
  return model_train_step_graph(m->impl, x, auto_loss, adam_m, adam_v, lr, step, loss,
                                (hipStream_t)stream);
}

int md2_model_set_params(md2_model* m, const float* flux, void* stream) {
  MD2_CHECK_ARG(m, "model");
  return model_set_params_flux(m->impl, flux, (hipStream_t)stream);
}
int md2_model_get_params(md2_model* m, float* flux, void* stream) {
  MD2_CHECK_ARG(m, "model");
  return model_get_params_flux(m->impl, flux, (hipStream_t)stream);
}
int md2_model_get_grads(md2_model* m, float* flux, void* stream) {
  MD2_CHECK_ARG(m, "model");
  return model_get_grads_flux(m->impl, flux, (hipStream_t)stream);
}
int md2_model_loss_cotangent(md2_model* m, float dloss, void* stream) {
  MD2_CHECK_ARG(m, "model");
  return model_scale_loss_cotangent(m->impl, dloss, (hipStream_t)stream);
}

int md2_model_set_profiling(md2_model* m, int on) {
  MD2_CHECK_ARG(m, "model");
  return model_set_profiling(m->impl, on);
}

int md2_model_profile_read(md2_model* m, double* out, int ncat) {
  MD2_CHECK_ARG(m, "model");
  return model_profile_read(m->impl, out, ncat);
}

int md2_model_profile_records(md2_model* m, int max, double* ms, double* work, int* cat, char* tags,
                              int tag_len, int* count) {
  MD2_CHECK_ARG(m, "model");
  return model_profile_records(m->impl, max, ms, work, cat, tags, tag_len, count);
}

int md2_model_set_disparity_bins(md2_model* m, const float* bins, void* stream) {
  MD2_CHECK_ARG(m, "model");
  return model_set_bins(m->impl, bins, (hipStream_t)stream);
}

int md2_model_outputs(md2_model* m, const float** disp, int* w, int* h, const float** pose) {
  MD2_CHECK_ARG(m, "model");
  return model_outputs(m->impl, disp, w, h, pose);
}

int md2_model_features(md2_model* m, const float** feat, int* c, int* h, int* w) {
  MD2_CHECK_ARG(m && feat && c && h && w, "model_features args");
  return model_features(m->impl, feat, c, h, w);
}

int md2_model_debug_tensor(md2_model* m, int index, const char** name, const void** ptr,
                           int* dims) {
  MD2_CHECK_ARG(m, "model");
  return model_debug_tensor(m->impl, index, name, ptr, dims);
}

int md2_model_eval_disparity(md2_model* m, const float* x, int n, const float** disp,
                             void* stream) {
  MD2_CHECK_ARG(m, "model");
  float* d[MAX_SCALES] = {};
  MD2_TRY(model_eval_disparity(m->impl, x, n, d, (hipStream_t)stream));
  if (disp)
    for (int i = 0; i < MAX_SCALES; ++i) disp[i] = d[i];
  return MD2_OK;
}

}  // extern "C"
