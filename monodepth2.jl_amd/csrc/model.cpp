// Model executor (see model.h).
//
// Data layout in HBM (all fp32, NCHW == Julia (W,H,C,N)):
//   * encoder batch is FRAME-MAJOR: image b = l*N + n holds frame l of sample n (the stem reads
//     x[n][l] through a batch map), so the target frames form the contiguous slice [N, 2N) that
//     the DepthDecoder reads as skips, and pose pairs (frame s, frame s+1) are (b, b+N).  BatchNorm
//     statistics run over all 3N frames exactly like ResNet.jl on reshape(x, (W,H,C,L*N)).
//   * parameters / gradients are caller-owned flat fp32 vectors in the order of
//     oracle/md2_oracle.py param_spec; conv weights are re-packed K-major after each update.
#include "model.h"
#include "head.h"

#include <algorithm>
#include <cmath>
#include <cstring>

namespace md2 {

namespace {

struct PConv {
  int cin = 0, cout = 0, k = 1, stride = 1, pad = 0, reflect = 0;
  bool bias = false;
  long w = -1, b = -1;
};
struct PBN {
  int c = 0;
  long g = -1, b = -1;
};
struct BlockSpec {
  std::vector<PConv> convs;
  std::vector<PBN> bns;
  bool down = false;
  PConv dconv;
  PBN dbn;
  int cin = 0, cout = 0, stride = 1;
};
struct BranchSpec {
  int bid = 0;
  PConv c1, c2;
  int cin = 0, cout = 0, cskip = 0;
  int head = -1;          // index into heads when a DecoderBlock head follows this branch
};
struct ArchSpec {
  std::vector<ParamEntry> table;
  long total = 0;
  PConv stem;
  PBN stem_bn;
  std::vector<std::vector<BlockSpec>> stages;
  int enc_ch[5];
  std::vector<BranchSpec> branches;
  std::vector<PConv> heads;
  std::vector<int> head_level;
  PConv squeezer, p1, p2, p3;
  long stage_begin[5];    // flat offsets: [0] stem, [1..4] layer1..4
  long depth_begin = 0;
};

ArchSpec build_spec(const ArchCfg& a) {
  ArchSpec S;
  auto add = [&](const std::string& name, std::initializer_list<int> shape) -> long {
    ParamEntry e;
    e.name = name;
    e.ndim = (int)shape.size();
    long n = 1;
    int i = 0;
    for (int s : shape) {
      e.shape[i++] = s;
      n *= s;
    }
    for (; i < 4; ++i) e.shape[i] = 1;
    e.offset = S.total;
    e.numel = n;
    S.total += n;
    S.table.push_back(e);
    return e.offset;
  };
  auto conv = [&](const std::string& name, int cin, int cout, int k, int stride, int pad,
                  int reflect, bool bias) {
    PConv c;
    c.cin = cin; c.cout = cout; c.k = k; c.stride = stride; c.pad = pad; c.reflect = reflect;
    c.bias = bias;
    c.w = add(name + ".weight", {cout, cin, k, k});
    if (bias) c.b = add(name + ".bias", {cout});
    return c;
  };
  auto bn = [&](const std::string& name, int c) {
    PBN b;
    b.c = c;
    b.g = add(name + ".gamma", {c});
    b.b = add(name + ".beta", {c});
    return b;
  };
  const bool bottleneck = a.arch >= 50;
  const int* layers;
  static const int L18[4] = {2, 2, 2, 2}, L34[4] = {3, 4, 6, 3};
  layers = (a.arch == 18) ? L18 : L34;
  const int exp = bottleneck ? 4 : 1;
  S.stage_begin[0] = 0;
  S.stem = conv("encoder.stem.conv", a.in_ch, 64, 7, 2, 3, 0, false);
  S.stem_bn = bn("encoder.stem.bn", 64);
  int cin = 64;
  const int widths[4] = {64, 128, 256, 512};
  S.stages.resize(4);
  for (int si = 0; si < 4; ++si) {
    S.stage_begin[si + 1] = S.total;
    for (int bi = 0; bi < layers[si]; ++bi) {
      const int stride = (bi == 0 && si > 0) ? 2 : 1;
      const std::string p = "encoder.layer" + std::to_string(si + 1) + "." + std::to_string(bi);
      const int width = widths[si], cout = width * exp;
      BlockSpec B;
      B.cin = cin;
      B.cout = cout;
      B.stride = stride;
      if (bottleneck) {
        B.convs.push_back(conv(p + ".conv1", cin, width, 1, 1, 0, 0, false));
        B.bns.push_back(bn(p + ".bn1", width));
        B.convs.push_back(conv(p + ".conv2", width, width, 3, stride, 1, 0, false));
        B.bns.push_back(bn(p + ".bn2", width));
        B.convs.push_back(conv(p + ".conv3", width, cout, 1, 1, 0, 0, false));
        B.bns.push_back(bn(p + ".bn3", cout));
      } else {
        B.convs.push_back(conv(p + ".conv1", cin, width, 3, stride, 1, 0, false));
        B.bns.push_back(bn(p + ".bn1", width));
        B.convs.push_back(conv(p + ".conv2", width, width, 3, 1, 1, 0, false));
        B.bns.push_back(bn(p + ".bn2", width));
      }
      if (stride != 1 || cin != cout) {
        B.down = true;
        B.dconv = conv(p + ".down", cin, cout, 1, stride, 0, 0, false);
        B.dbn = bn(p + ".down_bn", cout);
      }
      S.stages[si].push_back(B);
      cin = cout;
    }
  }
  const int enc18[5] = {64, 64, 128, 256, 512}, enc50[5] = {64, 256, 512, 1024, 2048};
  for (int i = 0; i < 5; ++i) S.enc_ch[i] = bottleneck ? enc50[i] : enc18[i];
  // DepthDecoder(; encoder_channels, scale_levels, embedding_levels=0) src/depth_decoder.jl:26-50
  S.depth_begin = S.total;
  const int dec[5] = {256, 128, 64, 32, 16};
  int encr[5];   // + embedding_levels in MPI mode (src/depth_decoder.jl:32)
  for (int i = 0; i < 5; ++i) encr[i] = S.enc_ch[4 - i] + a.emb;
  const int in_ch[5] = {encr[0], dec[0], dec[1], dec[2], dec[3]};
  const int skip[5] = {encr[1], encr[2], encr[3], encr[4], 0};
  int bstart = 1;
  for (int li = 0; li < a.nlevels; ++li) {
    const int slevel = a.levels[li];
    for (int bid = bstart; bid <= slevel; ++bid) {
      const int b = bid - 1;
      BranchSpec br;
      br.bid = bid;
      br.cin = in_ch[b];
      br.cout = dec[b];
      br.cskip = skip[b];
      br.c1 = conv("depth.branch" + std::to_string(bid) + ".c1", in_ch[b], dec[b], 3, 1, 1, 1, true);
      br.c2 = conv("depth.branch" + std::to_string(bid) + ".c2", dec[b] + skip[b], dec[b], 3, 1, 1, 1, true);
      S.branches.push_back(br);
    }
    S.heads.push_back(conv("depth.head" + std::to_string(slevel), dec[slevel - 1], 1, 3, 1, 1, 1, true));
    S.head_level.push_back(slevel);
    S.branches.back().head = (int)S.heads.size() - 1;
    bstart = slevel + 1;
  }
  // PoseDecoder(encoder_out_channels) src/pose_decoder.jl:13-21
  S.squeezer = conv("pose.squeezer", S.enc_ch[4], 256, 1, 1, 0, 0, true);
  S.p1 = conv("pose.conv1", 512, 256, 3, 1, 1, 0, true);
  S.p2 = conv("pose.conv2", 256, 256, 3, 1, 1, 0, true);
  S.p3 = conv("pose.conv3", 256, 6, 1, 1, 0, 0, true);
  return S;
}

inline int out_dim(int in, int k, int s, int p) { return (in + 2 * p - k) / s + 1; }

}  // namespace

std::vector<ParamEntry> build_param_table(const ArchCfg& a) { return build_spec(a).table; }

// ---------------------------------------------------------------------------------------------
// runtime structures
// ---------------------------------------------------------------------------------------------
struct RConv {
  PConv p;
  ConvShape s{};          // N filled per call
  float* wpf = nullptr;   // packed forward weights
  float* wpd = nullptr;   // packed dgrad weights
  int cat = PROF_CONV_OTHER;
};
struct RBN {
  PBN p;
  float *mean = nullptr, *invstd = nullptr, *rmean = nullptr, *rvar = nullptr;
  const double* part = nullptr;   // statistics partials of the current forward (bn_fwd)
  int parts = 0;
};
struct EncStage {
  RConv conv;
  RBN bn;
  float* y = nullptr;     // conv output
  float* a = nullptr;     // post BN (+ReLU); block output for the last stage
};
struct EncBlock {
  std::vector<EncStage> st;
  bool down = false;
  RConv dconv;
  RBN dbn;
  float* yd = nullptr;
  float* in = nullptr;
  float* d_in = nullptr;
  float* d_out = nullptr;
  int C = 0, H = 0, W = 0;      // output
  int Cin = 0, Hin = 0, Win = 0;
};
struct DecBranch {
  BranchSpec b;
  RConv c1, c2;
  int h = 0, w = 0;             // c1 resolution (input); output 2h x 2w
  float *o1 = nullptr, *up = nullptr, *o2 = nullptr, *d_o2 = nullptr;
  int head = -1;
  RConv hc;
  float* disp = nullptr;
  float* d_head = nullptr;      // gradient w.r.t. the head pre-activation (from the loss tail)
};

class Model {
 public:
  ModelCfg cfg;
  ArchSpec spec;
  float* params = nullptr;
  float* grads = nullptr;
  std::vector<void*> allocs;
  size_t bytes = 0;

  int N = 0, B = 0;             // samples, encoder images (3N)
  int H0 = 0, W0 = 0;           // stem output
  int Hm = 0, Wm = 0;           // maxpool output
  RConv stem;
  RBN stem_bn;
  float *y0 = nullptr, *f0 = nullptr, *mp = nullptr, *d_mp = nullptr, *d_f0 = nullptr;
  unsigned char* mp_arg = nullptr;
  std::vector<std::vector<EncBlock>> stages;
  float* feat[5] = {};
  int featC[5] = {}, featH[5] = {}, featW[5] = {};
  std::vector<DecBranch> br;
  float* d_skip[4] = {};
  // MPI mode (src/model.jl:31-55): E embedding channels, NP planes per sample, ND = N*NP decoder
  // images (image n*NP + p).  emb_in[f] = cat(repeat(target features f, P), repeat(embed(bins),
  // h, w)) is the decoder's input / skip of level f; d_emb[f] its gradient, block-summed over the
  // planes into the target features' gradient (the _repeat pullback, src/repeat.jl:44-53).
  int E = 0, NP = 1, ND = 0;
  // MPI mode: the E embedding channels of every decoder input are stored padded to Ep = E rounded
  // up to 16 (zero channels with zero weights), so C + Ep stays a multiple of 16 and the decoder
  // convs run on the tap-major kernels (conv_tap_major); the weights keep the reference's E
  int Ep = 0;
  float* emb_in[5] = {};
  float* d_emb[5] = {};
  float* bins = nullptr;                        // [N][P]
  float *pose_rep = nullptr, *d_pose_rep = nullptr, *amask_rep = nullptr;
  // pose
  RConv sq, p1, p2, p3;
  float *sqo = nullptr, *pc1 = nullptr, *pc2 = nullptr, *means = nullptr, *pose = nullptr;
  float *d_pose = nullptr, *d_pc1 = nullptr, *d_pin = nullptr, *d_sq = nullptr;
  // pose pair j of sample q = frames (pa[j], pb[j]) (src/model.jl:57-70); the default (target 2,
  // sources 1, 3) pairs are images (q, q+N) and read sqo in place, other ids gather into pin
  int pa[2] = {0, 1}, pb[2] = {1, 2};
  bool pairs_inplace = true;
  float* pin = nullptr;
  int T0 = 0;                   // image offset of the target frame's slice (target * N)
  // scratch
  float *DA = nullptr, *DY = nullptr, *G = nullptr, *DYD = nullptr;
  float *DPRE = nullptr, *DUP = nullptr, *DO1 = nullptr;
  ConvWorkspace cws{};
  // Side stream for independent branches, each with its OWN scratch (split-K workspace,
  // bias-gradient partials, activation-pullback buffer, BN partials slot 1) so they can run
  // beside the model stream:
  //  * the PoseDecoder depends only on the encoder's layer-4 features (forward) and on d_pose
  //    from the loss tail (backward): it runs beside the DepthDecoder and joins before the loss
  //    tail (poses) and before the decoder's first-branch dgrad accumulates into the layer-4
  //    feature gradient the squeezer's dgrad wrote (MD2_POSE_STREAM);
  //  * a downsampling block's 1x1 conv + BN depends only on the block input: its forward runs
  //    beside the block's 3x3 chain and joins before the residual BN apply; its backward runs
  //    beside the chain's backward and joins before the first conv's dgrad accumulates into the
  //    block's input gradient the 1x1 dgrad wrote (MD2_DOWN_STREAM);
  //  * the DepthDecoder's filter gradients beside its data gradients (MD2_DEC_WGRAD_STREAM, below).
  // The arithmetic is unchanged (same kernels, same buffers' contents): the step is
  // bit-identical with any switch off (=0, tests/test_gpu_fusion.py) and under the HIP-event
  // probe, which runs everything on the model stream so that its brackets time kernels alone.
  ConvWorkspace cws_side{};
  float* bp_ws_side = nullptr;
  float* DPRE_side = nullptr;
  bool side_ws = false;       // conv / act_bias calls of a side branch: its own scratch
  hipStream_t side = nullptr;
  hipEvent_t fork_ev = nullptr, join_ev = nullptr;
  // Per-segment optimiser update (model_adam_segment): ADAM over a backward segment's parameter
  // range and the re-pack of that segment's conv weights, on a stream of their own as soon as the
  // segment's gradient is final -- beside the remaining backward instead of after it.  Safe: no
  // later backward segment reads an earlier segment's parameters or packed weights (the segments
  // are decoders, layer 4, ..., stem: each reads only its own), and the next forward waits for the
  // updates (model_adam_join).
  hipStream_t upd = nullptr;
  hipEvent_t seg_ev = nullptr, upd_ev = nullptr;
  bool upd_recorded = false;   // upd_ev holds the newest adam_segment's completion
  struct SegPack {
    PackJob* jobs = nullptr;
    int njobs = 0;
    long blocks = 0;
  } seg_pack[6];
  const bool pose_stream = [] {
    const char* v = getenv("MD2_POSE_STREAM");
    return !(v && v[0] == '0');
  }();
  ConvWorkspace& ws_conv() { return side_ws ? cws_side : cws; }
  float* ws_bp() { return side_ws ? bp_ws_side : bp_ws; }
  const bool down_stream = [] {
    const char* v = getenv("MD2_DOWN_STREAM");
    return !(v && v[0] == '0');
  }();
  const bool dec_wgrad_stream = [] {
    const char* v = getenv("MD2_DEC_WGRAD_STREAM");
    return !(v && v[0] == '0');
  }();
  // DepthDecoder backward: each conv's filter gradient on the side stream beside its data
  // gradient and the rest of the branch (the decoder convs fill a fraction of the chip).  The
  // side reads DPRE / DO1 and the bias partials of the act_bias before it, so those buffers are
  // reused only after the side's event (bias partials double-buffered: bp_dec[0] for c2, [1] for c1)
  hipEvent_t ev_a = nullptr, ev_b = nullptr, ev_c2 = nullptr, ev_c1 = nullptr;
  float* bp_dec[2] = {nullptr, nullptr};
  bool pose_overlap() const { return pose_stream && side && !prof; }
  bool wgrad_overlap() const { return dec_wgrad_stream && side && !prof; }
  bool down_overlap() const { return down_stream && side && !prof; }
  // Encoder backward of the last stages (stages >= enc_wgrad_from: layers 2-4 by default; the convs
  // are small and split-K): each block conv's filter gradient on the side stream beside its data
  // gradient (interleaved A/B, 3 x 60 steps: off 1481, from layer 4 1493, from layer 3 1490,
  // from layer 2 1478 images/s -- the larger layers' convs fill the chip and only time-share).  The
  // conv's dY alternates between DY and DY2 so the data gradient's BN backward can write the next
  // dY while the side still reads the current one; a dY buffer is written again only after the
  // side's event for its last read (ev_y[j]); every stage segment ends with the side joined.
  const bool enc_wgrad_stream = [] {
    const char* v = getenv("MD2_ENC_WGRAD_STREAM");
    return !(v && v[0] == '0');
  }();
  // (round 6, with the LDS-halo kernels: from layer 2 (si = 1) 6.194 vs 6.211 ms and 6.159 vs 6.19
  // against layer 4 only, interleaved; from layer 1 6.167)
  const int enc_wgrad_from = tuning_knob("MD2_ENC_WGRAD_FROM", 1);
  // (1: -45 us per step, 6.555 vs 6.60 ms interleaved; the side stream was the longer path of the
  // layer-4 segment)
  const bool enc_wgrad_main0 = tuning_knob("MD2_ENC_WGRAD_MAIN0", 1) != 0;
  bool enc_overlap(int si) const { return enc_wgrad_stream && side && !prof && si >= enc_wgrad_from; }
  float* DY2 = nullptr;
  hipEvent_t ev_y[2] = {nullptr, nullptr};
  bool y_pending[2] = {false, false};
  int ycur = 0;
  float* ybuf(int j) { return j ? DY2 : DY; }
  int y_claim(int j, hipStream_t st) {   // the model stream is about to write dY buffer j
    if (y_pending[j]) MD2_HIP(hipStreamWaitEvent(st, ev_y[j], 0));
    y_pending[j] = false;
    return MD2_OK;
  }
  // the downsample branch's conv + BN statistics (slot 1), on `st`
  int down_fwd(EncBlock& b, int nimg, hipStream_t st) {
    side_ws = true;
    const long ohw = (long)b.H * b.W;
    const int rc = conv_f_bn(b.dconv, nimg, tin(b.in, b.Cin, (long)b.Hin * b.Win), b.yd, (long)b.C * ohw,
                             b.dbn, ohw, st, 1);
    side_ws = false;
    return rc;
  }
  // ops of `st2` wait for everything enqueued on `st1` so far
  int stream_wait(hipStream_t st1, hipStream_t st2, hipEvent_t e) {
    MD2_HIP(hipEventRecord(e, st1));
    MD2_HIP(hipStreamWaitEvent(st2, e, 0));
    return MD2_OK;
  }
  BNStatsWs bnws{};
  long bn_slot = 0;                 // doubles per partials slot (slot 1: the downsample BN of a block)
  double* bn_collapsed = nullptr;   // [2 slots][4096 channels][2]: collapsed epilogue partials
  void* tail_ws = nullptr;
  LossTailCfg tail{};
  float* loss_buf = nullptr;
  float* amask = nullptr;       // automasking_loss of the current batch when the caller passes none
  const float* eval_disp[MAX_SCALES] = {};

  ~Model() {
    if (g.exec) (void)hipGraphExecDestroy(g.exec);
    if (side) (void)hipStreamDestroy(side);
    if (upd) (void)hipStreamDestroy(upd);
    if (seg_ev) (void)hipEventDestroy(seg_ev);
    if (upd_ev) (void)hipEventDestroy(upd_ev);
    if (fork_ev) (void)hipEventDestroy(fork_ev);
    for (hipEvent_t e : {ev_a, ev_b, ev_c2, ev_c1, ev_y[0], ev_y[1]})
      if (e) (void)hipEventDestroy(e);
    if (join_ev) (void)hipEventDestroy(join_ev);
    if (g.st) (void)hipStreamDestroy(g.st);
    for (void* p : allocs) (void)hipFree(p);
    for (hipEvent_t e : evpool) (void)hipEventDestroy(e);
  }

  // graph-captured single-GPU step (model_train_step_graph): the executor owns the input copy,
  // the loss slot and the device ADAM step counter, so one capture replays for every batch/step
  struct StepGraph {
    hipGraphExec_t exec = nullptr;
    hipStream_t st = nullptr;
    float *x = nullptr, *autoloss = nullptr, *loss = nullptr, *bc = nullptr;
    int* step = nullptr;
    float *adam_m = nullptr, *adam_v = nullptr;
    float lr = 0.f;
    int with_auto = -1;
    int next_step = -1;
  } g;

  int alloc(float** p, size_t n) {
    void* q = nullptr;
    MD2_HIP(hipMalloc(&q, std::max<size_t>(n, 1) * sizeof(float)));
    allocs.push_back(q);
    bytes += n * sizeof(float);
    *p = (float*)q;
    return MD2_OK;
  }
  float* P(long off) { return off >= 0 ? params + off : nullptr; }
  float* Gd(long off) { return off >= 0 ? grads + off : nullptr; }

  int make_conv(RConv& r, const PConv& p, int H, int W, bool dgrad, size_t& ws_need, int cin_pad = 0) {
    r.p = p;
    r.s.N = 0;
    r.s.Cin = cin_pad > 0 ? cin_pad : p.cin;   // cin_pad: zero input channels beyond the weights' p.cin
    r.s.cin_w = cin_pad > 0 ? p.cin : 0;
    r.s.Cout = p.cout;
    r.s.H = H;
    r.s.W = W;
    r.s.KH = r.s.KW = p.k;
    r.s.stride = p.stride;
    r.s.pad = p.pad;
    r.s.reflect = p.reflect;
    r.s.Ho = out_dim(H, p.k, p.stride, p.pad);
    r.s.Wo = out_dim(W, p.k, p.stride, p.pad);
    // packed weights: the repack writes only real elements, the padding stays zero from here
    MD2_TRY(alloc(&r.wpf, conv_fwd_packed_elems(r.s)));
    MD2_HIP(hipMemset(r.wpf, 0, conv_fwd_packed_elems(r.s) * sizeof(float)));
    if (dgrad) {
      MD2_TRY(alloc(&r.wpd, conv_dgrad_packed_elems(r.s)));
      MD2_HIP(hipMemset(r.wpd, 0, conv_dgrad_packed_elems(r.s) * sizeof(float)));
    }
    return MD2_OK;
  }
  void need_ws(const RConv& r, int nimg, size_t& ws_need, bool dgrad) {
    ConvShape s = r.s;
    s.N = nimg;
    ws_need = std::max(ws_need, conv_fwd_workspace(s));
    ws_need = std::max(ws_need, conv_wgrad_workspace(s));
    if (dgrad) ws_need = std::max(ws_need, conv_dgrad_workspace(s));
  }
  int make_bn(RBN& r, const PBN& p) {
    r.p = p;
    MD2_TRY(alloc(&r.mean, p.c));
    MD2_TRY(alloc(&r.invstd, p.c));
    MD2_TRY(alloc(&r.rmean, p.c));
    MD2_TRY(alloc(&r.rvar, p.c));
    MD2_HIP(hipMemset(r.rmean, 0, p.c * sizeof(float)));
    std::vector<float> ones(p.c, 1.f);
    MD2_HIP(hipMemcpy(r.rvar, ones.data(), p.c * sizeof(float), hipMemcpyHostToDevice));
    return MD2_OK;
  }

  int build() {
    const ArchCfg& A = cfg.arch;
    spec = build_spec(A);
    N = cfg.N;
    B = 3 * N;
    E = A.emb;
    NP = E > 0 ? cfg.num_bins : 1;
    Ep = E > 0 ? (E + 15) / 16 * 16 : 0;
    ND = N * NP;
    const int C = A.in_ch;
    size_t wsn = 0, wsn_side = 0, scratch = 0;   // wsn_side: side-stream convs (downsample, pose, decoder wgrad)
    long bnmax = 0;
    auto track = [&](long n) { scratch = std::max(scratch, (size_t)n); };
    auto bnws_need = [&](int Cc, long HW) {
      bnmax = std::max(bnmax, (long)Cc * bn_parts(Cc, B, HW) * 2);
      bnmax = std::max(bnmax, (long)Cc * ((B * HW + 255) / 256) * 2);   // per-tile epilogue partials
    };
    // ---- encoder
    MD2_TRY(make_conv(stem, spec.stem, cfg.H, cfg.W, false, wsn));
    need_ws(stem, B, wsn, false);
    MD2_TRY(make_bn(stem_bn, spec.stem_bn));
    H0 = stem.s.Ho;
    W0 = stem.s.Wo;
    Hm = out_dim(H0, 3, 2, 1);
    Wm = out_dim(W0, 3, 2, 1);
    const long n0 = (long)B * 64 * H0 * W0, nm = (long)B * 64 * Hm * Wm;
    MD2_TRY(alloc(&y0, n0));
    MD2_TRY(alloc(&f0, n0));
    MD2_TRY(alloc(&d_f0, n0));
    MD2_TRY(alloc(&mp, nm));
    MD2_TRY(alloc(&d_mp, nm));
    {
      void* q;
      MD2_HIP(hipMalloc(&q, nm));
      allocs.push_back(q);
      mp_arg = (unsigned char*)q;
    }
    track(n0);
    bnws_need(64, (long)H0 * W0);
    feat[0] = f0; featC[0] = 64; featH[0] = H0; featW[0] = W0;
    float* cur = mp;
    float* dcur = d_mp;
    int cC = 64, cH = Hm, cW = Wm;
    stages.resize(4);
    for (int si = 0; si < 4; ++si) {
      for (auto& bs : spec.stages[si]) {
        EncBlock eb;
        eb.in = cur;
        eb.d_in = dcur;
        eb.Cin = cC; eb.Hin = cH; eb.Win = cW;
        int h = cH, w = cW;
        for (size_t k = 0; k < bs.convs.size(); ++k) {
          EncStage es;
          MD2_TRY(make_conv(es.conv, bs.convs[k], h, w, true, wsn));
          es.conv.cat = bs.convs[k].k == 3 ? PROF_CONV3_ENC : PROF_CONV_OTHER;
          need_ws(es.conv, B, wsn, true);
          need_ws(es.conv, B, wsn_side, false);   // filter gradient on the side (enc_overlap)
          MD2_TRY(make_bn(es.bn, bs.bns[k]));
          h = es.conv.s.Ho;
          w = es.conv.s.Wo;
          const long n = (long)B * bs.convs[k].cout * h * w;
          MD2_TRY(alloc(&es.y, n));
          MD2_TRY(alloc(&es.a, n));
          track(n);
          bnws_need(bs.convs[k].cout, (long)h * w);
          eb.st.push_back(es);
        }
        if (bs.down) {
          eb.down = true;
          MD2_TRY(make_conv(eb.dconv, bs.dconv, cH, cW, true, wsn_side));
          need_ws(eb.dconv, B, wsn_side, true);
          MD2_TRY(make_bn(eb.dbn, bs.dbn));
          MD2_TRY(alloc(&eb.yd, (long)B * bs.cout * h * w));
        }
        eb.C = bs.cout; eb.H = h; eb.W = w;
        MD2_TRY(alloc(&eb.d_out, (long)B * bs.cout * h * w));
        cur = eb.st.back().a;
        dcur = eb.d_out;
        cC = bs.cout; cH = h; cW = w;
        stages[si].push_back(eb);
      }
      feat[si + 1] = cur;
      featC[si + 1] = cC; featH[si + 1] = cH; featW[si + 1] = cW;
    }
    // ---- depth decoder (ND = N target images, times P planes in MPI mode)
    if (E > 0) {
      MD2_TRY(alloc(&bins, (long)N * NP));
      MD2_HIP(hipMemset(bins, 0, sizeof(float) * N * NP));
      MD2_TRY(alloc(&emb_in[4], (long)ND * (featC[4] + Ep) * featH[4] * featW[4]));
      MD2_TRY(alloc(&d_emb[4], (long)ND * (featC[4] + Ep) * featH[4] * featW[4]));
    }
    int h = featH[4], w = featW[4];
    for (auto& bs : spec.branches) {
      DecBranch d;
      d.b = bs;
      d.h = h;
      d.w = w;
      // MPI mode: the inputs carrying embedding channels run padded (Ep)
      const int pad1 = (E > 0 && bs.bid == 1) ? bs.c1.cin - E + Ep : 0;
      const int pad2 = (E > 0 && bs.cskip > 0) ? bs.c2.cin - E + Ep : 0;
      MD2_TRY(make_conv(d.c1, bs.c1, h, w, true, wsn, pad1));
      need_ws(d.c1, ND, wsn, true);
      MD2_TRY(make_conv(d.c2, bs.c2, 2 * h, 2 * w, true, wsn, pad2));
      need_ws(d.c2, ND, wsn, true);
      need_ws(d.c1, ND, wsn_side, false);   // filter gradients on the side stream (wgrad_overlap)
      need_ws(d.c2, ND, wsn_side, false);
      MD2_TRY(alloc(&d.o1, (long)ND * bs.cout * h * w));
      MD2_TRY(alloc(&d.up, (long)ND * bs.cout * 4 * h * w));
      MD2_TRY(alloc(&d.o2, (long)ND * bs.cout * 4 * h * w));
      MD2_TRY(alloc(&d.d_o2, (long)ND * bs.cout * 4 * h * w));
      track((long)ND * d.c2.s.Cin * 4 * h * w);
      if (bs.head >= 0) {
        d.head = bs.head;
        MD2_TRY(make_conv(d.hc, spec.heads[bs.head], 2 * h, 2 * w, true, wsn));
        need_ws(d.hc, ND, wsn, true);
        MD2_TRY(alloc(&d.disp, (long)ND * 4 * h * w));
        MD2_TRY(alloc(&d.d_head, (long)ND * 4 * h * w));
      }
      if (bs.bid <= 4) {
        const int fi = 4 - bs.bid;
        if (featH[fi] != 2 * h || featW[fi] != 2 * w) {
          set_error("decoder/encoder resolution mismatch (image sides must be multiples of 32)");
          return MD2_EINVAL;
        }
        MD2_TRY(alloc(&d_skip[fi], (long)N * featC[fi] * 4 * h * w));
        if (E > 0) {
          MD2_TRY(alloc(&emb_in[fi], (long)ND * (featC[fi] + Ep) * 4 * h * w));
          MD2_TRY(alloc(&d_emb[fi], (long)ND * (featC[fi] + Ep) * 4 * h * w));
        }
      }
      h *= 2;
      w *= 2;
      br.push_back(d);
    }
    if (h != cfg.H || w != cfg.W) {
      // the final branch must come back to full resolution for the loss (levels up to 5)
    }
    {
      HeadJob jobs[MAX_HEADS];
      const int nh = head_jobs(jobs, ND);
      if (nh > 0) MD2_TRY(alloc(&hws, heads_bwd_workspace(jobs, nh) / sizeof(float) + 64));
    }
    // ---- pose decoder (2N pairs)
    const int h4 = featH[4], w4 = featW[4];
    const long hw4 = (long)h4 * w4;
    MD2_TRY(make_conv(sq, spec.squeezer, h4, w4, true, wsn_side));
    need_ws(sq, B, wsn_side, true);
    MD2_TRY(make_conv(p1, spec.p1, h4, w4, true, wsn_side));
    need_ws(p1, 2 * N, wsn_side, true);
    MD2_TRY(make_conv(p2, spec.p2, h4, w4, true, wsn_side));
    need_ws(p2, 2 * N, wsn_side, true);
    p1.cat = p2.cat = PROF_CONV3_ENC;     // zero-padded 3x3 like the encoder's (same kernels)
    MD2_TRY(alloc(&sqo, (long)B * 256 * hw4));
    MD2_TRY(alloc(&d_sq, (long)B * 256 * hw4));
    MD2_TRY(alloc(&pc1, 2L * N * 256 * hw4));
    MD2_TRY(alloc(&d_pc1, 2L * N * 256 * hw4));
    MD2_TRY(alloc(&pc2, 2L * N * 256 * hw4));
    MD2_TRY(alloc(&d_pin, 2L * N * 512 * hw4));
    for (int j = 0; j < 2; ++j) {
      const int s = j ? cfg.src1 : cfg.src0;
      pa[j] = std::min(s, cfg.target);
      pb[j] = std::max(s, cfg.target);
    }
    pairs_inplace = pa[0] == 0 && pa[1] == 1 && pb[0] == 1 && pb[1] == 2;
    if (!pairs_inplace) MD2_TRY(alloc(&pin, 2L * N * 512 * hw4));
    T0 = cfg.target * N;
    MD2_TRY(alloc(&means, 2L * N * 256));
    MD2_TRY(alloc(&pose, 2L * N * 6));
    MD2_TRY(alloc(&d_pose, 2L * N * 6));
    track(2L * N * 512 * hw4);
    // ---- scratch / workspaces
    MD2_TRY(alloc(&DA, scratch));
    MD2_TRY(alloc(&DY, scratch));
    MD2_TRY(alloc(&DY2, scratch));
    MD2_TRY(alloc(&G, scratch));
    MD2_TRY(alloc(&DYD, scratch));
    MD2_TRY(alloc(&DPRE, scratch));
    MD2_TRY(alloc(&DUP, scratch));
    MD2_TRY(alloc(&DO1, scratch));
    {
      float* q;
      MD2_TRY(alloc(&q, wsn / sizeof(float) + 64));
      cws.ptr = q;
      cws.bytes = wsn + 256;
    }
    MD2_TRY(alloc(&bp_ws, BP_WS));
    {
      float* q;
      MD2_TRY(alloc(&q, wsn_side / sizeof(float) + 64));
      cws_side.ptr = q;
      cws_side.bytes = wsn_side + 256;
    }
    MD2_TRY(alloc(&bp_ws_side, BP_WS));
    MD2_TRY(alloc(&DPRE_side, 2L * N * 256 * hw4));
    MD2_HIP(hipStreamCreateWithFlags(&side, hipStreamNonBlocking));
    MD2_HIP(hipStreamCreateWithFlags(&upd, hipStreamNonBlocking));
    MD2_HIP(hipEventCreateWithFlags(&seg_ev, hipEventDisableTiming));
    MD2_HIP(hipEventCreateWithFlags(&upd_ev, hipEventDisableTiming));
    MD2_HIP(hipEventCreateWithFlags(&fork_ev, hipEventDisableTiming));
    MD2_HIP(hipEventCreateWithFlags(&join_ev, hipEventDisableTiming));
    for (hipEvent_t* e : {&ev_a, &ev_b, &ev_c2, &ev_c1, &ev_y[0], &ev_y[1]})
      MD2_HIP(hipEventCreateWithFlags(e, hipEventDisableTiming));
    MD2_TRY(alloc(&bp_dec[0], BP_WS));
    MD2_TRY(alloc(&bp_dec[1], BP_WS));
    {
      double* q;
      void* v;
      bn_slot = std::max<long>(bnmax, 2);
      MD2_HIP(hipMalloc(&v, 2 * bn_slot * sizeof(double)));
      allocs.push_back(v);
      q = (double*)v;
      bnws.partials = q;
      MD2_HIP(hipMalloc(&v, 2 * 4096 * 2 * sizeof(double)));
      allocs.push_back(v);
      bn_collapsed = (double*)v;
    }
    // ---- loss tail (src/training.jl:21-78).  MPI mode: the ND plane disparities are the batch
    // (training.jl:42-51 reshapes depth to (1, W*H, dn) with dn = num_bins*N); the poses and the
    // frames of the one sample broadcast over its planes (Project's batched_mul of the 3x3x1 R,
    // grid_sample and SSIM against the N = 1 images): x sample stride 0, poses / automask
    // repeated per plane
    if (E > 0) {
      MD2_TRY(alloc(&pose_rep, 2L * ND * 6));
      MD2_TRY(alloc(&d_pose_rep, 2L * ND * 6));
      if (cfg.automask) MD2_TRY(alloc(&amask_rep, (long)ND * cfg.H * cfg.W));
    }
    tail.N = ND;
    tail.C = C;
    tail.W = cfg.W;
    tail.H = cfg.H;
    tail.nscales = A.nlevels;
    int li = 0;
    for (auto& d : br)
      if (d.head >= 0) {
        tail.dw[li] = 2 * d.w;
        tail.dh[li] = 2 * d.h;
        tail.smooth_w[li] = cfg.smoothness * cfg.scales[li];
        ++li;
      }
    tail.divisor = (float)A.nlevels;
    tail.smooth_normalize = 1;
    std::memcpy(tail.K, cfg.K, sizeof(tail.K));
    std::memcpy(tail.invK, cfg.invK, sizeof(tail.invK));
    tail.min_depth = cfg.min_depth;
    tail.max_depth = cfg.max_depth;
    tail.x_frame_stride = (long)C * cfg.H * cfg.W;
    tail.x_sample_stride = E > 0 ? 0 : 3 * tail.x_frame_stride;   // MPI: N == 1, planes share x
    tail.target = cfg.target;
    tail.src0 = cfg.src0;
    tail.src1 = cfg.src1;
    tail.invert_mask = (cfg.src0 < cfg.target ? 1 : 0) | (cfg.src1 < cfg.target ? 2 : 0);
    tail.sigmoid_grad = 1;
    {
      float* q;
      MD2_TRY(alloc(&q, loss_tail_workspace_bytes(tail) / sizeof(float) + 64));
      tail_ws = q;
    }
    MD2_TRY(alloc(&loss_buf, 16));
    if (cfg.automask) MD2_TRY(alloc(&amask, (long)N * cfg.H * cfg.W));
    return build_pack_table();
  }

  // -------------------------------------------------------------------------------------------
  // ---- optional HIP-event profiling of the hot kernels (bench.py roofline) ----------------
  struct ProfRec {
    hipEvent_t a, b;
    int cat;
    double work;
    char tag[64];   // pass + shape of a conv record (per-layer table), "" otherwise
  };
  bool prof = false;
  std::vector<ProfRec> recs;
  std::vector<hipEvent_t> evpool;
  size_t evi = 0;
  hipEvent_t ev() {
    if (evi == evpool.size()) {
      hipEvent_t e;
      (void)hipEventCreate(&e);
      evpool.push_back(e);
    }
    return evpool[evi++];
  }
  hipEvent_t prof_begin(hipStream_t st) {
    if (!prof) return nullptr;
    hipEvent_t e = ev();
    (void)hipEventRecord(e, st);
    return e;
  }
  void prof_end(hipEvent_t a, int cat, double work, hipStream_t st, const char* pass = nullptr,
                const ConvShape* s = nullptr) {
    if (!prof) return;
    hipEvent_t b = ev();
    (void)hipEventRecord(b, st);
    ProfRec r{a, b, cat, work, {0}};
    if (pass && s) {
      const int ar = conv_last_arith();
      snprintf(r.tag, sizeof(r.tag), "%s %dx%d/%d%s %d->%d %dx%d n%d [%s]", pass, s->KH, s->KW, s->stride,
               s->reflect ? "r" : "", s->Cin, s->Cout, s->H, s->W, s->N,
               ar == 6 ? "bf16x6" : ar == 1 ? "fp32" : "valu");
    }
    else if (pass)
      snprintf(r.tag, sizeof(r.tag), "%s", pass);
    recs.push_back(r);
  }
  static double conv_flops(const ConvShape& s) {
    return 2.0 * s.N * (double)s.Ho * s.Wo * s.Cout * weight_cin(s) * s.KH * s.KW;   // algorithmic
  }

  int conv_f(RConv& c, int nimg, const TensorIn& in, float* out, long out_bs, int act,
             int accumulate, hipStream_t st) {
    ConvShape s = c.s;
    s.N = nimg;
    TensorOut o;
    o.p0 = out;
    o.bs0 = out_bs;
    o.bias = P(c.p.b);
    o.act = act;
    o.accumulate = accumulate;
    hipEvent_t e = prof_begin(st);
    MD2_TRY(conv_fwd(s, in, c.wpf, o, ws_conv(), st));
    prof_end(e, c.cat, conv_flops(s), st, "fwd", &s);
    return MD2_OK;
  }
  // conv + BatchNorm statistics: a split-K conv leaves its slabs to the statistics pass, which
  // sums them (bit-identical to the conv's own reduction), writes y and takes the partials in one
  // launch.  The profile bracket then includes that fused pass (conservative for the roofline).
  int conv_f_bn(RConv& c, int nimg, const TensorIn& in, float* y, long out_bs, RBN& bn, long HW,
                hipStream_t st, int slot = 0) {
    ConvShape s = c.s;
    s.N = nimg;
    TensorOut o;
    o.p0 = y;
    o.bs0 = out_bs;
    o.bias = P(c.p.b);
    SplitKDefer d;
    // the LDS-halo forward without split-K takes the statistics in its epilogue (MD2_FUSE_BNSTATS=0:
    // the separate bn_stats_partial pass; within 1 ulp of mean / invstd, not bit-identical: the
    // fp64 sums run in another order)
    BNStatsWs wst = bn_ws(bn, nimg, HW, slot);
    if (fuse_bnstats) d.stats = wst.partials;
    d.keep_reduce = !fuse_splitk;
    hipEvent_t e = prof_begin(st);
    MD2_TRY(conv_fwd(s, in, c.wpf, o, ws_conv(), st, fuse_splitk || fuse_bnstats ? &d : nullptr));
    if (d.stats_parts > 0) {
      // (the apply passes finalise the tile partials per block, behind their own loads;
      // MD2_BN_COLLAPSE=1: one collapse launch first -- measured slower, 6 us per launch)
      if (bn_collapse) {
        MD2_CHECK_ARG(bn.p.c <= 4096, "conv_f_bn: BN channels");
        double* col = bn_collapsed + (long)slot * 2 * 4096;
        MD2_TRY(bn_partials_collapse(wst.partials, bn.p.c, d.stats_parts, col, st));
        bn.part = col;
        bn.parts = 1;
      } else {
        bn.part = wst.partials;
        bn.parts = d.stats_parts;
      }
      prof_end(e, c.cat, conv_flops(s), st, "fwd", &s);
      return MD2_OK;
    }
    if (d.splits > 0) {
      BNStatsWs w = bn_ws(bn, nimg, HW, slot);
      MD2_TRY(bn_stats_partial_slabs(SlabIn{d.slab, d.splits}, y, nimg, bn.p.c, HW, w, st));
      prof_end(e, c.cat, conv_flops(s), st, "fwd", &s);
      return MD2_OK;
    }
    prof_end(e, c.cat, conv_flops(s), st, "fwd", &s);
    return bn_fwd(bn, y, nimg, HW, st, slot);
  }
  // MD2_FUSE_SKIP_BWD=0 restores the axpy of the decoder skip gradients (A/B, bit-identity test)
  const bool fuse_skip_bwd = [] {
    const char* v = getenv("MD2_FUSE_SKIP_BWD");
    return !(v && v[0] == '0');
  }();
  // MD2_FUSE_POOL_FWD=0 restores bn_apply_fused + maxpool_fwd for the stem (A/B, bit-identity test)
  const bool fuse_pool_fwd = [] {
    const char* v = getenv("MD2_FUSE_POOL_FWD");
    return !(v && v[0] == '0');
  }();
  // MD2_FUSE_POOL_BWD=0 restores the stem's separate skip-gradient axpy after maxpool_bwd (A/B,
  // bit-identity test)
  const bool fuse_pool_bwd = [] {
    const char* v = getenv("MD2_FUSE_POOL_BWD");
    return !(v && v[0] == '0');
  }();
  const bool bn_collapse = tuning_knob("MD2_BN_COLLAPSE", 0) != 0;
  // MD2_FUSE_BNSTATS=0 restores the statistics pass after the LDS-halo forward convs
  const bool fuse_bnstats = [] {
    const char* v = getenv("MD2_FUSE_BNSTATS");
    return !(v && v[0] == '0');
  }();
  // MD2_FUSE_SPLITK=0 restores the separate reduction launches (A/B measurement)
  const bool fuse_splitk = [] {
    const char* v = getenv("MD2_FUSE_SPLITK");
    return !(v && v[0] == '0');
  }();
  static TensorIn tin(const float* p, int C, long HW) {
    TensorIn t;
    t.p0 = p;
    t.c0 = C;
    t.bs0 = (long)C * HW;
    return t;
  }

  // one batched launch re-packs every conv weight (forward and dgrad layouts) after an update;
  // each weight is read once and written to both layouts
  PackJob* pack_jobs = nullptr;
  int pack_njobs = 0;
  long pack_blocks = 0;

  int build_pack_table() {
    std::vector<PackJob> jobs;
    auto pk = [&](RConv& c) { jobs.push_back(conv_pack_job(c.s, params + c.p.w, c.wpf, c.wpd)); };
    pk(stem);
    for (auto& sg : stages)
      for (auto& b : sg) {
        for (auto& e : b.st) pk(e.conv);
        if (b.down) pk(b.dconv);
      }
    for (auto& d : br) {
      pk(d.c1);
      pk(d.c2);
      if (d.head >= 0) pk(d.hc);
    }
    pk(sq);
    pk(p1);
    pk(p2);
    long blocks = 0;
    for (auto& j : jobs) {
      j.block_begin = blocks;
      blocks += conv_pack_job_blocks(j);
    }
    void* q = nullptr;
    MD2_HIP(hipMalloc(&q, jobs.size() * sizeof(PackJob)));
    allocs.push_back(q);
    MD2_HIP(hipMemcpy(q, jobs.data(), jobs.size() * sizeof(PackJob), hipMemcpyHostToDevice));
    pack_jobs = (PackJob*)q;
    pack_njobs = (int)jobs.size();
    pack_blocks = blocks;
    // the same jobs grouped by the backward segment that owns their parameters (each group with
    // its own block numbering)
    for (int k = 0; k < 6; ++k) {
      long b0, e0;
      segment_range(k, b0, e0);
      std::vector<PackJob> sj;
      long sb = 0;
      for (PackJob j : jobs) {
        const long off = (long)(j.w - params);
        if (off < b0 || off >= e0) continue;
        j.block_begin = sb;
        sb += conv_pack_job_blocks(j);
        sj.push_back(j);
      }
      seg_pack[k] = SegPack{};
      if (sj.empty()) continue;
      void* qs = nullptr;
      MD2_HIP(hipMalloc(&qs, sj.size() * sizeof(PackJob)));
      allocs.push_back(qs);
      MD2_HIP(hipMemcpy(qs, sj.data(), sj.size() * sizeof(PackJob), hipMemcpyHostToDevice));
      seg_pack[k] = SegPack{(PackJob*)qs, (int)sj.size(), sb};
    }
    return MD2_OK;
  }

  // the parameter range [b, e) of backward segment k (model_backward_segment)
  void segment_range(int k, long& b, long& e) const {
    const ArchSpec& S = spec;
    switch (k) {
      case 0: b = S.depth_begin; e = S.total; break;
      case 1: b = S.stage_begin[4]; e = S.depth_begin; break;
      case 2: b = S.stage_begin[3]; e = S.stage_begin[4]; break;
      case 3: b = S.stage_begin[2]; e = S.stage_begin[3]; break;
      case 4: b = S.stage_begin[1]; e = S.stage_begin[2]; break;
      default: b = 0; e = S.stage_begin[1]; break;
    }
  }

  // ADAM over segment k's parameters + the re-pack of its conv weights on `upd`, ordered after
  // everything enqueued on st so far (its backward segment, and a DP caller's all-reduce of the
  // bucket when st waits on it)
  int adam_segment(int k, float* am, float* av, float lr, float b1, float b2, float eps, float bc1,
                   float bc2, float gscale, hipStream_t st) {
    long b0, e0;
    segment_range(k, b0, e0);
    MD2_HIP(hipEventRecord(seg_ev, st));
    MD2_HIP(hipStreamWaitEvent(upd, seg_ev, 0));
    MD2_TRY(adam_step(params + b0, grads + b0, am + b0, av + b0, e0 - b0, lr, b1, b2, eps, bc1, bc2,
                      gscale, upd));
    if (seg_pack[k].njobs) MD2_TRY(conv_pack_batch(seg_pack[k].jobs, seg_pack[k].njobs, seg_pack[k].blocks, upd));
    MD2_HIP(hipEventRecord(upd_ev, upd));
    upd_recorded = true;
    return MD2_OK;
  }
  // st waits for every update enqueued by adam_segment.  The ordering is per stream, so once an
  // update was ever recorded EVERY join waits (an entry point on another stream -- a Python
  // executor sharing the parameters, a user stream for eval or get_params -- must see it too);
  // waiting on a completed event costs next to nothing.
  int adam_join(hipStream_t st) {
    if (upd_recorded) MD2_HIP(hipStreamWaitEvent(st, upd_ev, 0));
    return MD2_OK;
  }

  int repack(hipStream_t st) { return conv_pack_batch(pack_jobs, pack_njobs, pack_blocks, st); }

  // statistics partials only; the finalise is fused into the apply (bn_apply_fused)
  BNStatsWs bn_ws(RBN& bn, int nimg, long HW, int slot) {
    BNStatsWs w = bnws;
    w.partials += slot * bn_slot;
    w.parts = bn_parts(bn.p.c, nimg, HW);
    bn.part = w.partials;
    bn.parts = w.parts;
    return w;
  }
  int bn_fwd(RBN& bn, const float* y, int nimg, long HW, hipStream_t st, int slot = 0) {
    return bn_stats_partial(y, nimg, bn.p.c, HW, bn_ws(bn, nimg, HW, slot), st);
  }
  BNStatsIn bn_in(const RBN& bn) {
    BNStatsIn s;
    s.part = bn.part;
    s.parts = bn.parts;
    s.gamma = P(bn.p.g);
    s.beta = P(bn.p.b);
    s.mean = bn.mean;
    s.invstd = bn.invstd;
    s.run_mean = bn.rmean;
    s.run_var = bn.rvar;
    return s;
  }

  // ---- encoder forward over nimg images (input already mapped by `in`)
  int encoder_fwd(const TensorIn& in, int nimg, hipStream_t st) {
    const long hw0 = (long)H0 * W0;
    MD2_TRY(conv_f_bn(stem, nimg, in, y0, 64 * hw0, stem_bn, hw0, st));
    BNApplyFused ap{};
    ap.y = y0; ap.s1 = bn_in(stem_bn); ap.relu = 1;
    if (H0 % 2 == 0 && W0 % 2 == 0 && fuse_pool_fwd) {   // BN + ReLU + max pool in one pass
      MD2_TRY(bn_relu_maxpool(ap, f0, nimg, 64, H0, W0, mp, mp_arg, Hm, Wm, st));
    } else {
      MD2_TRY(bn_apply_fused(ap, f0, nimg, 64, hw0, st));
      MD2_TRY(maxpool_fwd(f0, nimg, 64, H0, W0, mp, mp_arg, Hm, Wm, st));
    }
    for (auto& sg : stages)
      for (auto& b : sg) {
        const float* x = b.in;
        int C = b.Cin;
        long HW = (long)b.Hin * b.Win;
        const bool dov = b.down && down_overlap();
        if (dov) {
          MD2_TRY(stream_wait(st, side, fork_ev));
          MD2_TRY(down_fwd(b, nimg, side));
          MD2_HIP(hipEventRecord(join_ev, side));
        }
        for (size_t k = 0; k < b.st.size(); ++k) {
          EncStage& e = b.st[k];
          const long ohw = (long)e.conv.s.Ho * e.conv.s.Wo;
          MD2_TRY(conv_f_bn(e.conv, nimg, tin(x, C, HW), e.y, (long)e.conv.p.cout * ohw, e.bn, ohw, st));
          if (k + 1 < b.st.size()) {
            BNApplyFused a{};
            a.y = e.y; a.s1 = bn_in(e.bn); a.relu = 1;
            MD2_TRY(bn_apply_fused(a, e.a, nimg, e.conv.p.cout, ohw, st));
          }
          x = e.a;
          C = e.conv.p.cout;
          HW = ohw;
        }
        EncStage& last = b.st.back();
        const long ohw = (long)b.H * b.W;
        BNApplyFused a{};
        a.y = last.y; a.s1 = bn_in(last.bn); a.relu = 1;
        if (b.down) {
          if (dov)
            MD2_HIP(hipStreamWaitEvent(st, join_ev, 0));
          else
            MD2_TRY(down_fwd(b, nimg, st));
          a.y2 = b.yd; a.s2 = bn_in(b.dbn);
        } else {
          a.res = b.in;
        }
        MD2_TRY(bn_apply_fused(a, last.a, nimg, b.C, ohw, st));
      }
    return MD2_OK;
  }

  // ---- depth decoder over nimg images whose features start at image offset `img0`
  // MPI mode: the decoder inputs of all levels from the target features of the last forward
  int mpi_embed(int nimg, int img0, hipStream_t st) {
    for (int fi = 0; fi < 5; ++fi)
      if (emb_in[fi]) {
        const long hw = (long)featH[fi] * featW[fi];
        MD2_TRY(mpi_embed_features(feat[fi] + (long)img0 * featC[fi] * hw, (long)featC[fi] * hw, nimg,
                                   featC[fi], featH[fi], featW[fi], bins, NP, (E - 1) / 2, emb_in[fi], st,
                                   featC[fi] + Ep));
      }
    return MD2_OK;
  }

  int decoder_fwd(int nimg, int img0, hipStream_t st) {
    const float* x = feat[4] + (long)img0 * featC[4] * featH[4] * featW[4];
    int C = featC[4];
    if (E > 0) {                       // decoder batch: nimg * P plane images
      MD2_TRY(mpi_embed(nimg, img0, st));
      x = emb_in[4];
      C = featC[4] + Ep;
      nimg *= NP;
    }
    for (auto& d : br) {
      const long hw = (long)d.h * d.w, hw2 = 4 * hw;
      const int co = d.b.cout;
      MD2_TRY(conv_f(d.c1, nimg, tin(x, C, hw), d.o1, co * hw, ACT_ELU, 0, st));
      MD2_TRY(upsample2_fwd(d.o1, nimg, co, d.h, d.w, d.up, st));
      TensorIn in = tin(d.up, co, hw2);
      if (d.b.cskip > 0) {
        const int fi = 4 - d.b.bid;
        if (E > 0) {
          in.p1 = emb_in[fi];
          in.bs1 = (long)(featC[fi] + Ep) * hw2;
        } else {
          in.p1 = feat[fi] + (long)img0 * featC[fi] * hw2;
          in.bs1 = (long)featC[fi] * hw2;
        }
      }
      MD2_TRY(conv_f(d.c2, nimg, in, d.o2, co * hw2, ACT_ELU, 0, st));
      x = d.o2;
      C = co;
    }
    {
      HeadJob jobs[MAX_HEADS];
      const int nh = head_jobs(jobs, nimg);
      hipEvent_t e = prof_begin(st);
      MD2_TRY(heads_fwd(jobs, nh, ACT_SIGMOID, st));
      prof_end(e, PROF_CONV_OTHER, heads_flops(nimg), st, "heads fwd");
    }
    return MD2_OK;
  }

  // the DepthDecoder's disparity heads run as one batch per pass (head.h)
  float* hws = nullptr;
  int head_jobs(HeadJob* jobs, int nimg) {
    int n = 0;
    for (auto& d : br) {
      if (d.head < 0) continue;
      HeadJob& j = jobs[n++];
      j = HeadJob{};
      const long hw2 = 4L * d.h * d.w;
      j.x = conv_head_in(tin(d.o2, d.b.cout, hw2));
      j.wf = conv_head_w(d.hc.s, 0, d.hc.wpf);
      j.wd = conv_head_w(d.hc.s, 1, d.hc.wpd);
      j.Cin = d.b.cout;
      j.H = 2 * d.h;
      j.W = 2 * d.w;
      j.N = nimg;
      j.bias = P(d.hc.p.b);
      j.y = d.disp;
      j.ybs = hw2;
      j.dy = d.d_head;
      j.dx = d.d_o2;
      j.dxbs = (long)d.b.cout * hw2;
      j.dw = grads + d.hc.p.w;
      j.db = Gd(d.hc.p.b);
    }
    return n;
  }
  double heads_flops(int nimg) const {
    double f = 0.0;
    for (auto& d : br)
      if (d.head >= 0) f += 2.0 * nimg * 4.0 * d.h * d.w * 9.0 * d.b.cout;
    return f;
  }

  // PoseDecoder input of the 2N pairs: in place for the default ids, else the gathered pin
  TensorIn pose_pairs_in(long hw4) {
    if (!pairs_inplace) return tin(pin, 512, hw4);
    TensorIn in = tin(sqo, 256, hw4);
    in.p1 = sqo + (long)N * 256 * hw4;   // pair (frame s, frame s+1) = images (q, q+N)
    in.bs1 = 256 * hw4;
    return in;
  }

  int pose_fwd(hipStream_t st) {
    side_ws = true;
    const int rc = pose_fwd_body(st);
    side_ws = false;
    return rc;
  }
  int pose_fwd_body(hipStream_t st) {
    const long hw4 = (long)featH[4] * featW[4];
    MD2_TRY(conv_f(sq, B, tin(feat[4], featC[4], hw4), sqo, 256 * hw4, ACT_RELU, 0, st));
    if (!pairs_inplace) MD2_TRY(pair_gather(sqo, N, 256, hw4, pa, pb, pin, st));
    MD2_TRY(conv_f(p1, 2 * N, pose_pairs_in(hw4), pc1, 256 * hw4, ACT_RELU, 0, st));
    MD2_TRY(conv_f(p2, 2 * N, tin(pc1, 256, hw4), pc2, 256 * hw4, ACT_RELU, 0, st));
    return pose_head_fwd(pc2, 2 * N, 256, hw4, P(spec.p3.w), P(spec.p3.b), means, pose, st);
  }

  // (m)(x, source_ids, target_id) (src/model.jl:31-55): encoder on the 3N frames, DepthDecoder on
  // the targets, PoseDecoder on the pairs -- disparities and poses, no loss tail
  int forward(const float* x, hipStream_t st) {
    const long fs = (long)cfg.arch.in_ch * cfg.H * cfg.W;
    TensorIn in;
    in.p0 = x;
    in.c0 = cfg.arch.in_ch;
    in.bdiv = N;          // image b = l*N + n  ->  x[n][l]
    in.bs0 = 3 * fs;
    in.bhi = fs;
    MD2_TRY(encoder_fwd(in, B, st));
    if (pose_overlap()) {
      MD2_TRY(stream_wait(st, side, fork_ev));
      MD2_TRY(pose_fwd(side));
      MD2_TRY(decoder_fwd(N, T0, st));
      MD2_TRY(stream_wait(side, st, join_ev));
    } else {
      MD2_TRY(decoder_fwd(N, T0, st));
      MD2_TRY(pose_fwd(st));
    }
    return MD2_OK;
  }

  int forward_loss(const float* x, const float* automask, float* loss, float* terms,
                   hipStream_t st) {
    MD2_TRY(forward(x, st));
    const float* disps[MAX_SCALES] = {};
    LossTailOut o{};
    int li = 0;
    for (auto& d : br)
      if (d.head >= 0) {
        disps[li] = d.disp;
        o.d_disp[li] = d.d_head;
        ++li;
      }
    o.loss = loss ? loss : loss_buf;
    o.terms = terms;
    o.d_pose = E > 0 ? d_pose_rep : d_pose;
    hipEvent_t pev[2 * MAX_SCALES] = {};
    if (prof) {
      for (int k = 0; k < 2; ++k) pev[k] = ev();
      o.photo_events = pev;
    }
    if (cfg.automask && !automask) {
      // automasking_loss(ssim, x, target; source_ids) (src/training.jl:9-11): identity
      // reprojection of the raw sources, the third candidate of every scale's per-pixel min
      MD2_TRY(launch_automask(x, tail.x_sample_stride, tail.x_frame_stride, tail.target, tail.src0,
                              tail.src1, N, cfg.arch.in_ch, cfg.H, cfg.W, amask, st));
      automask = amask;
    }
    const float* tail_pose = pose;
    if (E > 0) {
      // every plane of a sample warps with that sample's poses and is compared with its frames
      MD2_TRY(repeat_rows(pose, 2L * N, 6, NP, pose_rep, st));
      tail_pose = pose_rep;
      if (cfg.automask) {
        MD2_TRY(repeat_rows(automask, N, cfg.H * cfg.W, NP, amask_rep, st));
        automask = amask_rep;
      }
    }
    MD2_TRY(loss_tail_run(tail, disps, tail_pose, x, cfg.automask ? automask : nullptr, 1.f, o, tail_ws, st));
    if (E > 0) MD2_TRY(repeat_rows_adjoint(d_pose_rep, 2L * N, 6, NP, d_pose, st));
    if (prof) {
      // one launch for all scales; algorithmic bytes per full-res pixel and scale:
      // disparity 4 + target 4C + two sources 8C + d_disp 4
      const double bytes = (double)tail.nscales * ND * cfg.H * cfg.W * (8.0 + 12.0 * cfg.arch.in_ch);
      recs.push_back({pev[0], pev[1], PROF_PHOTO, bytes, "photometric (all scales)"});
    }
    return MD2_OK;
  }

  // per-record view of the same events (per-layer table); clears like profile_read
  int profile_records(int max, double* ms, double* work, int* cat, char* tags, int tag_len,
                      int* count) {
    int k = 0;
    for (auto& r : recs) {
      if (k >= max) break;
      MD2_HIP(hipEventSynchronize(r.b));
      float t = 0.f;
      MD2_HIP(hipEventElapsedTime(&t, r.a, r.b));
      ms[k] = t;
      work[k] = r.work;
      cat[k] = r.cat;
      if (tags && tag_len > 0) {
        strncpy(tags + (long)k * tag_len, r.tag, tag_len - 1);
        tags[(long)k * tag_len + tag_len - 1] = 0;
      }
      ++k;
    }
    *count = k;
    recs.clear();
    evi = 0;
    return MD2_OK;
  }

  int profile_read(double* out, int ncat) {
    for (int c = 0; c < ncat * 3; ++c) out[c] = 0.0;
    for (auto& r : recs) {
      MD2_HIP(hipEventSynchronize(r.b));
      float ms = 0.f;
      MD2_HIP(hipEventElapsedTime(&ms, r.a, r.b));
      if (r.cat < ncat) {
        out[r.cat * 3 + 0] += ms;
        out[r.cat * 3 + 1] += r.work;
        out[r.cat * 3 + 2] += 1.0;
      }
    }
    recs.clear();
    evi = 0;
    return MD2_OK;
  }

  // -------------------------------------------------------------------------------------------
  int conv_w(RConv& c, int nimg, const TensorIn& in, const float* dy, hipStream_t st) {
    ConvShape s = c.s;
    s.N = nimg;
    hipEvent_t e = prof_begin(st);
    MD2_TRY(conv_wgrad(s, in, dy, grads + c.p.w, Gd(c.p.b), 0, ws_conv(), st, c.p.b >= 0 ? bp_pending : nullptr,
                       bp_parts));
    bp_pending = nullptr;
    prof_end(e, c.cat, conv_flops(s), st, "wgrad", &s);
    return MD2_OK;
  }
  // filter and data gradient of one conv from the same dY.  (Running the filter gradient on a
  // second stream overlapped them but each slowed by as much, and the cross-queue fork/join
  // added ~1.3 ms/step of idle gaps: measured slower, so both stay on `st`.)
  int conv_wd(RConv& c, int nimg, const TensorIn& in, const float* dy, float* dx, long dx_bs,
              int acc, hipStream_t st, float* dx1 = nullptr, long dx1_bs = 0, int c0 = 1 << 30) {
    MD2_TRY(conv_w(c, nimg, in, dy, st));
    return conv_d(c, nimg, dy, dx, dx_bs, acc, st, dx1, dx1_bs, c0);
  }
  int conv_d(RConv& c, int nimg, const float* dy, float* dx, long dx_bs, int acc, hipStream_t st,
             float* dx1 = nullptr, long dx1_bs = 0, int c0 = 1 << 30) {
    ConvShape s = c.s;
    s.N = nimg;
    TensorOut o;
    o.p0 = dx;
    o.bs0 = dx_bs;
    o.p1 = dx1;
    o.bs1 = dx1_bs;
    o.c0 = c0;
    o.accumulate = acc;
    hipEvent_t e = prof_begin(st);
    MD2_TRY(conv_dgrad(s, dy, c.wpd, o, ws_conv(), st));
    prof_end(e, c.cat, conv_flops(s), st, "dgrad", &s);
    return MD2_OK;
  }
  // dgrad into DA followed by the backward of the residual-free BN+ReLU that produced the conv's
  // input (ReLU mask re-derived from y): a split-K dgrad leaves its slabs to bn_bwd_partial, which
  // forms DA in the same pass (profile bracket includes it, as conv_f_bn)
  int conv_d_bn(RConv& c, int nimg, const float* dy, float* da, long da_bs, RBN& bn, const float* y,
                long HW, float* dyprev, hipStream_t st) {
    ConvShape s = c.s;
    s.N = nimg;
    TensorOut o;
    o.p0 = da;
    o.bs0 = da_bs;
    SplitKDefer d;
    hipEvent_t e = prof_begin(st);
    MD2_TRY(conv_dgrad(s, dy, c.wpd, o, ws_conv(), st, fuse_splitk ? &d : nullptr));
    if (d.splits == 0) {
      prof_end(e, c.cat, conv_flops(s), st, "dgrad", &s);
      return bn_bwd(bn, da, nullptr, y, nimg, HW, dyprev, nullptr, 0, st, true);
    }
    BNStatsWs w = bnws;
    w.parts = bn_parts(bn.p.c, nimg, HW);
    MD2_TRY(bn_bwd_partial_slabs(SlabIn{d.slab, d.splits}, da, y, bn.mean, bn.invstd, nimg, bn.p.c,
                                 HW, w, st, P(bn.p.g), P(bn.p.b)));
    prof_end(e, c.cat, conv_flops(s), st, "dgrad", &s);
    return bn_bwd_apply_fused(da, nullptr, y, bn.mean, bn.invstd, P(bn.p.g), w, Gd(bn.p.g),
                              Gd(bn.p.b), nimg, bn.p.c, HW, dyprev, nullptr, 0, st, P(bn.p.b));
  }
  // activation pullback fused with the bias-gradient partials of the conv that produced `out`
  // (consumed by that conv's next conv_w)
  float* bp_ws = nullptr;
  const float* bp_pending = nullptr;
  int bp_parts = 0;
  int act_bias(const float* out, const float* dout, float* dpre, int nimg, int C, long HW, int act,
               hipStream_t st, float* bp_buf = nullptr) {
    if (HW % 4 != 0 || (long)C * act_bias_parts(C, nimg, HW) > BP_WS) {
      bp_pending = nullptr;
      return act_backward(out, dout, dpre, (long)nimg * C * HW, act, st);
    }
    float* bp = bp_buf ? bp_buf : ws_bp();
    MD2_TRY(act_backward_bias(out, dout, dpre, nimg, C, HW, act, bp, st));
    bp_pending = bp;
    bp_parts = act_bias_parts(C, nimg, HW);
    return MD2_OK;
  }
  static constexpr long BP_WS = 8192;

  // mask: the BN+ReLU output whose ReLU gates dout, or nullptr with relu_from_y for a residual-free
  // BN+ReLU (stem, intra-block): the mask is re-derived from y (bit-exact, one read less)
  int bn_bwd(RBN& bn, const float* dout, const float* mask, const float* y, int nimg, long HW,
             float* dy, float* dres, int dres_acc, hipStream_t st, bool relu_from_y = false,
             SkipAdd sk = SkipAdd{}, int slot = 0) {
    BNStatsWs w = bnws;
    w.partials += slot * bn_slot;
    w.parts = bn_parts(bn.p.c, nimg, HW);
    const float* mg = relu_from_y ? P(bn.p.g) : nullptr;
    const float* mb = relu_from_y ? P(bn.p.b) : nullptr;
    if (relu_from_y) mask = nullptr;
    MD2_TRY(bn_bwd_partial(dout, mask, y, bn.mean, bn.invstd, nimg, bn.p.c, HW, w, st, mg, mb, sk));
    return bn_bwd_apply_fused(dout, mask, y, bn.mean, bn.invstd, P(bn.p.g), w, Gd(bn.p.g),
                              Gd(bn.p.b), nimg, bn.p.c, HW, dy, dres, dres_acc, st, mb, sk);
  }
  // the decoder skip gradient d_skip[si] on the target slice of encoder feature si (si = 1..3, the
  // input of stage si = the output of stage si-1): added by stage si-1's last-block BN backward
  // when fused (MD2_FUSE_SKIP_BWD, HW % 4 == 0), else by an axpy after stage si's backward
  bool skip_fused(int si) const {
    return fuse_skip_bwd && si >= 1 && si <= 3 && d_skip[si] && ((long)featH[si] * featW[si]) % 4 == 0;
  }
  SkipAdd skip_add(int si) const {
    SkipAdd sk;
    if (!skip_fused(si)) return sk;
    const long fsz = (long)featC[si] * featH[si] * featW[si];
    sk.skip = d_skip[si];
    sk.lo = (long)T0 * fsz;
    sk.hi = (long)(T0 + N) * fsz;
    return sk;
  }

  int block_bwd(EncBlock& b, hipStream_t st, SkipAdd sk = SkipAdd{}, bool eov = false) {
    const int nimg = B;
    const long ohw = (long)b.H * b.W, ihw = (long)b.Hin * b.Win;
    const int ns = (int)b.st.size();
    EncStage& last = b.st.back();
    // last BN (+ residual, ReLU): g = (d_out [+ skip]) * relu'(out)
    MD2_TRY(y_claim(ycur, st));
    MD2_TRY(bn_bwd(last.bn, b.d_out, last.a, last.y, nimg, ohw, ybuf(ycur), b.down ? G : b.d_in, 0, st,
                   false, sk));
    const bool dov = b.down && down_overlap();
    if (b.down) {
      // downsample branch: BN backward (partials slot 1) + the 1x1 conv's filter and data
      // gradients (d_in written whole; the chain's first conv adds to it below)
      hipStream_t sd = dov ? side : st;
      if (dov) MD2_TRY(stream_wait(st, side, fork_ev));
      MD2_TRY(bn_bwd(b.dbn, G, nullptr, b.yd, nimg, ohw, DYD, nullptr, 0, sd, false, SkipAdd{}, 1));
      side_ws = true;
      const int rc = conv_wd(b.dconv, nimg, tin(b.in, b.Cin, ihw), DYD, b.d_in, (long)b.Cin * ihw, 0, sd);
      side_ws = false;
      MD2_TRY(rc);
      if (dov) MD2_HIP(hipEventRecord(join_ev, side));
    }
    for (int k = ns - 1; k >= 0; --k) {
      EncStage& e = b.st[k];
      const float* xin = k == 0 ? b.in : b.st[k - 1].a;
      const int cin = e.conv.p.cin;
      const long hin = (long)e.conv.s.H * e.conv.s.W;
      float* dy = ybuf(ycur);
      // MD2_ENC_WGRAD_MAIN0=1 (tuning): the first conv's filter gradient of each block stays on
      // the model stream, after its data gradient (balances the side stream's share)
      const bool wmain = eov && k == 0 && enc_wgrad_main0;
      if (eov && !wmain) {   // filter gradient beside the data gradient; dy untouched until ev_y[ycur]
        MD2_TRY(stream_wait(st, side, fork_ev));
        side_ws = true;
        const int rc = conv_w(e.conv, nimg, tin(xin, cin, hin), dy, side);
        side_ws = false;
        MD2_TRY(rc);
        MD2_HIP(hipEventRecord(ev_y[ycur], side));
        y_pending[ycur] = true;
      } else if (!wmain) {
        MD2_TRY(conv_w(e.conv, nimg, tin(xin, cin, hin), dy, st));
      }
      if (k > 0) {
        EncStage& pe = b.st[k - 1];
        const int nx = ycur ^ 1;
        MD2_TRY(y_claim(nx, st));
        MD2_TRY(conv_d_bn(e.conv, nimg, dy, DA, (long)cin * hin, pe.bn, pe.y, hin, ybuf(nx), st));
        ycur = nx;
      } else {
        if (dov) MD2_HIP(hipStreamWaitEvent(st, join_ev, 0));   // b.d_in written by the 1x1 dgrad
        MD2_TRY(conv_d(e.conv, nimg, dy, b.d_in, (long)cin * hin, 1, st));
        if (wmain) MD2_TRY(conv_w(e.conv, nimg, tin(xin, cin, hin), dy, st));
      }
    }
    return MD2_OK;
  }

  // PoseDecoder backward: d_pose -> pose parameter gradients and the layer-4 feature gradient
  // d_f4 (written whole by the squeezer's dgrad; the DepthDecoder's first branch adds to it)
  int pose_bwd(hipStream_t st) {
    side_ws = true;
    const int rc = pose_bwd_body(st);
    side_ws = false;
    return rc;
  }
  int pose_bwd_body(hipStream_t st) {
    const long hw4 = (long)featH[4] * featW[4];
    float* DP = DPRE_side;
    MD2_TRY(pose_head_bwd(d_pose, 2 * N, 256, hw4, P(spec.p3.w), means, DP, Gd(spec.p3.w),
                          Gd(spec.p3.b), st));
    MD2_TRY(act_bias(pc2, DP, DP, 2 * N, 256, hw4, ACT_RELU, st));
    MD2_TRY(conv_wd(p2, 2 * N, tin(pc1, 256, hw4), DP, d_pc1, 256 * hw4, 0, st));
    MD2_TRY(act_bias(pc1, d_pc1, d_pc1, 2 * N, 256, hw4, ACT_RELU, st));
    MD2_TRY(conv_wd(p1, 2 * N, pose_pairs_in(hw4), d_pc1, d_pin, 512 * hw4, 0, st));
    MD2_TRY(pair_grad_gather(d_pin, N, 256, hw4, pa, pb, d_sq, st));
    MD2_TRY(act_bias(sqo, d_sq, d_sq, B, 256, hw4, ACT_RELU, st));
    float* d_f4 = stages[3].back().d_out;
    return conv_wd(sq, B, tin(feat[4], featC[4], hw4), d_sq, d_f4, (long)featC[4] * hw4, 0, st);
  }

  int seg_decoder(hipStream_t st) {
    // ---- PoseDecoder backward: beside the DepthDecoder's on the side stream, or first
    const bool ov = pose_overlap();
    if (ov) {
      MD2_TRY(stream_wait(st, side, fork_ev));
      MD2_TRY(pose_bwd(side));
      MD2_HIP(hipEventRecord(join_ev, side));
    } else {
      MD2_TRY(pose_bwd(st));
    }
    float* d_f4 = stages[3].back().d_out;
    // ---- DepthDecoder backward (reverse branch order), over ND decoder images
    const int nb = (int)br.size();
    {
      // every head's data + filter gradient first (their d_head all come from the loss tail):
      // d_o2 of a head branch is then the head's dx, and the next branch's c1 dgrad adds to it
      HeadJob jobs[MAX_HEADS];
      const int nh = head_jobs(jobs, ND);
      hipEvent_t e = prof_begin(st);
      MD2_TRY(heads_bwd(jobs, nh, hws, heads_bwd_workspace(jobs, nh) + 256, st));
      prof_end(e, PROF_CONV_OTHER, 2.0 * heads_flops(ND), st, "heads bwd");
    }
    const bool wov = wgrad_overlap();
    // filter gradient of conv c on the side stream once the main stream has reached `ready`
    auto wgrad_side = [&](RConv& c, const TensorIn& in, const float* dy, hipEvent_t ready,
                          hipEvent_t done) -> int {
      MD2_TRY(stream_wait(st, side, ready));
      side_ws = true;
      const int rc = conv_w(c, ND, in, dy, side);
      side_ws = false;
      MD2_TRY(rc);
      MD2_HIP(hipEventRecord(done, side));
      return MD2_OK;
    };
    for (int i = nb - 1; i >= 0; --i) {
      DecBranch& d = br[i];
      const long hw = (long)d.h * d.w, hw2 = 4 * hw;
      const int co = d.b.cout;
      float* const dpre = DPRE;
      float* const do1 = DO1;
      const hipEvent_t evc2 = ev_c2, evc1 = ev_c1;
      float* const bpc2 = bp_dec[0];
      float* const bpc1 = bp_dec[1];
      if (wov && i < nb - 1) MD2_HIP(hipStreamWaitEvent(st, evc2, 0));   // dpre, bpc2 free
      MD2_TRY(act_bias(d.o2, d.d_o2, dpre, ND, co, hw2, ACT_ELU, st, wov ? bpc2 : nullptr));
      TensorIn in = tin(d.up, co, hw2);
      float* dskip = nullptr;
      long skip_bs = 0;
      if (d.b.cskip > 0) {
        const int fi = 4 - d.b.bid;
        if (E > 0) {
          in.p1 = emb_in[fi];
          in.bs1 = (long)(featC[fi] + Ep) * hw2;
          dskip = d_emb[fi];
          skip_bs = (long)(featC[fi] + Ep) * hw2;
        } else {
          in.p1 = feat[fi] + (long)T0 * featC[fi] * hw2;
          in.bs1 = (long)featC[fi] * hw2;
          dskip = d_skip[fi];
          skip_bs = (long)featC[fi] * hw2;
        }
      }
      if (wov) {
        MD2_TRY(wgrad_side(d.c2, in, dpre, ev_a, evc2));
        MD2_TRY(conv_d(d.c2, ND, dpre, DUP, co * hw2, 0, st, dskip, skip_bs, co));
      } else {
        MD2_TRY(conv_wd(d.c2, ND, in, dpre, DUP, co * hw2, 0, st, dskip, skip_bs, co));
      }
      if (E > 0 && d.b.cskip > 0) {
        // _repeat pullback: the skip gradient of the target features = sum over the planes
        const int fi = 4 - d.b.bid;
        MD2_TRY(plane_sum(d_emb[fi], N, NP, featC[fi] + Ep, featC[fi], hw2, d_skip[fi], 0, st));
      }
      if (wov && i < nb - 1) MD2_HIP(hipStreamWaitEvent(st, evc1, 0));   // do1, bpc1 free
      MD2_TRY(upsample2_bwd(DUP, ND, co, d.h, d.w, do1, st));
      MD2_TRY(act_bias(d.o1, do1, do1, ND, co, hw, ACT_ELU, st, wov ? bpc1 : nullptr));
      const float* xin;
      int cin;
      float* dx;
      int acc;
      if (i == 0 && ov) MD2_HIP(hipStreamWaitEvent(st, join_ev, 0));   // d_f4 written by the squeezer
      if (i == 0 && E > 0) {
        cin = featC[4] + Ep;
        xin = emb_in[4];
        dx = d_emb[4];
        acc = 0;
      } else if (i == 0) {
        cin = featC[4];
        xin = feat[4] + (long)T0 * cin * hw;
        dx = d_f4 + (long)T0 * cin * hw;
        acc = 1;
      } else {
        cin = br[i - 1].b.cout;
        xin = br[i - 1].o2;
        dx = br[i - 1].d_o2;
        acc = br[i - 1].head >= 0 ? 1 : 0;   // on top of the head's dx
      }
      if (wov) {
        MD2_TRY(wgrad_side(d.c1, tin(xin, cin, hw), do1, ev_b, evc1));
        MD2_TRY(conv_d(d.c1, ND, do1, dx, (long)cin * hw, acc, st));
      } else {
        MD2_TRY(conv_wd(d.c1, ND, tin(xin, cin, hw), do1, dx, (long)cin * hw, acc, st));
      }
      if (i == 0 && E > 0)
        MD2_TRY(plane_sum(d_emb[4], N, NP, cin, featC[4], hw, d_f4 + (long)T0 * featC[4] * hw, 1, st));
    }
    // every decoder filter gradient final: the side runs in order, so its last event covers all
    if (wov) MD2_HIP(hipStreamWaitEvent(st, ev_c1, 0));
    return MD2_OK;
  }

  int seg_stage(int si, hipStream_t st) {
    auto& sg = stages[si];
    for (int k = (int)sg.size() - 1; k >= 0; --k)
      MD2_TRY(block_bwd(sg[k], st, k == (int)sg.size() - 1 ? skip_add(si + 1) : SkipAdd{}, enc_overlap(si)));
    for (int j = 0; j < 2; ++j) MD2_TRY(y_claim(j, st));   // the stage's filter gradients final
    if (si >= 1 && !skip_fused(si)) {
      // d f_si (= block 0's d_in) += decoder skip gradient on the target slice
      const long n = (long)N * featC[si] * featH[si] * featW[si];
      MD2_TRY(axpy(sg[0].d_in + (long)T0 * featC[si] * featH[si] * featW[si], d_skip[si], n, st));
    }
    return MD2_OK;
  }

  int seg_stem(hipStream_t st) {
    const long hw0 = (long)H0 * W0;
    const long n = (long)N * 64 * hw0;
    if (W0 % 2 == 0 && fuse_pool_bwd && d_skip[0]) {
      // the decoder skip gradient added by the max-pool adjoint itself (no axpy pass)
      SkipAdd sk;
      sk.skip = d_skip[0];
      sk.lo = (long)T0 * 64 * hw0;
      sk.hi = sk.lo + n;
      MD2_TRY(maxpool_bwd(d_mp, mp_arg, B, 64, H0, W0, Hm, Wm, d_f0, st, sk));
    } else {
      MD2_TRY(maxpool_bwd(d_mp, mp_arg, B, 64, H0, W0, Hm, Wm, d_f0, st));
      MD2_TRY(axpy(d_f0 + (long)T0 * 64 * hw0, d_skip[0], n, st));
    }
    MD2_TRY(bn_bwd(stem_bn, d_f0, f0, y0, B, hw0, DY, nullptr, 0, st, true));
    const long fs = (long)cfg.arch.in_ch * cfg.H * cfg.W;
    TensorIn in;
    in.p0 = cur_x;
    in.c0 = cfg.arch.in_ch;
    in.bdiv = N;
    in.bs0 = 3 * fs;
    in.bhi = fs;
    return conv_w(stem, B, in, DY, st);
  }

  // caller cotangents (d disp per level, d pose) of a forward-only call: the head pullback and
  // the pose gradient buffers the backward segments read, as the fused loss tail writes them
  int set_cotangents(const float* const* d_disp, const float* d_pose_in, hipStream_t st) {
    int li = 0;
    for (auto& d : br)
      if (d.head >= 0) {
        MD2_TRY(sigmoid_cotangent(d_disp ? d_disp[li] : nullptr, d.disp, d.d_head, (long)ND * 4 * d.h * d.w, st));
        ++li;
      }
    if (d_pose_in) MD2_HIP(hipMemcpyAsync(d_pose, d_pose_in, sizeof(float) * 12 * N, hipMemcpyDefault, st));
    else MD2_HIP(hipMemsetAsync(d_pose, 0, sizeof(float) * 12 * N, st));
    return MD2_OK;
  }

  const float* cur_x = nullptr;
  // 0: the last forward was forward-only (the backward needs md2_model_set_cotangents first);
  // 1: the backward's cotangents are in place (forward_loss, or set_cotangents after forward)
  int cot_ready = 0;
  std::string dbg_name;   // storage behind model_debug_tensor's name
};

// ---------------------------------------------------------------------------------------------
// DepthDecoder(; scale_levels) (src/depth_decoder.jl:26-50): at most 5 levels in 1:5 (the
// reference's own error); levels that do not strictly increase are MD2_ENOTSUP (the reference
// then builds empty branches: a duplicate head for a repeated level, a channel mismatch at run
// time for a decreasing one)
int check_scale_levels(const ArchCfg& a) {
  MD2_CHECK_ARG(a.nlevels >= 1 && a.nlevels <= MAX_SCALES,
                "`scale_levels` should be at most of length 5 and have values in [1, 5] range.");
  for (int i = 0; i < a.nlevels; ++i)
    MD2_CHECK_ARG(a.levels[i] >= 1 && a.levels[i] <= 5,
                  "`scale_levels` should be at most of length 5 and have values in [1, 5] range.");
  for (int i = 1; i < a.nlevels; ++i)
    if (a.levels[i] <= a.levels[i - 1]) {
      set_error("scale_levels must be strictly increasing (repeated / decreasing levels: not supported)");
      return MD2_ENOTSUP;
    }
  return MD2_OK;
}

int model_create(const ModelCfg& cfg, float* params, float* grads, Model** out) {
  MD2_CHECK_ARG(out != nullptr && params != nullptr && grads != nullptr, "model_create args");
  MD2_CHECK_ARG(cfg.arch.arch == 18 || cfg.arch.arch == 34 || cfg.arch.arch == 50, "arch 18/34/50");
  MD2_CHECK_ARG(cfg.arch.in_ch == 1 || cfg.arch.in_ch == 3, "in_channels 1 or 3");
  MD2_CHECK_ARG(cfg.N >= 1 && cfg.W % 32 == 0 && cfg.H % 32 == 0 && cfg.W >= 64 && cfg.H >= 64,
                "width/height must be multiples of 32 (>= 64)");
  // TrainCache(target_id, source_ids) over triplets (src/Monodepth.jl:49-60): any frames of 3
  MD2_CHECK_ARG(cfg.target >= 0 && cfg.target < 3 && cfg.src0 >= 0 && cfg.src0 < 3 && cfg.src1 >= 0 &&
                    cfg.src1 < 3, "target / source ids must be frames of the triplet (1-based 1:3)");
  MD2_TRY(check_scale_levels(cfg.arch));
  MD2_CHECK_ARG(cfg.arch.emb == 0 || (cfg.arch.emb > 0 && cfg.arch.emb % 2 == 1),
                "embedding_levels must be 0 or 2L+1 (x, sin, cos of L octaves)");
  if (cfg.arch.emb > 0) {
    MD2_CHECK_ARG(cfg.num_bins >= 1, "num_bins >= 1");
    if (cfg.N != 1) {
      // src/training.jl:42-56 with planes merged into the batch is shape-consistent only for one
      // sample: Project / grid_sample broadcast the N = 1 poses and frames
      set_error("MPI mode (embedding_levels > 0) trains one sample per step (batch must be 1)");
      return MD2_ENOTSUP;
    }
  }
  Model* m = new Model();
  m->cfg = cfg;
  m->params = params;
  m->grads = grads;
  int rc = m->build();
  if (rc) {
    delete m;
    return rc;
  }
  *out = m;
  return MD2_OK;
}

void model_destroy(Model* m) { delete m; }

int model_forward_loss(Model* m, const float* x, const float* automask, float* loss, float* terms,
                       hipStream_t st) {
  MD2_CHECK_ARG(m && x, "model/x");
  MD2_TRY(m->adam_join(st));   // pending per-segment updates (model_adam_segment)
  m->cur_x = x;
  m->cot_ready = 1;
  return m->forward_loss(x, automask, loss, terms, st);
}

int model_forward(Model* m, const float* x, hipStream_t st) {
  MD2_CHECK_ARG(m && x, "model/x");
  MD2_TRY(m->adam_join(st));   // pending per-segment updates (model_adam_segment)
  m->cur_x = x;
  m->cot_ready = 0;
  return m->forward(x, st);
}

int model_set_cotangents(Model* m, const float* const* d_disp, const float* d_pose, hipStream_t st) {
  MD2_CHECK_ARG(m, "model");
  if (!m->cur_x) {
    set_error("set_cotangents: no pending forward (none yet, or eval_disparity ran since)");
    return MD2_ESTATE;
  }
  MD2_TRY(m->set_cotangents(d_disp, d_pose, st));
  m->cot_ready = 1;
  return MD2_OK;
}

int model_num_segments(Model* m) { return m ? 6 : 0; }

// ---------------------------------------------------------------------------------------------
// Graph-captured train step (forward + loss + every backward segment + ADAM + weight repack as
// ONE hipGraph): the ~320 launches of a step replay without per-launch host work.  Captured on
// the executor's own stream on first use (and again when adam_m / adam_v / lr / the automask
// input change); each call copies x (and auto_loss) into the executor's input buffers, replays
// on `st`, and copies the loss out.  ADAM's step count lives on the device (adam_prep), re-set
// only when the caller's `step` is not the one the graph expects next.
static int capture_step(Model* m, bool with_auto, float* adam_m, float* adam_v, float lr) {
  auto& g = m->g;
  if (g.exec) {
    MD2_HIP(hipGraphExecDestroy(g.exec));
    g.exec = nullptr;
  }
  if (!g.st) MD2_HIP(hipStreamCreateWithFlags(&g.st, hipStreamNonBlocking));
  if (!g.x) {
    const long xn = (long)m->N * 3 * m->cfg.arch.in_ch * m->cfg.H * m->cfg.W;
    MD2_TRY(m->alloc(&g.x, xn));
    MD2_TRY(m->alloc(&g.autoloss, (long)m->N * m->cfg.H * m->cfg.W));
    MD2_TRY(m->alloc(&g.loss, 4));
    MD2_TRY(m->alloc(&g.bc, 4));
    float* q;
    MD2_TRY(m->alloc(&q, 4));
    g.step = (int*)q;
  }
  MD2_HIP(hipStreamBeginCapture(g.st, hipStreamCaptureModeThreadLocal));
  auto body = [&]() -> int {
    m->cur_x = g.x;
    m->cot_ready = 1;
    MD2_TRY(m->forward_loss(g.x, with_auto ? g.autoloss : nullptr, g.loss, nullptr, g.st));
    for (int k = 0; k < model_num_segments(m); ++k) MD2_TRY(model_backward_segment(m, k, nullptr, nullptr, g.st));
    MD2_TRY(adam_prep(g.step, g.bc, 0.9f, 0.999f, g.st));
    MD2_TRY(adam_step_dev(m->params, m->grads, adam_m, adam_v, m->spec.total, lr, 0.9f, 0.999f, 1e-8f,
                          g.bc, 1.f, g.st));
    return m->repack(g.st);
  };
  const int rc = body();
  hipGraph_t graph = nullptr;
  const hipError_t e = hipStreamEndCapture(g.st, &graph);
  if (rc) {
    if (graph) (void)hipGraphDestroy(graph);
    return rc;
  }
  MD2_HIP(e);
  const hipError_t ei = hipGraphInstantiate(&g.exec, graph, nullptr, nullptr, 0);
  (void)hipGraphDestroy(graph);
  MD2_HIP(ei);
  g.adam_m = adam_m;
  g.adam_v = adam_v;
  g.lr = lr;
  g.with_auto = with_auto ? 1 : 0;
  g.next_step = -1;
  return MD2_OK;
}

int model_train_step_graph(Model* m, const float* x, const float* auto_loss, float* adam_m,
                           float* adam_v, float lr, int step, float* loss, hipStream_t st) {
  MD2_CHECK_ARG(m && x && adam_m && adam_v && loss && step >= 1, "train_step_graph args");
  auto& g = m->g;
  const bool with_auto = auto_loss != nullptr;
  if (m->prof) {   // per-launch HIP events cannot live in a replayed graph: eager step
    MD2_TRY(model_forward_loss(m, x, auto_loss, loss, nullptr, st));
    for (int k = 0; k < model_num_segments(m); ++k) MD2_TRY(model_backward_segment(m, k, nullptr, nullptr, st));
    return model_adam(m, adam_m, adam_v, lr, 0.9f, 0.999f, 1e-8f, step, 1.f, st);
  }
  // the replay reads and writes params, adam_m / adam_v and the packed weights: order it after
  // pending per-segment updates (outside the capture: the event lives outside the graph)
  MD2_TRY(m->adam_join(st));
  if (!g.exec || g.adam_m != adam_m || g.adam_v != adam_v || g.lr != lr || g.with_auto != (int)with_auto)
    MD2_TRY(capture_step(m, with_auto, adam_m, adam_v, lr));
  const size_t xb = sizeof(float) * (size_t)m->N * 3 * m->cfg.arch.in_ch * m->cfg.H * m->cfg.W;
  if (x != g.x) MD2_HIP(hipMemcpyAsync(g.x, x, xb, hipMemcpyDeviceToDevice, st));
  if (with_auto)
    MD2_HIP(hipMemcpyAsync(g.autoloss, auto_loss, sizeof(float) * (size_t)m->N * m->cfg.H * m->cfg.W,
                           hipMemcpyDeviceToDevice, st));
  if (step != g.next_step) MD2_TRY(set_device_int(g.step, step - 1, st));
  MD2_HIP(hipGraphLaunch(g.exec, st));
  MD2_HIP(hipMemcpyAsync(loss, g.loss, sizeof(float), hipMemcpyDeviceToDevice, st));
  m->cur_x = g.x;
  m->cot_ready = 1;
  g.next_step = step + 1;
  return MD2_OK;
}



int model_backward_segment(Model* m, int k, long* off, long* len, hipStream_t st) {
  MD2_CHECK_ARG(m, "model");
  if (!m->cur_x) {
    set_error("backward_segment: no pending forward_loss (none yet, or eval_disparity ran since)");
    return MD2_ESTATE;
  }
  if (!m->cot_ready) {
    set_error("backward_segment: forward-only call without cotangents (md2_model_set_cotangents)");
    return MD2_ESTATE;
  }
  MD2_CHECK_ARG(k >= 0 && k < 6, "segment index");
  long b = 0, e = 0;
  switch (k) {
    case 0: MD2_TRY(m->seg_decoder(st)); break;
    case 1: MD2_TRY(m->seg_stage(3, st)); break;
    case 2: MD2_TRY(m->seg_stage(2, st)); break;
    case 3: MD2_TRY(m->seg_stage(1, st)); break;
    case 4: MD2_TRY(m->seg_stage(0, st)); break;
    default: MD2_TRY(m->seg_stem(st)); break;
  }
  m->segment_range(k, b, e);
  if (off) *off = b;
  if (len) *len = e - b;
  return MD2_OK;
}

int model_adam(Model* m, float* adam_m, float* adam_v, float lr, float b1, float b2, float eps,
               int step, float grad_scale, hipStream_t st) {
  MD2_CHECK_ARG(m && adam_m && adam_v && step >= 1, "adam args");
  MD2_TRY(m->adam_join(st));   // pending per-segment updates (model_adam_segment)
  const double bc1 = 1.0 - std::pow((double)b1, step), bc2 = 1.0 - std::pow((double)b2, step);
  MD2_TRY(adam_step(m->params, m->grads, adam_m, adam_v, m->spec.total, lr, b1, b2, eps, (float)bc1,
                    (float)bc2, grad_scale, st));
  return m->repack(st);
}

int model_adam_segment(Model* m, int k, float* adam_m, float* adam_v, float lr, float b1, float b2,
                       float eps, int step, float grad_scale, hipStream_t st) {
  MD2_CHECK_ARG(m && adam_m && adam_v && step >= 1, "adam_segment args");
  MD2_CHECK_ARG(k >= 0 && k < 6, "segment index");
  const double bc1 = 1.0 - std::pow((double)b1, step), bc2 = 1.0 - std::pow((double)b2, step);
  return m->adam_segment(k, adam_m, adam_v, lr, b1, b2, eps, (float)bc1, (float)bc2, grad_scale, st);
}

int model_adam_join(Model* m, hipStream_t st) {
  MD2_CHECK_ARG(m, "model");
  return m->adam_join(st);
}

bool model_segment_update_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("MD2_SEG_UPDATE");
    return e && e[0] == '1';
  }();
  return on;
}

int model_repack(Model* m, hipStream_t st) {
  MD2_CHECK_ARG(m, "model");
  MD2_TRY(m->adam_join(st));   // pending per-segment updates write the same packed weights
  return m->repack(st);
}

int model_debug_tensor(Model* m, int index, const char** name, const void** ptr, int* dims) {
  MD2_CHECK_ARG(m && ptr && dims, "debug_tensor arguments");
  struct T {
    std::string name;
    const void* p;
    int n, c, h, w, u8;
  };
  const int B = m->B, N = m->N;
  std::vector<T> ts;
  ts.push_back({"stem.y", m->y0, B, 64, m->H0, m->W0, 0});
  ts.push_back({"stem.out", m->f0, B, 64, m->H0, m->W0, 0});
  ts.push_back({"maxpool.out", m->mp, B, 64, m->Hm, m->Wm, 0});
  ts.push_back({"maxpool.arg", m->mp_arg, B, 64, m->Hm, m->Wm, 1});
  for (size_t si = 0; si < m->stages.size(); ++si)
    for (size_t bi = 0; bi < m->stages[si].size(); ++bi) {
      auto& b = m->stages[si][bi];
      const std::string pre = "layer" + std::to_string(si + 1) + "." + std::to_string(bi);
      for (size_t k = 0; k < b.st.size(); ++k) {
        auto& e = b.st[k];
        const bool last = k + 1 == b.st.size();
        ts.push_back({pre + ".conv" + std::to_string(k + 1) + ".y", e.y, B, e.conv.p.cout,
                      e.conv.s.Ho, e.conv.s.Wo, 0});
        ts.push_back({pre + (last ? std::string(".out") : ".relu" + std::to_string(k + 1)), e.a, B,
                      e.conv.p.cout, e.conv.s.Ho, e.conv.s.Wo, 0});
      }
      if (b.down) ts.push_back({pre + ".down.y", b.yd, B, b.C, b.H, b.W, 0});
      ts.push_back({pre + ".d_out", b.d_out, B, b.C, b.H, b.W, 0});
    }
  const int h4 = m->featH[4], w4 = m->featW[4];
  ts.push_back({"pose.sq", m->sqo, B, 256, h4, w4, 0});
  ts.push_back({"pose.conv1", m->pc1, 2 * N, 256, h4, w4, 0});
  ts.push_back({"pose.conv2", m->pc2, 2 * N, 256, h4, w4, 0});
  for (int f = 0; f < 4; ++f)
    if (m->d_skip[f])
      ts.push_back({"d_skip" + std::to_string(f), m->d_skip[f], N, m->featC[f], m->featH[f],
                    m->featW[f], 0});
  // DepthDecoder intermediates of the last forward (forward-accuracy bisection, tools/forward_bisect.py)
  for (auto& d : m->br) {
    const std::string pre = "depth.branch" + std::to_string(d.b.bid);
    ts.push_back({pre + ".c1", d.o1, m->ND, d.b.cout, d.h, d.w, 0});
    ts.push_back({pre + ".up", d.up, m->ND, d.b.cout, 2 * d.h, 2 * d.w, 0});
    ts.push_back({pre + ".c2", d.o2, m->ND, d.b.cout, 2 * d.h, 2 * d.w, 0});
  }
  ts.push_back({"d_mp", m->d_mp, B, 64, m->Hm, m->Wm, 0});
  ts.push_back({"d_f0", m->d_f0, B, 64, m->H0, m->W0, 0});
  if (index < 0 || index >= (int)ts.size()) {
    set_error("debug_tensor: index out of range");
    return MD2_EINVAL;
  }
  m->dbg_name = ts[index].name;
  if (name) *name = m->dbg_name.c_str();
  *ptr = ts[index].p;
  dims[0] = ts[index].n;
  dims[1] = ts[index].c;
  dims[2] = ts[index].h;
  dims[3] = ts[index].w;
  dims[4] = ts[index].u8;
  return MD2_OK;
}

int model_outputs(Model* m, const float** disp, int* dw, int* dh, const float** pose) {
  MD2_CHECK_ARG(m, "model");
  int li = 0;
  for (auto& d : m->br)
    if (d.head >= 0) {
      if (disp) disp[li] = d.disp;
      if (dw) dw[li] = 2 * d.w;
      if (dh) dh[li] = 2 * d.h;
      ++li;
    }
  if (pose) *pose = m->pose;
  return MD2_OK;
}

int model_features(Model* m, const float** feat, int* c, int* h, int* w) {
  MD2_CHECK_ARG(m, "model");
  for (int k = 0; k < 5; ++k) {
    feat[k] = m->feat[k];
    c[k] = m->featC[k];
    h[k] = m->featH[k];
    w[k] = m->featW[k];
  }
  return MD2_OK;
}

int model_eval_disparity(Model* m, const float* x, int n, float** disp_out, hipStream_t st) {
  MD2_CHECK_ARG(m && x && n >= 1 && n <= m->N, "eval_disparity: 1 <= n <= batch");
  MD2_TRY(m->adam_join(st));   // pending per-segment updates (model_adam_segment)
  if (m->E > 0) {
    // src/model.jl:63 runs the decoder on the bare encoder features, which an
    // embedding_levels > 0 DepthDecoder cannot take (defect D4)
    set_error("eval_disparity: the MPI-mode DepthDecoder (embedding_levels > 0) has no mono input");
    return MD2_ENOTSUP;
  }
  // inference reuses the executor's activation buffers: a pending train forward is gone, and a
  // backward after this must fail instead of differentiating the eval batch
  m->cur_x = nullptr;
  TensorIn in = Model::tin(x, m->cfg.arch.in_ch, (long)m->cfg.H * m->cfg.W);
  MD2_TRY(m->encoder_fwd(in, n, st));
  MD2_TRY(m->decoder_fwd(n, 0, st));
  if (disp_out) {
    int li = 0;
    for (auto& d : m->br)
      if (d.head >= 0) disp_out[li++] = d.disp;
  }
  return MD2_OK;
}

int model_set_profiling(Model* m, int on) {
  MD2_CHECK_ARG(m, "model");
  m->prof = on != 0;
  m->recs.clear();
  m->evi = 0;
  return MD2_OK;
}

int model_profile_records(Model* m, int max, double* ms, double* work, int* cat, char* tags,
                          int tag_len, int* count) {
  MD2_CHECK_ARG(m && ms && work && cat && count && max >= 0, "profile_records args");
  return m->profile_records(max, ms, work, cat, tags, tag_len, count);
}

int model_profile_read(Model* m, double* out, int ncat) {
  MD2_CHECK_ARG(m && out && ncat > 0, "profile_read args");
  return m->profile_read(out, ncat);
}

// Flux-layout flat vectors (src/model.jl @functor order, conv weights as true convolutions) <->
// the library's flat vectors: a copy with every conv weight's taps reversed (md2_model_*_params)
static int flux_flip_copy(const Model* m, const float* src, float* dst, hipStream_t st) {
  MD2_CHECK_ARG(src && dst && src != dst, "params: distinct source and destination required");
  MD2_HIP(hipMemcpyAsync(dst, src, sizeof(float) * (size_t)m->spec.total, hipMemcpyDeviceToDevice, st));
  for (const ParamEntry& e : m->spec.table)
    if (e.ndim == 4 && e.shape[2] * e.shape[3] > 1)
      MD2_TRY(flip_taps(src + e.offset, dst + e.offset, (long)e.shape[0] * e.shape[1], e.shape[2],
                        e.shape[3], st));
  return MD2_OK;
}

int model_set_params_flux(Model* m, const float* flux, hipStream_t st) {
  MD2_CHECK_ARG(m, "model");
  MD2_TRY(m->adam_join(st));   // pending per-segment updates (model_adam_segment)
  MD2_TRY(flux_flip_copy(m, flux, m->params, st));
  return m->repack(st);
}

int model_get_params_flux(Model* m, float* flux, hipStream_t st) {
  MD2_CHECK_ARG(m, "model");
  MD2_TRY(m->adam_join(st));   // pending per-segment updates (model_adam_segment)
  return flux_flip_copy(m, m->params, flux, st);
}

int model_get_grads_flux(Model* m, float* flux, hipStream_t st) {
  MD2_CHECK_ARG(m, "model");
  MD2_TRY(m->adam_join(st));   // a DP per-segment update is ordered after its bucket's all-reduce
  return flux_flip_copy(m, m->grads, flux, st);
}

// train_loss pullback with an upstream cotangent: the fused loss tail formed d loss / d (disp,
// pose) for dloss = 1 during the forward; scale them before backward segment 0
int model_scale_loss_cotangent(Model* m, float dloss, hipStream_t st) {
  MD2_CHECK_ARG(m && m->cur_x && m->cot_ready, "loss cotangent before forward_loss");
  if (dloss == 1.f) return MD2_OK;
  for (auto& d : m->br)
    if (d.head >= 0) MD2_TRY(scale_inplace(d.d_head, (long)m->ND * 4 * d.h * d.w, dloss, st));
  return scale_inplace(m->d_pose, 2L * m->N * 6, dloss, st);
}

int model_set_bins(Model* m, const float* bins, hipStream_t st) {
  MD2_CHECK_ARG(m && bins, "set_bins args");
  if (m->E == 0) {
    set_error("set_bins: the model is not in MPI mode (embedding_levels = 0)");
    return MD2_ESTATE;
  }
  MD2_HIP(hipMemcpyAsync(m->bins, bins, sizeof(float) * m->N * m->NP, hipMemcpyDefault, st));
  return MD2_OK;
}

long model_param_count(Model* m) { return m ? m->spec.total : 0; }
float* model_grads(Model* m) { return m ? m->grads : nullptr; }
size_t model_device_bytes(Model* m) { return m ? m->bytes : 0; }

}  // namespace md2
