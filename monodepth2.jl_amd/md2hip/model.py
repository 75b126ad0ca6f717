"""Host mirror of the reference's model API over libmd2hip.so.

Reference (Julia): ``ResidualNetwork(18; in_channels, classes=nothing)`` (ResNet.jl),
``DepthDecoder(; encoder_channels, scale_levels, embedding_levels)`` (src/depth_decoder.jl:26),
``PoseDecoder(encoder_out_channels)`` (src/pose_decoder.jl:13), ``Model(encoder, depth_decoder,
pose_decoder)`` (src/model.jl:24-29), ``train_loss`` (src/training.jl:21), ``eval_disparity``
(src/model.jl:63) and the ``gradient(θ)`` / ``update!(ADAM)`` loop (scripts/script.jl:84-86).

The Julia objects are size-agnostic; the HIP executor is planned for one (batch, height, width,
TrainCache, Params) and cached per such key.  Parameters live in ONE flat fp32 device vector
(``Model.flat``) in the order of ``md2_arch_param_info``; ``Model.parameters()`` are views."""
from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import _lib
from ._lib import ModelCfg, check, lib, ptr, stream_of
from .loss import Params, TrainCache, depth10k_intrinsics, loss_tail


class ResidualNetwork:
    """``ResidualNetwork(depth; in_channels, classes=nothing)`` (ext ResNet.jl, torchvision
    topology).  ``stages`` gives the channel list used by the decoders (scripts/script.jl:78)."""

    def __init__(self, depth: int = 18, *, in_channels: int = 3, classes=None):
        if depth not in (18, 34, 50):
            raise ValueError("ResidualNetwork depth must be 18, 34 or 50")
        if classes is not None:
            raise NotImplementedError("the classification head is not part of the depth model")
        self.depth = depth
        self.in_channels = in_channels
        self.stages = (64, 64, 128, 256, 512) if depth in (18, 34) else (64, 256, 512, 1024, 2048)


ResNet = ResidualNetwork


class DepthDecoder:
    """``DepthDecoder(; encoder_channels, scale_levels, embedding_levels=21)``.  embedding_levels
    = 0 is the mono decoder of the measured step; 2L+1 (the reference's default 21) is the MPI-mode
    decoder whose inputs carry the plane embedding (src/model.jl:31-55, trained at batch 1)."""

    def __init__(self, *, encoder_channels, scale_levels, embedding_levels: int = 21):
        levels = list(scale_levels)
        if len(levels) > 5 or min(levels) < 1 or max(levels) > 5:   # src/depth_decoder.jl:27-29
            raise ValueError("`scale_levels` should be at most of length 5 and have values in [1, 5] range.")
        if embedding_levels < 0 or (embedding_levels and embedding_levels % 2 != 1):
            raise ValueError("embedding_levels must be 0 or 2L+1 (x, sin, cos of L octaves; src/model.jl:4-15)")
        if any(b <= a for a, b in zip(levels, levels[1:])):
            # the reference builds an empty branch here: a duplicate head for a repeated level, a
            # channel mismatch at run time for a decreasing one (library: MD2_ENOTSUP)
            raise NotImplementedError("scale_levels must be strictly increasing")
        self.encoder_channels = tuple(encoder_channels)
        self.scale_levels = tuple(levels)
        self.embedding_levels = embedding_levels


class PoseDecoder:
    """``PoseDecoder(encoder_out_channels)``."""

    def __init__(self, encoder_out_channels: int):
        self.encoder_out_channels = encoder_out_channels


@dataclass
class Pose:
    """``Pose{rvec (3,N), tvec (3,1,N)}`` (src/pose_decoder.jl:1-5) as [N,3] tensors."""
    rvec: object
    tvec: object


def _cfg(arch, in_ch, levels, batch=1, width=64, height=64, cache: Optional[TrainCache] = None,
         params: Optional[Params] = None, embedding_levels: int = 0, num_bins: int = 32) -> ModelCfg:
    c = ModelCfg()
    c.arch, c.in_channels, c.batch, c.width, c.height = arch, in_ch, batch, width, height
    c.embedding_levels, c.num_bins = embedding_levels, num_bins
    c.n_levels = len(levels)
    for i, l in enumerate(levels):
        c.scale_levels[i] = l
    if cache is not None:
        K = np.asarray(cache.K, dtype=np.float64).reshape(-1)
        iK = np.asarray(cache.invK, dtype=np.float64).reshape(-1)
        for i in range(9):
            c.K[i], c.invK[i] = float(K[i]), float(iK[i])
        for i, s in enumerate(cache.scales):
            c.scales[i] = float(s)
        ids = (cache.target_id, *cache.source_ids)
        if len(cache.source_ids) != 2:
            raise NotImplementedError("the HIP model takes exactly two source frames (TrainCache.source_ids)")
        if any(not 1 <= i <= 3 for i in ids):
            raise ValueError("target_id / source_ids must be frames of the triplet (1:3)")
        if len(cache.scales) != len(levels):
            raise ValueError("TrainCache.scales must have one entry per DepthDecoder scale level")
        c.target, c.src0, c.src1 = cache.target_id - 1, cache.source_ids[0] - 1, cache.source_ids[1] - 1
    if params is not None:
        c.min_depth, c.max_depth = params.min_depth, params.max_depth
        c.disparity_smoothness = params.disparity_smoothness
        c.automasking = int(params.automasking)
    return c


def param_table(arch=18, in_channels=3, scale_levels=(2, 3, 4, 5), embedding_levels=0):
    """[(name, shape, offset)] of the flat parameter vector (host-only library query)."""
    cfg = _cfg(arch, in_channels, scale_levels, embedding_levels=embedding_levels)
    ne, nel = C.c_longlong(), C.c_longlong()
    check(lib().md2_arch_param_count(C.byref(cfg), C.byref(ne), C.byref(nel)), "md2_arch_param_count")
    out = []
    name = C.create_string_buffer(128)
    nd, off = C.c_int(), C.c_longlong()
    shp = (C.c_int * 4)()
    for i in range(ne.value):
        check(lib().md2_arch_param_info(C.byref(cfg), i, name, 128, C.byref(nd), shp, C.byref(off)),
              "md2_arch_param_info")
        out.append((name.value.decode(), tuple(shp[j] for j in range(nd.value)), off.value))
    return out, nel.value


def flux_init(table, total, seed=42):
    """Flux defaults (glorot_uniform conv weights, zero bias, BN gamma=1 beta=0) on the host,
    float64 -> the caller casts.  Identical to oracle.init_params for the same seed."""
    import torch
    g = torch.Generator().manual_seed(seed)
    flat = torch.empty(total, dtype=torch.float64)
    for name, shape, off in table:
        n = int(np.prod(shape))
        if name.endswith(".weight"):
            cout, cin, kh, kw = shape
            lim = math.sqrt(6.0 / (cin * kh * kw + cout * kh * kw))
            v = (torch.rand(shape, generator=g, dtype=torch.float64) * 2 - 1) * lim
        elif name.endswith(".gamma"):
            v = torch.ones(n, dtype=torch.float64)
        else:
            v = torch.zeros(n, dtype=torch.float64)
        flat[off:off + n] = v.reshape(-1)
    return flat


class _Executor:
    """One libmd2hip model instance (activations/workspace) for a fixed problem size."""

    def __init__(self, model: "Model", batch, height, width, cache: TrainCache, params: Params,
                 num_bins: int = 32):
        self.model = model
        self.batch, self.height, self.width = batch, height, width
        self.emb = model.depth_decoder.embedding_levels
        self.num_bins = num_bins if self.emb else 1
        cfg = _cfg(model.encoder.depth, model.encoder.in_channels, model.depth_decoder.scale_levels,
                   batch, width, height, cache, params, self.emb, num_bins)
        h = C.c_void_p()
        check(lib().md2_model_create(C.byref(cfg), ptr(model.flat), ptr(model.grad), C.byref(h)),
              "md2_model_create")
        self.handle = h
        self.nseg = lib().md2_model_num_segments(h)
        self.automask = params.automasking
        self.forwarded = False              # a forward_loss ran since the last eval_disparity here
        self.pending = False                # ... and its backward has not run yet
        self.version = -1                   # Model.version its packed conv weights reflect
        self.sync()

    def sync(self):
        """Re-pack this executor's conv weights if the flat parameters changed since its last
        pack (ADAM through another executor, load_flat, direct writes via Model.touch())."""
        if self.version != self.model.version:
            check(lib().md2_model_repack(self.handle, stream_of(self.model.device)), "md2_model_repack")
            self.version = self.model.version

    def __del__(self):
        try:
            if self.handle:
                lib().md2_model_destroy(self.handle)
        except Exception:
            pass

    def device_bytes(self):
        return lib().md2_model_device_bytes(self.handle)

    PROF_CATS = ("conv3x3_encoder", "conv_other", "photometric")

    def set_profiling(self, on: bool):
        check(lib().md2_model_set_profiling(self.handle, int(on)), "md2_model_set_profiling")

    def profile_read(self):
        """{category: (ms, work, launches)} from HIP events recorded on the model's stream."""
        n = len(self.PROF_CATS)
        buf = (C.c_double * (3 * n))()
        check(lib().md2_model_profile_read(self.handle, buf, n), "md2_model_profile_read")
        return {c: (buf[3 * i], buf[3 * i + 1], int(buf[3 * i + 2])) for i, c in enumerate(self.PROF_CATS)}

    def profile_records(self, max_records=4096):
        """[(tag, category, ms, work)] per profiled launch (per-layer table), then clears."""
        ms = (C.c_double * max_records)()
        work = (C.c_double * max_records)()
        cat = (C.c_int * max_records)()
        tag_len = 64
        tags = C.create_string_buffer(max_records * tag_len)
        count = C.c_int(0)
        check(lib().md2_model_profile_records(self.handle, max_records, ms, work, cat, tags, tag_len,
                                              C.byref(count)), "md2_model_profile_records")
        raw = tags.raw
        return [(raw[i * tag_len:(i + 1) * tag_len].split(b"\0", 1)[0].decode(),
                 self.PROF_CATS[cat[i]] if cat[i] < len(self.PROF_CATS) else str(cat[i]), ms[i], work[i])
                for i in range(count.value)]

    def set_bins(self, bins):
        """MPI mode: the disparity bins [batch, num_bins] of the next forwards (the reference's
        ``uniformly_sample_disparity_from_linspace_bins`` draw, src/model.jl:17-21)."""
        import torch
        b = bins.to(self.model.device, torch.float32).contiguous()
        if tuple(b.shape) != (self.batch, self.num_bins):
            raise ValueError(f"bins must be [{self.batch}, {self.num_bins}]")
        check(lib().md2_model_set_disparity_bins(self.handle, ptr(b), stream_of(self.model.device)),
              "md2_model_set_disparity_bins")
        self._bins = b                       # the copy is async: keep the source alive

    def forward_loss(self, x, auto_loss=None, loss=None, terms=None):
        import torch
        loss = loss if loss is not None else torch.empty(1, dtype=torch.float32, device=x.device)
        self.sync()
        am = auto_loss.contiguous() if (self.automask and auto_loss is not None) else None
        check(lib().md2_model_forward_loss(self.handle, ptr(x), ptr(am), ptr(loss), ptr(terms),
                                           stream_of(x.device)), "md2_model_forward_loss")
        self.forwarded = self.pending = True
        return loss

    def forward(self, x):
        """``(m)(x, source_ids, target_id)`` alone (md2_model_forward): encoder, DepthDecoder and
        PoseDecoder, no loss tail.  A backward after it needs ``set_cotangents``."""
        self.sync()
        check(lib().md2_model_forward(self.handle, ptr(x), None, None, stream_of(x.device)),
              "md2_model_forward")
        self.forwarded = self.pending = True
        self.cotangents = False

    def set_cotangents(self, d_disps=None, d_pose=None):
        """The cotangents of the last forward's outputs (md2_model_set_cotangents): d_disps[l] like
        the level-l disparities (None: zero), d_pose like the [2N, 6] poses (None: zero)."""
        import torch
        keep = []
        arr = (C.c_void_p * 5)()
        for i, d in enumerate(d_disps or []):
            if d is not None:
                d = d.to(self.model.device, torch.float32).contiguous()
                keep.append(d)
                arr[i] = d.data_ptr()
        dp = None if d_pose is None else d_pose.to(self.model.device, torch.float32).contiguous()
        check(lib().md2_model_set_cotangents(self.handle, arr, ptr(dp), stream_of(self.model.device)),
              "md2_model_set_cotangents")
        self._cot_keep = (keep, dp)           # the copies are async: keep the sources alive
        self.cotangents = True

    def train_step_graph(self, x, opt: "ADAM", auto_loss=None, loss=None):
        """One full step (forward, loss, backward, Flux ADAM with opt's state) replayed as a
        captured hipGraph (md2_model_train_step_graph): the same kernels in the same order as
        forward_loss + backward + ADAM.update, without per-launch host work.  Returns the loss."""
        import torch
        if tuple(opt.beta) != (0.9, 0.999) or opt.eps != 1e-8:
            raise NotImplementedError("the captured step uses ADAM's defaults beta=(0.9, 0.999), eps=1e-8")
        loss = loss if loss is not None else torch.empty(1, dtype=torch.float32, device=x.device)
        self.sync()
        if opt.m is None:
            opt.m = torch.zeros_like(self.model.flat)
            opt.v = torch.zeros_like(self.model.flat)
        am = auto_loss.contiguous() if (self.automask and auto_loss is not None) else None
        opt.t += 1
        check(lib().md2_model_train_step_graph(self.handle, ptr(x), ptr(am), ptr(opt.m), ptr(opt.v), opt.eta,
                                               opt.t, ptr(loss), stream_of(x.device)),
              "md2_model_train_step_graph")
        self.forwarded = True
        self.model._last = self
        self.model.touch()
        self.version = self.model.version
        return loss

    def backward_segment(self, k):
        off, ln = C.c_longlong(), C.c_longlong()
        check(lib().md2_model_backward_segment(self.handle, k, C.byref(off), C.byref(ln),
                                               stream_of(self.model.device)), "md2_model_backward_segment")
        return off.value, ln.value

    def backward(self):
        r = [self.backward_segment(k) for k in range(self.nseg)]
        self.pending = False
        return r

    def outputs(self):
        """(disparities [N,1,h,w] views, poses [2N,6] view) of the last forward (device memory
        owned by the executor; clone to keep)."""
        import torch
        nl = len(self.model.depth_decoder.scale_levels)
        dptr = (C.c_void_p * 5)()
        w = (C.c_int * 5)()
        h = (C.c_int * 5)()
        pp = C.c_void_p()
        check(lib().md2_model_outputs(self.handle, dptr, w, h, C.byref(pp)), "md2_model_outputs")
        disps = [_wrap(dptr[i], (self.batch * self.num_bins, 1, h[i], w[i]), self.model.device)
                 for i in range(nl)]
        pose = _wrap(pp.value, (2 * self.batch, 6), self.model.device)
        return disps, pose

    def debug_tensors(self):
        """{name: copy} of the library's internal buffers of the last forward/backward (see
        md2_model_debug_tensor; parity diagnostics).  Images in frame-major encoder order."""
        import torch
        out = {}
        dims = (C.c_int * 5)()
        p = C.c_void_p()
        nm = C.c_char_p()
        i = 0
        while lib().md2_model_debug_tensor(self.handle, i, C.byref(nm), C.byref(p), dims) == 0:
            shape = tuple(dims[:4])
            out[nm.value.decode()] = _wrap(p.value, shape, self.model.device,
                                           torch.uint8 if dims[4] else torch.float32)
            i += 1
        return out


def _wrap(p, shape, device, dtype=None):
    """Copy library-owned device memory into a fresh torch tensor (md2_memcpy_d2d)."""
    import torch
    dtype = dtype or torch.float32
    n = int(np.prod(shape))
    out = torch.empty(shape, dtype=dtype, device=device)
    check(lib().md2_memcpy_d2d(ptr(out), C.c_void_p(p), n * out.element_size(), stream_of(device)),
          "md2_memcpy_d2d")
    return out


class Model:
    """``Model(encoder, depth_decoder, pose_decoder)`` (src/model.jl:24-29)."""

    def __init__(self, encoder: ResidualNetwork, depth_decoder: DepthDecoder,
                 pose_decoder: PoseDecoder, *, device="cuda", seed: int = 42):
        import torch
        if tuple(depth_decoder.encoder_channels) != tuple(encoder.stages):
            raise ValueError("DepthDecoder encoder_channels must equal encoder.stages")
        if pose_decoder.encoder_out_channels != encoder.stages[-1]:
            raise ValueError("PoseDecoder channels must equal encoder.stages[end]")
        self.encoder, self.depth_decoder, self.pose_decoder = encoder, depth_decoder, pose_decoder
        self.device = torch.device(device)
        self.table, self.numel = param_table(encoder.depth, encoder.in_channels, depth_decoder.scale_levels,
                                             depth_decoder.embedding_levels)
        self.flat = flux_init(self.table, self.numel, seed).to(self.device, torch.float32)
        self.grad = torch.zeros_like(self.flat)
        self._ex: Dict[tuple, _Executor] = {}
        self._last: Optional[_Executor] = None
        # bumped whenever the flat parameters change; every executor keeps its own packed copy of
        # the conv weights and re-packs lazily when it is behind (Model.executor / _Executor.sync)
        self.version = 0

    # -- parameters (Flux.params(model)) ----------------------------------------------------
    def parameters(self) -> Dict[str, object]:
        return {name: self.flat[off:off + int(np.prod(shape))].view(shape) for name, shape, off in self.table}

    def load_flat(self, flat):
        self.flat.copy_(flat.to(self.flat.device, self.flat.dtype))
        self.touch()

    def touch(self):
        """Declare that ``flat`` was modified in place (the executors re-pack before next use)."""
        self.version += 1

    def evict(self, batch=None):
        """Free the cached executors (all, or those of one batch size)."""
        for k in [k for k in self._ex if batch is None or k[0] == batch]:
            ex = self._ex.pop(k)
            if ex is self._last:
                self._last = None

    def executor(self, x_shape, cache: TrainCache, params: Params, num_bins: int = 32) -> _Executor:
        N, L, Cc, H, W = x_shape
        if L != 3 or Cc != self.encoder.in_channels:
            raise ValueError("x must be [N, 3, in_channels, H, W]")
        if (W, H) != tuple(params.target_size):
            raise ValueError("x size != Params.target_size")
        nb = num_bins if self.depth_decoder.embedding_levels else 1
        key = (N, H, W, tuple(np.asarray(cache.K).reshape(-1)), tuple(cache.scales), params.min_depth,
               params.max_depth, params.disparity_smoothness, params.automasking, nb)
        if key not in self._ex:
            self._ex[key] = _Executor(self, N, H, W, cache, params, nb)
        self._last = self._ex[key]
        self._last.sync()
        return self._last

    def eval_executor(self, N, H, W) -> _Executor:
        """An executor of batch >= N at (H, W) for eval_disparity (the loss configuration does not
        matter for inference) that holds no pending train forward -- inference overwrites the
        executor's activations, so an executor between train_loss and gradient() is never taken;
        a new one (default TrainCache/Params) only if none fits."""
        fits = [ex for k, ex in self._ex.items() if k[1] == H and k[2] == W and k[0] >= N
                and not ex.pending]
        if fits:
            ex = min(fits, key=lambda e: e.batch)
            ex.sync()
            return ex
        K, iK = depth10k_intrinsics(W, H)
        cache = TrainCache(K=K, invK=iK)
        params = Params(target_size=(W, H), batch_size=N, automasking=False)
        key = (N, H, W, tuple(np.asarray(cache.K).reshape(-1)), tuple(cache.scales), params.min_depth,
               params.max_depth, params.disparity_smoothness, params.automasking, 1)
        key = key + ("eval",) if key in self._ex else key          # that one has a pending forward
        ex = self._ex[key] = _Executor(self, N, H, W, cache, params)   # leaves _last (training) alone
        return ex

    def __call__(self, x, source_ids=(1, 3), target_id=2, cache: Optional[TrainCache] = None,
                 params: Optional[Params] = None, num_bins: int = 32, bins=None):
        """``(m::Model)(x, source_ids, target_id; num_bins=32)`` (src/model.jl:31-55): returns
        (disparities, [Pose, Pose]).  MPI mode (embedding_levels > 0): disparities of the
        N*num_bins plane images; ``bins`` [N, num_bins] (default: a fresh uniform draw, as the
        reference's CUDA.rand)."""
        N, L, Cc, H, W = x.shape
        if cache is None:
            K, iK = depth10k_intrinsics(W, H)
            cache = TrainCache(K=K, invK=iK, target_id=target_id, source_ids=tuple(source_ids))
        if params is None:
            params = Params(target_size=(W, H), batch_size=N, automasking=False)
        ex = self.executor(tuple(x.shape), cache, params, num_bins)
        if ex.emb:
            ex.set_bins(disparity_bins(N, num_bins, device=self.device) if bins is None else bins)
        ex.forward(x)                       # forward only (md2_model_forward): no loss tail
        disps, pose = ex.outputs()
        return disps, [Pose(pose[s * N:(s + 1) * N, 0:3], pose[s * N:(s + 1) * N, 3:6]) for s in range(2)]


def disparity_bins(batch: int, num_bins: int, u=None, device="cuda", near=1.0, far=0.001):
    """``uniformly_sample_disparity_from_linspace_bins(num_bins, batch_size)`` (src/model.jl:17-21):
    bins[n][p] = linspace(near, far, num_bins+1)[p] + u[n][p] * interval, u ~ U[0,1) (drawn here
    when not given -- the reference draws with CUDA.rand, defect D3) -> float32 [batch, num_bins]."""
    import torch
    if u is None:
        u = torch.rand(batch, num_bins, dtype=torch.float64)
    edges = torch.linspace(near, far, num_bins + 1, dtype=torch.float64)[:-1]
    interval = float(edges[1] - edges[0])
    return (edges.unsqueeze(0) + u.double().cpu() * interval).float().to(device).contiguous()


def train_loss(model: Model, x, auto_loss, cache: TrainCache, params: Params,
               do_visualization: bool = False, num_bins: int = 32, bins=None):
    """``train_loss(model, x, auto_loss, cache, params, do_visualization)`` (src/training.jl:21).
    Runs the forward and the fused loss-tail pullback; call ``gradient(model)`` for the rest of
    the backward.  Returns (loss, vis_disparity, vis_warped, vis_loss).  MPI mode (the model's
    DepthDecoder has embedding_levels > 0; batch 1): ``num_bins`` planes, ``bins`` [1, num_bins]
    (default: a fresh draw of md2hip.disparity_bins)."""
    ex = model.executor(tuple(x.shape), cache, params, num_bins)
    if ex.emb:
        ex.set_bins(disparity_bins(x.shape[0], num_bins, device=x.device) if bins is None else bins)
    loss = ex.forward_loss(x, auto_loss)
    if not do_visualization:
        return loss, None, None, None
    # training.jl:34-37,71-74: the last disparity, both warped sources and the per-pixel warp
    # loss of the last scale, on the host.  Recomputed from the model outputs by the loss-tail
    # kernels (forward only, after the step's own forward; the gradient state is untouched).
    disps, pose = ex.outputs()
    N, nb = x.shape[0], ex.num_bins
    poses = [(pose[s * N:(s + 1) * N, 0:3], pose[s * N:(s + 1) * N, 3:6]) for s in range(2)]
    xv = x.contiguous()
    if nb > 1:           # MPI: every plane against its sample's frames and poses
        xv = xv.repeat_interleave(nb, 0).contiguous()
        poses = [(r.repeat_interleave(nb, 0).contiguous(), t.repeat_interleave(nb, 0).contiguous())
                 for r, t in poses]
        if auto_loss is not None:
            auto_loss = auto_loss.repeat_interleave(nb, 0).contiguous()
    vis = loss_tail(disps, poses, xv, auto_loss, cache,
                    Params(target_size=params.target_size, batch_size=N * nb, min_depth=params.min_depth,
                           max_depth=params.max_depth, disparity_smoothness=params.disparity_smoothness,
                           automasking=params.automasking), grads=False, visualize=True)
    return (loss, disps[-1].cpu(), [w.cpu() for w in vis["vis_warped"].unbind(0)],
            vis["vis_loss"][-1].unsqueeze(1).cpu())


def gradient(model: Model, dloss: float = 1.0):
    """Backward of the last ``train_loss`` (Zygote ``gradient(θ)``): fills ``model.grad``.
    ``dloss`` is the upstream cotangent of the loss (the ``rrule`` pullback's input)."""
    ex = model._last
    if not ex.forwarded:
        raise RuntimeError("gradient() needs a preceding train_loss()")
    if dloss != 1.0:
        check(lib().md2_model_loss_cotangent(ex.handle, float(dloss), stream_of(model.device)),
              "md2_model_loss_cotangent")
    ex.backward()
    return model.grad


def pullback(model: Model, d_disps=None, d_poses=None):
    """The pullback of the last ``model(x, source_ids, target_id)`` call from caller cotangents --
    what Zygote runs when the caller differentiates its own loss of (disparities, poses): fills and
    returns ``model.grad``.  ``d_disps[l]`` like the level-l disparities [N*num_bins, 1, h, w]
    (None: zero); ``d_poses`` [Pose-like (d_rvec [N, 3], d_tvec [N, 3]) per source] or a [2N, 6]
    tensor (None: zero).  The backward segments are the fused path's (md2_model_set_cotangents)."""
    import torch
    ex = model._last
    if ex is None or not ex.forwarded:
        raise RuntimeError("pullback() needs a preceding model(x, source_ids, target_id) call")
    dp = d_poses
    if d_poses is not None and not torch.is_tensor(d_poses):
        dp = torch.cat([torch.cat([torch.as_tensor(r), torch.as_tensor(t)], 1) for r, t in d_poses], 0)
    ex.set_cotangents(d_disps, dp)
    ex.backward()
    return model.grad


def set_flux_params(model: Model, flux_flat):
    """Load a Flux-layout flat vector (``Flux.params`` order, conv kernels as true convolutions)
    into the model: taps flipped on the device (md2_model_set_params), every executor re-packs."""
    import torch
    src = flux_flat.to(device=model.device, dtype=torch.float32).contiguous()
    ex = model._last or next(iter(model._ex.values()), None)
    if ex is None:
        raise RuntimeError("set_flux_params needs an executor (run train_loss / eval_disparity once)")
    check(lib().md2_model_set_params(ex.handle, ptr(src), stream_of(model.device)), "md2_model_set_params")
    model.touch()
    ex.version = model.version


def flux_params(model: Model, grads: bool = False):
    """The flat parameters (or gradients) in Flux layout (md2_model_get_params / _get_grads)."""
    import torch
    ex = model._last or next(iter(model._ex.values()), None)
    if ex is None:
        raise RuntimeError("flux_params needs an executor")
    out = torch.empty_like(model.flat)
    fn = lib().md2_model_get_grads if grads else lib().md2_model_get_params
    check(fn(ex.handle, ptr(out), stream_of(model.device)), "md2_model_get_params")
    return out


class ADAM:
    """Flux ``ADAM(eta, (beta1, beta2))`` with eps = 1e-8 (scripts/script.jl:85)."""

    def __init__(self, eta=1e-3, beta=(0.9, 0.999), eps=1e-8):
        self.eta, self.beta, self.eps = eta, beta, eps
        self.t = 0
        self.m = self.v = None

    def update(self, model: Model, grad_scale: float = 1.0):
        """``Flux.Optimise.update!(opt, θ, ∇)`` on the flat vector (in place)."""
        import torch
        if self.m is None:
            self.m = torch.zeros_like(model.flat)
            self.v = torch.zeros_like(model.flat)
        self.t += 1
        ex = model._last
        if ex is None:
            raise RuntimeError("ADAM.update needs a preceding train_loss/gradient")
        # md2_model_adam updates flat (shared by every executor) and re-packs ex's weights only
        check(lib().md2_model_adam(ex.handle, ptr(self.m), ptr(self.v), self.eta, self.beta[0],
                                   self.beta[1], self.eps, self.t, grad_scale, stream_of(model.device)),
              "md2_model_adam")
        model.touch()
        ex.version = model.version

    def update_segment(self, model: Model, k: int, grad_scale: float = 1.0):
        """The update of backward segment k's parameters alone (md2_model_adam_segment), beside the
        rest of the backward; segment 0 opens the step.  ``finish`` closes it."""
        import torch
        if self.m is None:
            self.m = torch.zeros_like(model.flat)
            self.v = torch.zeros_like(model.flat)
        ex = model._last
        if ex is None:
            raise RuntimeError("ADAM.update_segment needs a preceding train_loss/gradient")
        if k == 0:
            self.t += 1
        check(lib().md2_model_adam_segment(ex.handle, k, ptr(self.m), ptr(self.v), self.eta, self.beta[0],
                                           self.beta[1], self.eps, self.t, grad_scale,
                                           stream_of(model.device)), "md2_model_adam_segment")

    def finish(self, model: Model):
        """After every segment's update_segment: the stream waits for them (the model's weights
        are current for the next forward)."""
        ex = model._last
        check(lib().md2_model_adam_join(ex.handle, stream_of(model.device)), "md2_model_adam_join")
        model.touch()
        ex.version = model.version


def train_step(model: Model, x, auto_loss, cache: TrainCache, params: Params, opt: ADAM):
    """One ``gradient(θ) do train_loss(...)[1] end`` + ``update!`` on one GPU."""
    loss, *_ = train_loss(model, x, auto_loss, cache, params)
    gradient(model)
    opt.update(model)
    return loss


def eval_disparity(model: Model, x, cache: Optional[TrainCache] = None):
    """``eval_disparity(m, x)`` (src/model.jl:63) for x [N, C, H, W] (train-mode BatchNorm, as
    the reference never calls testmode!).  Runs on any cached executor of batch >= N at (H, W)
    (``Model.eval_executor``; its weights are re-packed first if stale); ``cache`` is unused
    (inference has no loss) and kept for signature compatibility."""
    N, Cc, H, W = x.shape
    if Cc != model.encoder.in_channels:
        raise ValueError("x must be [N, in_channels, H, W]")
    if model.depth_decoder.embedding_levels:
        raise NotImplementedError("eval_disparity (src/model.jl:63) feeds the bare encoder features, which "
                                  "an embedding_levels > 0 DepthDecoder cannot take (defect D4)")
    ex = model.eval_executor(N, H, W)
    dptr = (C.c_void_p * 5)()
    ex.forwarded = False            # the library discards any pending forward of this executor
    check(lib().md2_model_eval_disparity(ex.handle, ptr(x), N, dptr, stream_of(x.device)),
          "md2_model_eval_disparity")
    out = []
    h, w = H, W
    nl = len(model.depth_decoder.scale_levels)
    shapes = []
    for l in model.depth_decoder.scale_levels:
        f = 2 ** (5 - l)
        shapes.append((N, 1, H // f, W // f))
    return [_wrap(dptr[i], shapes[i], x.device) for i in range(nl)]
