"""Host mirror of the reference's loss API (src/Monodepth.jl:37-60, src/training.jl) over the
C-ABI.  Tensors are torch CUDA tensors in C order ([N,C,H,W]; x is [N,L,C,H,W])."""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _lib
from ._lib import LossCfg, check, lib, ptr, ptr_array, stream_of


@dataclass
class Params:
    """``Params`` (src/Monodepth.jl:37-47)."""
    target_size: Tuple[int, int]            # (width, height)
    batch_size: int
    min_depth: float = 0.1
    max_depth: float = 100.0
    disparity_smoothness: float = 1e-3
    frame_ids: List[int] = field(default_factory=lambda: [1, 2, 3])
    automasking: bool = True


@dataclass
class TrainCache:
    """``TrainCache`` (src/Monodepth.jl:49-60): intrinsics, frame ids (1-based), scales."""
    K: np.ndarray
    invK: np.ndarray
    target_id: int = 2
    source_ids: Sequence[int] = (1, 3)
    scales: Sequence[float] = (0.125, 0.25, 0.5, 1.0)


def depth10k_intrinsics(width=416, height=128):
    """Depth10k K / invK (src/dtk.jl:15-21)."""
    f = 2648.0 / 4.63461538462
    K = np.array([[f, 0, width / 2.0], [0, f, height / 2.0], [0, 0, 1.0]])
    return K, np.linalg.inv(K)


def _check_ids(cache: TrainCache):
    if len(cache.source_ids) != 2:
        raise ValueError("the HIP loss supports exactly two source frames (TrainCache.source_ids)")


def make_loss_cfg(N, C_, W, H, disp_shapes, cache: TrainCache, params: Params, *,
                  smooth_weights=None, divisor=None, smooth_normalize=True,
                  L=3, sigmoid_grad=False) -> LossCfg:
    _check_ids(cache)
    cfg = LossCfg()
    cfg.n, cfg.c, cfg.width, cfg.height = N, C_, W, H
    cfg.nscales = len(disp_shapes)
    if cfg.nscales > _lib.MAX_SCALES:
        raise ValueError("at most 5 scales")
    for s, (h, w) in enumerate(disp_shapes):
        cfg.scale_w[s], cfg.scale_h[s] = w, h
        if smooth_weights is None:
            cfg.smooth_weight[s] = params.disparity_smoothness * float(cache.scales[s])
        else:
            cfg.smooth_weight[s] = smooth_weights[s]
    cfg.divisor = float(len(disp_shapes) if divisor is None else divisor)
    cfg.smooth_normalize = int(smooth_normalize)
    for i in range(9):
        cfg.K[i] = float(np.asarray(cache.K, dtype=np.float64).reshape(-1)[i])
        cfg.invK[i] = float(np.asarray(cache.invK, dtype=np.float64).reshape(-1)[i])
    cfg.min_depth, cfg.max_depth = params.min_depth, params.max_depth
    cfg.x_frame_stride = C_ * H * W
    cfg.x_sample_stride = L * C_ * H * W
    cfg.target = cache.target_id - 1
    cfg.src0, cfg.src1 = cache.source_ids[0] - 1, cache.source_ids[1] - 1
    cfg.invert_mask = sum(1 << s for s, sid in enumerate(cache.source_ids) if sid < cache.target_id)
    cfg.sigmoid_grad = int(sigmoid_grad)
    return cfg


def pack_poses(poses):
    """[(rvec [N,3], tvec [N,3])] x 2  ->  [2N, 6] (row s*N+i)."""
    import torch
    return torch.cat([torch.cat([r, t], 1) for r, t in poses], 0).contiguous()


def loss_tail(disparities, poses, x, auto_loss, cache: TrainCache, params: Params, *,
              grads=True, smooth_weights=None, divisor=None, smooth_normalize=True,
              dloss=1.0, sigmoid_grad=False, visualize=False, keep_workspace=False):
    """The body of ``train_loss`` after the model call (src/training.jl:25-77) and its pullback.

    disparities: list of [N,1,h,w] float32 CUDA tensors (one per scale); poses: list of
    (rvec [N,3], tvec [N,3]) per source; x: [N,L,C,H,W]; auto_loss: [N,1,H,W] or None.
    Returns a dict: loss [1], terms [nscales,2], d_disp (list), d_pose [2N,6] and, with
    ``visualize``, vis_loss / vis_sel [nscales,N,H,W] (training.jl:71-74 vis_loss) and
    vis_warped [2,N,C,H,W] (both sources warped by the last scale, training.jl:71-73).
    ``keep_workspace`` (diagnostics): also return the raw workspace as "workspace"."""
    import torch
    N, L, C_, H, W = x.shape
    dev = x.device
    for d in disparities:
        assert d.dtype == torch.float32 and d.is_contiguous() and d.device == dev
    assert x.dtype == torch.float32 and x.is_contiguous()
    shapes = [(d.shape[-2], d.shape[-1]) for d in disparities]
    cfg = make_loss_cfg(N, C_, W, H, shapes, cache, params, smooth_weights=smooth_weights,
                        divisor=divisor, smooth_normalize=smooth_normalize, L=L,
                        sigmoid_grad=sigmoid_grad)
    pose = pack_poses(poses).to(dev, torch.float32)
    ws_bytes = lib().md2_loss_workspace_size(C.byref(cfg))
    ws = torch.empty(ws_bytes // 4 + 64, dtype=torch.float32, device=dev)
    res = {"loss": torch.empty(1, dtype=torch.float32, device=dev),
           "terms": torch.empty(len(disparities), 2, dtype=torch.float32, device=dev),
           "d_disp": [torch.empty_like(d) for d in disparities] if grads else [None] * len(disparities),
           "d_pose": torch.empty(2 * N, 6, dtype=torch.float32, device=dev) if grads else None}
    if keep_workspace:
        res["workspace"] = ws
    if visualize:
        res["vis_loss"] = torch.empty(len(disparities), N, H, W, dtype=torch.float32, device=dev)
        res["vis_sel"] = torch.empty(len(disparities), N, H, W, dtype=torch.int8, device=dev)
        res["vis_warped"] = torch.empty(2, N, C_, H, W, dtype=torch.float32, device=dev)
        # per-pixel bilinear cells / border states of both sources (parity diagnostics)
        res["vis_cell"] = torch.empty(len(disparities), 2, N, H, W, dtype=torch.int32, device=dev)
    am = None
    if params.automasking:
        if auto_loss is None:        # automasking_loss(ssim, x, target; source_ids), on the GPU
            from .primitives import automasking_loss
            auto_loss = automasking_loss(x, cache.target_id, cache.source_ids)
        am = auto_loss.contiguous()
    out = _lib.LossOut()
    out.loss = res["loss"].data_ptr()
    out.terms = res["terms"].data_ptr()
    for i, d in enumerate(res["d_disp"]):
        out.d_disp[i] = None if d is None else d.data_ptr()
    out.d_pose = None if res["d_pose"] is None else res["d_pose"].data_ptr()
    out.vis_loss = res["vis_loss"].data_ptr() if visualize else None
    out.vis_sel = res["vis_sel"].data_ptr() if visualize else None
    out.vis_warped = res["vis_warped"].data_ptr() if visualize else None
    out.vis_cell = res["vis_cell"].data_ptr() if visualize else None
    disp_arr = ptr_array(disparities)
    check(lib().md2_loss_fwd_bwd(C.byref(cfg), C.cast(disp_arr, _lib.FP), ptr(pose), ptr(x), ptr(am),
                                 C.c_float(dloss), C.byref(out), ptr(ws), stream_of(dev)),
          "md2_loss_fwd_bwd")
    return res
