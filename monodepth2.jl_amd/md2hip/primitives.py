"""Op-level loss primitives of the reference (src/utils.jl, src/training.jl) as differentiable
host functions over the C-ABI -- the Python mirror of the ``ChainRulesCore.rrule`` seam the
Julia shim uses (julia/MD2HIP.jl): every op is a ``torch.autograd.Function`` whose forward calls
``md2_*_fwd`` and whose backward calls the matching ``md2_*_bwd`` pullback.  No CPU fallback.

Layouts follow the C-ABI (= the Julia arrays' memory): ``Backproject`` returns [N, W*H, 3] for
Julia's (3, W*H, N); ``Project`` takes R as [N, 3, 3] (row i, column j) and returns [N, W*H, 2];
``grid_sample_border`` takes grid [N, Ho, Wo, 2] for Julia's (2, Wo, Ho, N)."""
from __future__ import annotations

import ctypes as C
from typing import Optional, Sequence

import numpy as np

from ._lib import WarpCfg, check, lib, ptr, stream_of


def _f32(t):
    import torch
    if t.dtype != torch.float32 or not t.is_contiguous() or t.device.type != "cuda":
        raise ValueError("expected a contiguous float32 CUDA tensor")
    return t


def _mat(m, dev):
    """3x3 (numpy / tensor) -> contiguous row-major float32 device tensor."""
    import torch
    return torch.as_tensor(np.asarray(m, dtype=np.float64).reshape(3, 3), dtype=torch.float32).to(dev).contiguous()


def _ws(nbytes, dev):
    import torch
    return torch.empty(max(int(nbytes) // 4, 1) + 64, dtype=torch.float32, device=dev)


# ------------------------------------------------------------------------------------------------
def static_scores(x, target_id: int = 2, source_ids: Sequence[int] = (1, 3)):
    """Per-sample ``mean(automasking_loss(ssim, x_i, x_i[target]; source_ids))`` -- the score
    ``find_static`` (src/dtk.jl:51-69) thresholds.  x [N, 3, C, H, W] -> [N]."""
    import torch
    _f32(x)
    N, L, Cc, H, W = x.shape
    if L != 3 or len(source_ids) != 2:
        raise ValueError("x must hold 3 frames and source_ids two of them")
    out = torch.empty(N, dtype=torch.float32, device=x.device)
    ws = _ws(lib().md2_static_scores_workspace_size(N, H, W), x.device)
    check(lib().md2_static_scores(ptr(x), N, Cc, H, W, target_id - 1, source_ids[0] - 1,
                                  source_ids[1] - 1, ptr(out), ptr(ws), stream_of(x.device)),
          "md2_static_scores")
    return out


def automasking_loss(x, target_id: int = 2, source_ids: Sequence[int] = (1, 3)):
    """``automasking_loss(ssim, x, target; source_ids)`` (src/training.jl:9-11): x [N, 3, C, H, W]
    -> [N, 1, H, W] identity-reprojection loss (min over the raw sources).  Data only."""
    import torch
    _f32(x)
    N, L, Cc, H, W = x.shape
    if L != 3 or len(source_ids) != 2:
        raise ValueError("x must hold 3 frames and source_ids two of them")
    out = torch.empty(N, 1, H, W, dtype=torch.float32, device=x.device)
    check(lib().md2_automasking_loss(ptr(x), N, Cc, H, W, target_id - 1, source_ids[0] - 1,
                                     source_ids[1] - 1, ptr(out), stream_of(x.device)),
          "md2_automasking_loss")
    return out


# ------------------------------------------------------------------------------------------------
def _ssim_fn():
    import torch

    class _SSIM(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x, y):
            _f32(x), _f32(y)
            n, c, h, w = x.shape
            out = torch.empty_like(x)
            check(lib().md2_ssim_fwd(ptr(x), ptr(y), n, c, h, w, ptr(out), stream_of(x.device)), "md2_ssim_fwd")
            ctx.save_for_backward(x, y)
            return out

        @staticmethod
        def backward(ctx, dout):
            x, y = ctx.saved_tensors
            n, c, h, w = x.shape
            dx = torch.empty_like(x) if ctx.needs_input_grad[0] else None
            dy = torch.empty_like(y) if ctx.needs_input_grad[1] else None
            check(lib().md2_ssim_bwd(ptr(x), ptr(y), ptr(dout.contiguous()), n, c, h, w, ptr(dx), ptr(dy),
                                     stream_of(x.device)), "md2_ssim_bwd")
            return dx, dy
    return _SSIM


class SSIM:
    """``SSIM()`` (src/utils.jl:17-23): MeanPool((3,3); stride=1) on reflect-padded inputs,
    c1 = 0.01^2, c2 = 0.03^2.  ``(ssim)(x, y)`` -> [N, C, H, W] in [0, 1]."""
    c1, c2 = 0.01 ** 2, 0.03 ** 2

    def __call__(self, x, y):
        return _ssim_fn().apply(x, y)


# ------------------------------------------------------------------------------------------------
class Backproject:
    """``Backproject(; width, height)`` (src/utils.jl:45-69); ``(b)(depth, invK)``:
    depth [N, W*H] (or [N, 1, W*H]) -> camera points [N, W*H, 3] (1-based pixel grid)."""

    def __init__(self, *, width: int, height: int):
        self.width, self.height = width, height

    def __call__(self, depth, invK):
        import torch
        width, height = self.width, self.height

        class _BP(torch.autograd.Function):
            @staticmethod
            def forward(ctx, d):
                d = _f32(d.reshape(d.shape[0], width * height).contiguous())
                iK = _mat(invK, d.device)
                out = torch.empty(d.shape[0], width * height, 3, dtype=torch.float32, device=d.device)
                check(lib().md2_backproject_fwd(ptr(d), d.shape[0], width, height, ptr(iK), ptr(out),
                                                stream_of(d.device)), "md2_backproject_fwd")
                ctx.shape, ctx.iK = depth.shape, iK
                return out

            @staticmethod
            def backward(ctx, dout):
                n = dout.shape[0]
                dd = torch.empty(n, width * height, dtype=torch.float32, device=dout.device)
                check(lib().md2_backproject_bwd(ptr(dout.contiguous()), n, width, height, ptr(ctx.iK), ptr(dd),
                                                stream_of(dout.device)), "md2_backproject_bwd")
                return dd.reshape(ctx.shape)
        return _BP.apply(depth)


class Project:
    """``Project(; width, height)`` (src/utils.jl:71-103); ``(p)(points, K, R, t)``:
    points [N, W*H, 3], K 3x3, R [N, 3, 3], t [N, 3] -> normalised coordinates [N, W*H, 2]."""

    def __init__(self, *, width: int, height: int):
        self.width, self.height = width, height

    def __call__(self, points, K, R, t):
        import torch
        width, height = self.width, self.height

        class _PJ(torch.autograd.Function):
            @staticmethod
            def forward(ctx, pts, R_, t_):
                _f32(pts)
                n = pts.shape[0]
                Kd = _mat(K, pts.device)
                Rc, tc = _f32(R_.contiguous()), _f32(t_.reshape(n, 3).contiguous())
                out = torch.empty(n, width * height, 2, dtype=torch.float32, device=pts.device)
                check(lib().md2_project_fwd(ptr(pts), n, width, height, ptr(Kd), ptr(Rc), ptr(tc), ptr(out),
                                            stream_of(pts.device)), "md2_project_fwd")
                ctx.save_for_backward(pts, Rc, tc)
                ctx.Kd, ctx.tshape = Kd, t_.shape
                return out

            @staticmethod
            def backward(ctx, dout):
                pts, Rc, tc = ctx.saved_tensors
                n = pts.shape[0]
                dp = torch.empty_like(pts)
                dR = torch.empty(n, 3, 3, dtype=torch.float32, device=pts.device)
                dt = torch.empty(n, 3, dtype=torch.float32, device=pts.device)
                ws = _ws(lib().md2_project_workspace_size(n, width, height), pts.device)
                check(lib().md2_project_bwd(ptr(pts), n, width, height, ptr(ctx.Kd), ptr(Rc), ptr(tc),
                                            ptr(dout.contiguous()), ptr(dp), ptr(dR), ptr(dt), ptr(ws),
                                            stream_of(pts.device)), "md2_project_bwd")
                return dp, dR, dt.reshape(ctx.tshape)
        return _PJ.apply(points, R, t)


# ------------------------------------------------------------------------------------------------
def grid_sample_border(x, grid):
    """NNlib ``grid_sample(x, grid; padding_mode=:border)``, align_corners=true
    (src/training.jl:56): x [N, C, Hi, Wi], grid [N, Ho, Wo, 2] -> [N, C, Ho, Wo].  The x
    pullback is an atomic scatter (summation order not fixed), formed only when x needs grad."""
    import torch

    class _GS(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x_, g_):
            _f32(x_), _f32(g_)
            n, c, hi, wi = x_.shape
            _, ho, wo, two = g_.shape
            assert two == 2 and g_.shape[0] == n
            out = torch.empty(n, c, ho, wo, dtype=torch.float32, device=x_.device)
            check(lib().md2_grid_sample_border_fwd(ptr(x_), ptr(g_), n, c, hi, wi, ho, wo, ptr(out),
                                                   stream_of(x_.device)), "md2_grid_sample_border_fwd")
            ctx.save_for_backward(x_, g_)
            return out

        @staticmethod
        def backward(ctx, dout):
            x_, g_ = ctx.saved_tensors
            n, c, hi, wi = x_.shape
            _, ho, wo, _ = g_.shape
            dg = torch.empty_like(g_)
            dx = torch.empty_like(x_) if ctx.needs_input_grad[0] else None
            check(lib().md2_grid_sample_border_bwd(ptr(x_), ptr(g_), ptr(dout.contiguous()), n, c, hi, wi,
                                                   ho, wo, ptr(dg), ptr(dx), stream_of(x_.device)),
                  "md2_grid_sample_border_bwd")
            return dx, dg
    return _GS.apply(x, grid)


# ------------------------------------------------------------------------------------------------
def smooth_loss(disparity, image):
    """``smooth_loss(disparity, image)`` (src/utils.jl:163-177): disparity [N, H, W], image
    [N, C, H, W] -> scalar.  The pullback is formed w.r.t. the disparity (the image is data in
    every caller, src/training.jl:66 and src/simple_depth.jl:39)."""
    import torch

    class _SM(torch.autograd.Function):
        @staticmethod
        def forward(ctx, d, img):
            _f32(d), _f32(img)
            n, h, w = d.shape
            c = img.shape[1]
            out = torch.empty(1, dtype=torch.float32, device=d.device)
            ws = _ws(lib().md2_smooth_loss_workspace_size(n, w, h), d.device)
            check(lib().md2_smooth_loss_fwd(ptr(d), ptr(img), n, c, h, w, ptr(out), ptr(ws),
                                            stream_of(d.device)), "md2_smooth_loss_fwd")
            ctx.save_for_backward(d, img)
            return out[0]

        @staticmethod
        def backward(ctx, dl):
            d, img = ctx.saved_tensors
            n, h, w = d.shape
            dd = torch.empty_like(d)
            ws = _ws(lib().md2_smooth_loss_workspace_size(n, w, h), d.device)
            check(lib().md2_smooth_loss_bwd(ptr(d), ptr(img), n, img.shape[1], h, w, C.c_float(float(dl)),
                                            ptr(dd), ptr(ws), stream_of(d.device)), "md2_smooth_loss_bwd")
            return dd, None
    return _SM.apply(disparity, image)


# ------------------------------------------------------------------------------------------------
def compose_poses(pose, n: int, invert_mask: int):
    """``composeT(so3_exp_map(rvec), tvec, invert)`` for both sources (src/utils.jl:106-145,
    185-192): pose [2N, 6] (rvec, tvec rows s*N+i) -> Rt [2N, 12] (R row-major, t)."""
    import torch

    class _CT(torch.autograd.Function):
        @staticmethod
        def forward(ctx, p):
            _f32(p)
            Rt = torch.empty(2 * n, 12, dtype=torch.float32, device=p.device)
            check(lib().md2_so3_compose_fwd(ptr(p), n, invert_mask, ptr(Rt), stream_of(p.device)),
                  "md2_so3_compose_fwd")
            ctx.save_for_backward(p)
            return Rt

        @staticmethod
        def backward(ctx, dRt):
            p, = ctx.saved_tensors
            dp = torch.empty_like(p)
            check(lib().md2_so3_compose_bwd(ptr(p), n, invert_mask, ptr(dRt.contiguous()), ptr(dp),
                                            stream_of(p.device)), "md2_so3_compose_bwd")
            return dp
    return _CT.apply(pose)


def warp_cfg(N, Cc, W, H, dw, dh, K, invK, min_depth=0.1, max_depth=100.0, target_id=2,
             source_ids=(1, 3), L=3) -> WarpCfg:
    c = WarpCfg()
    c.n, c.c, c.width, c.height, c.dw, c.dh = N, Cc, W, H, dw, dh
    Kf, iKf = np.asarray(K, dtype=np.float64).reshape(-1), np.asarray(invK, dtype=np.float64).reshape(-1)
    for i in range(9):
        c.K[i], c.invK[i] = float(Kf[i]), float(iKf[i])
    c.min_depth, c.max_depth = min_depth, max_depth
    c.x_frame_stride = Cc * H * W
    c.x_sample_stride = L * Cc * H * W
    c.target, c.src0, c.src1 = target_id - 1, source_ids[0] - 1, source_ids[1] - 1
    return c


def warp_photometric(disparity, Rt, x, K, invK, *, min_depth=0.1, max_depth=100.0, target_id=2,
                     source_ids=(1, 3), automask=None, return_sel=False):
    """One scale of ``train_loss``'s loop (src/training.jl:43-62): upsample the disparity
    [N, 1, dh, dw] to x's resolution, depth, Backproject, Project with the composed poses Rt
    [2N, 12], border grid_sample of both sources, photometric loss, min over sources
    [, min with the automask]; -> warp_loss [N, 1, H, W].  Differentiable in disparity and Rt."""
    import torch
    N, L, Cc, H, W = x.shape
    dh, dw = disparity.shape[-2], disparity.shape[-1]
    cfg = warp_cfg(N, Cc, W, H, dw, dh, K, invK, min_depth, max_depth, target_id, source_ids, L)
    am = None if automask is None else _f32(automask.contiguous())
    sel = torch.empty(N, 1, H, W, dtype=torch.int8, device=x.device)

    class _WP(torch.autograd.Function):
        @staticmethod
        def forward(ctx, d, rt):
            _f32(d), _f32(rt), _f32(x)
            out = torch.empty(N, 1, H, W, dtype=torch.float32, device=d.device)
            ws = _ws(lib().md2_warp_photometric_workspace_size(C.byref(cfg)), d.device)
            check(lib().md2_warp_photometric_fwd(C.byref(cfg), ptr(d), ptr(rt), ptr(x), ptr(am), ptr(out),
                                                 ptr(sel), ptr(ws), stream_of(d.device)),
                  "md2_warp_photometric_fwd")
            ctx.save_for_backward(d, rt)
            return out

        @staticmethod
        def backward(ctx, dl):
            d, rt = ctx.saved_tensors
            dd = torch.empty_like(d)
            drt = torch.empty_like(rt)
            ws = _ws(lib().md2_warp_photometric_workspace_size(C.byref(cfg)), d.device)
            check(lib().md2_warp_photometric_bwd(C.byref(cfg), ptr(d), ptr(rt), ptr(x), ptr(am),
                                                 ptr(dl.contiguous()), ptr(dd), ptr(drt), ptr(ws),
                                                 stream_of(d.device)), "md2_warp_photometric_bwd")
            return dd, drt
    out = _WP.apply(disparity, Rt)
    return (out, sel) if return_sel else out
