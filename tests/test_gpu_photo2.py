"""GPU: the packed-fp32 photometric kernel (photo2.hip, the default) is bit-identical to the scalar
kernel it replaces (photo.hip, MD2_PHOTO_V1=1, read per launch): every output of the fused loss
tail (loss, per-scale terms, d disparity per scale, d pose, the per-pixel loss / argmin / bilinear
cell maps of the parity diagnostics) and of the op-level warp_photometric fwd / bwd with a
per-pixel cotangent map, at the bench shape (B=12, 416x128, 4 scales) and at odd shapes (one
channel, a 96-wide frame whose level-1 disparity is 6 columns, automasking, near-field poses)."""
import os

import pytest
import torch

from tests import _data as D

pytestmark = pytest.mark.gpu

SCALES = (0.125, 0.25, 0.5, 1.0)


def _tail(v1, disps, poses, x, K, invK, automask, visualize):
    import md2hip
    N, L, C, H, W = x.shape
    cache = md2hip.TrainCache(K=K.numpy(), invK=invK.numpy(), scales=SCALES[-len(disps):])
    params = md2hip.Params(target_size=(W, H), batch_size=N, automasking=automask is not None,
                           disparity_smoothness=1e-3)
    os.environ["MD2_PHOTO_V1"] = "1" if v1 else "0"
    try:
        r = md2hip.loss_tail(disps, poses, x, automask, cache, params, visualize=visualize)
        torch.cuda.synchronize()
    finally:
        os.environ.pop("MD2_PHOTO_V1", None)
    return r


def _same(a, b, what):
    if isinstance(a, list):
        for i, (u, v) in enumerate(zip(a, b)):
            _same(u, v, f"{what}[{i}]")
        return
    if a is None:
        assert b is None, what
        return
    assert a.shape == b.shape, what
    diff = (a != b) & ~(torch.isnan(a) & torch.isnan(b)) if a.is_floating_point() else (a != b)
    n = int(diff.sum())
    assert n == 0, f"{what}: {n} of {a.numel()} elements differ"


@pytest.mark.parametrize("N,C,H,W,nscales,sources,automask,near", [
    (12, 3, 128, 416, 4, "uniform", False, False),
    (12, 3, 128, 416, 4, "texture", True, False),
    (2, 1, 64, 96, 4, "texture", False, False),
    (3, 3, 64, 128, 2, "ramp", True, True),
], ids=["bench-uniform", "bench-texture-automask", "gray-96wide", "near-field-automask"])
@pytest.mark.parametrize("visualize", [False, True], ids=["plain", "cells"])
def test_photo2_bit_identical_to_scalar_kernel(N, C, H, W, nscales, sources, automask, near, visualize):
    dev = torch.device("cuda")
    if sources == "uniform":
        g = torch.Generator().manual_seed(3)
        x = torch.rand(N, 3, C, H, W, generator=g, dtype=torch.float32)
    else:
        x = D.triplets(N, C, H, W, seed=7, ramp_sources=sources == "ramp").float()
    x = x.to(dev).contiguous()
    K, invK = D.intrinsics(W, H)
    disps = [d.float().to(dev).contiguous() for d in D.disparities(N, H, W, nscales=nscales, seed=11)]
    kw = dict(forward=0.05, jitter=0.2) if near else {}
    poses = [(a.float().to(dev), b.float().to(dev)) for a, b in D.poses(N, seed=13, **kw)]
    am = None
    if automask:
        am = (0.2 * torch.rand(N, 1, H, W, generator=torch.Generator().manual_seed(5))).to(dev).contiguous()
    r1 = _tail(True, disps, poses, x, K, invK, am, visualize)
    r2 = _tail(False, disps, poses, x, K, invK, am, visualize)
    keys = sorted(set(r1) & set(r2) - {"workspace"})
    assert {"loss", "terms", "d_disp", "d_pose"} <= set(keys)
    for k in keys:
        _same(r1[k], r2[k], k)


@pytest.mark.parametrize("scale", [1, 4])
def test_photo2_warp_op_with_cotangent_map_bit_identical(scale):
    """md2_warp_photometric_fwd / _bwd (one scale, per-pixel cotangent map = the kernel's gmap
    path) through the op-level API."""
    from md2hip import primitives as Pm
    dev = torch.device("cuda")
    N, C, H, W = 4, 3, 128, 416
    x = D.triplets(N, C, H, W, seed=7).float().to(dev).contiguous()
    K, invK = D.intrinsics(W, H)
    d = D.disparities(N, H, W, nscales=4, seed=11)[-1 if scale == 1 else 0].float().to(dev).contiguous()
    rt = torch.randn(2 * N, 12, generator=torch.Generator().manual_seed(2)) * 0.01
    rt[:, 0] += 1
    rt[:, 4] += 1
    rt[:, 8] += 1
    rt = rt.to(dev)
    dl = torch.rand(N, 1, H, W, generator=torch.Generator().manual_seed(9)).to(dev)
    outs = []
    for v1 in (True, False):
        os.environ["MD2_PHOTO_V1"] = "1" if v1 else "0"
        try:
            dd = d.clone().requires_grad_(True)
            rr = rt.clone().requires_grad_(True)
            out, sel = Pm.warp_photometric(dd, rr, x, K.numpy(), invK.numpy(), return_sel=True)
            out.backward(dl)
            torch.cuda.synchronize()
            outs.append((out.detach(), sel, dd.grad, rr.grad))
        finally:
            os.environ.pop("MD2_PHOTO_V1", None)
    for name, a, b in zip(("loss_map", "sel", "d_disp", "d_Rt"), outs[0], outs[1]):
        _same(a, b, name)
