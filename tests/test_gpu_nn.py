"""GPU parity of the pooling / resampling kernels against fp64 torch-CPU references.

* MaxPool((3,3), pad=1, stride=2) (ResNet.jl stem): values bit-exact, the window
  index of the FIRST maximum (NNlib / torch.argmax tie rule) exact, the pullback exact (it only
  routes dy; a 2x2-block gather sums at most four routed values).
* upsample_bilinear(x, (2,2)) align_corners (src/depth_decoder.jl:18-19) and its adjoint:
  relative Frobenius error 1e-6 against fp64 F.interpolate / autograd.
"""
import pytest
import torch
import torch.nn.functional as F

from tests import _data as D

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def _ops():
    from md2hip import ops
    return ops


def _maxpool_ref(x):
    """first-maximum window index of a -inf padded 3x3/2 window; dx by scatter-add."""
    n, c, h, w = x.shape
    xp = F.pad(x, (1, 1, 1, 1), value=float("-inf"))
    win = xp.unfold(2, 3, 2).unfold(3, 3, 2)              # [n][c][ho][wo][3][3]
    flat = win.reshape(*win.shape[:4], 9)
    return flat.max(-1).values, flat.argmax(-1)


def _maxpool_bwd_ref(dy, arg, h, w):
    n, c, ho, wo = dy.shape
    kh, kw = arg // 3, arg % 3
    oh = torch.arange(ho).view(1, 1, ho, 1)
    ow = torch.arange(wo).view(1, 1, 1, wo)
    ih = 2 * oh - 1 + kh
    iw = 2 * ow - 1 + kw
    dx = torch.zeros(n, c, h * w, dtype=dy.dtype)
    dx.scatter_add_(2, (ih * w + iw).reshape(n, c, -1), dy.reshape(n, c, -1))
    return dx.view(n, c, h, w)


@pytest.mark.parametrize("shape", [(12, 64, 64, 208), (2, 3, 7, 9), (1, 2, 1, 1), (2, 4, 2, 3),
                                   (3, 5, 8, 5)])
def test_maxpool3s2(shape):
    ops = _ops()
    g = torch.Generator().manual_seed(7)
    x = torch.randn(*shape, generator=g)
    if shape[1] == 4:                        # ties: quantised values hit the first-max rule
        x = torch.round(x)
    y, arg = ops.maxpool3s2(x.to(DEV))
    yr, ar = _maxpool_ref(x)
    assert torch.equal(y.cpu(), yr)
    assert torch.equal(arg.cpu().long(), ar)
    dy = torch.randn(*yr.shape, generator=g)
    dx = ops.maxpool3s2_backward(dy.to(DEV), arg, shape)
    ref = _maxpool_bwd_ref(dy.double(), ar, shape[2], shape[3])
    assert D.rel_err(dx.cpu().double(), ref) < 1e-7


@pytest.mark.parametrize("shape", [(12, 16, 64, 208), (2, 256, 4, 13), (2, 3, 1, 1), (1, 2, 1, 5),
                                   (2, 2, 2, 2), (3, 4, 3, 7)])
def test_upsample2(shape):
    ops = _ops()
    g = torch.Generator().manual_seed(11)
    x = torch.randn(*shape, generator=g)
    y = ops.upsample2(x.to(DEV))
    xr = x.double().requires_grad_(True)
    yr = F.interpolate(xr, scale_factor=2, mode="bilinear", align_corners=True)
    assert D.rel_err(y.cpu().double(), yr.detach()) < 1e-6
    dy = torch.randn(*yr.shape, generator=g)
    (gx,) = torch.autograd.grad(yr, xr, dy.double())
    dx = ops.upsample2_backward(dy.to(DEV))
    assert D.rel_err(dx.cpu().double(), gx) < 1e-6


_UP_CHILD = r"""
import sys, numpy as np, torch
sys.path[:0] = [sys.argv[1], sys.argv[1] + "/monodepth2.jl_amd"]
from md2hip import ops
out = []
for shape in [(12, 16, 64, 208), (12, 32, 32, 104), (12, 256, 4, 13), (3, 4, 3, 7), (2, 3, 1, 1)]:
    g = torch.Generator().manual_seed(5)
    n, c, h, w = shape
    dy = torch.randn(n, c, 2 * h, 2 * w, generator=g).cuda()
    out.append(ops.upsample2_backward(dy).cpu().numpy().ravel())
np.save(sys.argv[2], np.concatenate(out))
"""


def test_upsample2_backward_tiled_bit_identical_to_gather(tmp_path):
    """The tiled adjoint (4 input rows per thread, round 6) equals the one-pixel-per-thread gather
    kernel (MD2_UP_TILED=0) bit for bit at the decoder's shapes and odd ones."""
    import os
    import subprocess
    import sys
    import numpy as np
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    base = {k: v for k, v in os.environ.items() if not k.startswith("MD2_")}
    res = {}
    for name, env in (("tiled", base), ("gather", dict(base, MD2_TUNING="1", MD2_UP_TILED="0"))):
        out = str(tmp_path / f"{name}.npy")
        r = subprocess.run([sys.executable, "-c", _UP_CHILD, root, out], env=env, capture_output=True,
                           text=True, timeout=200)
        assert r.returncode == 0, (name, r.stderr[-3000:])
        res[name] = np.load(out)
    assert np.array_equal(res["tiled"].view(np.uint32), res["gather"].view(np.uint32))
