"""Relative Frobenius error vs fp64 of the conv kernels (fwd / dgrad / wgrad) at the bench's
encoder and decoder shapes, on fp32-representable inputs (as tests/test_gpu_conv.py) -- to compare
kernel variants' arithmetic, e.g. the exact-fp32 MFMA (conv_px2) against the exact-product bf16x9
kernel (conv_px3: MD2_TUNING=1 MD2_PX3=1).   python tools/conv_accuracy.py [OUT.json]"""
import json
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, "monodepth2.jl_amd")]
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from md2hip import ops  # noqa: E402
from oracle import md2_oracle as O  # noqa: E402
from tests import _data as D  # noqa: E402

SH = [("l1", (36, 64, 32, 104), 64, 3, 1, 1, False), ("l2.0", (36, 64, 32, 104), 128, 3, 2, 1, False),
      ("l2", (36, 128, 16, 52), 128, 3, 1, 1, False), ("l3", (36, 256, 8, 26), 256, 3, 1, 1, False),
      ("l4.0", (36, 256, 8, 26), 512, 3, 2, 1, False), ("l4", (36, 512, 4, 13), 512, 3, 1, 1, False),
      ("down3", (36, 128, 16, 52), 256, 1, 2, 0, False), ("d3c2", (12, 128, 32, 104), 64, 3, 1, 1, True),
      ("b1c2", (12, 512, 8, 26), 256, 3, 1, 1, True)]
out = {}
for name, xs, cout, k, st, pd, rf in SH:
    g = torch.Generator().manual_seed(5)
    x = torch.randn(*xs, generator=g, dtype=torch.float64).float().double()
    w = (torch.randn(cout, xs[1], k, k, generator=g, dtype=torch.float64) / (xs[1] * k * k) ** 0.5).float().double()
    xr, wr = x.clone().requires_grad_(True), w.clone().requires_grad_(True)
    pre = F.conv2d(O.pad_reflect(xr, pd), wr, stride=st) if rf else F.conv2d(xr, wr, stride=st, padding=pd)
    dy = torch.randn(pre.shape, generator=g, dtype=torch.float64).float().double()
    pre.backward(dy)
    xg, wg = x.float().cuda(), w.float().cuda()
    y = ops.conv2d(xg, wg, None, stride=st, pad=pd, reflect=rf)
    dx = ops.conv2d_dgrad(dy.float().cuda(), wg, xs, stride=st, pad=pd, reflect=rf)
    dw, _ = ops.conv2d_wgrad(xg, dy.float().cuda(), tuple(w.shape), stride=st, pad=pd, reflect=rf, bias=False)
    torch.cuda.synchronize()
    # the fp32 floor: the same convolutions evaluated in fp32 on the CPU
    y32 = (F.conv2d(O.pad_reflect(x.float(), pd), w.float(), stride=st) if rf
           else F.conv2d(x.float(), w.float(), stride=st, padding=pd))
    out[name] = {"fwd": D.rel_err(y, pre.detach()), "dgrad": D.rel_err(dx, xr.grad), "wgrad": D.rel_err(dw, wr.grad),
                 "fwd_cpu_fp32": D.rel_err(y32, pre.detach())}
    print(name, {k_: f"{v:.2e}" for k_, v in out[name].items()}, flush=True)
if len(sys.argv) > 1:
    with open(sys.argv[1], "w") as f:
        json.dump({"env": {k: v for k, v in os.environ.items() if k.startswith("MD2_")}, "rel_err": out}, f, indent=1)
