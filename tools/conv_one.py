"""Run one conv shape (fwd, dgrad, wgrad) a few times -- for rocprofv3 counter collection."""
import os, sys, ctypes as C
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R); sys.path.insert(0, os.path.join(R, "monodepth2.jl_amd"))
import torch
from md2hip import ops
from md2hip._lib import lib, ptr, stream_of, check
SHAPES = {"l2": ((36, 128, 16, 52), 128, 3, 1, 1, 0), "l1": ((36, 64, 32, 104), 64, 3, 1, 1, 0),
          "l3": ((36, 256, 8, 26), 256, 3, 1, 1, 0), "l4": ((36, 512, 4, 13), 512, 3, 1, 1, 0), "d4": ((12, 96, 64, 208), 32, 3, 1, 1, 1),
          "stem": ((36, 3, 128, 416), 64, 7, 2, 3, 0),
          "s2l2": ((36, 64, 32, 104), 128, 3, 2, 1, 0), "s2l3": ((36, 128, 16, 52), 256, 3, 2, 1, 0),
          "s2l4": ((36, 256, 8, 26), 512, 3, 2, 1, 0)}
xs, cout, k, st, pd, rf = SHAPES[sys.argv[1] if len(sys.argv) > 1 else "l2"]
only = sys.argv[2] if len(sys.argv) > 2 else "all"
x = torch.randn(*xs, device="cuda")
w = torch.randn(cout, xs[1], k, k, device="cuda") * 0.05
d = ops.conv_desc(xs, tuple(w.shape), st, pd, bool(rf))
ws = torch.empty(lib().md2_conv2d_workspace_size(C.byref(d)) // 4 + 64, device="cuda")
ho, wo = ops.out_hw(xs[2], xs[3], k, st, pd)
y = torch.empty(xs[0], cout, ho, wo, device="cuda"); dy = torch.randn_like(y); dx = torch.empty_like(x); dw = torch.empty_like(w)
for _ in range(5):
    if only in ("all", "fwd"):
        check(lib().md2_conv2d_fwd(C.byref(d), ptr(x), ptr(w), None, ptr(y), ptr(ws), stream_of()))
    if only in ("all", "dgrad"):
        check(lib().md2_conv2d_dgrad(C.byref(d), ptr(dy), ptr(w), ptr(dx), ptr(ws), stream_of()))
    if only in ("all", "wgrad"):
        check(lib().md2_conv2d_wgrad(C.byref(d), ptr(x), ptr(dy), ptr(dw), None, ptr(ws), stream_of()))
torch.cuda.synchronize()
