"""Per-shape throughput of the conv kernels at the measured config (B=12 -> 36 encoder images)."""
import os, sys, ctypes as C
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R); sys.path.insert(0, os.path.join(R, "monodepth2.jl_amd"))
import torch
from md2hip import ops
from md2hip._lib import lib, ptr, stream_of, check
SH = [  # name, x_shape, cout, k, s, p, reflect
    ("stem", (36, 3, 128, 416), 64, 7, 2, 3, 0),
    ("l1", (36, 64, 32, 104), 64, 3, 1, 1, 0),
    ("l2.0", (36, 64, 32, 104), 128, 3, 2, 1, 0),
    ("l2", (36, 128, 16, 52), 128, 3, 1, 1, 0),
    ("l3.0", (36, 128, 16, 52), 256, 3, 2, 1, 0),
    ("l3", (36, 256, 8, 26), 256, 3, 1, 1, 0),
    ("l4.0", (36, 256, 8, 26), 512, 3, 2, 1, 0),
    ("l4", (36, 512, 4, 13), 512, 3, 1, 1, 0),
    ("d1c1", (12, 512, 4, 13), 256, 3, 1, 1, 1),
    ("d1c2", (12, 512, 8, 26), 256, 3, 1, 1, 1),
    ("d2c1", (12, 256, 8, 26), 128, 3, 1, 1, 1),
    ("d2c2", (12, 256, 16, 52), 128, 3, 1, 1, 1),
    ("d3c1", (12, 128, 16, 52), 64, 3, 1, 1, 1),
    ("d5c2", (12, 16, 128, 416), 16, 3, 1, 1, 1),
    ("d4c2", (12, 96, 64, 208), 32, 3, 1, 1, 1),
    ("d3c2", (12, 128, 32, 104), 64, 3, 1, 1, 1),
    ("d5c1", (12, 32, 64, 208), 16, 3, 1, 1, 1),
    ("d4c1", (12, 64, 32, 104), 32, 3, 1, 1, 1),
    ("h5", (12, 16, 128, 416), 1, 3, 1, 1, 1),
    ("h4", (12, 32, 64, 208), 1, 3, 1, 1, 1),
    ("h3", (12, 64, 32, 104), 1, 3, 1, 1, 1),
    ("h2", (12, 128, 16, 52), 1, 3, 1, 1, 1),
]
_only = [a.split("=", 1)[1].split(",") for a in sys.argv if a.startswith("--only=")]
if _only:
    SH = [t for t in SH if t[0] in _only[0]]
def timeit(fn, it=20):
    for _ in range(3): fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it): fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / it
tot = {"fwd": 0, "dgrad": 0, "wgrad": 0}
for name, xs, cout, k, st, pd, rf in SH:
    x = torch.randn(*xs, device="cuda")
    w = torch.randn(cout, xs[1], k, k, device="cuda") * 0.05
    d = ops.conv_desc(xs, tuple(w.shape), st, pd, bool(rf))
    ws = torch.empty(lib().md2_conv2d_workspace_size(C.byref(d)) // 4 + 64, device="cuda")
    ho, wo = ops.out_hw(xs[2], xs[3], k, st, pd)
    y = torch.empty(xs[0], cout, ho, wo, device="cuda")
    dy = torch.randn_like(y); dx = torch.empty_like(x); dw = torch.empty_like(w)
    flops = 2.0 * xs[0] * ho * wo * cout * xs[1] * k * k
    sm = stream_of()
    f = lambda: check(lib().md2_conv2d_fwd(C.byref(d), ptr(x), ptr(w), None, ptr(y), ptr(ws), sm))
    g = lambda: check(lib().md2_conv2d_dgrad(C.byref(d), ptr(dy), ptr(w), ptr(dx), ptr(ws), sm))
    h = lambda: check(lib().md2_conv2d_wgrad(C.byref(d), ptr(x), ptr(dy), ptr(dw), None, ptr(ws), sm))
    tf, tg, th = timeit(f), timeit(g), timeit(h)
    tot["fwd"] += tf; tot["dgrad"] += tg; tot["wgrad"] += th
    print(f"{name:6s} GF {flops/1e9:7.2f}  fwd {tf*1e3:8.1f}us {flops/tf/1e9:6.1f}TF  dgrad {tg*1e3:8.1f}us {flops/tg/1e9:6.1f}TF  wgrad {th*1e3:8.1f}us {flops/th/1e9:6.1f}TF", flush=True)
    if "--miopen" in sys.argv and not rf:   # MIOpen (torch conv, exact fp32) at the same shape
        wt = w.clone()
        tf2 = timeit(lambda: torch.nn.functional.conv2d(x, wt, None, st, pd))
        cb = lambda m: torch.ops.aten.convolution_backward(dy, x, wt, None, [st, st], [pd, pd], [1, 1], False, [0, 0], 1, m)
        tg2, th2 = timeit(lambda: cb([True, False, False])), timeit(lambda: cb([False, True, False]))
        print(f"{'miopen':6s} {'':10s}  fwd {tf2*1e3:8.1f}us {flops/tf2/1e9:6.1f}TF  dgrad {tg2*1e3:8.1f}us {flops/tg2/1e9:6.1f}TF  wgrad {th2*1e3:8.1f}us {flops/th2/1e9:6.1f}TF", flush=True)
print(tot)
