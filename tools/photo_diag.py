"""Where does the loss-tail d_disparity differ from the fp64 oracle?  Per scale: relative error,
and the error energy by column position in the 60-wide wave tiles, image edges and rows.
usage: python tools/photo_diag.py [N] [H] [W] [strict]"""
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
sys.path.insert(0, os.path.join(R, "monodepth2.jl_amd"))
import torch  # noqa: E402

from tests import _data as D  # noqa: E402
from tests.test_gpu_loss import SCALES, _gpu, _oracle  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1
H = int(sys.argv[2]) if len(sys.argv) > 2 else 128
W = int(sys.argv[3]) if len(sys.argv) > 3 else 416
strict = (sys.argv[4] != "0") if len(sys.argv) > 4 else True
x = D.triplets(N, 3, H, W, seed=7, ramp_sources=strict)
K, invK = D.intrinsics(W, H)
disps = D.disparities(N, H, W, seed=11)
poses = D.poses(N, seed=13)
g = _gpu(disps, poses, x, K, invK, None)
forced = [g["vis_sel"][s].unsqueeze(1).long() for s in range(len(SCALES))]
lo, dd_o, dp_o, _ = _oracle(disps, poses, x, K, invK, None, forced_sel=forced)
print(f"loss gpu {g['loss'].item():.8f} oracle {lo.item():.8f}")
for s in range(len(SCALES)):
    a, b = g["d_disp"][s].double(), dd_o[s].double()
    e = (a - b)
    print(f"scale {s} shape {tuple(a.shape)} rel {D.rel_err(a, b):.3e}")
    full = g["vis_sel"][s]
print("d_pose rel", D.rel_err(g["d_pose"], dp_o))
# full-res gradient map before the upsample adjoint is internal; look at the full-res scale
a, b = g["d_disp"][3].double()[:, 0], dd_o[3].double()[:, 0]
e2 = (a - b) ** 2
tot = e2.sum().item()
cols = torch.arange(W)
for name, m in [("col%60 in {0,1}", (cols % 60) < 2), ("col%60 in {58,59}", (cols % 60) >= 58),
                ("col 0..1", cols < 2), ("col W-2..W-1", cols >= W - 2)]:
    print(f"  {name:20s} share of error energy {e2[..., m].sum().item() / tot:.3f} (share of cols {m.float().mean():.3f})")
rows = torch.arange(H)
for name, m in [("row 0..1", rows < 2), ("row H-2..", rows >= H - 2), ("row%8 in {0,7}", (rows % 8 == 0) | (rows % 8 == 7))]:
    print(f"  {name:20s} share of error energy {e2[:, m].sum().item() / tot:.3f} (share of rows {m.float().mean():.3f})")
idx = torch.topk(e2.flatten(), 10).indices
for i in idx.tolist():
    n_, r_ = divmod(i, H * W)
    y, xx = divmod(r_, W)
    print(f"  worst n={n_} y={y} x={xx} gpu {a[n_, y, xx].item():.4e} ref {b[n_, y, xx].item():.4e}")
