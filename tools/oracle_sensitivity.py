"""Conditioning of the exact train_loss gradient (fp64 oracle): relative change of loss and
gradients under a tiny relative perturbation of the disparities, with the argmin held fixed.
Sets the floor for fp32-vs-fp64 gradient parity on textured inputs (tests/test_gpu_loss.py)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from tests import _data as D  # noqa: E402
from tests.test_gpu_loss import _oracle  # noqa: E402

N, C, H, W = 1, 3, 128, 416
x = D.triplets(N, C, H, W, seed=7)
K, invK = D.intrinsics(W, H)
disps = D.disparities(N, H, W, seed=11)
poses = D.poses(N, seed=13)
l0, d0, p0, per = _oracle(disps, poses, x, K, invK, None)
sel = [(per[s][1] < per[s][0]).long() for s in range(4)]
for eps in (1e-7, 1e-6):
    g = torch.Generator().manual_seed(1)
    dp = [d * (1 + eps * torch.randn(d.shape, generator=g, dtype=d.dtype)) for d in disps]
    l1, d1, p1, _ = _oracle(dp, poses, x, K, invK, None, forced_sel=sel)
    print(f"eps {eps:g}: loss {abs(l1 - l0).item() / l0.item():.2e}  d_disp "
          f"{[f'{D.rel_err(d1[s], d0[s]):.1e}' for s in range(4)]}  d_pose {D.rel_err(p1, p0):.1e}")
