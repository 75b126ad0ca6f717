"""Dump the GPU loss tail's outputs (loss, d_disp per scale, d_pose, argmin map, bilinear cells)
for seeded inputs to a .pt file, for CPU-side analysis against the oracle (tools/tail_analyze.py).
    python tools/tail_dump.py OUT.pt [sources=uniform|texture|ramp] [N H W]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monodepth2.jl_amd")]
import torch  # noqa: E402

from tests import _data as D  # noqa: E402
from tests._model_parity import inputs  # noqa: E402
from tests.test_gpu_loss import SCALES, _gpu  # noqa: E402

out = sys.argv[1]
src = sys.argv[2] if len(sys.argv) > 2 else "uniform"
N, H, W = (int(v) for v in sys.argv[3:6]) if len(sys.argv) > 5 else (2, 64, 128)
x = inputs(N, 3, H, W, src, 7)
K, invK = D.intrinsics(W, H)
disps = D.disparities(N, H, W, seed=11)
poses = D.poses(N, seed=13)
g = _gpu(disps, poses, x, K, invK, None)
torch.save({"x": x, "disps": disps, "poses": poses, "K": K, "invK": invK, "gpu": g, "scales": SCALES}, out)
print("dumped", out, {k: (tuple(v.shape) if hasattr(v, "shape") else len(v)) for k, v in g.items()})
