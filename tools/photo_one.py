"""Run the loss tail (4-scale photometric + smoothness, fwd+bwd) at the bench shape a few times --
for rocprofv3 kernel timing / counter collection of photometric_kernel in isolation.
usage: python tools/photo_one.py [N] [iters]"""
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
sys.path.insert(0, os.path.join(R, "monodepth2.jl_amd"))
import torch  # noqa: E402

import md2hip  # noqa: E402
from tests import _data as D  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 12
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 10
C, H, W = 3, 128, 416
SCALES = (0.125, 0.25, 0.5, 1.0)
dev = torch.device("cuda")
x = D.triplets(N, C, H, W, seed=7, ramp_sources=False).float().to(dev).contiguous()
K, invK = D.intrinsics(W, H)
disps = [d.float().to(dev).contiguous() for d in D.disparities(N, H, W, seed=11)]
poses = [(a.float().to(dev), b.float().to(dev)) for a, b in D.poses(N, seed=13)]
cache = md2hip.TrainCache(K=K.numpy(), invK=invK.numpy(), scales=SCALES)
params = md2hip.Params(target_size=(W, H), batch_size=N, automasking=False,
                       disparity_smoothness=1e-3)
start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for it in range(iters):
    if it == 2:
        start.record()
    md2hip.loss_tail(disps, poses, x, None, cache, params)
end.record()
torch.cuda.synchronize()
print(f"loss tail {start.elapsed_time(end) / max(iters - 2, 1) * 1e3:.1f} us/iter (N={N})")
