"""Golden trajectory of BASELINE config 1 at the reference's length: ``slow_depth``
(src/simple_depth.jl:16-42) -- 500 ADAM(3e-4) iterations on one 416x128 triplet -- from the CPU
oracle (oracle/md2_oracle.py slow_depth_loss + Adam), in fp64 (the reference values) and in fp32
(the floor: what a plain fp32 evaluation of the same loop drifts from fp64).

Two starts, as tests/test_gpu_slow_depth.py sets them up (seed 5, textured frames):
  reference  disp = 0.5, rvec = [0, 0, 0.01], tvec = 0 (src/simple_depth.jl:8-13);
  textured   disparity and poses from tests/_data.py (seeds 9 and 11), fp32-grid values.
Stored per start and precision: the per-iteration loss, the final pose rows, and the final
disparity update disp_500 - disp_0 (float32; the GPU test compares directions and norms).

    python tests/golden/make_slow_depth_traj.py     # rewrites tests/golden/slow_depth_traj_416x128.npz
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
for p in (ROOT, os.path.join(ROOT, "monodepth2.jl_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

from oracle import md2_oracle as O  # noqa: E402
from tests import _data as D  # noqa: E402

H, W, ITERS, SEED = 128, 416, 500, 5


def start(kind):
    """(disp [1,1,H,W], pose rows [2, 6]) of the start, fp32-grid values as float64."""
    if kind == "reference":
        disp = torch.full((1, 1, H, W), 0.5, dtype=torch.float64)
        rows = torch.zeros(2, 6, dtype=torch.float64)
        rows[:, 2] = 0.01
        return disp, rows
    disp = D.disparities(1, H, W, seed=SEED + 4)[-1].float().double()
    rows = torch.zeros(2, 6, dtype=torch.float64)
    for s, (r, t) in enumerate(D.poses(1, seed=SEED + 6)):
        rows[s, :3] = r.float().double()[0]
        rows[s, 3:] = t.float().double()[0]
    return disp, rows


def loop(disp, rows, x, K, invK, dt, iters=ITERS):
    """The reference loop (src/simple_depth.jl:22-42) in dtype dt."""
    opt = O.Adam(eta=3e-4)
    disp = disp.to(dt).clone()
    rv = [rows[s:s + 1, :3].to(dt).clone() for s in range(2)]
    tv = [rows[s:s + 1, 3:].to(dt).clone() for s in range(2)]
    x, K, invK = x.to(dt), K.to(dt), invK.to(dt)
    losses = []
    for _ in range(iters):
        disp.requires_grad_(True)
        for t in rv + tv:
            t.requires_grad_(True)
        loss = O.slow_depth_loss(disp, rv, tv, x, K, invK)
        loss.backward()
        losses.append(loss.item())
        with torch.no_grad():
            opt.step("disp", disp, disp.grad)
            for k, t in enumerate(rv + tv):
                opt.step(f"p{k}", t, t.grad)
        disp = disp.detach()
        rv = [t.detach() for t in rv]
        tv = [t.detach() for t in tv]
    rows_out = torch.cat([torch.cat([r, t], 1) for r, t in zip(rv, tv)], 0)
    return np.array(losses), disp.double(), rows_out.double()


def main():
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    x = D.triplets(1, 3, H, W, seed=SEED, ramp_sources=False)
    K, invK = D.intrinsics(W, H)
    out = {}
    for kind in ("reference", "textured"):
        d0, r0 = start(kind)
        for tag, dt in (("64", torch.float64), ("32", torch.float32)):
            losses, d, r = loop(d0, r0, x, K, invK, dt)
            out[f"{kind}_loss{tag}"] = losses
            out[f"{kind}_rows{tag}"] = r.numpy()
            out[f"{kind}_dupdate{tag}"] = (d - d0).float().numpy()
            print(kind, tag, "loss", losses[0], "->", losses[-1], flush=True)
    np.savez_compressed(os.path.join(HERE, "slow_depth_traj_416x128.npz"), **out)


if __name__ == "__main__":
    main()
