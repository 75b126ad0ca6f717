"""Accuracy of the slow_depth pose gradient (config 1) per entry: the GPU (md2hip.SlowDepth,
the fused photometric kernel) and the oracle in fp32 (CPU, and torch on the GPU) against the
fp64 oracle, with the GPU's per-pixel source choice imposed -- at the textured start of
tests/test_gpu_slow_depth.py (seed 5) and after a few ADAM steps.

    python tools/pose_grad_acc.py [--height 64] [--width 128] [--steps 0,4,8]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monodepth2.jl_amd")]

import torch

from oracle import md2_oracle as O
from tests import _data as D
from tests.test_gpu_slow_depth import _setup


def oracle(sd, x, K, invK, sel, dt, dev="cpu", cells=None):
    N = sd.N
    with torch.device(dev):
        disp = sd.disp.detach().to(dev, dt).clone().requires_grad_(True)
        rows = sd.pose_rows.detach().to(dev, dt)
        rv = [rows[s * N:(s + 1) * N, :3].clone().requires_grad_(True) for s in range(2)]
        tv = [rows[s * N:(s + 1) * N, 3:].clone().requires_grad_(True) for s in range(2)]
        loss = O.slow_depth_loss(disp, rv, tv, x.to(dev, dt), K.to(dev, dt), invK.to(dev, dt),
                                 forced_sel=sel.to(dev), forced_cells=None if cells is None else cells.to(dev))
        loss.backward()
        dpose = torch.cat([torch.cat([r.grad, t.grad], 1) for r, t in zip(rv, tv)], 0)
    return disp.grad.double().cpu(), dpose.double().cpu()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--height", type=int, default=64)
    ap.add_argument("--width", type=int, default=128)
    ap.add_argument("--steps", default="0,1,4,8")
    a = ap.parse_args()
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    sd, x, K, invK = _setup(1, a.height, a.width, seed=5, strict=False, textured_theta=True)
    done = 0
    for target in [int(v) for v in a.steps.split(",")]:
        while done < target:
            sd.step()
            done += 1
        r = sd.evaluate(visualize=True)
        torch.cuda.synchronize()
        sel = r["vis_sel"][0].cpu().unsqueeze(1).long()
        g_d, g_p = r["d_disp"][0].double().cpu(), r["d_pose"].double().cpu()
        d64, p64 = oracle(sd, x, K, invK, sel, torch.float64)
        d32, p32 = oracle(sd, x, K, invK, sel, torch.float32)
        dg32, pg32 = oracle(sd, x, K, invK, sel, torch.float32, "cuda")
        cells = r["vis_cell"][0].cpu()
        dc64, pc64 = oracle(sd, x, K, invK, sel, torch.float64, cells=cells)
        print(f"   with the GPU's bilinear cells imposed: d_pose gpu {D.rel_err(g_p, pc64):.2e}, d_disp gpu "
              f"{D.rel_err(g_d.reshape(dc64.shape), dc64):.2e}; decisions that differ from fp64's move d_pose "
              f"by {D.rel_err(pc64, p64):.2e}")
        print(f"after {done} steps: d_pose rel err  gpu {D.rel_err(g_p, p64):.2e}  cpu32 {D.rel_err(p32, p64):.2e}  "
              f"gpu32(torch) {D.rel_err(pg32, p64):.2e};  d_disp  gpu {D.rel_err(g_d.reshape(d64.shape), d64):.2e}  "
              f"cpu32 {D.rel_err(d32, d64):.2e}  gpu32 {D.rel_err(dg32, d64):.2e}")
        print("   per entry |gpu - fp64| / |fp64|:", ((g_p - p64).abs() / p64.abs()).numpy().round(7).tolist())
        print("   per entry |cpu32 - fp64| / |fp64|:", ((p32 - p64).abs() / p64.abs()).numpy().round(7).tolist())
        print("   fp64 d_pose:", p64.numpy().tolist())


if __name__ == "__main__":
    main()
