"""Time the fused MINE render_tgt_rgb_depth kernel (md2_render_tgt_rgb_depth, src/render.jl:96-114)
with HIP events on its stream, and the unfused reference chain of our own ops (pack -> sample ->
clamp -> plane_volume_rendering) for comparison.  Algorithmic bytes: 28 B read (7 channels) + 4 B
written (depth volume) per pixel and plane, + 16 B per pixel (rgb out, mask).

    python tools/bench_mine.py [out.json]"""
import json
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
sys.path.insert(0, os.path.join(R, "monodepth2.jl_amd"))
import torch  # noqa: E402

import md2hip  # noqa: E402
from md2hip import render as Rn  # noqa: E402

PEAK_HBM = 8.0e12


def timed(fn, iters=50, warm=5):
    for _ in range(warm):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def case(B, N, H, W):
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    rgb = torch.rand(B, N, 3, H, W, device=dev, generator=g)
    sigma = torch.rand(B, N, 1, H, W, device=dev, generator=g)
    xyz = torch.rand(B, N, H, W, 3, device=dev, generator=g)
    disp = torch.linspace(1.0, 0.001, N, device=dev).repeat(B, 1).contiguous()
    pose = md2hip.Pose(0.05 * torch.randn(B, 3, device=dev, generator=g), 0.1 * torch.randn(B, 3, device=dev, generator=g))
    f = 2648.0 / 4.63461538462
    K = [[f, 0, W / 2], [0, f, H / 2], [0, 0, 1]]
    iK = torch.linalg.inv(torch.tensor(K, dtype=torch.float64)).tolist()
    fused = timed(lambda: Rn.render_tgt_rgb_depth(rgb, sigma, disp, xyz, pose, iK, K))

    def chain():
        packed = torch.cat([rgb, sigma, xyz.permute(0, 1, 4, 2, 3)], 2).reshape(B * N, 7, H, W).contiguous()
        tgt, valid = Rn.sample(packed, (1.0 / disp).contiguous(), pose, K, iK)
        tgt = tgt.view(B, N, 7, H, W)
        s = tgt[:, :, 3:4]
        s = (s * (s >= 0)).contiguous()
        Rn.plane_volume_rendering(tgt[:, :, 0:3].contiguous(), s, tgt[:, :, 4:7].permute(0, 1, 3, 4, 2).contiguous())
        valid.view(B, N, H, W).sum(1)
    unfused = timed(chain, iters=10)
    alg = B * N * H * W * 32 + B * H * W * 16
    return {"B": B, "N": N, "H": H, "W": W, "fused_ms": round(fused, 4), "op_chain_ms": round(unfused, 4),
            "algorithmic_bytes": alg, "fused_GBps": round(alg / (fused * 1e-3) / 1e9, 1),
            "fused_frac_hbm": round(alg / (fused * 1e-3) / PEAK_HBM, 3)}


def main():
    out = {"kernel": "md2::mine_render_kernel (render_tgt_rgb_depth, fused)", "peak_GBps": PEAK_HBM / 1e9,
           "cases": [case(2, 32, 100, 200), case(2, 32, 256, 384), case(8, 32, 256, 384), case(4, 64, 384, 640)]}
    for c in out["cases"]:
        print(c, flush=True)
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
