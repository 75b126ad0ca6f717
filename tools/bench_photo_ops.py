"""HBM roofline of the reference-structured warp + SSIM kernels (the op-level C-ABI that
julia/MD2HIP.jl binds per ChainRulesCore rrule: grid_sample(:border) and SSIM forward and
pullback, src/training.jl:56-59, src/utils.jl:17-43) at the bench's full-resolution scale: B=12
samples x 2 sources, 3 channels, 416x128.  The production step runs the fused single-pass kernel
(photo.hip) instead; this measures how close the per-op kernels of the same path come to the
HBM peak.  Per kernel: median of HIP-event timings over `reps` launches, algorithmic bytes
(each tensor read / written once; the bilinear source image counted once), GB/s and fraction of
the 8 TB/s peak.  One JSON line per kernel.

    python tools/bench_photo_ops.py [reps]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monodepth2.jl_amd")]

PEAK = 8000.0   # GB/s, MI355X HBM3E (MI355X_MICROARCH.md)


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    import torch
    from md2hip._lib import check, lib, ptr, stream_of
    torch.cuda.set_device(0)
    g = torch.Generator(device="cuda").manual_seed(0)
    n, c, h, w = 24, 3, 128, 416            # 12 samples x 2 sources
    px = n * h * w
    src = torch.rand(n, c, h, w, device="cuda", generator=g)
    tgt = torch.rand(n, c, h, w, device="cuda", generator=g)
    # a smooth warp (small shifts) like the training step's, in normalised [-1, 1] coordinates
    ys, xs = torch.meshgrid(torch.linspace(-1, 1, h, device="cuda"), torch.linspace(-1, 1, w, device="cuda"),
                            indexing="ij")
    shift = 0.02 * torch.rand(n, 1, 1, 2, device="cuda", generator=g)
    grid = (torch.stack([xs, ys], -1)[None] * 0.98 + shift).contiguous()
    warped = torch.empty_like(src)
    ssim = torch.empty_like(src)
    dout = torch.rand_like(src)
    dx = torch.empty_like(src)
    dy = torch.empty_like(src)
    dgrid = torch.empty_like(grid)
    st = stream_of()
    B4 = 4
    kernels = {
        # grid (8 B/px) + source image (c*4) read, warped (c*4) written
        "grid_sample_border_fwd": (lambda: lib().md2_grid_sample_border_fwd(
            ptr(src), ptr(grid), n, c, h, w, h, w, ptr(warped), st), px * (8 + 2 * c * B4)),
        # grid + source image + dout read, d_grid written (the d_x scatter is off: frames are data)
        "grid_sample_border_bwd": (lambda: lib().md2_grid_sample_border_bwd(
            ptr(src), ptr(grid), ptr(dout), n, c, h, w, h, w, ptr(dgrid), None, st), px * (8 + 2 * c * B4 + 8)),
        # x, y read, SSIM map written
        "ssim_fwd": (lambda: lib().md2_ssim_fwd(ptr(warped), ptr(tgt), n, c, h, w, ptr(ssim), st),
                     px * c * 3 * B4),
        # x, y, dout read, dx, dy written
        "ssim_bwd": (lambda: lib().md2_ssim_bwd(ptr(warped), ptr(tgt), ptr(dout), n, c, h, w, ptr(dx), ptr(dy),
                                                st), px * c * 5 * B4),
    }
    for name, (fn, byt) in kernels.items():
        for _ in range(5):
            check(fn(), name)
        ts = []
        for _ in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            check(fn(), name)
            b.record()
            b.synchronize()
            ts.append(a.elapsed_time(b))
        t = sorted(ts)[len(ts) // 2]
        gbs = byt / (t * 1e-3) / 1e9
        print(json.dumps({"kernel": name, "shape": f"n={n} c={c} {w}x{h}", "us": round(t * 1e3, 2),
                          "algorithmic_bytes": byt, "GBps": round(gbs, 1), "frac_hbm": round(gbs / PEAK, 4)}),
              flush=True)


if __name__ == "__main__":
    main()
