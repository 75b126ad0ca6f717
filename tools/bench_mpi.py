"""MPI-mode train step on one MI355X (src/model.jl:1-55, src/repeat.jl:44-69):
ResNet-18 encoder + DepthDecoder(embedding_levels=21) over num_bins plane images at batch 1,
4-scale photometric loss with the planes as its batch, full backward (plane_sum = the _repeat
pullback) and ADAM.  Prints one JSON line: samples/s, plane images/s and the HIP-event split of
the step (zero-padded 3x3 convs vs the other convs, e.g. the 32x-batched decoder), each with its
fraction of the fp32 MFMA peak.

    python tools/bench_mpi.py [--bins 32] [--height 128] [--width 416] [--steps 20]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monodepth2.jl_amd")]

PEAK = 157.3   # TFLOP/s, fp32 MFMA (MI355X_MICROARCH.md)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bins", type=int, default=32)
    ap.add_argument("--height", type=int, default=128)
    ap.add_argument("--width", type=int, default=416)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--layers", default="", help="write the per-layer conv table (markdown) here")
    args = ap.parse_args()
    import torch
    import md2hip
    import md2hip.dist
    torch.cuda.set_device(0)
    H, W, nb = args.height, args.width, args.bins
    enc = md2hip.ResNet(18, in_channels=3)
    model = md2hip.Model(enc, md2hip.DepthDecoder(encoder_channels=enc.stages, scale_levels=[2, 3, 4, 5],
                                                  embedding_levels=21),
                         md2hip.PoseDecoder(512), seed=42)
    K, invK = md2hip.depth10k_intrinsics(W, H)
    cache = md2hip.TrainCache(K=K, invK=invK)
    params = md2hip.Params(target_size=(W, H), batch_size=1, automasking=False)
    x = md2hip.dist.synthetic_triplets(1, H, W, 0, torch.device("cuda", 0))
    ex = model.executor(tuple(x.shape), cache, params, nb)
    ex.set_bins(md2hip.disparity_bins(1, nb))
    opt = md2hip.ADAM(1e-4)
    loss = torch.empty(1, dtype=torch.float32, device="cuda")

    def step():
        md2hip.dist.train_step(ex, model, opt, x, loss=loss)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / args.steps * 1e3
    prof = None
    ex.set_profiling(True)
    for _ in range(5):
        step()
        torch.cuda.synchronize()
        p = ex.profile_read()
        prof = p if prof is None else {c: min(prof[c], p[c]) for c in p}
    ex.set_profiling(False)
    if args.layers:
        from collections import defaultdict
        acc = defaultdict(lambda: [0.0, 0.0, 0])
        for _ in range(3):
            ex.set_profiling(True)
            step()
            torch.cuda.synchronize()
            for t, cat, tms, work in ex.profile_records():
                if cat == "photometric":
                    continue
                a = acc[t]
                a[0] += tms / 3
                a[1] = work
                a[2] += 1
            ex.set_profiling(False)
        rows = sorted(acc.items(), key=lambda kv: -kv[1][0])
        lines = [f"# MPI-mode per-layer conv table: {nb} planes, {W}x{H}, batch 1 (HIP events, mean of 3 steps)", "",
                 "| layer pass | calls | GFLOP/call | ms/step | TFLOP/s | % fp32 MFMA peak |", "|---|---|---|---|---|---|"]
        for t, (tms, work, n) in rows:
            per = n / 3
            tf = work * per / (tms * 1e-3) / 1e12 if tms > 0 else 0.0
            lines.append(f"| `{t}` | {per:.0f} | {work / 1e9:.2f} | {tms:.3f} | {tf:.1f} | {100 * tf / PEAK:.1f} |")
        with open(args.layers, "w") as f:
            f.write("\n".join(lines) + "\n")
    out = {"workload": f"MPI train step resnet18, DepthDecoder(embedding_levels=21), batch 1, {nb} planes, "
                       f"{W}x{H}, 4 scales, ADAM",
           "ms_per_step": round(ms, 4), "samples_per_s": round(1e3 / ms, 2),
           "plane_images_per_s": round(nb * 1e3 / ms, 1), "loss": loss.item()}
    for cat in ("conv3x3_encoder", "conv_other"):
        t, flop, n = prof[cat]
        tf = flop / (t * 1e-3) / 1e12 if t > 0 else 0.0
        out[cat] = {"ms_per_step": round(t, 4), "gflop": round(flop / 1e9, 2), "launches": n,
                    "tflops": round(tf, 2), "frac_fp32_mfma": round(tf / PEAK, 4)}
    t, byt, n = prof["photometric"]
    out["photometric"] = {"ms_per_step": round(t, 4), "launches": n}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
