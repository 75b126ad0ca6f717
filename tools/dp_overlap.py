"""DP overlap budget from a world-1 step: per backward segment (= gradient
bucket of the RCCL all-reduce, md2_model_backward_allreduce) its gradient bytes, its own
backward time, and the backward time still REMAINING after it (the window its all-reduce can hide
in), against that bucket's ring all-reduce time at 8 ranks for assumed RCCL bus bandwidths.
    python tools/dp_overlap.py [OUT.json] [--arch 18|50 --height H --width W --batch B]
Defaults: BASELINE config 4's per-rank workload (ResNet-18 416x128, 12 triplets); config 5 is
--arch 50 --height 192 --width 640 --batch 8."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monodepth2.jl_amd")]
import torch  # noqa: E402

import md2hip  # noqa: E402
from md2hip.dist import synthetic_triplets  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("out", nargs="?")
ap.add_argument("--arch", type=int, default=18)
ap.add_argument("--height", type=int, default=128)
ap.add_argument("--width", type=int, default=416)
ap.add_argument("--batch", type=int, default=12)
args = ap.parse_args()
B, H, W, RANKS = args.batch, args.height, args.width, 8
BUSBW = (150.0, 300.0, 600.0)     # GB/s: one xGMI link .. RCCL multi-channel over the 7 links
LAT_US = 25.0                     # per-collective latency assumed for small buckets
names = ["pose+depth decoders", "layer4", "layer3", "layer2", "layer1", "stem"]

enc = md2hip.ResNet(args.arch, in_channels=3)
model = md2hip.Model(enc, md2hip.DepthDecoder(encoder_channels=enc.stages, scale_levels=[2, 3, 4, 5],
                                              embedding_levels=0), md2hip.PoseDecoder(enc.stages[-1]), seed=42)
K, invK = md2hip.depth10k_intrinsics(W, H)
cache = md2hip.TrainCache(K=K, invK=invK)
params = md2hip.Params(target_size=(W, H), batch_size=B, automasking=False)
ex = model.executor((B, 3, 3, H, W), cache, params)
x = synthetic_triplets(B, H, W, 0, "cuda")
rows = None
samples = []
for it in range(8):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(ex.nseg + 2)]
    ev[0].record()
    ex.forward_loss(x)
    ev[1].record()
    rng = []
    for k in range(ex.nseg):
        rng.append(ex.backward_segment(k))
        ev[k + 2].record()
    torch.cuda.synchronize()
    if it >= 3:
        samples.append([ev[k + 1].elapsed_time(ev[k + 2]) for k in range(ex.nseg)] + [ev[0].elapsed_time(ev[1])])
med = [sorted(s[k] for s in samples)[len(samples) // 2] for k in range(ex.nseg + 1)]
seg_ms, fwd_ms = med[:ex.nseg], med[ex.nseg]
out = {"arch": args.arch, "batch_per_gpu": B, "size": [W, H], "ranks": RANKS, "forward_ms": fwd_ms,
       "backward_ms": sum(seg_ms), "busbw_GBps": BUSBW, "latency_us": LAT_US, "buckets": []}
for k, (off, ln) in enumerate(rng):
    bytes_ = 4 * ln
    remaining = sum(seg_ms[k + 1:])
    ar = {str(b): LAT_US / 1e3 + 2 * (RANKS - 1) / RANKS * bytes_ / (b * 1e9) * 1e3 for b in BUSBW}
    out["buckets"].append({"segment": k, "name": names[k] if k < len(names) else str(k),
                           "MB": bytes_ / 1e6, "segment_ms": seg_ms[k], "remaining_backward_ms": remaining,
                           "allreduce_ms": ar,
                           "hidden": {b: ar[b] <= remaining for b in ar}})
# the buckets run back to back on the comm stream: the exposed tail is what the last collectives
# add after the backward ends (a queue of collectives, each starting when its segment is done)
for b in map(str, BUSBW):
    t_free = 0.0
    t_seg_end = 0.0
    for k in range(len(rng)):
        t_seg_end += seg_ms[k]
        t_free = max(t_free, t_seg_end) + out["buckets"][k]["allreduce_ms"][b]
    out.setdefault("exposed_ms", {})[b] = max(0.0, t_free - t_seg_end)
print(json.dumps(out, indent=1))
if args.out:
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)
