"""Per-layer conv table of the bench step (B=12 416x128 ResNet-18 unless told otherwise): HIP
events around every conv pass on the model stream (md2_model_profile_records), GFLOP, time,
fraction of the fp32 MFMA peak (the reference's arithmetic) and fraction of the ceiling of the
instructions the pass's kernel actually issues (the record's [arith] label: bf16x6 split products
2516 / 6 = 419.3 TFLOP/s fp32-equivalent, fp32 MFMA and VALU 157.3), sorted by time.  Writes
profiles/<tag>_layers.md.

    python tools/layer_table.py <tag> [batch] [steps]"""
import os
import sys
from collections import defaultdict

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
sys.path.insert(0, os.path.join(R, "monodepth2.jl_amd"))
import torch  # noqa: E402

import md2hip  # noqa: E402
import md2hip.dist  # noqa: E402

PEAK = 157.3
CEIL = {"bf16x6": 2516.0 / 6, "fp32": 157.3, "valu": 157.3}
tag = sys.argv[1] if len(sys.argv) > 1 else "cur"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 12
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
H, W = 128, 416
dev = torch.device("cuda", 0)
enc = md2hip.ResNet(18, in_channels=3)
model = md2hip.Model(enc, md2hip.DepthDecoder(encoder_channels=enc.stages, scale_levels=[2, 3, 4, 5],
                                              embedding_levels=0), md2hip.PoseDecoder(512), device=dev, seed=42)
K, invK = md2hip.depth10k_intrinsics(W, H)
cache = md2hip.TrainCache(K=K, invK=invK, scales=(0.125, 0.25, 0.5, 1.0))
params = md2hip.Params(target_size=(W, H), batch_size=B, automasking=False)
opt = md2hip.ADAM(1e-4)
x = md2hip.dist.synthetic_triplets(B, H, W, 0, dev)
ex = model.executor(tuple(x.shape), cache, params)
comm = md2hip.dist.GradAllReduce(force=False)
for _ in range(3):
    md2hip.dist.train_step(ex, model, opt, x, comm)
torch.cuda.synchronize()
acc = defaultdict(lambda: [0.0, 0.0, 0, ""])
for _ in range(steps):
    ex.set_profiling(True)
    md2hip.dist.train_step(ex, model, opt, x, comm)
    torch.cuda.synchronize()
    for t, cat, ms, work in ex.profile_records():
        a = acc[t]
        a[0] += ms / steps
        a[1] = work
        a[2] += 1
        a[3] = cat
    ex.set_profiling(False)
rows = sorted(acc.items(), key=lambda kv: -kv[1][0])
conv = [(t, v) for t, v in rows if v[3] != "photometric"]
tot_ms = sum(v[0] for _, v in conv)
tot_fl = sum(v[1] * v[2] / steps for _, v in conv)
lines = [f"# Per-layer conv table ({tag}): ResNet-18 train step, B={B}, {W}x{H}, 1x MI355X",
         "",
         f"HIP events around every conv pass on the model stream (md2_model_profile_records), mean of {steps} "
         f"profiled steps; `calls` per step.  All convs: **{tot_ms:.3f} ms/step, {tot_fl / 1e9:.1f} GFLOP, "
         f"{tot_fl / (tot_ms * 1e-3) / 1e12:.1f} TFLOP/s = {100 * tot_fl / (tot_ms * 1e-3) / 1e12 / PEAK:.1f}% of "
         f"{PEAK} TFLOP/s fp32 MFMA**.  Tag: pass, kernel/stride (r = reflect pad), Cin->Cout, input HxW, images.",
         "`% fp32 peak`: fp32-equivalent TFLOP/s over 157.3; `% own ceiling`: over the ceiling of the "
         "kernel's issued arithmetic (`arith`: bf16x6 419.3, fp32 MFMA / VALU 157.3) -- the column that "
         "stays below 100%.",
         "", "| layer pass | arith | category | calls | GFLOP/call | ms/step | TFLOP/s | % fp32 peak | % own ceiling | ms lost vs 60% fp32 |",
         "|---|---|---|---|---|---|---|---|---|---|"]
by_arith = defaultdict(lambda: [0.0, 0.0])
for t, (ms, work, n, cat) in conv:
    per = n / steps
    tf = work * per / (ms * 1e-3) / 1e12 if ms > 0 else 0.0
    lost = ms - work * per / (0.6 * PEAK * 1e12) * 1e3
    ar = t.rsplit("[", 1)[1].rstrip("]") if t.endswith("]") else "fp32"
    name = t.rsplit(" [", 1)[0]
    by_arith[ar][0] += ms
    by_arith[ar][1] += work * per
    lines.append(f"| `{name}` | {ar} | {cat} | {per:.0f} | {work / 1e9:.2f} | {ms:.3f} | {tf:.1f} | "
                 f"{100 * tf / PEAK:.1f} | {100 * tf / CEIL.get(ar, PEAK):.1f} | {lost:.3f} |")
lines += ["", "| arith | ms/step | GFLOP/step | TFLOP/s | % fp32 peak | % own ceiling |", "|---|---|---|---|---|---|"]
for ar, (ms, fl) in sorted(by_arith.items()):
    tf = fl / (ms * 1e-3) / 1e12
    lines.append(f"| {ar} | {ms:.3f} | {fl / 1e9:.1f} | {tf:.1f} | {100 * tf / PEAK:.1f} | {100 * tf / CEIL.get(ar, PEAK):.1f} |")
out = os.path.join(R, "profiles", f"{tag}_layers.md")
with open(out, "w") as f:
    f.write("\n".join(lines) + "\n")
print("\n".join(lines[:12]))
print("wrote", out)
