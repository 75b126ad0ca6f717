"""Independent fp32 evaluations of the reference step vs the fp64 oracle (parity diagnostics).

The end-to-end "fp32 floor" of a parameter tensor's gradient is the error of a plain fp32
evaluation of the reference against fp64.  One evaluation is one sample of that error; for the
cancelling sums (a head's bias gradient sums ~1e6 pixel gradients of both signs) the samples
scatter by large factors.  This runs, with every GPU branch decision imposed and on the same
inputs and parameters:
  md2     this library's train step on the GPU (the product);
  cpu32   the oracle in fp32 on the CPU (torch / oneDNN kernels);
  gpu32   the same oracle in fp32 on the GPU (torch / MIOpen kernels, TF32 off);
  gpu64   the oracle in fp64 on the GPU (a check of the fp64 reference itself),
all against the fp64 oracle on the CPU, and prints per tensor the three fp32 errors.

    python tools/fp32_realizations.py [--batch 12] [--sources uniform] [--out FILE.json]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monodepth2.jl_amd")]

import torch

from tests import _model_parity as MP


def to_dev(v, dev):
    if isinstance(v, torch.Tensor):
        return v.to(dev)
    if isinstance(v, dict):
        return {k: to_dev(x, dev) for k, x in v.items()}
    if isinstance(v, list):
        return [to_dev(x, dev) for x in v]
    if isinstance(v, tuple):
        return tuple(to_dev(x, dev) for x in v)
    return v


def on_gpu_oracle(g, dt, kw):
    torch.backends.cudnn.allow_tf32 = False
    torch.backends.cuda.matmul.allow_tf32 = False
    gd = to_dev(g, "cuda")
    with torch.device("cuda"):
        grad, fwd, loss, _ = MP._oracle_grad(gd, dt, **kw)
    torch.cuda.synchronize()
    return grad.cpu(), loss


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=12)
    ap.add_argument("--height", type=int, default=128)
    ap.add_argument("--width", type=int, default=416)
    ap.add_argument("--arch", type=int, default=18)
    ap.add_argument("--sources", default="uniform")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    g, o, e_md2 = MP.run(N=a.batch, H=a.height, W=a.width, arch=a.arch, strict=False, sources=a.sources)
    kw = dict(arch=a.arch, levels=(2, 3, 4, 5), target_id=2, source_ids=(1, 3))
    g32, _, l32, spec = MP._oracle_grad(g, torch.float32, **kw)
    e_cpu32 = MP.per_tensor(spec, g32, o["grad"])
    gg32, _ = on_gpu_oracle(g, torch.float32, kw)
    e_gpu32 = MP.per_tensor(spec, gg32, o["grad"])
    gg64, _ = on_gpu_oracle(g, torch.float64, kw)
    e_gpu64 = MP.per_tensor(spec, gg64, o["grad"])
    # more independent fp32 realisations of the same function: the samples reordered (every
    # batch reduction adds in another order), on the GPU and on the CPU
    N = a.batch
    perms = [list(range(N))[::-1], [(3 * i + 1) % N for i in range(N)] if N % 3 else list(range(1, N)) + [0]]
    e_perm = []
    for pi, perm in enumerate(perms):
        gp = MP.permute_samples(g, perm)
        gg, _ = on_gpu_oracle(gp, torch.float32, kw)
        e_perm.append(("gpu32_perm%d" % pi, MP.per_tensor(spec, gg, o["grad"])))
        gc, _, _, _ = MP._oracle_grad(gp, torch.float32, **kw)
        e_perm.append(("cpu32_perm%d" % pi, MP.per_tensor(spec, gc, o["grad"])))
        gc64, _, _, _ = MP._oracle_grad(gp, torch.float64, **kw)
        e_perm.append(("cpu64_perm%d" % pi, MP.per_tensor(spec, gc64, o["grad"])))
    rows = []
    for k in e_md2:
        fl = max(e_cpu32[k], e_gpu32[k])
        r = {"tensor": k, "md2": e_md2[k], "cpu32": e_cpu32[k], "gpu32": e_gpu32[k], "gpu64": e_gpu64[k]}
        for name, e in e_perm:
            r[name] = e[k]
        f32s = [r[c] for c in r if "32" in c]
        r["fp32_rms"] = (sum(v * v for v in f32s) / len(f32s)) ** 0.5
        r["fp32_max"] = max(f32s)
        r["md2_over_max_fp32"] = e_md2[k] / max(r["fp32_max"], 1e-30)
        r["md2_over_rms_fp32"] = e_md2[k] / max(r["fp32_rms"], 1e-30)
        rows.append(r)
    rows.sort(key=lambda r: -r["md2_over_rms_fp32"])
    cols = ["md2", "cpu32", "gpu32"] + [n for n, _ in e_perm if "32" in n] + ["fp32_rms", "md2_over_rms_fp32", "md2_over_max_fp32"]
    print(f"{'tensor':30s} " + " ".join(f"{c[:10]:>10s}" for c in cols))
    for r in rows:
        print(f"{r['tensor']:30s} " + " ".join(f"{r[c]:10.2e}" for c in cols))
    print("fp64 realisations (gpu64, cpu64 permuted) worst:", max(r["gpu64"] for r in rows),
          max(r[n] for r in rows for n, _ in e_perm if "64" in n))
    worst = {c: max(r[c] for r in rows) for c in ("md2", "cpu32", "gpu32", "gpu64", "fp32_rms")}
    print("worst:", worst)
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"config": vars(a), "rows": rows, "worst": worst}, f, indent=1)


if __name__ == "__main__":
    main()
