"""Forward-accuracy bisection of the GPU train-step forward (VERDICT r04 "what's next" item 2).

At one configuration (default: BASELINE config 3, B=12 416x128 with the bench's uniform frames)
runs the GPU forward (md2hip.train_loss) and the fp64 / fp32 oracle forward with every GPU branch
decision imposed, and prints, per intermediate tensor (encoder stage outputs, pose convs,
DepthDecoder branch outputs, disparities, poses), the GPU's relative Frobenius error against fp64
next to the fp32 oracle's (the "fp32 floor" of that tensor) and their ratio -- the first tensor
whose ratio jumps locates the kernel that loses accuracy.

    python tools/forward_bisect.py [--batch 12] [--sources uniform] [--out FILE.json]
(knobs such as MD2_TUNING=1 MD2_PX3=0 swap kernels for the A/B.)"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monodepth2.jl_amd")]

import torch
import torch.nn.functional as F

import md2hip
from oracle import md2_oracle as O
from tests import _data as D
from tests import _model_parity as MP


def oracle_intermediates(P, x, arch, levels, source_ids, target_id, dec):
    """fp32 / fp64 oracle forward (decisions imposed), capturing what the GPU exposes."""
    out = {}
    N, L, C, H, W = x.shape
    with O.forced_decisions(dec):
        feats = O.resnet_stages(P, x.reshape(N * L, C, H, W), arch)
        for i, f in enumerate(feats):
            out[f"feat{i}"] = f
        feats = [f.reshape(N, L, *f.shape[1:]) for f in feats]
        tf = [f[:, target_id - 1] for f in feats]
        # DepthDecoder with its intermediates (O.depth_decoder, unrolled)
        xx, skips = tf[-1], tf[:-1][::-1]
        bstart, disps = 1, []
        for slevel in levels:
            for bid in range(bstart, slevel + 1):
                y = O._decoder_block(P, f"depth.branch{bid}.c1", xx, F.elu)
                out[f"depth.branch{bid}.c1"] = y
                y = O.upsample_bilinear_x2(y)
                out[f"depth.branch{bid}.up"] = y
                if bid <= len(skips):
                    y = torch.cat([y, skips[bid - 1]], dim=1)
                xx = O._decoder_block(P, f"depth.branch{bid}.c2", y, F.elu)
                out[f"depth.branch{bid}.c2"] = xx
            disps.append(O._decoder_block(P, f"depth.head{slevel}", xx, torch.sigmoid))
            bstart = slevel + 1
        for s, d in enumerate(disps):
            out[f"disp{s}"] = d
        poses = []
        for j, i in enumerate(source_ids):
            fa, fb = (feats[-1][:, i - 1], feats[-1][:, target_id - 1]) if i < target_id else \
                     (feats[-1][:, target_id - 1], feats[-1][:, i - 1])
            r, t = O.pose_decoder(P, fa, fb, tag=f"pose{j}")
            poses.append(torch.cat([r, t], 1))
        out["pose"] = torch.cat(poses, 0)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=12)
    ap.add_argument("--height", type=int, default=128)
    ap.add_argument("--width", type=int, default=416)
    ap.add_argument("--arch", type=int, default=18)
    ap.add_argument("--sources", default="uniform")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    N, H, W, arch = a.batch, a.height, a.width, a.arch
    levels, target_id, source_ids = (2, 3, 4, 5), 2, (1, 3)
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    x = MP.inputs(N, 3, H, W, a.sources, 7)
    K, invK = D.intrinsics(W, H)
    enc = md2hip.ResNet(arch, in_channels=3)
    model = md2hip.Model(enc, md2hip.DepthDecoder(encoder_channels=enc.stages, scale_levels=list(levels),
                                                  embedding_levels=0), md2hip.PoseDecoder(enc.stages[-1]), seed=42)
    cache = md2hip.TrainCache(K=K.numpy(), invK=invK.numpy(), target_id=target_id, source_ids=source_ids,
                              scales=tuple(MP.DEFAULT_SCALES[l] for l in levels))
    params = md2hip.Params(target_size=(W, H), batch_size=N, automasking=False)
    xg = x.float().cuda().contiguous()
    md2hip.train_loss(model, xg, None, cache, params)
    disps, pose = model._last.outputs()
    torch.cuda.synchronize()
    t = {k: v.cpu() for k, v in model._last.debug_tensors().items()}
    dec = MP.gpu_decisions(model, N, arch, target_id=target_id, source_ids=source_ids)

    def nmajor(v, L=3):
        return v.reshape(L, N, *v.shape[1:]).transpose(0, 1).reshape(L * N, *v.shape[1:])

    g = {"feat0": nmajor(t["stem.out"])}
    nb = O.RESNET_LAYERS[arch]
    for si in range(4):
        g[f"feat{si + 1}"] = nmajor(t[f"layer{si + 1}.{nb[si] - 1}.out"])
    for k, v in t.items():
        if k.startswith("depth.branch"):
            g[k] = v
    for s, d in enumerate(disps):
        g[f"disp{s}"] = d.cpu()
    g["pose"] = pose.cpu()

    spec = O.param_spec(arch, 3, levels)
    flat = model.flat.detach().double().cpu()
    ref = {}
    for dt in (torch.float64, torch.float32):
        P = O.unflatten(flat.to(dt), spec)
        with torch.no_grad():
            ref[dt] = oracle_intermediates(P, x.to(dt), arch, levels, source_ids, target_id, dec)
    rows = []
    order = [k for k in ref[torch.float64] if k in g]
    # z = sum(e) / sqrt(sum(e^2)) of the error e = t - fp64: ~N(0, 1) for unbiased independent
    # roundings, |z| >> 3 for a coherent (biased) error -- what a cancelling gradient sum sees
    def zscore(e):
        e = e.reshape(-1)
        return (e.sum() / e.pow(2).sum().clamp_min(1e-300).sqrt()).item()

    print(f"{'tensor':24s} {'gpu vs fp64':>12s} {'fp32 vs fp64':>13s} {'ratio':>7s} {'z gpu':>9s} {'z fp32':>9s}")
    for k in order:
        r64 = ref[torch.float64][k].double()
        gk = g[k].double().reshape(r64.shape)
        o32 = ref[torch.float32][k].double()
        eg = D.rel_err(gk, r64)
        e32 = D.rel_err(o32, r64)
        zg, z32 = zscore(gk - r64), zscore(o32 - r64)
        rows.append({"tensor": k, "gpu": eg, "fp32": e32, "ratio": eg / max(e32, 1e-30), "z_gpu": zg, "z_fp32": z32})
        print(f"{k:24s} {eg:12.3e} {e32:13.3e} {eg / max(e32, 1e-30):7.2f} {zg:9.1f} {z32:9.1f}", flush=True)
    knobs = {k: v for k, v in os.environ.items() if k.startswith("MD2_")}
    res = {"config": {"batch": N, "height": H, "width": W, "arch": arch, "sources": a.sources},
           "knobs": knobs, "rows": rows}
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
