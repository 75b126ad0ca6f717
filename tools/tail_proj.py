"""Where a head-bias gradient's error comes from (GPU box): one model parity run (tests/_model_parity
run()), then per scale the GPU loss tail's d_disparity against the fp64 and fp32 oracle tails
evaluated AT the GPU's outputs with its decisions imposed -- Frobenius error, and the error of
the projection onto sigmoid'(z) = d (1 - d), which is that scale's head-bias gradient (a heavily
cancelling sum).  Then the model's head-bias gradients against the same projections.
    python tools/tail_proj.py CONFIG   (mpi4 | r50 | levels12345)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monodepth2.jl_amd")]
import torch  # noqa: E402

from oracle import md2_oracle as O  # noqa: E402
from tests import _data as D  # noqa: E402
from tests._model_parity import DEFAULT_SCALES, per_tensor, run  # noqa: E402

torch.set_num_threads(16)
cfg = sys.argv[1] if len(sys.argv) > 1 else "mpi4"
kw = {"mpi4": dict(N=1, H=64, W=128, sources="texture", num_bins=4),
      "r50": dict(N=8, H=192, W=640, arch=50, sources="texture"),
      "uniform12": dict(N=12, H=128, W=416, sources="uniform"),
      "levels12345": dict(N=2, H=64, W=128, strict=False, levels=(1, 2, 3, 4, 5), target_id=2,
                          source_ids=(3, 1))}[cfg]
g, o, errs = run(**kw)
x = g["x"]
N, L, C, H, W = x.shape
nb = g["bins"].shape[1] if g.get("bins") is not None else 1
levels = g["levels"]
K, invK = D.intrinsics(W, H)
scales = tuple(DEFAULT_SCALES[l] for l in levels)
forced = [s.unsqueeze(1).long() for s in g["sel"]]


def tail(dt, smooth=1e-3):
    ds = [d.to(dt).clone().requires_grad_(True) for d in g["disps"]]
    pg = g["pose"].to(dt)
    ps = [(pg[k * N:(k + 1) * N, :3].repeat_interleave(nb, 0).clone().requires_grad_(True),
           pg[k * N:(k + 1) * N, 3:].repeat_interleave(nb, 0).clone().requires_grad_(True)) for k in range(2)]
    xt = x.to(dt).repeat_interleave(nb, 0) if nb > 1 else x.to(dt)
    cache = O.TrainCache(K=K.to(dt), invK=invK.to(dt), target_id=g["target_id"],
                         source_ids=g["source_ids"], scales=scales)
    l = O.loss_from_outputs(ds, ps, xt, None, cache, O.Params(target_size=(W, H), batch_size=N * nb,
                                                                automasking=False,
                                                                disparity_smoothness=smooth),
                            forced_sel=forced, forced_cells=g["cells"])
    l.backward()
    return [d.grad.double() for d in ds]


t64, t32 = tail(torch.float64), tail(torch.float32)
for s in range(len(scales)):
    d = g["disps"][s].double()
    sp = d * (1 - d)
    ref = (t64[s] * sp).sum().item()
    mass = (t64[s] * sp).abs().sum().item()
    gp = (g["tail_d_disp"][s].double() * sp).sum().item()
    fp = (t32[s] * sp).sum().item()
    print(f"scale {s} ({tuple(d.shape)}): d_disp gpu {D.rel_err(g['tail_d_disp'][s], t64[s]):.2e} "
          f"fp32 {D.rel_err(t32[s], t64[s]):.2e} | bias-proj f64 {ref:+.4e} (mass {mass:.2e}) "
          f"gpu rel {abs(gp - ref) / abs(ref):.2e} fp32 rel {abs(fp - ref) / abs(ref):.2e}")
    e = (g["tail_d_disp"][s].double() - t64[s])
    print(f"   gpu err: mean {e.mean().item():+.3e} (x count {e.mean().item() * e.numel():+.3e}), "
          f"rms {e.pow(2).mean().sqrt().item():.3e}; proj err {(e * sp).sum().item():+.3e}; "
          f"fp32 err mean {(t32[s] - t64[s]).mean().item():+.3e}")
    top = torch.topk(e.abs().flatten(), 6).indices
    hs, ws = e.shape[-2:]
    print("   worst native pixels (n, y, x, gpu, f64, f32):",
          [(i // (hs * ws), (i % (hs * ws)) // ws, i % ws, f"{g['tail_d_disp'][s].flatten()[i].item():+.3e}",
            f"{t64[s].flatten()[i].item():+.3e}", f"{t32[s].flatten()[i].item():+.3e}") for i in top.tolist()])
    rel = (e / t64[s].abs().clamp_min(1e-30))
    print(f"   gpu err / |g| : mean {rel.mean().item():+.2e} median {rel.median().item():+.2e}; "
          f"corr(err, g) {torch.corrcoef(torch.stack([e.flatten(), t64[s].flatten()]))[0, 1].item():+.3f}")


def gpu_tail(smooth):
    import md2hip
    xt = x.float().cuda().repeat_interleave(nb, 0).contiguous()
    pg = g["pose"].cuda()
    ps = [(pg[k * N:(k + 1) * N, :3].repeat_interleave(nb, 0).contiguous(),
           pg[k * N:(k + 1) * N, 3:].repeat_interleave(nb, 0).contiguous()) for k in range(2)]
    cache = md2hip.TrainCache(K=K.numpy(), invK=invK.numpy(), target_id=g["target_id"],
                              source_ids=g["source_ids"], scales=scales)
    r = md2hip.loss_tail([d.cuda().contiguous() for d in g["disps"]], ps, xt, None, cache,
                         md2hip.Params(target_size=(W, H), batch_size=N * nb, automasking=False,
                                       disparity_smoothness=smooth))
    return [t.cpu().double() for t in r["d_disp"]]


p64 = tail(torch.float64, 0.0)
gp0 = gpu_tail(0.0)
gp1 = gpu_tail(1e-3)
for s in range(len(scales)):
    ep = gp0[s] - p64[s]
    es = (gp1[s] - gp0[s]) - (t64[s] - p64[s])
    bad = (gp1[s] != g["tail_d_disp"][s].double())
    if bad.any():
        idx = bad.nonzero()[:5].tolist()
        print(f"   visualize / plain kernels differ at {int(bad.sum())} pixels, e.g. {idx}: "
              f"{[(g['tail_d_disp'][s][tuple(i)].item(), gp1[s][tuple(i)].item()) for i in idx]}")
    print(f"scale {s}: photometric-only DC err {ep.mean().item():+.2e} (rms {ep.pow(2).mean().sqrt().item():.2e}); "
          f"smoothness-part DC err {es.mean().item():+.2e} (rms {es.pow(2).mean().sqrt().item():.2e}); "
          f"smooth part mean {(t64[s] - p64[s]).mean().item():+.2e}; gpu rerun == model tail: "
          f"{torch.equal(gp1[s], g['tail_d_disp'][s].double())}")
print("model head biases: gpu vs oracle", {k: f"{v:.2e}" for k, v in errs.items() if "head" in k and "bias" in k})
if len(sys.argv) > 2:
    torch.save({"g": {k: v for k, v in g.items() if k not in ("decisions", "flat", "grad")},
                "t64": t64, "t32": t32}, sys.argv[2])
