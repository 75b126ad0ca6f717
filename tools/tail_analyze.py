"""CPU analysis of a tools/tail_dump.py file: the GPU loss-tail gradients against the fp64 oracle
and the fp32 oracle, both with the GPU's argmin and bilinear cells imposed, per scale; for the
full-resolution scale the per-pixel error distribution and the worst pixels.
    python tools/tail_analyze.py DUMP.pt"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monodepth2.jl_amd")]
import torch  # noqa: E402

from oracle import md2_oracle as O  # noqa: E402
from tests import _data as D  # noqa: E402

d = torch.load(sys.argv[1], weights_only=False)
g = d["gpu"]
x, disps, poses, K, invK, SC = d["x"], d["disps"], d["poses"], d["K"], d["invK"], d["scales"]
N, L, C, H, W = x.shape
sel = [g["vis_sel"][s].unsqueeze(1).long() for s in range(len(SC))]
cells = g["vis_cell"]


def tail(dt):
    ds = [a.to(dt).clone().requires_grad_(True) for a in disps]
    ps = [(r.to(dt).clone().requires_grad_(True), t.to(dt).clone().requires_grad_(True)) for r, t in poses]
    l = O.loss_from_outputs(ds, ps, x.to(dt), None, O.TrainCache(K=K.to(dt), invK=invK.to(dt), scales=SC),
                            O.Params(target_size=(W, H), batch_size=N, automasking=False),
                            forced_sel=sel, forced_cells=cells)
    l.backward()
    return l.item(), [a.grad.double() for a in ds], torch.cat([torch.cat([r.grad, t.grad], 1) for r, t in ps]).double()


l64, g64, p64 = tail(torch.float64)
l32, g32, p32 = tail(torch.float32)
print(f"loss gpu {g['loss'].item():.8f} f64 {l64:.8f} f32 {l32:.8f}")
for s in range(len(SC)):
    print(f"scale {s}: d_disp gpu {D.rel_err(g['d_disp'][s], g64[s]):.2e}  fp32-oracle {D.rel_err(g32[s], g64[s]):.2e}")
print(f"d_pose gpu {D.rel_err(g['d_pose'], p64):.2e}  fp32-oracle {D.rel_err(p32, p64):.2e}")
s = int(os.environ.get("SCALE", len(SC) - 1))
e = (g["d_disp"][s].double() - g64[s]).abs().flatten()
e32 = (g32[s] - g64[s]).abs().flatten()
rms = g64[s].pow(2).mean().sqrt().item()
print(f"scale {s}: rms |g| {rms:.3e}; gpu err quantiles (/rms)",
      [f"{q:.1e}" for q in (torch.quantile(e, torch.tensor([0.5, 0.9, 0.99, 0.999, 1.0], dtype=e.dtype)) / rms).tolist()])
print("           fp32-oracle err quantiles (/rms)",
      [f"{q:.1e}" for q in (torch.quantile(e32, torch.tensor([0.5, 0.9, 0.99, 0.999, 1.0], dtype=e.dtype)) / rms).tolist()])
top = torch.topk(e, 10).indices
for i in top.tolist():
    hs, ws = g64[s].shape[-2:]
    n, r = divmod(i, hs * ws)
    yy, xx = divmod(r, ws)
    cs = cells[s, :, n, yy, xx] if hs == H else cells[s, :, n, 0, 0]
    print(f"  n{n} ({yy},{xx}) g64 {g64[s].flatten()[i]:+.3e} gpu {g['d_disp'][s].flatten()[i].item():+.3e} "
          f"f32 {g32[s].flatten()[i]:+.3e} sel {sel[s][n, 0, yy, xx].item() if hs == H else '-'} states {[(c.item() >> 22) & 15 for c in cs]}")
