"""Which full-resolution pixels carry a scale's gradient error (GPU box).  One model parity run
(tests/_model_parity run()), then the loss tail again with scale S's disparity upsampled to full
resolution beforehand (so the GPU returns its full-res gradient), against the fp64 oracle with the
GPU's decisions imposed; prints the worst pixels with their decisions and the oracle's values at
each branch point (per-source loss, |target - warped| per channel, SSIM before the clamp).
    python tools/scale0_probe.py CONFIG [S]    (CONFIG as tools/tail_proj.py)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monodepth2.jl_amd")]
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import md2hip  # noqa: E402
from oracle import md2_oracle as O  # noqa: E402
from tests import _data as D  # noqa: E402
from tests._model_parity import DEFAULT_SCALES, run  # noqa: E402

torch.set_num_threads(16)
cfg = sys.argv[1] if len(sys.argv) > 1 else "uniform12"
S = int(sys.argv[2]) if len(sys.argv) > 2 else 0
kw = {"uniform12": dict(N=12, H=128, W=416, sources="uniform"),
      "mpi4": dict(N=1, H=64, W=128, sources="texture", num_bins=4)}[cfg]
g, o, errs = run(**kw)
x = g["x"]
N, L, C, H, W = x.shape
K, invK = D.intrinsics(W, H)
scales = tuple(DEFAULT_SCALES[l] for l in g["levels"])
disps = [d.cuda() for d in g["disps"]]


def kernel_upsample(d):
    """The photometric kernel's own fp32 upsample (photo.hip issue_disp / the rx, ry of
    loss_tail.cpp ratio()), fmaf emulated in fp64 (a*b exact, one rounding of the sum)."""
    import numpy as np
    d = d.cpu().numpy().astype(np.float32)
    n_, _, dh, dw = d.shape
    f32 = np.float32
    rx, ry = f32(dw - 1) / f32(W - 1), f32(dh - 1) / f32(H - 1)
    X = np.arange(W, dtype=np.float32)
    Y = np.arange(H, dtype=np.float32)
    usx = (rx * X).astype(f32)
    ux0 = np.minimum(usx.astype(np.int64), dw - 1)
    ux1 = np.minimum(ux0 + 1, dw - 1)
    ufx = (usx - ux0.astype(f32)).astype(f32)
    sy = (ry * Y).astype(f32)
    uy0 = np.minimum(sy.astype(np.int64), dh - 1)
    uy1 = np.minimum(uy0 + 1, dh - 1)
    fy = (sy - uy0.astype(f32)).astype(f32)

    def fma(a, b, c):
        return (a.astype(np.float64) * b.astype(np.float64) + c.astype(np.float64)).astype(f32)
    out = np.empty((n_, 1, H, W), dtype=f32)
    for n in range(n_):
        a = d[n, 0]
        d00, d01 = a[uy0][:, ux0], a[uy0][:, ux1]
        d10, d11 = a[uy1][:, ux0], a[uy1][:, ux1]
        top = fma(ufx[None, :], (d01 - d00).astype(f32), d00)
        bot = fma(ufx[None, :], (d11 - d10).astype(f32), d10)
        out[n, 0] = fma(fy[:, None], (bot - top).astype(f32), top)
    return torch.from_numpy(out).cuda()


disps[S] = kernel_upsample(disps[S]).contiguous()
pg = g["pose"].cuda()
ps = [(pg[k * N:(k + 1) * N, :3].contiguous(), pg[k * N:(k + 1) * N, 3:].contiguous()) for k in range(2)]
cache = md2hip.TrainCache(K=K.numpy(), invK=invK.numpy(), scales=scales)
prm = md2hip.Params(target_size=(W, H), batch_size=N, automasking=False)
r = md2hip.loss_tail(disps, ps, x.float().cuda().contiguous(), None, cache, prm, visualize=True)
torch.cuda.synchronize()
gd = r["d_disp"][S].cpu().double()
sel = [v.unsqueeze(1).long() for v in r["vis_sel"].cpu()]
cells = r["vis_cell"].cpu()

ds = [d.cpu().double().clone().requires_grad_(True) for d in disps]
pos = [(a.cpu().double().clone().requires_grad_(True), b.cpu().double().clone().requires_grad_(True)) for a, b in ps]
ocache = O.TrainCache(K=K, invK=invK, scales=scales)
l = O.loss_from_outputs(ds, pos, x, None, ocache, O.Params(target_size=(W, H), batch_size=N, automasking=False),
                        forced_sel=sel, forced_cells=cells)
l.backward()
go = ds[S].grad
e = (gd - go).abs()
print(f"scale {S} full-res gradient: rel err {D.rel_err(gd, go):.2e}; rms |g| {go.pow(2).mean().sqrt():.2e}")
top = torch.topk(e.flatten(), 12).indices
Ps = O.poses_to_transforms([(a.detach(), b.detach()) for a, b in pos], (1, 3), 2)
warped = O.warp(ds[S].detach(), x, Ps, K, invK, (1, 3), 0.1, 100.0, cells=cells[S])
tgt = x[:, 1]
pool = lambda t: F.avg_pool2d(t, 3, stride=1)  # noqa: E731
ssim_raw = []
for p in warped:
    xr, yr = O.pad_reflect(p), O.pad_reflect(tgt)
    mx, my = pool(xr), pool(yr)
    sx, sy, sxy = pool(xr * xr) - mx * mx, pool(yr * yr) - my * my, pool(xr * yr) - mx * my
    ssim_raw.append((1 - (2 * mx * my + 1e-4) * (2 * sxy + 9e-4) / ((mx * mx + my * my + 1e-4) * (sx + sy + 9e-4))) * 0.5)
for i in top.tolist():
    n, rr = divmod(i, H * W)
    yy, xx = divmod(rr, W)
    c = [int(cells[S, j, n, yy, xx].item()) & 0xFFFFFFFF for j in range(2)]
    print(f"  n{n} ({yy},{xx}) gpu {gd[n, 0, yy, xx]:+.4e} f64 {go[n, 0, yy, xx]:+.4e} sel {sel[S][n, 0, yy, xx].item()} "
          f"states {[(v >> 22) & 15 for v in c]} l1 {[bin(v >> 26) for v in c]} "
          f"|t-p| {[[f'{v:.1e}' for v in (tgt[n, :, yy, xx] - w_[n, :, yy, xx]).abs().tolist()] for w_ in warped]} "
          f"ssim-term {[f'{s_[n, :, yy, xx].min().item():.3f}..{s_[n, :, yy, xx].max().item():.3f}' for s_ in ssim_raw]}")

# the same tail with scale S at its native resolution (what the model runs): its native gradient
# against the fp64 adjoint of the full-res GPU gradient above (isolates the upsample adjoint)
nat = [d.cuda() for d in g["disps"]]
r2 = md2hip.loss_tail(nat, ps, x.float().cuda().contiguous(), None, cache, prm, visualize=True)
torch.cuda.synchronize()
gn = r2["d_disp"][S].cpu().double()
d0 = g["disps"][S].double().clone().requires_grad_(True)
up = F.interpolate(d0, size=(H, W), mode="bilinear", align_corners=True)
(up * gd).sum().backward()
adj = d0.grad
e2 = (gn - adj).abs()
print(f"native gradient vs fp64 adjoint of the full-res GPU gradient: rel {D.rel_err(gn, adj):.2e}")
hs, ws = gn.shape[-2:]
for i in torch.topk(e2.flatten(), 6).indices.tolist():
    n, rr = divmod(i, hs * ws)
    yy, xx = divmod(rr, ws)
    print(f"  n{n} ({yy},{xx}) native {gn[n, 0, yy, xx]:+.4e} adjoint {adj[n, 0, yy, xx]:+.4e}")
cells_n = r2["vis_cell"].cpu()[S]
print("cells differ (native vs full-res input):", int((cells_n != cells[S]).sum()),
      "sel differ:", int((r2["vis_sel"].cpu()[S] != r["vis_sel"].cpu()[S]).sum()))

# the native run's own full-resolution photometric gradient (loss-tail workspace, g_full[S]; no
# smoothness) against the fp64 oracle's gradient w.r.t. the upsampled disparity, both with the
# native run's decisions imposed
prm0 = md2hip.Params(target_size=(W, H), batch_size=N, automasking=False, disparity_smoothness=0.0)
r3 = md2hip.loss_tail(nat, ps, x.float().cuda().contiguous(), None, cache, prm0, visualize=True,
                      keep_workspace=True)
torch.cuda.synchronize()
al = lambda b: (b + 255) // 256 * 256  # noqa: E731
off = 2 * al(4 * 2 * N * 12) + al(8 * len(scales) * N * 64)
for s_ in range(S):
    raise SystemExit("probe supports S = 0 only")
gfull = r3["workspace"].view(torch.uint8)[off:off + 4 * N * H * W].view(torch.float32).view(N, 1, H, W).cpu().double()
sel3 = [v.unsqueeze(1).long() for v in r3["vis_sel"].cpu()]
ds3 = [d.cpu().double().clone() for d in nat]
ds3[S] = O.upsample_bilinear_size(ds3[S], (H, W))
ds3 = [d.requires_grad_(True) for d in ds3]
l3 = O.loss_from_outputs(ds3, [(a.detach(), b.detach()) for a, b in pos], x, None, ocache,
                         O.Params(target_size=(W, H), batch_size=N, automasking=False, disparity_smoothness=0.0),
                         forced_sel=sel3, forced_cells=r3["vis_cell"].cpu())
l3.backward()
gf = ds3[S].grad
e3 = (gfull - gf).abs()
print(f"native run full-res photometric gradient vs fp64: rel {D.rel_err(gfull, gf):.2e}")
cl = r3["vis_cell"].cpu()[S]
for i in torch.topk(e3.flatten(), 8).indices.tolist():
    n, rr = divmod(i, H * W)
    yy, xx = divmod(rr, W)
    c = [int(cl[j, n, yy, xx].item()) & 0xFFFFFFFF for j in range(2)]
    print(f"  n{n} ({yy},{xx}) gpu {gfull[n, 0, yy, xx]:+.4e} f64 {gf[n, 0, yy, xx]:+.4e} sel {sel3[S][n, 0, yy, xx].item()} "
          f"cells {[(v & 0x7FF, (v >> 11) & 0x7FF, (v >> 22) & 15, bin(v >> 26)) for v in c]}")

# scale S alone (so vis_warped holds its warps): GPU warped values against the oracle's forced warp
cache1 = md2hip.TrainCache(K=K.numpy(), invK=invK.numpy(), scales=(scales[S],))
r4 = md2hip.loss_tail([nat[S]], ps, x.float().cuda().contiguous(), None, cache1, prm0, visualize=True,
                      keep_workspace=True)
torch.cuda.synchronize()
gw = r4["vis_warped"].cpu().double()
c4 = r4["vis_cell"].cpu()[0]
up4 = O.upsample_bilinear_size(nat[S].cpu().double(), (H, W))
ow = O.warp(up4, x, Ps, K, invK, (1, 3), 0.1, 100.0, cells=c4)
for j in range(2):
    ew = (gw[j] - ow[j]).abs()
    print(f"source {j}: warped rel {D.rel_err(gw[j], ow[j]):.2e}, max abs {ew.max():.2e}")
    for i in torch.topk(ew.flatten(), 4).indices.tolist():
        n, rr = divmod(i, C * H * W)
        c, rr = divmod(rr, H * W)
        yy, xx = divmod(rr, W)
        v = int(c4[j, n, yy, xx].item()) & 0xFFFFFFFF
        print(f"   n{n} c{c} ({yy},{xx}) gpu {gw[j, n, c, yy, xx]:.6f} oracle {ow[j][n, c, yy, xx]:.6f} "
              f"cell {(v & 0x7FF, (v >> 11) & 0x7FF, (v >> 22) & 15)}")
print("n2 row 109 cols 360-366 source-1 gpu", [f"{v:.5f}" for v in gw[1, 2, 0, 109, 360:367].tolist()])
print("                            oracle", [f"{v:.5f}" for v in ow[1][2, 0, 109, 360:367].tolist()])
for j in range(2):
    p = ow[j]
    xr, yr = O.pad_reflect(p), O.pad_reflect(tgt)
    mx, my = pool(xr), pool(yr)
    sx, sy, sxy = pool(xr * xr) - mx * mx, pool(yr * yr) - my * my, pool(xr * yr) - mx * my
    raw = (1 - (2 * mx * my + 1e-4) * (2 * sxy + 9e-4) / ((mx * mx + my * my + 1e-4) * (sx + sy + 9e-4))) * 0.5
    print(f"source {j} ssim-term n2 row 109 cols 360-366:", [[f"{v:.4f}" for v in raw[2, c, 109, 360:367].tolist()] for c in range(C)])
    gwj = gw[j]
    xr, yr = O.pad_reflect(gwj), O.pad_reflect(tgt)
    mx, my = pool(xr), pool(yr)
    sx, sy, sxy = pool(xr * xr) - mx * mx, pool(yr * yr) - my * my, pool(xr * yr) - mx * my
    raw = (1 - (2 * mx * my + 1e-4) * (2 * sxy + 9e-4) / ((mx * mx + my * my + 1e-4) * (sx + sy + 9e-4))) * 0.5
    print(f"   (from the GPU's warped values)        :", [[f"{v:.4f}" for v in raw[2, c, 109, 360:367].tolist()] for c in range(C)])
print("sel r4 n2 row 109 cols 360-366:", r4["vis_sel"][0, 2, 109, 360:367].tolist(), "loss", [f"{v:.4f}" for v in r4["vis_loss"][0, 2, 109, 360:367].tolist()])
print("cells r4 src1 rows 108-110:", [[((int(v) & 0xFFFFFFFF) >> 22) & 15 for v in c4[1, 2, rr, 360:367].tolist()] for rr in (108, 109, 110)])
print("cells r4 src0 rows 108-110:", [[((int(v) & 0xFFFFFFFF) >> 22) & 15 for v in c4[0, 2, rr, 360:367].tolist()] for rr in (108, 109, 110)])
print("gpu g_full n2 rows 107-111 cols 359-367 (x1e6):")
for rr in range(107, 112):
    print("  ", " ".join(f"{v * 1e6:+7.3f}" for v in gfull[2, 0, rr, 359:368].tolist()), " | f64 ",
          " ".join(f"{v * 1e6:+7.3f}" for v in gf[2, 0, rr, 359:368].tolist()))
# hypothesis: the GPU treats the bottom-clamped source-1 samples as interior in y
c5 = r3["vis_cell"].cpu().clone()
v = c5[S].long() & 0xFFFFFFFF
st = (v >> 22) & 15
fixed = torch.where(st == 8, v & ~(15 << 22), v)
c5[S] = torch.where(fixed >= 2**31, fixed - 2**32, fixed).int()
ds5 = [d.detach().clone().requires_grad_(True) for d in ds3]
l5 = O.loss_from_outputs(ds5, [(a.detach(), b.detach()) for a, b in pos], x, None, ocache,
                         O.Params(target_size=(W, H), batch_size=N, automasking=False, disparity_smoothness=0.0),
                         forced_sel=sel3, forced_cells=c5)
l5.backward()
print("oracle with bottom clamps released (x1e6):")
for rr in range(107, 112):
    print("  ", " ".join(f"{v * 1e6:+7.3f}" for v in ds5[S].grad[2, 0, rr, 359:368].tolist()))
thr = 0.1 * gf.pow(2).mean().sqrt().item()
bad = (e3 > thr).nonzero().tolist()
print(f"outliers (|err| > {thr:.2e}): {len(bad)}")
for n, _, yy, xx in bad[:40]:
    c = [int(cl[j, n, yy, xx].item()) & 0xFFFFFFFF for j in range(2)]
    print(f"  n{n} ({yy},{xx}) err {gfull[n, 0, yy, xx] - gf[n, 0, yy, xx]:+.2e} g {gf[n, 0, yy, xx]:+.2e} sel {sel3[S][n, 0, yy, xx].item()} "
          f"states {[(v >> 22) & 15 for v in c]} cells {[(v & 0x7FF, (v >> 11) & 0x7FF) for v in c]} x%60 {(xx + 0) % 60}")
dep = O.disparity_to_depth(ds3[S].detach(), 0.1, 100.0)
coords = O.backproject(dep.reshape(N, 1, H * W), invK, W, H)
for j, (R_, t_) in enumerate(Ps):
    cam = K @ (R_ @ coords + t_.unsqueeze(-1))
    ixy = cam[:, :2] / (cam[:, 2:3] + 1e-7) - 1.0
    for xx in range(361, 366):
        p = 109 * W + xx
        print(f"  src{j} n2 (109,{xx}) depth {dep[2, 0, 109, xx]:.5f} cam {[f'{v:.4f}' for v in cam[2, :, p].tolist()]} ix,iy {[f'{v:.4f}' for v in ixy[2, :, p].tolist()]}")
pl = [O.photometric_loss(w_, tgt) for w_ in ow]
for rr in (108, 109, 110, 111):
    print(f"  row {rr} l0-l1 rel:", [f"{((pl[0][2, 0, rr, xx] - pl[1][2, 0, rr, xx]) / pl[0][2, 0, rr, xx]).item():+.1e}" for xx in range(360, 367)],
          "sel", r4["vis_sel"][0, 2, rr, 360:367].tolist())
