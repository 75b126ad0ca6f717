import sys, os
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R); sys.path.insert(0, os.path.join(R, "monodepth2.jl_amd"))
import torch
from oracle import md2_oracle as O
from tests import _data as D
from tests.test_gpu_loss import _gpu, _oracle, SCALES
N, C, H, W = 1, 3, 128, 416
x = D.triplets(N, C, H, W, seed=7); K, invK = D.intrinsics(W, H)
disps = D.disparities(N, H, W, seed=11); poses = D.poses(N, seed=13)
g = _gpu(disps, poses, x, K, invK, None)
forced = [g["vis_sel"][s].unsqueeze(1).long() for s in range(4)]
lo, dd_o, dp_o, per = _oracle(disps, poses, x, K, invK, None, forced_sel=forced)
# ix, iy per source at full res for scale 3
s = 3
Ps = O.poses_to_transforms(poses, (1, 3), 2)
depth = O.disparity_to_depth(disps[s], 0.1, 100.0)
pts = O.backproject(depth.reshape(N, 1, H * W), invK, W, H)
for sc in range(4):
    e = (g["d_disp"][sc].double() - dd_o[sc]).abs()[0, 0]
    print("scale", sc, "rel", D.rel_err(g["d_disp"][sc], dd_o[sc]))
    flat = torch.topk(e.flatten(), 6)
    for v, i in zip(flat.values, flat.indices):
        yy, xx = divmod(i.item(), e.shape[1])
        print(f"   ({yy},{xx}) err {v.item():.3e} gpu {g['d_disp'][sc][0,0,yy,xx].item():.4e} ref {dd_o[sc][0,0,yy,xx].item():.4e}")
e = (g["d_disp"][3].double() - dd_o[3]).abs()[0, 0]
flat = torch.topk(e.flatten(), 4)
for i in flat.indices:
    yy, xx = divmod(i.item(), W)
    print("pixel", yy, xx, "sel nbhd", g["vis_sel"][3][0, max(0,yy-1):yy+2, max(0,xx-1):xx+2].tolist())
    for k, (Rm, t) in enumerate(Ps):
        uv = O.project(pts, K, Rm, t, W, H)[0, :, yy * W + xx]
        ix = (uv[0] + 1) / 2 * (W - 1); iy = (uv[1] + 1) / 2 * (H - 1)
        print(f"    src{k}: ix {ix.item():.6f} iy {iy.item():.6f} l={per[3][k][0,0,yy,xx].item():.6f}")
print("pose rel", D.rel_err(g["d_pose"], dp_o), "loss", g["loss"].item(), lo.item())
