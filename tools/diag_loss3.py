import sys, os
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R); sys.path.insert(0, os.path.join(R, "monodepth2.jl_amd"))
import torch
from oracle import md2_oracle as O
from tests import _data as D
from tests.test_gpu_loss import _gpu, _oracle, SCALES
N, C, H, W = 2, 3, 32, 64
for smooth in (1e-3, 0.0):
    x = D.triplets(N, C, H, W, seed=7, ramp_sources=True); K, invK = D.intrinsics(W, H)
    disps = D.disparities(N, H, W, seed=11); poses = D.poses(N, seed=13)
    g = _gpu(disps, poses, x, K, invK, None, smoothness=smooth)
    forced = [g["vis_sel"][s].unsqueeze(1).long() for s in range(4)]
    lo, dd_o, dp_o, per = _oracle(disps, poses, x, K, invK, None, forced_sel=forced, smoothness=smooth)
    print("smooth", smooth, [D.rel_err(g["d_disp"][s], dd_o[s]) for s in range(4)], "pose", D.rel_err(g["d_pose"], dp_o))
    e = (g["d_disp"][3].double() - dd_o[3]).abs()
    flat = torch.topk(e.flatten(), 8)
    for v, i in zip(flat.values, flat.indices):
        idx = torch.unravel_index(i, e.shape)
        print("   ", [int(t) for t in idx], f"err {v.item():.3e} gpu {g['d_disp'][3][idx].item():.4e} ref {dd_o[3][idx].item():.4e}")
    print("   ref abs mean", dd_o[3].abs().mean().item(), "err mean", e.mean().item())
