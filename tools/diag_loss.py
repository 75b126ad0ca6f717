import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "monodepth2.jl_amd"))
import torch
from oracle import md2_oracle as O
from tests import _data as D
import md2hip

def run(N, C, H, W, smooth):
    x = D.triplets(N, C, H, W); K, invK = D.intrinsics(W, H)
    disps = D.disparities(N, H, W); poses = D.poses(N)
    scales = (0.125, 0.25, 0.5, 1.0)
    dd = [d.clone().requires_grad_(True) for d in disps]
    pp = [(r.clone().requires_grad_(True), t.clone().requires_grad_(True)) for r, t in poses]
    cache = O.TrainCache(K=K, invK=invK, scales=scales)
    p = O.Params(target_size=(W, H), batch_size=N, automasking=False, disparity_smoothness=smooth)
    lo = O.loss_from_outputs(dd, pp, x, None, cache, p); lo.backward()
    c2 = md2hip.TrainCache(K=K.numpy(), invK=invK.numpy(), scales=scales)
    p2 = md2hip.Params(target_size=(W, H), batch_size=N, automasking=False, disparity_smoothness=smooth)
    lg, terms, dg, dp = md2hip.loss_tail([d.float().cuda().contiguous() for d in disps],
        [(r.float().cuda(), t.float().cuda()) for r, t in poses], x.float().cuda().contiguous(), None, c2, p2)
    torch.cuda.synchronize()
    print(f"N{N} C{C} {H}x{W} smooth={smooth} loss {lg.item():.7f} vs {lo.item():.7f}")
    for s in range(4):
        a, b = dg[s].cpu().double(), dd[s].grad
        e = (a - b).abs()
        idx = torch.argmax(e)
        print(f"  scale {s} rel {D.rel_err(a,b):.3e} max abs err {e.max().item():.3e} at {torch.unravel_index(idx, e.shape)} ref max {b.abs().max().item():.3e}")
        # error by row / col
        er = e[0,0]
        print("    err row-sum top:", torch.topk(er.sum(1), 3).indices.tolist(), " col-sum top:", torch.topk(er.sum(0), 3).indices.tolist())
    dpo = torch.cat([torch.cat([r.grad, t.grad], 1) for r, t in pp], 0)
    print("  pose rel", D.rel_err(dp.cpu(), dpo))

run(1, 3, 128, 416, 1e-3)
run(1, 3, 128, 416, 0.0)
run(1, 3, 64, 128, 0.0)
run(1, 3, 32, 64, 0.0)
