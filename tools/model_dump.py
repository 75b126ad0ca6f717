"""Dump one GPU train step (tests/_model_parity.run) -- inputs, flat parameters, the GPU's
decisions, disparities / poses, the loss tail's d_disp / d_pose at those outputs and the flat
gradient -- to a .pt file for CPU-side decomposition of gradient errors (tools/model_analyze.py).
    python tools/model_dump.py OUT.pt SOURCES [N H W]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monodepth2.jl_amd")]
import torch  # noqa: E402

import md2hip  # noqa: E402
from tests import _data as D  # noqa: E402
from tests import _model_parity as MP  # noqa: E402

out, src = sys.argv[1], sys.argv[2]
N, H, W = (int(v) for v in sys.argv[3:6]) if len(sys.argv) > 5 else (2, 64, 128)
g, o, errs = MP.run(N=N, H=H, W=W, sources=src)
# the loss tail's own pullback at the GPU's outputs
x = g["x"].float().cuda().contiguous()
K, invK = D.intrinsics(W, H)
cache = md2hip.TrainCache(K=K.numpy(), invK=invK.numpy())
params = md2hip.Params(target_size=(W, H), batch_size=N, automasking=False)
pose = g["pose"].cuda()
tail = md2hip.loss_tail([d.cuda().contiguous() for d in g["disps"]],
                        [(pose[:N, :3].contiguous(), pose[:N, 3:].contiguous()),
                         (pose[N:, :3].contiguous(), pose[N:, 3:].contiguous())], x, None, cache, params)
torch.cuda.synchronize()
g["tail_d_disp"] = [t.cpu() for t in tail["d_disp"]]
g["tail_d_pose"] = tail["d_pose"].cpu()
torch.save({"g": g, "errs": errs}, out)
print("dumped", out, sorted(errs.items(), key=lambda kv: -kv[1])[:3])
