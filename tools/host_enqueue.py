"""Is the train step host-bound?  Times the host-side enqueue of K steps (no synchronisation)
against the wall time until the GPU has finished them (bench.py's workload, B=12 416x128)."""
import os
import sys
import time

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, "monodepth2.jl_amd")]
import torch  # noqa: E402

import md2hip  # noqa: E402
import md2hip.dist  # noqa: E402
from bench import synthetic_batch  # noqa: E402

B, H, W = 12, 128, 416
dev = torch.device("cuda", 0)
enc = md2hip.ResNet(18, in_channels=3)
model = md2hip.Model(enc, md2hip.DepthDecoder(encoder_channels=enc.stages, scale_levels=[2, 3, 4, 5],
                                              embedding_levels=0), md2hip.PoseDecoder(512), device=dev, seed=42)
K, invK = md2hip.depth10k_intrinsics(W, H)
cache = md2hip.TrainCache(K=K, invK=invK)
params = md2hip.Params(target_size=(W, H), batch_size=B, automasking=False)
opt = md2hip.ADAM(1e-4)
x = synthetic_batch(B, H, W, 0, dev)
ex = model.executor(tuple(x.shape), cache, params)
comm = md2hip.dist.GradAllReduce()
loss = torch.empty(1, device=dev)
for _ in range(5):
    md2hip.dist.train_step(ex, model, opt, x, comm, loss=loss)
torch.cuda.synchronize()
for K_ in (1, 5, 20):
    t0 = time.perf_counter()
    for _ in range(K_):
        md2hip.dist.train_step(ex, model, opt, x, comm, loss=loss)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"{K_:3d} steps: host enqueue {(t1 - t0) / K_ * 1e3:.3f} ms/step, wall {(t2 - t0) / K_ * 1e3:.3f} ms/step")
