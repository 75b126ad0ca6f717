"""Golden train_loss of the bench's first step (BASELINE config 3) from the fp64 CPU oracle.

bench.py's step 1 runs train_loss on: Flux-default parameters (seed 42; md2hip.model.flux_init
== oracle.init_params), 12 uniform [0,1) RGB 416x128 triplets from md2hip.dist.synthetic_triplets
(global sample indices 0..11, seed 1234), Depth10k K, scales (1/8, 1/4, 1/2, 1), automasking off.
The loss is a continuous function of the inputs (ReLU / max-pool / per-pixel min are continuous),
so no branch decision needs imposing for the VALUE.

    python tests/golden/make_bench_loss.py     # rewrites tests/golden/bench_first_loss.json
"""
import json
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
for p in (ROOT, os.path.join(ROOT, "monodepth2.jl_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

from oracle import md2_oracle as O  # noqa: E402

B, H, W = 12, 128, 416


def bench_first_loss():
    from md2hip.dist import synthetic_triplets       # pure torch-CPU data generator
    x = synthetic_triplets(B, H, W, 0, "cpu").double()
    spec = O.param_spec(18, 3, (2, 3, 4, 5))
    flat = O.init_params(spec, 42).float().double()  # the GPU runs the fp32 cast of the init
    P = O.unflatten(flat, spec)
    K, invK = O.depth10k_K(W, H)
    cache = O.TrainCache(K=K, invK=invK, scales=(0.125, 0.25, 0.5, 1.0))
    params = O.Params(target_size=(W, H), batch_size=B, automasking=False)
    with torch.no_grad():
        loss = O.train_loss(P, x, None, cache, params, arch=18)
    return float(loss)


if __name__ == "__main__":
    v = bench_first_loss()
    with open(os.path.join(HERE, "bench_first_loss.json"), "w") as f:
        json.dump({"config": f"train_loss resnet18 B={B} {W}x{H} RGB, bench.py step 1",
                   "loss": v}, f, indent=1)
    print(v)
