"""Generates the golden vectors under tests/golden/ from the fp64 CPU oracle (oracle/md2_oracle.py).

The reference (Julia/Flux) cannot run here, so the oracle is pinned by the
reference's own known answers (tests/test_oracle_known_answers.py, test/runtests.jl) and these
fixtures freeze its outputs on seeded inputs: tests/test_golden.py re-derives them on the CPU
(oracle drift) and checks the HIP path against them on the GPU.

    python tests/golden/make_golden.py          # rewrites the .npz / .json files
"""
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import md2_oracle as O  # noqa: E402
from tests import _data as D  # noqa: E402

SCALES = (0.125, 0.25, 0.5, 1.0)


def loss_tail_case(N=2, C=3, H=32, W=64, seed=7):
    """Fused loss tail (src/training.jl:25-77) fwd + pullback on affine-ramp sources."""
    x = D.triplets(N, C, H, W, seed=seed, ramp_sources=True, grid32=False)
    K, invK = D.intrinsics(W, H, grid32=False)
    disps = D.disparities(N, H, W, seed=seed + 4, grid32=False)
    poses = D.poses(N, seed=seed + 6, grid32=False)
    dv = [d.clone().requires_grad_(True) for d in disps]
    pv = [(r.clone().requires_grad_(True), t.clone().requires_grad_(True)) for r, t in poses]
    per_source = []
    loss, parts = O.loss_from_outputs(dv, pv, x, None, O.TrainCache(K=K, invK=invK, scales=SCALES),
                                      O.Params(target_size=(W, H), batch_size=N, automasking=False),
                                      return_parts=True, per_source=per_source)
    loss.backward()
    out = {"x": x, "K": K, "invK": invK, "loss": loss.detach().reshape(1),
           "terms": torch.tensor([[float(a.detach()), float(b.detach())] for a, b in parts]),
           "d_pose": torch.cat([torch.cat([r.grad, t.grad], 1) for r, t in pv], 0)}
    for s in range(len(SCALES)):
        out[f"disp{s}"] = disps[s]
        out[f"d_disp{s}"] = dv[s].grad
        out[f"l0_{s}"] = per_source[s][0].detach()
        out[f"l1_{s}"] = per_source[s][1].detach()
    for j, (r, t) in enumerate(poses):
        out[f"rvec{j}"] = r
        out[f"tvec{j}"] = t
    return {k: v.numpy() for k, v in out.items()}


def so3_case():
    """so3_exp_map + composeT (src/utils.jl:106-121, 185-192) incl. theta < 1e-4 and 0."""
    g = torch.Generator().manual_seed(11)
    r = torch.randn(8, 3, generator=g, dtype=torch.float64) * 0.3
    r[5] = torch.tensor([3e-5, -2e-5, 1e-5], dtype=torch.float64)    # theta' = max(theta, 1e-4)
    r[6] = 0.0
    r[7] = torch.tensor([3.0, 0.5, -1.0], dtype=torch.float64)       # |theta| near pi
    t = torch.randn(8, 3, generator=g, dtype=torch.float64)
    out = {"rvec": r, "tvec": t, "R": O.so3_exp_map(r)}
    for inv in (0, 1):
        R, tt = O.composeT(r, t, bool(inv))
        out[f"R_inv{inv}"], out[f"t_inv{inv}"] = R, tt
    return {k: v.numpy() for k, v in out.items()}


def model_digest(N=1, C=3, H=64, W=128, seed=7):
    """Full train_loss + gradient of the mono model (ResNet-18, scale_levels 2:5, Flux init seed
    42) at 64x128: loss, outputs and per-tensor gradient digests (norm, sum, 4 sampled entries)."""
    x = D.triplets(N, C, H, W, seed=seed, ramp_sources=True, grid32=False)
    K, invK = D.intrinsics(W, H, grid32=False)
    spec = O.param_spec(18, C, (2, 3, 4, 5))
    flat = O.init_params(spec, 42).double().requires_grad_(True)
    P = O.unflatten(flat, spec)
    d_o, p_o = O.model_forward(P, x, arch=18)
    loss = O.loss_from_outputs(d_o, p_o, x, None, O.TrainCache(K=K, invK=invK),
                               O.Params(target_size=(W, H), batch_size=N, automasking=False))
    loss.backward()
    dig, off = {}, 0
    for name, shape in spec:
        n = int(np.prod(shape))
        gsl = flat.grad[off:off + n]
        idx = [0, n // 3, (2 * n) // 3, n - 1]
        dig[name] = {"norm": gsl.norm().item(), "sum": gsl.sum().item(),
                     "idx": idx, "val": [gsl[i].item() for i in idx]}
        off += n
    return {"config": {"N": N, "C": C, "H": H, "W": W, "seed": seed, "param_seed": 42, "arch": 18,
                       "ramp_sources": True},
            "loss": loss.item(),
            "disp_sums": [d.sum().item() for d in d_o],
            "poses": [torch.cat([r, t], 1).detach().reshape(-1).tolist() for r, t in p_o],
            "grad": dig}


def main():
    torch.set_default_dtype(torch.float64)
    np.savez_compressed(os.path.join(HERE, "loss_tail_2x3x32x64.npz"), **loss_tail_case())
    np.savez_compressed(os.path.join(HERE, "so3_compose.npz"), **so3_case())
    with open(os.path.join(HERE, "model_digest_1x3x64x128.json"), "w") as f:
        json.dump(model_digest(), f, indent=1)


if __name__ == "__main__":
    main()
