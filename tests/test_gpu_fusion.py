"""GPU: the launch-boundary split-K reduce (a split-K conv's slabs summed by the BatchNorm
statistics pass / the BN-backward partial pass, conv_f_bn / conv_d_bn in model.cpp) and the float4
split-K reduction change no bit of the train step: parameters, ADAM moments and losses after
several steps at the benchmarked configuration (B=12, 416x128: layer3/layer4 convs run split-K)
equal those of the separate-reduction path (MD2_FUSE_SPLITK=0).  Likewise the fused stem passes:
BN + ReLU + max pool in one forward kernel (MD2_FUSE_POOL_FWD), the stem's decoder skip gradient
added by the max-pool adjoint (MD2_FUSE_POOL_BWD), and the encoder stages' skip gradients added
inside the BN-backward passes instead of by axpy (MD2_FUSE_SKIP_BWD).  And the PoseDecoder on its own
stream beside the DepthDecoder, and the downsampling blocks' 1x1 conv + BN beside the block's 3x3
chain, and the DepthDecoder's and the late encoder stages' filter gradients beside their data
gradients, each with its own scratch (MD2_POSE_STREAM, MD2_DOWN_STREAM, MD2_DEC_WGRAD_STREAM,
MD2_ENC_WGRAD_STREAM)."""
import os

import pytest
import torch

from tests import _data as D

pytestmark = pytest.mark.gpu


def _setup(fuse, H, W, B, switch="MD2_FUSE_SPLITK"):
    import md2hip
    old = os.environ.get(switch)
    os.environ[switch] = "1" if fuse else "0"
    try:
        enc = md2hip.ResNet(18, in_channels=3)
        model = md2hip.Model(enc, md2hip.DepthDecoder(encoder_channels=enc.stages, scale_levels=[2, 3, 4, 5],
                                                      embedding_levels=0), md2hip.PoseDecoder(512), seed=42)
        K, invK = D.intrinsics(W, H)
        cache = md2hip.TrainCache(K=K.numpy(), invK=invK.numpy())
        params = md2hip.Params(target_size=(W, H), batch_size=B, automasking=True)
        opt = md2hip.ADAM(1e-4)
        ex = model.executor((B, 3, 3, H, W), cache, params)   # the executor reads the switch here
    finally:
        if old is None:
            os.environ.pop(switch, None)
        else:
            os.environ[switch] = old
    return model, ex, opt


@pytest.mark.parametrize("switch", ["MD2_FUSE_SPLITK", "MD2_FUSE_POOL_FWD", "MD2_FUSE_POOL_BWD",
                                    "MD2_FUSE_SKIP_BWD", "MD2_POSE_STREAM", "MD2_DOWN_STREAM",
                                    "MD2_DEC_WGRAD_STREAM", "MD2_ENC_WGRAD_STREAM"])
@pytest.mark.parametrize("B,H,W", [(12, 128, 416), (2, 64, 128)])
def test_fused_splitk_bn_bitwise(B, H, W, switch):
    import md2hip.dist
    xs = [D.triplets(B, 3, H, W, seed=s).float().cuda().contiguous() for s in (5, 6, 7)]
    mf, exf, of = _setup(True, H, W, B, switch)
    mu, exu, ou = _setup(False, H, W, B, switch)
    comm = md2hip.dist.GradAllReduce(force=False)
    for i, x in enumerate(xs):
        lf = md2hip.dist.train_step(exf, mf, of, x, comm).clone()
        lu = md2hip.dist.train_step(exu, mu, ou, x, comm).clone()
        torch.cuda.synchronize()
        assert torch.equal(lf, lu), (i, lf, lu)
        assert torch.equal(mf.flat, mu.flat), i
        assert torch.equal(of.m, ou.m) and torch.equal(of.v, ou.v), i


@pytest.mark.parametrize("B,H,W", [(12, 128, 416), (2, 64, 128)])
def test_fused_bnstats_close(B, H, W):
    """BatchNorm statistics from the LDS-halo forward's epilogue (per-tile fp64 partials,
    MD2_FUSE_BNSTATS) against the separate statistics pass: the same fp64 sums in another order,
    so mean / invstd agree to an ulp, not bitwise.  Losses within 1e-6 relative at every step;
    parameters within ADAM's per-step bound (lr per step: an update can flip where a gradient
    component sits at the rounding level)."""
    import md2hip.dist
    xs = [D.triplets(B, 3, H, W, seed=s).float().cuda().contiguous() for s in (5, 6, 7)]
    mf, exf, of = _setup(True, H, W, B, "MD2_FUSE_BNSTATS")
    mu, exu, ou = _setup(False, H, W, B, "MD2_FUSE_BNSTATS")
    comm = md2hip.dist.GradAllReduce(force=False)
    for i, x in enumerate(xs):
        lf = md2hip.dist.train_step(exf, mf, of, x, comm).clone()
        lu = md2hip.dist.train_step(exu, mu, ou, x, comm).clone()
        torch.cuda.synchronize()
        assert abs(float(lf) - float(lu)) <= 1e-6 * abs(float(lu)), (i, float(lf), float(lu))
        dp = (mf.flat - mu.flat).abs().max().item()
        assert dp <= 2.0 * 1e-4 * (i + 1) + 1e-7, (i, dp)


_KNOB_CHILD = r"""
import os, sys
root, out = sys.argv[1], sys.argv[2]
sys.path[:0] = [root, os.path.join(root, "monodepth2.jl_amd")]
import numpy as np, torch, md2hip, md2hip.dist
from tests import _data as D
B, H, W = 2, 64, 128
enc = md2hip.ResNet(18, in_channels=3)
m = md2hip.Model(enc, md2hip.DepthDecoder(encoder_channels=enc.stages, scale_levels=[2, 3, 4, 5],
                                          embedding_levels=0), md2hip.PoseDecoder(512), seed=42)
K, invK = D.intrinsics(W, H)
ex = m.executor((B, 3, 3, H, W), md2hip.TrainCache(K=K.numpy(), invK=invK.numpy()),
                md2hip.Params(target_size=(W, H), batch_size=B, automasking=False))
opt = md2hip.ADAM(1e-4)
for s in (5, 6):
    md2hip.dist.train_step(ex, m, opt, D.triplets(B, 3, H, W, seed=s).float().cuda().contiguous(),
                           md2hip.dist.GradAllReduce(force=False))
torch.cuda.synchronize()
np.save(out, m.flat.cpu().numpy())
"""

# settings every one of which an A/B sweep has run before (tools/*_sweep.sh, tools/ab_*.sh)
KNOBS = {"MD2_PX_TARGET": "1024", "MD2_W_TILE": "2", "MD2_W_TARGET": "1024", "MD2_PX_V2": "0",
         "MD2_HEAD_STRIP": "0", "MD2_UP_TILED": "0", "MD2_PHOTO_WAVES": "1024", "MD2_W16": "0",
         "MD2_PX16": "0"}


@pytest.mark.timeout(240)
def test_tuning_knobs_ignored_without_md2_tuning(tmp_path):
    """The kernel / planner tuning knobs (common.h tuning_knob) change nothing unless MD2_TUNING=1:
    two steps with nine knobs set (and no MD2_TUNING) give bit-identical parameters to a clean
    environment; with MD2_TUNING=1 the same knobs do take effect (other kernels, other roundings)."""
    import subprocess
    import sys
    import numpy as np
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    base = {k: v for k, v in os.environ.items() if not k.startswith("MD2_")}
    runs = {"clean": base, "knobs": dict(base, **KNOBS), "tuned": dict(base, MD2_TUNING="1", **KNOBS)}
    res = {}
    for name, env in runs.items():
        out = str(tmp_path / f"{name}.npy")
        r = subprocess.run([sys.executable, "-c", _KNOB_CHILD, root, out], env=env, capture_output=True,
                           text=True, timeout=200)
        assert r.returncode == 0, r.stderr[-3000:]
        res[name] = np.load(out)
    assert np.array_equal(res["clean"], res["knobs"])
    assert not np.array_equal(res["clean"], res["tuned"])


# round-5 placement / regrouping switches: each regroups the same arithmetic (other streams, other
# buffers, another loop order with the same per-output fma chain), so the step must not move a bit
BITWISE_TUNING = {"MD2_ENC_WGRAD_MAIN0": "0"}


@pytest.mark.timeout(420)
def test_bitwise_tuning_switches(tmp_path):
    """MD2_ENC_WGRAD_MAIN0=0 (every layer-4 filter gradient on the side stream): two train steps at
    B=2 64x128 give parameters bit-identical to the defaults.  (The round-5 opt-ins measured
    neutral -- the decoder ping-pong buffers, the row-walking heads forward, the per-branch
    decoder filter-gradient placement, the small-map whalo target -- were deleted in round 6.)"""
    import subprocess
    import sys
    import numpy as np
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    base = {k: v for k, v in os.environ.items() if not k.startswith("MD2_")}
    runs = {"clean": base}
    for k, v in BITWISE_TUNING.items():
        runs[k] = dict(base, MD2_TUNING="1", **{k: v})
    res = {}
    for name, env in runs.items():
        out = str(tmp_path / f"{name}.npy")
        r = subprocess.run([sys.executable, "-c", _KNOB_CHILD, root, out], env=env, capture_output=True,
                           text=True, timeout=200)
        assert r.returncode == 0, (name, r.stderr[-3000:])
        res[name] = np.load(out)
    for k in BITWISE_TUNING:
        assert np.array_equal(res["clean"], res[k]), k
