"""GPU: the launch-boundary split-K reduce (a split-K conv's slabs summed by the BatchNorm
statistics pass / the BN-backward partial pass, conv_f_bn / conv_d_bn in model.cpp) and the float4
split-K reduction change no bit of the train step: parameters, ADAM moments and losses after
several steps at the benchmarked configuration (B=12, 416x128: layer3/layer4 convs run split-K)
equal those of the separate-reduction path (MD2_FUSE_SPLITK=0).  Likewise the fused stem passes:
BN + ReLU + max pool in one forward kernel (MD2_FUSE_POOL_FWD), the stem's decoder skip gradient
added by the max-pool adjoint (MD2_FUSE_POOL_BWD), and the encoder stages' skip gradients added
inside the BN-backward passes instead of by axpy (MD2_FUSE_SKIP_BWD)."""
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
                                    "MD2_FUSE_SKIP_BWD"])
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
