"""GPU: the graph-captured train step (md2_model_train_step_graph) equals the eager step --
forward_loss + backward segments + ADAM.update -- bit for bit: parameters, ADAM moments and
losses over several steps with changing batches, a jump of the step counter, and automasking
computed inside the step."""
import pytest
import torch

from tests import _data as D

pytestmark = pytest.mark.gpu


def _setup(automasking):
    import md2hip
    enc = md2hip.ResNet(18, in_channels=3)
    model = md2hip.Model(enc, md2hip.DepthDecoder(encoder_channels=enc.stages, scale_levels=[2, 3, 4, 5],
                                                  embedding_levels=0), md2hip.PoseDecoder(512), seed=42)
    K, invK = D.intrinsics(128, 64)
    cache = md2hip.TrainCache(K=K.numpy(), invK=invK.numpy())
    params = md2hip.Params(target_size=(128, 64), batch_size=2, automasking=automasking)
    return model, cache, params, md2hip.ADAM(1e-3)


@pytest.mark.parametrize("automasking", [False, True])
def test_graph_step_bitwise_equals_eager(automasking):
    import md2hip.dist
    xs = [D.triplets(2, 3, 64, 128, seed=s).float().cuda().contiguous() for s in (1, 2, 3, 4)]
    me, cache, params, oe = _setup(automasking)
    mg, _, _, og = _setup(automasking)
    ex_e = me.executor(tuple(xs[0].shape), cache, params)
    ex_g = mg.executor(tuple(xs[0].shape), cache, params)
    comm = md2hip.dist.GradAllReduce(force=False)
    for i, x in enumerate(xs):
        if i == 3:                       # the device step counter is re-set when t jumps
            oe.t += 5
            og.t += 5
        le = md2hip.dist.train_step(ex_e, me, oe, x, comm).clone()
        lg = ex_g.train_step_graph(x, og).clone()
        torch.cuda.synchronize()
        assert torch.equal(le, lg), (i, le, lg)
        assert torch.equal(me.flat, mg.flat), i
        assert torch.equal(oe.m, og.m) and torch.equal(oe.v, og.v), i
    # an eager call on the graph model after replays sees the replayed parameters
    le = md2hip.dist.train_step(ex_e, me, oe, xs[0], comm)
    lg = md2hip.dist.train_step(ex_g, mg, og, xs[0], comm)
    torch.cuda.synchronize()
    assert torch.equal(le, lg) and torch.equal(me.flat, mg.flat)


def test_segment_update_bitwise_equals_single_update(monkeypatch):
    """MD2_SEG_UPDATE=1: ADAM + re-pack of each backward segment on the executor's update stream
    beside the remaining backward (md2_model_adam_segment / md2_model_adam_join) equals the one
    update after the backward bit for bit -- parameters, moments, losses -- over steps that each
    read the previous step's re-packed weights."""
    import md2hip.dist
    xs = [D.triplets(2, 3, 64, 128, seed=s).float().cuda().contiguous() for s in (5, 6, 7)]
    ma, cache, params, oa = _setup(False)
    mb, _, _, ob = _setup(False)
    ex_a = ma.executor(tuple(xs[0].shape), cache, params)
    ex_b = mb.executor(tuple(xs[0].shape), cache, params)
    comm = md2hip.dist.GradAllReduce(force=False)
    for i, x in enumerate(xs):
        monkeypatch.setenv("MD2_SEG_UPDATE", "0")
        la = md2hip.dist.train_step(ex_a, ma, oa, x, comm).clone()
        monkeypatch.setenv("MD2_SEG_UPDATE", "1")
        lb = md2hip.dist.train_step(ex_b, mb, ob, x, comm).clone()
        torch.cuda.synchronize()
        assert torch.equal(la, lb), (i, la, lb)
        assert torch.equal(ma.flat, mb.flat), i
        assert torch.equal(oa.m, ob.m) and torch.equal(oa.v, ob.v), i
