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
