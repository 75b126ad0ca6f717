"""MPI mode end to end (src/model.jl:1-55, src/repeat.jl:44-69): the Model
with DepthDecoder(embedding_levels=21) trained at batch 1 on the executor's kernels --
encoder, plane embedding of every decoder level (md2_mpi_embed_features), the 21-channel-wider
DepthDecoder over the num_bins plane images, the loss with the planes as its batch (each plane
warped with the sample's poses against the sample's frames), and the backward including the
_repeat pullback (block sum over the planes, plane_sum) -- against the fp64 oracle's
O.mpi_train_loss with every GPU decision imposed; bounds as tests/test_gpu_model.py."""
import pytest
import torch

from tests import _data as D

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(600)
@pytest.mark.parametrize("H,W,nb", [(64, 128, 4), (96, 320, 4), (128, 416, 32)],
                         ids=["64x128-4planes", "96x320-4planes", "416x128-32planes"])
def test_mpi_train_step_parity(H, W, nb):
    """96x320: the level-4 map is 3x10 = 30 pixels, not a multiple of 4 -- the _repeat pullback
    takes its one-pixel-per-thread path."""
    from tests._model_parity import check_step, oracle_bounds, run
    g, o, errs = run(N=1, H=H, W=W, sources="texture", num_bins=nb)
    assert len(g["disps"]) == 4 and g["disps"][-1].shape == (nb, 1, H, W)
    assert g["loss"] == g["tail_loss"]
    # the plane axis is live: different bins, different disparities of the same sample
    assert (g["disps"][-1][0] - g["disps"][-1][1]).abs().max() > 0
    b = oracle_bounds(g, o)
    check_step(g, o, errs, b, label=f"MPI {W}x{H} planes {nb}")


def test_mpi_mode_contract():
    """MPI mode trains one sample per step (the reference's shape-consistent case), has no
    eval_disparity (defect D4), and an ADAM step through it updates the parameters."""
    import md2hip
    from md2hip._lib import MD2Error
    enc = md2hip.ResNet(18, in_channels=3)
    m = md2hip.Model(enc, md2hip.DepthDecoder(encoder_channels=enc.stages, scale_levels=[2, 3, 4, 5],
                                              embedding_levels=21), md2hip.PoseDecoder(512), seed=42)
    K, invK = D.intrinsics(128, 64)
    cache = md2hip.TrainCache(K=K.numpy(), invK=invK.numpy())
    x2 = D.triplets(2, 3, 64, 128, seed=3).float().cuda()
    with pytest.raises(MD2Error, match="batch must be 1"):
        md2hip.train_loss(m, x2, None, cache, md2hip.Params(target_size=(128, 64), batch_size=2,
                                                            automasking=False), num_bins=4)
    with pytest.raises(NotImplementedError):
        md2hip.eval_disparity(m, x2[:, 1].contiguous())
    x1 = x2[:1].contiguous()
    params = md2hip.Params(target_size=(128, 64), batch_size=1, automasking=True)
    before = m.flat.clone()
    opt = md2hip.ADAM(1e-4)
    for _ in range(2):
        loss, *_ = md2hip.train_loss(m, x1, None, cache, params, num_bins=8)
        md2hip.gradient(m)
        opt.update(m)
    torch.cuda.synchronize()
    assert torch.isfinite(loss).all() and torch.isfinite(m.flat).all()
    assert not torch.equal(before, m.flat)
    disps, poses = m(x1, num_bins=8)
    assert disps[-1].shape == (8, 1, 64, 128) and poses[0].rvec.shape == (1, 3)
