"""GPU: the Flux-layout parameter boundary (md2_model_set_params / get_params / get_grads: conv
kernels as Flux's true convolutions, taps reversed against the library's cross-correlation) and
the train_loss pullback cotangent (md2_model_loss_cotangent)."""
import pytest
import torch

from tests import _data as D

pytestmark = pytest.mark.gpu


def _model():
    import md2hip
    enc = md2hip.ResNet(18, in_channels=3)
    m = md2hip.Model(enc, md2hip.DepthDecoder(encoder_channels=enc.stages, scale_levels=[2, 3, 4, 5],
                                              embedding_levels=0), md2hip.PoseDecoder(512), seed=42)
    K, invK = D.intrinsics(128, 64)
    cache = md2hip.TrainCache(K=K.numpy(), invK=invK.numpy())
    params = md2hip.Params(target_size=(128, 64), batch_size=2, automasking=False)
    return m, cache, params


def _flip_reference(flat, table):
    out = flat.clone()
    for name, shape, off in table:
        if len(shape) == 4 and shape[2] * shape[3] > 1:
            n = 1
            for v in shape:
                n *= v
            out[off:off + n] = flat[off:off + n].view(*shape).flip(2, 3).reshape(-1)
    return out


def test_flux_params_roundtrip_and_flip():
    import md2hip
    m, cache, params = _model()
    x = D.triplets(2, 3, 64, 128, seed=1).float().cuda().contiguous()
    md2hip.train_loss(m, x, None, cache, params)
    lib_flat = m.flat.detach().clone()
    flux = md2hip.flux_params(m)
    assert torch.equal(flux.cpu(), _flip_reference(lib_flat.cpu(), m.table))
    # a Flux-layout vector loaded back reproduces the library flat exactly, and the loss with it
    loss0 = md2hip.train_loss(m, x, None, cache, params)[0].item()
    m.flat.data.zero_()
    md2hip.set_flux_params(m, flux)
    assert torch.equal(m.flat.detach(), lib_flat)
    assert md2hip.train_loss(m, x, None, cache, params)[0].item() == loss0


def test_flux_grads_and_loss_cotangent():
    import md2hip
    m, cache, params = _model()
    x = D.triplets(2, 3, 64, 128, seed=2).float().cuda().contiguous()
    md2hip.train_loss(m, x, None, cache, params)
    g1 = md2hip.gradient(m).detach().clone()
    assert torch.equal(md2hip.flux_params(m, grads=True).cpu(), _flip_reference(g1.cpu(), m.table))
    md2hip.train_loss(m, x, None, cache, params)
    g25 = md2hip.gradient(m, dloss=2.5).detach().clone()
    err = ((g25 - 2.5 * g1).abs().max() / (2.5 * g1).abs().max()).item()
    assert err < 1e-5, err          # scaling before vs after the fp32 backward: rounding only
