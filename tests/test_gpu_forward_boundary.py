"""The Model boundary without the loss tail: ``(m)(x, source_ids, target_id)``
forward only (md2_model_forward, src/model.jl:31-55) and its pullback from caller cotangents
(md2_model_set_cotangents / md2_model_backward_from), all through the C-ABI.

  * the forward-only outputs are bit-identical to md2_model_forward_loss's;
  * fed the loss tail's own d disparity / d pose (md2_loss_fwd_bwd with sigmoid_grad = 0 at the
    forward's outputs), the pullback's flat gradient is bit-identical to the fused path's;
  * the pullback is linear: zero cotangents give a zero gradient, doubled cotangents exactly
    twice the gradient (every rounding commutes with a power-of-two scale);
  * a backward after a forward-only call without cotangents is refused (MD2_ESTATE)."""
import pytest
import torch

from tests import _data as D

pytestmark = pytest.mark.gpu


def _setup(N, H, W, arch=18, emb=0):
    import md2hip
    enc = md2hip.ResNet(arch, in_channels=3)
    m = md2hip.Model(enc, md2hip.DepthDecoder(encoder_channels=enc.stages, scale_levels=[2, 3, 4, 5],
                                              embedding_levels=emb), md2hip.PoseDecoder(enc.stages[-1]), seed=42)
    K, invK = D.intrinsics(W, H)
    cache = md2hip.TrainCache(K=K.numpy(), invK=invK.numpy())
    params = md2hip.Params(target_size=(W, H), batch_size=N, automasking=False)
    x = D.triplets(N, 3, H, W).float().cuda().contiguous()
    return m, cache, params, x


@pytest.mark.parametrize("N,H,W", [(2, 64, 128), (12, 128, 416)], ids=["b2-64x128", "bench-b12-416x128"])
def test_forward_only_and_pullback_bit_identical_to_fused(N, H, W):
    import md2hip
    m, cache, params, x = _setup(N, H, W)
    ex = m.executor(tuple(x.shape), cache, params)
    loss_a = ex.forward_loss(x).clone()
    d_a, p_a = ex.outputs()
    ex.backward()
    torch.cuda.synchronize()
    g_a = m.grad.clone()

    m.grad.fill_(float("nan"))
    disps, poses = m(x, cache=cache, params=params)           # md2_model_forward
    d_b, p_b = ex.outputs()
    for a, b, c in zip(d_a, d_b, disps):
        assert torch.equal(a, b) and torch.equal(b, c)
    assert torch.equal(p_a, p_b)
    for s in range(2):
        assert torch.equal(poses[s].rvec, p_a[s * N:(s + 1) * N, 0:3])
        assert torch.equal(poses[s].tvec, p_a[s * N:(s + 1) * N, 3:6])

    # the reference's train_loss body on the model's outputs (src/training.jl:25-77), w.r.t. the
    # disparities themselves (no fused sigmoid derivative)
    tail = md2hip.loss_tail([d.contiguous() for d in d_b], [(p.rvec, p.tvec) for p in poses], x, None,
                            cache, params, sigmoid_grad=False)
    assert torch.equal(tail["loss"], loss_a)
    g_b = md2hip.pullback(m, tail["d_disp"], tail["d_pose"]).clone()
    torch.cuda.synchronize()
    assert torch.isfinite(g_b).all()
    diff = (g_a != g_b).sum().item()
    assert diff == 0, f"{diff} of {g_a.numel()} gradient entries differ from the fused path"

    # linearity: 2x the cotangents -> exactly 2x the gradient; zero cotangents -> zero
    m(x, cache=cache, params=params)
    g2 = md2hip.pullback(m, [2 * d for d in tail["d_disp"]], 2 * tail["d_pose"]).clone()
    assert torch.equal(g2, 2 * g_b)
    m(x, cache=cache, params=params)
    g0 = md2hip.pullback(m, None, None)
    assert (g0 == 0).all()


def test_pose_only_cotangent_touches_no_depth_decoder_weight():
    """d pose alone: the DepthDecoder's parameters get exactly zero, the PoseDecoder's do not."""
    import md2hip
    m, cache, params, x = _setup(2, 64, 128)
    m(x, cache=cache, params=params)
    dp = torch.randn(4, 6, device="cuda")
    g = md2hip.pullback(m, None, dp)
    torch.cuda.synchronize()
    for name, shape, off in m.table:
        n = 1
        for s in shape:
            n *= s
        t = g[off:off + n]
        if name.startswith("depth."):
            assert (t == 0).all(), name
    pose_w = [g[off:off + 10] for name, _, off in m.table if name.startswith("pose.conv3")]
    assert any((t != 0).any() for t in pose_w)


def test_backward_after_forward_only_needs_cotangents():
    import md2hip
    m, cache, params, x = _setup(1, 64, 128)
    m(x, cache=cache, params=params)
    with pytest.raises(md2hip.MD2Error, match="cotangents"):
        m._last.backward_segment(0)


def test_mpi_forward_only_matches_forward_loss():
    """MPI mode (embedding_levels = 21, 4 planes): the forward-only plane disparities and poses
    equal the fused forward's."""
    import md2hip
    m, cache, params, x = _setup(1, 64, 128, emb=21)
    bins = md2hip.disparity_bins(1, 4, u=torch.rand(1, 4, dtype=torch.float64, generator=torch.Generator().manual_seed(3)))
    ex = m.executor(tuple(x.shape), cache, params, num_bins=4)
    ex.set_bins(bins)
    ex.forward_loss(x)
    d_a, p_a = ex.outputs()
    d_b, poses = m(x, cache=cache, params=params, num_bins=4, bins=bins)
    for a, b in zip(d_a, d_b):
        assert a.shape[0] == 4 and torch.equal(a, b)
    assert torch.equal(p_a[0:1, 0:3], poses[0].rvec)
