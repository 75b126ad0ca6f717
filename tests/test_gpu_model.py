"""Full train step (Model + train_loss + pullback + ADAM) on the GPU vs the fp64 CPU oracle.

Same flat parameters (Flux-default init, seed 42) and inputs; the GPU's per-pixel argmin is
imposed on the oracle (see test_gpu_loss.py for why).  Tolerances:
  * forward: disparities / poses relative 1e-5, loss relative 1e-6;
  * gradients, per parameter tensor (tests/_model_parity.py check_step):
      - backward: within max(4 x its fp32 floor, 2e-5) of the fp64 oracle evaluated AT THE GPU's
        own forward outputs (the exact gradient at the GPU's forward point);
      - end to end: within max(4 x the fp32 floor, 2e-5) of the plain fp64 oracle, the floor
        being the max over four fp32 realisations of the reference (tests/_model_parity.py);
  * every GPU branch decision is imposed on the oracle, including grid_sample's bilinear cells
    and border clamps, so textured and uniform-random source frames get the same bounds as
    kink-free affine ramps."""
import numpy as np
import pytest
import torch

from oracle import md2_oracle as O
from tests import _data as D

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("arch,sources", [(18, "ramp"), (18, "texture"), (18, "uniform"), (34, "ramp"),
                                          (50, "texture")],
                         ids=["r18-ramp", "r18-texture", "r18-uniform", "r34-ramp", "r50-texture"])
def test_model_train_loss_parity(arch, sources):
    """ResNet-18 (the measured config), ResNet-34 and the Bottleneck ResNet-50 of config 5."""
    from tests._model_parity import check_step, oracle_bounds, run
    g, o, errs = run(sources=sources, arch=arch)
    assert g["loss"] == g["tail_loss"]
    b = oracle_bounds(g, o, arch=arch)
    check_step(g, o, errs, b, label=f"R{arch} {sources}")


@pytest.mark.parametrize("levels,target_id,source_ids,W", [((1, 3, 5), 1, (2, 3), 128), ((2, 4), 3, (1, 2), 128),
                                                        ((1, 2, 3, 4, 5), 2, (3, 1), 128),
                                                        ((1, 3, 5), 2, (1, 3), 96)],
                         ids=["levels135-target1", "levels24-target3", "levels12345-sources31",
                              "levels135-96wide"])
def test_model_general_levels_and_frame_ids(levels, target_id, source_ids, W):
    """Any strictly increasing scale_levels in 1:5 (src/depth_decoder.jl:26-50, incl. the 1/16
    level 1 and a decoder that stops short of full resolution) and any target / two source frames
    of the triplet (src/Monodepth.jl:49-60; pose pairs _get_pose_features, src/model.jl:64-69).
    At width 96 the level-1 head is 6 pixels wide: its kernels move 2-pixel vectors."""
    from tests._model_parity import check_step, oracle_bounds, run
    kw = dict(levels=levels, target_id=target_id, source_ids=source_ids)
    g, o, errs = run(sources="texture", W=W, **kw)
    assert len(g["disps"]) == len(levels)
    for l, d in zip(levels, g["disps"]):
        assert d.shape[-2:] == (64 // 2 ** (5 - l), W // 2 ** (5 - l))
    b = oracle_bounds(g, o, **kw)
    check_step(g, o, errs, b, label=f"{kw} W{W}")


def test_backward_segments_cover_params():
    import md2hip
    from tests._model_parity import run  # noqa: F401
    enc = md2hip.ResNet(18, in_channels=3)
    m = md2hip.Model(enc, md2hip.DepthDecoder(encoder_channels=enc.stages, scale_levels=[2, 3, 4, 5],
                                              embedding_levels=0), md2hip.PoseDecoder(512))
    K, invK = D.intrinsics(128, 64)
    x = D.triplets(1, 3, 64, 128).float().cuda()
    md2hip.train_loss(m, x, None, md2hip.TrainCache(K=K.numpy(), invK=invK.numpy()),
                      md2hip.Params(target_size=(128, 64), batch_size=1, automasking=False))
    ranges = m._last.backward()
    covered = np.zeros(m.numel, dtype=np.int32)
    for off, ln in ranges:
        covered[off:off + ln] += 1
    assert (covered == 1).all()


def test_adam_matches_flux_rule():
    """ADAM kernel vs Flux.Optimise.apply!(::ADAM) restated in numpy, on the GPU's own gradient."""
    import md2hip
    enc = md2hip.ResNet(18, in_channels=3)
    m = md2hip.Model(enc, md2hip.DepthDecoder(encoder_channels=enc.stages, scale_levels=[2, 3, 4, 5],
                                              embedding_levels=0), md2hip.PoseDecoder(512))
    K, invK = D.intrinsics(128, 64)
    cache = md2hip.TrainCache(K=K.numpy(), invK=invK.numpy())
    params = md2hip.Params(target_size=(128, 64), batch_size=2, automasking=False)
    opt = md2hip.ADAM(1e-4)
    p = m.flat.double().cpu().numpy().copy()
    mm = np.zeros_like(p)
    vv = np.zeros_like(p)
    for step in range(1, 3):
        x = D.triplets(2, 3, 64, 128, seed=step).float().cuda()
        md2hip.train_loss(m, x, None, cache, params)
        md2hip.gradient(m)
        gr = m.grad.double().cpu().numpy()
        opt.update(m)
        mm = 0.9 * mm + 0.1 * gr
        vv = 0.999 * vv + 0.001 * gr * gr
        p = p - (mm / (1 - 0.9 ** step)) / (np.sqrt(vv / (1 - 0.999 ** step)) + 1e-8) * 1e-4
        got = m.flat.double().cpu().numpy()
        assert np.abs(got - p).max() < 1e-6, np.abs(got - p).max()
        p = got.copy()


def test_eval_disparity_parity():
    import md2hip
    from oracle import md2_oracle as O
    enc = md2hip.ResNet(18, in_channels=3)
    m = md2hip.Model(enc, md2hip.DepthDecoder(encoder_channels=enc.stages, scale_levels=[2, 3, 4, 5],
                                              embedding_levels=0), md2hip.PoseDecoder(512))
    x = D.triplets(2, 3, 64, 128)[:, 1].contiguous()
    got = md2hip.eval_disparity(m, x.float().cuda())
    P = O.unflatten(m.flat.double().cpu(), O.param_spec(18, 3, (2, 3, 4, 5)))
    ref = O.eval_disparity(P, x)
    for a, b in zip(got, ref):
        assert D.rel_err(a.cpu(), b) < 1e-5


@pytest.mark.parametrize("arch", [18])
def test_encoder_layers_parity(arch):
    """Every encoder layer of the GPU forward vs fp64 torch evaluated on the GPU's OWN input to
    that layer (md2_model_debug_tensor): conv outputs, BN(+residual)+ReLU, max-pool.  Catches
    wiring errors that train-mode BN would hide from the final outputs (a per-channel affine
    error in a conv output cancels in the forward but not in the backward)."""
    import torch.nn.functional as F
    import md2hip
    from oracle import md2_oracle as O
    N, C, H, W = 2, 3, 64, 128
    x = D.triplets(N, C, H, W, seed=7)
    enc = md2hip.ResNet(arch, in_channels=C)
    model = md2hip.Model(enc, md2hip.DepthDecoder(encoder_channels=enc.stages, scale_levels=[2, 3, 4, 5],
                                                  embedding_levels=0),
                         md2hip.PoseDecoder(enc.stages[-1]), seed=42)
    K, invK = D.intrinsics(W, H)
    cache = md2hip.TrainCache(K=K.numpy(), invK=invK.numpy())
    params = md2hip.Params(target_size=(W, H), batch_size=N, automasking=False)
    md2hip.train_loss(model, x.float().cuda().contiguous(), None, cache, params)
    t = {k: v.double().cpu() for k, v in model._last.debug_tensors().items()}
    P = O.unflatten(model.flat.detach().double().cpu(), O.param_spec(arch, C, (2, 3, 4, 5)))

    def bn(y, name):
        return F.batch_norm(y, None, None, P[name + ".gamma"], P[name + ".beta"], training=True,
                            eps=1e-5)

    errs = {}
    frames = x.float().double().transpose(0, 1).reshape(3 * N, C, H, W)   # frame-major batch
    errs["stem.y"] = D.rel_err(t["stem.y"], F.conv2d(frames, P["encoder.stem.conv.weight"], stride=2, padding=3))
    errs["stem.out"] = D.rel_err(t["stem.out"], F.relu(bn(t["stem.y"], "encoder.stem.bn")))
    errs["maxpool.out"] = D.rel_err(t["maxpool.out"], F.max_pool2d(t["stem.out"], 3, 2, 1))
    cur = t["maxpool.out"]
    for si, nblocks in enumerate(O.RESNET_LAYERS[arch]):
        for bi in range(nblocks):
            q, p = f"layer{si + 1}.{bi}", f"encoder.layer{si + 1}.{bi}"
            stride = 2 if (bi == 0 and si > 0) else 1
            errs[q + ".conv1.y"] = D.rel_err(t[q + ".conv1.y"], F.conv2d(cur, P[p + ".conv1.weight"], stride=stride, padding=1))
            errs[q + ".relu1"] = D.rel_err(t[q + ".relu1"], F.relu(bn(t[q + ".conv1.y"], p + ".bn1")))
            errs[q + ".conv2.y"] = D.rel_err(t[q + ".conv2.y"], F.conv2d(t[q + ".relu1"], P[p + ".conv2.weight"], padding=1))
            if q + ".down.y" in t:
                errs[q + ".down.y"] = D.rel_err(t[q + ".down.y"], F.conv2d(cur, P[p + ".down.weight"], stride=2))
                res = bn(t[q + ".down.y"], p + ".down_bn")
            else:
                res = cur
            errs[q + ".out"] = D.rel_err(t[q + ".out"], F.relu(bn(t[q + ".conv2.y"], p + ".bn2") + res))
            cur = t[q + ".out"]
    sq = F.relu(F.conv2d(cur, P["pose.squeezer.weight"], P["pose.squeezer.bias"]))
    errs["pose.sq"] = D.rel_err(t["pose.sq"], sq)
    pin = torch.cat([t["pose.sq"][:2 * N], t["pose.sq"][N:]], 1)   # pairs (q, q + N)
    errs["pose.conv1"] = D.rel_err(t["pose.conv1"], F.relu(F.conv2d(pin, P["pose.conv1.weight"], P["pose.conv1.bias"], padding=1)))
    errs["pose.conv2"] = D.rel_err(t["pose.conv2"], F.relu(F.conv2d(t["pose.conv1"], P["pose.conv2.weight"], P["pose.conv2.bias"], padding=1)))
    bad = {k: v for k, v in errs.items() if v > 1e-5}
    assert not bad, bad


def test_train_loss_visualization():
    """train_loss(..., do_visualization=true) returns (loss, vis_disparity, vis_warped, vis_loss)
    (src/training.jl:34-37,71-74); the warped sources match the oracle's warp of the model's own
    last disparity and poses."""
    import md2hip
    N, H, W = 2, 64, 128
    enc = md2hip.ResNet(18, in_channels=3)
    model = md2hip.Model(enc, md2hip.DepthDecoder(encoder_channels=enc.stages, scale_levels=[2, 3, 4, 5],
                                                  embedding_levels=0), md2hip.PoseDecoder(512), seed=42)
    K, invK = md2hip.depth10k_intrinsics(W, H)
    cache = md2hip.TrainCache(K=K, invK=invK)
    params = md2hip.Params(target_size=(W, H), batch_size=N, automasking=False)
    x = D.triplets(N, 3, H, W, seed=3, ramp_sources=True).float().cuda().contiguous()
    loss, vd, vw, vl = md2hip.train_loss(model, x, None, cache, params, True)
    torch.cuda.synchronize()
    assert vd.shape == (N, 1, H, W) and vl.shape == (N, 1, H, W) and len(vw) == 2
    assert all(w.shape == (N, 3, H, W) for w in vw)
    assert torch.isfinite(vl).all() and (vl >= 0).all()
    disps, pose = model._last.outputs()
    pose = pose.cpu().double()
    poses = [(pose[s * N:(s + 1) * N, 0:3], pose[s * N:(s + 1) * N, 3:6]) for s in range(2)]
    Ps = O.poses_to_transforms(poses, (1, 3), 2)
    ref = O.warp(vd.double(), x.cpu().double(), Ps, torch.tensor(K, dtype=torch.float64),
                 torch.tensor(invK, dtype=torch.float64), (1, 3), 0.1, 100.0)
    for s in range(2):
        assert D.rel_err(vw[s], ref[s]) < 1e-5, s
    # the gradient path still works after a visualising train_loss
    md2hip.gradient(model)
    torch.cuda.synchronize()
    assert torch.isfinite(model.grad).all()


def test_executors_see_updated_weights():
    """Every cached executor keeps its own packed conv weights; after an ADAM step through one of
    them the others must re-pack before use.  Sequence: train_loss + gradient at
    N=2, eval_disparity at N=1 (a second executor, built between gradient() and update!),
    ADAM update, then eval_disparity at N=1 and a forward at N=2 -- all against the oracle on the
    UPDATED flat parameters."""
    import md2hip
    enc = md2hip.ResNet(18, in_channels=3)
    m = md2hip.Model(enc, md2hip.DepthDecoder(encoder_channels=enc.stages, scale_levels=[2, 3, 4, 5],
                                              embedding_levels=0), md2hip.PoseDecoder(512), seed=42)
    K, invK = D.intrinsics(128, 64)
    cache = md2hip.TrainCache(K=K.numpy(), invK=invK.numpy())
    params = md2hip.Params(target_size=(128, 64), batch_size=2, automasking=False)
    x2 = D.triplets(2, 3, 64, 128, seed=3).float().cuda()
    x1 = D.triplets(1, 3, 64, 128, seed=4)[:, 1].contiguous()
    opt = md2hip.ADAM(1e-3)                       # 10x Flux's step: stale weights are obvious
    md2hip.train_loss(m, x2, None, cache, params)
    md2hip.gradient(m)
    before = md2hip.eval_disparity(m, x1.float().cuda())
    opt.update(m)
    after = md2hip.eval_disparity(m, x1.float().cuda())
    P = O.unflatten(m.flat.double().cpu(), O.param_spec(18, 3, (2, 3, 4, 5)))
    ref = O.eval_disparity(P, x1.float().double())
    for s, (a, b) in enumerate(zip(after, ref)):
        assert D.rel_err(a.cpu(), b) < 1e-5, s
    assert D.rel_err(before[-1].cpu(), ref[-1]) > 1e-3       # the update did change the output
    print(f"\nstale-vs-updated disparity difference {D.rel_err(before[-1].cpu(), ref[-1]):.3e}")
    disps, _ = m(x2)
    ref2, _ = O.model_forward(P, x2.cpu().double())
    for s, (a, b) in enumerate(zip(disps, ref2)):
        assert D.rel_err(a.cpu(), b) < 1e-5, s


def test_eval_between_train_loss_and_gradient():
    """eval_disparity between train_loss and gradient() must not change the gradient
    (inference runs on an executor without a pending forward), and the library refuses a backward
    on an executor whose forward an eval_disparity discarded (MD2_ESTATE)."""
    import md2hip
    from md2hip._lib import MD2Error
    K, invK = D.intrinsics(128, 64)
    cache = md2hip.TrainCache(K=K.numpy(), invK=invK.numpy())
    params = md2hip.Params(target_size=(128, 64), batch_size=2, automasking=False)
    x = D.triplets(2, 3, 64, 128, seed=3).float().cuda()
    xe = D.triplets(2, 3, 64, 128, seed=9)[:, 1].float().cuda().contiguous()
    grads = []
    for with_eval in (False, True):
        enc = md2hip.ResNet(18, in_channels=3)
        m = md2hip.Model(enc, md2hip.DepthDecoder(encoder_channels=enc.stages, scale_levels=[2, 3, 4, 5],
                                                  embedding_levels=0), md2hip.PoseDecoder(512), seed=42)
        md2hip.train_loss(m, x, None, cache, params)
        if with_eval:
            md2hip.eval_disparity(m, xe)
        md2hip.gradient(m)
        grads.append(m.grad.clone())
    assert torch.equal(grads[0], grads[1])
    # the C-ABI contract: eval on the training executor itself discards its forward
    ex = m._last
    md2hip.train_loss(m, x, None, cache, params)
    dptr = (__import__("ctypes").c_void_p * 5)()
    from md2hip._lib import check, lib, ptr, stream_of
    check(lib().md2_model_eval_disparity(ex.handle, ptr(xe), 2, dptr, stream_of()))
    with pytest.raises(MD2Error, match="no pending forward_loss"):
        ex.backward_segment(0)
