"""GPU: MINE plane rendering (src/render.jl:21-114) through the C-ABI against the fp64 oracle --
get_src_xyz_from_plane_disparity, get_tgt_xyz_from_plane_disparity, sample, plane_volume_rendering
and the fused render_tgt_rgb_depth, at the reference cross-check scripts' shape (B=2, N=32,
100x200, test/test_render_tgt_rgb_depth.jl:16) and small/ragged ones.

Tolerance: fp32 kernels vs fp64 oracle on the same fp32 inputs, |err| <= 1e-4 (abs) + 1e-4 (rel)
for sampled / rendered values, 1e-5 relative for the pointwise xyz maps.  Discontinuities are
excluded explicitly: the valid mask flips where u or v is within 1e-3 of 0 (chained comparison,
render.jl:83) and the homography is singular where |u| or |v| exceeds 1e4 (a2 ~ 0: fp32 and fp64
can land on opposite borders); pixels touching either are left out of the comparison and their
count is bounded."""
import pytest
import torch

from oracle import md2_oracle as O

pytestmark = pytest.mark.gpu

CASES = [(2, 32, 100, 200, "moderate"), (1, 5, 37, 61, "moderate"), (3, 8, 64, 96, "wide")]


def _inputs(B, N, H, W, poses, seed):
    g = torch.Generator().manual_seed(seed)
    rgb = torch.rand(B, N, 3, H, W, generator=g)
    sigma = torch.randn(B, N, 1, H, W, generator=g)      # negative sigmas exercise the clamp
    xyz = torch.rand(B, N, H, W, 3, generator=g)
    u = torch.rand(B, N, generator=g)
    disp = (O.disparity_bins(N, u.double()) if N > 1 else 0.5 + 0.5 * u.double()).float()   # MINE's bins
    if poses == "moderate":
        rvec, tvec = 0.05 * torch.randn(B, 3, generator=g), 0.1 * torch.randn(B, 3, generator=g)
    else:                                                 # the reference scripts' randn poses
        rvec, tvec = torch.randn(B, 3, generator=g), torch.randn(B, 3, generator=g)
    K, iK = O.depth10k_K(W, H)
    return rgb, sigma, xyz, disp, rvec, tvec, K.float(), iK.float()


def _d(t):
    return t.double()


def _ambiguous(coords, H, W):
    u, v, _ = coords
    return (u.abs() < 1e-3) | (v.abs() < 1e-3) | (u.abs() > 1e4) | (v.abs() > 1e4)   # [BN, HW]


def _close(got, ref, keep, rtol=1e-4, atol=1e-4, floor=None):
    """|got - ref| - rtol |ref| <= max(atol, 4 x the fp32 floor) over the kept pixels, where the
    floor is the same excess of the oracle run in fp32 (torch CPU) on the same inputs."""
    def excess(a):
        a = a.double().cpu()[keep]
        return ((a - ref[keep]).abs() - rtol * ref[keep].abs()).max().item() if a.numel() else 0.0
    err = excess(got)
    tol = max(atol, 4 * excess(floor)) if floor is not None else atol
    assert err <= tol, (err, tol)


@pytest.mark.parametrize("B,N,H,W,poses", CASES)
def test_src_and_tgt_xyz(B, N, H, W, poses):
    from md2hip import render as R
    rgb, sigma, xyz, disp, rvec, tvec, K, iK = _inputs(B, N, H, W, poses, 1)
    mg = R.create_meshgrid(H, W, "cuda")
    assert torch.equal(mg.cpu().double(), O.create_meshgrid(H, W))
    got = R.get_src_xyz_from_plane_disparity(mg, disp.cuda(), iK)
    ref = O.get_src_xyz_from_plane_disparity(O.create_meshgrid(H, W), _d(disp), _d(iK))
    assert torch.allclose(got.cpu().double(), ref, rtol=1e-5, atol=1e-6)
    pose = torch.cat([rvec, tvec], 1)
    gt = R.get_tgt_xyz_from_plane_disparity(got, R_pose(rvec, tvec))
    rt = O.get_tgt_xyz_from_plane_disparity(got.cpu().double(), _d(rvec), _d(tvec))
    assert torch.allclose(gt.cpu().double(), rt, rtol=1e-5, atol=1e-4)
    assert torch.equal(R.get_tgt_xyz_from_plane_disparity(got, pose.cuda()), gt)


def R_pose(rvec, tvec):
    import md2hip
    return md2hip.Pose(rvec.cuda(), tvec.cuda())


@pytest.mark.parametrize("B,N,H,W,poses", CASES)
@pytest.mark.parametrize("C", [7, 3])
def test_sample_matches_oracle(B, N, H, W, poses, C):
    from md2hip import render as R
    _, _, _, disp, rvec, tvec, K, iK = _inputs(B, N, H, W, poses, 2)
    g = torch.Generator().manual_seed(5)
    src = torch.rand(B * N, C, H, W, generator=g)
    depth = 1.0 / disp
    tgt, valid = R.sample(src.cuda(), depth.cuda(), R_pose(rvec, tvec), K, iK)
    rt, rv, coords = O.mine_sample(_d(src), _d(depth), _d(rvec), _d(tvec), _d(K), _d(iK), return_coords=True)
    amb = _ambiguous(coords, H, W)
    assert amb.double().mean().item() < 0.02
    keep = ~amb
    assert torch.equal(valid.cpu().bool()[keep], rv[keep])
    _close(tgt.view(B * N, C, H * W).permute(0, 2, 1), rt.view(B * N, C, H * W).permute(0, 2, 1), keep)


@pytest.mark.parametrize("B,N,H,W", [(2, 32, 100, 200), (1, 1, 9, 13), (2, 3, 16, 40)])
def test_plane_volume_rendering_matches_oracle(B, N, H, W):
    from md2hip import render as R
    rgb, sigma, xyz, *_ = _inputs(B, N, H, W, "moderate", 3)
    sigma = sigma.abs()
    out, acc, w = R.plane_volume_rendering(rgb.cuda(), sigma.cuda(), xyz.cuda())
    ro, ra, rw = O.plane_volume_rendering(_d(rgb), _d(sigma), _d(xyz))
    for got, ref in ((out, ro), (acc, ra), (w, rw)):
        assert torch.allclose(got.cpu().double(), ref, rtol=1e-4, atol=1e-5), (got.cpu().double() - ref).abs().max()


@pytest.mark.parametrize("B,N,H,W,poses", CASES)
def test_render_tgt_rgb_depth_matches_oracle(B, N, H, W, poses):
    from md2hip import render as R
    rgb, sigma, xyz, disp, rvec, tvec, K, iK = _inputs(B, N, H, W, poses, 4)
    out, depth, mask = R.render_tgt_rgb_depth(rgb.cuda(), sigma.cuda(), disp.cuda(), xyz.cuda(),
                                              R_pose(rvec, tvec), iK, K)
    ro, rd, rm, coords = O.render_tgt_rgb_depth(_d(rgb), _d(sigma), _d(disp), _d(xyz), _d(rvec), _d(tvec),
                                                _d(iK), _d(K), return_coords=True)
    fo, fd, _ = O.render_tgt_rgb_depth(rgb, sigma, disp, xyz, rvec, tvec, iK, K)   # fp32 floor
    amb = _ambiguous(coords, H, W).view(B, N, H * W).any(1)          # [B, HW]
    assert amb.double().mean().item() < 0.3        # the "wide" randn poses fold planes behind the camera
    keep = ~amb
    assert torch.equal(mask.cpu().double().view(B, H * W)[keep], rm.view(B, H * W)[keep])
    px = lambda t, c: t.reshape(B, c, H * W).permute(0, 2, 1)   # noqa: E731
    _close(px(out, 3), px(ro, 3), keep, floor=px(fo, 3))
    _close(px(depth, N), px(rd, N), keep, floor=px(fd, N))


def test_render_equals_composition_of_ops():
    """The fused kernel equals the reference's chain of its own ops (cat -> sample -> clamp ->
    plane_volume_rendering -> sum of the valid mask), all on the GPU."""
    from md2hip import render as R
    B, N, H, W = 2, 6, 48, 80
    rgb, sigma, xyz, disp, rvec, tvec, K, iK = _inputs(B, N, H, W, "moderate", 6)
    rgb, sigma, xyz, disp = rgb.cuda(), sigma.cuda(), xyz.cuda(), disp.cuda()
    pose = R_pose(rvec, tvec)
    out, depth, mask = R.render_tgt_rgb_depth(rgb, sigma, disp, xyz, pose, iK, K)
    packed = torch.cat([rgb, sigma, xyz.permute(0, 1, 4, 2, 3)], 2).reshape(B * N, 7, H, W).contiguous()
    tgt, valid = R.sample(packed, (1.0 / disp).contiguous(), pose, K, iK)
    tgt = tgt.view(B, N, 7, H, W)
    s = tgt[:, :, 3:4]
    s = (s * (s >= 0)).contiguous()
    ro, ra, _ = R.plane_volume_rendering(tgt[:, :, 0:3].contiguous(), s,
                                         tgt[:, :, 4:7].permute(0, 1, 3, 4, 2).contiguous())
    assert torch.allclose(out, ro, rtol=1e-5, atol=1e-6)
    assert torch.allclose(depth, ra, rtol=1e-5, atol=1e-6)
    assert torch.equal(mask.view(B, H, W), valid.view(B, N, H, W).sum(1))


def test_render_rejects_bad_shapes():
    from md2hip import render as R
    B, N, H, W = 1, 2, 8, 8
    rgb, sigma, xyz, disp, rvec, tvec, K, iK = _inputs(B, N, H, W, "moderate", 7)
    with pytest.raises(ValueError):
        R.render_tgt_rgb_depth(rgb.cuda(), sigma.cuda(), disp.cuda(), xyz.cuda()[:, :, :4], R_pose(rvec, tvec), iK, K)
    with pytest.raises(ValueError):
        R.render_tgt_rgb_depth(rgb, sigma, disp, xyz, R_pose(rvec, tvec), iK, K)   # host tensors
