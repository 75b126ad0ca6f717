"""CPU: the MINE rendering restatement (oracle, src/render.jl:21-114) pinned by analytic known
answers of the reference's formulas.  The reference's own MINE checks (test/test_sample.jl,
test_plane_volume_rendering.jl, test_render_tgt_rgb_depth.jl, ...) compare against an external
PyTorch MINE checkout that is absent, so they hold no vectors; these properties pin the same
functions instead."""
import math

import numpy as np
import torch

from oracle import md2_oracle as O

D = torch.float64


def _K(W, H):
    return O.depth10k_K(W, H)


def test_meshgrid_is_one_based_w_h_1():
    g = O.create_meshgrid(3, 5)
    assert g.shape == (3, 5, 3)
    assert g[0, 0].tolist() == [1, 1, 1] and g[2, 4].tolist() == [5, 3, 1] and g[1, 3].tolist() == [4, 2, 1]


def test_src_xyz_depth_is_inverse_disparity():
    H, W = 4, 6
    K, iK = _K(W, H)
    disp = torch.tensor([[0.5, 0.25], [1.0, 0.1]], dtype=D)
    xyz = O.get_src_xyz_from_plane_disparity(O.create_meshgrid(H, W), disp, iK)
    assert xyz.shape == (2, 2, H, W, 3)
    assert torch.allclose(xyz[..., 2], (1 / disp).view(2, 2, 1, 1).expand(2, 2, H, W))
    # projecting back with K returns the 1-based pixel grid
    pix = xyz @ K.T
    assert torch.allclose(pix[..., :2] / pix[..., 2:], O.create_meshgrid(H, W)[..., :2].expand(2, 2, H, W, 2))


def test_volume_rendering_empty_and_opaque_first_plane():
    B, N, H, W = 1, 5, 2, 3
    g = torch.Generator().manual_seed(0)
    rgb = torch.rand(B, N, 3, H, W, generator=g, dtype=D)
    xyz = torch.rand(B, N, H, W, 3, generator=g, dtype=D)
    out, acc, w = O.plane_volume_rendering(rgb, torch.zeros(B, N, 1, H, W, dtype=D), xyz)
    assert torch.all(out == 0) and torch.all(w == 0)
    for n in range(N):      # exclusive cumprod of (T + 1e-6) with T = 1
        assert torch.allclose(acc[:, n], torch.full_like(acc[:, n], (1 + 1e-6) ** n))
    sigma = torch.zeros(B, N, 1, H, W, dtype=D)
    sigma[:, 0] = 1e9
    out, acc, w = O.plane_volume_rendering(rgb, sigma, xyz)
    assert torch.allclose(out, rgb[:, 0]) and torch.allclose(acc[:, 1], torch.full_like(acc[:, 1], 1e-6))


def test_volume_rendering_last_plane_distance_is_1e3():
    B, N, H, W = 1, 2, 1, 1
    rgb = torch.ones(B, N, 3, H, W, dtype=D)
    xyz = torch.tensor([0.0, 0, 0, 3, 4, 0], dtype=D).view(B, N, H, W, 3)   # |diff| = 5
    sigma = torch.tensor([0.1, 1e-3], dtype=D).view(B, N, 1, H, W)
    out, acc, w = O.plane_volume_rendering(rgb, sigma, xyz)
    T0, T1 = math.exp(-0.5), math.exp(-1.0)
    assert math.isclose(w[0, 0].item(), 1 - T0, rel_tol=1e-12)
    assert math.isclose(acc[0, 1].item(), T0 + 1e-6, rel_tol=1e-12)
    assert math.isclose(w[0, 1].item(), (T0 + 1e-6) * (1 - T1), rel_tol=1e-12)


def test_homography_is_plane_induced():
    """H_src_tgt maps a target pixel to the source pixel of the same point on the fronto-parallel
    plane z = d of the source camera: X_tgt = R X + t (render.jl:68-79)."""
    H, W = 40, 60
    K, iK = _K(W, H)
    g = torch.Generator().manual_seed(1)
    rvec = 0.05 * torch.randn(2, 3, generator=g, dtype=D)
    tvec = 0.2 * torch.randn(2, 3, generator=g, dtype=D)
    depth = torch.tensor([[2.0, 7.0, 30.0], [1.5, 4.0, 100.0]], dtype=D)
    Hst = O.mine_homographies(depth, rvec, tvec, K, iK).view(2, 3, 3, 3)
    R = O.so3_exp_map(rvec)
    p = torch.tensor([17.0, 9.0, 1.0], dtype=D)
    for b in range(2):
        for n in range(3):
            X = depth[b, n] * (iK @ p)
            Xt = R[b] @ X + tvec[b]
            pt = K @ Xt
            pt = pt / pt[2]
            back = Hst[b, n] @ pt
            assert torch.allclose(back / back[2], p, atol=1e-9)


def test_sample_identity_pose_and_chained_valid_mask():
    """Identity pose: H = I, so u = x, v = y (0-based); the chained comparison is u > 0 & v > 0
    and the grid is (x + 0.5)/(W/2) unnormalised by align_corners (render.jl:80-90)."""
    H, W, C = 5, 7, 2
    K, iK = _K(W, H)
    g = torch.Generator().manual_seed(2)
    src = torch.rand(1, C, H, W, generator=g, dtype=D)
    z = torch.zeros(1, 3, dtype=D)
    tgt, valid = O.mine_sample(src, torch.tensor([[3.0]], dtype=D), z, z, K, iK)
    v = valid.view(H, W)
    assert not v[0].any() and not v[:, 0].any() and v[1:, 1:].all()
    s = src[0].numpy()
    for y in range(H):
        for x in range(W):
            ix = min(max(((x + 0.5) / (W / 2) + 1) / 2 * (W - 1), 0), W - 1)
            iy = min(max(((y + 0.5) / (H / 2) + 1) / 2 * (H - 1), 0), H - 1)
            x0, y0 = int(np.floor(ix)), int(np.floor(iy))
            x1, y1 = min(x0 + 1, W - 1), min(y0 + 1, H - 1)
            wx, wy = ix - x0, iy - y0
            ref = (s[:, y0, x0] * (1 - wx) * (1 - wy) + s[:, y0, x1] * wx * (1 - wy) +
                   s[:, y1, x0] * (1 - wx) * wy + s[:, y1, x1] * wx * wy)
            assert np.allclose(tgt[0, :, y, x].numpy(), ref, atol=1e-12)


def test_render_identity_pose_is_rendering_of_the_resampled_planes():
    B, N, H, W = 1, 4, 6, 8
    K, iK = _K(W, H)
    g = torch.Generator().manual_seed(3)
    rgb = torch.rand(B, N, 3, H, W, generator=g, dtype=D)
    sigma = torch.randn(B, N, 1, H, W, generator=g, dtype=D)
    xyz = torch.rand(B, N, H, W, 3, generator=g, dtype=D)
    disp = torch.tensor([[1.0, 0.5, 0.2, 0.05]], dtype=D)
    z = torch.zeros(B, 3, dtype=D)
    out, depth, mask = O.render_tgt_rgb_depth(rgb, sigma, disp, xyz, z, z, iK, K)
    packed = torch.cat([rgb, sigma, xyz.permute(0, 1, 4, 2, 3)], 2).view(N, 7, H, W)
    tgt, valid = O.mine_sample(packed, 1 / disp, z, z, K, iK)
    s = tgt[:, 3:4].clamp(min=0).unsqueeze(0)
    ref = O.plane_volume_rendering(tgt[:, 0:3].unsqueeze(0), s, tgt[:, 4:7].permute(0, 2, 3, 1).unsqueeze(0))
    assert torch.allclose(out, ref[0]) and torch.allclose(depth, ref[1])
    assert torch.equal(mask[0, 0], valid.view(N, H, W).sum(0).to(D))
    assert mask[0, 0, 0, 0] == 0 and mask[0, 0, 1, 1] == N
