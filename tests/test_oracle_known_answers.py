"""The reference's own known answers (test/runtests.jl) re-expressed against the CPU oracle.

These pin the oracle before it is trusted as the parity checker."""
import math

import numpy as np
import pytest
import torch
from scipy.spatial.transform import Rotation

from oracle import md2_oracle as O



@pytest.fixture(autouse=True)
def _float64_default():
    """fp64 like the reference's CPU runtests; restored afterwards (no import-time side effect)."""
    old = torch.get_default_dtype()
    torch.set_default_dtype(torch.float64)
    yield
    torch.set_default_dtype(old)


def rotvec(v):
    """Stand-in for Rotations.jl ``RotationVec`` (test/runtests.jl:18)."""
    return torch.tensor(Rotation.from_rotvec(np.asarray(v, dtype=np.float64)).as_matrix())


def test_rotations():
    """test/runtests.jl:14-29: so3_exp_map(v) == RotationVec(v...) (atol 1e-5)."""
    g = torch.Generator().manual_seed(0)
    for _ in range(16):
        v = torch.rand(1, 3, generator=g)
        assert torch.allclose(O.so3_exp_map(v)[0], rotvec(v[0]), atol=1e-5)


def test_hat_rrule_fd():
    """test/runtests.jl:21 test_rrule(hat, v): finite differences on a scalar of hat(v)."""
    v = torch.rand(4, 3, requires_grad=True)
    w = torch.rand(4, 3, 3)
    torch.autograd.gradcheck(lambda a: (O.hat(a) * w).sum(), (v,))
    # the hand-written pullback (src/utils.jl:134-145), restated
    d = w
    gv = torch.stack([d[:, 2, 1] - d[:, 1, 2], -d[:, 2, 0] + d[:, 0, 2], d[:, 1, 0] - d[:, 0, 1]], 1)
    (O.hat(v) * w).sum().backward()
    assert torch.allclose(v.grad, gv)


def test_transformation():
    """test/runtests.jl:31-50: composeT forward and exact inverse."""
    g = torch.Generator().manual_seed(1)
    rvec, tvec, p = torch.rand(1, 3, generator=g), torch.rand(1, 3, generator=g), torch.rand(1, 3, generator=g)
    R, t = O.composeT(rvec, tvec, False)
    tp = rotvec(rvec[0]) @ p[0] + t[0]
    np_ = (R @ p.unsqueeze(-1)).squeeze(-1) + t
    assert torch.allclose(np_[0], tp, atol=1e-6)
    R, t = O.composeT(rvec, tvec, True)
    invR = rotvec(rvec[0]).T
    tp2 = invR @ np_[0] - invR @ tvec[0]
    op = (R @ np_.unsqueeze(-1)).squeeze(-1) + t
    assert torch.allclose(op[0], tp2, atol=1e-6)
    assert torch.allclose(op, p, atol=1e-6)


def test_ssim_known_answers():
    """test/runtests.jl:52-68."""
    ones = torch.ones(1, 1, 2, 2)
    assert torch.allclose(O.ssim(ones, ones), torch.zeros(1, 1, 2, 2))
    s = O.ssim(ones, torch.zeros(1, 1, 2, 2))
    assert torch.all((s - 0.5).abs() <= 0.1)
    # exact value under the restated semantics: (1 - c1*c2/((1+c1)*c2))/2
    assert torch.allclose(s, torch.full_like(s, (1 - 1e-4 / (1 + 1e-4)) / 2))
    g = torch.Generator().manual_seed(2)
    a, b = torch.rand(2, 1, 2, 2, generator=g), torch.rand(2, 1, 2, 2, generator=g)
    assert torch.allclose(O.ssim(a, b), O.ssim(b, a))


def _julia_2x2(vals):
    """reshape(transpose(reshape(vals, (2,2))), (2,2,1,1)) as torch [1,1,H,W]."""
    v = list(vals)
    # Julia d[w,h]: d[1,1]=v0, d[2,1]=v2, d[1,2]=v1, d[2,2]=v3  -> torch t[h][w]
    return torch.tensor([[v[0], v[2]], [v[1], v[3]]]).view(1, 1, 2, 2)


def test_smooth_loss_known_answers():
    """test/runtests.jl:70-83 (0.2542 +- 1e-4)."""
    disp = _julia_2x2([0.0, 0.1, 0.2, 0.3])
    image = torch.ones(1, 1, 2, 2)
    sl = O.smooth_loss(disp[:, 0], image)
    tl = (disp[..., :-1] - disp[..., 1:]).abs().mean() + (disp[..., :-1, :] - disp[..., 1:, :]).abs().mean()
    assert torch.allclose(sl, tl)
    image = _julia_2x2([0.1, 0.2, 0.3, 0.4])
    sl = O.smooth_loss(disp[:, 0], image)
    assert abs(sl.item() - 0.2542) <= 1e-4
    assert abs(sl.item() - (0.2 * math.exp(-0.2) + 0.1 * math.exp(-0.1))) < 1e-12


def test_disparity_to_depth_bounds():
    """test/runtests.jl:85-92."""
    d = O.disparity_to_depth(torch.rand(2, 32, 32), 0.1, 100.0)
    assert d.min() >= 0.1 and d.max() <= 100.0


def test_identity_warp():
    """test/runtests.jl:94-122: backproject -> project(R=I, t=0) -> grid_sample == image."""
    res, N = 16, 2
    g = torch.Generator().manual_seed(3)
    image = torch.rand(N, 1, res, res, generator=g)
    depth = torch.rand(N, 1, res * res, generator=g)
    K = torch.tensor([[910.0, 0, res / 2], [0, 910.0, res / 2], [0, 0, 1]])
    invK = torch.linalg.inv(K)
    R = O.so3_exp_map(torch.zeros(N, 3))
    t = torch.zeros(N, 3)
    pts = O.backproject(depth, invK, res, res)
    uv = O.project(pts, K, R, t, res, res)
    grid = uv.reshape(N, 2, res, res).permute(0, 2, 3, 1)
    sampled = O.grid_sample_zeros(image, grid)
    assert torch.allclose(image, sampled, atol=1e-3)


def test_pose_derivative():
    """test/runtests.jl:124-142 (no assertion upstream; SURVEY section 4 restated values)."""
    x = torch.tensor([3.0, 2, 1]).view(1, 3, 1)
    target = torch.tensor([1.0, 2, 3]).view(1, 3, 1)
    r = torch.tensor([[1.0, 0, 0]], requires_grad=True)
    t = torch.zeros(1, 3, requires_grad=True)
    R = O.so3_exp_map(r)
    l = torch.sqrt(((R @ x + t.unsqueeze(-1)) - target).pow(2).sum(1)).sum()
    l.backward()
    assert abs(l.item() - 2.775608) < 1e-6
    assert torch.allclose(r.grad[0], torch.tensor([1.343521, 1.100367, -2.868871]), atol=1e-6)
    assert torch.allclose(t.grad[0], torch.tensor([0.720563, -0.634407, -0.279851]), atol=1e-6)
