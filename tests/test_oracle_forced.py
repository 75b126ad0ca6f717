"""The oracle's forced-decision grid sampler (O.grid_sample_border_forced, the test hook that
imposes the GPU's bilinear cells / border clamps) is NNlib's grid_sample(:border) wherever the
imposed decisions are the oracle's own: same values and same gradients (grid and image)."""
import torch

from oracle import md2_oracle as O


def cells_of(grid, W, H):
    """The photometric kernel's decision rule (photo.hip issue_gathers) in fp64: clamp, cell
    corner min(floor, W-2), border state 0 interior / 1 clamped to 0 / 2 clamped to W-1."""
    ix = (grid[..., 0] + 1) * 0.5 * (W - 1)
    iy = (grid[..., 1] + 1) * 0.5 * (H - 1)
    xc, yc = ix.clamp(0, W - 1), iy.clamp(0, H - 1)
    xi = torch.clamp(xc.floor().long(), max=W - 2)
    yi = torch.clamp(yc.floor().long(), max=H - 2)
    sx = torch.where(ix <= 0, 1, torch.where(ix >= W - 1, 2, 0))
    sy = torch.where(iy <= 0, 1, torch.where(iy >= H - 1, 2, 0))
    return (xi | (yi << 11) | (sx << 22) | (sy << 24)).int()


def test_forced_sampler_matches_grid_sample():
    g = torch.Generator().manual_seed(3)
    N, C, H, W = 2, 3, 9, 13
    img = torch.rand(N, C, H, W, generator=g, dtype=torch.float64)
    grid = 2.6 * torch.rand(N, 7, 11, 2, generator=g, dtype=torch.float64) - 1.3   # ~30 % clamped
    grid[0, 0, 0] = torch.tensor([-1.0, 1.0])                                    # exact corners
    grid[0, 0, 1] = torch.tensor([1.0, -1.0])
    cells = cells_of(grid, W, H)
    a_img, a_grid = img.clone().requires_grad_(True), grid.clone().requires_grad_(True)
    b_img, b_grid = img.clone().requires_grad_(True), grid.clone().requires_grad_(True)
    ya = O.grid_sample_border(a_img, a_grid)
    yb = O.grid_sample_border_forced(b_img, b_grid, cells)
    assert torch.allclose(ya, yb, rtol=0, atol=1e-14)
    w = torch.rand(ya.shape, generator=g, dtype=torch.float64)
    (ya * w).sum().backward()
    (yb * w).sum().backward()
    assert torch.allclose(a_grid.grad, b_grid.grad, rtol=0, atol=1e-12)
    assert torch.allclose(a_img.grad, b_img.grad, rtol=0, atol=1e-12)


def test_forced_sampler_continues_the_imposed_cell():
    """A coordinate just below an integer, forced into the cell ABOVE it (what an fp32 GPU that
    rounded across the edge decided): the value is continuous and the gradient is that cell's."""
    img = torch.tensor([[[[0.0, 1.0, 5.0]]]], dtype=torch.float64).expand(1, 1, 2, 3).contiguous()
    x = 1.0 - 1e-9                                     # pixel coordinate (0-based), cell 0 by floor
    grid = torch.tensor([[[[2 * x / 2 - 1, 0.0]]]], dtype=torch.float64).requires_grad_(True)
    forced = torch.tensor([[[1]]], dtype=torch.int32)  # cell 1, interior
    y = O.grid_sample_border_forced(img, grid, forced)
    assert abs(y.item() - 1.0) < 1e-8
    y.sum().backward()
    # d value / d pixel-x in cell [1, 2] is 5 - 1 = 4; d pixel-x / d grid-x = (W - 1) / 2 = 1
    assert abs(grid.grad[0, 0, 0, 0].item() - 4.0) < 1e-12


def test_forced_l1_sign_decoding_and_branch():
    """vis_cell's L1 branch codes (bits 26 + 2c: 1 warped below target, 2 above, 3 equal, 0 not
    recorded) decode to (recorded, sign); a recorded branch opposite to the fp64 difference flips
    abs' at that pixel only, a recorded tie gives abs'(0) = 0, with the value unchanged up to the
    rounding-sized difference itself."""
    code = (2 << 26) | (1 << 28) | (2 << 30)                     # channels: above, below, above
    cell = torch.tensor([[[0, code - 2**32, (1 << 26) | (3 << 28) | (1 << 30)]]], dtype=torch.int32).expand(1, 2, 3)
    rec, s = O.forced_l1_sign(cell, 3)
    assert rec.shape == s.shape == (1, 3, 2, 3)
    assert rec[0, :, 0, 0].tolist() == [False] * 3
    assert rec[0, :, 0, 1].tolist() == [True] * 3 and s[0, :, 0, 1].tolist() == [1, -1, 1]
    assert rec[0, :, 0, 2].tolist() == [True] * 3 and s[0, :, 0, 2].tolist() == [-1, 0, -1]
    tgt = torch.zeros(1, 3, 2, 3, dtype=torch.float64)
    pred = torch.full((1, 3, 2, 3), -1e-9, dtype=torch.float64).requires_grad_(True)
    l = O.photometric_loss(pred, tgt, alpha=0.0, l1_sign=(rec, s))
    l.sum().backward()
    assert abs(l[0, 0, 0, 1].item()) < 1e-8
    # pixel 0 unforced: abs' = sign(pred - tgt) = -1; pixel 1 forced [+, -, +]; pixel 2 [-, 0, -]
    assert torch.allclose(pred.grad[0, :, 0, 0], torch.full((3,), -1 / 3, dtype=torch.float64))
    assert torch.allclose(pred.grad[0, :, 0, 1], torch.tensor([1 / 3, -1 / 3, 1 / 3], dtype=torch.float64))
    assert torch.allclose(pred.grad[0, :, 0, 2], torch.tensor([-1 / 3, 0.0, -1 / 3], dtype=torch.float64))
