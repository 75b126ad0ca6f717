"""Seeded synthetic inputs shared by the parity tests (KITTI-shape triplets).

Every input is rounded to the fp32 grid (kept in the requested dtype): the GPU receives fp32
copies, so the fp64 oracle must be handed exactly those values -- otherwise the input rounding
(in K and invK a COHERENT perturbation of every pixel's warp) shows up as a GPU error.
``grid32=False``: the unrounded values the committed golden fixtures were generated from."""
import math

import torch
import torch.nn.functional as F


def fp32_grid(t):
    """t rounded to the nearest fp32 value, in t's dtype."""
    return t.float().to(t.dtype)


def smooth_field(g, n, c, h, w, base=8, dtype=torch.float64):
    """Low-frequency random texture in [0,1] with a little high-frequency detail."""
    lo = torch.rand(n, c, max(2, h // base), max(2, w // base), generator=g, dtype=dtype)
    up = F.interpolate(lo, size=(h, w), mode="bicubic", align_corners=True)
    hi = torch.rand(n, c, h, w, generator=g, dtype=dtype)
    return (0.85 * up + 0.15 * hi).clamp(0, 1)


def ramp(g, n, c, h, w, dtype=torch.float64):
    """Affine image a*u + b*v + c0 per channel: bilinear sampling of it has no kinks."""
    u = torch.linspace(0, 1, w, dtype=dtype).view(1, 1, 1, w)
    v = torch.linspace(0, 1, h, dtype=dtype).view(1, 1, h, 1)
    a = 0.4 * torch.rand(n, c, 1, 1, generator=g, dtype=dtype) + 0.1
    b = 0.4 * torch.rand(n, c, 1, 1, generator=g, dtype=dtype) - 0.2
    c0 = 0.2 + 0.2 * torch.rand(n, c, 1, 1, generator=g, dtype=dtype)
    return a * u + b * v + c0


def triplets(n, c, h, w, seed=7, dtype=torch.float64, ramp_sources=False, grid32=True):
    """[n, 3, c, h, w] frames; frame 1 (the target) is textured; with ``ramp_sources`` the two
    source frames are affine ramps (kink-free bilinear gradients)."""
    g = torch.Generator().manual_seed(seed)
    frames = [smooth_field(g, n, c, h, w, dtype=dtype) for _ in range(3)]
    if ramp_sources:
        frames[0] = ramp(g, n, c, h, w, dtype)
        frames[2] = ramp(g, n, c, h, w, dtype)
    x = torch.stack(frames, 1).contiguous()
    return fp32_grid(x) if grid32 else x


def intrinsics(w, h, grid32=True):
    f = (2648.0 / 4.63461538462) * (w / 416.0)
    K = torch.tensor([[f, 0, w / 2.0], [0, f, h / 2.0], [0, 0, 1.0]], dtype=torch.float64)
    invK = torch.linalg.inv(K)
    return (fp32_grid(K), fp32_grid(invK)) if grid32 else (K, invK)


def disparities(n, h, w, nscales=4, seed=11, dtype=torch.float64, lo=0.01, hi=0.1, grid32=True):
    """Per-scale disparity maps in [lo, hi] (depth = 1/(d*9.99+0.01): [0.01,0.1] -> 1-9 m)."""
    g = torch.Generator().manual_seed(seed)
    out = []
    for s in range(nscales):
        f = 2 ** (nscales - 1 - s)
        hh, ww = h // f, w // f
        z = smooth_field(g, n, 1, hh, ww, base=4, dtype=dtype)
        d = (lo + (hi - lo) * torch.sigmoid(4.0 * (z - 0.5))).contiguous()
        out.append(fp32_grid(d) if grid32 else d)
    return out


def poses(n, seed=13, dtype=torch.float64, forward=0.3, jitter=0.05, grid32=True):
    """rvec ~ N(0, 0.01^2), tvec = (0, 0, -+forward) + N(0, jitter^2)  (SURVEY.md 8d)."""
    g = torch.Generator().manual_seed(seed)
    res = []
    for sign in (-1.0, 1.0):
        r = 0.01 * torch.randn(n, 3, generator=g, dtype=dtype)
        t = jitter * torch.randn(n, 3, generator=g, dtype=dtype)
        t[:, 2] += forward * sign
        res.append((fp32_grid(r), fp32_grid(t)) if grid32 else (r, t))
    return res


def rel_err(a, b):
    a = a.double().cpu()
    b = b.double().cpu()
    return ((a - b).norm() / max(b.norm().item(), 1e-30)).item()
