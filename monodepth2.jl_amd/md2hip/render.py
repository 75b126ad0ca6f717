"""MINE plane rendering of the MPI mode (src/render.jl:21-114) over the C-ABI -- the host mirror
of ``create_meshgrid``, ``get_src_xyz_from_plane_disparity``, ``plane_volume_rendering``,
``get_tgt_xyz_from_plane_disparity``, ``sample`` and ``render_tgt_rgb_depth``.  Forward only, as
upstream (no rrule).  No CPU fallback: every call runs a HIP kernel of libmd2hip.so.

Tensors are the Julia arrays' memory in C order (float32, contiguous, on the GPU):
  rgb (W,H,3,N,B) = [B,N,3,H,W]      sigma (W,H,1,N,B) = [B,N,1,H,W]
  xyz (3,W,H,N,B) = [B,N,H,W,3]      disparity / depth (N,B) = [B,N]
  sample's src (W,H,C,N*B) = [B*N,C,H,W], valid (W*H, N*B) = [B*N, H*W]
  pose: ``Pose(rvec, tvec)`` with [B,3] tensors, or a [B,6] (rvec, tvec) tensor
  K, invK: 3x3 (numpy / tensor / nested lists), host side.
The reference's semantics are kept as written (DESIGN.md "MINE rendering"): the valid mask is
the chained comparison ``u .< W .* u .>= 0`` (u > 0), the sample grid is (u + 0.5)/(W/2) without
the -1, and render_tgt_rgb_depth's ``depth`` is the transparency_acc volume."""
from __future__ import annotations

import numpy as np

from ._lib import check, lib, ptr, stream_of


def _f32(t, shape=None, name="tensor"):
    import torch
    if t.dtype != torch.float32 or not t.is_contiguous() or t.device.type != "cuda":
        raise ValueError(f"{name}: expected a contiguous float32 CUDA tensor")
    if shape is not None and tuple(t.shape) != tuple(shape):
        raise ValueError(f"{name}: shape {tuple(t.shape)} != {tuple(shape)}")
    return t


def _host3(m):
    a = np.ascontiguousarray(np.asarray(m.cpu() if hasattr(m, "cpu") else m, dtype=np.float32).reshape(3, 3))
    return a, a.ctypes.data


def _pose6(pose, B, dev):
    import torch
    if hasattr(pose, "rvec"):
        p = torch.cat([pose.rvec.reshape(B, 3), pose.tvec.reshape(B, 3)], 1)
    else:
        p = pose.reshape(B, 6)
    return p.to(device=dev, dtype=torch.float32).contiguous()


def create_meshgrid(H: int, W: int, device=None):
    """``create_meshgrid(H, W)`` (src/render.jl:21-23): Julia (3,W,H) of 1-based (w, h, 1) as
    [H,W,3] float32."""
    import torch
    w = torch.arange(1, W + 1, dtype=torch.float32, device=device).view(1, W).expand(H, W)
    h = torch.arange(1, H + 1, dtype=torch.float32, device=device).view(H, 1).expand(H, W)
    return torch.stack([w, h, torch.ones(H, W, dtype=torch.float32, device=device)], -1).contiguous()


def get_src_xyz_from_plane_disparity(meshgrid_src_homo, mpi_disparity_src, K_src_inv):
    """src/render.jl:25-30: xyz [B,N,H,W,3] = K^-1 [w, h, 1] / disparity.  The kernel generates
    the pixel grid itself; ``meshgrid_src_homo`` must be ``create_meshgrid(H, W)`` (the only grid
    the reference passes) and fixes H, W."""
    import torch
    H, W, _ = meshgrid_src_homo.shape
    d = _f32(mpi_disparity_src, name="mpi_disparity_src")
    B, N = d.shape
    if not torch.equal(meshgrid_src_homo.to(d.device, torch.float32), create_meshgrid(H, W, d.device)):
        raise ValueError("meshgrid_src_homo must be create_meshgrid(H, W)")
    iK, iKp = _host3(K_src_inv)
    out = torch.empty(B, N, H, W, 3, dtype=torch.float32, device=d.device)
    check(lib().md2_mine_src_xyz(ptr(d), N, B, H, W, iKp, ptr(out), stream_of(d.device)), "md2_mine_src_xyz")
    return out


def get_tgt_xyz_from_plane_disparity(xyz_src, pose):
    """src/render.jl:51-64: R(rvec_b) xyz + t_b, [B,N,H,W,3] -> [B,N,H,W,3]."""
    import torch
    x = _f32(xyz_src, name="xyz_src")
    B, N, H, W, _ = x.shape
    p = _pose6(pose, B, x.device)
    out = torch.empty_like(x)
    check(lib().md2_mine_tgt_xyz(ptr(x), ptr(p), N, B, H, W, ptr(out), stream_of(x.device)), "md2_mine_tgt_xyz")
    return out


def sample(src, depth_src, pose, K, K_inv):
    """``sample(src, depth_src, pose, K, K_inv)`` (src/render.jl:66-94): per-plane homography
    warp of src [B*N,C,H,W] with depth_src [B,N] -> (tgt [B*N,C,H,W], valid [B*N,H*W] as 0/1)."""
    import torch
    s = _f32(src, name="src")
    d = _f32(depth_src, name="depth_src")
    B, N = d.shape
    BN, Cc, H, W = s.shape
    if BN != B * N:
        raise ValueError(f"src holds {BN} planes, depth_src {B}x{N}")
    p = _pose6(pose, B, s.device)
    k, kp = _host3(K)
    ik, ikp = _host3(K_inv)
    out = torch.empty_like(s)
    valid = torch.empty(BN, H * W, dtype=torch.float32, device=s.device)
    check(lib().md2_mine_sample(ptr(s), Cc, ptr(d), ptr(p), N, B, H, W, kp, ikp, ptr(out), ptr(valid),
                                stream_of(s.device)), "md2_mine_sample")
    return out, valid


def plane_volume_rendering(rgb, sigma, xyz):
    """src/render.jl:32-49: rgb [B,N,3,H,W], sigma [B,N,1,H,W], xyz [B,N,H,W,3] ->
    (rgb_out [B,3,H,W], transparency_acc [B,N,1,H,W], weights [B,N,1,H,W])."""
    import torch
    r = _f32(rgb, name="rgb")
    B, N, _, H, W = r.shape
    s = _f32(sigma, (B, N, 1, H, W), "sigma")
    x = _f32(xyz, (B, N, H, W, 3), "xyz")
    out = torch.empty(B, 3, H, W, dtype=torch.float32, device=r.device)
    acc = torch.empty(B, N, 1, H, W, dtype=torch.float32, device=r.device)
    w = torch.empty_like(acc)
    check(lib().md2_plane_volume_rendering(ptr(r), ptr(s), ptr(x), N, B, H, W, ptr(out), ptr(acc), ptr(w),
                                           stream_of(r.device)), "md2_plane_volume_rendering")
    return out, acc, w


def render_tgt_rgb_depth(rgb, sigma, disparity_src, xyz_tgt, pose, K_inv, K):
    """src/render.jl:96-114, one fused HIP kernel: -> (rgb [B,3,H,W], depth [B,N,1,H,W] (the
    transparency_acc volume), mask [B,1,H,W] (per-pixel count of valid planes))."""
    import torch
    r = _f32(rgb, name="rgb")
    B, N, _, H, W = r.shape
    s = _f32(sigma, (B, N, 1, H, W), "sigma")
    d = _f32(disparity_src, (B, N), "disparity_src")
    x = _f32(xyz_tgt, (B, N, H, W, 3), "xyz_tgt")
    p = _pose6(pose, B, r.device)
    ik, ikp = _host3(K_inv)
    k, kp = _host3(K)
    out = torch.empty(B, 3, H, W, dtype=torch.float32, device=r.device)
    depth = torch.empty(B, N, 1, H, W, dtype=torch.float32, device=r.device)
    mask = torch.empty(B, 1, H, W, dtype=torch.float32, device=r.device)
    check(lib().md2_render_tgt_rgb_depth(ptr(r), ptr(s), ptr(d), ptr(x), ptr(p), ikp, kp, N, B, H, W, ptr(out),
                                         ptr(depth), ptr(mask), stream_of(r.device)), "md2_render_tgt_rgb_depth")
    return out, depth, mask
