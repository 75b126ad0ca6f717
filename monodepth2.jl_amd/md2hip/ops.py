"""Op-level host mirror: Flux ``Conv`` forward and its NNlib pullbacks (∇conv_data,
∇conv_filter) over the C-ABI.  Weights are cross-correlation [Cout, Cin, KH, KW]."""
from __future__ import annotations

import ctypes as C

from . import _lib
from ._lib import ConvDesc, check, lib, ptr, stream_of

ACT = {None: 0, "identity": 0, "relu": 1, "elu": 2, "sigmoid": 3}


def conv_desc(x_shape, w_shape, stride=1, pad=0, reflect=False, act=None) -> ConvDesc:
    n, cin, h, w = x_shape
    cout, cin2, kh, kw = w_shape
    if cin != cin2:
        raise ValueError(f"channel mismatch {cin} vs {cin2}")
    d = ConvDesc()
    d.n, d.cin, d.h, d.w, d.cout, d.kh, d.kw = n, cin, h, w, cout, kh, kw
    d.stride, d.pad, d.reflect, d.act = stride, pad, int(reflect), ACT[act]
    return d


def _ws(d, dev):
    import torch
    nbytes = lib().md2_conv2d_workspace_size(C.byref(d))
    return torch.empty(max(nbytes // 4, 1) + 64, dtype=torch.float32, device=dev)


def out_hw(h, w, k, stride, pad):
    return (h + 2 * pad - k) // stride + 1, (w + 2 * pad - k) // stride + 1


def conv2d(x, weight, bias=None, stride=1, pad=0, reflect=False, act=None):
    """y = act(conv(x, w) + b) -- Flux ``Conv((k,k), cin=>cout, act; stride, pad)`` (cross-corr.)
    with ``reflect`` = ``DecoderBlock`` semantics (pad_reflect then valid conv)."""
    import torch
    d = conv_desc(tuple(x.shape), tuple(weight.shape), stride, pad, reflect, act)
    ho, wo = out_hw(d.h, d.w, d.kh, stride, pad)
    y = torch.empty(d.n, d.cout, ho, wo, dtype=torch.float32, device=x.device)
    check(lib().md2_conv2d_fwd(C.byref(d), ptr(x), ptr(weight), ptr(bias), ptr(y),
                               ptr(_ws(d, x.device)), stream_of(x.device)), "md2_conv2d_fwd")
    return y


def conv2d_dgrad(dy, weight, x_shape, stride=1, pad=0, reflect=False):
    """NNlib ``∇conv_data``: dx from the pre-activation output gradient."""
    import torch
    d = conv_desc(tuple(x_shape), tuple(weight.shape), stride, pad, reflect)
    dx = torch.empty(*x_shape, dtype=torch.float32, device=dy.device)
    check(lib().md2_conv2d_dgrad(C.byref(d), ptr(dy), ptr(weight), ptr(dx), ptr(_ws(d, dy.device)),
                                 stream_of(dy.device)), "md2_conv2d_dgrad")
    return dx


def conv2d_wgrad(x, dy, w_shape, stride=1, pad=0, reflect=False, bias=True):
    """NNlib ``∇conv_filter`` (+ the bias gradient)."""
    import torch
    d = conv_desc(tuple(x.shape), tuple(w_shape), stride, pad, reflect)
    dw = torch.empty(*w_shape, dtype=torch.float32, device=x.device)
    db = torch.empty(w_shape[0], dtype=torch.float32, device=x.device) if bias else None
    check(lib().md2_conv2d_wgrad(C.byref(d), ptr(x), ptr(dy), ptr(dw), ptr(db), ptr(_ws(d, x.device)),
                                 stream_of(x.device)), "md2_conv2d_wgrad")
    return dw, db


def act_backward(out, dout, act):
    import torch
    dpre = torch.empty_like(dout)
    check(lib().md2_act_backward(ptr(out), ptr(dout), ptr(dpre), dout.numel(), ACT[act],
                                 stream_of(out.device)), "md2_act_backward")
    return dpre


def maxpool3s2(x):
    """ResNet stem ``MaxPool((3,3), pad=1, stride=2)``: (y, arg) with arg the uint8 window index
    of the first maximum, kept for :func:`maxpool3s2_backward`."""
    import torch
    n, c, h, w = x.shape
    y = torch.empty(n, c, (h + 1) // 2, (w + 1) // 2, dtype=torch.float32, device=x.device)
    arg = torch.empty(y.shape, dtype=torch.uint8, device=x.device)
    check(lib().md2_maxpool3s2_fwd(ptr(x), n, c, h, w, ptr(y), ptr(arg), stream_of(x.device)),
          "md2_maxpool3s2_fwd")
    return y, arg


def maxpool3s2_backward(dy, arg, x_shape):
    import torch
    n, c, h, w = x_shape
    dx = torch.empty(n, c, h, w, dtype=torch.float32, device=dy.device)
    check(lib().md2_maxpool3s2_bwd(ptr(dy), ptr(arg), n, c, h, w, ptr(dx), stream_of(dy.device)),
          "md2_maxpool3s2_bwd")
    return dx


def upsample2(x):
    """``upsample_bilinear(x, (2,2))`` with align_corners (src/depth_decoder.jl:18-19)."""
    import torch
    n, c, h, w = x.shape
    y = torch.empty(n, c, 2 * h, 2 * w, dtype=torch.float32, device=x.device)
    check(lib().md2_upsample2_fwd(ptr(x), n, c, h, w, ptr(y), stream_of(x.device)),
          "md2_upsample2_fwd")
    return y


def upsample2_backward(dy):
    import torch
    n, c, h2, w2 = dy.shape
    dx = torch.empty(n, c, h2 // 2, w2 // 2, dtype=torch.float32, device=dy.device)
    check(lib().md2_upsample2_bwd(ptr(dy), n, c, h2 // 2, w2 // 2, ptr(dx), stream_of(dy.device)),
          "md2_upsample2_bwd")
    return dx
