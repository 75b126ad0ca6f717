"""GPU parity of the implicit-GEMM conv kernels (fwd / ∇conv_data / ∇conv_filter) against
fp64 torch-CPU convolutions (the oracle's F.conv2d, cross-correlation semantics).

Tolerance: relative Frobenius error 1e-5 (exact-fp32 MFMA accumulation over K <= 8k terms)."""
import os

import pytest
import torch
import torch.nn.functional as F

from oracle import md2_oracle as O
from tests import _data as D

pytestmark = pytest.mark.gpu

# (x_shape, cout, k, stride, pad, reflect, act, bias)   -- shapes of the ResNet-18 / decoders
CASES = [
    ((2, 3, 64, 208), 64, 7, 2, 3, False, None, False),          # stem 7x7/2 (Wo = 104: conv_px)
    # the stem on the space-to-depth kernel (conv_stem.inc, Wo % 16 == 0): two subtiles per row,
    # a 2-row map (every s2d row window crosses a border) with an odd subtile count, 640 wide
    # (8 staged records per thread, one block per CU)
    ((3, 3, 32, 64), 64, 7, 2, 3, False, None, False),
    ((2, 3, 4, 96), 64, 7, 2, 3, False, None, False),
    ((1, 3, 10, 640), 64, 7, 2, 3, False, None, False),
    ((2, 64, 32, 104), 64, 3, 1, 1, False, None, False),         # layer1
    ((2, 64, 32, 104), 128, 3, 2, 1, False, None, False),        # layer2.0.conv1 (stride 2)
    ((2, 64, 32, 104), 128, 1, 2, 0, False, None, False),        # downsample 1x1/2
    ((2, 256, 8, 26), 512, 3, 2, 1, False, None, False),         # layer4.0.conv1 (split-K)
    ((3, 512, 4, 13), 512, 3, 1, 1, False, None, False),         # layer4 3x3 (split-K)
    ((2, 96, 16, 52), 32, 3, 1, 1, True, "elu", True),           # decoder c2 (reflect, ELU)
    ((2, 16, 32, 64), 16, 3, 1, 1, True, "elu", True),           # decoder branch5
    ((2, 16, 32, 64), 1, 3, 1, 1, True, "sigmoid", True),        # disparity head
    ((4, 512, 4, 13), 256, 3, 1, 1, False, "relu", True),        # pose conv1
    ((4, 256, 4, 13), 6, 1, 1, 0, False, None, True),            # pose conv3
    ((6, 512, 4, 13), 256, 1, 1, 0, False, "relu", True),        # pose squeezer
    ((2, 8, 2, 3), 4, 3, 1, 1, True, "elu", True),               # reflect on a 2x3 map
    ((3, 5, 9, 11), 7, 3, 2, 1, False, "relu", True),            # ragged everything
    # tap-major K order (channels % 16 == 0): reflect borders, CW = 16/32/64 wgrad tap blocks,
    # stride-2 dgrad phases, 1x1/2 with few channels
    ((2, 16, 2, 4), 16, 3, 1, 1, True, "elu", True),             # reflect, every pixel a border
    ((2, 32, 4, 5), 32, 3, 1, 1, True, "elu", True),             # reflect, mixed border waves
    ((2, 48, 8, 12), 64, 3, 1, 1, False, "relu", True),          # Cin 48 -> CW 16
    ((2, 32, 9, 13), 16, 3, 2, 1, False, None, False),           # stride-2 dgrad, Cout 16
    ((2, 16, 7, 9), 32, 1, 2, 0, False, None, False),            # 1x1/2, 16 channels
    ((2, 64, 6, 10), 48, 3, 1, 1, True, "elu", True),            # reflect, CW 64, Cout 48
    # bf16 split-product wgrad (conv_wgrad_px3: pixel pairs): a pair wrapping to the next row (odd
    # Wo), an odd pixel count per image (fp32 tap kernel fallback), Cout 96 (ragged row tile)
    ((2, 64, 6, 7), 96, 3, 1, 1, True, "elu", True),
    ((3, 64, 5, 7), 64, 3, 1, 1, False, None, False),
    ((2, 128, 9, 14), 64, 3, 2, 1, False, "relu", True),
    # 4 pixels per lane (64-row tiles, 64 / 128-channel tap blocks): groups wrapping a row (odd Wo),
    # reflect borders inside a group
    ((2, 64, 4, 13), 64, 3, 1, 1, False, None, False),
    ((2, 128, 4, 7), 64, 3, 1, 1, True, "elu", True),
    # the model-parity configuration (6 frames of 64x128): tiny deep maps
    ((6, 64, 16, 32), 64, 3, 1, 1, False, None, False),          # layer1
    ((6, 64, 16, 32), 128, 3, 2, 1, False, None, False),         # layer2.0.conv1
    ((6, 128, 8, 16), 256, 3, 2, 1, False, None, False),         # layer3.0.conv1
    ((6, 256, 4, 8), 512, 3, 2, 1, False, None, False),          # layer4.0.conv1
    ((6, 512, 2, 4), 512, 3, 1, 1, False, None, False),          # layer4 3x3 on 2x4
    ((6, 256, 4, 8), 512, 1, 2, 0, False, None, False),          # layer4 downsample
    ((2, 512, 2, 4), 256, 3, 1, 1, True, "elu", True),           # branch1.c1 reflect 2x4
    ((4, 512, 2, 4), 256, 3, 1, 1, False, "relu", True),         # pose conv1 on 2x4
    # M <= 16 (16x16x4 MFMA kernel): Cout = 16 forward / Cin = 16 dgrad, reflect and zero padding,
    # ragged pixel tiles, both block widths (BN 128 / 256), the bench-size branch-5 convs
    ((2, 16, 24, 70), 16, 3, 1, 1, True, "elu", True),
    ((2, 32, 12, 40), 16, 3, 1, 1, True, "elu", True),
    ((3, 16, 9, 17), 16, 3, 1, 1, False, "relu", False),
    ((2, 48, 5, 7), 8, 3, 1, 1, True, None, True),
    ((12, 16, 128, 416), 16, 3, 1, 1, True, "elu", True),
    ((12, 32, 64, 208), 16, 3, 1, 1, True, "elu", True),
    # Cout <= 16 wgrad (conv_wgrad16_kernel: 16-channel groups, K split over waves and slabs)
    ((5, 64, 33, 47), 16, 3, 1, 1, False, None, True),           # 4 channel groups, ragged K
    ((1, 16, 3, 5), 12, 3, 1, 1, True, "elu", True),             # K < one 64-pixel chunk
    ((3, 32, 10, 30), 20, 3, 1, 1, False, "relu", True),         # Cout 20: ragged second row tile
    ((12, 96, 64, 208), 32, 3, 1, 1, True, "elu", True),         # decoder level-4 conv2 at bench size
    # Cout = 1 heads (VALU kernels of head.hip): reflect folds on 2/3-wide maps, zero padding,
    # ragged and > 8-channel groups, the bench-size full-resolution head
    ((2, 16, 2, 2), 1, 3, 1, 1, True, "sigmoid", True),          # every pixel folds twice
    ((2, 8, 3, 3), 1, 3, 1, 1, True, "sigmoid", True),           # q = 1 = n-2 folds both ways
    ((3, 5, 7, 11), 1, 3, 1, 1, True, "sigmoid", True),          # ragged channel group
    ((2, 13, 6, 9), 1, 3, 1, 1, False, None, True),              # zero padding, no act
    ((2, 32, 16, 52), 1, 3, 1, 1, True, "sigmoid", True),        # head4 geometry
    ((2, 128, 4, 13), 1, 3, 1, 1, True, "sigmoid", True),        # head2 (16 channel groups)
    ((12, 16, 128, 416), 1, 3, 1, 1, True, "sigmoid", True),     # head5 at bench size
    # column-strip head kernels (W >= 64): ragged segments / bands / channel blocks, zero padding,
    # both row folds inside one strip, the head3 geometry
    ((2, 37, 13, 70), 1, 3, 1, 1, True, "sigmoid", True),
    ((2, 7, 9, 66), 1, 3, 1, 1, False, None, True),
    ((4, 8, 130, 256), 1, 3, 1, 1, False, None, True),           # zero padding, strip fwd/wgrad
    ((1, 16, 4, 64), 1, 3, 1, 1, True, "sigmoid", True),
    ((2, 64, 32, 104), 1, 3, 1, 1, True, "sigmoid", True),
    # LDS-halo kernel (conv_halo.inc) edges: a 256-pixel tile spanning many small images (W = 7:
    # 40 halo rows), ragged N, C = 32 (two channel chunks, split-K of one), M = 128 (two row
    # tiles), a map too wide for the halo image (W = 200: conv_px3 instead)
    ((5, 64, 5, 7), 64, 3, 1, 1, False, None, False),
    ((3, 32, 13, 97), 128, 3, 1, 1, False, "relu", True),
    ((2, 128, 9, 29), 128, 3, 1, 1, False, None, False),
    ((2, 64, 6, 200), 64, 3, 1, 1, False, None, False),
    # LDS-halo filter gradient (conv_whalo): chunks of 4 rows (80 pixels, 5 k-steps), and of 3
    # rows (108 pixels + 4 zero pad) with one 32-channel tile and two 64-filter tiles
    ((3, 64, 12, 20), 64, 3, 1, 1, False, None, False),
    ((2, 32, 6, 36), 128, 3, 1, 1, False, "relu", True),
    # reflect-padded dgrad on the halo kernel (the zero-padded adjoint of the (H+2) x (W+2) grid,
    # then the fold): many small padded images per tile, a 2-row map (every row folds)
    ((3, 64, 7, 5), 64, 3, 1, 1, True, "elu", True),
    ((4, 128, 2, 9), 64, 3, 1, 1, True, None, False),
    # stride-2 data gradient on the LDS halo (conv_halo3s2: the four output-parity classes from
    # one staged dY image): 128-point tiles over many 3x7 images, a 1x1 dY map, 64- and 65-wide dY
    # rows (the widest its 416-pixel halo plane takes), a 100-wide one (too wide: conv_px3's merged
    # classes), Cout 64 (4 chunks, split-K of 2)
    ((5, 64, 6, 14), 64, 3, 2, 1, False, None, False),
    ((2, 64, 2, 2), 64, 3, 2, 1, False, None, False),
    ((2, 64, 4, 128), 64, 3, 2, 1, False, None, False),
    ((1, 128, 6, 130), 64, 3, 2, 1, False, "relu", True),
    ((2, 64, 4, 200), 64, 3, 2, 1, False, None, False),
    ((3, 192, 10, 30), 64, 3, 2, 1, False, None, False),
    # every conv of the benchmarked step (BASELINE config 3: B=12 triplets, 416x128) at its bench
    # shape -- the encoder on 36 frames, the pose decoder on 24 pairs, the depth decoder on the 12
    # targets -- so each planner choice the bench runs (tile, split-K count, stride-2 phase launch,
    # wgrad kernel) is pinned against fp64
    ((36, 3, 128, 416), 64, 7, 2, 3, False, None, False),        # stem 7x7/2
    ((36, 64, 32, 104), 64, 3, 1, 1, False, None, False),        # layer1 3x3
    ((36, 64, 32, 104), 128, 3, 2, 1, False, None, False),       # layer2.0.conv1 (stride 2)
    ((36, 64, 32, 104), 128, 1, 2, 0, False, None, False),       # layer2.0 downsample
    ((36, 128, 16, 52), 128, 3, 1, 1, False, None, False),       # layer2 3x3
    ((36, 128, 16, 52), 256, 3, 2, 1, False, None, False),       # layer3.0.conv1
    ((36, 128, 16, 52), 256, 1, 2, 0, False, None, False),       # layer3.0 downsample
    ((36, 256, 8, 26), 256, 3, 1, 1, False, None, False),        # layer3 3x3
    ((36, 256, 8, 26), 512, 3, 2, 1, False, None, False),        # layer4.0.conv1 (split-K)
    ((36, 256, 8, 26), 512, 1, 2, 0, False, None, False),        # layer4.0 downsample
    ((36, 512, 4, 13), 512, 3, 1, 1, False, None, False),        # layer4 3x3 (split-K)
    ((36, 512, 4, 13), 256, 1, 1, 0, False, "relu", True),       # pose squeezer
    ((24, 512, 4, 13), 256, 3, 1, 1, False, "relu", True),       # pose conv1
    ((24, 256, 4, 13), 256, 3, 1, 1, False, "relu", True),       # pose conv2
    ((24, 256, 4, 13), 6, 1, 1, 0, False, None, True),           # pose conv3
    ((12, 512, 4, 13), 256, 3, 1, 1, True, "elu", True),         # branch1.c1
    ((12, 512, 8, 26), 256, 3, 1, 1, True, "elu", True),         # branch1.c2 (256 up + 256 skip)
    ((12, 256, 8, 26), 128, 3, 1, 1, True, "elu", True),         # branch2.c1
    ((12, 256, 16, 52), 128, 3, 1, 1, True, "elu", True),        # branch2.c2
    ((12, 128, 16, 52), 1, 3, 1, 1, True, "sigmoid", True),      # head2
    ((12, 128, 16, 52), 64, 3, 1, 1, True, "elu", True),         # branch3.c1
    ((12, 128, 32, 104), 64, 3, 1, 1, True, "elu", True),        # branch3.c2
    ((12, 64, 32, 104), 1, 3, 1, 1, True, "sigmoid", True),      # head3
    ((12, 64, 32, 104), 32, 3, 1, 1, True, "elu", True),         # branch4.c1
    ((12, 32, 64, 208), 1, 3, 1, 1, True, "sigmoid", True),      # head4
]


def _ref_act(y, act):
    return {None: y, "relu": F.relu(y), "elu": F.elu(y), "sigmoid": torch.sigmoid(y)}[act]


def _ref_conv(x, w, b, stride, pad, reflect):
    if reflect:
        return F.conv2d(O.pad_reflect(x, pad), w, b, stride=stride)
    return F.conv2d(x, w, b, stride=stride, padding=pad)


@pytest.mark.parametrize("case", CASES, ids=[f"{c[0]}-{c[1]}-k{c[2]}s{c[3]}{'r' if c[5] else ''}" for c in CASES])
def test_conv_fwd_bwd(case):
    from md2hip import ops
    xs, cout, k, stride, pad, reflect, act, has_bias = case
    g = torch.Generator().manual_seed(5)
    # fp32-representable inputs: the fp64 reference sees exactly what the kernels see, so the
    # tolerance measures the kernels' accumulation error alone (a cancelling bias-gradient sum
    # would otherwise inherit the fp32 rounding of dy)
    x = torch.randn(*xs, generator=g, dtype=torch.float64).float().double()
    w = (torch.randn(cout, xs[1], k, k, generator=g, dtype=torch.float64) / (xs[1] * k * k) ** 0.5).float().double()
    b = torch.randn(cout, generator=g, dtype=torch.float64).float().double() if has_bias else None
    xr = x.clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    br = b.clone().requires_grad_(True) if has_bias else None
    pre = _ref_conv(xr, wr, br, stride, pad, reflect)
    y_ref = _ref_act(pre, act)
    dy = torch.randn(pre.shape, generator=g, dtype=torch.float64).float().double()
    pre.backward(dy)

    dev = torch.device("cuda")
    xg, wg = x.float().to(dev), w.float().to(dev)
    bg = b.float().to(dev) if has_bias else None
    y = ops.conv2d(xg, wg, bg, stride=stride, pad=pad, reflect=reflect, act=act)
    dx = ops.conv2d_dgrad(dy.float().to(dev), wg, xs, stride=stride, pad=pad, reflect=reflect)
    dw, db = ops.conv2d_wgrad(xg, dy.float().to(dev), tuple(w.shape), stride=stride, pad=pad,
                              reflect=reflect, bias=has_bias)
    torch.cuda.synchronize()
    assert D.rel_err(y, y_ref.detach()) < 1e-5
    assert D.rel_err(dx, xr.grad) < 1e-5
    assert D.rel_err(dw, wr.grad) < 1e-5
    if has_bias:
        assert D.rel_err(db, br.grad) < 1e-5


@pytest.mark.parametrize("act", ["relu", "elu", "sigmoid"])
def test_act_backward(act):
    from md2hip import ops
    g = torch.Generator().manual_seed(9)
    pre = torch.randn(1000, generator=g, dtype=torch.float64).requires_grad_(True)
    out = _ref_act(pre, act)
    dout = torch.randn(1000, generator=g, dtype=torch.float64)
    out.backward(dout)
    got = ops.act_backward(out.detach().float().cuda(), dout.float().cuda(), act)
    torch.cuda.synchronize()
    assert D.rel_err(got, pre.grad) < 1e-5


_VARIANT_CHILD = r"""
import sys, json
root = sys.argv[1]
sys.path[:0] = [root, root + "/monodepth2.jl_amd"]
import torch, torch.nn.functional as F
from md2hip import ops
from oracle import md2_oracle as O
from tests import _data as D
out = {}
shapes = [((36, 64, 32, 104), 64, 3, 1, 1, False), ((36, 128, 16, 52), 256, 3, 2, 1, False),
          ((36, 512, 4, 13), 512, 3, 1, 1, False), ((12, 128, 32, 104), 64, 3, 1, 1, True),
          ((36, 128, 16, 52), 256, 1, 2, 0, False)]
if len(sys.argv) > 2:
    shapes = [(tuple(a), b, c, d, e, f) for a, b, c, d, e, f in json.loads(sys.argv[2])]
for xs, cout, k, st, pd, rf in shapes:
    g = torch.Generator().manual_seed(5)
    x = torch.randn(*xs, generator=g, dtype=torch.float64).float().double()
    w = (torch.randn(cout, xs[1], k, k, generator=g, dtype=torch.float64) / (xs[1] * k * k) ** 0.5).float().double()
    xr, wr = x.clone().requires_grad_(True), w.clone().requires_grad_(True)
    pre = F.conv2d(O.pad_reflect(xr, pd), wr, stride=st) if rf else F.conv2d(xr, wr, stride=st, padding=pd)
    dy = torch.randn(pre.shape, generator=g, dtype=torch.float64).float().double()
    pre.backward(dy)
    xg, wg = x.float().cuda(), w.float().cuda()
    y = ops.conv2d(xg, wg, None, stride=st, pad=pd, reflect=rf)
    dx = ops.conv2d_dgrad(dy.float().cuda(), wg, xs, stride=st, pad=pd, reflect=rf)
    dw, _ = ops.conv2d_wgrad(xg, dy.float().cuda(), tuple(w.shape), stride=st, pad=pd, reflect=rf, bias=False)
    torch.cuda.synchronize()
    out[str((xs, cout, k, st, rf))] = [D.rel_err(y, pre.detach()), D.rel_err(dx, xr.grad), D.rel_err(dw, wr.grad)]
print(json.dumps(out))
"""


@pytest.mark.parametrize("env", [{"MD2_PX3": "0", "MD2_WPX3": "0"}, {"MD2_PX3_TERMS": "9"}],
                         ids=["fp32-mfma", "bf16x9"])
def test_conv_kernel_variants(env):
    _variant(env)


def test_halo2d_dgrad_variant():
    """The 2D-tile halo kernel's data-gradient forms (MD2_HALO2D=3: off by default, measured
    slower in the step): the reflect dgrad on the padded grid + fold at the decoder's 96->32
    64x208 shape and a ragged one, the zero-padded dgrad with 32-row M tiles; within 1e-5 of fp64."""
    _variant({"MD2_HALO2D": "3"}, [[[12, 96, 64, 208], 32, 3, 1, 1, True], [[3, 96, 20, 70], 32, 3, 1, 1, True],
                                   [[2, 32, 24, 200], 64, 3, 1, 1, False], [[2, 96, 16, 60], 48, 3, 1, 1, False]])


def test_halo_s2_off_variant():
    """MD2_HALO_S2=0: the stride-2 data gradients back on conv_px3's merged parity classes (the
    path the halo kernel replaced), at the encoder's three bench shapes; within 1e-5 of fp64."""
    _variant({"MD2_HALO_S2": "0"}, [[[36, 64, 32, 104], 128, 3, 2, 1, False], [[36, 128, 16, 52], 256, 3, 2, 1, False],
                                    [[36, 256, 8, 26], 512, 3, 2, 1, False]])


def _variant(env, shapes=None):
    """The selectable conv kernels (MD2_TUNING=1): the exact-fp32 MFMA kernels (conv_px2 for
    fwd / dgrad, conv_wgrad_tap for wgrad) and the nine-product bf16x9 form of conv_px3 /
    conv_wgrad_px3, on encoder / decoder shapes, within
    1e-5 of fp64 like the default bf16x6 (test_conv_fwd_bwd)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    e = {k: v for k, v in os.environ.items() if not k.startswith("MD2_")}
    e.update(MD2_TUNING="1", **env)
    argv = [sys.executable, "-c", _VARIANT_CHILD, root] + ([json.dumps(shapes)] if shapes else [])
    r = subprocess.run(argv, env=e, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    errs = json.loads(r.stdout.strip().splitlines()[-1])
    bad = {k: v for k, v in errs.items() if max(v) >= 1e-5}
    assert not bad, bad
