"""CPU: the host data pipeline -- Depth10k triplet split (src/dtk.jl:29-46),
grayscale, KITTI calib/intrinsics and triplet indexing (src/kitty.jl:19-61), DChain bins
(src/dchain.jl), FlipX, and the DataLoader's rank sharding / collation.  Synthetic PNGs written
here (the reference ships no dataset; res/image.png is not read at test time)."""
import os

import numpy as np
import pytest
import torch

from PIL import Image


def _write_rgb(path, arr):
    Image.fromarray((arr * 255).round().astype(np.uint8), mode="RGB").save(path)


@pytest.fixture
def dtk(tmp_path):
    rng = np.random.default_rng(0)
    files = []
    for i in range(6):
        a = rng.random((128, 3 * 416, 3))
        name = f"s{i}.png"
        _write_rgb(str(tmp_path / name), a)
        files.append(name)
    return str(tmp_path), files


def _expect(path):
    a = np.asarray(Image.open(path), dtype=np.float32) / 255.0          # [H, 3W, 3]
    return np.stack([a[:, 416 * j:416 * (j + 1)].transpose(2, 0, 1) for j in range(3)], 0)


def test_depth10k_split_and_layout(dtk):
    import md2hip
    d, files = dtk
    ds = md2hip.Depth10k(d, files)
    assert len(ds) == 6 and ds.resolution == (416, 128)
    x = ds[2]
    assert x.shape == (3, 3, 128, 416) and x.dtype == np.float32
    np.testing.assert_array_equal(x, _expect(os.path.join(d, files[2])))
    f = 2648.0 / 4.63461538462
    np.testing.assert_allclose(ds.K, [[f, 0, 208], [0, f, 64], [0, 0, 1]])
    np.testing.assert_allclose(ds.K @ ds.invK, np.eye(3), atol=1e-12)


def test_depth10k_grayscale(dtk):
    import md2hip
    d, files = dtk
    g = md2hip.Depth10k(d, files, grayscale=True)[0]
    rgb = _expect(os.path.join(d, files[0]))
    assert g.shape == (3, 1, 128, 416)
    ref = 0.299 * rgb[:, 0] + 0.587 * rgb[:, 1] + 0.114 * rgb[:, 2]
    np.testing.assert_allclose(g[:, 0], ref, atol=1e-6)


def test_flipx_all_frames_together(dtk):
    import md2hip
    d, files = dtk
    plain = md2hip.Depth10k(d, files)
    always = md2hip.Depth10k(d, files, augmentations=md2hip.FlipX(1.0))
    never = md2hip.Depth10k(d, files, augmentations=md2hip.FlipX(0.0))
    np.testing.assert_array_equal(always[1], plain[1][..., ::-1])
    np.testing.assert_array_equal(never[1], plain[1])
    half = md2hip.Depth10k(d, files * 20, augmentations=md2hip.FlipX(0.5))
    flips = sum(bool(np.array_equal(half[i], plain[i % 6][..., ::-1])) for i in range(len(half)))
    assert 30 <= flips <= 90
    assert np.array_equal(half.getobs(4, seed=3), half.getobs(4, seed=3))     # deterministic


def test_kitti_calib_and_triplets(tmp_path):
    import md2hip
    seq = tmp_path / "sequences" / "03" / "image_0"
    seq.mkdir(parents=True)
    (tmp_path / "sequences" / "03" / "calib.txt").write_text(
        "P0: 7.215377e+02 0.000000e+00 6.095593e+02 0.000000e+00 0.000000e+00 7.215377e+02 "
        "1.728540e+02 0.000000e+00 0.000000e+00 0.000000e+00 1.000000e+00 0.000000e+00\n")
    rng = np.random.default_rng(1)
    frames = []
    for k in range(7):                        # 7 frames -> 2 triplets
        a = (rng.random((256, 832)) * 255).round().astype(np.uint8)
        Image.fromarray(a, mode="L").save(str(seq / ("%06d.png" % k)))
        frames.append(a.astype(np.float32) / 255.0)
    ds = md2hip.KittyDataset(str(tmp_path), "03", target_size=(128, 416))
    assert len(ds) == 2 and ds.resolution == (416, 128)
    fx = 0.5 * 7.215377e+02                    # mean((128,416)./(256,832)) * K[1,1]
    np.testing.assert_allclose(ds.K, [[fx, 0, 208], [0, fx, 64], [0, 0, 1]])
    x = ds[1]
    assert x.shape == (3, 1, 128, 416)
    # frames 3, 4, 5; a 2x bilinear downsample of the PNG keeps the frame's mean
    for j in range(3):
        assert abs(x[j, 0].mean() - frames[3 + j].mean()) < 2e-3


def test_dchain_bins(dtk):
    import md2hip
    d, files = dtk
    a = md2hip.Depth10k(d, files[:2])
    b = md2hip.Depth10k(d, files[2:])
    ch = md2hip.DChain([a, b])
    assert len(ch) == 6 and ch.bins == [2, 6]
    np.testing.assert_array_equal(ch[1], a[1])
    np.testing.assert_array_equal(ch[2], b[0])
    np.testing.assert_array_equal(ch[5], b[3])
    with pytest.raises(IndexError):
        ch[6]


def test_dataloader_batches_and_shards(dtk):
    import md2hip
    d, files = dtk
    ds = md2hip.Depth10k(d, files)
    full = md2hip.DataLoader(ds, 4, shuffle=True, seed=5, workers=2)
    batches = list(full)
    assert len(batches) == 1 and batches[0].shape == (4, 3, 3, 128, 416)   # trailing 2 dropped
    idx = full.batch_indices(0)[0]
    np.testing.assert_array_equal(batches[0].numpy(), np.stack([ds[i] for i in idx], 0))
    # two ranks of 2: the union of their shards is the single-rank batch, in order
    shards = [md2hip.DataLoader(ds, 2, shuffle=True, seed=5, rank=r, world=2).batch_indices(0)
              for r in range(2)]
    assert shards[0][0] + shards[1][0] == idx
    # a new epoch reshuffles
    assert full.batch_indices(1) != full.batch_indices(0) or len(ds) < 3


def test_dataloader_surfaces_decode_errors(tmp_path):
    import md2hip
    (tmp_path / "bad.png").write_bytes(b"not a png")
    ds = md2hip.Depth10k(str(tmp_path), ["bad.png"])
    with pytest.raises(Exception):
        list(md2hip.DataLoader(ds, 1, shuffle=False, workers=1))


def test_imresize_known_answers():
    """ImageTransformations.imresize restated (md2hip.data.imresize; src/kitty.jl:52): output
    pixel i samples the input at sf*(i - 1/2) + 1/2 (1-based) bilinearly, no antialiasing."""
    from md2hip.data import imresize
    rng = np.random.default_rng(3)
    # constant -> constant, both directions
    c = np.full((1, 10, 14), 77, dtype=np.uint8)
    assert (imresize(c, 4, 5) == 77).all() and (imresize(c, 23, 31) == 77).all()
    # an exact 2x downsample is the 2x2 box average (sample points fall between pixel pairs)
    a = rng.integers(0, 256, (1, 8, 12)).astype(np.float64)
    box = a.reshape(1, 4, 2, 6, 2).mean(axis=(2, 4))
    np.testing.assert_allclose(imresize(a, 4, 6), box, rtol=0, atol=1e-12)
    # N0f8 in -> N0f8 out: rounded to the nearest 1/255 (round half to even)
    u = np.array([[[0, 1, 2, 3]]], dtype=np.uint8)
    np.testing.assert_array_equal(imresize(u, 1, 2), [[[0, 2]]])        # 0.5 -> 0, 2.5 -> 2
    # an affine ramp is reproduced exactly at the mapped coordinates (bilinear of affine)
    H0, W0, H1, W1 = 37, 53, 16, 24
    yy, xx = np.meshgrid(np.arange(H0), np.arange(W0), indexing="ij")
    ramp = (0.3 * xx + 0.7 * yy + 2.0)[None].astype(np.float64)
    py = (H0 / H1) * (np.arange(1, H1 + 1) - 0.5) + 0.5 - 1
    px = (W0 / W1) * (np.arange(1, W1 + 1) - 0.5) + 0.5 - 1
    np.testing.assert_allclose(imresize(ramp, H1, W1)[0], 0.3 * px[None, :] + 0.7 * py[:, None] + 2.0,
                               rtol=0, atol=1e-12)
    # upsampling clamps the sample positions to the image
    up = imresize(np.array([[[0.0, 1.0]]]), 1, 4)
    np.testing.assert_allclose(up, [[[0.0, 0.25, 0.75, 1.0]]], atol=1e-12)


def test_imresize_matches_half_pixel_bilinear():
    """The same map as torch's interpolate(align_corners=False, antialias=False), at KITTI's
    1241x376 -> 416x128 and for an upsample (cross-check of the restatement, in fp64)."""
    import torch.nn.functional as F
    from md2hip.data import imresize
    rng = np.random.default_rng(4)
    for (h0, w0, h1, w1) in [(376, 1241, 128, 416), (20, 30, 64, 90)]:
        a = rng.random((1, h0, w0))
        ref = F.interpolate(torch.from_numpy(a)[None], size=(h1, w1), mode="bilinear",
                            align_corners=False, antialias=False)[0].numpy()
        np.testing.assert_allclose(imresize(a, h1, w1), ref, rtol=0, atol=1e-12)


def test_u8_samples_match_float_samples(dtk, tmp_path):
    """getobs_u8 is the same sample as getobs, as bytes: Float32(u) / 255f0 of it is bit-identical
    (RGB Depth10k with FlipX, KITTI after imresize); grayscale Depth10k has no byte form."""
    import md2hip
    from md2hip.data import _unorm
    d, files = dtk
    ds = md2hip.Depth10k(d, files, augmentations=md2hip.FlipX(0.5))
    for i in range(len(ds)):
        np.testing.assert_array_equal(_unorm(ds.getobs_u8(i, seed=2)), ds.getobs(i, seed=2))
    with pytest.raises(TypeError):
        md2hip.Depth10k(d, files, grayscale=True).getobs_u8(0)
    seq = tmp_path / "k" / "sequences" / "00" / "image_0"
    seq.mkdir(parents=True)
    (tmp_path / "k" / "sequences" / "00" / "calib.txt").write_text("P0: " + " ".join(["1.0"] * 12) + "\n")
    rng = np.random.default_rng(5)
    for k in range(3):
        Image.fromarray(rng.integers(0, 256, (376, 1241)).astype(np.uint8), mode="L").save(str(seq / ("%06d.png" % k)))
    kd = md2hip.KittyDataset(str(tmp_path / "k"), "00", target_size=(128, 416))
    u = kd.getobs_u8(0)
    assert u.dtype == np.uint8 and u.shape == (3, 1, 128, 416)
    np.testing.assert_array_equal(_unorm(u), kd[0])


def _write_png_filters(path, img):
    """A PNG whose rows cycle through all five filter types (None, Sub, Up, Average, Paeth), to
    pin the native decoder's unfiltering (PIL picks its own filters)."""
    import struct
    import zlib
    h, w = img.shape[:2]
    c = 1 if img.ndim == 2 else img.shape[2]
    a = img.reshape(h, w * c).astype(np.int64)
    raw = bytearray()
    for y in range(h):
        ft = y % 5
        cur, prev = a[y], (a[y - 1] if y else np.zeros_like(a[0]))
        left = np.concatenate([np.zeros(c, np.int64), cur[:-c]])
        ul = np.concatenate([np.zeros(c, np.int64), prev[:-c]])
        if ft == 0:
            f = cur
        elif ft == 1:
            f = cur - left
        elif ft == 2:
            f = cur - prev
        elif ft == 3:
            f = cur - (left + prev) // 2
        else:
            p = left + prev - ul
            pa, pb, pc = np.abs(p - left), np.abs(p - prev), np.abs(p - ul)
            pred = np.where((pa <= pb) & (pa <= pc), left, np.where(pb <= pc, prev, ul))
            f = cur - pred
        raw += bytes([ft]) + bytes((f % 256).astype(np.uint8))
    def chunk(t, d):
        return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xffffffff)
    ihdr = struct.pack(">IIBBBBB", w, h, 8, {1: 0, 3: 2, 4: 6}[c], 0, 0, 0)
    idat = zlib.compress(bytes(raw), 6)
    with open(path, "wb") as f:   # split IDAT in two chunks: the decoder must stream them
        f.write(b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", ihdr) + chunk(b"IDAT", idat[:len(idat) // 2]) +
                chunk(b"IDAT", idat[len(idat) // 2:]) + chunk(b"IEND", b""))


def test_native_png_decoder_all_filters(tmp_path):
    """md2_load_triplets_u8 / md2_load_kitti_u8 decode every PNG row filter bit-exactly (PIL
    agrees on the same files), RGBA drops alpha."""
    import ctypes as C
    import md2hip
    from md2hip._lib import lib
    rng = np.random.default_rng(7)
    rgb = rng.integers(0, 256, (16, 3 * 20, 3), dtype=np.uint8)
    _write_png_filters(str(tmp_path / "a.png"), rgb)
    np.testing.assert_array_equal(np.asarray(Image.open(str(tmp_path / "a.png"))), rgb)
    rgba = np.concatenate([rgb, rng.integers(0, 256, (16, 60, 1), dtype=np.uint8)], 2)
    _write_png_filters(str(tmp_path / "b.png"), rgba)
    out = np.empty((2, 3, 3, 16, 20), dtype=np.uint8)
    paths = (C.c_char_p * 2)(str(tmp_path / "a.png").encode(), str(tmp_path / "b.png").encode())
    flips = np.array([0, 1], dtype=np.uint8)
    assert lib().md2_load_triplets_u8(paths, 2, 20, 16, flips.ctypes.data_as(C.c_void_p),
                                      C.c_void_p(out.ctypes.data), 2) == 0
    ref = np.stack([rgb[:, 20 * j:20 * (j + 1)].transpose(2, 0, 1) for j in range(3)], 0)
    np.testing.assert_array_equal(out[0], ref)
    np.testing.assert_array_equal(out[1], ref[..., ::-1])
    w, h, c = C.c_int(), C.c_int(), C.c_int()
    assert lib().md2_png_info(str(tmp_path / "b.png").encode(), C.byref(w), C.byref(h), C.byref(c)) == 0
    assert (w.value, h.value, c.value) == (60, 16, 4)
    # a bad file fails loudly with its name
    (tmp_path / "bad.png").write_bytes(b"garbage")
    paths = (C.c_char_p * 1)(str(tmp_path / "bad.png").encode())
    assert lib().md2_load_triplets_u8(paths, 1, 20, 16, None, C.c_void_p(out.ctypes.data), 1) != 0
    assert b"bad.png" in lib().md2_last_error()


def test_native_batches_match_python_path(dtk, tmp_path):
    """Depth10k + FlipX, KittyDataset (imresize 1241x376 -> 416x128 + FlipX) and a DChain of
    both kinds: the native batch loader is bit-identical to the per-sample Python path, and the
    host DataLoader (native, float) delivers the same samples as getobs."""
    import md2hip
    d, files = dtk
    ds = md2hip.Depth10k(d, files, augmentations=md2hip.FlipX(0.5))
    idx = [5, 0, 3, 2]
    got = ds.batch_u8(idx, seed=4, threads=3)
    np.testing.assert_array_equal(got, np.stack([ds.getobs_u8(i, seed=4) for i in idx]))
    seq = tmp_path / "k" / "sequences" / "01" / "image_0"
    seq.mkdir(parents=True)
    (tmp_path / "k" / "sequences" / "01" / "calib.txt").write_text("P0: " + " ".join(["2.0"] * 12) + "\n")
    rng = np.random.default_rng(8)
    for k in range(9):
        _write_png_filters(str(seq / ("%06d.png" % k)), rng.integers(0, 256, (376, 1241), dtype=np.uint8))
    kd = md2hip.KittyDataset(str(tmp_path / "k"), "01", target_size=(128, 416), augmentations=md2hip.FlipX(0.5))
    got = kd.batch_u8([2, 0, 1], seed=1, threads=4)
    np.testing.assert_array_equal(got, np.stack([kd.getobs_u8(i, seed=1) for i in (2, 0, 1)]))
    loader = md2hip.DataLoader(ds, 2, shuffle=True, seed=5, workers=4)
    for b, x in zip(loader.batch_indices(0), loader):
        np.testing.assert_array_equal(x.numpy(), np.stack([ds.getobs(i, seed=5) for i in b]))


def test_native_png_decoder_rejects_corrupt_headers(tmp_path):
    """truncated data, a repeated IHDR, a short IHDR, an absurd size and a size other
    than the caller's all fail with an error naming the file (never a crash or an allocation sized
    by the header)."""
    import ctypes as C
    import struct
    import zlib
    from md2hip._lib import lib
    rng = np.random.default_rng(3)
    rgb = rng.integers(0, 256, (16, 60, 3), dtype=np.uint8)
    good = tmp_path / "good.png"
    _write_png_filters(str(good), rgb)
    blob = good.read_bytes()

    def chunk(t, d):
        return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xffffffff)
    sig, ihdr_end = blob[:8], 8 + 25
    ihdr = blob[8:ihdr_end]
    cases = {
        "trunc.png": blob[:len(blob) // 2],                                   # IDAT cut short
        "dup.png": sig + ihdr + ihdr + blob[ihdr_end:],                       # second IHDR
        "short.png": sig + chunk(b"IHDR", ihdr[8:8 + 10]) + blob[ihdr_end:],  # 10-byte IHDR
        "huge.png": sig + chunk(b"IHDR", struct.pack(">IIBBBBB", 0x80000000, 0x7fffffff, 8, 2, 0, 0, 0))
                    + blob[ihdr_end:],
        "size.png": None,                                                     # valid, wrong size
    }
    other = rng.integers(0, 256, (16, 63, 3), dtype=np.uint8)
    _write_png_filters(str(tmp_path / "size.png"), other)
    out = np.empty((1, 3, 3, 16, 20), dtype=np.uint8)
    for name, data in cases.items():
        if data is not None:
            (tmp_path / name).write_bytes(data)
        paths = (C.c_char_p * 1)(str(tmp_path / name).encode())
        assert lib().md2_load_triplets_u8(paths, 1, 20, 16, None, C.c_void_p(out.ctypes.data), 1) != 0, name
        assert name.encode() in lib().md2_last_error(), (name, lib().md2_last_error())
    paths = (C.c_char_p * 1)(str(good).encode())
    assert lib().md2_load_triplets_u8(paths, 1, 20, 16, None, C.c_void_p(out.ctypes.data), 1) == 0
