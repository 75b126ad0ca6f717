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
