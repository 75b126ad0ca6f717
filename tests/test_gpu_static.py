"""GPU: the static-scene filter find_static (src/dtk.jl:51-69) -- per-triplet mean identity-
reprojection loss (md2_static_scores) against the fp64 oracle, and the dataset filter over
Depth10k PNG triplets written here (static, nearly static and moving triplets mixed)."""
import numpy as np
import pytest
import torch
from PIL import Image

from oracle import md2_oracle as O
from tests import _data as D

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("N,C,H,W", [(4, 3, 64, 128), (3, 1, 32, 64), (2, 3, 128, 416)])
def test_static_scores_match_oracle(N, C, H, W):
    from md2hip.primitives import static_scores
    x = D.triplets(N, C, H, W, seed=3)
    x[0, 0] = x[0, 1]                       # sample 0: frames 1 and 2 identical -> score 0
    x[0, 2] = x[0, 1]
    got = static_scores(x.float().cuda().contiguous()).cpu().double()
    ref = O.static_scores(x.float().double())
    assert got[0].item() <= 1e-6
    assert torch.allclose(got, ref, rtol=1e-5, atol=1e-7), (got, ref)


def _write_triplet(path, frames):
    arr = np.concatenate([f.transpose(1, 2, 0) for f in frames], axis=1)
    Image.fromarray((arr * 255).round().astype(np.uint8), mode="RGB").save(path)


def test_find_static_filters_depth10k(tmp_path):
    import md2hip
    rng = np.random.default_rng(5)
    files = []
    for i in range(7):
        base = rng.random((3, 128, 416))
        if i % 3 == 0:                      # static: the same frame three times
            frames = [base, base, base]
        elif i % 3 == 1:                    # nearly static: faint noise
            frames = [np.clip(base + 0.01 * rng.standard_normal(base.shape), 0, 1), base,
                      np.clip(base + 0.01 * rng.standard_normal(base.shape), 0, 1)]
        else:                               # moving: unrelated frames
            frames = [rng.random((3, 128, 416)), base, rng.random((3, 128, 416))]
        name = f"t{i}.png"
        _write_triplet(str(tmp_path / name), frames)
        files.append(name)
    ds = md2hip.Depth10k(str(tmp_path), files)
    samples = [torch.from_numpy(ds.getobs(i)).double() for i in range(len(ds))]
    scores = [O.static_scores(s.unsqueeze(0))[0].item() for s in samples]
    alpha = 0.5 * (scores[1] + max(scores[0], 1e-9))      # between "static" and "nearly static"
    got = md2hip.find_static(ds, alpha, batch=3)
    assert got == O.find_static(samples, files, alpha)
    assert "t0.png" not in got and "t2.png" in got
