"""GPU: the DataLoader's pinned-memory side-stream copies deliver exactly the decoded samples,
and its batches drive the HIP train step."""
import numpy as np
import pytest
import torch
from PIL import Image

pytestmark = pytest.mark.gpu


def test_dataloader_feeds_train_step(tmp_path):
    import md2hip
    rng = np.random.default_rng(0)
    files = []
    for i in range(4):
        a = (rng.random((128, 3 * 416, 3)) * 255).round().astype(np.uint8)
        Image.fromarray(a, mode="RGB").save(str(tmp_path / f"{i}.png"))
        files.append(f"{i}.png")
    ds = md2hip.Depth10k(str(tmp_path), files, augmentations=md2hip.FlipX(0.5))
    loader = md2hip.DataLoader(ds, 2, shuffle=True, seed=1, workers=2, device="cuda")
    idx = loader.batch_indices(0)
    enc = md2hip.ResNet(18, in_channels=3)
    model = md2hip.Model(enc, md2hip.DepthDecoder(encoder_channels=enc.stages, scale_levels=[2, 3, 4, 5],
                                                  embedding_levels=0), md2hip.PoseDecoder(512), seed=42)
    cache = md2hip.TrainCache(K=ds.K, invK=ds.invK)
    params = md2hip.Params(target_size=ds.resolution, batch_size=2, automasking=False)
    opt = md2hip.ADAM(1e-4)
    for b, x in enumerate(loader):
        assert x.is_cuda and x.shape == (2, 3, 3, 128, 416)
        ref = np.stack([ds.getobs(i, seed=1) for i in idx[b]], 0)
        np.testing.assert_array_equal(x.cpu().numpy(), ref)
        loss = md2hip.train_step(model, x, None, cache, params, opt)
        torch.cuda.synchronize()
        assert torch.isfinite(loss).all()
    assert b == 1
