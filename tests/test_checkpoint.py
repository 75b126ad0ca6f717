"""CPU: checkpoint / resume -- flat parameters + ADAM state round-trip
through safetensors bit-exactly, and a file written for another architecture is refused."""
import pytest
import torch


def _model(arch=18, levels=(2, 3, 4, 5), seed=42):
    import md2hip
    enc = md2hip.ResNet(arch, in_channels=3)
    return md2hip.Model(enc, md2hip.DepthDecoder(encoder_channels=enc.stages, scale_levels=list(levels),
                                                 embedding_levels=0),
                        md2hip.PoseDecoder(enc.stages[-1]), device="cpu", seed=seed)


def test_checkpoint_roundtrip(tmp_path):
    import md2hip
    a = _model(seed=42)
    opt = md2hip.ADAM(1e-4)
    g = torch.Generator().manual_seed(0)
    opt.m = torch.randn(a.numel, generator=g)
    opt.v = torch.rand(a.numel, generator=g)
    opt.t = 17
    path = str(tmp_path / "ck.safetensors")
    md2hip.save_checkpoint(path, a, opt, extra={"epoch": 3})

    b = _model(seed=7)
    assert not torch.equal(a.flat, b.flat)
    opt2 = md2hip.ADAM(3e-4, beta=(0.5, 0.5))
    extra = md2hip.load_checkpoint(path, b, opt2)
    assert extra == {"epoch": 3}
    assert torch.equal(a.flat, b.flat)
    assert torch.equal(opt.m, opt2.m) and torch.equal(opt.v, opt2.v)
    assert (opt2.t, opt2.eta, opt2.beta, opt2.eps) == (17, 1e-4, (0.9, 0.999), 1e-8)


def test_checkpoint_without_moments(tmp_path):
    import md2hip
    a = _model()
    path = str(tmp_path / "p.safetensors")
    md2hip.save_checkpoint(path, a)
    b = _model(seed=1)
    md2hip.load_checkpoint(path, b)
    assert torch.equal(a.flat, b.flat)
    with pytest.raises(ValueError):
        md2hip.load_checkpoint(path, b, md2hip.ADAM())


def test_checkpoint_refuses_other_architecture(tmp_path):
    import md2hip
    path = str(tmp_path / "r18.safetensors")
    md2hip.save_checkpoint(path, _model(18))
    with pytest.raises(ValueError):
        md2hip.load_checkpoint(path, _model(34))
    with pytest.raises(ValueError):
        md2hip.load_checkpoint(path, _model(18, levels=(3, 4, 5)))
