"""CPU: the library's flat parameter table (md2_arch_param_info, host-only) equals the oracle's
param_spec, and the host-side Flux initialiser equals the oracle's."""
import numpy as np
import pytest
import torch

from oracle import md2_oracle as O


@pytest.mark.parametrize("arch,in_ch,levels", [(18, 3, (2, 3, 4, 5)), (18, 1, (2, 3, 4, 5)),
                                               (50, 3, (2, 3, 4, 5)), (34, 3, (3, 5)),
                                               (18, 3, (1, 2, 3, 4, 5)), (18, 3, (1, 3)), (18, 3, (4,))])
def test_param_table_matches_oracle(arch, in_ch, levels):
    import md2hip
    table, total = md2hip.param_table(arch, in_ch, levels)
    spec = O.param_spec(arch, in_ch, levels)
    assert [t[0] for t in table] == [s[0] for s in spec]
    assert [tuple(t[1]) for t in table] == [tuple(s[1]) for s in spec]
    off = 0
    for (name, shape, o) in table:
        assert o == off
        off += int(np.prod(shape))
    assert off == total


def test_resnet18_param_count():
    """ResNet-18 encoder 11.17M + depth decoder 3.15M + pose decoder 1.90M."""
    import md2hip
    table, total = md2hip.param_table(18, 3, (2, 3, 4, 5))
    enc = sum(int(np.prod(s)) for n, s, _ in table if n.startswith("encoder"))
    dep = sum(int(np.prod(s)) for n, s, _ in table if n.startswith("depth"))
    pos = sum(int(np.prod(s)) for n, s, _ in table if n.startswith("pose"))
    assert abs(enc / 1e6 - 11.17) < 0.01 and abs(dep / 1e6 - 3.15) < 0.01 and abs(pos / 1e6 - 1.90) < 0.01


def test_flux_init_matches_oracle():
    import md2hip
    from md2hip.model import flux_init
    table, total = md2hip.param_table(18, 3, (2, 3, 4, 5))
    a = flux_init(table, total, seed=42)
    b = O.init_params(O.param_spec(18, 3, (2, 3, 4, 5)), seed=42)
    assert torch.equal(a, b)


@pytest.mark.parametrize("levels,rc", [((3, 3), 3), ((4, 2), 3), ((0, 5), 1), ((2, 6), 1),
                                       ((1, 2, 3, 4, 5, 5), 1)])
def test_rejected_scale_levels(levels, rc):
    """Levels outside 1:5 or more than 5 of them: MD2_EINVAL (the reference's own error,
    src/depth_decoder.jl:27-29); repeated / decreasing levels: MD2_ENOTSUP (the reference builds
    empty branches: a duplicate head, or a channel mismatch at run time)."""
    import ctypes as C
    import md2hip
    from md2hip._lib import ModelCfg, lib
    c = ModelCfg()
    c.arch, c.in_channels, c.n_levels = 18, 3, min(len(levels), 5)
    for i, l in enumerate(levels[:5]):
        c.scale_levels[i] = l
    if len(levels) > 5:
        c.n_levels = 6
    n, e = C.c_longlong(), C.c_longlong()
    assert lib().md2_arch_param_count(C.byref(c), C.byref(n), C.byref(e)) == rc
    with pytest.raises(NotImplementedError if rc == 3 else ValueError):
        md2hip.DepthDecoder(encoder_channels=(64, 64, 128, 256, 512), scale_levels=list(levels), embedding_levels=0)


@pytest.mark.parametrize("target_id,source_ids,exc", [(4, (1, 3), ValueError), (2, (0, 3), ValueError),
                                                      (2, (1,), NotImplementedError),
                                                      (2, (1, 3, 3), NotImplementedError)])
def test_rejected_frame_ids(target_id, source_ids, exc):
    import md2hip
    from md2hip.model import _cfg
    K, iK = md2hip.depth10k_intrinsics(128, 64)
    cache = md2hip.TrainCache(K=K, invK=iK, target_id=target_id, source_ids=source_ids)
    with pytest.raises(exc):
        _cfg(18, 3, (2, 3, 4, 5), cache=cache)


def test_general_frame_ids_accepted():
    import md2hip
    from md2hip.model import _cfg
    K, iK = md2hip.depth10k_intrinsics(128, 64)
    for t, s in [(1, (2, 3)), (3, (1, 2)), (2, (3, 1))]:
        c = _cfg(18, 3, (1, 3, 5), cache=md2hip.TrainCache(K=K, invK=iK, target_id=t, source_ids=s,
                                                           scales=(0.0625, 0.25, 1.0)))
        assert (c.target, c.src0, c.src1) == (t - 1, s[0] - 1, s[1] - 1)


@pytest.mark.parametrize("arch,levels", [(18, (2, 3, 4, 5)), (50, (2, 3, 4, 5)), (18, (1, 3, 5))])
def test_mpi_param_table_matches_oracle(arch, levels):
    """MPI mode: DepthDecoder(; embedding_levels=21) widens every decoder input by the embedding
    (src/depth_decoder.jl:32) -- the library table equals the oracle's spec."""
    import md2hip
    table, total = md2hip.param_table(arch, 3, levels, embedding_levels=21)
    spec = O.param_spec(arch, 3, levels, embedding_levels=21)
    assert [(t[0], tuple(t[1])) for t in table] == [(s[0], tuple(s[1])) for s in spec]
    d = {t[0]: tuple(t[1]) for t in table}
    enc = O.encoder_stage_channels(arch)
    assert d["depth.branch1.c1.weight"][1] == enc[4] + 21


def test_disparity_bins_definition():
    """uniformly_sample_disparity_from_linspace_bins (src/model.jl:17-21)."""
    import md2hip
    u = torch.tensor([[0.0, 0.5, 0.25]], dtype=torch.float64)
    b = md2hip.disparity_bins(1, 3, u=u, device="cpu")
    edges = np.linspace(1.0, 0.001, 4)[:-1]
    iv = edges[1] - edges[0]
    np.testing.assert_allclose(b.numpy()[0], (edges + u.numpy()[0] * iv).astype(np.float32))
    assert b.dtype == torch.float32
