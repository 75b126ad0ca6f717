"""CPU: the library's flat parameter table (md2_arch_param_info, host-only) equals the oracle's
param_spec, and the host-side Flux initialiser equals the oracle's."""
import numpy as np
import pytest
import torch

from oracle import md2_oracle as O


@pytest.mark.parametrize("arch,in_ch,levels", [(18, 3, (2, 3, 4, 5)), (18, 1, (2, 3, 4, 5)),
                                               (50, 3, (2, 3, 4, 5)), (34, 3, (3, 5))])
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
