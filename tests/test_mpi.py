"""MPI mode (forward parity only as upstream).

CPU: the embedding DepthDecoder's parameter table equals the oracle's param_spec with
embedding_levels = 21; the oracle's embed / bin sampler match the reference's definitions
(src/model.jl:4-21).
GPU: ``mpi_forward`` (encoder -> md2_mpi_embed_features -> 21-channel-wider DepthDecoder on the
HIP conv / upsample / concat kernels) against the fp64 oracle, relative 5e-5 per scale (fp32
accumulation over an encoder + 10-conv decoder; the mono forward's tolerance is 1e-5 at the
model output)."""
import math

import pytest
import torch

from oracle import md2_oracle as O
from tests import _data as D


def test_mpi_decoder_param_table_matches_oracle():
    from md2hip import mpi
    enc = O.encoder_stage_channels(18)
    tab = mpi.decoder_param_table(enc, (2, 3, 4, 5), 21)
    spec = [s for s in O.param_spec(18, 3, (2, 3, 4, 5), embedding_levels=21) if s[0].startswith("depth.")]
    assert [(n, tuple(s)) for n, s in tab] == [(n, tuple(s)) for n, s in spec]
    assert dict(tab)["depth.branch1.c1.weight"] == (256, 512 + 21, 3, 3)
    assert dict(tab)["depth.branch1.c2.weight"] == (256, 256 + 256 + 21, 3, 3)


def test_embed_and_bins_definitions():
    x = torch.tensor([[0.3, 0.7]], dtype=torch.float64)
    e = O.embed(x, 10)
    assert e.shape == (1, 2, 21)
    assert e[0, 1, 0] == 0.7
    assert abs(e[0, 1, 1 + 2 * 3] - math.sin(8 * 0.7)) < 1e-15        # sin(2^3 x)
    assert abs(e[0, 1, 2 + 2 * 3] - math.cos(8 * 0.7)) < 1e-15        # cos(2^3 x)
    u = torch.zeros(1, 32, dtype=torch.float64)
    b = O.disparity_bins(32, u)
    assert b[0, 0] == 1.0 and abs(b[0, 1] - (1.0 - 0.999 / 32)) < 1e-15


@pytest.mark.gpu
@pytest.mark.parametrize("N,nb", [(1, 4), (2, 3)])
def test_mpi_forward_parity(N, nb):
    import md2hip
    H, W = 64, 128
    enc = md2hip.ResNet(18, in_channels=3)
    model = md2hip.Model(enc, md2hip.DepthDecoder(encoder_channels=enc.stages, scale_levels=[2, 3, 4, 5],
                                                  embedding_levels=0), md2hip.PoseDecoder(512), seed=42)
    dec = md2hip.MPIDepthDecoder(enc.stages, (2, 3, 4, 5), 21, seed=43)
    x = D.triplets(N, 3, H, W, seed=11).float()
    u = torch.rand(N, nb, generator=torch.Generator().manual_seed(3), dtype=torch.float64)
    disps, poses = md2hip.mpi_forward(model, dec, x.cuda().contiguous(), u.float())
    torch.cuda.synchronize()
    P = O.unflatten(model.flat.cpu().double(), O.param_spec(18, 3, (2, 3, 4, 5)))
    P.update({k: v.cpu().double() for k, v in dec.params.items()})
    ref = O.mpi_model_forward(P, x.double(), u.float().double())
    assert len(disps) == 4
    for d, r in zip(disps, ref):
        assert d.shape == r.shape and d.shape[0] == N * nb
        assert D.rel_err(d, r) < 5e-5
    # the plane axis is live: different bins give different disparities for the same sample
    assert (disps[-1][0] - disps[-1][1]).abs().max() > 0
