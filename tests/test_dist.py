"""Data-parallel path on CPU with the gloo backend, world size 2.

Covers what the multi-GPU bench relies on, without a GPU: global-index sharding of the
synthetic data, the bucketed async all-reduce over backward segments (each gradient entry summed
exactly once), and train_step's orchestration (segment -> bucket -> wait -> ADAM with 1/world)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from md2hip import dist as D


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class _FakeExecutor:
    """Stands in for the HIP executor: segment k writes a rank-dependent gradient slice."""

    def __init__(self, model, segments, rank):
        self.model, self.segments, self.rank = model, segments, rank
        self.nseg = len(segments)
        self.calls = []

    def forward_loss(self, x, auto_loss=None, loss=None):
        self.calls.append("fwd")
        return torch.tensor([float(self.rank)])

    def backward_segment(self, k):
        off, ln = self.segments[k]
        self.model.grad[off:off + ln] = torch.arange(off, off + ln, dtype=torch.float32) * (self.rank + 1)
        self.calls.append(k)
        return off, ln


class _FakeModel:
    def __init__(self, n):
        self.grad = torch.full((n,), float("nan"))


class _RecordingOpt:
    def __init__(self):
        self.scale = None

    def update(self, model, grad_scale=1.0):
        self.scale = grad_scale
        self.grad = model.grad.clone()


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n = 1000
        # reverse-layer-order buckets, as the library's segments: decoder tail first
        segments = [(700, 300), (400, 300), (150, 250), (0, 150)]
        D.check_segments_cover(segments, n)
        model, opt = _FakeModel(n), _RecordingOpt()
        ex = _FakeExecutor(model, segments, rank)
        comm = D.GradAllReduce()
        D.train_step(ex, model, opt, x=None, comm=comm)
        expect = torch.arange(n, dtype=torch.float32) * sum(r + 1 for r in range(world))
        q.put((rank, bool(torch.equal(opt.grad, expect)), opt.scale, ex.calls))
    finally:
        dist.destroy_process_group()


def test_train_step_allreduce_gloo_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ok, scale, calls in res:
        assert ok, f"rank {rank}: all-reduced gradient != sum over ranks"
        assert scale == pytest.approx(1.0 / world)
        assert calls == ["fwd", 0, 1, 2, 3]


def test_shards_are_gpu_count_invariant():
    B, H, W = 4, 8, 16
    whole = D.synthetic_triplets(B, H, W, 0, "cpu")
    for world in (2, 4):
        parts = []
        for r in range(world):
            b, e = D.shard_range(B, world, r)
            parts.append(D.synthetic_triplets(e - b, H, W, b, "cpu"))
        assert torch.equal(torch.cat(parts, 0), whole)
    with pytest.raises(ValueError):
        D.shard_range(10, 4, 0)


def test_segment_cover_check():
    D.check_segments_cover([(5, 5), (0, 5)], 10)
    with pytest.raises(AssertionError):
        D.check_segments_cover([(0, 5), (6, 4)], 10)
    with pytest.raises(AssertionError):
        D.check_segments_cover([(0, 5), (5, 4)], 10)


def test_single_process_comm_is_identity():
    comm = D.GradAllReduce()
    g = torch.ones(10)
    comm.bucket_ready(g, 0, 10)
    comm.wait()
    assert comm.grad_scale == 1.0 and torch.equal(g, torch.ones(10))
