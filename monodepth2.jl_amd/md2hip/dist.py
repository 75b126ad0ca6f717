"""Data-parallel train step: one process per GPU, RCCL (torch.distributed "nccl") over xGMI.

SURVEY.md section 8(e): triplets are independent and every loss term is a mean over pixels and
batch, so with equal shards the global gradient is the mean of the shard gradients.  The only
exchange is a sum all-reduce of the flat fp32 gradient, scaled by 1/world inside ADAM.  It is
bucketed by the library's backward segments (decoder+pose first, then encoder stages 4..1,
stem) and each bucket's collective is launched as soon as that segment's kernels are enqueued,
so RCCL (on its own stream, ordered after the segment by the process group) overlaps the
remaining backward.  BatchNorm statistics stay per GPU (the reference is single-device; no
SyncBN) -- the one documented difference from a single-device run of the global batch.

The same code runs with the gloo backend on CPU tensors (tests/test_dist.py)."""
from __future__ import annotations

import os
from typing import List, Optional, Sequence, Tuple


def shard_range(global_batch: int, world: int, rank: int) -> Tuple[int, int]:
    """[begin, end) global sample indices of ``rank`` (equal shards, global_batch % world == 0)."""
    if global_batch % world:
        raise ValueError(f"global batch {global_batch} is not divisible by {world} ranks")
    per = global_batch // world
    return rank * per, (rank + 1) * per


def synthetic_triplets(batch: int, height: int, width: int, first_index: int, device, seed: int = 1234,
                       channels: int = 3):
    """Uniform [0,1) triplets [batch, 3 frames, C, H, W] keyed by GLOBAL sample index, so the
    union of the shards is the same data for every GPU count."""
    import torch
    xs = []
    for i in range(batch):
        g = torch.Generator().manual_seed(seed + first_index + i)
        xs.append(torch.rand(3, channels, height, width, generator=g))
    return torch.stack(xs, 0).to(device).contiguous()


class GradAllReduce:
    """Overlapped bucket all-reduce of slices of one flat gradient vector."""

    def __init__(self, group=None, force: bool = False):
        import torch.distributed as dist
        self.group = group
        on = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(group) if on else 1
        self.backend = dist.get_backend(group) if on else None
        self.force = force and on           # run the collective even at world size 1 (tests)
        self._handles: List = []
        self.calls = 0                      # collectives launched and their payload (bench.py)
        self.bytes = 0

    def bucket_ready(self, flat_grad, off: int, length: int):
        """Launch the sum all-reduce of flat_grad[off:off+length] (returns immediately)."""
        if (self.world == 1 and not self.force) or length == 0:
            return
        import torch.distributed as dist
        sl = flat_grad[off:off + length]
        self.calls += 1
        self.bytes += length * sl.element_size()
        if self.backend == "gloo" and sl.is_cuda:
            # host control-plane backend (CPU tests, same-device rehearsal): stage through the host
            h = sl.cpu()
            dist.all_reduce(h, group=self.group)
            sl.copy_(h)
            return
        self._handles.append(dist.all_reduce(sl, group=self.group, async_op=True))

    def wait(self):
        """Make the current stream wait for every launched bucket."""
        for h in self._handles:
            h.wait()
        self._handles.clear()

    @property
    def grad_scale(self) -> float:
        return 1.0 / self.world

    @property
    def active(self) -> bool:
        """Whether bucket_ready launches collectives (world > 1, or forced)."""
        return self.world > 1 or self.force


def train_step(executor, model, opt, x, comm: Optional[GradAllReduce] = None, loss=None):
    """forward_loss -> backward segments (each followed by its bucket all-reduce) -> ADAM with
    gradient scale 1/world.  Returns the device loss tensor (this rank's shard loss)."""
    comm = comm or GradAllReduce()
    out = executor.forward_loss(x, None, loss=loss)
    # one update after the last bucket unless MD2_SEG_UPDATE=1 (concurrent per-segment updates
    # measured 2% slower at N=1, profiles/r04_seg_update_ab.txt)
    if comm.active or os.environ.get("MD2_SEG_UPDATE") != "1":
        for k in range(executor.nseg):
            off, ln = executor.backward_segment(k)
            comm.bucket_ready(model.grad, off, ln)
        comm.wait()
        opt.update(model, grad_scale=comm.grad_scale)
        return out
    # no exchange: each segment's update runs beside the remaining backward (same arithmetic)
    for k in range(executor.nseg):
        executor.backward_segment(k)
        opt.update_segment(model, k)
    opt.finish(model)
    return out


def check_segments_cover(segments: Sequence[Tuple[int, int]], total: int):
    """The backward buckets must partition [0, total) (each gradient reduced exactly once)."""
    cov = sorted(segments)
    pos = 0
    for off, ln in cov:
        if off != pos or ln <= 0:
            raise AssertionError(f"segments do not tile the gradient at {pos}: {cov}")
        pos += ln
    if pos != total:
        raise AssertionError(f"segments cover {pos} of {total} gradient entries")
