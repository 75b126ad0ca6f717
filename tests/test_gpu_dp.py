"""Data-parallel correctness on the real HIP executor.

1. Bucket finality: the DP all-reduce of bucket k starts as soon as backward segment k is
   enqueued, which is only correct if no later segment writes into [off, off+len).  Snapshot
   each bucket right after its segment and compare with the final gradient, bit for bit.
2. The C-ABI RCCL path (md2_comm_*, md2_model_backward_allreduce, md2_model_train_step_dp) at
   world size 1 on the box: same parameters after ADAM as the plain step (sum over one rank is the
   identity), exercising RCCL init, the comm stream and the bucket events on real hardware.
3. World size 2, both ranks on cuda:0 with the real executor (gloo control plane, host-staged
   bucket reduce): the reduced gradient equals the sum of the two shard gradients computed
   sequentially, bit for bit, and both ranks end with identical parameters.  BatchNorm
   statistics are per shard, as designed (no SyncBN; the reference is single-device)."""
import os
import socket

import pytest
import torch

from tests import _data as D

pytestmark = pytest.mark.gpu

H, W = 64, 128


def _model(seed=42):
    import md2hip
    enc = md2hip.ResNet(18, in_channels=3)
    return md2hip.Model(enc, md2hip.DepthDecoder(encoder_channels=enc.stages, scale_levels=[2, 3, 4, 5],
                                                 embedding_levels=0), md2hip.PoseDecoder(512), seed=seed)


def _setup(model, N):
    import md2hip
    K, invK = md2hip.depth10k_intrinsics(W, H)
    cache = md2hip.TrainCache(K=K, invK=invK)
    params = md2hip.Params(target_size=(W, H), batch_size=N, automasking=False)
    return model.executor((N, 3, 3, H, W), cache, params)


def test_backward_buckets_final_when_segment_returns():
    from md2hip.dist import synthetic_triplets
    m = _model()
    ex = _setup(m, 2)
    x = synthetic_triplets(2, H, W, 0, "cuda")
    m.grad.fill_(float("nan"))
    ex.forward_loss(x)
    snaps = []
    for k in range(ex.nseg):
        off, ln = ex.backward_segment(k)
        torch.cuda.synchronize()
        snaps.append((off, ln, m.grad[off:off + ln].clone()))
    torch.cuda.synchronize()
    covered = 0
    for off, ln, s in snaps:
        assert torch.isfinite(s).all()
        assert torch.equal(s, m.grad[off:off + ln]), f"bucket [{off}, {off + ln}) changed after its segment"
        covered += ln
    assert covered == m.numel


def test_rccl_comm_world1_matches_single_gpu_step():
    import md2hip
    from md2hip import comm as MC
    from md2hip.dist import synthetic_triplets
    x = synthetic_triplets(2, H, W, 0, "cuda")
    flats = []
    for use_comm in (False, True):
        m = _model()
        ex = _setup(m, 2)
        opt = md2hip.ADAM(1e-4)
        c = MC.Comm(0, 1, MC.unique_id(), 0) if use_comm else None
        for _ in range(2):
            MC.train_step_dp(ex, m, opt, x, c)
        torch.cuda.synchronize()
        # the generic in-place all-reduce on the caller's stream
        if c is not None:
            t = torch.arange(10, dtype=torch.float32, device="cuda")
            c.allreduce_sum(t)
            torch.cuda.synchronize()
            assert torch.equal(t.cpu(), torch.arange(10, dtype=torch.float32))
            c.close()
        flats.append(m.flat.cpu())
    assert torch.equal(flats[0], flats[1])


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _dp_worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "monodepth2.jl_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch.distributed as dist
    import md2hip
    from md2hip import dist as MD
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        per = 2
        x = MD.synthetic_triplets(per, H, W, rank * per, "cuda")
        m = _model()
        ex = _setup(m, per)
        # this shard's own gradient (no exchange)
        ex.forward_loss(x)
        ex.backward()
        torch.cuda.synchronize()
        local = m.grad.cpu().numpy().copy()
        # the DP step: bucketed all-reduce after each segment, ADAM with 1/world
        opt = md2hip.ADAM(1e-4)
        MD.train_step(ex, m, opt, x, MD.GradAllReduce())
        torch.cuda.synchronize()
        q.put((rank, local, m.grad.cpu().numpy().copy(), m.flat.cpu().numpy().copy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(240)
def test_world2_same_device_reduced_gradient_is_shard_sum():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        r, local, reduced, flat = q.get(timeout=200)     # numpy: no fd sharing with the child
        res[r] = (torch.from_numpy(local), torch.from_numpy(reduced), torch.from_numpy(flat))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    total = res[0][0] + res[1][0]
    assert not torch.equal(res[0][0], res[1][0])             # different shards
    assert torch.equal(res[0][1], total) and torch.equal(res[1][1], total)
    assert torch.equal(res[0][2], res[1][2])                  # replicas stay identical
