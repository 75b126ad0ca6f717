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
   statistics are per shard, as designed (no SyncBN; the reference is single-device).  Run at a
   small shape and at the per-rank workloads of BASELINE configs 4 (ResNet-18 416x128, 12
   triplets per rank) and 5 (ResNet-50 640x192, 8 per rank) -- scripts/script.jl:84-86.
4. The bucket order through a call-recording RCCL stand-in, at the small and the config-4 shape."""
import os
import socket

import pytest
import torch

from tests import _data as D

pytestmark = pytest.mark.gpu

H, W = 64, 128


# (arch, H, W, triplets per rank)
SHAPES = {"r18-64x128-b2": (18, 64, 128, 2),
          "config4-r18-416x128-b12": (18, 128, 416, 12),
          "config5-r50-640x192-b8": (50, 192, 640, 8)}


def _model(seed=42, arch=18):
    import md2hip
    enc = md2hip.ResNet(arch, in_channels=3)
    return md2hip.Model(enc, md2hip.DepthDecoder(encoder_channels=enc.stages, scale_levels=[2, 3, 4, 5],
                                                 embedding_levels=0), md2hip.PoseDecoder(enc.stages[-1]),
                        seed=seed)


def _setup(model, N, h=H, w=W):
    import md2hip
    K, invK = md2hip.depth10k_intrinsics(w, h)
    cache = md2hip.TrainCache(K=K, invK=invK)
    params = md2hip.Params(target_size=(w, h), batch_size=N, automasking=False)
    return model.executor((N, 3, 3, h, w), cache, params)


@pytest.mark.parametrize("shape", list(SHAPES), ids=list(SHAPES))
def test_backward_buckets_final_when_segment_returns(shape):
    from md2hip.dist import synthetic_triplets
    arch, h, w, per = SHAPES[shape]
    m = _model(arch=arch)
    ex = _setup(m, per, h, w)
    x = synthetic_triplets(per, h, w, 0, "cuda")
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


def _dp_worker(rank, world, port, q, shape):
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
        arch, h, w, per = shape
        x = MD.synthetic_triplets(per, h, w, rank * per, "cuda")
        m = _model(arch=arch)
        ex = _setup(m, per, h, w)
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


@pytest.mark.timeout(300)
@pytest.mark.parametrize("shape", list(SHAPES), ids=list(SHAPES))
def test_world2_same_device_reduced_gradient_is_shard_sum(shape):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dp_worker, args=(r, 2, port, q, SHAPES[shape])) for r in range(2)]
    for p in procs:
        p.start()
    import queue
    import time
    res = {}
    t0 = time.time()
    while len(res) < 2:
        try:
            r, local, reduced, flat = q.get(timeout=5)   # numpy: no fd sharing with the child
        except queue.Empty:
            # a rank that died (exception, crash) never reports: fail now, not at the timeout
            dead = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
            assert not dead, f"DP worker exited with {dead}"
            assert time.time() - t0 < 260, "DP workers did not report"
            print(f"waiting for DP workers ({time.time() - t0:.0f} s)", flush=True)
            continue
        res[r] = (torch.from_numpy(local), torch.from_numpy(reduced), torch.from_numpy(flat))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    total = res[0][0] + res[1][0]
    assert not torch.equal(res[0][0], res[1][0])             # different shards
    assert torch.equal(res[0][1], total) and torch.equal(res[1][1], total)
    assert torch.equal(res[0][2], res[1][2])                  # replicas stay identical


_STUB_CHILD = r"""
import ctypes as C, os, sys
root = sys.argv[1]
sys.path[:0] = [root, os.path.join(root, "monodepth2.jl_amd")]
import torch, md2hip
from md2hip import comm as MC
from md2hip.dist import synthetic_triplets
from tests.test_gpu_dp import _model, _setup, SHAPES
arch, H, W, per = SHAPES[sys.argv[2]]
stub = C.CDLL(os.environ["MD2_RCCL_LIB"])
stub.stub_get.argtypes = [C.c_int] + [C.POINTER(C.c_void_p), C.POINTER(C.c_size_t), C.POINTER(C.c_void_p), C.POINTER(C.c_void_p)]
m = _model(arch=arch)
ex = _setup(m, per, H, W)
x = synthetic_triplets(per, H, W, 0, "cuda")
dev = torch.cuda.current_device()
c = MC.Comm(0, 2, bytes(128), 0)                     # "world 2": the stub never reduces
assert torch.cuda.current_device() == dev
m.grad.fill_(float("nan"))
ex.forward_loss(x)
caller = torch.cuda.current_stream().cuda_stream
MC.backward_allreduce(ex, c)
torch.cuda.synchronize()
n = stub.stub_count()
assert n == ex.nseg, (n, ex.nseg)
base, end = m.grad.data_ptr(), m.numel
streams = set()
for i in range(n):
    recv, cnt, st, snap = C.c_void_p(), C.c_size_t(), C.c_void_p(), C.c_void_p()
    assert stub.stub_get(i, C.byref(recv), C.byref(cnt), C.byref(st), C.byref(snap)) == 0
    off = (recv.value - base) // 4
    # bucket i = backward segment i, issued in segment order: decoders, layer4 .. layer1, stem,
    # i.e. contiguous ranges walking DOWN the flat vector
    assert off + cnt.value == end, (i, off, cnt.value, end)
    end = off
    streams.add(st.value)
    got = torch.empty(cnt.value, dtype=torch.float32, device="cuda")
    md2hip._lib.check(md2hip._lib.lib().md2_memcpy_d2d(C.c_void_p(got.data_ptr()), snap, 4 * cnt.value, None))
    torch.cuda.synchronize()
    fin = m.grad[off:off + cnt.value]
    assert torch.isfinite(got).all(), f"bucket {i} snapshot holds unwritten gradient"
    assert torch.equal(got, fin), f"bucket {i}'s collective ran before its segment finished"
assert end == 0
assert len(streams) == 1 and caller not in streams, "buckets must run on the comm stream"
stub.stub_reset()
c.close()
print("STUB_OK", n)
"""


def _stub_lib():
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    so = os.path.join(root, "tests", "stubs", "librccl_stub.so")
    if not os.path.exists(so):
        import subprocess
        subprocess.run(["/opt/rocm/bin/hipcc", "-O1", "-std=c++17", "-shared", "-fPIC",
                        os.path.join(root, "tests", "stubs", "rccl_stub.cpp"), "-o", so], check=True)
    return root, so


@pytest.mark.timeout(180)
@pytest.mark.parametrize("shape", ["r18-64x128-b2", "config4-r18-416x128-b12"])
def test_library_bucket_allreduce_order_with_recording_stub(shape):
    """md2_model_backward_allreduce through a call-recording RCCL stand-in (tests/stubs): ONE
    collective per backward segment, in segment order, each covering exactly that segment's final
    gradient range, all on the communicator's own stream (not the caller's), and each ordered
    after its segment by the per-bucket event -- the stub's in-stream snapshot of every bucket is
    bit-identical to the final gradient (prefilled with NaN, so an early copy would show).  Also:
    md2_comm_init leaves the caller's current device unchanged."""
    import subprocess
    import sys
    root, so = _stub_lib()
    env = dict(os.environ, MD2_RCCL_LIB=so, MD2_TUNING="1")
    r = subprocess.run([sys.executable, "-c", _STUB_CHILD, root, shape], env=env, capture_output=True,
                       text=True, timeout=170)
    assert r.returncode == 0 and "STUB_OK" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]


_SEG_CHILD = r"""
import ctypes as C, os, sys
root, out = sys.argv[1], sys.argv[2]
sys.path[:0] = [root, os.path.join(root, "monodepth2.jl_amd")]
import numpy as np, torch, md2hip
from md2hip import comm as MC
from md2hip._lib import lib, check, ptr, stream_of
from tests import _data as D
from tests.test_gpu_dp import _model, _setup
st = stream_of(torch.device("cuda", 0))
res = {}
for path in ("dp", "single"):
    m = _model()
    ex = _setup(m, 2)
    am, av = torch.zeros_like(m.flat), torch.zeros_like(m.flat)
    loss = torch.empty(1, device="cuda")
    c = MC.Comm(0, 2, bytes(128), 0) if path == "dp" else None   # stub "world 2": grad_scale 1/2
    losses = []
    for t in range(1, 4):
        x = D.triplets(2, 3, 64, 128, seed=10 + t).float().cuda().contiguous()
        if path == "dp":
            check(lib().md2_model_train_step_dp(ex.handle, c.handle, ptr(x), None, ptr(am), ptr(av),
                                                1e-3, 0.9, 0.999, 1e-8, t, ptr(loss), st), "train_step_dp")
        else:
            check(lib().md2_model_train_step(ex.handle, ptr(x), None, ptr(am), ptr(av), 1e-3, t,
                                             ptr(loss), st), "train_step")
        torch.cuda.synchronize()
        losses.append(loss.item())
    if c is not None:
        calls, nbytes = c.stats()
        assert calls == 3 * ex.nseg and nbytes == 3 * 4 * m.numel, (calls, nbytes)
        assert c.query() == (0, 2)
        c.close()
    for k, v in (("flat", m.flat), ("m", am), ("v", av)):
        res[f"{path}_{k}"] = v.cpu().numpy()
    res[f"{path}_loss"] = np.array(losses)
np.savez(out, **res)
print("SEG_OK")
"""


@pytest.mark.timeout(240)
def test_c_train_steps_segment_update_bitwise(tmp_path):
    """the C entry points' per-segment update paths -- md2_model_train_step_dp with a
    communicator (each bucket's ADAM + re-pack on the update stream after its all-reduce; here the
    recording stub at "world 2", so grad_scale = 1/2 and no values change in the collective) and
    md2_model_train_step -- give the same parameters, ADAM moments and losses bit for bit with
    MD2_SEG_UPDATE=1 as with the default single update, over three steps that each read the
    previous step's re-packed weights.  Also: md2_comm_stats counts one all-reduce per segment
    with the whole gradient's bytes, md2_comm_rank reports the communicator's (rank, size)."""
    import subprocess
    import sys
    import numpy as np
    root, so = _stub_lib()
    outs = {}
    for seg in ("0", "1"):
        out = str(tmp_path / f"seg{seg}.npz")
        env = dict(os.environ, MD2_RCCL_LIB=so, MD2_TUNING="1", MD2_SEG_UPDATE=seg)
        r = subprocess.run([sys.executable, "-c", _SEG_CHILD, root, out], env=env, capture_output=True,
                           text=True, timeout=200)
        assert r.returncode == 0 and "SEG_OK" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]
        outs[seg] = np.load(out)
    for k in outs["0"].files:
        assert np.array_equal(outs["0"][k], outs["1"][k]), k
    assert not np.array_equal(outs["0"]["dp_flat"], outs["0"]["single_flat"])   # scale 1/2 differs
