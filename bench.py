#!/usr/bin/env python3
"""Train-step throughput of the MI355X-native Monodepth2 hot path (BASELINE.json metric).

One step = Model forward on B synthetic 416x128 RGB triplets (ResNet-18 encoder on 3B frames,
DepthDecoder, PoseDecoder) + train_loss (4 scales, warp+SSIM+L1, smoothness) + full backward +
gradient all-reduce over RCCL (N > 1, bucketed per backward segment and overlapped with the
remaining backward) + Flux ADAM update.  Inputs are resident in HBM before timing.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

``--gpus N`` with N > 1 and no launcher around it (WORLD_SIZE unset) starts the N local ranks
itself (torchrun-style, before anything touches the GPU) and exits with their status; it exits
non-zero when fewer than N devices are visible or when WORLD_SIZE disagrees with --gpus -- it
never runs fewer ranks than asked.  The JSON line carries the communicator's own rank count
(md2_comm_rank) and the all-reduce calls / bytes per step it counted (md2_comm_stats).

Rank 0 prints ONE JSON line.  ``value`` = images (training triplets) per second for the whole
job; ``roofline`` is measured live with HIP events on the model's stream around every
encoder 3x3 conv launch (fwd + dgrad + wgrad, the MFMA-bound kernels); ``roofline_photometric``
does the same for the fused warp+SSIM kernel (HBM-bound); ``cpu_baseline`` times the CPU
restatement (oracle/) of the same step on this host (rank 0, N = 1 only)."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "monodepth2.jl_amd"))
sys.path.insert(0, ROOT)

METRIC = "train-step images/sec, ResNet-18 416×128; 1/2/4/8 MI355X + roofline %"
PEAK_FP32_MFMA_TFLOPS = 157.3      # MI355X_MICROARCH.md: Peak FP32 (matrix), dense
PEAK_HBM_GBS = 8000.0              # MI355X_MICROARCH.md: HBM3E 8 TB/s
# the 3x3 convs (fwd, dgrad, wgrad) run bf16x6 (conv_px3 / conv_wgrad_px3: every fp32 operand
# split exactly into 3 bf16 terms, the 6 partial products down to 2^-16 on the bf16 MFMA, fp32
# sums): their own ceiling is the dense bf16 MFMA rate / 6
PEAK_BF16_MFMA_TFLOPS = 2516.0     # MI355X_MICROARCH.md: ~2.5 PF dense bf16
PEAK_BF16X6_TFLOPS = PEAK_BF16_MFMA_TFLOPS / 6


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=12, help="triplets per GPU")
    ap.add_argument("--height", type=int, default=128)
    ap.add_argument("--width", type=int, default=416)
    ap.add_argument("--arch", type=int, default=18)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-probe", action="store_true", help="skip the HIP-event roofline probe")
    ap.add_argument("--probe-steps", type=int, default=5,
                    help="profiled steps after the timed region (per-category minimum is reported)")
    ap.add_argument("--graph", action="store_true",
                    help="single GPU: replay the step as its captured hipGraph (measured neutral at "
                         "B=12: 1338 vs 1342 images/s eager -- the GPU is never starved of launches)")
    ap.add_argument("--comm", choices=("md2", "torch"), default="md2",
                    help="gradient all-reduce for N > 1: the library's own RCCL communicator "
                         "(md2_comm_*, gloo only as the host control plane) or torch.distributed nccl")
    ap.add_argument("--force-dp", action="store_true",
                    help="run the data-parallel step (process group, all-reduce) even at N = 1")
    ap.add_argument("--launcher-selftest", action="store_true",
                    help="test hook (tests/test_bench_launcher.py): the ranks run only the gloo "
                         "control plane (one all-reduce, no GPU) and rank 0 prints the JSON line")
    return ap.parse_args()


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


KFD_NODES = "/sys/class/kfd/kfd/topology/nodes"


def _kfd_gpus(root=KFD_NODES) -> int:
    """GPU agents in the KFD topology (nodes whose properties report SIMDs), -1 if unreadable --
    read from sysfs, so no HIP runtime is loaded."""
    try:
        names = os.listdir(root)
    except OSError:
        return -1
    n = 0
    for d in names:
        try:
            with open(os.path.join(root, d, "properties")) as f:
                props = dict(line.split(None, 1) for line in f if len(line.split(None, 1)) == 2)
        except OSError:
            continue
        if int(props.get("simd_count", "0").strip() or 0) > 0:
            n += 1
    return n


def _visible_devices(selftest: bool) -> int:
    """GPUs this process can see, counted WITHOUT initialising HIP, so that the parent may still
    start the ranks: the KFD topology in sysfs, capped by HIP_VISIBLE_DEVICES /
    ROCR_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES.  -1 when the topology is unreadable (no fallback
    to a HIP device query).  The launcher self-test takes MD2_BENCH_FAKE_DEVICES instead
    (CPU-only containers)."""
    if selftest and "MD2_BENCH_FAKE_DEVICES" in os.environ:
        return int(os.environ["MD2_BENCH_FAKE_DEVICES"])
    n = _kfd_gpus()
    if n < 0:
        return -1
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([t for t in v.split(",") if t.strip()]))
    return n


def _under_profiler() -> bool:
    """rocprofv3 initialises the GPU in every process it wraps (its preloaded tool library), so a
    launcher parent under it would spawn ranks from a GPU-initialised process."""
    return any(k.startswith(("ROCPROF", "ROCP_")) for k in os.environ)


def launch_local(args) -> int:
    """Start args.gpus ranks of this script on this node (RANK / LOCAL_RANK / WORLD_SIZE /
    MASTER_ADDR=127.0.0.1 / MASTER_PORT, as torch.distributed.run sets them) and wait for all of
    them.  Rank 0 prints the JSON line on the inherited stdout.  A rank that fails ends the others
    (their exact PIDs) and its exit status is returned."""
    import signal
    import subprocess
    n = args.gpus
    if _under_profiler() and not args.launcher_selftest:
        print("bench.py: --gpus N > 1 under a profiler: the profiler initialises the GPU in this "
              "parent; launch the ranks with `python -m torch.distributed.run` from a clean shell",
              file=sys.stderr, flush=True)
        return 2
    have = _visible_devices(args.launcher_selftest)
    if have < 0:
        print("bench.py: cannot count GPUs without initialising HIP (no KFD topology in sysfs); "
              "launch the ranks with `python -m torch.distributed.run`", file=sys.stderr, flush=True)
        return 2
    if have < n:
        print(f"bench.py: --gpus {n} needs {n} visible GPUs, found {have}; refusing to run "
              f"fewer ranks", file=sys.stderr, flush=True)
        return 2
    port = str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    print(f"bench.py: started {n} ranks (pids {[p.pid for p in procs]}), master 127.0.0.1:{port}",
          file=sys.stderr, flush=True)
    def stop(live, grace=10.0):
        for q in live:
            if q.poll() is None:
                q.terminate()
        t_end = time.time() + grace
        for q in live:
            try:
                q.wait(timeout=max(0.1, t_end - time.time()))
            except subprocess.TimeoutExpired:
                q.kill()

    # a SIGTERM / SIGINT to the launcher (a driver's timeout) ends the ranks it started -- their
    # exact PIDs -- instead of orphaning them on the GPUs and the rendezvous port
    def on_signal(signum, frame):
        print(f"bench.py: signal {signum}: stopping ranks {[p.pid for p in procs]}", file=sys.stderr, flush=True)
        stop(procs)
        sys.exit(128 + signum)

    old_handlers = {sig: signal.signal(sig, on_signal) for sig in (signal.SIGTERM, signal.SIGINT)}
    rc = 0
    live = list(procs)
    try:
        while live:
            for p in list(live):
                code = p.poll()
                if code is None:
                    continue
                live.remove(p)
                if code != 0 and rc == 0:
                    rc = code if code > 0 else 128 - code
                    print(f"bench.py: rank pid {p.pid} exited with {code}; stopping the others",
                          file=sys.stderr, flush=True)
                    stop(live)
            time.sleep(0.05)
    finally:
        stop(procs)
        for sig, h in old_handlers.items():
            signal.signal(sig, h)
    return rc


def _selftest_rank(json_fd) -> None:
    """--launcher-selftest body of one rank: gloo process group, one all-reduce of a ones vector
    (its sum is the number of ranks that took part), rank 0 prints the JSON line."""
    import torch
    import torch.distributed as dist
    world = int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo")
    t = torch.ones(4)
    dist.all_reduce(t)
    got = int(t[0].item())
    pids = [None] * world
    dist.all_gather_object(pids, os.getpid())
    if dist.get_rank() == 0:
        line = {"metric": METRIC, "selftest": True, "n_gpus": world,
                "comm": {"nranks": dist.get_world_size(), "allreduce_ranks_seen": got,
                         "rank_pids": pids}}
        os.write(json_fd, (json.dumps(line) + "\n").encode())
    dist.destroy_process_group()
    if got != world:
        raise SystemExit(f"all-reduce saw {got} ranks, expected {world}")


def synthetic_batch(batch, height, width, rank, device):
    """Uniform [0,1) triplets keyed by GLOBAL sample index (GPU-count invariant shards)."""
    from md2hip.dist import synthetic_triplets
    return synthetic_triplets(batch, height, width, rank * batch, device)


def _host_cpu():
    """Host CPU model, logical CPU count of the machine and the CPUs this process may run on."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        avail = os.cpu_count() or 1
    # a container's CPU quota (cgroup v2 cpu.max / v1 cfs quota) caps the usable cores below
    # what the affinity mask shows: more threads than that only oversubscribe the quota
    quota = None
    for path, parse in (("/sys/fs/cgroup/cpu.max", lambda t: t.split()),
                        ("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", lambda t: [t.strip(), None])):
        try:
            with open(path) as f:
                q, p = parse(f.read())
            if q not in ("max", "-1"):
                if p is None:
                    with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                        p = f.read().strip()
                quota = max(1, int(int(q) // int(p)))
            break
        except (OSError, ValueError):
            continue
    if quota is not None:
        avail = min(avail, quota)
    return model, os.cpu_count() or 1, avail


def _median_time(fn, warmup, min_steps, seconds):
    """2 untimed warm-ups, then the median of >= min_steps timed calls (more while time allows)."""
    import statistics
    for _ in range(warmup):
        fn()
    times = []
    t_end = time.perf_counter() + seconds
    while len(times) < min_steps or time.perf_counter() < t_end:
        t0 = time.perf_counter()
        fn()
        times.append(time.perf_counter() - t0)
        print(f"cpu baseline: step {len(times)} {times[-1]:.2f} s", file=sys.stderr, flush=True)
        if len(times) >= 50:
            break
    return statistics.median(times), len(times)


def cpu_baseline(args, seconds):
    """The oracle (torch-CPU fp32 restatement of the reference step, oracle/md2_oracle.py) on the
    host cores: forward + train_loss + autograd backward + Flux ADAM (BASELINE config 3), and
    eval_disparity (config 2), same shapes and batch.  Threads = every CPU this process may run on
    (the box's per-GPU CPU share; `nproc` reports the whole machine)."""
    import torch
    from oracle import md2_oracle as O
    model, nproc, avail = _host_cpu()
    threads = avail
    torch.set_num_threads(threads)
    print(f"cpu baseline: {threads} threads ({nproc} logical CPUs on the host, {model})",
          file=sys.stderr, flush=True)
    B, H, W = args.batch, args.height, args.width
    spec = O.param_spec(args.arch, 3, (2, 3, 4, 5))
    flat = O.init_params(spec, 42, dtype=torch.float32).requires_grad_(True)
    K, invK = O.depth10k_K(W, H, torch.float32)
    cache = O.TrainCache(K=K, invK=invK)
    params = O.Params(target_size=(W, H), batch_size=B, automasking=False)
    opt = O.Adam(1e-4)
    x = synthetic_batch(B, H, W, 0, "cpu")

    def step():
        P = O.unflatten(flat, spec)
        loss = O.train_loss(P, x, None, cache, params, arch=args.arch)
        g, = torch.autograd.grad(loss, flat)
        with torch.no_grad():
            opt.step("flat", flat, g)
        return loss.item()

    t, n = _median_time(step, 2, 5, seconds)
    out = {"value": round(B / t, 3), "unit": "images/s", "cores": threads, "kind": "port",
           "nproc": nproc, "cpu_model": model,
           "sample": f"median of {n} full train steps at batch {B} {W}x{H} after 2 warm-ups "
                     f"(fp32 torch-CPU restatement of the Flux/Zygote reference, oracle/md2_oracle.py; "
                     f"baseline only)"}

    def evald():
        with torch.no_grad():
            P = O.unflatten(flat.detach(), spec)
            O.eval_disparity(P, x[:, 1].contiguous(), arch=args.arch)

    t2, n2 = _median_time(evald, 2, 5, seconds / 3)
    out["eval_disparity"] = {"value": round(B / t2, 3), "unit": "images/s",
                             "sample": f"median of {n2} eval_disparity calls at batch {B} (BASELINE config 2)"}
    return out


def pmc_traffic():
    """HBM bytes per launch of the roofline kernel set from the newest committed PMC profile
    (tools/profile_round.sh + tools/prof_summary.py: separate FETCH_SIZE / WRITE_SIZE passes,
    FETCH doubled per the gfx950 note).  PMC cannot run inside the timed bench."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc.json")))
    if not files:
        return None, None
    with open(files[-1]) as f:
        t = json.load(f).get("traffic")
    if not t:
        return None, None
    return round(t["bytes_per_launch"]), os.path.relpath(files[-1], ROOT)


def pmc_mfma_busy():
    """MFMA pipe busy fraction of the roofline set (per family and overall) from the newest
    committed profile carrying it (tools/profile_round.sh's SQ_VALU_MFMA_BUSY_CYCLES pass)."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc.json")), reverse=True):
        with open(path) as f:
            m = json.load(f).get("mfma_busy")
        if m:
            return m, os.path.relpath(path, ROOT)
    return None, None


def pmc_photo_traffic(batch):
    """HBM bytes per launch of the photometric kernel at this batch from the newest committed
    tools/pmc_photo.sh profile (profiles/r*_pmc_photo.json; FETCH doubled per the gfx950 note,
    uncalibrated for 4-byte gathers) -- PMC cannot run inside the timed bench."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_photo.json")))
    if not files:
        return None, None, None
    with open(files[-1]) as f:
        d = json.load(f)
    row = d.get("by_batch", {}).get(str(batch))
    if not row or d.get("scales_per_launch") != 4:
        return None, None, None
    src = os.path.relpath(files[-1], ROOT)
    # what bounds the kernel, from the same profile's counters (tools/pmc_photo_summary.py)
    note = (f"{src} at B={batch}: {row['avg_us']:.1f} us/launch under the profiler, VALU issue "
            f"utilisation {row['valu_issue_utilisation']:.2f}, waves active {row['active_inst_any']:.0%} / "
            f"waiting {row['wait_any']:.0%}, {row['valu_insts_per_pixel_scale']:.0f} VALU instr per "
            f"pixel-scale; traffic {row['traffic_bytes'] / row['algorithmic_bytes']:.2f}x algorithmic (DESIGN.md sec. 4)")
    return row["traffic_bytes"], src, note


def main():
    args = parse()
    if args.gpus < 1:
        print("bench.py: --gpus must be >= 1", file=sys.stderr)
        sys.exit(2)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # no launcher around us: start the ranks here, before this process touches the GPU
        sys.exit(launch_local(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}; refusing to guess",
              file=sys.stderr)
        sys.exit(2)
    # libraries print banners on fd 1 (RCCL's version block, gloo's peer count): keep stdout for
    # the ONE JSON line -- everything else goes to stderr until it is printed
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)
    if args.launcher_selftest:
        _selftest_rank(json_fd)
        return
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dp = world > 1 or args.force_dp
    if local >= torch.cuda.device_count():
        print(f"bench.py: rank {rank} wants device {local}, {torch.cuda.device_count()} visible",
              file=sys.stderr)
        sys.exit(2)
    if dp:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        os.environ.setdefault("RANK", str(rank))
        os.environ.setdefault("WORLD_SIZE", str(world))
        torch.cuda.set_device(local)
        if args.comm == "md2":
            dist.init_process_group("gloo")            # host control plane only
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    import md2hip
    import md2hip.comm
    import md2hip.dist
    B, H, W = args.batch, args.height, args.width
    enc = md2hip.ResNet(args.arch, in_channels=3)
    model = md2hip.Model(enc, md2hip.DepthDecoder(encoder_channels=enc.stages, scale_levels=[2, 3, 4, 5],
                                                  embedding_levels=0),
                         md2hip.PoseDecoder(enc.stages[-1]), device=dev, seed=42)
    K, invK = md2hip.depth10k_intrinsics(W, H)
    cache = md2hip.TrainCache(K=K, invK=invK, scales=(0.125, 0.25, 0.5, 1.0))
    params = md2hip.Params(target_size=(W, H), batch_size=B, automasking=False, disparity_smoothness=1e-3)
    opt = md2hip.ADAM(1e-4)
    x = synthetic_batch(B, H, W, rank, dev)
    ex = model.executor(tuple(x.shape), cache, params)
    loss_buf = torch.empty(1, dtype=torch.float32, device=dev)
    comm = None
    if dp and args.comm == "md2":
        comm = md2hip.comm.Comm(rank, world, md2hip.comm.broadcast_id(rank), local)
        crank, cranks = comm.query()
        if (crank, cranks) != (rank, world):
            raise SystemExit(f"RCCL communicator reports rank {crank} of {cranks}, expected {rank} of {world}")

        def step():
            md2hip.comm.train_step_dp(ex, model, opt, x, comm, loss=loss_buf)
    elif not dp and args.graph:
        # single GPU: the whole step replays as one captured hipGraph (same kernels, same order,
        # bit-identical to the eager step: tests/test_gpu_graph.py)
        def step():
            ex.train_step_graph(x, opt, loss=loss_buf)
    else:
        comm = md2hip.dist.GradAllReduce(force=args.force_dp)

        def step():
            md2hip.dist.train_step(ex, model, opt, x, comm, loss=loss_buf)

    def barrier():
        torch.cuda.synchronize()
        if dp:
            dist.barrier()
        torch.cuda.synchronize()

    step()                                   # step 1 (warm-up): its loss is pinned by a test
    torch.cuda.synchronize()
    loss_first = loss_buf.item()
    for _ in range(max(args.warmup - 1, 0)):
        step()
    def comm_counts():
        if comm is None:
            return 0, 0
        if isinstance(comm, md2hip.comm.Comm):
            return comm.stats()
        return comm.calls, comm.bytes

    barrier()
    c0 = comm_counts()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    barrier()
    elapsed = time.perf_counter() - t0
    c1 = comm_counts()
    if comm is None or not dp:
        comm_info = None            # single GPU: no transport, no all-reduce
    elif isinstance(comm, md2hip.comm.Comm):
        comm_info = {"transport": "md2_comm (RCCL, library-owned)", "nranks": comm.query()[1]}
    else:
        comm_info = {"transport": f"torch.distributed {comm.backend}", "nranks": comm.world}
    if comm_info is not None:
        comm_info["allreduce_calls_per_step"] = (c1[0] - c0[0]) / args.steps
        comm_info["allreduce_bytes_per_step"] = (c1[1] - c0[1]) / args.steps
        comm_info["grad_bytes"] = model.grad.numel() * model.grad.element_size()
    if dp:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev if args.comm == "torch" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    loss_val = loss_buf.item()

    prof = None
    if not args.no_probe:
        # the event brackets of ONE step are at the mercy of host jitter (a late launch leaves
        # its bracket open while the GPU idles) and the first profiled step also creates the
        # event pool; take each category's minimum over a few profiled steps
        ex.set_profiling(True)
        samples = []
        for _ in range(args.probe_steps):
            step()
            torch.cuda.synchronize()
            samples.append(ex.profile_read())
        ex.set_profiling(False)
        import statistics
        # per category: the median step (reported) and the fastest one (beside it)
        prof = {c: statistics.median_low([s_[c] for s_ in samples]) for c in samples[0]}
        prof_min = {c: min(s_[c] for s_ in samples) for c in samples[0]}

    if rank == 0:
        imgs = world * B * args.steps
        out = {
            "metric": METRIC,
            "value": round(imgs / elapsed, 3),
            "unit": "images/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "arithmetic": "fp32 tensors and sums; the 3x3 convs contract on the bf16 MFMA with every fp32 "
                          "operand split exactly into 3 bf16 terms and the 6 largest partial products "
                          "(bf16x6, error vs fp64 below the fp32-MFMA kernel's; DESIGN.md sec. 4)",
            "data": f"synthetic: uniform [0,1) RGB {W}x{H} triplets keyed by global sample index; "
                    "Flux-default random init (seed 42)",
            "config": {"workload": f"train_step resnet{args.arch} depth+pose decoders, 4-scale photometric loss, ADAM",
                       "batch_per_gpu": B, "global_batch": B * world, "height": H, "width": W,
                       "parallelism": f"dp{world}",
                       "allreduce": ("rccl md2_comm (bucketed, overlapped with backward)" if args.comm == "md2"
                                     else "rccl torch.distributed (bucketed, overlapped)") if dp else None},
            "comm": comm_info,
            "loss": loss_val,
            "loss_first_step": loss_first,   # == tests/golden/bench_first_loss.json (fp64 oracle) at B=12 416x128
        }
        if prof:
            ms, flop, n = prof["conv3x3_encoder"]
            ach = flop / (ms * 1e-3) / 1e12 if ms > 0 else 0.0
            ms_min = prof_min["conv3x3_encoder"][0]
            ach_min = flop / (ms_min * 1e-3) / 1e12 if ms_min > 0 else 0.0
            # the committed PMC profiles are of the default workload (ResNet-18, B=12, 416x128)
            default = (args.arch, B, H, W) == (18, 12, 128, 416)
            traffic, tsrc = pmc_traffic() if default else (None, None)
            busy, bsrc = pmc_mfma_busy() if default else (None, None)
            out["roofline"] = {"bound": "mfma", "kernel": "implicit-GEMM zero-padded 3x3 convs (encoder+pose): fwd+dgrad conv_halo3 (LDS halo, stride 1) / conv_px3 (stride 2), wgrad conv_whalo (LDS halo, layers 2-4 + pose) / conv_wgrad_px3 (bf16x6 split products, fp32 sums), + split-K / wgrad reduce",
                               "achieved": round(ach, 3), "peak": PEAK_FP32_MFMA_TFLOPS, "unit": "TFLOP/s",
                               "frac": round(ach / PEAK_FP32_MFMA_TFLOPS, 4), "traffic": traffic,
                               "peak_note": "peak = fp32 MFMA (the reference's arithmetic, algorithmic fp32 FLOPs); "
                                            f"the bf16x6 kernels issue 6 bf16 MFMAs per fp32 product: their own "
                                            f"ceiling is {PEAK_BF16X6_TFLOPS:.1f} TFLOP/s (frac_issued)",
                               "peak_issued": round(PEAK_BF16X6_TFLOPS, 1),
                               "frac_issued": round(ach / PEAK_BF16X6_TFLOPS, 4),
                               "mfma_busy": busy, "mfma_busy_source": bsrc,
                               "traffic_source": tsrc,
                               "launches": n, "algorithmic_flop_per_step": flop, "kernel_ms_per_step": round(ms, 4),
                               "probe": f"median of {args.probe_steps} profiled steps; fastest step "
                                        f"{ms_min:.4f} ms = frac {ach_min / PEAK_FP32_MFMA_TFLOPS:.4f}"}
            ms, byt, n = prof["photometric"]
            gbs = byt / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
            ptraffic, psrc, pnote = pmc_photo_traffic(B) if (H, W) == (128, 416) else (None, None, None)
            out["roofline_photometric"] = {"bound": "hbm", "kernel": "photo_stream_kernel (fused warp+SSIM+L1 fwd+bwd, all 4 scales in one launch)",
                                           "achieved": round(gbs, 2), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                                           "frac": round(gbs / PEAK_HBM_GBS, 4), "traffic": ptraffic,
                                           "traffic_source": psrc,
                                           "note": pnote,
                                           "launches": n, "algorithmic_bytes_per_step": byt,
                                           "kernel_ms_per_step": round(ms, 4),
                                           "probe": f"median of {args.probe_steps} profiled steps; fastest "
                                                    f"{prof_min['photometric'][0]:.4f} ms"}
            ms2, flop2, n2 = prof["conv_other"]
            out["conv_other"] = {"ms_per_step": round(ms2, 4), "tflops": round(flop2 / max(ms2, 1e-9) / 1e9, 3),
                                 "launches": n2}
        if world == 1 and not args.no_cpu_baseline:
            try:
                out["cpu_baseline"] = cpu_baseline(args, args.cpu_seconds)
            except Exception as e:  # pragma: no cover - report, never fake
                out["cpu_baseline"] = {"error": repr(e)}
        sys.stdout.flush()
        os.write(json_fd, (json.dumps(out) + "\n").encode())
    if dp:
        if args.comm == "md2":
            comm.close()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
