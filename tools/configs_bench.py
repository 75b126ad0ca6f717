"""Measure BASELINE.json configs 1 and 2 on one MI355X (bench.py measures config 3; config 5
per GPU is ``bench.py --arch 50 --width 640 --height 192 --batch 8``):

  config 1  slow_depth (src/simple_depth.jl): one 416x128 triplet, ADAM(3e-4) on disparity +
            poses -- GPU ms/iteration, and the fp32 torch-CPU restatement timed on the host
            cores for a few iterations (the reference is CPU Flux/Zygote; baseline only);
  config 2  eval_disparity (src/model.jl:63): ResNet-18 + DepthDecoder forward, B=12 -- images/s.

Prints one JSON line per config.  usage: python tools/configs_bench.py [--cpu-iters N]
"""
import argparse
import json
import os
import sys
import time

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
sys.path.insert(0, os.path.join(R, "monodepth2.jl_amd"))
import torch  # noqa: E402

import md2hip  # noqa: E402
from tests import _data as D  # noqa: E402


def timed(fn, iters, warmup=3):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def config1(cpu_iters):
    W, H = 416, 128
    x = D.triplets(1, 3, H, W, seed=7).float()
    K, invK = D.intrinsics(W, H)
    sd = md2hip.SlowDepth(x.cuda(), K.numpy(), invK.numpy())
    ms = timed(sd.step, 100)
    out = {"config": "1: slow_depth 416x128 single triplet, ADAM(3e-4)", "gpu_ms_per_iter": round(ms, 4),
           "gpu_s_500_iters": round(ms * 0.5, 4)}
    if cpu_iters > 0:
        from oracle import md2_oracle as O
        # the box's CPU share is 16 cores (os.cpu_count() reports the whole host)
        torch.set_num_threads(min(16, int(os.environ.get("OMP_NUM_THREADS", "16")), os.cpu_count() or 1))
        disp, rv, tv = O.slow_depth_init(W, H, dtype=torch.float32)
        Kf, iKf = K.float(), invK.float()
        opt = O.Adam(eta=3e-4)
        t0 = time.perf_counter()
        for _ in range(cpu_iters):
            disp.requires_grad_(True)
            for t in rv + tv:
                t.requires_grad_(True)
            loss = O.slow_depth_loss(disp, rv, tv, x, Kf, iKf)
            loss.backward()
            with torch.no_grad():
                opt.step("d", disp, disp.grad)
                for k, t in enumerate(rv + tv):
                    opt.step(k, t, t.grad)
            disp = disp.detach()
            rv = [t.detach() for t in rv]
            tv = [t.detach() for t in tv]
        cpu_ms = (time.perf_counter() - t0) / cpu_iters * 1e3
        out.update({"cpu_ms_per_iter": round(cpu_ms, 2), "cpu_threads": torch.get_num_threads(),
                    "cpu_kind": "port (fp32 torch restatement, oracle/md2_oracle.py)",
                    "gpu_vs_cpu": round(cpu_ms / ms, 1)})
    print(json.dumps(out))


def config2():
    W, H, N = 416, 128, 12
    enc = md2hip.ResNet(18, in_channels=3)
    m = md2hip.Model(enc, md2hip.DepthDecoder(encoder_channels=enc.stages, scale_levels=[2, 3, 4, 5],
                                              embedding_levels=0), md2hip.PoseDecoder(512))
    x = torch.rand(N, 3, H, W, device="cuda")
    ms = timed(lambda: md2hip.eval_disparity(m, x), 50)
    print(json.dumps({"config": "2: eval_disparity ResNet-18 + DepthDecoder forward, 416x128 B=12",
                      "ms_per_batch": round(ms, 4), "images_per_s": round(N / ms * 1e3, 1)}))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--cpu-iters", type=int, default=3)
    a = ap.parse_args()
    config1(a.cpu_iters)
    config2()
