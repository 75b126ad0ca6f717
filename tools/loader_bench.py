"""Host data-pipeline throughput: decoded triplets/s of the
DataLoader for Depth10k (+FlipX; src/dtk.jl:29-46) and KittyDataset (imresize 1241x376 ->
416x128; src/kitty.jl:45-61) on synthetic PNGs written here (natural-image-like content: a smooth
random field plus 8 % pixel noise, 8-bit), host-only and into the GPU (N0f8 bytes over PCIe +
md2_unorm8_to_float, and the float path for comparison).  Compared with the train step's
images/s (bench.py), which the loader must exceed to keep the GPU fed.
    python tools/loader_bench.py [OUT.json] [workers ...]"""
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monodepth2.jl_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from PIL import Image  # noqa: E402

import md2hip  # noqa: E402


def natural(rng, h, w, c):
    lo = rng.random((max(2, h // 16), max(2, w // 16), c))
    img = np.asarray(Image.fromarray((lo * 255).astype(np.uint8).squeeze()).resize((w, h), Image.BICUBIC),
                     dtype=np.float64) / 255.0
    img = img.reshape(h, w, c) if c > 1 else img.reshape(h, w)
    img = 0.92 * img + 0.08 * rng.random(img.shape)
    return (img.clip(0, 1) * 255).round().astype(np.uint8)


def rate(loader, batches):
    it = iter(loader)
    x = next(it)                       # warm-up batch (thread pool start)
    if x.is_cuda:
        torch.cuda.synchronize()
    t, n = time.perf_counter(), 0
    for x in it:
        n += x.shape[0]
        if n >= batches * x.shape[0]:
            break
    if x.is_cuda:
        torch.cuda.synchronize()
    return n / (time.perf_counter() - t)


def main():
    out_path = sys.argv[1] if len(sys.argv) > 1 else None
    workers = [int(v) for v in sys.argv[2:]] or [8, 16]
    rng = np.random.default_rng(0)
    B = 12
    res = {"batch": B, "cpu_quota": os.environ.get("OMP_NUM_THREADS"), "results": []}
    with tempfile.TemporaryDirectory() as d:
        files = []
        for i in range(240):
            Image.fromarray(natural(rng, 128, 3 * 416, 3), mode="RGB").save(os.path.join(d, f"{i}.png"))
            files.append(f"{i}.png")
        kd = os.path.join(d, "kitti", "sequences", "00")
        os.makedirs(os.path.join(kd, "image_0"))
        with open(os.path.join(kd, "calib.txt"), "w") as f:
            f.write("P0: 7.188560e+02 0 6.071928e+02 0 0 7.188560e+02 1.852157e+02 0 0 0 1 0\n")
        for i in range(3 * 120):
            Image.fromarray(natural(rng, 376, 1241, 1), mode="L").save(os.path.join(kd, "image_0", "%06d.png" % i))
        sets = {"Depth10k+FlipX": md2hip.Depth10k(d, files, augmentations=md2hip.FlipX(0.5)),
                "KittyDataset(imresize)": md2hip.KittyDataset(os.path.join(d, "kitti"), "00", target_size=(128, 416))}
        for name, ds in sets.items():
            nb = len(ds) // B - 1
            for w in workers:
                row = {"dataset": name, "workers": w}
                row["host_triplets_per_s"] = rate(md2hip.DataLoader(ds, B, workers=w, seed=1), nb)
                if torch.cuda.is_available():
                    row["gpu_bytes_triplets_per_s"] = rate(md2hip.DataLoader(ds, B, workers=w, seed=1, device="cuda"), nb)
                    row["gpu_float_triplets_per_s"] = rate(md2hip.DataLoader(ds, B, workers=w, seed=1, device="cuda",
                                                                             bytes_h2d=False), nb)
                print(json.dumps(row), flush=True)
                res["results"].append(row)
    if out_path:
        with open(out_path, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
