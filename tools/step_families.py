"""Per-step time by kernel family from a rocprofv3 --stats CSV (profiles/<tag>_kernel_stats.csv).

    python tools/step_families.py profiles/r02e_kernel_stats.csv [steps=13]
"""
import csv
import re
import sys

FAMILIES = [
    ("conv 3x3/1x1/7x7 implicit GEMM (fwd/dgrad/wgrad)", r"conv_(px|px2|px3|px16|wgrad|wgrad_tap|wgrad16|wgrad_stem|wgrad_px3|halo3|whalo)_kernel|fold_reflect"),
    ("split-K / wgrad reductions", r"(splitk_reduce|wgrad_reduce)"),
    ("BatchNorm (+ fused stem max pool)", r"bn_|maxpool"),
    ("disparity heads (Cout=1)", r"head_"),
    ("photometric (warp+SSIM fwd+bwd)", r"photo_stream"),
    ("loss tail rest (smooth, means, adjoint, finalize, so3)", r"(smooth|disp_sum|up_adjoint|loss_|so3_|pose_grad_reduce)"),
    ("decoder upsample / activations", r"(upsample2|act_bias|act_backward|axpy|concat)"),
    ("ADAM + weight repack", r"(adam|pack_)"),
    ("pose head / pairs", r"(pose_|pair_)"),
]


def main(path, steps=13):
    rows = list(csv.DictReader(open(path)))
    out = {name: 0.0 for name, _ in FAMILIES}
    other = 0.0
    others = []
    for r in rows:
        t = float(r["TotalDurationNs"]) / steps / 1e3
        for name, pat in FAMILIES:
            if re.search(pat, r["Name"]):
                out[name] += t
                break
        else:
            other += t
            others.append((t, r["Name"][:100], r["Calls"]))
    total = sum(out.values()) + other
    for name, v in sorted(out.items(), key=lambda x: -x[1]):
        print(f"{v:8.1f} us/step  {100 * v / total:5.1f}%  {name}")
    print(f"{other:8.1f} us/step  {100 * other / total:5.1f}%  other (runtime fills/copies, torch)")
    print(f"{total:8.1f} us/step  total")
    for t, n, c in sorted(others, reverse=True)[:8]:
        print(f"    other: {t:8.1f} us/step  calls {c:>6s}  {n}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 13)
