"""Per-kernel-family time of the train step with every kernel on the model stream (bench.py's
HIP-event probe steps: no side-stream overlap, so durations are the kernels' own) from a
rocprofv3 kernel trace of `bench.py --probe-steps P`: the last P steps (one photometric launch
each) are averaged.

    python tools/isolated_kernels.py run_kernel_trace.csv P [top]"""
import csv
import sys
from collections import defaultdict


def family(n):
    n = n.replace("void ", "").replace("md2::", "").replace("(anonymous namespace)::", "")
    return n.split("(")[0][:64]


def main():
    rows = sorted((r for r in csv.DictReader(open(sys.argv[1])) if "md2::" in r["Kernel_Name"]),
                  key=lambda r: int(r["Start_Timestamp"]))
    P = int(sys.argv[2])
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    photo = [i for i, r in enumerate(rows) if "photo" in r["Kernel_Name"]]
    # step s spans from the kernel after photo launch s-1's step start... take the window between
    # the (P+1)-th last photometric launch and the last one, shifted to whole steps: kernels from
    # the first encoder launch after photo[-P-1] up to photo[-1]'s step end (the next step's start
    # is not traced after the last probe step, so the tail runs to the end of the trace)
    a = photo[-P - 1]
    # the backward + ADAM of step -P-1 follow its photometric launch; skip to the next pack/adam
    i0 = a
    while i0 < len(rows) and "pack_batch" not in rows[i0]["Kernel_Name"]:
        i0 += 1
    win = rows[i0 + 1:]
    fam = defaultdict(lambda: [0.0, 0])
    for r in win:
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        k = family(r["Kernel_Name"])
        fam[k][0] += d
        fam[k][1] += 1
    tot = sum(v[0] for v in fam.values())
    span = int(win[-1]["End_Timestamp"]) - int(win[0]["Start_Timestamp"])
    print(f"{P} isolated steps: kernel sum {tot / 1e6 / P:.3f} ms/step, span {span / 1e6 / P:.3f} ms/step")
    for k, (t, c) in sorted(fam.items(), key=lambda kv: -kv[1][0])[:top]:
        print(f"  {t / 1e3 / P:8.1f} us/step  {c / P:5.1f}x  avg {t / 1e3 / c:7.1f}  {k}")


if __name__ == "__main__":
    main()
