"""Per-shape median durations of the conv_halo3 / conv_px3 kernels in a rocprofv3 kernel trace
(tools/bench_conv.py under rocprofv3):  python tools/halo_shapes.py DIR [DIR ...]"""
import collections
import csv
import sys

for d in sys.argv[1:]:
    rows = list(csv.DictReader(open(f"{d}/run_kernel_trace.csv")))
    t = collections.defaultdict(list)
    for r in rows:
        n = r["Kernel_Name"]
        if "halo3" in n or "conv_px3_kernel" in n:
            key = (n.split("(")[0].replace("void md2::", "")[-36:], r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"])
            t[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
    print("==", d)
    for k, v in t.items():
        v = sorted(v)
        print(f"  {k[0]:38s} grid {k[1]:>7s} x {k[2]:>2s} x {k[3]:>2s}  n={len(v):3d}  median {v[len(v) // 2]:7.1f} us  min {v[0]:7.1f}")
