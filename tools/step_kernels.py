"""Per-step kernel list from a rocprofv3 kernel trace: the launches between the last two ADAM
kernels (one full train step), optionally filtered by a substring, plus a by-name summary.
usage: python tools/step_kernels.py <run_kernel_trace.csv> [filter] [--top N]"""
import collections
import csv
import re
import sys


def main():
    path = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else None
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 40
    rows = list(csv.DictReader(open(path)))
    idx = [i for i, r in enumerate(rows) if "adam_kernel" in r["Kernel_Name"]]
    a, b = idx[-2], idx[-1]
    step = rows[a + 1:b + 1]
    tot = 0.0
    agg = collections.defaultdict(lambda: [0.0, 0])
    for r in step:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
        tot += d
        name = re.sub(r"\(.*", "", r["Kernel_Name"])
        key = re.sub(r"^void ", "", name)[:100]
        agg[key][0] += d
        agg[key][1] += 1
        if filt and filt in name:
            print(f"{d:8.1f} {key} grid={r['Grid_Size_X']}x{r['Grid_Size_Y']}x{r['Grid_Size_Z']}")
    print(f"step kernel time {tot:.1f} us, {len(step)} launches, span "
          f"{(int(step[-1]['End_Timestamp']) - int(step[0]['Start_Timestamp'])) / 1000:.1f} us")
    for k, (t, n) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:top]:
        print(f"{t:8.1f} {n:4d}  {k}")


if __name__ == "__main__":
    main()
