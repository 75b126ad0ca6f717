"""Where the model stream waits (rocprofv3 kernel trace of bench.py): per queue busy time, and the
gaps on the busiest queue (the model stream) with the kernels around them -- a gap there is the
step waiting on the side stream or on the host.

    python tools/critical_path.py run_kernel_trace.csv STEPS [top]"""
import csv
import sys
from collections import defaultdict


def short(n):
    n = n.replace("void ", "").replace("md2::", "").replace("(anonymous namespace)::", "")
    return n.split("(")[0][:48]


def main():
    rows = [r for r in csv.DictReader(open(sys.argv[1])) if "md2::" in r["Kernel_Name"]]
    steps = int(sys.argv[2])
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 15
    byq = defaultdict(list)
    for r in rows:
        byq[r["Queue_Id"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    for q in byq:
        byq[q].sort()
    main_q = max(byq, key=lambda q: len(byq[q]))
    t0 = min(v[0][0] for v in byq.values())
    t1 = max(max(e for _, e, _ in v) for v in byq.values())
    print(f"span {(t1 - t0) / 1e6 / steps:.3f} ms/step over {steps} steps")
    for q, v in sorted(byq.items(), key=lambda kv: -len(kv[1])):
        busy = sum(e - s for s, e, _ in v)
        print(f"queue {q}{' (model)' if q == main_q else ''}: {len(v) / steps:.0f} kernels/step, "
              f"busy {busy / 1e6 / steps:.3f} ms/step")
    m = byq[main_q]
    gaps = defaultdict(lambda: [0, 0])
    tot = 0
    for (s0, e0, n0), (s1, e1, n1) in zip(m, m[1:]):
        g = s1 - e0
        if g > 2000:          # > 2 us
            k = (short(n0), short(n1))
            gaps[k][0] += g
            gaps[k][1] += 1
            tot += g
    print(f"model-stream gaps > 2 us: {tot / 1e6 / steps:.3f} ms/step")
    for (a, b), (g, c) in sorted(gaps.items(), key=lambda kv: -kv[1][0])[:top]:
        print(f"  {g / 1e3 / steps:8.1f} us/step  x{c / steps:.1f}  after {a}  before {b}")


if __name__ == "__main__":
    main()
