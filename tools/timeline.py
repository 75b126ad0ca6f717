"""Concurrency / gap analysis of a rocprofv3 kernel trace (md2 kernels): python tools/timeline.py trace.csv [steps]"""
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "md2::" in r["Kernel_Name"]]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"], r["Kernel_Name"]) for r in rows)
t0, t1 = iv[0][0], max(e for _, e, _, _ in iv)
busy, cur_s, cur_e = 0, None, None
for s, e, _, _ in iv:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
tot = sum(e - s for s, e, _, _ in iv)
queues = sorted(set(q for _, _, q, _ in iv))
print(f"span {(t1 - t0) / 1e6 / steps:.3f} ms/step  busy(union) {busy / 1e6 / steps:.3f}  sum {tot / 1e6 / steps:.3f}  "
      f"idle {(t1 - t0 - busy) / 1e6 / steps:.3f}  queues {queues}  kernels/step {len(iv) / steps:.0f}")
