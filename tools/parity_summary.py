"""Condense the check_step parity records of a -m gpu run (gpurun_out/parity/*.json, written by
tests/_model_parity.py before it asserts) into one committed file: per record the loss / forward
errors and the 8 tensors closest to their bounds, with the worst ratios to bound and ceiling.
    python tools/parity_summary.py [PARITY_DIR] OUT.json [full-record label -> OUT_full.json]"""
import glob
import json
import os
import sys

src = sys.argv[1] if len(sys.argv) > 2 else "gpurun_out/parity"
out = sys.argv[2] if len(sys.argv) > 2 else sys.argv[1]
if len(sys.argv) < 2 or os.path.isfile(src) or os.path.exists(out) or not os.path.isdir(src):
    # the output must be a NEW file: a committed record passed as the only argument would
    # otherwise be overwritten by the summary of gpurun_out/parity
    sys.exit(f"usage: parity_summary.py [PARITY_DIR] NEW_OUT.json  (refusing: src={src!r}, out={out!r} "
             "exists or src is not a directory)")
recs = {}
for f in sorted(glob.glob(os.path.join(src, "*.json"))):
    d = json.load(open(f))
    t = d.get("tensors")
    if not t:                                   # non-check_step records (e.g. a trajectory) verbatim
        recs[os.path.basename(f)] = d
        continue
    rb = {k: v["bwd_err"] / v["bwd_bound"] for k, v in t.items()}
    rc = {k: v["bwd_err"] / v["bwd_ceiling"] for k, v in t.items()}
    eb = {k: v["e2e_err"] / v["e2e_bound"] for k, v in t.items()}
    ef = {k: v["e2e_err"] / max(v["floor"], 1e-30) for k, v in t.items()}
    worst = sorted(t, key=lambda k: -max(rb[k], eb[k]))[:8]
    fwd = d.get("forward", {})
    recs[d["label"]] = {"loss_rel_err": d["loss_rel_err"], "pose_rel_err": d["pose_rel_err"],
                        "disp_rel_err": d["disp_rel_err"], "disp_floor": d.get("disp_floor"),
                        "forward_over_bound_max": max((v["err"] / v["bound"] for v in fwd.values()), default=None),
                        "worst_bwd": d["worst_bwd"], "worst_e2e": d["worst_e2e"],
                        "max_bwd_err": max(v["bwd_err"] for v in t.values()),
                        "max_bwd_over_bound": max(rb.values()), "max_bwd_over_ceiling": max(rc.values()),
                        "max_e2e_over_bound": max(eb.values()), "max_e2e_over_fp32_floor": max(ef.values()),
                        "tensors_worst8": {k: t[k] for k in worst}, "n_tensors": len(t)}
ok = all(r.get("max_bwd_over_ceiling", 0) < 1 and r.get("max_bwd_over_bound", 0) < 1 and
         r.get("max_e2e_over_bound", 0) < 1 and (r.get("forward_over_bound_max") or 0) < 1
         for r in recs.values())
first = next((json.load(open(f)) for f in sorted(glob.glob(os.path.join(src, "*.json"))) if "bounds" in json.load(open(f))), {})
json.dump({"source": "tests/_model_parity.py check_step records (gpurun_out/parity/*.json) of a -m gpu run on MI355X",
           "bounds": first.get("bounds"),
           "all_within_bounds": ok,
           "note": "per record: the 8 tensors closest to their bounds; ratios < 1 pass; end to end bound = "
                   "max(1e-3, 4 x the fp32 floor = max over 4 independent fp32 evaluations)",
           "records": recs}, open(out, "w"), indent=1)
print(out, "records", len(recs), "all within bounds:", ok)
