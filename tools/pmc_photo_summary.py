"""Condense tools/pmc_photo.sh output into profiles/<tag>_pmc_photo.json.

    python tools/pmc_photo_summary.py gpurun_out/pmc_photo_<tag> <tag> [scales_per_launch]

Per batch size N (tools/photo_one.py N: the loss tail at 416x128, 4 scales): the photometric
kernel's average duration (kernel trace), PMC counters per launch (one pass per counter group),
HBM traffic (FETCH_SIZE doubled per the gfx950 note of MI355X_MICROARCH.md, WRITE_SIZE as read;
both uncalibrated for 4-byte gathers/stores), the algorithmic bytes (44 B per
full-resolution pixel and scale) and the VALU issue utilisation."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEY = "photo"
W, H, C, NSCALES = 416, 128, 3, 4
VALU_CYCLES = 4           # wave64 f32 VALU issue on gfx950, measured (tools/micro/valu_rate.hip, profiles/r04_valu_rate.txt)
SIMDS = 256 * 4


def counters(d):
    per = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(os.path.join(d, "*", "run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if KEY not in r["Kernel_Name"] or "md2::" not in r["Kernel_Name"]:
                continue
            per[(f, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    agg = defaultdict(list)
    for cs in per.values():
        for c, v in cs.items():
            agg[c].append(v)
    return {c: sum(v) / len(v) for c, v in agg.items()}


def main():
    src, tag = sys.argv[1], sys.argv[2]
    per_launch = int(sys.argv[3]) if len(sys.argv) > 3 else NSCALES   # r01 kernel: 1 scale a launch
    out = {"scales_per_launch": per_launch, "source": "tools/pmc_photo.sh + tools/photo_one.py (loss tail, 416x128, 4 scales, textured synthetic triplets)",
           "units": "per launch", "by_batch": {}}
    for nd in sorted(glob.glob(os.path.join(src, "*")), key=lambda p: int(os.path.basename(p))):
        N = int(os.path.basename(nd))
        stats = list(csv.DictReader(open(os.path.join(nd, "trace", "run_kernel_stats.csv"))))
        row = [r for r in stats if KEY in r["Name"] and "md2::" in r["Name"]][0]
        avg_us = float(row["AverageNs"]) / 1e3
        c = counters(nd)
        alg = per_launch * N * H * W * (8 + 12 * C)
        fetch = 2 * c["FETCH_SIZE"] * 1024
        write = c["WRITE_SIZE"] * 1024
        valu = c["SQ_INSTS_VALU"]
        out["by_batch"][str(N)] = {
            "kernel": row["Name"][:80], "avg_us": round(avg_us, 2),
            "algorithmic_bytes": alg, "algorithmic_GBps": round(alg / (avg_us * 1e-6) / 1e9, 1),
            "hbm_fetch_bytes_x2": round(fetch), "hbm_write_bytes": round(write),
            "traffic_bytes": round(fetch + write),
            "valu_insts": valu, "valu_insts_per_pixel_scale": round(valu * 64 / (per_launch * N * H * W), 1),
            "valu_issue_utilisation": round(valu * VALU_CYCLES / SIMDS / (avg_us * 1e-6 * 2.4e9), 3),
            "waves": c.get("SQ_WAVES"), "wave_cycles_quad": c.get("SQ_WAVE_CYCLES"),
            "wait_any": round(c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"], 3),
            "wait_inst_any": round(c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"], 3),
            "active_inst_any": round(c["SQ_ACTIVE_INST_ANY"] / c["SQ_WAVE_CYCLES"], 3),
            "lds_bank_conflict_cycles": c.get("SQ_LDS_BANK_CONFLICT"),
            "counters": {k: round(v) for k, v in sorted(c.items())}}
    o = os.path.join(ROOT, "profiles", f"{tag}_pmc_photo.json")
    with open(o, "w") as f:
        json.dump(out, f, indent=1)
    for N, v in out["by_batch"].items():
        print(N, {k: v[k] for k in ("avg_us", "algorithmic_GBps", "traffic_bytes", "algorithmic_bytes",
                                  "valu_insts_per_pixel_scale", "valu_issue_utilisation")})
    print("wrote", o)


if __name__ == "__main__":
    main()
