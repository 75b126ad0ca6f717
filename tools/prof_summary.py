"""Condense a tools/profile_round.sh run into profiles/<tag>_*.

    python tools/prof_summary.py gpurun_out/prof_r01 r01

Writes
  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (verbatim)
  profiles/<tag>_bench.json         the bench line of the un-profiled run
  profiles/<tag>_summary.md         top kernels, per-step category times, the roofline cross-check
  profiles/<tag>_pmc.json           FETCH_SIZE / WRITE_SIZE per launch of the roofline kernels

Roofline kernel set (matches bench.py's HIP-event category 0): implicit-GEMM conv kernels with a
3x3 zero-padded filter (conv_px{,2,3}_kernel / conv_halo3_kernel / conv_wgrad_*kernel / conv_whalo_kernel
with KH=3, RFL=0) plus the split-K / wgrad reduction kernels dispatched right after each of them."""
import csv
import json
import os
import re
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def targs(name):
    m = re.search(r"<([^<>]*)>\(md2::ConvArgs\)", name)
    return [int(v) for v in m.group(1).split(",")] if m else None


def is_conv3(name):
    a = targs(name)
    if a is None:
        return False
    if "conv_px2_kernel" in name or "conv_px3_kernel" in name:   # <MODE, BM, BN, WM, WN, KH, KW, S, RFL, ...>
        return a[5] == 3 and a[8] == 0
    if "conv_px_kernel" in name:          # <MODE, TAP, BM, BN, BK, WM, WN, KH, KW, S, RFL>
        return a[7] == 3 and a[10] == 0
    if "conv_wgrad_stem_kernel" in name:   # <CIN>: the 7x7/2 stem
        return False
    if "conv_halo3_kernel" in name:        # <MODE, NT, ITEMS, DBG, RFL, EXT>: stride-1 3x3
        return (len(a) < 5 or a[4] == 0) and (len(a) < 6 or a[5] == 0)
    if "conv_halo3s2_kernel" in name:      # <ITEMS>: stride-2 3x3 data gradient
        return True
    if "conv_whalo_kernel" in name:        # <ITEMS, KS>: stride-1 3x3 zero-padded filter gradient
        return True
    if "conv_wgrad_px3_kernel" in name:    # <BM, BN, WM, WN, KH, KW, S, RFL, CW, NT>
        return a[4] == 3 and a[7] == 0
    if "conv_wgrad16_kernel" in name:      # <MT, KH, KW, RFL>
        return a[1] == 3 and a[3] == 0
    if "conv_wgrad" in name:               # <BM, BN, BK, WM, WN, KH, KW, S, RFL[, CW]>
        return a[5] == 3 and a[8] == 0
    return False


def is_reduce(name):
    return "splitk_reduce" in name or "wgrad_reduce" in name


def read_csv(path):
    with open(path, newline="") as f:
        return list(csv.DictReader(f))


def short(name, n=90):
    name = name.replace("void ", "").replace("md2::", "")
    return name if len(name) <= n else name[:n - 3] + "..."


def conv3_groups(trace):
    """[(main kernel row, [reduce rows])] for the roofline kernel set, in dispatch order."""
    rows = sorted(trace, key=lambda r: int(r["Dispatch_Id"]))
    out, cur = [], None
    for r in rows:
        nm = r["Kernel_Name"]
        if is_conv3(nm):
            cur = (r, [])
            out.append(cur)
        elif is_reduce(nm) and cur is not None:
            cur[1].append(r)
        else:
            cur = None
    return out


def dur(r):
    return int(r["End_Timestamp"]) - int(r["Start_Timestamp"])


def conv3_family(name):
    """fwd / dgrad / wgrad and kernel of a roofline-set launch (None outside the set)."""
    if not is_conv3(name):
        return None
    a = targs(name)
    if "conv_halo3s2_kernel" in name:
        return "dgrad halo3s2 (stride 2)"
    if "conv_halo3_kernel" in name:
        return ("fwd" if a[0] == 0 else "dgrad") + " halo3"
    if "conv_whalo_kernel" in name:
        return "wgrad whalo"
    if "conv_px3_kernel" in name or "conv_px2_kernel" in name:
        return ("fwd" if a[0] == 0 else "dgrad") + " px3 (stride 2)"
    return "wgrad px3"


def mfma_busy(path):
    """MFMA pipe busy fraction of the roofline set per family, from one --pmc pass of
    SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE: busy / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs)
    summed over the family's dispatches (tools/pmc_report.py's formula)."""
    if not os.path.exists(path):
        return None
    per = defaultdict(lambda: defaultdict(float))
    names = {}
    for r in read_csv(path):
        i = int(r["Dispatch_Id"])
        per[i][r["Counter_Name"]] += float(r["Counter_Value"])
        names[i] = r["Kernel_Name"]
    fam = defaultdict(lambda: [0.0, 0.0, 0.0, 0])
    for i, c in per.items():
        f = conv3_family(names[i])
        if f is None or "GRBM_GUI_ACTIVE" not in c:
            continue
        for key in (f, "set"):
            fam[key][0] += c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
            fam[key][1] += c["GRBM_GUI_ACTIVE"] / 8 * 1024
            fam[key][2] += c.get("SQ_INSTS_MFMA", 0.0)
            fam[key][3] += 1
    return {k: {"busy": round(v[0] / v[1], 4) if v[1] else None, "mfma_insts": v[2], "dispatches": v[3]}
            for k, v in sorted(fam.items())}


def main(src, tag):
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    stats = os.path.join(src, "trace", "run_kernel_stats.csv")
    shutil.copy(stats, os.path.join(prof, f"{tag}_kernel_stats.csv"))
    bench = None
    with open(os.path.join(src, "bench_plain.json")) as f:
        for line in f:
            if line.startswith("{"):
                bench = json.loads(line)
    with open(os.path.join(prof, f"{tag}_bench.json"), "w") as f:
        json.dump(bench, f, indent=1)
    with open(os.path.join(src, "bench_trace.json")) as f:
        traced = [json.loads(l) for l in f if l.startswith("{")][0]
    steps_traced = traced["steps"] + traced["warmup"]       # --no-probe: no extra step

    st = read_csv(stats)
    total_ns = sum(float(r["TotalDurationNs"]) for r in st)
    trace = read_csv(os.path.join(src, "trace", "run_kernel_trace.csv"))
    groups = conv3_groups(trace)
    g_main = sum(dur(m) for m, _ in groups)
    g_all = sum(dur(m) + sum(dur(r) for r in rs) for m, rs in groups)
    per_step_ms = g_all / steps_traced / 1e6
    md2_ns = sum(dur(r) for r in trace if "md2::" in r["Kernel_Name"])

    # PMC: sum per dispatch over the roofline set (counters are per dispatch rows)
    pmc = {}
    for cname, sub in (("FETCH_SIZE", "fetch"), ("WRITE_SIZE", "write")):
        path = os.path.join(src, sub, "run_counter_collection.csv")
        if not os.path.exists(path):
            continue
        rows = read_csv(path)
        per_disp = defaultdict(float)
        names = {}
        for r in rows:
            if r["Counter_Name"] == cname:
                per_disp[int(r["Dispatch_Id"])] += float(r["Counter_Value"])
                names[int(r["Dispatch_Id"])] = r["Kernel_Name"]
        ids = sorted(per_disp)
        tot, n_main, cur = 0.0, 0, False
        for i in ids:
            nm = names[i]
            if is_conv3(nm):
                tot += per_disp[i]
                n_main += 1
                cur = True
            elif is_reduce(nm) and cur:
                tot += per_disp[i]
            else:
                cur = False
        pmc[cname] = {"kib_total": tot, "launches": n_main}
    traffic = None
    if "FETCH_SIZE" in pmc and "WRITE_SIZE" in pmc and pmc["FETCH_SIZE"]["launches"]:
        n = pmc["FETCH_SIZE"]["launches"]
        fetch_b = pmc["FETCH_SIZE"]["kib_total"] * 1024 / n * 2     # gfx950: FETCH_SIZE = 1/2 of bytes
        write_b = pmc["WRITE_SIZE"]["kib_total"] * 1024 / n
        traffic = {"bytes_per_launch": fetch_b + write_b, "fetch_bytes_per_launch_x2": fetch_b,
                   "write_bytes_per_launch": write_b, "launches": n,
                   "note": "FETCH_SIZE doubled per MI355X_MICROARCH.md (gfx950 reports 1/2 of wide-read "
                           "bytes); these kernels mix 4-B gathers and 16-B loads, so the absolute is "
                           "uncalibrated; ratios between rounds are exact"}
    mfma = mfma_busy(os.path.join(src, "mfma", "run_counter_collection.csv"))
    with open(os.path.join(prof, f"{tag}_pmc.json"), "w") as f:
        json.dump({"counters": pmc, "traffic": traffic, "mfma_busy": mfma}, f, indent=1)

    lines = [f"# Profile {tag}: bench.py on 1x MI355X (rocprofv3 --kernel-trace --stats)", ""]
    if bench:
        lines += [f"Un-profiled bench: **{bench['value']} {bench['unit']}**, {bench['ms_per_step']} ms/step "
                  f"(B={bench['config']['batch_per_gpu']}, {bench['config']['width']}x{bench['config']['height']}).", ""]
    lines += [f"Traced run: {steps_traced} steps (incl. warm-up); md2 kernels {md2_ns / steps_traced / 1e6:.3f} ms/step, "
              f"all kernels {total_ns / steps_traced / 1e6:.3f} ms/step.", ""]
    lines += ["## Roofline kernel set (zero-padded 3x3 implicit-GEMM convs + their split-K reductions)", "",
              f"- rocprof: {len(groups) / steps_traced:.0f} launches/step, main kernels "
              f"{g_main / steps_traced / 1e6:.3f} ms/step, with reductions **{per_step_ms:.3f} ms/step**"]
    if bench and "roofline" in bench:
        rf = bench["roofline"]
        lines += [f"- bench HIP events (same set, event-to-event on the model stream): "
                  f"**{rf['kernel_ms_per_step']} ms/step**, {rf['launches']} launches -> "
                  f"{rf['achieved']} TFLOP/s = {rf['frac'] * 100:.1f}% of {rf['peak']} TFLOP/s fp32 MFMA"]
        lines += [f"- agreement: rocprof / events = {per_step_ms / rf['kernel_ms_per_step']:.3f} "
                  "(events also include the launch gaps inside each bracket)"]
    if traffic:
        lines += [f"- HBM traffic per launch (PMC, separate passes): {traffic['bytes_per_launch'] / 1e6:.2f} MB "
                  f"(fetch x2 {traffic['fetch_bytes_per_launch_x2'] / 1e6:.2f} MB + write "
                  f"{traffic['write_bytes_per_launch'] / 1e6:.2f} MB)"]
    lines += ["", "## Top kernels (whole traced run)", "", "| kernel | calls | total ms | avg us | % |", "|---|---|---|---|---|"]
    for r in sorted(st, key=lambda r: -float(r["TotalDurationNs"]))[:25]:
        lines.append(f"| `{short(r['Name'])}` | {r['Calls']} | {float(r['TotalDurationNs']) / 1e6:.2f} | "
                     f"{float(r['AverageNs']) / 1e3:.1f} | {float(r['Percentage']):.1f} |")
    with open(os.path.join(prof, f"{tag}_summary.md"), "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines[:14]))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "r01")
