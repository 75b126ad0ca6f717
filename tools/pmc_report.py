"""Average per-dispatch PMC values per md2 kernel from tools/pmc_conv.sh output dirs."""
import csv, glob, sys
from collections import defaultdict
root = sys.argv[1]
vals = defaultdict(lambda: defaultdict(list))
for f in glob.glob(f"{root}/*/run_counter_collection.csv"):
    per = defaultdict(lambda: defaultdict(float))
    names = {}
    for r in csv.DictReader(open(f)):
        if "md2::" not in r["Kernel_Name"]:
            continue
        d = int(r["Dispatch_Id"])
        per[d][r["Counter_Name"]] += float(r["Counter_Value"])
        names[d] = r["Kernel_Name"].replace("void md2::", "")[:70]
    for d, cs in per.items():
        for c, v in cs.items():
            vals[names[d]][c].append(v)
for k, cs in vals.items():
    print("==", k)
    avg = {c: sum(v) / len(v) for c, v in cs.items()}
    for c in sorted(avg):
        print(f"   {c:28s} {avg[c]:14.0f}")
    if "SQ_WAVE_CYCLES" in avg:
        w = avg["SQ_WAVE_CYCLES"]
        print(f"   wait_any {avg['SQ_WAIT_ANY']/w:.2f} wait_inst {avg['SQ_WAIT_INST_ANY']/w:.2f} active {avg['SQ_ACTIVE_INST_ANY']/w:.2f}")
    if "SQ_VALU_MFMA_BUSY_CYCLES" in avg and "GRBM_GUI_ACTIVE" in avg:
        print(f"   MFMA util {avg['SQ_VALU_MFMA_BUSY_CYCLES'] / (avg['GRBM_GUI_ACTIVE'] / 8 * 1024):.3f}")
