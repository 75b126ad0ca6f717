#!/bin/bash
# Counters + kernel times of the photometric kernel, scalar (MD2_PHOTO_V1=1) vs packed, at B=12
# (tools/photo_one.py).  Output: gpurun_out/pmc_photo_ab/<v>/{trace,a,b}; summary on stdout.
set -uo pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
P="$R/tools/photo_one.py 12 6"
for v in 1 0 1 0; do
  OUT=$R/gpurun_out/pmc_photo_ab/v$v
  mkdir -p "$OUT"
  MD2_PHOTO_V1=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 $P > /dev/null 2>&1 || exit 1
  python3 - "$OUT/trace/run_kernel_stats.csv" "$v" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "photo" in r["Name"]:
        print(f"V1={sys.argv[2]} {r['Name'][:40]} avg_us={float(r['AverageNs'])/1000:.1f} min_us={float(r['MinNs'])/1000:.1f}")
PY
done
for v in 1 0; do
  OUT=$R/gpurun_out/pmc_photo_ab/v$v
  MD2_PHOTO_V1=$v timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU -d "$OUT/a" -o run --output-format csv -- python3 $P > /dev/null 2>&1 || exit 1
  MD2_PHOTO_V1=$v timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE -d "$OUT/b" -o run --output-format csv -- python3 $P > /dev/null 2>&1 || exit 1
  echo "=== V1=$v"
  python3 $R/tools/pmc_report.py $OUT | grep -A 30 "photo" | head -32
done
