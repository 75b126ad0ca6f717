#!/bin/bash
# timing-only variants of the s2d stem forward (MD2_STEM_DBG)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for d in 0 16 2 4 8 14; do
  MD2_TUNING=1 MD2_STEM_DBG=$d timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_stemdbg_$d -o run --output-format csv -- python3 $R/tools/conv_one.py stem fwd > /dev/null 2>&1 || exit 21
  python3 - $R/gpurun_out/prof_stemdbg_$d/run_kernel_stats.csv $d <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "stem" in r["Name"]:
        print(f"DBG={sys.argv[2]:3s} {r['Name'][:60]:60s} calls={r['Calls']} avg_us={float(r['AverageNs'])/1000:.1f} min_us={float(r['MinNs'])/1000:.1f}")
PY
done
