#!/bin/bash
# timing-only variants of the s2d stem filter gradient (MD2_WSTEM_DBG)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for d in 0 1 2 4 6 7 15; do
  MD2_TUNING=1 MD2_WSTEM_DBG=$d timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_wsdbg_$d -o run --output-format csv -- python3 $R/tools/conv_one.py stem wgrad > /dev/null 2>&1 || exit 21
  python3 - $R/gpurun_out/prof_wsdbg_$d/run_kernel_stats.csv $d <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "stem" in r["Name"]:
        print(f"DBG={sys.argv[2]:3s} {r['Name'][:60]:60s} avg_us={float(r['AverageNs'])/1000:.1f} min_us={float(r['MinNs'])/1000:.1f}")
PY
done
