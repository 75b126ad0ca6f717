#!/bin/bash
# loss-tail kernel timings per library variant (kernel trace of tools/photo_one.py)
set -uo pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for v in base ${VARIANTS:-}; do
  lib=$R/monodepth2.jl_amd/lib/libmd2hip.so
  [ "$v" != base ] && lib=$R/lib_var/$v/libmd2hip.so
  MD2HIP_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/abp_$v -o run --output-format csv -- python3 $R/tools/photo_one.py 12 10 > /dev/null 2>&1 || { echo "variant $v failed"; exit 1; }
  echo "== $v"
  python3 - /tmp/abp_$v/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if any(k in n for k in ("photo", "smooth_kernel", "up_adjoint", "disp_sum")):
        print(f"{n[:60]:60s} calls={r['Calls']} avg_us={float(r['AverageNs'])/1000:.1f}")
PY
done
