#!/bin/bash
# Loss-tail kernel timings per setting (kernel trace of tools/photo_one.py N 10): one block per
# library variant (VARIANTS="name ..." under lib_var/) and per environment setting
# (CONFIGS="ENV1=a ENV2=b;ENV1=c", run with MD2_TUNING=1).  Usage: tools/ab_photo.sh [N]
set -uo pipefail
R=$GRAFT_REPO_ROOT
N=${1:-12}
cd /tmp && export TMPDIR=/tmp
summ() {
  python3 - "$1" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if any(k in n for k in ("photo", "smooth_kernel", "up_adjoint", "disp_sum")):
        print(f"{n[:60]:60s} calls={r['Calls']} avg_us={float(r['AverageNs'])/1000:.1f}")
PY
}
for v in base ${VARIANTS:-}; do
  lib=$R/monodepth2.jl_amd/lib/libmd2hip.so
  [ "$v" != base ] && lib=$R/lib_var/$v/libmd2hip.so
  MD2HIP_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/abp_$v -o run --output-format csv -- python3 $R/tools/photo_one.py $N 10 > /dev/null 2>&1 || { echo "variant $v failed"; exit 1; }
  echo "== $v"
  summ /tmp/abp_$v/run_kernel_stats.csv
done
IFS=';' read -ra CFG <<< "${CONFIGS:-}"
i=0
for c in "${CFG[@]}"; do
  i=$((i + 1))
  env MD2_TUNING=1 $c timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/abc_$i -o run --output-format csv -- python3 $R/tools/photo_one.py $N 10 > /dev/null 2>&1 || { echo "config '$c' failed"; exit 1; }
  echo "== $c"
  summ /tmp/abc_$i/run_kernel_stats.csv
done
