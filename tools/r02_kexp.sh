#!/bin/bash
# Kernel experiment check: GPU tests + bench, then a kernel trace of the bench whose per-kernel
# averages are compared with profiles/r02f_kernel_stats.csv (kernels matching $1).
set -o pipefail
PAT=${1:-upsample}
PROFILE=0 bash tools/r02_check.sh || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_kexp -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-probe > /dev/null 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python3 - "$PAT" <<'PY'
import csv, sys
a = {r['Name']: float(r['AverageNs']) for r in csv.DictReader(open('profiles/r02f_kernel_stats.csv'))}
for r in csv.DictReader(open('gpurun_out/prof_kexp/run_kernel_stats.csv')):
    if sys.argv[1] in r['Name']:
        print(f"{a.get(r['Name'], 0) / 1e3:7.1f} -> {float(r['AverageNs']) / 1e3:7.1f} us  {r['Name'][:90]}")
PY
