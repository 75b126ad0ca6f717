#!/bin/bash
# s2d stem kernels: conv parity, per-kernel time, step A/B
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_conv.py -k "k7" -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r06o_conv.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_r06o_conv.log; [ $rc -eq 0 ] || { grep -E "^E " gpurun_out/pytest_r06o_conv.log | head -20; exit $rc; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_stem_o -o run --output-format csv -- python3 $R/tools/bench_conv.py --only=stem > $R/gpurun_out/stem_o.txt 2>&1 || exit 21
grep stem $R/gpurun_out/stem_o.txt
python3 - $R/gpurun_out/prof_stem_o/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if any(k in r["Name"] for k in ("stem", "wgrad_reduce")):
        print(f"  {r['Name'][:70]:70s} calls={r['Calls']} avg_us={float(r['AverageNs'])/1000:.1f} min_us={float(r['MinNs'])/1000:.1f}")
PY
cd $R
for rep in 1 2; do
for v in 1 0; do
  MD2_TUNING=1 MD2_STEM_S2D=$v MD2_WSTEM_S2D=$v timeout -k 10 200 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/ab_r06o.json 2>/dev/null || exit 23
  python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_r06o.json')); print('MD2_STEM_S2D=%s %9.1f img/s  %.3f ms' % (sys.argv[1], d['value'], d['ms_per_step']))" "$v"
done; done
