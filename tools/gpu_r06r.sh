#!/bin/bash
# stem filter gradient: 1 vs 2 M tiles per wave (MD2_WSTEM_MV), parity + kernel time
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_conv.py -k "k7" -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r06r_conv.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_r06r_conv.log; [ $rc -eq 0 ] || { grep -E "^E " gpurun_out/pytest_r06r_conv.log | head -20; exit $rc; }
cd /tmp && export TMPDIR=/tmp
for mv in 2 1 2 1; do
  MD2_TUNING=1 MD2_WSTEM_MV=$mv timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_wstem_$mv -o run --output-format csv -- python3 $R/tools/conv_one.py stem wgrad > /dev/null 2>&1 || exit 21
  python3 - $R/gpurun_out/prof_wstem_$mv/run_kernel_stats.csv $mv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "stem" in r["Name"]:
        print(f"MV={sys.argv[2]} {r['Name'][:60]:60s} calls={r['Calls']} avg_us={float(r['AverageNs'])/1000:.1f} min_us={float(r['MinNs'])/1000:.1f}")
PY
done
cd $R
timeout -k 10 200 python3 -u tools/layer_table.py r06 > gpurun_out/layers_r06.txt 2>&1 || exit 24
cp profiles/r06_layers.md gpurun_out/ 2>/dev/null
for rep in 1 2; do
for mv in 2 1; do
  MD2_TUNING=1 MD2_WSTEM_MV=$mv timeout -k 10 200 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/ab_r06r.json 2>/dev/null || exit 23
  python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_r06r.json')); print('MD2_WSTEM_MV=%s %9.1f img/s  %.3f ms' % (sys.argv[1], d['value'], d['ms_per_step']))" "$mv"
done; done
