#!/bin/bash
# stem filter gradient with the K-steps split between a filter quarter's two waves: stem conv
# tests, rocprof timing vs the tile-split kernel (variant library), interleaved bench pairs
set -o pipefail
R=$GRAFT_REPO_ROOT
V=$R/monodepth2.jl_amd/lib_var_tmp/stemold/libmd2hip.so
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_conv.py -x -q --timeout 120 --timeout-method thread -k "k7s2" > gpurun_out/pytest_r06ai.log 2>&1 || { tail -30 gpurun_out/pytest_r06ai.log; exit 30; }
tail -1 gpurun_out/pytest_r06ai.log
cd /tmp && export TMPDIR=/tmp
for v in new old; do
  if [ $v = old ]; then export MD2HIP_LIB=$V; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_ws_$v -o run --output-format csv -- python3 $R/tools/conv_one.py stem wgrad > /dev/null 2>&1 || exit 21
  unset MD2HIP_LIB
  python3 - $R/gpurun_out/prof_ws_$v/run_kernel_stats.csv $v <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "stem" in r["Name"]:
        print(f"{sys.argv[2]:4s} {r['Name'][:60]:60s} calls={r['Calls']} avg_us={float(r['AverageNs'])/1000:.1f}")
PY
done
cd $R
for rep in 1 2 3; do
for v in old new; do
  if [ $v = old ]; then L="MD2HIP_LIB=$V"; else L=""; fi
  env $L timeout -k 10 200 python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/ab_r06ai.json 2>/dev/null || exit 23
  python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_r06ai.json')); print('%-4s %9.1f img/s  %.3f ms' % (sys.argv[1], d['value'], d['ms_per_step']))" "$v"
done; done
