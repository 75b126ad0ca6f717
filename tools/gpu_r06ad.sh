#!/bin/bash
# host enqueue order (heads backward before the pose branch's side-stream launches; encoder data
# gradient before its side-stream filter gradient) -- digest + interleaved A/B; and the M = 96
# reflect dgrad (decoder level-1 c2) on 32-row px3 tiles (MD2_PX_TILE=6 / 2) vs 64 x 64
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
V=$R/monodepth2.jl_amd/lib_var_tmp/order/libmd2hip.so
cd $R
timeout -k 10 200 python3 tools/step_digest.py > gpurun_out/dig_o0.txt 2>&1 || exit 25
MD2HIP_LIB=$V timeout -k 10 200 python3 tools/step_digest.py > gpurun_out/dig_o1.txt 2>&1 || exit 26
tail -1 gpurun_out/dig_o0.txt | cut -c1-200; tail -1 gpurun_out/dig_o1.txt | cut -c1-200
cd /tmp && export TMPDIR=/tmp
for t in -1 6 2; do
  MD2_TUNING=1 MD2_PX_TILE=$t timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_tile_$t -o run --output-format csv -- python3 $R/tools/conv_one.py d4 dgrad > /dev/null 2>&1 || exit 21
  python3 - $R/gpurun_out/prof_tile_$t/run_kernel_stats.csv $t <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(f"TILE={sys.argv[2]:3s} {r['Name'][:70]:70s} calls={r['Calls']} avg_us={float(r['AverageNs'])/1000:.1f} min_us={float(r['MinNs'])/1000:.1f}")
PY
done
cd $R
for rep in 1 2 3; do
for v in base order; do
  if [ $v = base ]; then L=""; else L="MD2HIP_LIB=$V"; fi
  env $L timeout -k 10 200 python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/ab_r06ad.json 2>/dev/null || exit 23
  python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_r06ad.json')); print('%-6s %9.1f img/s  %.3f ms' % (sys.argv[1], d['value'], d['ms_per_step']))" "$v"
done; done
