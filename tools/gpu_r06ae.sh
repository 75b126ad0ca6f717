#!/bin/bash
# stride-2 data gradient on the LDS halo (conv_halo3s2): conv tests, per-shape rocprof timing vs
# conv_px3's merged classes (MD2_HALO_S2=0), interleaved bench A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_conv.py -x -q --timeout 120 --timeout-method thread -k "s2 or halo_s2 or 36-" > gpurun_out/pytest_r06ae.log 2>&1 || { tail -30 gpurun_out/pytest_r06ae.log; exit 30; }
tail -3 gpurun_out/pytest_r06ae.log
cd /tmp && export TMPDIR=/tmp
for sh in s2l2 s2l3 s2l4; do for v in 0 1; do
  MD2_TUNING=1 MD2_HALO_S2=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_s2_${sh}_$v -o run --output-format csv -- python3 $R/tools/conv_one.py $sh dgrad > /dev/null 2>&1 || exit 21
  python3 - $R/gpurun_out/prof_s2_${sh}_$v/run_kernel_stats.csv "$sh S2=$v" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "md2::" in r["Name"] and "pack" not in r["Name"]:
        print(f"{sys.argv[2]:10s} {r['Name'][:64]:64s} calls={r['Calls']} avg_us={float(r['AverageNs'])/1000:.1f}")
PY
done; done
cd $R
for rep in 1 2 3; do
for v in 0 1; do
  MD2_TUNING=1 MD2_HALO_S2=$v timeout -k 10 200 python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/ab_r06ae.json 2>/dev/null || exit 23
  python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_r06ae.json')); print('S2=%s %9.1f img/s  %.3f ms' % (sys.argv[1], d['value'], d['ms_per_step']))" "$v"
done; done
