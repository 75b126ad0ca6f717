#!/bin/bash
# BN reduction passes with 8 float4 units in flight per thread (variant library) -- digest + A/B
set -o pipefail
mkdir -p gpurun_out
V=$GRAFT_REPO_ROOT/monodepth2.jl_amd/lib_var_tmp/bn8/libmd2hip.so
timeout -k 10 200 python3 tools/step_digest.py > gpurun_out/dig_b4.txt 2>&1 || exit 25
MD2HIP_LIB=$V timeout -k 10 200 python3 tools/step_digest.py > gpurun_out/dig_b8.txt 2>&1 || exit 26
tail -1 gpurun_out/dig_b4.txt | cut -c1-200; tail -1 gpurun_out/dig_b8.txt | cut -c1-200
for rep in 1 2 3; do
for v in base bn8; do
  if [ $v = base ]; then L=""; else L="MD2HIP_LIB=$V"; fi
  env $L timeout -k 10 200 python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/ab_r06ab.json 2>/dev/null || exit 23
  python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_r06ab.json')); print('%-6s %9.1f img/s  %.3f ms' % (sys.argv[1], d['value'], d['ms_per_step']))" "$v"
done; done
