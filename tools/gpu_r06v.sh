#!/bin/bash
# 2D-tile halo kernel: step A/B per pass (MD2_HALO2D bit 0 forward, bit 1 data gradient)
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2 3; do
for v in 3 1 0; do
  MD2_TUNING=1 MD2_HALO2D=$v timeout -k 10 200 python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/ab_r06v.json 2>/dev/null || exit 23
  python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_r06v.json')); print('MD2_HALO2D=%s %9.1f img/s  %.3f ms' % (sys.argv[1], d['value'], d['ms_per_step']))" "$v"
done; done
