#!/bin/bash
# encoder filter gradients beside the data gradients from stage FROM (MD2_ENC_WGRAD_FROM) -- A/B
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2 3; do
for v in 3 2 1; do
  MD2_TUNING=1 MD2_ENC_WGRAD_FROM=$v timeout -k 10 200 python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/ab_r06y.json 2>/dev/null || exit 23
  python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_r06y.json')); print('MD2_ENC_WGRAD_FROM=%s %9.1f img/s  %.3f ms' % (sys.argv[1], d['value'], d['ms_per_step']))" "$v"
done; done
