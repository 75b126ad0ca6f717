#!/bin/bash
# stream balance with the layer 2-4 filter gradients on the side: MD2_ENC_WGRAD_MAIN0 A/B
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2 3; do
for v in "MD2_ENC_WGRAD_MAIN0=1" "MD2_ENC_WGRAD_MAIN0=0" "MD2_ENC_WGRAD_FROM=0 MD2_ENC_WGRAD_MAIN0=0"; do
  env MD2_TUNING=1 $v timeout -k 10 200 python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/ab_r06aa.json 2>/dev/null || exit 23
  python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_r06aa.json')); print('%-45s %9.1f img/s  %.3f ms' % (sys.argv[1], d['value'], d['ms_per_step']))" "$v"
done; done
