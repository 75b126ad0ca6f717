#!/bin/bash
# side-stream priority (MD2_SIDE_PRIO: 1 least, -1 greatest) -- interleaved bench A/B
set -o pipefail
mkdir -p gpurun_out
MD2_TUNING=1 MD2_SIDE_PRIO=1 MD2_PRIO_PRINT=1 timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline 2>&1 >/dev/null | grep -m1 "priority range" || true
for rep in 1 2 3; do
for v in 0 1 -1; do
  MD2_TUNING=1 MD2_SIDE_PRIO=$v timeout -k 10 200 python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/ab_r06ah.json 2>/dev/null || exit 23
  python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_r06ah.json')); print('PRIO=%-3s %9.1f img/s  %.3f ms' % (sys.argv[1], d['value'], d['ms_per_step']))" "$v"
done; done
