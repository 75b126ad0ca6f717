#!/bin/bash
# after restoring conv_halo3's LDS size: smoke()'s parity case, the full conv suite, and the
# stride-2 halo dgrad A/B again (interleaved bench pairs)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python3 tools/smoke_ab.py > gpurun_out/sab_one.txt 2>&1 || { tail -5 gpurun_out/sab_one.txt; exit 31; }
tail -1 gpurun_out/sab_one.txt
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_conv.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r06ag.log 2>&1 || { tail -30 gpurun_out/pytest_r06ag.log; exit 30; }
tail -2 gpurun_out/pytest_r06ag.log
for rep in 1 2 3; do
for v in 0 1; do
  MD2_TUNING=1 MD2_HALO_S2=$v timeout -k 10 200 python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/ab_r06ag.json 2>/dev/null || exit 23
  python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_r06ag.json')); print('S2=%s %9.1f img/s  %.3f ms' % (sys.argv[1], d['value'], d['ms_per_step']))" "$v"
done; done
