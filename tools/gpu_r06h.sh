#!/bin/bash
# BN apply + ReLU in the LDS-halo staging: fusion bit-identity, model parity (R18/R34/R50), A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_fusion.py tests/test_gpu_model.py tests/test_gpu_conv.py -m gpu -q -x --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r06h.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_r06h.log; [ $rc -eq 0 ] || { grep -E "^E " gpurun_out/pytest_r06h.log | head -20; exit $rc; }
for rep in 1 2 3; do
for v in default "MD2_FUSE_BNSTAGE=0"; do
  if [ "$v" = default ]; then E=""; else E="$v"; fi
  env $E timeout -k 10 200 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/ab_r06h.json 2>/dev/null || exit 23
  python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_r06h.json')); print('%-30s %9.1f img/s  %.3f ms' % (sys.argv[1], d['value'], d['ms_per_step']))" "$v"
done; done
