#!/bin/bash
# 4-pixel reflect fold: conv parity, bit-identity through the fusion tests, step A/B (MD2_FOLD4)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_conv.py tests/test_gpu_fusion.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r06w.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_r06w.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_r06w.log | head -20; exit $rc; }
MD2HIP_DIGEST_OUT=gpurun_out/dig1.txt timeout -k 10 200 python3 tools/step_digest.py > gpurun_out/dig1.txt 2>&1 || exit 25
MD2_TUNING=1 MD2_FOLD4=0 timeout -k 10 200 python3 tools/step_digest.py > gpurun_out/dig0.txt 2>&1 || exit 26
tail -1 gpurun_out/dig1.txt; tail -1 gpurun_out/dig0.txt
for rep in 1 2 3; do
for v in 1 0; do
  MD2_TUNING=1 MD2_FOLD4=$v timeout -k 10 200 python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/ab_r06w.json 2>/dev/null || exit 23
  python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_r06w.json')); print('MD2_FOLD4=%s %9.1f img/s  %.3f ms' % (sys.argv[1], d['value'], d['ms_per_step']))" "$v"
done; done
