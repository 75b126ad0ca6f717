#!/bin/bash
# encoder filter gradients from layer 2 on the side stream: digest vs layer-4-only, model suites
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python3 tools/step_digest.py > gpurun_out/digz1.txt 2>&1 || exit 25
MD2_TUNING=1 MD2_ENC_WGRAD_FROM=3 timeout -k 10 200 python3 tools/step_digest.py > gpurun_out/digz3.txt 2>&1 || exit 26
tail -1 gpurun_out/digz1.txt; tail -1 gpurun_out/digz3.txt
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_fusion.py tests/test_gpu_model.py tests/test_gpu_bench_parity.py tests/test_gpu_dp.py -m gpu -q -x --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r06z.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_r06z.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_r06z.log | head -20; exit $rc; }
