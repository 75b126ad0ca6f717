#!/bin/bash
# Cin = 32 reflect data gradients on the 2D-tile halo kernel (MD2_HALO2D bit 2): parity, A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_conv.py tests/test_gpu_model.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r06x.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_r06x.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_r06x.log | head -20; exit $rc; }
for v in 5 1; do
  MD2_TUNING=1 MD2_HALO2D=$v timeout -k 10 200 python3 tools/bench_conv.py --only=d5c1,d4c1 > gpurun_out/bc_r06x_$v.txt 2>&1 || exit 22
  echo "MD2_HALO2D=$v"; grep -v "^{\|amdgpu.ids" gpurun_out/bc_r06x_$v.txt
done
for rep in 1 2 3; do
for v in 5 1; do
  MD2_TUNING=1 MD2_HALO2D=$v timeout -k 10 200 python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/ab_r06x.json 2>/dev/null || exit 23
  python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_r06x.json')); print('MD2_HALO2D=%s %9.1f img/s  %.3f ms' % (sys.argv[1], d['value'], d['ms_per_step']))" "$v"
done; done
