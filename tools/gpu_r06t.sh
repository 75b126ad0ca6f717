#!/bin/bash
# 2D-tile halo kernel (decoder Cout = 32 forwards, Cin = 96 / 32-row data gradients, 64x208 maps):
# conv parity, per-shape kernel times, step A/B (MD2_HALO2D)
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_conv.py -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r06t_conv.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_r06t_conv.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_r06t_conv.log | head -20; exit $rc; }
for v in 1 0; do
  MD2_TUNING=1 MD2_HALO2D=$v timeout -k 10 200 python3 tools/bench_conv.py --only=d1c2,d2c2,d3c1,d3c2,d4c1,d4c2,d5c1 > gpurun_out/bc_r06t_$v.txt 2>&1 || exit 22
  echo "MD2_HALO2D=$v"; cat gpurun_out/bc_r06t_$v.txt | grep -v "^{"
done
for rep in 1 2; do
for v in 1 0; do
  MD2_TUNING=1 MD2_HALO2D=$v timeout -k 10 200 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/ab_r06t.json 2>/dev/null || exit 23
  python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_r06t.json')); print('MD2_HALO2D=%s %9.1f img/s  %.3f ms' % (sys.argv[1], d['value'], d['ms_per_step']))" "$v"
done; done
