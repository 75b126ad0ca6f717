#!/bin/bash
# stem BN statistics: in the s2d forward's epilogue vs the separate pass (MD2_STEM_BNSTATS=0)
set -o pipefail
mkdir -p gpurun_out
#timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fusion.py tests/test_gpu_model.py -m gpu -q -x --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r06q.log 2>&1
#rc=$?; tail -2 gpurun_out/pytest_r06q.log; [ $rc -eq 0 ] || { grep -E "^E " gpurun_out/pytest_r06q.log | head -20; exit $rc; }
for rep in 1 2 3; do
for v in 1 0; do
  MD2_TUNING=1 MD2_STEM_BNSTATS=$v timeout -k 10 200 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/ab_r06q.json 2>/dev/null || exit 23
  python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_r06q.json')); print('MD2_STEM_BNSTATS=%s %9.1f img/s  %.3f ms' % (sys.argv[1], d['value'], d['ms_per_step']))" "$v"
done; done
