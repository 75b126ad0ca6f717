#!/bin/bash
# photo2: bit-identity vs the scalar kernel, loss parity, kernel timing A/B, one bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_photo2.py tests/test_gpu_loss.py -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r06b.log 2>&1
rc1=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/pytest_r06b.log | tail -25
[ $rc1 -eq 0 ] || [ $rc1 -eq 1 ] || exit $rc1
CONFIGS="MD2_PHOTO_V1=1;MD2_PHOTO_V1=0" timeout -k 10 400 bash tools/ab_photo.sh 12 > gpurun_out/ab_photo_r06b.txt 2>&1
rc2=$?
cat gpurun_out/ab_photo_r06b.txt
[ $rc2 -eq 0 ] || exit $rc2
timeout -k 10 240 python3 bench.py --no-cpu-baseline > gpurun_out/bench_r06b.json 2> gpurun_out/bench_r06b.err
rc3=$?
cut -c1-300 gpurun_out/bench_r06b.json
python3 -c "import json; d=json.loads(open('gpurun_out/bench_r06b.json').read()); print(d['roofline_photometric'])"
exit $((rc1 + rc3))
