#!/bin/bash
# Photometric kernel check on the GPU box: its parity tests, the A/B kernel timings (split vs
# the two-source-per-lane kernel) at B=12 and 96, and a bench line per kernel.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_loss.py tests/test_gpu_ops.py tests/test_golden.py tests/test_gpu_bench_parity.py -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/photo_tests.log 2>&1
rc=$?; tail -3 gpurun_out/photo_tests.log; [ $rc -gt 1 ] && exit $rc
CONFIGS="MD2_PHOTO_SPLIT=0;MD2_PHOTO_SPLIT=1" timeout -k 10 300 bash tools/ab_photo.sh 12 > gpurun_out/ab_photo12.txt 2>&1 || exit 5
CONFIGS="MD2_PHOTO_SPLIT=0;MD2_PHOTO_SPLIT=1" timeout -k 10 300 bash tools/ab_photo.sh 96 > gpurun_out/ab_photo96.txt 2>&1 || exit 6
cat gpurun_out/ab_photo12.txt gpurun_out/ab_photo96.txt
for s in 0 1; do
  MD2_TUNING=1 MD2_PHOTO_SPLIT=$s timeout -k 10 200 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/bench_split$s.json 2> gpurun_out/bench_split$s.err || exit 7
  python3 -c "import json;d=json.load(open('gpurun_out/bench_split$s.json'));print('split=$s', d['value'], d['roofline_photometric']['kernel_ms_per_step'], d['roofline']['frac'])"
done
exit $rc
