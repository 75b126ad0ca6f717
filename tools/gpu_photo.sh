#!/bin/bash
# Photometric kernel check on the GPU box: its parity tests, then the kernel timings of the
# library and each lib_var/ variant (VARIANTS) at B=12 and 96, and a bench line per library.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_loss.py tests/test_gpu_ops.py tests/test_golden.py tests/test_gpu_bench_parity.py -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/photo_tests.log 2>&1
rc=$?; tail -3 gpurun_out/photo_tests.log; [ $rc -gt 1 ] && exit $rc
timeout -k 10 400 bash tools/ab_photo.sh 12 > gpurun_out/ab_photo12.txt 2>&1 || exit 5
timeout -k 10 400 bash tools/ab_photo.sh 96 > gpurun_out/ab_photo96.txt 2>&1 || exit 6
grep -h "==\|photo_stream" gpurun_out/ab_photo12.txt gpurun_out/ab_photo96.txt
for v in base ${VARIANTS:-}; do
  lib=$PWD/monodepth2.jl_amd/lib/libmd2hip.so
  [ "$v" != base ] && lib=$PWD/lib_var/$v/libmd2hip.so
  MD2HIP_LIB=$lib timeout -k 10 200 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/bench_$v.json 2> gpurun_out/bench_$v.err || exit 7
  python3 -c "import json;d=json.load(open('gpurun_out/bench_$v.json'));print('$v', d['value'], d['roofline_photometric']['kernel_ms_per_step'], d['roofline']['frac'])"
done
exit $rc
