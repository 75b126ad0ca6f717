set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_slow_depth.py -m gpu -v -s --timeout 280 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_sd2.log 2>&1; grep -E "PASSED|FAILED|passed|failed" gpurun_out/pytest_sd2.log | tail -12
timeout -k 10 900 python3 -u tools/fp32_realizations.py --out gpurun_out/f32r2.json > gpurun_out/f32r2.txt 2>&1; rc=$?
head -30 gpurun_out/f32r2.txt | cut -c1-200; tail -3 gpurun_out/f32r2.txt; exit $rc
