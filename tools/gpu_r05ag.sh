set -o pipefail
mkdir -p gpurun_out
T=${1:-r05ag}
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_fusion.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_${T}.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_${T}.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_${T}.log | head -20; exit $rc; }
SKIP_TESTS=1 bash tools/gpu_ab.sh $T default || exit 27
python3 - <<'PY'
import csv
for r in csv.DictReader(open('gpurun_out/prof_r05ag/run_kernel_stats.csv')):
    if 'splitk_reduce' in r['Name']: print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1), round(float(r['TotalDurationNs'])/13e3,1))
PY
