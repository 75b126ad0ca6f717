set -o pipefail
mkdir -p gpurun_out
T=${1:-r05v}
timeout -k 10 900 python -u -m pytest tests/test_gpu_loss.py tests/test_gpu_ops.py tests/test_gpu_fusion.py tests/test_gpu_slow_depth.py tests/test_gpu_model.py tests/test_gpu_bench_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_${T}.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_${T}.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_${T}.log | head -20; exit $rc; }
bash tools/gpu_whxdbg.sh $T || exit 26
SKIP_TESTS=1 bash tools/gpu_ab.sh $T default || exit 27
python3 tools/step_families.py gpurun_out/prof_$T/run_kernel_stats.csv | grep -E "smooth|heads|total" 
python3 - <<'PY'
import csv
for r in csv.DictReader(open('gpurun_out/prof_r05v/run_kernel_stats.csv')):
    if 'smooth' in r['Name']: print(r['Name'][:40], float(r['AverageNs'])/1e3)
PY
