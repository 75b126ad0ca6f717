set -o pipefail
mkdir -p gpurun_out
T=${1:-r05aj}
timeout -k 10 900 python -u -m pytest tests/test_gpu_fusion.py tests/test_gpu_nn.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_${T}.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_${T}.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_${T}.log | head -20; exit $rc; }
SKIP_TESTS=1 bash tools/gpu_ab.sh $T default "MD2_FUSE_BNSTATS=0" || exit 27
python3 - <<'PY'
import csv
for r in csv.DictReader(open('gpurun_out/prof_r05aj/run_kernel_stats.csv')):
    if 'bn_apply_fused' in r['Name'] or 'bn_stats' in r['Name']: print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1))
PY
