# parity tests of the model step (check_step records -> gpurun_out/parity) + slow_depth
set -o pipefail
T=${1:-par}
mkdir -p gpurun_out
K=${2:-}
ARGS=(tests/test_gpu_slow_depth.py tests/test_gpu_bench_parity.py tests/test_gpu_model.py tests/test_gpu_mpi_train.py tests/test_gpu_ops.py -m gpu -v -s --timeout 400 --timeout-method thread -p no:cacheprovider)
[ -n "$K" ] && ARGS+=(-k "$K")
timeout -k 10 1050 python3 -u -m pytest "${ARGS[@]}" > gpurun_out/pytest_$T.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/pytest_$T.log | tail -60
exit $rc
