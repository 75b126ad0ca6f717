set -o pipefail
mkdir -p gpurun_out
T=${1:-r05ah}
timeout -k 10 900 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_fusion.py tests/test_gpu_model.py tests/test_gpu_bench_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_${T}.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_${T}.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_${T}.log | head -20; exit $rc; }
SKIP_TESTS=1 bash tools/gpu_ab.sh $T default "MD2_FUSE_BNSTATS=0" || exit 27
