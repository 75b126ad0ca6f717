set -o pipefail
mkdir -p gpurun_out
T=${1:-r05y}
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_${T}.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_${T}.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_${T}.log | head -20; exit $rc; }
bash tools/gpu_whxdbg.sh $T || exit 26
bash tools/gpu_knobconv.sh $T l1,l2,l3,l4 default || exit 28
SKIP_TESTS=1 bash tools/gpu_ab.sh $T default || exit 27
