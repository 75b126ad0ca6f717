set -o pipefail
mkdir -p gpurun_out
T=${1:-r05h}
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_${T}_conv.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_${T}_conv.log; [ $rc -eq 0 ] || { grep -E "^E " gpurun_out/pytest_${T}_conv.log | head -20; exit $rc; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_${T}_w -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/bench_conv.py --only=l1,l2,l3,l4 > $GRAFT_REPO_ROOT/gpurun_out/bench_conv_${T}.txt 2>&1 || exit 21
MD2_TUNING=1 MD2_WHALO=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_${T}_wold -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/bench_conv.py --only=l1,l2,l3,l4 > $GRAFT_REPO_ROOT/gpurun_out/bench_conv_${T}_old.txt 2>&1 || exit 22
cd $GRAFT_REPO_ROOT
grep -E "^l[1-4]" gpurun_out/bench_conv_${T}.txt gpurun_out/bench_conv_${T}_old.txt
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err && cut -c1-200 gpurun_out/bench_$T.json
