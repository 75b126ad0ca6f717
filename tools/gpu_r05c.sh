# halo conv iteration: conv tests, per-shape rocprof of the halo kernels, PMC of l2 fwd, bench
set -o pipefail
mkdir -p gpurun_out
T=${1:-r05c}
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_${T}_conv.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_${T}_conv.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_${T}_halo -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/bench_conv.py --only=l1,l2,l3,l4 > $GRAFT_REPO_ROOT/gpurun_out/bench_conv_${T}_halo.txt 2>&1 || exit 21
cd $GRAFT_REPO_ROOT
PMC_TAG=_$T bash tools/pmc_conv.sh l2 fwd > /dev/null 2>&1 || exit 22
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err && cat gpurun_out/bench_$T.json | cut -c1-400
