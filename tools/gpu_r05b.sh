set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r05b_conv.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_r05b_conv.log; [ $rc -le 1 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r05b_halo -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/bench_conv.py --only=l1,l2,l3,l4 > $GRAFT_REPO_ROOT/gpurun_out/bench_conv_r05b_halo.txt 2>&1 || exit 21
MD2_TUNING=1 MD2_HALO=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r05b_px3 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/bench_conv.py --only=l1,l2,l3,l4 > $GRAFT_REPO_ROOT/gpurun_out/bench_conv_r05b_px3.txt 2>&1 || exit 22
cd $GRAFT_REPO_ROOT
[ $rc -eq 0 ] || exit 1
timeout -k 10 500 python -u -m pytest tests/test_gpu_dp.py tests/test_gpu_graph.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r05b_dp.log 2>&1; tail -3 gpurun_out/pytest_r05b_dp.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench_r05b.json 2> gpurun_out/bench_r05b.err && cat gpurun_out/bench_r05b.json
