#!/bin/bash
# upsample adjoint (4 rows / thread) + knob deletion: nn / fusion tests, bench, kernel stats
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_nn.py tests/test_gpu_fusion.py tests/test_gpu_photo2.py -m gpu -q --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r06f.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_r06f.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python3 bench.py --no-cpu-baseline > gpurun_out/bench_r06f.json 2> gpurun_out/bench_r06f.err || exit 1
cut -c1-260 gpurun_out/bench_r06f.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r06f -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-probe > /dev/null 2>&1 || exit 1
grep -E "upsample|photo2" $GRAFT_REPO_ROOT/gpurun_out/prof_r06f/run_kernel_stats.csv | cut -c1-160
