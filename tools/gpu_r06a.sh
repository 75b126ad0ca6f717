#!/bin/bash
# round-6 first GPU pass: the new boundary tests, the whole -m gpu suite, one bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python3 -u -m pytest tests/test_gpu_forward_boundary.py -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r06a_boundary.log 2>&1
rc1=$?
tail -5 gpurun_out/pytest_r06a_boundary.log
[ $rc1 -eq 0 ] || [ $rc1 -eq 1 ] || exit $rc1
timeout -k 10 700 python3 -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r06a.log 2>&1
rc2=$?
tail -15 gpurun_out/pytest_r06a.log
[ $rc2 -eq 0 ] || [ $rc2 -eq 1 ] || exit $rc2
timeout -k 10 240 python3 bench.py --cpu-seconds 5 > gpurun_out/bench_r06a.json 2> gpurun_out/bench_r06a.err
rc3=$?
cat gpurun_out/bench_r06a.json | cut -c1-600
exit $((rc1 + rc2 + rc3))
