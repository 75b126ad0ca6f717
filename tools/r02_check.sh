#!/bin/bash
# Round-2 check on one MI355X: the whole -m gpu suite, the default bench, then the per-round
# profile (tools/profile_round.sh TAG).  Outputs under gpurun_out/.
set -o pipefail
TAG=${1:-r02c}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gputest.log; tail -4 gpurun_out/gputest.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || exit 1
tail -1 gpurun_out/bench.log
[ "${PROFILE:-1}" = "1" ] || exit 0
bash tools/profile_round.sh $TAG > gpurun_out/profile.log 2>&1 || { tail -20 gpurun_out/profile.log; exit 1; }
echo profiled
