#!/bin/bash
# final pass: smoke(), the -m gpu suite, then the measurement pass (round_final.sh without the suite)
set -o pipefail
mkdir -p gpurun_out
TAG=${1:?tag}
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_$TAG.txt 2>&1 || { tail -20 gpurun_out/smoke_$TAG.txt; exit 30; }
tail -1 gpurun_out/smoke_$TAG.txt
NO_PROFILE=1 bash tools/gpu_check.sh $TAG || exit $?
