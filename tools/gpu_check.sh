#!/bin/bash
# One GPU-box pass (run from the repo root under gpurun): the -m gpu suite with its parity records
# (gpurun_out/parity/*.json), then -- only if pytest ended normally (0 = green, 1 = failures) --
# the DP overlap table at configs 4 and 5 and the per-round profile (tools/profile_round.sh TAG).
#   tools/gpu_check.sh TAG [pytest -k expression]
TAG=${1:?tag}
K=${2:-}
mkdir -p gpurun_out
ARGS=(tests -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider)
[ -n "$K" ] && ARGS+=(-k "$K")
timeout -k 10 1000 python -u -m pytest "${ARGS[@]}" > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_$TAG.log
if [ $rc -gt 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
[ -n "${NO_PROFILE:-}" ] && exit $rc
timeout -k 10 200 python -u tools/dp_overlap.py gpurun_out/dp_overlap_c4_$TAG.json > /dev/null || exit 3
timeout -k 10 200 python -u tools/dp_overlap.py gpurun_out/dp_overlap_c5_$TAG.json --arch 50 --height 192 --width 640 --batch 8 > /dev/null || exit 3
bash tools/profile_round.sh $TAG || exit 4
exit $rc
