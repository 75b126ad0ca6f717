#!/bin/bash
# photo2 bit-identity + A/B, then the HEAD profile (trace, FETCH, WRITE, MFMA-busy passes) and
# the photometric PMC at B=12
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python3 -u -m pytest tests/test_gpu_photo2.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r06e.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_r06e.log; [ $rc -eq 0 ] || exit $rc
bash tools/pmc_photo_ab.sh > gpurun_out/pmc_photo_ab_r06e.txt 2>&1 || exit 1
grep -E "V1=|SQ_INSTS_VALU|wait_any" gpurun_out/pmc_photo_ab_r06e.txt
bash tools/profile_round.sh r06e > gpurun_out/profile_r06e.txt 2>&1 || { tail -5 gpurun_out/profile_r06e.txt; exit 1; }
bash tools/pmc_photo.sh r06e 12 > gpurun_out/pmc_photo_r06e.txt 2>&1 || { tail -5 gpurun_out/pmc_photo_r06e.txt; exit 1; }
echo all done
