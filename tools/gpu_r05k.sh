set -o pipefail
mkdir -p gpurun_out
T=${1:-r05k}
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_fusion.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_${T}_conv.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_${T}_conv.log; [ $rc -eq 0 ] || { grep -E "^E " gpurun_out/pytest_${T}_conv.log | head -20; exit $rc; }
bash tools/profile_round.sh $T || exit 22
python3 tools/step_families.py gpurun_out/prof_$T/trace > gpurun_out/families_$T.txt 2>&1; tail -30 gpurun_out/families_$T.txt
cut -c1-300 gpurun_out/prof_$T/bench_plain.json
