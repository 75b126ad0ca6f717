# A/B of planner knobs on the full bench step (run on the GPU box from the repo root):
#   bash tools/gpu_ab.sh TAG "ENV1" "ENV2" ...   ("default" = no knob; knobs need MD2_TUNING=1)
set -o pipefail
mkdir -p gpurun_out
T=$1; shift
[ -n "$SKIP_TESTS" ] || timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_fusion.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_${T}_conv.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_${T}_conv.log; [ $rc -eq 0 ] || { grep -E "^E " gpurun_out/pytest_${T}_conv.log | head -20; exit $rc; }
for rep in 1 2; do
for v in "$@"; do
  if [ "$v" = default ]; then E=""; else E="MD2_TUNING=1 $v"; fi
  env $E timeout -k 10 200 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/ab_${T}.json 2>/dev/null || exit 23
  python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_${T}.json')); print('%-40s %9.1f img/s  %.3f ms' % (sys.argv[1], d['value'], d['ms_per_step']))" "$v"
done; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$T -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-probe > /dev/null 2>&1 || exit 24
