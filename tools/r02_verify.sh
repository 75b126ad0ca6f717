set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1; echo "pytest rc=$?" >> gpurun_out/gputest.log
tail -5 gpurun_out/gputest.log
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || exit 1
tail -2 gpurun_out/bench.log
for cfg in "-1 0" "2 0" "2 1152" "2 2304"; do set -- $cfg; echo "== wtile $1 tgt $2"; MD2_W_TILE=$1 MD2_W_TARGET=$2 timeout -k 10 120 python tools/bench_conv.py --only=l1,l2,l3,l4 || exit 1; done > gpurun_out/wsweep.log 2>&1
cat gpurun_out/wsweep.log
