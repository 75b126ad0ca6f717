# forward-accuracy bisection at config 3 (uniform frames) under kernel knobs + a step trace
set -o pipefail
T=${1:-bis}
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/forward_bisect.py --out gpurun_out/${T}_default.json > gpurun_out/${T}_default.txt 2>&1 || exit 11
MD2_TUNING=1 MD2_PX3=0 timeout -k 10 300 python3 -u tools/forward_bisect.py --out gpurun_out/${T}_px3off.json > gpurun_out/${T}_px3off.txt 2>&1 || exit 12
cat gpurun_out/${T}_default.txt; echo ==== PX3=0; cat gpurun_out/${T}_px3off.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_${T}_step -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-probe > $GRAFT_REPO_ROOT/gpurun_out/bench_${T}_trace.json 2>/dev/null || exit 13
