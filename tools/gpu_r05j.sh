set -o pipefail
mkdir -p gpurun_out
T=${1:-r05j}
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_fusion.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_${T}_conv.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_${T}_conv.log; [ $rc -eq 0 ] || { grep -E "^E " gpurun_out/pytest_${T}_conv.log | head -20; exit $rc; }
cd /tmp && export TMPDIR=/tmp
for v in "default" "MD2_HALO_RFL_DGRAD=0"; do
MD2_TUNING=1 env $( [ "$v" = default ] || echo $v ) timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_${T}_${v%%=*} -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/bench_conv.py --only=d3c2,d4c2,l2,l3 > $GRAFT_REPO_ROOT/gpurun_out/bench_conv_${T}_${v%%=*}.txt 2>&1 || exit 21
done
cd $GRAFT_REPO_ROOT
grep -hE "^(d|l)[0-9]" gpurun_out/bench_conv_${T}_*.txt
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err && cut -c1-200 gpurun_out/bench_$T.json
