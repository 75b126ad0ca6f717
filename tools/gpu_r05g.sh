set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 ./tools/micro/mfma_round > gpurun_out/mfma_round.txt 2>&1 || exit 9
cat gpurun_out/mfma_round.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r05g_conv.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_r05g_conv.log; [ $rc -eq 0 ] || exit $rc
for v in "default" "MD2_PX3_TERMS=9" "MD2_PX3_M32=0" "MD2_PX3=0"; do
  env MD2_TUNING=1 $( [ "$v" = default ] || echo $v ) timeout -k 10 300 python3 -u tools/forward_bisect.py --out gpurun_out/bis3_${v%%=*}.json > gpurun_out/bis3_${v%%=*}.txt 2>&1 || exit 11
  echo "== $v"; grep -E "branch[345]|disp|feat4" gpurun_out/bis3_${v%%=*}.txt
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_r05g.json 2> gpurun_out/bench_r05g.err && cut -c1-300 gpurun_out/bench_r05g.json
