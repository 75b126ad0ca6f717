set -o pipefail
mkdir -p gpurun_out
T=${1:-r05p}
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_${T}_conv.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_${T}_conv.log; [ $rc -eq 0 ] || { grep -E "^E " gpurun_out/pytest_${T}_conv.log | head -20; exit $rc; }
bash tools/gpu_dec.sh $T || exit 25
for rep in 1 2; do for v in default "MD2_HALO_RFL_DGRAD=0"; do
  if [ "$v" = default ]; then E=""; else E="MD2_TUNING=1 $v"; fi
  env $E timeout -k 10 200 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/ab_${T}.json 2>/dev/null || exit 23
  python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_${T}.json')); print('%-40s %9.1f img/s  %.3f ms' % (sys.argv[1], d['value'], d['ms_per_step']))" "$v"
done; done
