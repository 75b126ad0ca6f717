# per-shape conv timings under planner knobs: bash tools/gpu_knobconv.sh TAG SHAPES "ENV1" "ENV2" ...
set -o pipefail
mkdir -p gpurun_out
T=$1; SH=$2; shift 2
for v in "$@"; do
  if [ "$v" = default ]; then E=""; else E="MD2_TUNING=1 $v"; fi
  echo "== $v"
  env $E timeout -k 10 200 python3 tools/bench_conv.py --only=$SH 2>&1 | grep -E "^[a-z0-9.]+ +GF" || exit 21
done
