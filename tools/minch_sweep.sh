#!/bin/bash
# Whole-step A/B of the split-K planners' minimum K chunks per split (MD2_PX_MINCH, MD2_W_MINCH):
# bench.py (B=12, 416x128) per setting, one JSON line each.
export MD2_TUNING=1   # kernel / planner knobs are honoured only with this (common.h tuning_knob)
set -o pipefail
mkdir -p gpurun_out
for cfg in "8 8" "4 8" "8 4" "4 4" "2 2" "8 8"; do
  set -- $cfg
  v=$(MD2_PX_MINCH=$1 MD2_W_MINCH=$2 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 --warmup 5 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['frac'], d['conv_other']['ms_per_step'])") || exit 1
  echo "px_minch $1 w_minch $2 : $v"
done
