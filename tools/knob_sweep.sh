#!/bin/bash
# Whole-step A/B of planner knobs: bench.py (B=12, 416x128, no CPU baseline) once per setting
# ("-" = defaults), printing images/s, the conv-set roofline fraction and conv_other ms/step.
set -o pipefail
export MD2_TUNING=1   # kernel / planner knobs are honoured only with this (common.h tuning_knob)
mkdir -p gpurun_out
for kv in "$@"; do
  if [ "$kv" = "-" ]; then envs=""; else envs="${kv//,/ }"; fi
  v=$(env $envs timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 --warmup 5 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['frac'], d['conv_other']['ms_per_step'])") || exit 1
  echo "$kv : $v"
done
