#!/bin/bash
export MD2_TUNING=1   # kernel / planner knobs are honoured only with this (common.h tuning_knob)
set -uo pipefail
for CFG in "5 1536" "4 1536" "3 1536" "0 768" "0 1536"; do
  set -- $CFG
  echo "=== tile $1 target $2"
  MD2_PX_TILE=$1 MD2_PX_TARGET=$2 timeout -k 10 120 python3 tools/bench_conv.py || exit 1
done
