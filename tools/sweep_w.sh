#!/bin/bash
export MD2_TUNING=1   # kernel / planner knobs are honoured only with this (common.h tuning_knob)
set -uo pipefail
for CFG in "-1 512" "0 1024" "2 512" "2 1024" "2 2048" "3 1024" "1 1024"; do
  set -- $CFG
  echo "=== wtile $1 target $2"
  MD2_PX_TILE=5 MD2_PX_TARGET=1536 MD2_W_TILE=$1 MD2_W_TARGET=$2 timeout -k 10 120 python3 tools/bench_conv.py || exit 1
done
