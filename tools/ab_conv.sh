#!/bin/bash
export MD2_TUNING=1   # kernel / planner knobs are honoured only with this (common.h tuning_knob)
set -uo pipefail
echo "=== w1"; MD2_W_V2=0 timeout -k 10 120 python3 tools/bench_conv.py || exit 1
echo "=== w2"; timeout -k 10 120 python3 tools/bench_conv.py || exit 1
echo "=== w2 target1024"; MD2_W_TARGET=1024 timeout -k 10 120 python3 tools/bench_conv.py || exit 1
echo "=== w2 tile64x64 t1024"; MD2_W_TILE=2 MD2_W_TARGET=1024 timeout -k 10 120 python3 tools/bench_conv.py || exit 1
