#!/bin/bash
# Split-K block-target sweep of the conv planner (MD2_PX_TARGET for fwd/dgrad, MD2_W_TARGET /
# MD2_W64_TARGET for wgrad): one per-layer table per setting under gpurun_out/sweep/.
export MD2_TUNING=1   # kernel / planner knobs are honoured only with this (common.h tuning_knob)
set -uo pipefail
mkdir -p gpurun_out/sweep
for t in ${PX_TARGETS:-}; do
  MD2_PX_TARGET=$t timeout -k 10 200 python tools/layer_table.py px$t 12 3 > /dev/null 2>&1 || exit 1
  mv profiles/px${t}_layers.md gpurun_out/sweep/
done
for t in ${W_TARGETS:-}; do
  MD2_W_TARGET=$t timeout -k 10 200 python tools/layer_table.py w$t 12 3 > /dev/null 2>&1 || exit 1
  mv profiles/w${t}_layers.md gpurun_out/sweep/
done
echo sweep done
