#!/bin/bash
# stem wgrad split-K target sweep (conv_wgrad_stem_kernel): per-layer table stem rows per target
export MD2_TUNING=1   # kernel / planner knobs are honoured only with this (common.h tuning_knob)
set -uo pipefail
for t in ${TARGETS:-256 512 1024 2048}; do
  MD2_WSTEM_TARGET=$t timeout -k 10 200 python tools/layer_table.py sweep 12 3 > /dev/null 2>&1 || exit 1
  echo "target $t: $(grep 'wgrad 7x7' profiles/sweep_layers.md | cut -c1-120)"
done
