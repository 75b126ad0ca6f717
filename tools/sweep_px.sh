#!/bin/bash
# px-kernel tiling sweep over the bench conv shapes (planner overrides via env)
set -uo pipefail
for CFG in "5 1536" "5 3072" "5 6144" "6 1536" "6 3072" "2 1536"; do
  set -- $CFG
  echo "=== tile $1 target $2"
  MD2_PX_TILE=$1 MD2_PX_TARGET=$2 timeout -k 10 120 python3 tools/bench_conv.py || exit 1
done
