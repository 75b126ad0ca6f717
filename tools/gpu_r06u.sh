#!/bin/bash
# per-layer event tables with / without the 2D-tile halo kernel
set -o pipefail
mkdir -p gpurun_out
for v in 1 0; do
  MD2_TUNING=1 MD2_HALO2D=$v timeout -k 10 200 python3 -u tools/layer_table.py h2d$v > /dev/null 2>&1 || exit 24
  cp profiles/h2d${v}_layers.md gpurun_out/
done
