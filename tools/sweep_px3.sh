#!/bin/bash
# conv_px3 (bf16x9) vs conv_px2 (fp32 MFMA) per encoder layer over forced tile shapes
# (MD2_PX_TILE: 0 128x128, 1 64x256, 3 64x128, 5 64x64) -- tools/bench_conv.py
mkdir -p gpurun_out
O=gpurun_out/sweep_px3.txt
: > $O
for px3 in 0 1; do
  for t in 5 3 1 0; do
    echo "== PX3=$px3 TILE=$t" >> $O
    MD2_TUNING=1 MD2_PX3=$px3 MD2_PX_TILE=$t timeout -k 10 120 python -u tools/bench_conv.py --only=l1,l2,l3,l4 >> $O 2>&1 || { echo "failed PX3=$px3 TILE=$t" >> $O; exit 3; }
  done
done
grep -v amdgpu.ids $O
