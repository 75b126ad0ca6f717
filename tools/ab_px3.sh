#!/bin/bash
# bf16x9 conv kernel selection A/B: the default (conv_px3 on the large-map shapes, conv_px2
# elsewhere) vs conv_px2 everywhere (MD2_TUNING=1 MD2_PX3=0) vs conv_px3 on every conv_px2 shape
# (MD2_PX3=1): accuracy vs fp64, per-layer kernel times and a bench line each.
mkdir -p gpurun_out
L=l1,l2.0,l2,l3.0,l3,l4.0,l4,d3c2,d4c2
for v in -1 0 1; do
  env MD2_TUNING=1 MD2_PX3=$v timeout -k 10 300 python -u tools/conv_accuracy.py gpurun_out/acc_px3_$v.json > gpurun_out/acc_px3_$v.log 2>&1 || exit 3
  env MD2_TUNING=1 MD2_PX3=$v timeout -k 10 300 python -u tools/bench_conv.py --only=$L > gpurun_out/bc_px3_$v.log 2>&1 || exit 5
  env MD2_TUNING=1 MD2_PX3=$v timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/bench_px3_$v.json 2> gpurun_out/bench_px3_$v.err || exit 7
done
for v in -1 0 1; do
  echo "== MD2_PX3=$v"
  grep -v amdgpu.ids gpurun_out/bc_px3_$v.log
  python3 -c "import json;d=json.load(open('gpurun_out/bench_px3_$v.json'));print('bench', d['value'], d['roofline']['achieved'], d['roofline']['frac'], d['conv_other'])"
done
