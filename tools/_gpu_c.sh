mkdir -p gpurun_out
timeout -k 10 60 tools/micro/valu_rate > gpurun_out/valu_rate.txt 2>&1 || exit 2
export MD2_SEGV_TRACE=1
timeout -k 10 300 python -u tools/conv_accuracy.py gpurun_out/acc_px2.json > gpurun_out/acc_px2.log 2>&1 || exit 3
MD2_TUNING=1 MD2_PX3=1 timeout -k 10 300 python -u tools/conv_accuracy.py gpurun_out/acc_px3.json > gpurun_out/acc_px3.log 2>&1 || exit 4
timeout -k 10 300 python -u tools/bench_conv.py --only=l1,l2.0,l2,l3.0,l3,l4.0,l4 > gpurun_out/bc_px2.log 2>&1 || exit 5
MD2_TUNING=1 MD2_PX3=1 timeout -k 10 300 python -u tools/bench_conv.py --only=l1,l2.0,l2,l3.0,l3,l4.0,l4 > gpurun_out/bc_px3.log 2>&1 || exit 6
timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/bench_px2.json 2> gpurun_out/bench_px2.err || exit 7
MD2_TUNING=1 MD2_PX3=1 timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/bench_px3.json 2> gpurun_out/bench_px3.err || exit 8
cat gpurun_out/acc_px2.log gpurun_out/acc_px3.log gpurun_out/bc_px2.log gpurun_out/bc_px3.log
