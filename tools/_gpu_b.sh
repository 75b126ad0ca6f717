mkdir -p gpurun_out
MD2_SEGV_TRACE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py -v -s --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/graph_r04.log 2>&1
rc=$?; tail -5 gpurun_out/graph_r04.log; if [ $rc -gt 1 ]; then echo "graph rc=$rc"; exit $rc; fi
timeout -k 10 900 python -u -m pytest tests/test_gpu_bench_parity.py tests/test_gpu_loss.py tests/test_gpu_mine.py tests/test_gpu_model.py tests/test_gpu_mpi_train.py tests/test_gpu_nn.py tests/test_gpu_ops.py tests/test_gpu_params_abi.py tests/test_gpu_slow_depth.py tests/test_gpu_static.py tests/test_golden.py -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/rest_r04.log 2>&1
rc=$?; tail -5 gpurun_out/rest_r04.log; exit $rc
