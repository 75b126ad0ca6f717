#!/bin/bash
set -uo pipefail
echo "=== v1"; MD2_PX_V2=0 timeout -k 10 120 python3 tools/bench_conv.py || exit 1
echo "=== v2 d2"; timeout -k 10 120 python3 tools/bench_conv.py || exit 1
echo "=== v2 d3"; MD2HIP_LIB=$PWD/monodepth2.jl_amd/lib_d3/libmd2hip.so timeout -k 10 120 python3 tools/bench_conv.py || exit 1
