#!/bin/bash
set -uo pipefail
echo "=== base"; timeout -k 10 120 python3 tools/bench_conv.py || exit 1
echo "=== bk32"; MD2_PX_BK=32 timeout -k 10 120 python3 tools/bench_conv.py || exit 1
echo "=== prio"; MD2HIP_LIB=$PWD/monodepth2.jl_amd/lib_prio/libmd2hip.so timeout -k 10 120 python3 tools/bench_conv.py || exit 1
echo "=== prio+bk32"; MD2_PX_BK=32 MD2HIP_LIB=$PWD/monodepth2.jl_amd/lib_prio/libmd2hip.so timeout -k 10 120 python3 tools/bench_conv.py || exit 1
