#!/bin/bash
# Build a variant libmd2hip.so with one translation unit recompiled under extra flags, for A/B
# runs on the GPU box (select it with MD2HIP_LIB=<repo>/lib_var/<name>/libmd2hip.so).
#   tools/build_variant.sh <name> <unit.hip> "<extra hipcc flags>"
set -euo pipefail
NAME=$1; UNIT=$2; FLAGS=${3:-}
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/monodepth2.jl_amd/csrc
make -C "$C" -j16 > /dev/null
OUT=${VAR_DIR:-$R/lib_var}/$NAME
mkdir -p "$OUT"
base=$(basename "${UNIT%.*}")
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall -Wno-unused-function --offload-arch=gfx950 $FLAGS \
  -c "$C/$UNIT" -o "$OUT/$base.o"
objs=$(ls "$C"/build/*.o | grep -v "/$base.o$")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$OUT/libmd2hip.so" $objs "$OUT/$base.o" -lz
echo "$OUT/libmd2hip.so"
