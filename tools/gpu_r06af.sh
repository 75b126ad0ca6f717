#!/bin/bash
# smoke()'s parity case under kernel switches (which change moved its loss)
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/sab.txt
for env in "" "" "MD2_TUNING=1 MD2_HALO_S2=0" "MD2_TUNING=1 MD2_STEM_S2D=0" "MD2_TUNING=1 MD2_HALO2D=0" "MD2_TUNING=1 MD2_HALO=0"; do
  env $env timeout -k 10 200 python3 tools/smoke_ab.py > gpurun_out/sab_one.txt 2>&1 || { tail -5 gpurun_out/sab_one.txt; exit 31; }
  tail -1 gpurun_out/sab_one.txt | tee -a gpurun_out/sab.txt
done
