#!/bin/bash
# Counters of the loss-tail kernels (photometric_kernel et al.) at the bench shape, one pass per
# counter group (tools/photo_one.py N iters).  Usage: tools/pmc_photo.sh TAG [N...]
# Output: gpurun_out/pmc_photo_<TAG>/<N>/{trace,a,b,c,fetch,write}; summarise with
#   python tools/pmc_report.py gpurun_out/pmc_photo_<TAG>/<N>
set -euo pipefail
TAG=${1:-cur}
shift || true
NS=${*:-12 96}
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for N in $NS; do
  OUT=$R/gpurun_out/pmc_photo_$TAG/$N
  mkdir -p "$OUT"
  P="$R/tools/photo_one.py $N 6"
  timeout -k 10 120 python3 $P > "$OUT/plain.txt" 2>&1
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 $P > /dev/null
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU -d "$OUT/a" -o run --output-format csv -- python3 $P > /dev/null
  timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d "$OUT/b" -o run --output-format csv -- python3 $P > /dev/null
  timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_FLAT SQ_INST_LEVEL_LDS SQ_WAIT_INST_ANY -d "$OUT/c" -o run --output-format csv -- python3 $P > /dev/null
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv -- python3 $P > /dev/null
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv -- python3 $P > /dev/null
done
echo "pmc done"
