#!/bin/bash
# SQ/GRBM counters of the conv kernels on one shape (tools/conv_one.py SHAPE [fwd|dgrad|wgrad|all]),
# separate passes; PMC_TAG suffixes the output directory (e.g. per kernel variant).
set -euo pipefail
SHAPE=${1:-l1}
ONLY=${2:-all}
OUT=$PWD/gpurun_out/pmc_${SHAPE}_${ONLY}${PMC_TAG:-}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
P="$GRAFT_REPO_ROOT/tools/conv_one.py $SHAPE $ONLY"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU -d "$OUT/a" -o run --output-format csv -- python3 $P
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d "$OUT/b" -o run --output-format csv -- python3 $P
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_INST_CYCLES_VMEM_RD SQ_LDS_DATA_FIFO_FULL SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC -d "$OUT/c" -o run --output-format csv -- python3 $P
echo done
