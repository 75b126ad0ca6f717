#!/bin/bash
# Per-round profile of the bench on ONE MI355X (run on the GPU box from the repo root):
#   1. rocprofv3 --kernel-trace --stats  (per-kernel time; must agree with bench.py's HIP events)
#   2. two separate --pmc passes: FETCH_SIZE, WRITE_SIZE (HBM traffic; MI355X_MICROARCH.md HBM)
# Outputs under gpurun_out/prof_<tag>/; tools/prof_summary.py condenses them into profiles/.
set -euo pipefail
TAG=${1:-r01}
STEPS=${STEPS:-10}
OUT=$PWD/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
BENCH="$GRAFT_REPO_ROOT/bench.py --steps $STEPS --warmup 3 --no-cpu-baseline"
timeout -k 10 300 python3 $BENCH > "$OUT/bench_plain.json"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 $BENCH --no-probe > "$OUT/bench_trace.json"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv -- python3 $BENCH --no-probe > "$OUT/bench_fetch.json"
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv -- python3 $BENCH --no-probe > "$OUT/bench_write.json"
# MFMA pipe occupancy of every kernel (SQ_VALU_MFMA_BUSY_CYCLES over GRBM_GUI_ACTIVE / 8 x 1024 SIMDs)
timeout -k 10 400 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_BUSY_CYCLES -d "$OUT/mfma" -o run --output-format csv -- python3 $BENCH --no-probe > "$OUT/bench_mfma.json"
echo "profile done: $OUT"
