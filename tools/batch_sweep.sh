#!/bin/bash
# Batch sweep of the train step on ONE MI355X (B up to 96 per GPU), one bench line
# per batch size into gpurun_out/sweep.jsonl.
set -uo pipefail
OUT=${OUT:-gpurun_out/sweep.jsonl}
: > "$OUT"
for B in ${BATCHES:-6 12 24 48 96}; do
  timeout -k 10 200 python3 bench.py --batch "$B" --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline >> "$OUT" \
    || { echo "batch $B failed"; exit 1; }
  echo "batch $B done"
done
