#!/bin/bash
# Model-level A/B of planner / kernel env settings: one bench line per setting.
#   CONFIGS="ENV1=a ENV2=b;ENV1=c" bash tools/ab_bench.sh
set -uo pipefail
IFS=';' read -ra CFG <<< "${CONFIGS:-}"
for c in "" "${CFG[@]}"; do
  out=$(env $c timeout -k 10 150 python3 bench.py --steps ${STEPS:-30} --warmup 5 --no-cpu-baseline --no-probe 2>/dev/null | tail -1) || { echo "[$c] failed"; exit 1; }
  echo "[${c:-default}] $(echo "$out" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], "img/s", d["ms_per_step"], "ms")')"
done
