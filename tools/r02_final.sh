#!/bin/bash
# End-of-round measurement on one MI355X: tests + bench + profile (tools/r02_check.sh TAG), the
# per-layer conv table, configs 1/2 and config 5 per GPU.  Results under gpurun_out/.
set -o pipefail
TAG=${1:-r02f}
bash tools/r02_check.sh $TAG || exit 1
timeout -k 10 300 python tools/layer_table.py $TAG > gpurun_out/layers.log 2>&1 || { tail -5 gpurun_out/layers.log; exit 1; }
cp profiles/${TAG}_layers.md gpurun_out/ || exit 1
timeout -k 10 400 python tools/configs_bench.py > gpurun_out/configs.jsonl 2> gpurun_out/configs.err || { tail -5 gpurun_out/configs.err; exit 1; }
timeout -k 10 300 python bench.py --arch 50 --width 640 --height 192 --batch 8 --no-cpu-baseline > gpurun_out/bench_r50.json 2> gpurun_out/bench_r50.err || exit 1
cat gpurun_out/configs.jsonl gpurun_out/bench_r50.json
