#!/bin/bash
# End-of-round measurement pass on ONE MI355X (run under gpurun from the repo root):
#   the -m gpu suite, the default bench line, the rocprof/PMC profile (profile_round.sh TAG),
#   the DP overlap tables at configs 4 and 5, configs 1 / 2 / 5 and the MPI step.
# Every step has its own time limit; the script stops at the first failure.
TAG=${1:?tag}
mkdir -p gpurun_out
# SKIP_SUITE=1: the suite already ran green on this build
if [ -z "${SKIP_SUITE:-}" ]; then NO_PROFILE=1 bash tools/gpu_check.sh $TAG || exit $?; fi
timeout -k 10 300 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 11
bash tools/profile_round.sh $TAG > /dev/null 2>&1 || exit 12
timeout -k 10 200 python -u tools/dp_overlap.py gpurun_out/dp_overlap_c4_$TAG.json > /dev/null 2>&1 || exit 13
timeout -k 10 200 python -u tools/dp_overlap.py gpurun_out/dp_overlap_c5_$TAG.json --arch 50 --height 192 --width 640 --batch 8 > /dev/null 2>&1 || exit 14
timeout -k 10 300 python -u tools/configs_bench.py > gpurun_out/configs_$TAG.jsonl 2> gpurun_out/configs_$TAG.err || exit 15
timeout -k 10 300 python -u bench.py --arch 50 --width 640 --height 192 --batch 8 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_c5_$TAG.json 2> gpurun_out/bench_c5_$TAG.err || exit 16
timeout -k 10 200 python -u tools/bench_mpi.py --layers gpurun_out/mpi_layers_$TAG.md > gpurun_out/mpi_$TAG.json 2> gpurun_out/mpi_$TAG.err || exit 17
python3 -c "import json;d=json.load(open('gpurun_out/bench_$TAG.json'));print('bench', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline_photometric']['frac'])"
echo "round_final done"
