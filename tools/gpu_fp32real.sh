set -o pipefail
T=${1:-f32r}
mkdir -p gpurun_out
timeout -k 10 900 python3 -u tools/fp32_realizations.py --out gpurun_out/${T}.json > gpurun_out/${T}.txt 2>&1; rc=$?
head -60 gpurun_out/${T}.txt; tail -3 gpurun_out/${T}.txt; exit $rc
