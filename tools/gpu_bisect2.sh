set -o pipefail
T=${1:-bis2}
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/forward_bisect.py --out gpurun_out/${T}_default.json > gpurun_out/${T}_default.txt 2>&1 || exit 11
cat gpurun_out/${T}_default.txt
