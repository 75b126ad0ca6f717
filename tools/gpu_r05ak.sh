set -o pipefail
mkdir -p gpurun_out
T=${1:-r05ak}
timeout -k 10 200 python3 tools/step_digest.py 12 3 > gpurun_out/digest_${T}_default.txt 2>&1 || exit 31
MD2_TUNING=1 MD2_HEAD_ROWS=1 timeout -k 10 200 python3 tools/step_digest.py 12 3 > gpurun_out/digest_${T}_rows.txt 2>&1 || exit 32
MD2_TUNING=1 MD2_HEAD_ROWS=1 timeout -k 10 200 python3 tools/step_digest.py 2 3 > gpurun_out/digest_${T}_rows_b2.txt 2>&1 || exit 33
timeout -k 10 200 python3 tools/step_digest.py 2 3 > gpurun_out/digest_${T}_default_b2.txt 2>&1 || exit 34
tail -1 gpurun_out/digest_${T}_default.txt; tail -1 gpurun_out/digest_${T}_rows.txt; tail -1 gpurun_out/digest_${T}_default_b2.txt; tail -1 gpurun_out/digest_${T}_rows_b2.txt
SKIP_TESTS=1 bash tools/gpu_ab.sh $T default "MD2_HEAD_ROWS=1" "MD2_SEG_UPDATE=1" "MD2_HX_TARGET=384" || exit 27
