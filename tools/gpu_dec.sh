set -o pipefail
mkdir -p gpurun_out
T=${1:-dec}
cd /tmp && export TMPDIR=/tmp
for v in "default" "MD2_HALO_RFL_DGRAD=0"; do
MD2_TUNING=1 env $( [ "$v" = default ] || echo $v ) timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_${T}_${v%%=*} -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/bench_conv.py --only=d1c1,d1c2,d2c1,d2c2,d3c1,d3c2,d4c1 > $GRAFT_REPO_ROOT/gpurun_out/bench_conv_${T}_${v%%=*}.txt 2>&1 || exit 21
done
cd $GRAFT_REPO_ROOT
grep -hE "^d[0-9]" gpurun_out/bench_conv_${T}_*.txt
