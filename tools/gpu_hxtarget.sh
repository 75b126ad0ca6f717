# halo kernel split target A/B (MD2_HX_TARGET blocks), same box
set -o pipefail
T=${1:-hxt}
cd /tmp && export TMPDIR=/tmp
for t in 512 256 384; do
  MD2_TUNING=1 MD2_HX_TARGET=$t timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_${T}_$t -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/bench_conv.py --only=l1,l2,l3,l4 > /dev/null 2>&1 || exit 20
done
cd $GRAFT_REPO_ROOT
for t in 512 256 384; do echo "TARGET=$t"; python3 tools/halo_shapes.py gpurun_out/prof_${T}_$t | grep halo3; done
