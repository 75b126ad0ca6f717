# timing-only variants of the halo kernel (MD2_HX_DBG: 1 no A loads, 2 no staging, 4 no MFMA)
set -o pipefail
T=${1:-hxdbg_l1}
cd /tmp && export TMPDIR=/tmp
for d in 0 1 2 3 4 6; do
  MD2_TUNING=1 MD2_HX_DBG=$d timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_${T}_$d -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/bench_conv.py --only=l1,l2 > /dev/null 2>&1 || exit 20
done
cd $GRAFT_REPO_ROOT
for d in 0 1 2 3 4 6; do echo "DBG=$d"; python3 tools/halo_shapes.py gpurun_out/prof_${T}_$d | grep halo3; done
