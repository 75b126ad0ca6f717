# timing-only whalo variants (MD2_WHX_DBG) on the layer-2 shape: kernel time per variant
set -o pipefail
mkdir -p gpurun_out
T=${1:-whxdbg}
cd /tmp && export TMPDIR=/tmp
for d in 0 1 2 3 4 8 11 12; do
  MD2_TUNING=1 MD2_WHX_DBG=$d timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_${T}_$d -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/bench_conv.py --only=l2 > /dev/null 2>&1 || exit 21
  python3 - "$GRAFT_REPO_ROOT/gpurun_out/prof_${T}_$d" "$d" <<'PY'
import csv, glob, sys
p = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(p)):
    if "whalo" in r["Name"]:
        print(f"DBG={sys.argv[2]:>2s}  {r['Name'][:50]:50s} avg {float(r['AverageNs'])/1e3:7.1f} us  min {float(r['MinNs'])/1e3:7.1f}")
PY
done
