set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  timeout -k 10 200 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/an_eager.json 2>/dev/null || exit 41
  timeout -k 10 200 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --graph > gpurun_out/an_graph.json 2>/dev/null || exit 42
  python3 -c "import json; a=json.load(open('gpurun_out/an_eager.json')); b=json.load(open('gpurun_out/an_graph.json')); print('eager %.1f %.3f  graph %.1f %.3f' % (a['value'], a['ms_per_step'], b['value'], b['ms_per_step']))"
done
