#!/bin/bash
# r03w: full GPU suite + smoke + C2 bench + rocprof, then C3/C4/C5 bench lines
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_check.sh r03w || exit 1
for c in C3 C4 C5; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_r03w_$c.json 2> gpurun_out/bench_r03w_$c.err || { echo "BENCH FAIL $c"; tail -20 gpurun_out/bench_r03w_$c.err; exit 1; }
  python -c "import json; r=json.load(open('gpurun_out/bench_r03w_$c.json')); print('$c', r['value'], r['ms_per_step'])"
done
