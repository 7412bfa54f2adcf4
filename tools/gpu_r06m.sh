#!/bin/bash
# Round-5 milestone: full GPU suite + smoke + C2 bench + rocprof (gpu_check.sh), the other configs'
# bench lines, then the PMC passes of the round-5 kernels.
set -o pipefail
TAG=${1:-r06m}
cd $GRAFT_REPO_ROOT
bash tools/gpu_check.sh $TAG || exit 1
for c in C3 C4 C5; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_${TAG}_$c.json 2> gpurun_out/bench_${TAG}_$c.err || { echo "BENCH FAIL $c"; exit 1; }
  cut -c1-200 gpurun_out/bench_${TAG}_$c.json
done
bash tools/gpu_pmc_r06.sh pmc_$TAG
