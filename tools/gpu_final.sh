#!/bin/bash
# end-of-round check: full GPU suite + smoke + C2 bench + rocprof (gpu_check.sh), C3/C4/C5 bench lines
#   gpurun -- bash tools/gpu_final.sh TAG
set -o pipefail
TAG=${1:-final}
cd $GRAFT_REPO_ROOT
bash tools/gpu_check.sh $TAG || exit 1
grep -q "TESTS EXIT 0" gpurun_out/tests_$TAG.log || { grep -E "^FAILED" gpurun_out/tests_$TAG.log | head; exit 1; }
for c in C3 C4 C5; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_${TAG}_$c.json 2> gpurun_out/bench_${TAG}_$c.err || { echo "BENCH FAIL $c"; exit 1; }
  cut -c1-200 gpurun_out/bench_${TAG}_$c.json
done
