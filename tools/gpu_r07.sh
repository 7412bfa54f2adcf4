#!/bin/bash
# Round-5 milestone check: full GPU suite + smoke + C2 bench + rocprof (gpu_check.sh), then bench lines of
# the configs given (default C4).  gpurun -- bash tools/gpu_r07.sh TAG [configs...]
set -o pipefail
TAG=${1:-r07}; shift
cd $GRAFT_REPO_ROOT
bash tools/gpu_check.sh $TAG || exit 1
grep -q "TESTS EXIT 0" gpurun_out/tests_$TAG.log || { grep -E "^FAILED" gpurun_out/tests_$TAG.log | head; exit 1; }
for c in ${@:-C4}; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_${TAG}_$c.json 2> gpurun_out/bench_${TAG}_$c.err || { echo "BENCH FAIL $c"; exit 1; }
  cut -c1-200 gpurun_out/bench_${TAG}_$c.json
done
