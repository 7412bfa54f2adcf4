#!/bin/bash
# GPU tests for the precision modes, then one bench line per BASELINE config.  usage: bash tools/gpu_configs.sh TAG
set -o pipefail
TAG=${1:-cfg}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_bf16_gpu.py tests/test_split_gpu.py -x -q -p no:cacheprovider > gpurun_out/cfgtests_$TAG.log 2>&1 || { echo "TESTS FAIL"; tail -30 gpurun_out/cfgtests_$TAG.log; exit 1; }
tail -1 gpurun_out/cfgtests_$TAG.log
for c in C2 C3 C4 C5; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_${TAG}_$c.json 2> gpurun_out/bench_${TAG}_$c.err || { echo "BENCH FAIL $c"; tail -20 gpurun_out/bench_${TAG}_$c.err; exit 1; }
  cut -c1-250 gpurun_out/bench_${TAG}_$c.json
done
