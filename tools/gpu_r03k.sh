#!/bin/bash
# r03k: parity of 256-row split tiles and bf16 weight gradients; layer A/B vs x3s<128>; C3 bench + rocprof
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -s --durations=0 --timeout 300 --timeout-method thread \
  tests/test_bf16_gpu.py tests/test_bench_plans_gpu.py -k "bf16 or C3" > gpurun_out/r03k_tests.log 2>&1 \
  || { tail -40 gpurun_out/r03k_tests.log; exit 1; }
grep -E "256-row|bf16 wgrad|C3:|passed|failed" gpurun_out/r03k_tests.log | tail -20
true
timeout -k 10 300 python bench.py --config C3 --steps 10 --warmup 3 > gpurun_out/r03k_bench_C3.json 2> gpurun_out/r03k_bench_C3.err || { tail -20 gpurun_out/r03k_bench_C3.err; exit 1; }
cat gpurun_out/r03k_bench_C3.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r03k_prof_C3 -o p --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config C3 --steps 5 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/r03k_prof_C3.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/r03k_prof_C3.log; exit 1; }
echo DONE
