#!/bin/bash
# r03j: 256-row split tiles: parity (wide tests, bench-plan step tests), layer timing vs x3s<128> (tools/_abl/nohalo)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v -s --durations=0 --timeout 300 --timeout-method thread \
  tests/test_wide_gpu.py tests/test_bench_plans_gpu.py > gpurun_out/r03j_tests.log 2>&1 \
  || { tail -40 gpurun_out/r03j_tests.log; exit 1; }
grep -E "256-row|passed|failed|s call" gpurun_out/r03j_tests.log | tail -20
bash tools/gpu_libab.sh r03j_ab "g_a.2 conv fwd,g_a.2 conv dgrad,g_s.4 tconv fwd,g_s.4 tconv dgrad" 2 nohalo
