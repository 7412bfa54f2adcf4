#!/bin/bash
# r03h: halo kernel parity (new halo tests, plan tests at C2 shapes, split tests), then layer timing
# in-tree (halo) against tools/_abl/nohalo (ig_kernel_x3s)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -v -s --durations=0 --timeout 600 --timeout-method thread \
  tests/test_bench_plans_gpu.py -k C5 tests/test_split_gpu.py > gpurun_out/r03h_tests.log 2>&1 \
  || { tail -40 gpurun_out/r03h_tests.log; exit 1; }
grep -E "halo|passed|failed|s call" gpurun_out/r03h_tests.log | tail -20
bash tools/gpu_libab.sh r03h_ab "g_a.2 conv fwd,g_a.2 conv dgrad,g_s.4 tconv fwd,g_s.4 tconv dgrad,g_a.1 conv fwd,g_s.3 tconv fwd" 2 nohalo
