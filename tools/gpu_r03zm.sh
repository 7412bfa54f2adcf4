#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_split_gpu.py tests/test_ops_gpu.py tests/test_bench_plans_gpu.py > gpurun_out/r03zm_t.log 2>&1; echo "tests rc=$?"; tail -3 gpurun_out/r03zm_t.log
bash tools/gpu_libab.sh r03zm_ab "g_a.0 conv3->192 fwd,g_s.6 tconv192->3 dgrad,g_a.0 conv3->192 wgrad" 2
