#!/bin/bash
# r03x: double-buffered edge_wgrad: parity (edge tests, split model) + edge layer timing vs tools/_abl/oldedge
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -k "edge or model or few or C2" \
  tests/test_split_gpu.py tests/test_ops_gpu.py tests/test_bench_plans_gpu.py > gpurun_out/r03x_tests.log 2>&1 \
  || { tail -40 gpurun_out/r03x_tests.log; exit 1; }
tail -1 gpurun_out/r03x_tests.log
bash tools/gpu_libab.sh r03x_ab "g_a.0,g_s.6" 2 oldedge
