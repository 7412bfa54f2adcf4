#!/bin/bash
# g_s.6 forward (tconv_few2_kernel) grid in one round of 256 blocks: edge / split tests, C5 bench + profile
set -o pipefail
TAG=${1:-r08e}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_split_gpu.py tests/test_bench_plans_gpu.py > gpurun_out/t_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/t_$TAG.log; [ $rc -eq 0 ] || { echo "TESTS FAIL rc=$rc"; grep -E "Error|assert|FAIL" gpurun_out/t_$TAG.log | head -20; exit 1; }
bash tools/gpu_cfgprof.sh $TAG C5 C2
