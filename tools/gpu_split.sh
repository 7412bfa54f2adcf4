#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_split_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/split_tests.log 2>&1
rc=$?; tail -15 gpurun_out/split_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/layer_bench.py --math 2 > gpurun_out/layers_x3.txt 2>&1 || exit $?
cat gpurun_out/layers_x3.txt
