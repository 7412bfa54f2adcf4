#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_split_gpu.py tests/test_ops_gpu.py -k "gdn" > gpurun_out/r03zt_t.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r03zt_t.log; [ $rc -eq 0 ] || exit 1
bash tools/gpu_libab.sh r03zt_ab "gdn_bwd" 2 oldgdn
