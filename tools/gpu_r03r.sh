#!/bin/bash
# r03r: x3d with split K on mid/small maps: split-arithmetic parity, then layer timing vs tools/_abl/big (x3d only >= 256 tiles)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_dma_gpu.py tests/test_split_gpu.py > gpurun_out/r03r_tests.log 2>&1 \
  || { tail -40 gpurun_out/r03r_tests.log; exit 1; }
tail -1 gpurun_out/r03r_tests.log
bash tools/gpu_libab.sh r03r_ab "conv fwd,conv dgrad,conv3x3 fwd,conv3x3 dgrad" 2 big
