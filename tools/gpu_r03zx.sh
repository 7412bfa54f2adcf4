#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
IMGCOMP_LIB=$PWD/tools/_abl/dma2/libimgcomp.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_dma_gpu.py > gpurun_out/r03zx_t.log 2>&1; rc=$?; echo "tests(dma1 dma2) rc=$rc"; tail -2 gpurun_out/r03zx_t.log; [ $rc -eq 0 ] || exit 1
bash tools/gpu_libab.sh r03zx_ab "g_a.2 conv fwd,g_s.4 tconv fwd,g_a.2 conv dgrad,g_a.4 conv fwd" 2 dma1 dma2
bash tools/gpu_libstep.sh r03zx_step dma1 dma2
