#!/bin/bash
# x3d two wave groups a half-step apart (IG_X3D_PP = lag in n-tiles): DMA-tile parity under the variant, layer and C2-step A/B
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
IMGCOMP_LIB=$PWD/tools/_abl/pp3/libimgcomp.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_dma_gpu.py > gpurun_out/r04d_t.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r04d_t.log; [ $rc -eq 0 ] || exit 1
bash tools/gpu_libab.sh r04d_ab "g_a.2 conv fwd,g_s.4 tconv fwd,g_a.2 conv dgrad,g_a.4 conv fwd" 2 pp2 pp3 pp4 || exit 1
bash tools/gpu_libstep.sh r04d_step pp3
