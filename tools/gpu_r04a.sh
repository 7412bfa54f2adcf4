#!/bin/bash
# x3d software-pipelined chunk loop: DMA-tile parity tests, then layer and C2-step A/B against the
# single-barrier loop (old) and two barrier placements
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_dma_gpu.py tests/test_bench_plans_gpu.py > gpurun_out/r04a_t.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r04a_t.log; [ $rc -eq 0 ] || exit 1
bash tools/gpu_libab.sh r04a_ab "g_a.2 conv fwd,g_s.4 tconv fwd,g_a.2 conv dgrad,g_a.4 conv fwd" 2 old jb10 jb6 || exit 1
bash tools/gpu_libstep.sh r04a_step old jb10
