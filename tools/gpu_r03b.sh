#!/bin/bash
# r03b: parity of the register-A split implicit GEMM + timing vs ig_kernel_x3s + determinism probes
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_split_gpu.py tests/test_bench_plans_gpu.py tests/test_model_gpu.py \
  tests/test_ddp_gpu.py tests/test_step_gpu.py tests/test_threads_gpu.py -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/t_r03b.log 2>&1
rc=$?; tail -8 gpurun_out/t_r03b.log; [ $rc -le 1 ] || exit $rc
bash tools/gpu_libab.sh ab_x3r "g_a.2 conv fwd,g_a.2 conv dgrad,g_s.4 tconv fwd,g_s.4 tconv dgrad" 2 x3s || exit 1
timeout -k 10 300 python tools/determinism_probe.py --reps 6 > gpurun_out/det_r03b.log 2>&1 || exit 1
tail -12 gpurun_out/det_r03b.log
PYTORCH_NO_CUDA_MEMORY_CACHING=1 timeout -k 10 300 python tools/determinism_probe.py --reps 6 > gpurun_out/det_nocache_r03b.log 2>&1 || exit 1
tail -4 gpurun_out/det_nocache_r03b.log
