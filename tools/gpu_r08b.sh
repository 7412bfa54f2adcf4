#!/bin/bash
# ig_kernel_b16r (ring of 32-channel slots, DMA S-1 chunks ahead) vs ig_kernel_b16d (tools/_abl/nob16r):
# bf16 tests, C3 layer timing, C3 bench alternating, C3 step profile
set -o pipefail
TAG=${1:-r08b}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_bf16_gpu.py tests/test_bench_plans_gpu.py > gpurun_out/t_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/t_$TAG.log; [ $rc -eq 0 ] || { echo "TESTS FAIL rc=$rc"; grep -E "Error|assert|FAIL" gpurun_out/t_$TAG.log | head -20; exit 1; }
bash tools/gpu_libab.sh layers_$TAG "g_a.2 conv,g_a.4 conv,g_s.2 tconv,g_s.4 tconv" 1 nob16r || exit 1
for rep in 1 2; do
  timeout -k 10 300 python bench.py --config C3 --steps 20 --warmup 5 --no-cpu-baseline --no-roofline > gpurun_out/bench_${TAG}_C3.json 2>gpurun_out/bench_${TAG}_C3.err || { echo BENCH FAIL; tail gpurun_out/bench_${TAG}_C3.err; exit 1; }
  cut -c1-150 gpurun_out/bench_${TAG}_C3.json
  IMGCOMP_LIB=$PWD/tools/_abl/nob16r/libimgcomp.so timeout -k 10 300 python bench.py --config C3 --steps 20 --warmup 5 --no-cpu-baseline --no-roofline > gpurun_out/bench_${TAG}_C3_old.json 2>gpurun_out/bench_${TAG}_C3_old.err || { echo BENCH2 FAIL; tail gpurun_out/bench_${TAG}_C3_old.err; exit 1; }
  cut -c1-150 gpurun_out/bench_${TAG}_C3_old.json
done
bash tools/gpu_cfgprof.sh $TAG C3
