#!/bin/bash
# ig_kernel_x3pc (x3d with the LDS-DMA on producer waves, IG_X3D_PC=1) vs ig_kernel_x3d (tools/_abl/nopc):
# DMA / split tests, C2 layer timing of every x3d op, C2 bench alternating, C2 step profile
set -o pipefail
TAG=${1:-r08g}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_dma_gpu.py tests/test_split_gpu.py > gpurun_out/t_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/t_$TAG.log; [ $rc -eq 0 ] || { echo "TESTS FAIL rc=$rc"; grep -E "Error|assert|FAIL" gpurun_out/t_$TAG.log | head -20; exit 1; }
bash tools/gpu_libab.sh layers_$TAG "g_a.2 conv,g_a.4 conv,g_s.2 tconv,g_s.4 tconv" 2 nopc || exit 1
for rep in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline > gpurun_out/bench_${TAG}_C2.json 2>gpurun_out/bench_${TAG}_C2.err || { echo BENCH FAIL; tail gpurun_out/bench_${TAG}_C2.err; exit 1; }
  cut -c1-150 gpurun_out/bench_${TAG}_C2.json
  IMGCOMP_LIB=$PWD/tools/_abl/nopc/libimgcomp.so timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline > gpurun_out/bench_${TAG}_C2_old.json 2>gpurun_out/bench_${TAG}_C2_old.err || { echo BENCH2 FAIL; tail gpurun_out/bench_${TAG}_C2_old.err; exit 1; }
  cut -c1-150 gpurun_out/bench_${TAG}_C2_old.json
done
bash tools/gpu_cfgprof.sh $TAG C2
