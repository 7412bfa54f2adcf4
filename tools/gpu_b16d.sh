#!/bin/bash
# bf16 DMA conv (C3): parity tests, layer timing vs ig_kernel_bf16 (nob16d), C3 bench.
set -o pipefail
TAG=${1:-r07n}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_bf16_gpu.py tests/test_bench_plans_gpu.py > gpurun_out/b16tests_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/b16tests_$TAG.log; [ $rc -eq 0 ] || { echo "TESTS FAIL rc=$rc"; grep -E "Error|assert|FAIL" gpurun_out/b16tests_$TAG.log | head -20; exit 1; }
bash tools/gpu_libab.sh b16time_$TAG "g_a.2 conv fwd,g_a.4 conv fwd,g_s.2 tconv dgrad,g_s.4 tconv dgrad" 1 nob16d || exit 1
timeout -k 10 300 python bench.py --config C3 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_${TAG}_C3.json 2> gpurun_out/bench_${TAG}_C3.err || { echo BENCH FAIL; tail gpurun_out/bench_${TAG}_C3.err; exit 1; }
cut -c1-220 gpurun_out/bench_${TAG}_C3.json
IMGCOMP_LIB=$PWD/tools/_abl/nob16d/libimgcomp.so timeout -k 10 300 python bench.py --config C3 --steps 20 --warmup 5 --no-cpu-baseline --no-roofline > gpurun_out/bench_${TAG}_C3_nob16d.json 2>/dev/null || { echo BENCH2 FAIL; exit 1; }
cut -c1-220 gpurun_out/bench_${TAG}_C3_nob16d.json
