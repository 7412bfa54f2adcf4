#!/bin/bash
# bf16 weight gradients from the bf16 copies (C3): tests, layer timing, C3 A/B vs WG_X3P_B16=0
set -o pipefail
TAG=${1:-r07y}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_bf16_gpu.py tests/test_bench_plans_gpu.py > gpurun_out/b16w_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/b16w_$TAG.log; [ $rc -eq 0 ] || { echo "TESTS FAIL rc=$rc"; grep -E "Error|assert|FAIL" gpurun_out/b16w_$TAG.log | head -20; exit 1; }
for rep in 1 2; do
  timeout -k 10 300 python bench.py --config C3 --steps 20 --warmup 5 --no-cpu-baseline --no-roofline > gpurun_out/bench_${TAG}_C3.json 2>/dev/null || { echo BENCH FAIL; exit 1; }
  cut -c1-150 gpurun_out/bench_${TAG}_C3.json
  IMGCOMP_LIB=$PWD/tools/_abl/nowgb16/libimgcomp.so timeout -k 10 300 python bench.py --config C3 --steps 20 --warmup 5 --no-cpu-baseline --no-roofline > gpurun_out/bench_${TAG}_C3_old.json 2>/dev/null || { echo BENCH2 FAIL; exit 1; }
  cut -c1-150 gpurun_out/bench_${TAG}_C3_old.json
done
bash tools/gpu_cfgprof.sh $TAG C3
