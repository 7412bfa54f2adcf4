#!/bin/bash
# bf16 copies from the GDN kernels (C3): tests, C3 bench vs IG_B16D=0, C3 step profile
set -o pipefail
TAG=${1:-r07p}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_bf16_gpu.py tests/test_bench_plans_gpu.py > gpurun_out/b16tests_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/b16tests_$TAG.log; [ $rc -eq 0 ] || { echo "TESTS FAIL rc=$rc"; grep -E "Error|assert|FAIL" gpurun_out/b16tests_$TAG.log | head -20; exit 1; }
for rep in 1 2; do
timeout -k 10 300 python bench.py --config C3 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_${TAG}_C3.json 2> gpurun_out/bench_${TAG}_C3.err || { echo BENCH FAIL; tail gpurun_out/bench_${TAG}_C3.err; exit 1; }
cut -c1-160 gpurun_out/bench_${TAG}_C3.json
IMGCOMP_LIB=$PWD/tools/_abl/nob16d/libimgcomp.so timeout -k 10 300 python bench.py --config C3 --steps 20 --warmup 5 --no-cpu-baseline --no-roofline > gpurun_out/bench_${TAG}_C3_nob16d.json 2>/dev/null || { echo BENCH2 FAIL; exit 1; }
cut -c1-160 gpurun_out/bench_${TAG}_C3_nob16d.json
done
bash tools/gpu_cfgprof.sh $TAG C3
