#!/bin/bash
# producer/consumer wgrad: parity tests, layer timing vs the tap-group kernel, C2 bench.
#   gpurun -- bash tools/gpu_wgp.sh TAG ABLTAG
set -o pipefail
TAG=$1; ABL=$2
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
  tests/test_split_gpu.py tests/test_bf16_gpu.py tests/test_ops_gpu.py -k "conv or wgrad or layer" > gpurun_out/wgtests_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/wgtests_$TAG.log; [ $rc -eq 0 ] || { echo "TESTS FAIL rc=$rc"; grep -E "Error|assert|FAIL" gpurun_out/wgtests_$TAG.log | head -20; exit 1; }
bash tools/gpu_libab.sh wgtime_$TAG "g_a.2 conv wgrad,g_s.4 tconv wgrad,g_a.4 conv wgrad,g_s.2 tconv wgrad" 2 $ABL || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo BENCH FAIL; exit 1; }
cut -c1-220 gpurun_out/bench_$TAG.json
