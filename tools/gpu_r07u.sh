#!/bin/bash
# C3 GDN backward on the pipelined one-wave kernel (bf16): tests, GDN timing (split: unchanged sums), C3 A/B
set -o pipefail
TAG=${1:-r07u}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_bf16_gpu.py tests/test_split_gpu.py -k "gdn or GDN or c3" > gpurun_out/gdnbf_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/gdnbf_$TAG.log; [ $rc -eq 0 ] || { echo "TESTS FAIL rc=$rc"; grep -E "Error|assert|FAIL" gpurun_out/gdnbf_$TAG.log | head -20; exit 1; }
timeout -k 10 120 python tools/gdn_bwd_time.py --sizes 128,64 > gpurun_out/gdntime_$TAG.txt 2>&1 || exit 1
timeout -k 10 120 python tools/gdn_bwd_time.py --sizes 128,64 --math 3 >> gpurun_out/gdntime_$TAG.txt 2>&1 || exit 1
IMGCOMP_LIB=$PWD/tools/_abl/oldgdnbf/libimgcomp.so timeout -k 10 120 python tools/gdn_bwd_time.py --sizes 128,64 --math 3 >> gpurun_out/gdntime_$TAG.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/gdntime_$TAG.txt
for rep in 1 2; do
  timeout -k 10 300 python bench.py --config C3 --steps 20 --warmup 5 --no-cpu-baseline --no-roofline > gpurun_out/bench_${TAG}_C3.json 2>/dev/null || { echo BENCH FAIL; exit 1; }
  cut -c1-150 gpurun_out/bench_${TAG}_C3.json
  IMGCOMP_LIB=$PWD/tools/_abl/oldgdnbf/libimgcomp.so timeout -k 10 300 python bench.py --config C3 --steps 20 --warmup 5 --no-cpu-baseline --no-roofline > gpurun_out/bench_${TAG}_C3_old.json 2>/dev/null || { echo BENCH2 FAIL; exit 1; }
  cut -c1-150 gpurun_out/bench_${TAG}_C3_old.json
done
