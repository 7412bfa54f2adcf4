#!/bin/bash
# GDN backward: parity tests, timing of the in-tree lib against an ablation build, then optional config profiles.
#   gpurun -- bash tools/gpu_gdnb.sh TAG ABLTAG [configs...]
set -o pipefail
TAG=$1; ABL=$2; shift 2
R=$GRAFT_REPO_ROOT
cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  tests/test_split_gpu.py tests/test_ops_gpu.py tests/test_bf16_gpu.py -k "gdn or GDN" > gpurun_out/gdntests_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/gdntests_$TAG.log; [ $rc -eq 0 ] || { echo "TESTS FAIL rc=$rc"; grep -E "Error|assert|FAIL" gpurun_out/gdntests_$TAG.log | head -20; exit 1; }
timeout -k 10 120 python tools/gdn_bwd_time.py > gpurun_out/gdntime_$TAG.txt 2>&1 || { echo TIME FAIL; tail gpurun_out/gdntime_$TAG.txt; exit 1; }
IMGCOMP_LIB=$R/tools/_abl/$ABL/libimgcomp.so timeout -k 10 120 python tools/gdn_bwd_time.py >> gpurun_out/gdntime_$TAG.txt 2>&1 || { echo TIME2 FAIL; exit 1; }
timeout -k 10 120 python tools/gdn_bwd_time.py >> gpurun_out/gdntime_$TAG.txt 2>&1 || { echo TIME3 FAIL; exit 1; }
grep -v amdgpu.ids gpurun_out/gdntime_$TAG.txt
if [ -n "$FULL" ]; then
  timeout -k 10 900 python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread tests -m gpu \
    > gpurun_out/gputests_$TAG.log 2>&1; rc=$?; tail -3 gpurun_out/gputests_$TAG.log
  [ $rc -eq 0 ] || { echo "FULL TESTS rc=$rc"; grep -E "^FAILED|Error" gpurun_out/gputests_$TAG.log | head; exit 1; }
fi
[ $# -gt 0 ] && bash tools/gpu_cfgprof.sh $TAG "$@"
echo DONE
