#!/bin/bash
# MS-SSIM: parity tests, timing against an ablation build, C4 bench + profile.  gpurun -- bash tools/gpu_ssim.sh TAG ABL
set -o pipefail
TAG=$1; ABL=$2
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
  tests/test_ops_gpu.py tests/test_model_gpu.py tests/test_eval.py tests/test_bench_plans_gpu.py -k "ssim or SSIM or msssim or C4 or eval or psnr" \
  > gpurun_out/ssimtests_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/ssimtests_$TAG.log; [ $rc -eq 0 ] || { echo "TESTS FAIL rc=$rc"; grep -E "Error|assert|FAIL" gpurun_out/ssimtests_$TAG.log | head -20; exit 1; }
for lib in "" "$GRAFT_REPO_ROOT/tools/_abl/$ABL/libimgcomp.so" ""; do
  IMGCOMP_LIB=$lib timeout -k 10 120 python tools/msssim_time.py 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/ssimtime_$TAG.txt || exit 1
done
bash tools/gpu_cfgprof.sh $TAG C4
