#!/bin/bash
# MS-SSIM parity + timing, then C4 bench: concurrent vs serial hyperprior.  gpurun -- bash tools/gpu_c4ab.sh TAG ABL
set -o pipefail
TAG=$1; ABL=$2
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
  tests/test_ops_gpu.py tests/test_model_gpu.py tests/test_eval.py -k "ssim or SSIM or msssim or eval or psnr" \
  > gpurun_out/ssimtests_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/ssimtests_$TAG.log; [ $rc -eq 0 ] || { echo "TESTS FAIL rc=$rc"; grep -E "Error|assert|FAIL" gpurun_out/ssimtests_$TAG.log | head -20; exit 1; }
for lib in "" "$GRAFT_REPO_ROOT/tools/_abl/$ABL/libimgcomp.so"; do
  IMGCOMP_LIB=$lib timeout -k 10 120 python tools/msssim_time.py 2>&1 | grep -E "^lib|x3x" | tee -a gpurun_out/ssimtime_$TAG.txt || exit 1
done
for rep in 1 2; do
  for mode in "" "--serial-hyperprior"; do
    timeout -k 10 300 python bench.py --config C4 --steps 10 --warmup 3 --no-cpu-baseline --no-roofline $mode > gpurun_out/bench_${TAG}_C4$mode.json 2>/dev/null || { echo BENCH FAIL; exit 1; }
    python -c "import json,sys; r=json.load(open(sys.argv[1])); print(sys.argv[2] or 'concurrent', r['value'], r['ms_per_step'])" gpurun_out/bench_${TAG}_C4$mode.json "$mode"
  done
done
