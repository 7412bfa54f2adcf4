#!/bin/bash
# MS-SSIM backward tile 32 x 22 (bth22) vs 32 x 16 (base): MS-SSIM and C4 tests, then C4 interleaved three times.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_ops_gpu.py tests/test_eval.py tests/test_bench_plans_gpu.py -k "ssim or C4 or eval" > gpurun_out/tests_r09zj.log 2>&1
rc=$?; tail -2 gpurun_out/tests_r09zj.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for v in base bth22; do
    IMGCOMP_LIB=$R/tools/_abl/$v/libimgcomp.so timeout -k 10 200 python3 bench.py --config C4 --no-cpu-baseline --no-roofline \
      > gpurun_out/r09zj_C4_$v.json 2>gpurun_out/r09zj_C4_$v.err || { tail gpurun_out/r09zj_C4_$v.err; exit 1; }
    echo "C4 $v $(python3 -c "import json;d=json.load(open('gpurun_out/r09zj_C4_$v.json'));print(d['value'], d['ms_per_step'])")" | tee -a gpurun_out/r09zj_ab.txt
  done
done
