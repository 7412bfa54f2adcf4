#!/bin/bash
# Split-K reduction with all partial loads (and the bias) issued together (igr) vs base: conv / model /
# whole-step tests, the split-K layers in isolation, then C2 / C3 / C4 interleaved twice.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_split_gpu.py tests/test_bf16_gpu.py tests/test_model_gpu.py tests/test_bench_plans_gpu.py > gpurun_out/tests_r09zl.log 2>&1
rc=$?; tail -2 gpurun_out/tests_r09zl.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_libab.sh r09zl_layers "g_a.6 conv fwd,g_s.0 tconv dgrad" 2 base igr || exit 1
for i in 1 2; do
  for c in C4 C2 C3; do
    for v in base igr; do
      IMGCOMP_LIB=$R/tools/_abl/$v/libimgcomp.so timeout -k 10 200 python3 bench.py --config $c --no-cpu-baseline --no-roofline \
        > gpurun_out/r09zl_${c}_$v.json 2>gpurun_out/r09zl_${c}_$v.err || { tail gpurun_out/r09zl_${c}_$v.err; exit 1; }
      echo "$c $v $(python3 -c "import json;d=json.load(open('gpurun_out/r09zl_${c}_$v.json'));print(d['value'], d['ms_per_step'])")" | tee -a gpurun_out/r09zl_ab.txt
    done
  done
done
