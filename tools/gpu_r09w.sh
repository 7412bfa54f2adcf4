#!/bin/bash
# bf16 edge conv on two blocks per CU (grid 512) vs one (round-6 base): its tests, g_a.0 fwd / g_s.6 dgrad
# in isolation, then C3 (and C2, unaffected) interleaved twice.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_bf16_gpu.py > gpurun_out/tests_r09w.log 2>&1
rc=$?; tail -2 gpurun_out/tests_r09w.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_libab.sh r09w_layers "g_a.0 conv3->192 fwd,g_s.6 tconv192->3 dgrad" 1 base ec2 || exit 1
for i in 1 2; do
  for c in C3 C2; do
    for v in base ec2; do
      IMGCOMP_LIB=$R/tools/_abl/$v/libimgcomp.so timeout -k 10 200 python3 bench.py --config $c --no-cpu-baseline --no-roofline \
        > gpurun_out/r09w_${c}_$v.json 2>gpurun_out/r09w_${c}_$v.err || { tail gpurun_out/r09w_${c}_$v.err; exit 1; }
      echo "$c $v $(python3 -c "import json;d=json.load(open('gpurun_out/r09w_${c}_$v.json'));print(d['value'], d['ms_per_step'])")" | tee -a gpurun_out/r09w_ab.txt
    done
  done
done
