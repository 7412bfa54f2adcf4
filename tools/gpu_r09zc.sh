#!/bin/bash
# Edge wgrad with its G tile double-buffered (one block per CU) vs base (single buffer, two blocks per
# CU): tests, g_a.0 / g_s.6 weight gradients in isolation (split and bf16), then C2 / C3 twice.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_split_gpu.py tests/test_bf16_gpu.py > gpurun_out/tests_r09zc.log 2>&1
rc=$?; tail -2 gpurun_out/tests_r09zc.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_libab.sh r09zc_layers "g_a.0 conv3->192 wgrad,g_s.6 tconv192->3 wgrad" 2 base ewdb || exit 1
bash tools/gpu_libab.sh r09zc_layers_bf16 "g_a.0 conv3->192 wgrad,g_s.6 tconv192->3 wgrad" 1 base ewdb || exit 1
for i in 1 2; do
  for c in C3 C2; do
    for v in base ewdb; do
      IMGCOMP_LIB=$R/tools/_abl/$v/libimgcomp.so timeout -k 10 200 python3 bench.py --config $c --no-cpu-baseline --no-roofline \
        > gpurun_out/r09zc_${c}_$v.json 2>gpurun_out/r09zc_${c}_$v.err || { tail gpurun_out/r09zc_${c}_$v.err; exit 1; }
      echo "$c $v $(python3 -c "import json;d=json.load(open('gpurun_out/r09zc_${c}_$v.json'));print(d['value'], d['ms_per_step'])")" | tee -a gpurun_out/r09zc_ab.txt
    done
  done
done
