#!/bin/bash
# Loads batched instead of serialised behind per-element branches (edge conv weight fragments, weight
# pack tiles, the implicit-GEMM epilogue's bias) vs base: conv / edge / model tests, g_a.0 and g_a.2
# forward in isolation, then C2 / C3 / C4 twice.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_split_gpu.py tests/test_bf16_gpu.py tests/test_model_gpu.py > gpurun_out/tests_r09ze.log 2>&1
rc=$?; tail -2 gpurun_out/tests_r09ze.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_libab.sh r09ze_layers "g_a.0 conv3->192 fwd,g_a.2 conv fwd" 2 base ldb || exit 1
for i in 1 2; do
  for c in C2 C3 C4; do
    for v in base ldb; do
      IMGCOMP_LIB=$R/tools/_abl/$v/libimgcomp.so timeout -k 10 200 python3 bench.py --config $c --no-cpu-baseline --no-roofline \
        > gpurun_out/r09ze_${c}_$v.json 2>gpurun_out/r09ze_${c}_$v.err || { tail gpurun_out/r09ze_${c}_$v.err; exit 1; }
      echo "$c $v $(python3 -c "import json;d=json.load(open('gpurun_out/r09ze_${c}_$v.json'));print(d['value'], d['ms_per_step'])")" | tee -a gpurun_out/r09ze_ab.txt
    done
  done
done
