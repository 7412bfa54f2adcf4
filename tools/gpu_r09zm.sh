#!/bin/bash
# tconv_few2 with compile-time channel / tap counts for Cin 192, k 5 (tf2) vs base: tests, g_s.6 fwd in
# isolation (split and bf16), then C2 / C3 interleaved twice.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_split_gpu.py tests/test_bf16_gpu.py tests/test_model_gpu.py > gpurun_out/tests_r09zm.log 2>&1
rc=$?; tail -2 gpurun_out/tests_r09zm.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_libab.sh r09zm_layers "g_s.6 tconv192->3 fwd" 2 base tf2 || exit 1
bash tools/gpu_libab.sh r09zm_layers_bf16 "g_s.6 tconv192->3 fwd" 1 base tf2 || exit 1
for i in 1 2; do
  for c in C3 C2; do
    for v in base tf2; do
      IMGCOMP_LIB=$R/tools/_abl/$v/libimgcomp.so timeout -k 10 200 python3 bench.py --config $c --no-cpu-baseline --no-roofline \
        > gpurun_out/r09zm_${c}_$v.json 2>gpurun_out/r09zm_${c}_$v.err || { tail gpurun_out/r09zm_${c}_$v.err; exit 1; }
      echo "$c $v $(python3 -c "import json;d=json.load(open('gpurun_out/r09zm_${c}_$v.json'));print(d['value'], d['ms_per_step'])")" | tee -a gpurun_out/r09zm_ab.txt
    done
  done
done
