#!/bin/bash
# Transposed convs' four phases on the DMA tiles with K split (IG_X3D_MPH, in-tree) vs the 64-row register-
# staged tiles (tools/_abl/mph0): whole-step parity at the bench batch, layer times, C2/C3/C4 alternating.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread -p no:cacheprovider \
  tests/test_bench_plans_gpu.py tests/test_split_gpu.py > gpurun_out/tests_r09l.log 2>&1
rc=$?; tail -3 gpurun_out/tests_r09l.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/tests_r09l.log | head -20; exit $rc; }
bash tools/gpu_libab.sh r09l_layers "g_s.0 tconv,g_a.6 conv dgrad,g_s.2 tconv" 2 mph0 || exit 1
for c in C2 C3 C4; do
  for i in 1 2; do
    for v in base mph0; do
      lib=""; [ $v = base ] || lib=$R/tools/_abl/$v/libimgcomp.so
      IMGCOMP_LIB=$lib timeout -k 10 200 python3 bench.py --config $c --no-cpu-baseline --no-roofline > gpurun_out/r09l_${c}_${v}.json 2>gpurun_out/r09l_$v.err || { tail gpurun_out/r09l_$v.err; exit 1; }
      echo "$c $v $(python3 -c "import json;d=json.load(open('gpurun_out/r09l_${c}_${v}.json'));print(d['value'], d['ms_per_step'])")" | tee -a gpurun_out/r09l_ab.txt
    done
  done
done
