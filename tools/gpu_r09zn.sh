#!/bin/bash
# ig_kernel_x3d with row tile 1's A split interleaved among row tile 0's MFMAs (sched_group_barrier;
# i2 / i3: over the first 2 / 3 n-tiles) vs base: split tests on i2, x3d layers, then C2 / C4 interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
IMGCOMP_LIB=$R/tools/_abl/i2/libimgcomp.so timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_split_gpu.py tests/test_model_gpu.py > gpurun_out/tests_r09zn.log 2>&1
rc=$?; tail -2 gpurun_out/tests_r09zn.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_libab.sh r09zn_layers "g_a.2 conv,g_s.4 tconv" 2 base i2 i3 || exit 1
for i in 1 2; do
  for c in C2 C4; do
    for v in base i2 i3; do
      IMGCOMP_LIB=$R/tools/_abl/$v/libimgcomp.so timeout -k 10 200 python3 bench.py --config $c --no-cpu-baseline --no-roofline \
        > gpurun_out/r09zn_${c}_$v.json 2>gpurun_out/r09zn_${c}_$v.err || { tail gpurun_out/r09zn_${c}_$v.err; exit 1; }
      echo "$c $v $(python3 -c "import json;d=json.load(open('gpurun_out/r09zn_${c}_$v.json'));print(d['value'], d['ms_per_step'])")" | tee -a gpurun_out/r09zn_ab.txt
    done
  done
done
