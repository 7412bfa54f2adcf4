#!/bin/bash
# The new isolated b16d emulation test; ig_kernel_x3d on 64 x 96 wave tiles (IG_X3D_WM=64: 35 % fewer LDS
# fragment bytes per chunk, each A row split by two waves) vs 32 x 192, in isolation and in the C2 step.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_bf16_gpu.py -k "b16d_vs" > gpurun_out/tests_r09o.log 2>&1
rc=$?; grep -E "vs fp64|passed|failed" gpurun_out/tests_r09o.log | tail -6; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_libab.sh r09o_layers "g_a.2 conv fwd,g_a.2 conv dgrad" 2 wm64 || exit 1
for i in 1 2; do
  for v in base wm64; do
    lib=""; [ $v = base ] || lib=$R/tools/_abl/$v/libimgcomp.so
    IMGCOMP_LIB=$lib timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-roofline > gpurun_out/r09o_${v}.json 2>gpurun_out/r09o_$v.err || { tail gpurun_out/r09o_$v.err; exit 1; }
    echo "C2 $v $(python3 -c "import json;d=json.load(open('gpurun_out/r09o_${v}.json'));print(d['value'], d['ms_per_step'])")" | tee -a gpurun_out/r09o_ab.txt
  done
done
