#!/bin/bash
# Split-K reduction on float4 columns (ig_reduce4_kernel, in-tree = r4) vs the scalar ig_reduce_kernel (base):
# the GPU suite on the in-tree build, outputs bitwise across the two builds, the split-K layers, then
# C4 / C2 / C3 interleaved twice.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/tests_r09zo.log 2>&1
rc=$?; tail -2 gpurun_out/tests_r09zo.log; [ $rc -eq 0 ] || exit $rc
IMGCOMP_LIB=$R/tools/_abl/base/libimgcomp.so timeout -k 10 200 python3 tools/reduce4_bitwise.py --out gpurun_out/r09zo_base.pt \
  > gpurun_out/r09zo_bitwise.txt 2>&1 || { tail gpurun_out/r09zo_bitwise.txt; exit 1; }
IMGCOMP_LIB=$R/tools/_abl/r4/libimgcomp.so timeout -k 10 200 python3 tools/reduce4_bitwise.py --ref gpurun_out/r09zo_base.pt \
  >> gpurun_out/r09zo_bitwise.txt 2>&1 || { tail gpurun_out/r09zo_bitwise.txt; exit 1; }
rm -f gpurun_out/r09zo_base.pt
tail -3 gpurun_out/r09zo_bitwise.txt
bash tools/gpu_libab.sh r09zo_layers "g_a.6 conv fwd,g_s.0 tconv dgrad,g_a.4 conv fwd,g_s.2 tconv dgrad" 2 base r4 || exit 1
for i in 1 2; do
  for c in C4 C2 C3; do
    for v in base r4; do
      IMGCOMP_LIB=$R/tools/_abl/$v/libimgcomp.so timeout -k 10 200 python3 bench.py --config $c --no-cpu-baseline --no-roofline \
        > gpurun_out/r09zo_${c}_$v.json 2>gpurun_out/r09zo_${c}_$v.err || { tail gpurun_out/r09zo_${c}_$v.err; exit 1; }
      echo "$c $v $(python3 -c "import json;d=json.load(open('gpurun_out/r09zo_${c}_$v.json'));print(d['value'], d['ms_per_step'])")" | tee -a gpurun_out/r09zo_ab.txt
    done
  done
done
