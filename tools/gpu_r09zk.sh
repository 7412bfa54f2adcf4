#!/bin/bash
# MS-SSIM loss fwd+bwd at C4's shape, base vs 32 x 22 backward tiles, alternating, plus the C4 step.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
for i in 1 2 3; do
  for v in base bth22; do
    echo -n "$v: " | tee -a gpurun_out/r09zk.txt
    IMGCOMP_LIB=$R/tools/_abl/$v/libimgcomp.so timeout -k 10 120 python3 tools/ssim_time.py 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/r09zk.txt || exit 1
  done
done
for i in 1 2; do
  for v in base bth22; do
    IMGCOMP_LIB=$R/tools/_abl/$v/libimgcomp.so timeout -k 10 200 python3 bench.py --config C4 --no-cpu-baseline --no-roofline \
      > gpurun_out/r09zk_C4_$v.json 2>gpurun_out/r09zk_C4_$v.err || { tail gpurun_out/r09zk_C4_$v.err; exit 1; }
    echo "C4 $v $(python3 -c "import json;d=json.load(open('gpurun_out/r09zk_C4_$v.json'));print(d['value'], d['ms_per_step'])")" | tee -a gpurun_out/r09zk.txt
  done
done
