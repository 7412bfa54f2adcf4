#!/bin/bash
# r09zo follow-up: C3 three times interleaved (pass 1 of r09zo had a C3 outlier), C5 and C2 once, base vs r4.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
for c in C3 C3 C3 C5 C2; do
  for v in base r4; do
    IMGCOMP_LIB=$R/tools/_abl/$v/libimgcomp.so timeout -k 10 200 python3 bench.py --config $c --no-cpu-baseline --no-roofline \
      > gpurun_out/r09zo2_${c}_$v.json 2>gpurun_out/r09zo2_${c}_$v.err || { tail gpurun_out/r09zo2_${c}_$v.err; exit 1; }
    echo "$c $v $(python3 -c "import json;d=json.load(open('gpurun_out/r09zo2_${c}_$v.json'));print(d['value'], d['ms_per_step'])")" | tee -a gpurun_out/r09zo2_ab.txt
  done
done
