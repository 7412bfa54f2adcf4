#!/bin/bash
# C2 / C4 three-way: base, all three load-batching changes (ldb), and without the pack change (ldb2).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
for i in 1 2 3; do
  for c in C2 C4; do
    for v in base ldb ldb2; do
      IMGCOMP_LIB=$R/tools/_abl/$v/libimgcomp.so timeout -k 10 200 python3 bench.py --config $c --no-cpu-baseline --no-roofline \
        > gpurun_out/r09zf_${c}_$v.json 2>gpurun_out/r09zf_${c}_$v.err || { tail gpurun_out/r09zf_${c}_$v.err; exit 1; }
      echo "$c $v $(python3 -c "import json;d=json.load(open('gpurun_out/r09zf_${c}_$v.json'));print(d['value'], d['ms_per_step'])")" | tee -a gpurun_out/r09zf_ab.txt
    done
  done
done
