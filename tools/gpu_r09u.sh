#!/bin/bash
# Edge conv with the k-step count as a template constant (no branch between the MFMA groups) vs round-6
# base: g_a.0 fwd and g_s.6 dgrad in isolation (split and bf16), then C2 / C3 interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
bash tools/gpu_libab.sh r09u_layers "g_a.0 conv3->192 fwd,g_s.6 tconv192->3 dgrad" 2 base s3 || exit 1
bash tools/gpu_libab.sh r09u_layers_bf16 "g_a.0 conv3->192 fwd,g_s.6 tconv192->3 dgrad" 1 base s3 || exit 1
for i in 1 2; do
  for c in C2 C3; do
    for v in base s3; do
      IMGCOMP_LIB=$R/tools/_abl/$v/libimgcomp.so timeout -k 10 200 python3 bench.py --config $c --no-cpu-baseline --no-roofline \
        > gpurun_out/r09u_${c}_$v.json 2>gpurun_out/r09u_${c}_$v.err || { tail gpurun_out/r09u_${c}_$v.err; exit 1; }
      echo "$c $v $(python3 -c "import json;d=json.load(open('gpurun_out/r09u_${c}_$v.json'));print(d['value'], d['ms_per_step'])")" | tee -a gpurun_out/r09u_ab.txt
    done
  done
done
