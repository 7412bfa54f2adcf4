#!/bin/bash
# Ablations of ig_kernel_x3d (no A split, no DMA) and edge_conv_x3 (no stores, no loads) on their
# C2 layers, and C3 with the hyperprior convs on bf16 operands (A/B alternating).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
OUT=gpurun_out/r09b.txt
bash tools/gpu_libab.sh r09b_abl "g_a.2 conv fwd,g_a.0 conv3->192 fwd" 2 x3dnosplit x3dnodma ecnostore ecnoload || exit 1
for i in 1 2; do
  for v in split bf16; do
    IMGCOMP_C3_HYPER=$v timeout -k 10 200 python3 bench.py --config C3 --no-cpu-baseline --no-roofline > gpurun_out/r09b_c3_$v.json 2>gpurun_out/r09b_c3_$v.err || { echo FAIL; tail gpurun_out/r09b_c3_$v.err; exit 1; }
    echo "C3 hyper=$v $(python3 -c "import json;d=json.load(open('gpurun_out/r09b_c3_$v.json'));print(d['value'], d['ms_per_step'])")" | tee -a $OUT
  done
done
