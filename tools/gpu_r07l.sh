#!/bin/bash
# x3w re-slicing (tests + timing vs X3W_SLICE=1) and the x3p producer-priority A/B
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
bash tools/gpu_gdnb.sh r07l x3wslice1 || exit 1
bash tools/gpu_libab.sh wgprio_r07l "g_a.2 conv wgrad,g_s.4 tconv wgrad" 2 wgprio1 wgprio2 wgprio3 wgp16 || exit 1
