#!/bin/bash
# wg_x3p_kernel ablations (diagnostic, wrong results): G stored unsplit (WG_X3P_ABL 64), nothing split (16)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for i in 1 2; do
  bash tools/gpu_libab.sh r09k_abl_$i "g_a.2 conv wgrad,g_s.4 tconv wgrad" 2 wgnogsplit wgnosplit || exit 1
done
