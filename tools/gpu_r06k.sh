#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
bash tools/gpu_libab.sh r06k_wgstag "g_a.2 conv wgrad,g_s.4 tconv wgrad" 2 wgnostag wgabl1 wgabl2 wgabl3 wgabl4 || exit 1
bash tools/gpu_envab.sh r06k IMGCOMP_SIDE_PRIORITY "0 -1" "C4 C2" 2
