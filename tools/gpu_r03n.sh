#!/bin/bash
# r03n: layer timing of the all-DMA split kernel (in-tree) vs the x3s<128> build (tools/_abl/nodma), twice
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
bash tools/gpu_libab.sh r03n_ab "g_a.2 conv fwd,g_a.2 conv dgrad,g_s.4 tconv fwd,g_s.4 tconv dgrad" 2 nodma || exit 1
bash tools/gpu_libab.sh r03n_ab2 "g_a.2 conv fwd,g_a.2 conv dgrad,g_s.4 tconv fwd,g_s.4 tconv dgrad" 2 nodma
