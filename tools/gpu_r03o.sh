#!/bin/bash
# r03o: ablations of ig_kernel_x3d (1 no DMA, 2 no split, 3 neither) + SQ PMC of the in-tree kernel
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
bash tools/gpu_libab.sh r03o_ab "g_a.2 conv fwd,g_s.4 tconv fwd" 2 abl1 abl2 abl3 nodma || exit 1
MATH=2 bash tools/gpu_sqpmc.sh "g_a.2 conv fwd" r03o_sq_dma
