#!/bin/bash
# r03i: layer timing in-tree (halo) vs nohalo (x3s), then SQ PMC of g_a.2 fwd for both
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
bash tools/gpu_libab.sh r03i_ab "g_a.2 conv fwd,g_a.2 conv dgrad,g_s.4 tconv fwd,g_s.4 tconv dgrad,g_a.4 conv fwd,g_s.2 tconv fwd" 2 nohalo || exit 1
MATH=2 bash tools/gpu_sqpmc.sh "g_a.2 conv fwd" r03i_sq_halo || exit 1
IMGCOMP_LIB=$GRAFT_REPO_ROOT/tools/_abl/nohalo/libimgcomp.so MATH=2 bash tools/gpu_sqpmc.sh "g_a.2 conv fwd" r03i_sq_x3s || exit 1
