#!/bin/bash
# SQ counters of the edge conv (g_a.0 fwd) in split and bf16 arithmetic, for what bounds it.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
MATH=2 bash tools/gpu_sqpmc.sh "g_a.0 conv3->192 fwd" r09y_sq_split || exit 1
MATH=1 bash tools/gpu_sqpmc.sh "g_a.0 conv3->192 fwd" r09y_sq_bf16 || exit 1
