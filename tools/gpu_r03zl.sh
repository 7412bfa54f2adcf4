#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
MATH=2 bash tools/gpu_sqpmc.sh "g_a.0 conv3->192 fwd" r03zl_sq && python3 tools/sq_summary.py gpurun_out/r03zl_sq edge > gpurun_out/r03zl_sq.txt; cat gpurun_out/r03zl_sq.txt
