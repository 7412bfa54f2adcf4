#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
bash tools/gpu_libab.sh r03zb_ab "g_a.0 conv3->192 fwd" 2 ec1 ec2 ec4 ec7
