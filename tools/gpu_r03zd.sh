#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
bash tools/gpu_libab.sh r03zd_ab "g_a.0 conv3->192 fwd,g_s.6 tconv192->3 dgrad" 2 ec1 ec2 ec4 ec8 ec6
