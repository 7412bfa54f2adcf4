#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
bash tools/gpu_libab.sh r03zg_ab "g_a.0 conv3->192 fwd,g_s.6 tconv192->3 dgrad,g_a.0 conv3->192 wgrad" 2 skew ec1 ec3 ec5 ec9 ec13 2
