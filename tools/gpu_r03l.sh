#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 200 python -u tools/bf16_model_probe.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r03l_model_probe.txt
