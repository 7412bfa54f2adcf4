#!/bin/bash
# host-vs-GPU pacing of the eager step per config: gpurun -- bash tools/gpu_pace.sh TAG [configs]
set -o pipefail
TAG=$1; shift
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for c in ${@:-C4 C2}; do
  timeout -k 10 240 python tools/host_pace.py --config $c 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/pace_$TAG.txt || exit 1
done
