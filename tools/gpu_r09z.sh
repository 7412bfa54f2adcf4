#!/bin/bash
# Phase stamps of the edge conv (stamp build), split and bf16.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for m in 2 1; do
  IMGCOMP_LIB=$PWD/tools/_abl/ecst/libimgcomp.so timeout -k 10 120 python3 tools/edge_stamps.py --math $m 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/r09z_edge_stamps.txt || exit 1
done
