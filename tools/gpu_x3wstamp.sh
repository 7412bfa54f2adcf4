#!/bin/bash
# Phase cycles of gdn_bwd_x3w_kernel under stamp builds: gpurun -- bash tools/gpu_x3wstamp.sh OUT tag...
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
OUT=$1; shift
for t in "$@"; do
  echo "== $t" | tee -a gpurun_out/$OUT.txt
  IMGCOMP_LIB=$PWD/tools/_abl/$t/libimgcomp.so timeout -k 10 120 python tools/x3w_stamps.py 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/$OUT.txt || exit 1
done
