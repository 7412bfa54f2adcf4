#!/bin/bash
# Time the GDN backward under the in-tree lib and each tools/_abl/<tag>/libimgcomp.so (alternating twice).
#   gpurun -- bash tools/gpu_gdnvar.sh OUT tag1 tag2 ...
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
OUT=$1; shift
for rep in 1 2; do
  timeout -k 10 120 python tools/gdn_bwd_time.py 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/$OUT.txt || exit 1
  for t in "$@"; do
    IMGCOMP_LIB=$PWD/tools/_abl/$t/libimgcomp.so timeout -k 10 120 python tools/gdn_bwd_time.py 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/$OUT.txt || exit 1
  done
done
