#!/bin/bash
# Time layer ops under the in-tree lib and each tools/_abl/<tag>/libimgcomp.so:
#   gpurun -- bash tools/gpu_libab.sh OUT "ONLY" MATH tag1 tag2 ...
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
OUT=$1; ONLY=$2; MATH=$3; shift 3
echo "== base" | tee gpurun_out/$OUT.txt
timeout -k 10 120 python tools/layer_bench.py --math $MATH --only "$ONLY" --reps 20 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/$OUT.txt || exit 1
for t in "$@"; do
  echo "== $t" | tee -a gpurun_out/$OUT.txt
  IMGCOMP_LIB=$PWD/tools/_abl/$t/libimgcomp.so timeout -k 10 120 python tools/layer_bench.py --math $MATH --only "$ONLY" --reps 20 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/$OUT.txt || exit 1
done
