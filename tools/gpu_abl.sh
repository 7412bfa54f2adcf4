#!/bin/bash
# Time one layer op under each ablation lib: bash tools/gpu_abl.sh "ONLY" MATH tag1 tag2 ...
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
ONLY=$1; MATH=$2; shift 2
echo "== base" | tee gpurun_out/abl.txt
timeout -k 10 120 python tools/layer_bench.py --math $MATH --only "$ONLY" --reps 20 2>&1 | grep -v amdgpu.ids | tail -60 | tee -a gpurun_out/abl.txt || exit $?
for t in "$@"; do
  echo "== $t" | tee -a gpurun_out/abl.txt
  IMGCOMP_LIB=$PWD/tools/_abl/lib_$t.so timeout -k 10 120 python tools/layer_bench.py --math $MATH --only "$ONLY" --reps 20 2>&1 | grep -v amdgpu.ids | tail -60 | tee -a gpurun_out/abl.txt || exit $?
done
