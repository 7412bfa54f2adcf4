#!/bin/bash
# One A/B round of a kernel variant built by tools/abl_build.sh into tools/_abl/<tag>/ (this replaces
# the per-experiment tools/gpu_r0*.sh records of rounds 1-3; their results are under profiles/):
#   gpurun -- bash tools/gpu_variant.sh OUT TAG [-t "pytest selection"] [-l "layer ops" MATH] [-s]
#     -t  parity tests run under the variant first (stops here when they fail)
#     -l  tools/layer_bench.py ops, base vs variant (tools/gpu_libab.sh)
#     -s  the C2 bench step, base vs variant alternating twice (tools/gpu_libstep.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
OUT=$1; TAG=$2; shift 2
while [ $# -gt 0 ]; do
  case $1 in
    -t) IMGCOMP_LIB=$PWD/tools/_abl/$TAG/libimgcomp.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 \
          --timeout-method thread -m gpu $2 > gpurun_out/${OUT}_t.log 2>&1; rc=$?
        echo "tests under $TAG rc=$rc"; tail -2 gpurun_out/${OUT}_t.log; [ $rc -eq 0 ] || exit 1; shift 2;;
    -l) bash tools/gpu_libab.sh ${OUT}_ab "$2" $3 $TAG || exit 1; shift 3;;
    -s) bash tools/gpu_libstep.sh ${OUT}_step $TAG || exit 1; shift;;
    *) echo "unknown option $1"; exit 2;;
  esac
done
