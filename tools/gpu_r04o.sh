#!/bin/bash
# tconv_few2 with product-outer MFMA order (TF2_POUTER): parity under the variant, then layer A/B
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
IMGCOMP_LIB=$PWD/tools/_abl/pouter/libimgcomp.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_split_gpu.py -k tconv_few > gpurun_out/r04o_t.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r04o_t.log; [ $rc -eq 0 ] || exit 1
bash tools/gpu_libab.sh r04o_ab "g_s.6 tconv192->3 fwd" 2 pouter && bash tools/gpu_libab.sh r04o_ab2 "g_s.6 tconv192->3 fwd" 2 pouter
