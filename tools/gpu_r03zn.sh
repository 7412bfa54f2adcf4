#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
PYTHONPATH=. IMGCOMP_LIB=tools/_abl/stamp/libimgcomp.so timeout -k 10 120 python3 tools/ec3_stamp.py 32 > gpurun_out/r03zn_stamp.txt 2>&1; rc=$?; cat gpurun_out/r03zn_stamp.txt; exit $rc
