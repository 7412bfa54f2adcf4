#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_split_gpu.py > gpurun_out/r03zo_t.log 2>&1; echo "tests rc=$?"; tail -2 gpurun_out/r03zo_t.log
PYTHONPATH=. IMGCOMP_LIB=tools/_abl/stamp/libimgcomp.so timeout -k 10 120 python3 tools/ec3_stamp.py 32 > gpurun_out/r03zo_stamp.txt 2>&1; cat gpurun_out/r03zo_stamp.txt
bash tools/gpu_libab.sh r03zo_ab "g_a.0 conv3->192 fwd,g_s.6 tconv192->3 dgrad" 2
