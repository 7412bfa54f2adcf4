#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
O=gpurun_out/diag2_$1.txt
: > $O
run() { echo "== $*" >> $O; timeout -k 10 240 python -u tools/model_err.py "$@" 2>&1 | grep -v "Warning\|va, vb\|Consider\|amdgpu.ids" | head -24 >> $O || { echo "FAIL $*" >> $O; exit 1; }; }
run --n 16 --size 256 --math fp32_split --bwd-math 0
run --n 16 --size 256 --math fp32 --bwd-math 2
run --n 16 --size 256 --math fp32_split --hyper-math 0
