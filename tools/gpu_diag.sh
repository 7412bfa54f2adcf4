#!/bin/bash
# Error report of the model step at the benched plans (tools/model_err.py), one line per config.
# usage: gpurun -- bash tools/gpu_diag.sh TAG
set -o pipefail
TAG=${1:-d}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
O=gpurun_out/diag_$TAG.txt
: > $O
run() { echo "== $*" >> $O; timeout -k 10 240 python -u tools/model_err.py "$@" >> $O 2>&1 || { echo "FAIL rc=$? $*" >> $O; exit 1; }; }
run --n 2 --size 128 --math fp32_split
run --n 2 --size 128 --math fp32
run --n 16 --size 256 --math fp32_split
run --n 16 --size 256 --math fp32
run --n 4 --size 512 --math fp32_split
run --n 16 --size 256 --math fp32_split --loss msssim --lam 64
run --n 16 --size 256 --math bf16 --latent 320 --lam 4096
cat $O
