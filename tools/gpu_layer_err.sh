#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 60 tools/_abl/mfma_round > gpurun_out/mfma_round.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/layer_err.py --n 16 --size 256 > gpurun_out/layer_err_$1.txt 2>&1
