#!/bin/bash
# Quick GPU iteration: parity tests + per-layer timings.  usage: gpurun -- bash tools/gpu_quick.sh TAG
set -o pipefail
TAG=${1:-q}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -rf -p no:cacheprovider > gpurun_out/tests_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/tests_$TAG.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/tests_$TAG.log | head -20; exit $rc; }
timeout -k 10 300 python tools/layer_bench.py --json gpurun_out/layers_$TAG.json > gpurun_out/layers_$TAG.txt 2>&1 || exit $?
cat gpurun_out/layers_$TAG.txt
