#!/bin/bash
# kernel + HIP runtime API trace of a few bench steps (when each launch was enqueued vs when it ran).
#   gpurun -- bash tools/gpu_apitrace.sh TAG CONFIG
set -o pipefail
TAG=$1; C=${2:-C4}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace -d $R/gpurun_out/api_${TAG}_$C -o run --output-format csv \
  -- python3 $R/bench.py --config $C --steps 3 --warmup 2 --no-cpu-baseline --no-roofline --profile-step-only \
  > $R/gpurun_out/api_${TAG}_$C.log 2>&1 || { echo "PROF FAIL"; tail -20 $R/gpurun_out/api_${TAG}_$C.log; exit 1; }
ls -la $R/gpurun_out/api_${TAG}_$C/*
