#!/bin/bash
# kernel trace of the two-rank one-GPU DDP rehearsal (tools/ddp_trace.py), per-process timelines
set -o pipefail
TAG=${1:-r07v}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $R/gpurun_out/ddp_$TAG -o run --output-format csv \
  -- python3 $R/tools/ddp_trace.py > $R/gpurun_out/ddp_$TAG.log 2>&1 || { echo "DDP TRACE FAIL"; tail -20 $R/gpurun_out/ddp_$TAG.log; exit 1; }
tail -2 $R/gpurun_out/ddp_$TAG.log
for f in $(find $R/gpurun_out/ddp_$TAG -name "*kernel_trace.csv"); do
  echo "== $f"; python3 $R/tools/trace_timeline.py $f 2>&1 | head -20
done
