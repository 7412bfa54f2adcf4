#!/bin/bash
# PMC passes (one counter group per run) for the dominant kernel: HBM bytes per launch;
# then a plain --kernel-trace --stats run of the same command (its average duration).
set -o pipefail
R=$GRAFT_REPO_ROOT; TAG=${1:-pmc}; MATH=${2:-fp32}
mkdir -p $R/gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $R/gpurun_out/$TAG/fetch -o fetch --output-format csv -- python3 $R/tools/dominant_kernel.py 10 $MATH > $R/gpurun_out/$TAG/fetch.log 2>&1 || { tail -20 $R/gpurun_out/$TAG/fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $R/gpurun_out/$TAG/write -o write --output-format csv -- python3 $R/tools/dominant_kernel.py 10 $MATH > $R/gpurun_out/$TAG/write.log 2>&1 || { tail -20 $R/gpurun_out/$TAG/write.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$TAG/stats -o stats --output-format csv -- python3 $R/tools/dominant_kernel.py 20 $MATH > $R/gpurun_out/$TAG/stats.log 2>&1 || { tail -20 $R/gpurun_out/$TAG/stats.log; exit 1; }
find $R/gpurun_out/$TAG -name "*.csv" | head
echo DONE
