#!/bin/bash
# PMC passes (FETCH_SIZE, WRITE_SIZE: one counter per run) and a stats pass over the layer_bench ops matching $1
#   gpurun -- bash tools/gpu_pmc_layers.sh "g_a.0,g_s.6" TAG [MATH]
set -o pipefail
R=$GRAFT_REPO_ROOT; F="$1"; TAG=${2:-pmcl}; MATH=${3:-2}
mkdir -p $R/gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace -d $R/gpurun_out/$TAG/$c -o $c --output-format csv -- python3 $R/tools/layer_bench.py --only "$F" --reps 3 --math $MATH > $R/gpurun_out/$TAG/$c.log 2>&1 || { tail -20 $R/gpurun_out/$TAG/$c.log; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$TAG/stats -o stats --output-format csv -- python3 $R/tools/layer_bench.py --only "$F" --reps 20 --math $MATH > $R/gpurun_out/$TAG/stats.log 2>&1 || { tail -20 $R/gpurun_out/$TAG/stats.log; exit 1; }
echo DONE
