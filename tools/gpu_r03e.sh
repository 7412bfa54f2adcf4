#!/bin/bash
# r03e: the factorized backward's reduction through LDS alone (in-tree) vs the shuffle block sum
# (tools/_abl/factshfl): concurrent C2 steps with the per-launch recompute check
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u tools/race_probe.py --reps 120 --pattern conc --check-fact > gpurun_out/race_fact_lds.log 2>&1 || { tail -5 gpurun_out/race_fact_lds.log; exit 1; }
grep -v "^ " gpurun_out/race_fact_lds.log | tail -4
IMGCOMP_LIB=$GRAFT_REPO_ROOT/tools/_abl/factshfl/libimgcomp.so timeout -k 10 400 python -u tools/race_probe.py --reps 120 --pattern conc --check-fact > gpurun_out/race_fact_shfl.log 2>&1 || { tail -5 gpurun_out/race_fact_shfl.log; exit 1; }
grep -v "^ " gpurun_out/race_fact_shfl.log | tail -4
