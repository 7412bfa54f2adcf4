#!/bin/bash
# r03d: is the rare CDF-gradient mismatch an in-kernel fault of the factorized backward?
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u tools/race_probe.py --reps 120 --pattern conc --check-fact > gpurun_out/race_fact.log 2>&1 || { tail -5 gpurun_out/race_fact.log; exit 1; }
grep -v "^ " gpurun_out/race_fact.log | tail -12
