#!/bin/bash
# GPU parity suite + smoke (+ optional extra python tool): usage gpurun -- bash tools/gpu_tests.sh TAG [pytest args]
set -o pipefail
TAG=${1:-t}; shift
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -rfP -p no:cacheprovider "$@" > gpurun_out/tests_$TAG.log 2>&1
rc=$?
tail -40 gpurun_out/tests_$TAG.log | grep -E "passed|failed|FAILED|ERROR|Error" | head -40
case $rc in 0|1) ;; *) echo "abort rc=$rc"; exit $rc;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo SMOKE FAIL; tail -5 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
exit $rc
