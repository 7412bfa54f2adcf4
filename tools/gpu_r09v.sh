#!/bin/bash
# CDF MLPs of any geometry (the wide kernels): the factorized entropy model against the fp64 oracle over
# eight (DIMS, BIN) geometries, train and eval; the reference's DIMS golden fixtures; then the C2 line.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_ops_gpu.py -k "factorized" tests/test_model_gpu.py -k "factorized or dims" > gpurun_out/tests_r09v.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|error|passed|failed" gpurun_out/tests_r09v.log | tail -30; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-roofline | cut -c1-200
