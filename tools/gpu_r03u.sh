#!/bin/bash
# r03u: 8-wave whole-split GDN backward: parity (GDN tests, split model, C2 step) + gdn_bwd timing vs tools/_abl/oldgdn
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -k "gdn or model or C2" \
  tests/test_split_gpu.py tests/test_ops_gpu.py tests/test_bench_plans_gpu.py > gpurun_out/r03u_tests.log 2>&1 \
  || { tail -40 gpurun_out/r03u_tests.log; exit 1; }
tail -1 gpurun_out/r03u_tests.log
bash tools/gpu_libab.sh r03u_ab "gdn_bwd" 2 oldgdn
