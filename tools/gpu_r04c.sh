#!/bin/bash
# eval-mode weight cache: eval / model / step / ops tests, then the eval-path timing with a rocprof summary
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_eval.py tests/test_model_gpu.py tests/test_step_gpu.py tests/test_solver.py > gpurun_out/r04c_t.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r04c_t.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python tools/eval_bench.py > gpurun_out/r04c_eval.json 2>gpurun_out/r04c_eval.err || { tail gpurun_out/r04c_eval.err; exit 1; }
cat gpurun_out/r04c_eval.json
