#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_eval.py > gpurun_out/r03zs_t.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r03zs_t.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 tools/eval_bench.py > gpurun_out/r03zs_eval.json 2> gpurun_out/r03zs_eval.err || { tail -20 gpurun_out/r03zs_eval.err; exit 1; }
cat gpurun_out/r03zs_eval.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r03zs_prof -o eval --output-format csv -- python3 $R/tools/eval_bench.py --images 8 --reps 1 > $R/gpurun_out/r03zs_prof.log 2>&1 || { tail -20 $R/gpurun_out/r03zs_prof.log; exit 1; }
echo DONE
