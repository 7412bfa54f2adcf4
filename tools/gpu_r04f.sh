#!/bin/bash
# tconv_few2 column segments (any input width): parity at the fp32 bar, model/eval tests, eval-path timing
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_split_gpu.py tests/test_eval.py tests/test_ops_gpu.py > gpurun_out/r04f_t.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r04f_t.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python tools/eval_bench.py > gpurun_out/r04f_eval.json 2>gpurun_out/r04f_eval.err || { tail gpurun_out/r04f_eval.err; exit 1; }
cat gpurun_out/r04f_eval.json
timeout -k 10 200 python tools/layer_bench.py --math 2 --gdn-math 2 --reps 10 --only "g_s.6" --batch 32 > gpurun_out/r04f_gs6.txt 2>&1 && cat gpurun_out/r04f_gs6.txt
