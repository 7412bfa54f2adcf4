#!/bin/bash
# r03s: split-K DMA tiles on one-phase mid/small maps: parity; C2 bench in-tree vs tools/_abl/big, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_dma_gpu.py tests/test_split_gpu.py tests/test_bench_plans_gpu.py > gpurun_out/r03s_tests.log 2>&1 \
  || { tail -40 gpurun_out/r03s_tests.log; exit 1; }
tail -1 gpurun_out/r03s_tests.log
for v in base big base big; do
  if [ $v = base ]; then unset IMGCOMP_LIB; else export IMGCOMP_LIB=$GRAFT_REPO_ROOT/tools/_abl/$v/libimgcomp.so; fi
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r03s_bench_$v.json 2>gpurun_out/r03s_bench.err || { tail -5 gpurun_out/r03s_bench.err; exit 1; }
  python -c "import json; r=json.load(open('gpurun_out/r03s_bench_$v.json')); print('$v', r['value'], r['ms_per_step'], r['roofline']['ms_per_launch'])"
done
