#!/bin/bash
# r03v: bf16 DMA kernel (x3d<1>): C3 parity, layer A/B (math 1) and C3 bench vs tools/_abl/nobfdma
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -k "bf16 or C3 or c2_" \
  tests/test_bf16_gpu.py tests/test_bench_plans_gpu.py > gpurun_out/r03v_tests.log 2>&1 \
  || { tail -40 gpurun_out/r03v_tests.log; exit 1; }
tail -1 gpurun_out/r03v_tests.log
bash tools/gpu_libab.sh r03v_ab "g_a.2 conv fwd,g_a.2 conv dgrad,g_s.4 tconv fwd,g_s.4 tconv dgrad" 1 nobfdma || exit 1
for v in base nobfdma base nobfdma; do
  if [ $v = base ]; then unset IMGCOMP_LIB; else export IMGCOMP_LIB=$GRAFT_REPO_ROOT/tools/_abl/$v/libimgcomp.so; fi
  timeout -k 10 300 python bench.py --config C3 --steps 20 --warmup 5 > gpurun_out/r03v_bench_$v.json 2>gpurun_out/r03v_bench.err || { tail -5 gpurun_out/r03v_bench.err; exit 1; }
  python -c "import json; r=json.load(open('gpurun_out/r03v_bench_$v.json')); print('$v', r['value'], r['ms_per_step'], r['roofline'] and r['roofline']['ms_per_launch'])"
done
