#!/bin/bash
# r03y: x3d with tap-pair 16-channel chunks: parity; layer + step A/B vs tools/_abl/nopair; PMC traffic
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_dma_gpu.py tests/test_split_gpu.py tests/test_bench_plans_gpu.py -k "not C3 and not C4" > gpurun_out/r03y_tests.log 2>&1 \
  || { tail -40 gpurun_out/r03y_tests.log; exit 1; }
tail -1 gpurun_out/r03y_tests.log
bash tools/gpu_libab.sh r03y_ab "g_a.2 conv fwd,g_a.2 conv dgrad,g_s.4 tconv fwd,g_s.4 tconv dgrad,g_a.4 conv fwd,g_s.2 tconv dgrad" 2 nopair || exit 1
for v in base nopair base nopair; do
  if [ $v = base ]; then unset IMGCOMP_LIB; else export IMGCOMP_LIB=$GRAFT_REPO_ROOT/tools/_abl/$v/libimgcomp.so; fi
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r03y_bench_$v.json 2>gpurun_out/r03y_bench.err || { tail -5 gpurun_out/r03y_bench.err; exit 1; }
  python -c "import json; r=json.load(open('gpurun_out/r03y_bench_$v.json')); print('$v', r['value'], r['ms_per_step'], r['roofline']['ms_per_launch'])"
done
unset IMGCOMP_LIB
bash tools/gpu_pmc.sh r03y_pmc fp32_split || exit 1
cd $GRAFT_REPO_ROOT && PMC_KERNEL="ig_kernel_x3d" python tools/pmc_summary.py gpurun_out/r03y_pmc gpurun_out/r03y_pmc_dominant.json
