#!/bin/bash
# edge_conv_x3 with LDS-DMA patches (EC_LF): parity tests, layer timings, the C2 bench; the clock
# (GRBM_GUI_ACTIVE per launch) of ig_kernel_x3d with and without its DMA.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_split_gpu.py tests/test_bf16_gpu.py -k "conv_split or tconv_few or edges" > gpurun_out/tests_r09d.log 2>&1
rc=$?; tail -3 gpurun_out/tests_r09d.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_model_gpu.py "tests/test_bench_plans_gpu.py::test_config_step_vs_oracle_and_bench_plans[C2]" >> gpurun_out/tests_r09d.log 2>&1
rc=$?; tail -3 gpurun_out/tests_r09d.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/layer_bench.py --math 2 --only "g_a.0 conv3->192 fwd,g_s.6 tconv192->3 dgrad,g_s.6 tconv192->3 fwd" --reps 20 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r09d_layers.txt || exit 1
timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/r09d_c2.json 2> gpurun_out/r09d_c2.err || { tail gpurun_out/r09d_c2.err; exit 1; }
cut -c1-260 gpurun_out/r09d_c2.json
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for v in base x3dnodma; do
  lib=""; [ $v = base ] || lib=$R/tools/_abl/$v/libimgcomp.so
  IMGCOMP_LIB=$lib timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d $R/gpurun_out/pmc_clk_$v -o run --output-format csv \
    -- python3 $R/tools/layer_bench.py --math 2 --only "g_a.2 conv fwd" --reps 5 > $R/gpurun_out/pmc_clk_$v.log 2>&1 || { echo PMC FAIL $v; tail $R/gpurun_out/pmc_clk_$v.log; exit 1; }
done
echo DONE
