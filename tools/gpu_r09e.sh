#!/bin/bash
# edge_conv_x3: DMA patches (in-tree) vs register-staged (EC_LF=0) alternating; per-kernel clock of
# the C2 step (GRBM_GUI_ACTIVE, kernels serialized by the counter collection).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
for i in 1 2; do
  for v in base eclf0; do
    lib=""; [ $v = base ] || lib=$R/tools/_abl/$v/libimgcomp.so
    echo "== $v" | tee -a gpurun_out/r09e_ab.txt
    IMGCOMP_LIB=$lib timeout -k 10 120 python tools/layer_bench.py --math 2 --only "g_a.0 conv3->192 fwd,g_s.6 tconv192->3 dgrad" --reps 30 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/r09e_ab.txt || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --pmc GRBM_GUI_ACTIVE -d $R/gpurun_out/pmc_clkstep -o run --output-format csv \
  -- python3 $R/bench.py --profile-step-only --steps 3 --warmup 2 --no-cpu-baseline --no-roofline --serial-hyperprior > $R/gpurun_out/pmc_clkstep.log 2>&1 || { echo PMC FAIL; tail $R/gpurun_out/pmc_clkstep.log; exit 1; }
python3 $R/tools/clock_map.py $R/gpurun_out/pmc_clkstep/run_counter_collection.csv | tee $R/gpurun_out/r09e_clock_map.txt
