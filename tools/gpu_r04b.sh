#!/bin/bash
# Full per-layer table (fp32_split) and HBM PMC traffic of g_a.4 fwd (split-K DMA tiles) and the big split wgrad
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 200 python tools/layer_bench.py --math 2 --gdn-math 2 --reps 10 > gpurun_out/r04b_layers.txt 2>&1 || { tail gpurun_out/r04b_layers.txt; exit 1; }
cat gpurun_out/r04b_layers.txt
bash tools/gpu_pmc_layers.sh "g_a.4 conv fwd,g_a.2 conv wgrad,g_s.4 tconv wgrad" r04b_pmc 2 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r04b_lstats -o l --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/layer_bench.py --math 2 --gdn-math 2 --reps 3 > $GRAFT_REPO_ROOT/gpurun_out/r04b_lstats.log 2>&1
cd $GRAFT_REPO_ROOT && bash tools/gpu_libab.sh r04b_prio_ab "g_a.2 conv fwd,g_s.4 tconv fwd,g_a.2 conv dgrad,g_a.4 conv fwd" 2 prio1 prio3
