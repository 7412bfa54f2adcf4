#!/bin/bash
# r03c: race probe (many concurrent C2 steps vs a serial reference), SQ counters of g_a.2 fwd for
# ig_kernel_x3s (in-tree lib) and ig_kernel_x3r (tools/_abl/lib_x3r.so)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/race_probe.py --reps 60 --pattern alt > gpurun_out/race_alt.log 2>&1 || { tail -5 gpurun_out/race_alt.log; exit 1; }
tail -3 gpurun_out/race_alt.log
timeout -k 10 300 python -u tools/race_probe.py --reps 80 --pattern conc > gpurun_out/race_conc.log 2>&1 || { tail -5 gpurun_out/race_conc.log; exit 1; }
tail -3 gpurun_out/race_conc.log
MATH=2 bash tools/gpu_sqpmc.sh "g_a.2 conv fwd" sq_x3s || exit 1
MATH=2 IMGCOMP_LIB=$GRAFT_REPO_ROOT/tools/_abl/lib_x3r.so bash tools/gpu_sqpmc.sh "g_a.2 conv fwd" sq_x3r || exit 1
python3 tools/sq_summary.py gpurun_out/sq_x3r ig_kernel
python3 tools/sq_summary.py gpurun_out/sq_x3s ig_kernel
