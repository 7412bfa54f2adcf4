#!/bin/bash
# Fresh PMC (round 6): the dominant kernel in isolation (ig_kernel_x3d, g_a.2 fwd, fp32_split) and the
# C2 step's kernels (FETCH_SIZE / WRITE_SIZE / stats in separate passes) for the edge kernels.
set -o pipefail
R=$GRAFT_REPO_ROOT; TAG=r09j
cd $R && bash tools/gpu_pmc.sh ${TAG}_dom fp32_split || exit 1
mkdir -p $R/gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE stats; do
  if [ $c = stats ]; then
    timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$TAG/c2/stats -o p --output-format csv \
      -- python3 $R/bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-roofline --profile-step-only > $R/gpurun_out/$TAG/c2.stats.log 2>&1 || { echo "FAIL stats"; tail -5 $R/gpurun_out/$TAG/c2.stats.log; exit 1; }
  else
    timeout -k 10 -s KILL 200 rocprofv3 --pmc $c --kernel-trace -d $R/gpurun_out/$TAG/c2/$c -o p --output-format csv \
      -- python3 $R/bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-roofline --profile-step-only > $R/gpurun_out/$TAG/c2.$c.log 2>&1 || { echo "FAIL $c"; tail -5 $R/gpurun_out/$TAG/c2.$c.log; exit 1; }
  fi
done
cd $R
PMC_KERNEL=ig_kernel_x3d python3 tools/pmc_summary.py gpurun_out/${TAG}_dom gpurun_out/${TAG}_pmc_dominant.json || exit 1
cat gpurun_out/${TAG}_pmc_dominant.json
python3 tools/pmc_kernels.py gpurun_out/$TAG/c2 "edge_conv_x3_kernel=428e6" "edge_wgrad_kernel=428e6" "tconv_few2_kernel=428e6" | tee gpurun_out/$TAG/summary.txt
echo DONE
