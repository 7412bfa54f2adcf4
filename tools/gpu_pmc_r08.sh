#!/bin/bash
# PMC of the C3 bf16 weight gradient on the bf16 copies (wg_x3p_kernel<false, 1, true>) inside the C3
# step (the copies exist only there), FETCH_SIZE / WRITE_SIZE / stats in separate passes.
#   gpurun -- bash tools/gpu_pmc_r08.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT; TAG=${1:-pmc8}
mkdir -p $R/gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE stats; do
  if [ $c = stats ]; then
    timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$TAG/c3/stats -o p --output-format csv \
      -- python3 $R/bench.py --config C3 --steps 3 --warmup 2 --no-cpu-baseline --no-roofline > $R/gpurun_out/$TAG/c3.stats.log 2>&1 || { echo "FAIL stats"; tail -5 $R/gpurun_out/$TAG/c3.stats.log; exit 1; }
  else
    timeout -k 10 -s KILL 200 rocprofv3 --pmc $c --kernel-trace -d $R/gpurun_out/$TAG/c3/$c -o p --output-format csv \
      -- python3 $R/bench.py --config C3 --steps 3 --warmup 2 --no-cpu-baseline --no-roofline > $R/gpurun_out/$TAG/c3.$c.log 2>&1 || { echo "FAIL $c"; tail -5 $R/gpurun_out/$TAG/c3.$c.log; exit 1; }
  fi
done
cd $R
python3 tools/pmc_kernels.py gpurun_out/$TAG/c3 "wg_x3p_kernel<false, 1, true>=252e6" "ig_kernel_b16d=303e6" | tee gpurun_out/$TAG/summary.txt
echo DONE
