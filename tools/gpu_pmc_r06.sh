#!/bin/bash
# PMC HBM traffic (FETCH_SIZE and WRITE_SIZE in separate passes) + kernel stats of the round-5 kernels:
# the GDN backward at 128^2, the g_a.2 split weight gradient, the MS-SSIM tile kernels at C4.
#   gpurun -- bash tools/gpu_pmc_r06.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT; TAG=${1:-pmc6}
mkdir -p $R/gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp
run() {  # name counter-or-stats cmd...
  local n=$1 c=$2; shift 2
  if [ $c = stats ]; then
    timeout -k 10 -s KILL 150 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$TAG/$n/stats -o p --output-format csv -- "$@" > $R/gpurun_out/$TAG/$n.stats.log 2>&1 || { echo "FAIL $n stats"; tail -5 $R/gpurun_out/$TAG/$n.stats.log; exit 1; }
  else
    timeout -k 10 -s KILL 150 rocprofv3 --pmc $c --kernel-trace -d $R/gpurun_out/$TAG/$n/$c -o p --output-format csv -- "$@" > $R/gpurun_out/$TAG/$n.$c.log 2>&1 || { echo "FAIL $n $c"; tail -5 $R/gpurun_out/$TAG/$n.$c.log; exit 1; }
  fi
}
for c in FETCH_SIZE WRITE_SIZE stats; do
  run gdn $c python3 $R/tools/gdn_bwd_time.py --sizes 128 --reps 3
  run wg $c python3 $R/tools/layer_bench.py --math 2 --only "g_a.2 conv wgrad" --reps 5
  run ssim $c python3 $R/tools/msssim_time.py --reps 3
done
cd $R
python3 tools/pmc_kernels.py gpurun_out/$TAG/gdn "gdn_bwd_x3w=1611e6" | tee gpurun_out/$TAG/summary.txt
python3 tools/pmc_kernels.py gpurun_out/$TAG/wg "wg_x3g=507e6" | tee -a gpurun_out/$TAG/summary.txt
python3 tools/pmc_kernels.py gpurun_out/$TAG/ssim "ssim_fwd_tile=0" "ssim_bwd_tile=0" | tee -a gpurun_out/$TAG/summary.txt
echo DONE
