#!/bin/bash
# Round-5 (second half) PMC: the C3 dominant kernel (ig_kernel_b16d, g_a.2 fwd, bench roofline `traffic`) and
# the producer/consumer split weight gradient (wg_x3p, g_a.2), FETCH_SIZE / WRITE_SIZE in separate passes.
#   gpurun -- bash tools/gpu_pmc_r07.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT; TAG=${1:-pmc7}
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
  run dom $c python3 $R/tools/dominant_kernel.py 10 bf16
  run wg $c python3 $R/tools/layer_bench.py --math 2 --only "g_a.2 conv wgrad" --reps 5
done
cd $R
mkdir -p gpurun_out/$TAG/dompmc && cp -r gpurun_out/$TAG/dom/FETCH_SIZE gpurun_out/$TAG/dompmc/fetch && cp -r gpurun_out/$TAG/dom/WRITE_SIZE gpurun_out/$TAG/dompmc/write
PMC_KERNEL=ig_kernel_b16d python3 tools/pmc_summary.py gpurun_out/$TAG/dompmc gpurun_out/$TAG/${TAG}_bf16_pmc_dominant.json
python3 tools/pmc_kernels.py gpurun_out/$TAG/dom "ig_kernel_b16d=303e6" "ig_cvt_bf16=604e6" | tee gpurun_out/$TAG/summary.txt
python3 tools/pmc_kernels.py gpurun_out/$TAG/wg "wg_x3p=507e6" | tee -a gpurun_out/$TAG/summary.txt
echo DONE
