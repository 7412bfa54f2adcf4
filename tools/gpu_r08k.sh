#!/bin/bash
# WG_X3P_PRIO=0 (tools/_abl/prio0: weight-gradient producers at normal issue priority) vs the in-tree 1, C3 bench alternating
set -o pipefail
TAG=${1:-r08k}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for rep in 1 2; do
  timeout -k 10 300 python bench.py --config C3 --steps 20 --warmup 5 --no-cpu-baseline --no-roofline > gpurun_out/bench_${TAG}_C3.json 2>gpurun_out/bench_${TAG}_C3.err || { echo BENCH FAIL; tail gpurun_out/bench_${TAG}_C3.err; exit 1; }
  cut -c1-150 gpurun_out/bench_${TAG}_C3.json
  IMGCOMP_LIB=$PWD/tools/_abl/prio0/libimgcomp.so timeout -k 10 300 python bench.py --config C3 --steps 20 --warmup 5 --no-cpu-baseline --no-roofline > gpurun_out/bench_${TAG}_C3_v.json 2>gpurun_out/bench_${TAG}_C3_v.err || { echo BENCH2 FAIL; tail gpurun_out/bench_${TAG}_C3_v.err; exit 1; }
  cut -c1-150 gpurun_out/bench_${TAG}_C3_v.json
done
echo DONE
