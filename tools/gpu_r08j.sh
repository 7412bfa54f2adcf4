#!/bin/bash
# IG_X3D_MINT=16 (tools/_abl/mint16: one-phase maps of 16-31 tiles of 256 rows on ig_kernel_x3d with split K)
# vs the in-tree 32: C4 bench alternating, then the C4 step profile under the variant
set -o pipefail
TAG=${1:-r08j}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for rep in 1 2; do
  timeout -k 10 300 python bench.py --config C4 --steps 20 --warmup 5 --no-cpu-baseline --no-roofline > gpurun_out/bench_${TAG}_C4.json 2>gpurun_out/bench_${TAG}_C4.err || { echo BENCH FAIL; tail gpurun_out/bench_${TAG}_C4.err; exit 1; }
  cut -c1-150 gpurun_out/bench_${TAG}_C4.json
  IMGCOMP_LIB=$PWD/tools/_abl/mint16/libimgcomp.so timeout -k 10 300 python bench.py --config C4 --steps 20 --warmup 5 --no-cpu-baseline --no-roofline > gpurun_out/bench_${TAG}_C4_v.json 2>gpurun_out/bench_${TAG}_C4_v.err || { echo BENCH2 FAIL; tail gpurun_out/bench_${TAG}_C4_v.err; exit 1; }
  cut -c1-150 gpurun_out/bench_${TAG}_C4_v.json
done
echo DONE
