#!/bin/bash
# One gpurun call: GPU parity tests, smoke, bench (with CPU baseline), rocprof kernel stats.
# usage: gpurun -- bash tools/gpu_check.sh TAG
set -o pipefail
TAG=${1:-run}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -m pytest tests -m gpu -q -rf -s -p no:cacheprovider > gpurun_out/tests_$TAG.log 2>&1
echo "TESTS EXIT $?" | tee -a gpurun_out/tests_$TAG.log
rc=$(tail -1 gpurun_out/tests_$TAG.log | awk '{print $3}')
case $rc in 0|1) ;; *) echo "abort after tests rc=$rc"; exit $rc;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo SMOKE FAIL; cat gpurun_out/smoke_$TAG.log | tail -20; exit 1; }
timeout -k 10 400 python bench.py ${BENCH_ARGS:---steps 20 --warmup 5} > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo BENCH FAIL; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $R/gpurun_out/prof_$TAG.log 2>&1 || { echo PROF FAIL; tail -20 $R/gpurun_out/prof_$TAG.log; exit 1; }
# the dominant kernel's launches the roofline times live (g_a.2 fwd: the first main-queue ig_kernel_x3d of each
# step) from the same trace, to set beside bench's live figure
python3 $R/tools/trace_timeline.py $(find $R/gpurun_out/prof_$TAG -name "*kernel_trace.csv" | head -1) --first ig_kernel_x3d > $R/gpurun_out/first_$TAG.txt 2>&1
head -2 $R/gpurun_out/first_$TAG.txt
echo DONE
