#!/bin/bash
# rocprofv3 kernel trace + stats of bench steps of the given configs, plus a per-step timeline.
#   gpurun -- bash tools/gpu_cfgprof.sh TAG C4 C5 ...
set -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for c in "$@"; do
  timeout -k 10 300 python3 $R/bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline --no-roofline \
    > $R/gpurun_out/bench_${TAG}_$c.json 2> $R/gpurun_out/bench_${TAG}_$c.err || { echo "BENCH FAIL $c"; tail -20 $R/gpurun_out/bench_${TAG}_$c.err; exit 1; }
  cut -c1-200 $R/gpurun_out/bench_${TAG}_$c.json
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${TAG}_$c -o run --output-format csv \
    -- python3 $R/bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline --no-roofline --profile-step-only \
    > $R/gpurun_out/prof_${TAG}_$c.log 2>&1 || { echo "PROF FAIL $c"; tail -20 $R/gpurun_out/prof_${TAG}_$c.log; exit 1; }
  f=$(find $R/gpurun_out/prof_${TAG}_$c -name "*kernel_trace.csv" | head -1)
  python3 $R/tools/trace_timeline.py $f > $R/gpurun_out/timeline_${TAG}_$c.txt 2>&1
  head -12 $R/gpurun_out/timeline_${TAG}_$c.txt
done
echo DONE
