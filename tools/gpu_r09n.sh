#!/bin/bash
# Round-6 end-of-round check on the final tree: the full GPU suite, smoke, the C2 bench line (roofline +
# CPU baseline), C3 / C4 / C5 lines, and the C2 kernel trace + per-step timeline (profiles/r09n_*).
set -o pipefail
TAG=${1:-r09n}
R=$GRAFT_REPO_ROOT
cd $R; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/tests_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 400 python3 bench.py > gpurun_out/bench_${TAG}_line_C2.json 2> gpurun_out/bench_${TAG}_line_C2.err || { tail gpurun_out/bench_${TAG}_line_C2.err; exit 1; }
cut -c1-300 gpurun_out/bench_${TAG}_line_C2.json
for c in C3 C4 C5; do
  timeout -k 10 300 python3 bench.py --config $c --no-cpu-baseline > gpurun_out/bench_${TAG}_$c.json 2> gpurun_out/bench_${TAG}_$c.err || { tail gpurun_out/bench_${TAG}_$c.err; exit 1; }
  cut -c1-200 gpurun_out/bench_${TAG}_$c.json
done
bash tools/gpu_cfgprof.sh ${TAG} C2 || exit 1
f=$(find $R/gpurun_out/prof_${TAG}_C2 -name "*kernel_trace.csv" | head -1)
python3 $R/tools/trace_timeline.py $f --first ig_kernel_x3d > $R/gpurun_out/first_${TAG}.txt 2>&1
head -2 $R/gpurun_out/first_${TAG}.txt
