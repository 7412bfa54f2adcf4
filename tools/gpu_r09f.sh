#!/bin/bash
# Full GPU suite after the round-6 housekeeping (dead kernel variants removed), smoke, C2/C3/C4 bench
# lines, and a C3 kernel trace with the hyperprior on bf16 operands.
set -o pipefail
TAG=${1:-r09f}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/tests_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
for c in C2 C3 C4; do
  timeout -k 10 300 python3 bench.py --config $c --no-cpu-baseline > gpurun_out/bench_${TAG}_$c.json 2> gpurun_out/bench_${TAG}_$c.err || { tail gpurun_out/bench_${TAG}_$c.err; exit 1; }
  cut -c1-240 gpurun_out/bench_${TAG}_$c.json
done
bash tools/gpu_cfgprof.sh ${TAG} C3
