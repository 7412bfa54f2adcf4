#!/bin/bash
# C2 bench (no CPU baseline) alternating environment settings, twice each:
#   gpurun -- bash tools/gpu_envab.sh OUT "VAR=a" "VAR=b" ...
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
OUT=$1; shift
: > gpurun_out/$OUT.txt
for rep in 1 2; do
  for e in "$@"; do
    echo "== $e" >> gpurun_out/$OUT.txt
    env $e timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline 2>>gpurun_out/$OUT.err | python -c "import json,sys; b=json.loads(sys.stdin.read()); print(b['value'], b['ms_per_step'])" >> gpurun_out/$OUT.txt || exit 1
  done
done
cat gpurun_out/$OUT.txt
