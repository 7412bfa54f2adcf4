#!/bin/bash
# C2 step: eager vs hipGraph replay (TrainStep), alternating
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
: > gpurun_out/r04g.txt
for rep in 1 2; do
  for mode in "" "--graph"; do
    echo "== eager$mode" >> gpurun_out/r04g.txt
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline $mode 2>>gpurun_out/r04g.err | python -c "import json,sys; b=json.loads(sys.stdin.read()); print(b['value'], b['ms_per_step'], b['config']['workload'][-30:])" >> gpurun_out/r04g.txt || exit 1
  done
done
cat gpurun_out/r04g.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r04g -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --graph > $GRAFT_REPO_ROOT/gpurun_out/prof_r04g.log 2>&1
