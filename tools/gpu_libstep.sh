#!/bin/bash
# C2 bench (no CPU baseline) under the in-tree lib and each tools/_abl/<tag>/libimgcomp.so (with a copy of
# libimgcomp_torch.so beside it, which loads its sibling), alternating twice:
#   gpurun -- bash tools/gpu_libstep.sh OUT tag1 tag2 ...
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
OUT=$1; shift
: > gpurun_out/$OUT.txt
for rep in 1 2; do
  echo "== base" >> gpurun_out/$OUT.txt
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline 2>>gpurun_out/$OUT.err | python -c "import json,sys; b=json.loads(sys.stdin.read()); print(b['value'], b['ms_per_step'])" >> gpurun_out/$OUT.txt || exit 1
  for t in "$@"; do
    echo "== $t" >> gpurun_out/$OUT.txt
    IMGCOMP_LIB=$PWD/tools/_abl/$t/libimgcomp.so timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline 2>>gpurun_out/$OUT.err | python -c "import json,sys; b=json.loads(sys.stdin.read()); print(b['value'], b['ms_per_step'])" >> gpurun_out/$OUT.txt || exit 1
  done
done
cat gpurun_out/$OUT.txt
