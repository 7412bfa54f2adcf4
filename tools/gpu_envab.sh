#!/bin/bash
# bench A/B of an environment knob, alternating: gpurun -- bash tools/gpu_envab.sh TAG VAR "v1 v2" "C4 C2" [reps]
set -o pipefail
TAG=$1; VAR=$2; VALS=$3; CFGS=$4; REPS=${5:-2}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for c in $CFGS; do
  for rep in $(seq 1 $REPS); do
    for v in $VALS; do
      env $VAR=$v timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline --no-roofline \
        > gpurun_out/envab_${TAG}_${c}_$v.json 2>/dev/null || { echo BENCH FAIL; exit 1; }
      python -c "import json,sys; r=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], r['value'], r['ms_per_step'])" \
        gpurun_out/envab_${TAG}_${c}_$v.json "$c" "$VAR=$v" | tee -a gpurun_out/envab_$TAG.txt
    done
  done
done
